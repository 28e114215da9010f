set -o pipefail
export PYTEST_SEL="tests/test_gather_tiled.py tests/test_gpu_parity.py -k gather_or_tiled"
export PYTEST_SEL="tests/test_gather_tiled.py tests/test_gpu_parity.py"
bash tools/probes/r06.sh sel || exit 1
FCG_LIB=gsoa10 PYTEST_SEL="tests/test_gather_tiled.py" bash tools/probes/r06.sh sel || exit 1
FCG_LIB=gt11 PYTEST_SEL="tests/test_gather_tiled.py" bash tools/probes/r06.sh sel || exit 1
LIBS="default gold gblk9" ABTAG=totlag ETARGS="--n 100 --renumber --path gather --kinem totlag --reps 30" bash tools/probes/r06.sh libab || exit 1
LIBS="default gold gblk9 gsoa gsoa10 gt11 gw9" ABTAG=linear ETARGS="--n 100 --renumber --path gather --kinem linear --reps 30" bash tools/probes/r06.sh libab || exit 1
