#!/bin/bash
# hex27 LDS layout round: parity of the hex27 element, slab, overlap and matrix-free paths, then
# same-box A/B of the element kernel (h27old = round-5 layouts, h27gpf = padded factors only) and of
# the matrix-free action (apold = its round-5 layout)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
PYTEST_SEL="tests/test_h27_slab.py tests/test_h27_overlap.py tests/test_tangent_apply.py tests/test_fullsize.py tests/test_multigrid.py" bash tools/probes/r06.sh sel || exit 1
PYTEST_SEL="tests/test_gpu_parity.py -k 27" bash tools/probes/r06.sh sel || exit 1
LIBS="default h27old h27noxu h27xul" bash tools/probes/r06.sh h27ab || exit 1
mkdir -p gpurun_out/r06
KIN=totlag bash tools/probes/apply_ab.sh default h27old apv1 > gpurun_out/r06/apply_ab.txt 2>&1 || exit 1
KIN=linear bash tools/probes/apply_ab.sh default h27old apv1 >> gpurun_out/r06/apply_ab.txt 2>&1 || exit 1
cat gpurun_out/r06/apply_ab.txt
bash tools/probes/r06.sh suite smoke || exit 1
