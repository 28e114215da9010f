#!/bin/bash
# hex27 TotLag K image blocks 10 apart (product build) against rows of 9 (kimg9), hex27 parity,
# then the full suite on the product build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/r06
PYTEST_SEL="tests/test_h27_slab.py tests/test_h27_overlap.py tests/test_fullsize.py tests/test_gpu_parity.py" bash tools/probes/r06.sh sel || exit 1
for i in 1 2; do LIBS="default kimg9" bash tools/probes/r06.sh h27ab || exit 1; done
bash tools/probes/r06.sh suite smoke || exit 1
