#!/bin/bash
# A/B timing of two builds on one box: alternates tools/eval_timing.py between the default
# library and lib/libfourc_gpu_$1.so (FCG_LIB), $2 rounds, remaining args to eval_timing.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
ALT=$1; R=$2; shift 2
for i in $(seq "$R"); do
  timeout -k 10 120 python tools/eval_timing.py "$@" | tail -1 | sed "s/^/base /" || exit 1
  FCG_LIB=$ALT timeout -k 10 120 python tools/eval_timing.py "$@" | tail -1 | sed "s/^/$ALT /" || exit 1
done
