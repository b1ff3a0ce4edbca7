#!/bin/bash
# Full GPU suite on the current build, then the BASELINE config matrix.  usage: bash tools/r02g_check.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
tag=${1:-r02g}; mkdir -p gpurun_out/$tag
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$tag/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/$tag/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
bash tools/bench_matrix.sh ${tag}_matrix
