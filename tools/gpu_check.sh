#!/bin/bash
# One GPU-box pass: parity tests, then a short bench (used with gpurun).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rocm-smi --showproductname > gpurun_out/gpu_info.txt 2>&1 || true
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-seconds 1.0 > gpurun_out/bench1.json 2> gpurun_out/bench1.err
echo "bench rc=$?"; cat gpurun_out/bench1.json; tail -5 gpurun_out/bench1.err
