#!/bin/bash
# One iteration on the GPU box: parity tests, then short benches of the AES variants given in $VARIANTS.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for v in ${VARIANTS:-0}; do
  QPP_AES_VARIANT=$v timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu $BENCH_ARGS > gpurun_out/bench_v$v.json 2> gpurun_out/bench_v$v.err || { tail -5 gpurun_out/bench_v$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_v$v.json')); print('variant $v', d['value'], d['config']['seal_ms'], d['config']['open_ms'], d['roofline']['frac'])"
done
