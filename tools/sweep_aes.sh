#!/bin/bash
# Parity tests, then the bench for every AES kernel variant (QPP_AES_VARIANT), one process each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tag=${1:-sweep}
mkdir -p gpurun_out/$tag
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/$tag/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/$tag/pytest.log
[ $rc -eq 0 ] || exit $rc
for v in ${VARIANTS:-0 1 2 3 4 5}; do
  QPP_AES_VARIANT=$v timeout -k 10 200 python bench.py --steps 6 --warmup 2 --no-cpu > gpurun_out/$tag/bench_v$v.json 2> gpurun_out/$tag/bench_v$v.err || { echo "variant $v failed"; tail -5 gpurun_out/$tag/bench_v$v.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/$tag/bench_v$v.json')); print('variant $v', d['value'], 'GiB/s', d['config']['seal_ms'], d['config']['open_ms'], d['roofline']['frac'])"
done
