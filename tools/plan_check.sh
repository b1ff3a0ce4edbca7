#!/bin/bash
# parity tests, then kernel stats of a short default bench (plan + AES kernel times), then the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
mkdir -p gpurun_out/plan
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/plan/pytest.log 2>&1 || { tail -30 gpurun_out/plan/pytest.log; exit 1; }
tail -1 gpurun_out/plan/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/plan/trace -o trace -- python3 bench.py --steps 4 --warmup 1 --no-cpu > gpurun_out/plan/trace.log 2>&1 || { tail -20 gpurun_out/plan/trace.log; exit 1; }
find gpurun_out/plan/trace -name "*kernel_stats.csv" -exec cut -d, -f1-4 {} \; | cut -c1-160
timeout -k 10 300 python bench.py > gpurun_out/plan/bench.json 2> gpurun_out/plan/bench.err || { tail -20 gpurun_out/plan/bench.err; exit 1; }
cat gpurun_out/plan/bench.json
