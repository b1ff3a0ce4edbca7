#!/bin/bash
# round-2 check: GPU tests (one process), then the default bench and the C5 e2e line
set -o pipefail
mkdir -p gpurun_out/r02
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/r02/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 > gpurun_out/r02/bench.json 2> gpurun_out/r02/bench.err
rc=$?
echo "bench rc=$rc"; cat gpurun_out/r02/bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --mode e2e --packets 2097152 --keys 4096 --rotate --steps 3 --no-cpu > gpurun_out/r02/e2e_c5.json 2> gpurun_out/r02/e2e_c5.err
rc=$?
echo "e2e c5 rc=$rc"; cat gpurun_out/r02/e2e_c5.json
exit $rc
