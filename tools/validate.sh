#!/bin/bash
# Round-end style validation on one GPU box: parity tests, smoke(), default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/val_pytest.log 2>&1 || { tail -30 gpurun_out/val_pytest.log; exit 1; }
tail -2 gpurun_out/val_pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/val_smoke.log 2>&1 || { tail -20 gpurun_out/val_smoke.log; exit 1; }
cat gpurun_out/val_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/val_bench.json 2> gpurun_out/val_bench.err || { tail -20 gpurun_out/val_bench.err; exit 1; }
cat gpurun_out/val_bench.json
