#!/bin/bash
# lifetime GPU tests alone (optionally against another build: QPP_LIB=ab/x.so bash tools/gpu_lifetime.sh tag)
set -o pipefail
O=gpurun_out/lt_${1:-cur}; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_lifetime.py -x -v --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -12 $O/pytest.log; exit $rc
