# A/B: the next interior group's first 1 / 2 payload blocks loaded at the end of the current group
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
QPP_LIB=$PWD/ab/pf2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pf2_pytest.log 2>&1; tail -1 gpurun_out/pf2_pytest.log; grep -q " passed" gpurun_out/pf2_pytest.log && ! grep -q "failed" gpurun_out/pf2_pytest.log || exit 1
CFGS="ab/base.so:0 ab/pf1.so:0 ab/pf2.so:0" ROUNDS=3 bash tools/ab.sh r03pf
