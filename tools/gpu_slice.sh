set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lifetime.py tests/test_gpu_c5.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/slice_tests.log 2>&1; rc=$?
tail -3 gpurun_out/slice_tests.log; [ $rc -eq 0 ] || exit 1
ROUNDS=2 STEPS=8 CFGS="ab/base.so:0 ab/slice.so:0" bash tools/ab.sh s1 | grep median || exit 1
ROUNDS=2 STEPS=8 CFGS="ab/base.so:0 ab/slice.so:0" BENCH_ARGS="--keys 64" bash tools/ab.sh s64 | grep median || exit 1
ROUNDS=2 STEPS=8 CFGS="ab/base.so:0 ab/slice.so:0" BENCH_ARGS="--suite aes256gcm --keys 64" bash tools/ab.sh s256 | grep median || exit 1
ROUNDS=2 STEPS=8 CFGS="ab/base.so:0 ab/slice.so:0" BENCH_ARGS="--pt 8000 --packets 131072" bash tools/ab.sh s8k | grep median
