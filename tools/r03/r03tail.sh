# the quad kernel's last group with 1..4 blocks per lane (ab/tail = libqpp) vs 3..4 (ab/base): parity, then A/B
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tail_pytest.log 2>&1; tail -1 gpurun_out/tail_pytest.log; grep -q " passed" gpurun_out/tail_pytest.log && ! grep -q "failed" gpurun_out/tail_pytest.log || exit 1
CFGS="ab/base.so:0 ab/tail.so:0" ROUNDS=2 BENCH_ARGS="--pt 300 --packets 4194304" bash tools/ab.sh r03tail300 && \
CFGS="ab/base.so:0 ab/tail.so:0" ROUNDS=2 BENCH_ARGS="--pt 600 --packets 2097152" bash tools/ab.sh r03tail600 && \
CFGS="ab/base.so:0 ab/tail.so:0" ROUNDS=2 bash tools/ab.sh r03tail1200 && \
CFGS="ab/base.so:0 ab/tail.so:0" ROUNDS=2 BENCH_ARGS="--suite aes256gcm --keys 64" bash tools/ab.sh r03tail256
