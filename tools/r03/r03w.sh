set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 120 python -u tools/diag/server_mismatch.py > gpurun_out/mis_server.txt 2>&1 && tail -3 gpurun_out/mis_server.txt && \
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/val_pytest.log 2>&1; tail -3 gpurun_out/val_pytest.log; \
timeout -k 10 120 python bench.py --mode txq --inflight 1 --no-cpu > gpurun_out/txq_server.json 2> gpurun_out/txq_server.err && cat gpurun_out/txq_server.json && \
timeout -k 10 120 python bench.py --mode txq --inflight 1 --txq-launch --no-cpu > gpurun_out/txq_launch.json 2> gpurun_out/txq_launch.err && cat gpurun_out/txq_launch.json && \
CFGS="ab/base.so:0 ab/noio.so:0 ab/nocrypto.so:0" ROUNDS=2 BENCH_ARGS="--no-check" bash tools/ab.sh r03io
