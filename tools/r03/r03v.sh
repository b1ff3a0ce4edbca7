# round-3 validation + txq latency + I/O-vs-compute A/B of the quad kernel
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
bash tools/validate.sh && \
timeout -k 10 120 python bench.py --mode txq --inflight 1 --no-cpu > gpurun_out/txq_server.json 2> gpurun_out/txq_server.err && cat gpurun_out/txq_server.json && \
timeout -k 10 120 python bench.py --mode txq --inflight 1 --txq-launch --no-cpu > gpurun_out/txq_launch.json 2> gpurun_out/txq_launch.err && cat gpurun_out/txq_launch.json && \
CFGS="ab/base.so:0 ab/noio.so:0 ab/nocrypto.so:0" ROUNDS=2 BENCH_ARGS="--no-check" bash tools/ab.sh r03io
