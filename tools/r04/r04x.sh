# round 4 step x: the wave-per-packet AES runs the last pass of an odd count as one chain (not a pair with a discarded
# chain): tests, then small-packet batches same-box against the previous build (ab/pre_single.so), and txq flushes
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; o=gpurun_out/r04x; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_txq_server.py tests/test_gpu_txq.py tests/test_gpu_packet_server.py tests/test_gpu_fuzz.py -q -x --timeout 120 --timeout-method thread > $o/pytest.log 2>&1; rc=$?
tail -3 $o/pytest.log
[ $rc -eq 0 ] || exit 1
CFGS="s2n-quic_amd/libqpp.so:new ab/pre_single.so:pre" BENCH_ARGS="--packets 4096 --pt 300" ROUNDS=3 bash tools/ab.sh r04x_300 && \
CFGS="s2n-quic_amd/libqpp.so:new ab/pre_single.so:pre" BENCH_ARGS="--packets 4096 --pt 1452" ROUNDS=3 bash tools/ab.sh r04x_1452 || exit 1
for pt in 300 1200 1452; do
  timeout -k 10 120 python bench.py --mode txq --inflight 1 --pt $pt --no-cpu > $o/txq1_$pt.json 2>$o/txq1_$pt.err || exit 1
  echo "txq1 $pt: $(python -c "import json; print(json.load(open('$o/txq1_$pt.json'))['value'])")"
done
