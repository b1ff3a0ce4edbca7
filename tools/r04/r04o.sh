# round 4 step o: the quad-split ChaCha20 header-protection block: ChaCha tests, then the ChaCha latency faces
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; o=gpurun_out/r04o; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_packet_server.py tests/test_gpu_txq_server.py tests/test_gpu_txq.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py -q -x --timeout 120 --timeout-method thread > $o/pytest.log 2>&1; rc=$?
tail -3 $o/pytest.log
[ $rc -eq 0 ] || exit 1
run() { local tag=$1; shift; timeout -k 10 120 "$@" > $o/$tag.json 2> $o/$tag.err || { echo "FAIL $tag"; tail -5 $o/$tag.err; exit 1; }; echo "$tag: $(head -c 330 $o/$tag.json)"; }
run txq1_chacha python bench.py --mode txq --suite chacha20poly1305 --inflight 1 --no-cpu && \
run txq1_aes python bench.py --mode txq --inflight 1 --no-cpu && \
run packet_chacha python bench.py --mode packet --suite chacha20poly1305 --no-cpu && \
run c3_chacha_64 python bench.py --suite chacha20poly1305 --keys 64 --no-cpu
