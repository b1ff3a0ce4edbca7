# round 4 step i: the packet server -- its tests and the per-packet tests that now run through it, then the
# per-packet latency (server vs launch per call, every suite)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; o=gpurun_out/r04i; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_packet_server.py tests/test_gpu_parity.py tests/test_gpu_fips.py tests/test_gpu_lifetime.py tests/test_gpu_txq_server.py tests/test_gpu_txrx.py -q -x --timeout 120 --timeout-method thread > $o/pytest.log 2>&1; rc=$?
tail -15 $o/pytest.log
[ $rc -eq 0 ] || exit 1
run() { local tag=$1; shift; timeout -k 10 120 "$@" > $o/$tag.json 2> $o/$tag.err || { echo "FAIL $tag"; tail -5 $o/$tag.err; exit 1; }; echo "$tag: $(cat $o/$tag.json)"; }
run packet_aes python bench.py --mode packet --no-cpu && \
run packet_aes256 python bench.py --mode packet --suite aes256gcm --no-cpu && \
run packet_chacha python bench.py --mode packet --suite chacha20poly1305 --no-cpu && \
run packet_aes_launch python bench.py --mode packet --no-server --no-cpu
