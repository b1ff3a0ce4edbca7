# round 4 step k: server without scratch spills (gmul with 8 positions in flight, round keys from LDS), ring reads past
# the caches instead of a per-flush acquire, the received tag / header bytes read up front: tests, latency, trace
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; o=gpurun_out/r04k; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_packet_server.py tests/test_gpu_txq_server.py tests/test_gpu_txq.py tests/test_gpu_txrx.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py -q -x --timeout 120 --timeout-method thread > $o/pytest.log 2>&1; rc=$?
tail -5 $o/pytest.log
[ $rc -eq 0 ] || exit 1
run() { local tag=$1; shift; timeout -k 10 120 "$@" > $o/$tag.json 2> $o/$tag.err || { echo "FAIL $tag"; tail -5 $o/$tag.err; exit 1; }; echo "$tag: $(head -c 420 $o/$tag.json)"; }
run packet_aes python bench.py --mode packet --no-cpu && \
run packet_aes256 python bench.py --mode packet --suite aes256gcm --no-cpu && \
run packet_chacha python bench.py --mode packet --suite chacha20poly1305 --no-cpu && \
run txq1_aes python bench.py --mode txq --inflight 1 --no-cpu && \
run txq1_chacha python bench.py --mode txq --suite chacha20poly1305 --inflight 1 --no-cpu && \
QPP_LIB=ab/sT.so timeout -k 10 120 python tools/diag/server_trace.py 1 1200 2>&1 | tee $o/trace_1.txt && \
QPP_LIB=ab/sT.so timeout -k 10 120 python tools/diag/server_trace.py 64 1200 2>&1 | tee $o/trace_64.txt
