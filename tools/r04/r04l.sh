# round 4 step l: the whole GPU suite, smoke and the default bench line on the current build, then the latency faces
# (per-packet seal/open through the packet server, txq flushes) and the server's phase trace
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; o=gpurun_out/r04l; mkdir -p $o
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $o/pytest.log 2>&1; rc=$?
tail -3 $o/pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 && cat $o/smoke.log && \
timeout -k 10 300 python bench.py > $o/bench.json 2> $o/bench.err && head -c 700 $o/bench.json && echo || exit 1
run() { local tag=$1; shift; timeout -k 10 120 "$@" > $o/$tag.json 2> $o/$tag.err || { echo "FAIL $tag"; tail -5 $o/$tag.err; exit 1; }; echo "$tag: $(head -c 300 $o/$tag.json)"; }
run packet_aes python bench.py --mode packet --no-cpu && \
run packet_aes256 python bench.py --mode packet --suite aes256gcm --no-cpu && \
run packet_chacha python bench.py --mode packet --suite chacha20poly1305 --no-cpu && \
run txq1_aes python bench.py --mode txq --inflight 1 --no-cpu && \
run txq1_chacha python bench.py --mode txq --suite chacha20poly1305 --inflight 1 --no-cpu && \
QPP_LIB=ab/sT.so timeout -k 10 120 python tools/diag/server_trace.py 1 1200 2>&1 | tee $o/trace_1.txt
