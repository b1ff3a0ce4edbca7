# round 4 step q: the final build -- GPU suite, smoke, the default bench line, the rx-mode rocprof trace (exit status),
# the rocprof kernel trace + PMC passes of the default bench command (tools/profile.sh), traffic, the latency faces
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; o=gpurun_out/r04q; mkdir -p $o
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $o/pytest.log 2>&1; rc=$?
tail -3 $o/pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 && cat $o/smoke.log && \
timeout -k 10 300 python bench.py > $o/bench.json 2> $o/bench.err && head -c 600 $o/bench.json && echo && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/rxtrace -o trace -- python3 bench.py --mode rx --keys 64 --steps 4 --warmup 1 --no-cpu > $o/rxtrace.log 2>&1; echo "rx trace exit $?" | tee $o/rxtrace.rc
bash tools/profile.sh r04q_prof && python tools/summarize_prof.py gpurun_out/r04q_prof > $o/prof_summary.txt && head -12 $o/prof_summary.txt && \
python tools/traffic.py gpurun_out/r04q_prof aes128gcm/1200/1 1048576 $o/traffic.json || exit 1
run() { local tag=$1; shift; timeout -k 10 120 "$@" > $o/$tag.json 2> $o/$tag.err || { echo "FAIL $tag"; tail -5 $o/$tag.err; exit 1; }; echo "$tag: $(head -c 250 $o/$tag.json)"; }
run packet_aes python bench.py --mode packet --no-cpu && \
run packet_chacha python bench.py --mode packet --suite chacha20poly1305 --no-cpu && \
run txq1_aes python bench.py --mode txq --inflight 1 --no-cpu && \
run txq1_chacha python bench.py --mode txq --suite chacha20poly1305 --inflight 1 --no-cpu
