# round 4 step f: validation of the current build on one box -- GPU suite, smoke, the default bench line, the rx-mode
# rocprof trace (exit status: the round-3 crash at exit), the PMC profile of the default bench command
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; o=gpurun_out/r04f; mkdir -p $o
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $o/pytest.log 2>&1; rc=$?
tail -3 $o/pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 && cat $o/smoke.log && \
timeout -k 10 300 python bench.py > $o/bench.json 2> $o/bench.err && cat $o/bench.json && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/rxtrace -o trace -- python3 bench.py --mode rx --keys 64 --steps 4 --warmup 1 --no-cpu > $o/rxtrace.log 2>&1; echo "rx trace exit $?" | tee $o/rxtrace.rc
bash tools/profile.sh r04f_prof && python tools/summarize_prof.py gpurun_out/r04f_prof > $o/prof_summary.txt && head -30 $o/prof_summary.txt && \
python tools/traffic.py gpurun_out/r04f_prof aes128gcm/1200/1 1048576 $o/traffic.json
