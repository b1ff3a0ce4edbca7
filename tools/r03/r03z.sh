# end-of-session validation: GPU suite, smoke, the default bench line, and the rocprof trace + PMC of the same
# bench command on the same box (kernel time per step vs ms_per_step), traffic per launch
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; o=gpurun_out/${R03Z_TAG:-r03z}; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $o/pytest.log 2>&1; tail -2 $o/pytest.log; grep -q " passed" $o/pytest.log && ! grep -q "failed\|error" $o/pytest.log || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 && cat $o/smoke.log && \
timeout -k 10 300 python bench.py > $o/bench.json 2> $o/bench.err && cat $o/bench.json && \
bash tools/profile.sh ${R03Z_TAG:-r03z}_prof && python tools/summarize_prof.py gpurun_out/${R03Z_TAG:-r03z}_prof > $o/prof_summary.txt && head -4 $o/prof_summary.txt && \
python tools/traffic.py gpurun_out/${R03Z_TAG:-r03z}_prof aes128gcm/1200/1 1048576 $o/traffic.json
