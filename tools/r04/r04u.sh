# round 4 step u: HEAD at the end of the session -- GPU suite, smoke, default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; o=gpurun_out/r04u; mkdir -p $o
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $o/pytest.log 2>&1; rc=$?
tail -3 $o/pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 && cat $o/smoke.log && \
timeout -k 10 300 python bench.py > $o/bench.json 2> $o/bench.err && head -c 400 $o/bench.json && echo
