# Round-end validation on one GPU: full GPU test suite, smoke, rocprof trace + PMC passes of the default workload,
# the default bench line (as the driver runs it).  usage: bash tools/round_final.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
tag=${1:-final}; mkdir -p gpurun_out/$tag
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$tag/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/$tag/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$tag/smoke.log 2>&1 || { tail -5 gpurun_out/$tag/smoke.log; exit 1; }
tail -1 gpurun_out/$tag/smoke.log
bash tools/profile.sh ${tag}_prof || exit 1
timeout -k 10 300 python bench.py > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err || { tail -5 gpurun_out/$tag/bench.err; exit 1; }
cat gpurun_out/$tag/bench.json
