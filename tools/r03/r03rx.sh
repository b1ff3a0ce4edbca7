# fused receive with the header rewrite deferred to the open phase (ab/rxdefer = libqpp) vs the previous (ab/base)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; o=gpurun_out/r03rx4; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_rx_fused.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py -k "rx or unprotect or receive or fused or random" -x -q --timeout 200 --timeout-method thread > $o/pytest.log 2>&1; tail -2 $o/pytest.log; grep -q " passed" $o/pytest.log && ! grep -q "failed" $o/pytest.log || exit 1
for r in 1 2; do for lib in ab/rxdefer.so ab/base.so; do
QPP_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --mode rx --keys 64 --no-cpu > $o/rx_$(basename $lib .so)_$r.json 2>$o/err.txt || { tail -3 $o/err.txt; exit 1; }; echo "$lib $(python3 -c "import json;print(json.load(open('$o/rx_$(basename $lib .so)_$r.json'))['value'])")"; done; done
