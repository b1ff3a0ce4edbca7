# the fused receive kernel with 64 keys: parity, phase times (QPP_RX_TRACE build), rate vs the previous build (ab/base)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; o=gpurun_out/r03rx3; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_rx_fused.py tests/test_gpu_parity.py -k "rx or unprotect or receive or fused" -x -q --timeout 200 --timeout-method thread > $o/pytest.log 2>&1; tail -2 $o/pytest.log; grep -q " passed" $o/pytest.log && ! grep -q "failed" $o/pytest.log || exit 1
QPP_LIB=$PWD/ab/rxT.so timeout -k 10 120 python3 bench.py --mode rx --keys 64 --steps 2 --warmup 1 --no-cpu > $o/rx_trace.txt 2>&1; tail -4 $o/rx_trace.txt
for r in 1 2; do for lib in s2n-quic_amd/libqpp.so ab/base.so; do
QPP_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --mode rx --keys 64 --no-cpu > $o/rx_$(basename $lib .so)_$r.json 2>$o/err.txt || { tail -3 $o/err.txt; exit 1; }; echo "$lib $(cat $o/rx_$(basename $lib .so)_$r.json)"; done; done
