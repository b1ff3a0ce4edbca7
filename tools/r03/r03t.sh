# txq latency after the deferred telemetry store; per-packet latency vs the previous build (ab/prev); GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; o=gpurun_out/r03t2; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest.log 2>&1; tail -2 $o/pytest.log; grep -q " passed" $o/pytest.log && ! grep -q "failed" $o/pytest.log || exit 1
for r in 1 2; do
for lib in s2n-quic_amd/libqpp.so ab/prev.so; do
  b=$(basename $lib .so)
  QPP_LIB=$PWD/$lib timeout -k 10 120 python bench.py --mode txq --inflight 1 --no-cpu > $o/txq1_${b}_$r.json 2>$o/err.txt || { tail -5 $o/err.txt; exit 1; }
  QPP_LIB=$PWD/$lib timeout -k 10 120 python bench.py --mode packet --no-cpu > $o/packet_${b}_$r.json 2>$o/err.txt || { tail -5 $o/err.txt; exit 1; }
  echo "$lib txq1 $(python -c "import json;d=json.load(open('$o/txq1_${b}_$r.json'));print(d['value'],d['p10_us'],d['p90_us'])") packet $(python -c "import json;d=json.load(open('$o/packet_${b}_$r.json'));print(d['value'],d['decrypt_us'])")"
done; done
QPP_LIB=$PWD/ab/sT2.so timeout -k 10 120 python tools/diag/server_trace.py > $o/server_trace.txt 2>&1; cat $o/server_trace.txt
