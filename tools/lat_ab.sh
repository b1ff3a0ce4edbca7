#!/bin/bash
# Same-box latency A/B of library builds: per-packet qpp_seal (packet server), one 64 x 1200 B txq flush (persistent
# server), a 4096-packet batch (wave-per-packet burst kernel); ROUNDS alternating rounds.
# usage: LIBS="ab/a.so s2n-quic_amd/libqpp.so" bash tools/lat_ab.sh tag
cd $GRAFT_REPO_ROOT
tag=${1:-latab}; mkdir -p gpurun_out/$tag
for round in $(seq 1 ${ROUNDS:-2}); do
  for lib in $LIBS; do
    n=$(basename $lib .so)
    for m in "packet|--mode packet" "txq|--mode txq --inflight 1" "b4k|--packets 4096 --steps 50"; do
      name=${m%%|*}; args=${m#*|}
      QPP_LIB=$PWD/$lib timeout -k 10 120 python bench.py $args --no-cpu > gpurun_out/$tag/r${round}_${n}_$name.json 2> gpurun_out/$tag/err.txt || { echo "fail $n $name"; tail -5 gpurun_out/$tag/err.txt; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/$tag/r${round}_${n}_$name.json').read().strip().splitlines()[-1]); c=d.get('config',{}); print('$round $n $name', d['value'], d['unit'], c.get('seal_ms',''), d.get('decrypt_us',''), d.get('hp_mask_us',''))"
    done
  done
done
