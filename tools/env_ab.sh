#!/bin/bash
# Same-box latency A/B of one library under two environments: per-packet qpp_seal / open / mask (packet server), one
# 64 x 1200 B txq flush (persistent server); ROUNDS alternating rounds.
# usage: ENVS="QPP_X=0 QPP_X=1" bash tools/env_ab.sh tag
cd $GRAFT_REPO_ROOT
tag=${1:-envab}; mkdir -p gpurun_out/$tag
for round in $(seq 1 ${ROUNDS:-2}); do
  for e in $ENVS; do
    for m in "packet|--mode packet" "packetcc|--mode packet --suite chacha20poly1305" "txq|--mode txq --inflight 1"; do
      name=${m%%|*}; args=${m#*|}
      env $e timeout -k 10 120 python bench.py $args --no-cpu > gpurun_out/$tag/r${round}_${e}_$name.json 2> gpurun_out/$tag/err.txt || { echo "fail $e $name"; tail -5 gpurun_out/$tag/err.txt; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/$tag/r${round}_${e}_$name.json').read().strip().splitlines()[-1]); print('$round $e $name', d['value'], d['unit'], d.get('decrypt_us',''), d.get('hp_mask_us',''))"
    done
  done
done
