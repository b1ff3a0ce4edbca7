#!/bin/bash
set -o pipefail
O=gpurun_out/r02e; mkdir -p $O
for s in aes128gcm chacha20poly1305; do
  for kcz in "8 1 256" "8 4 256" "16 4 256" "32 4 256" "16 8 1024" "32 8 1024" "64 16 1024"; do
    set -- $kcz
    QPP_TXQ_ZC_MAX=$3 timeout -k 10 120 python -u bench.py --mode txq --suite $s --inflight $1 --coalesce $2 --steps 40 --no-cpu > $O/txqn_${s}_$1_$2_$3.json 2>&1 || { tail -5 $O/txqn_${s}_$1_$2_$3.json; exit 1; }
    echo "txq $s inflight $1 coalesce $2 zc $3: $(python3 -c "import json;d=json.load(open('$O/txqn_${s}_$1_$2_$3.json'));print(d['value'],d['unit'],d['us_per_burst'])")"
  done
done
QPP_TXQ_ZC_MAX=1024 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof2 -o prof -- python3 bench.py --mode txq --inflight 32 --coalesce 8 --steps 10 --no-cpu > $O/prof2.log 2>&1 || exit 1
find $O/prof2 -name "*kernel_stats.csv" | head -1 | xargs cat | head -5
