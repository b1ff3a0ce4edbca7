#!/bin/bash
# BASELINE configs[3]: AES-128-GCM seal + HP, GSO-style 64-packet bursts through qpp_txq, payload sweep
set -o pipefail
O=gpurun_out/c4; mkdir -p $O
for pt in 300 1200 1452 8000; do
  timeout -k 10 120 python -u bench.py --mode txq --pt $pt --steps 40 --no-cpu > $O/lat_$pt.json 2>&1 || { tail -5 $O/lat_$pt.json; exit 1; }
  timeout -k 10 120 python -u bench.py --mode txq --pt $pt --inflight 32 --coalesce 8 --steps 40 --no-cpu > $O/rate_$pt.json 2>&1 || { tail -5 $O/rate_$pt.json; exit 1; }
  echo "pt $pt: latency $(python3 -c "import json;d=json.load(open('$O/lat_$pt.json'));print(d['value'],d['unit'])") sustained $(python3 -c "import json;d=json.load(open('$O/rate_$pt.json'));print(d['value'],d['unit'],d['us_per_burst'])")"
done
