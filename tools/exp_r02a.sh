#!/bin/bash
# round-2 experiment A: batched key retirement (lifetime tests), mixed-key locality (random keys vs key runs),
# e2e C5 chunk sizes
set -o pipefail
O=gpurun_out/r02a; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_lifetime.py tests/test_gpu_c5.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
B="timeout -k 10 200 python -u bench.py --no-cpu --steps 10"
for kr in 1 64 1024; do
  $B --keys 64 --key-run $kr > $O/k64_run$kr.json 2>&1 || exit 1
  echo "keys64 run$kr: $(python3 -c "import json,sys;d=json.load(open('$O/k64_run$kr.json'));print(d['value'],d['config']['seal_ms'],d['config']['open_ms'])")"
done
$B --keys 4096 --packets 2097152 > $O/k4096.json 2>&1 || exit 1
echo "keys4096 2Mi: $(python3 -c "import json;d=json.load(open('$O/k4096.json'));print(d['value'],d['config']['seal_ms'])")"
for pipe in 65536,96,4 131072,192,4 524288,768,4 2097152,2600,2; do
  timeout -k 10 300 python -u bench.py --mode e2e --packets 2097152 --keys 4096 --rotate --steps 3 --pipe $pipe > $O/e2e_$pipe.json 2>&1 || exit 1
  echo "e2e c5 pipe $pipe: $(python3 -c "import json;d=json.load(open('$O/e2e_$pipe.json'));print(d['value'],d['ms_per_step'])")"
done
