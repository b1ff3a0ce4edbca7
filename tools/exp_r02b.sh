#!/bin/bash
# round-2 experiment B: wave-item kernel for many keys: parity, then lane vs wave on the many-key configs
set -o pipefail
O=gpurun_out/r02b; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
B="timeout -k 10 200 python -u bench.py --no-cpu --steps 10"
j() { python3 -c "import json;d=json.load(open('$1'));c=d['config'];print(d['value'],c.get('seal_ms'),c.get('open_ms'),d['ms_per_step'])"; }
$B > $O/c2.json && echo "c2 auto: $(j $O/c2.json)"
for k in lane wave; do
  QPP_AES_KERNEL=$k $B --keys 64 > $O/k64_$k.json && echo "keys64 $k: $(j $O/k64_$k.json)"
  QPP_AES_KERNEL=$k $B --keys 64 --key-run 64 > $O/k64r64_$k.json && echo "keys64 run64 $k: $(j $O/k64r64_$k.json)"
  QPP_AES_KERNEL=$k $B --keys 4096 --packets 2097152 > $O/k4096_$k.json && echo "keys4096 2Mi $k: $(j $O/k4096_$k.json)"
  QPP_AES_KERNEL=$k $B --keys 64 --suite aes256gcm > $O/k64_256_$k.json && echo "aes256 keys64 $k: $(j $O/k64_256_$k.json)"
done
$B --suite aes256gcm > $O/c2_256.json && echo "aes256 1 key: $(j $O/c2_256.json)"
for pipe in 65536,96,4 262144,384,4 524288,768,4; do
  timeout -k 10 300 python -u bench.py --mode e2e --packets 2097152 --keys 4096 --rotate --steps 3 --pipe $pipe > $O/e2e_$pipe.json 2>&1 || exit 1
  echo "e2e c5 pipe $pipe: $(j $O/e2e_$pipe.json)"
done
