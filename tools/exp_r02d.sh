#!/bin/bash
# async txq parity + sustained GSO-burst rate; FETCH/WRITE calibration of the coop chunk pattern
set -o pipefail
O=gpurun_out/r02d; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "txq" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for s in aes128gcm chacha20poly1305; do
  for k in 1 8 16; do
    timeout -k 10 120 python -u bench.py --mode txq --suite $s --inflight $k --steps 20 --no-cpu > $O/txq_${s}_$k.json 2>&1 || { tail -5 $O/txq_${s}_$k.json; exit 1; }
    echo "txq $s inflight $k: $(cat $O/txq_${s}_$k.json)"
  done
done
bash tools/ubench/run_copy_pattern.sh 2>&1 | tail -40
