#!/bin/bash
# Fused receive kernel: parity tests, then the rx bench fused vs two-launch (QPP_RX_FUSED=0), 3 alternating rounds,
# AES-128 and AES-256, and a kernel trace of the fused rx bench.  usage: bash tools/rx_fused_check.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
tag=${1:-rxf}; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rx_fused.py tests/test_gpu_parity.py -k "rx or unprotect" -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1; rc=$?
tail -6 $out/pytest.log; [ $rc -eq 0 ] || exit 1
for r in 1 2 3; do
  for suite in aes128gcm aes256gcm; do
    for f in 1 0; do
      QPP_RX_FUSED=$f timeout -k 10 200 python bench.py --mode rx --suite $suite --steps 10 --warmup 3 > $out/r${r}_${suite}_f$f.json 2> $out/err.txt || { tail -5 $out/err.txt; exit 1; }
      python -c "import json; d=json.load(open('$out/r${r}_${suite}_f$f.json')); print('$r $suite fused=$f', d['value'], d['ms_per_step'])"
    done
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o trace -- python3 bench.py --mode rx --steps 5 --warmup 2 > $out/trace.log 2>&1 || { tail -20 $out/trace.log; exit 1; }
echo done
