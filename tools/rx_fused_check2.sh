#!/bin/bash
# Full GPU suite, then the receive bench fused vs two-launch (QPP_RX_FUSED=0) for ChaCha20-Poly1305 64 keys and
# AES-128-GCM 1 key, 3 alternating rounds.  usage: bash tools/rx_fused_check2.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
tag=${1:-rxf2}; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?
tail -3 $out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
for r in 1 2 3; do
  for cfg in "chacha20poly1305 64" "aes128gcm 1"; do
    set -- $cfg
    for f in 1 0; do
      QPP_RX_FUSED=$f timeout -k 10 200 python bench.py --mode rx --suite $1 --keys $2 --steps 8 --warmup 3 > $out/r${r}_$1_f$f.json 2> $out/err.txt || { tail -5 $out/err.txt; exit 1; }
      python -c "import json; d=json.load(open('$out/r${r}_$1_f$f.json')); print('$r $1 fused=$f', d['value'], d['ms_per_step'])"
    done
  done
done
