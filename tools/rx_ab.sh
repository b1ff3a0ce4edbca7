#!/bin/bash
# RX parity tests on the in-tree build, then the rx bench A/B of two libraries (QPP_LIB), 3 alternating rounds, for
# AES-128-GCM 64 keys and ChaCha20-Poly1305 64 keys.  usage: A=<so> B=<so> bash tools/rx_ab.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
tag=${1:-rxab}; out=gpurun_out/$tag; mkdir -p $out
[ -n "$A" ] && [ -n "$B" ] || { echo "set A and B to two library paths"; exit 2; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_rx_fused.py tests/test_gpu_parity.py -k "rx or unprotect" -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1; rc=$?
tail -2 $out/pytest.log; [ $rc -eq 0 ] || exit 1
for r in 1 2 3; do
  for suite in aes128gcm chacha20poly1305; do
    for lib in $A $B; do
      nm=$(basename $lib .so)
      QPP_LIB=$PWD/$lib timeout -k 10 200 python bench.py --mode rx --suite $suite --keys 64 --steps 8 --warmup 3 > $out/r${r}_${suite}_$nm.json 2> $out/err.txt || { tail -5 $out/err.txt; exit 1; }
      python -c "import json; d=json.load(open('$out/r${r}_${suite}_$nm.json')); print('$r $suite $nm', d['value'], d['ms_per_step'])"
    done
  done
done
