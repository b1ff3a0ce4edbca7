#!/bin/bash
# Same-box receive-path A/B of library builds (QPP_LIB), ROUNDS alternating rounds, over the rx configurations given.
# usage: LIBS="ab/a.so s2n-quic_amd/libqpp.so" CFGS="1 64" bash tools/rx_ab2.sh <tag>   (CFGS: key counts, AES-128)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
tag=${1:-rxab}; out=gpurun_out/$tag; mkdir -p $out
for r in $(seq 1 ${ROUNDS:-3}); do
  for k in ${CFGS:-1 64}; do
    for lib in $LIBS; do
      nm=$(basename $lib .so)
      QPP_LIB=$PWD/$lib timeout -k 10 200 python bench.py --mode rx --keys $k --steps 10 --warmup 3 --no-cpu > $out/r${r}_k${k}_$nm.json 2> $out/err.txt || { tail -5 $out/err.txt; exit 1; }
      python -c "import json; d=json.load(open('$out/r${r}_k${k}_$nm.json')); print('$r k$k $nm', d['value'], d['ms_per_step'])"
    done
  done
done
