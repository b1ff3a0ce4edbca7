#!/bin/bash
# Latency A/B of two engine builds: each run installs the build as s2n-quic_amd/libqpp.so (the native txq driver links
# it by path), then times a 64-packet txq flush (1 in flight) and the one-packet qpp_seal, 3 alternating rounds.
# usage: A=<so> B=<so> bash tools/lat_ab.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
tag=${1:-latab}; out=gpurun_out/$tag; mkdir -p $out
[ -n "$A" ] && [ -n "$B" ] || { echo "set A and B"; exit 2; }
cp s2n-quic_amd/libqpp.so $out/orig.so
for r in 1 2 3; do
  for lib in $A $B; do
    nm=$(basename $lib .so); cp $lib s2n-quic_amd/libqpp.so
    for mode in txq packet; do
      timeout -k 10 200 python bench.py --mode $mode --steps 200 --warmup 20 --no-cpu > $out/r${r}_${mode}_$nm.json 2> $out/err.txt || { tail -5 $out/err.txt; cp $out/orig.so s2n-quic_amd/libqpp.so; exit 1; }
      python -c "import json; d=json.load(open('$out/r${r}_${mode}_$nm.json')); print('$r $mode $nm', d['value'], d['unit'])"
    done
  done
done
cp $out/orig.so s2n-quic_amd/libqpp.so
