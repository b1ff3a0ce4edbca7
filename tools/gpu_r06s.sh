# payload alignment vs store cost (same library; ABL=2 = no interior stores), 3 alternating rounds
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
o=gpurun_out/r06s; mkdir -p $o
for r in 1 2 3; do
  for cfg in "a21:--aad 21" "a32:--aad 32" "a64:--aad 64 --stride 1280" "a128:--aad 128 --stride 1408"; do
    n=${cfg%%:*}; args=${cfg#*:}
    for lib in s2n-quic_amd/libqpp.so ab/abl2.so; do
      b=$(basename $lib .so)
      QPP_LIB=$PWD/$lib timeout -k 10 120 python bench.py --no-cpu --no-check --steps 6 --warmup 2 $args > $o/r${r}_${n}_$b.json 2> $o/err.txt || { tail -5 $o/err.txt; exit 1; }
      python3 -c "import json; d=json.load(open('$o/r${r}_${n}_$b.json')); print('$r $n $b', d['config']['seal_ms'], d['config']['open_ms'])"
    done
  done
done
