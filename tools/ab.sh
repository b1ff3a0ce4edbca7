#!/bin/bash
# Same-box A/B: alternate benches of library builds (QPP_LIB) and AES variants (QPP_AES_VARIANT), 3 rounds.
# usage: CFGS="ab/a.so:0 ab/b.so:0 s2n-quic_amd/libqpp.so:1" [BENCH_ARGS="--suite aes256gcm --keys 64"] bash tools/ab.sh tag
#   CFGS: space-separated <library path>:<variant index> pairs; BENCH_ARGS: extra bench.py arguments
set -o pipefail
[ -n "$CFGS" ] || { echo "CFGS is empty: nothing to compare (see the usage line)"; exit 2; }
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tag=${1:-ab}; mkdir -p gpurun_out/$tag
for round in 1 2 3; do
  for cfg in $CFGS; do
    lib=${cfg%%:*}; var=${cfg##*:}
    QPP_LIB=$PWD/$lib QPP_AES_VARIANT=$var timeout -k 10 200 python bench.py --steps 6 --warmup 2 --no-cpu $BENCH_ARGS > gpurun_out/$tag/r${round}_$(basename $lib .so)_$var.json 2>gpurun_out/$tag/err.txt || { echo "fail $cfg"; tail -5 gpurun_out/$tag/err.txt; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/$tag/r${round}_$(basename $lib .so)_$var.json')); print('$round $cfg', d['value'], d['config']['seal_ms'], d['config']['open_ms'])"
  done
done
