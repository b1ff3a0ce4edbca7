#!/bin/bash
# Same-box A/B: alternate benches of two library builds (QPP_LIB) and variants; usage: A=<so> B=<so> bash tools/ab.sh tag
set -o pipefail
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
