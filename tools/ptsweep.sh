#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/ptsweep; mkdir -p $out
run() { name=$1; shift; timeout -k 10 240 python bench.py --steps 5 --warmup 2 --no-cpu "$@" > $out/$name.json 2> $out/$name.err || { echo "FAIL $name"; tail -5 $out/$name.err; return 1; }; python -c "import json;d=json.load(open('$out/$name.json'));print('$name', d['value'], d.get('unit'), d.get('ms_per_step'), d.get('roofline',{}).get('frac'))"; }
run pt1200 && run pt2400 --pt 2400 --packets 524288 && run pt4000 --pt 4000 --packets 262144 && run pt8000 --pt 8000 --packets 131072 && run pt8000x2 --pt 8000 --packets 262144 && run pt8000x4 --pt 8000 --packets 524288
