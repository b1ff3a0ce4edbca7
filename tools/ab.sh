#!/bin/bash
# Same-box A/B: alternate benches of library builds (QPP_LIB), ROUNDS rounds (default 3).
# usage: CFGS="ab/a.so:0 ab/b.so:0 s2n-quic_amd/libqpp.so:1" [BENCH_ARGS="--suite aes256gcm --keys 64"] bash tools/ab.sh tag
#   CFGS: space-separated <library path>:<label> pairs; BENCH_ARGS: extra bench.py arguments
set -o pipefail
[ -n "$CFGS" ] || { echo "CFGS is empty: nothing to compare (see the usage line)"; exit 2; }
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tag=${1:-ab}; mkdir -p gpurun_out/$tag
ROUNDS=${ROUNDS:-3}; STEPS=${STEPS:-6}
for round in $(seq 1 $ROUNDS); do
  for cfg in $CFGS; do
    lib=${cfg%%:*}; var=${cfg##*:}
    QPP_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps $STEPS --warmup 2 --no-cpu $BENCH_ARGS > gpurun_out/$tag/r${round}_$(basename $lib .so)_$var.json 2>gpurun_out/$tag/err.txt || { echo "fail $cfg"; tail -5 gpurun_out/$tag/err.txt; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/$tag/r${round}_$(basename $lib .so)_$var.json')); print('$round $cfg', d['value'], d['config']['seal_ms'], d['config']['open_ms'])"
  done
done
python - "$tag" <<'PY'
import glob, json, statistics, sys, collections
t = sys.argv[1]
by = collections.defaultdict(list)
for f in glob.glob(f"gpurun_out/{t}/r*_*.json"):
    d = json.load(open(f))
    by[f.split("/")[-1].split("_", 1)[1][:-5]].append(d["config"]["seal_ms"])
for k, v in sorted(by.items()):
    print(f"median seal_ms {k}: {statistics.median(v):.4f}  min {min(v):.4f}  (n={len(v)})")
PY
