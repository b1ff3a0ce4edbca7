#!/bin/bash
# Same-box comparison of 1 key vs 64 keys (a mixed-key batch within 10 % of the single-key rate),
# AES-128-GCM and AES-256-GCM, 1 Mi x 1200 B, alternating, ROUNDS rounds.  Lines -> gpurun_out/<tag>/lines.jsonl
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=${1:-keys_vs_single}; mkdir -p gpurun_out/$tag
ROUNDS=${ROUNDS:-3}
for round in $(seq 1 $ROUNDS); do
  for suite in aes128gcm aes256gcm; do
    for keys in 1 64; do
      timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --suite $suite --keys $keys \
        > gpurun_out/$tag/r${round}_${suite}_${keys}.json 2> gpurun_out/$tag/err.txt || { echo "fail $suite $keys"; tail -5 gpurun_out/$tag/err.txt; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/$tag/r${round}_${suite}_${keys}.json')); d['tag']='$suite keys=$keys round $round'; print(json.dumps(d))" >> gpurun_out/$tag/lines.jsonl
      tail -1 gpurun_out/$tag/lines.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['tag'], d['value'], d['config']['seal_ms'], d['config']['open_ms'])"
    done
  done
done
python - "$tag" <<'PY'
import json, statistics, sys, collections
t = sys.argv[1]
by = collections.defaultdict(list)
for l in open(f"gpurun_out/{t}/lines.jsonl"):
    d = json.loads(l)
    by[d["tag"].rsplit(" round", 1)[0]].append(d["value"])
med = {k: statistics.median(v) for k, v in by.items()}
for k, v in sorted(med.items()):
    print(f"median {k}: {v:.1f} GiB/s (n={len(by[k])})")
for s in ("aes128gcm", "aes256gcm"):
    print(f"{s}: 64 keys / 1 key = {med[s + ' keys=64'] / med[s + ' keys=1']:.3f}")
PY
