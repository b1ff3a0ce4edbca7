#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration of the coop 64-B chunk pattern (tools/ubench/copy_pattern.hip): one PMC pass per
# counter, as MI355X_MICROARCH.md prescribes; summary -> gpurun_out/copycal/summary.json
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/copycal; mkdir -p $O
for m in 0 1 2 3 4; do
  timeout -k 10 60 tools/ubench/copy_pattern $m > $O/time_$m.json || exit 1
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d $O/m${m}_$c -o pmc -- tools/ubench/copy_pattern $m 1048576 3 > $O/m${m}_$c.log 2>&1 || { echo "pmc $m $c failed"; tail -5 $O/m${m}_$c.log; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob, json
out = {}
for m in (0, 1, 2, 3, 4):
    t = json.load(open(f"gpurun_out/copycal/time_{m}.json"))
    row = dict(t)
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        vals = [float(r["Counter_Value"]) for f in glob.glob(f"gpurun_out/copycal/m{m}_{c}/**/*counter_collection.csv", recursive=True)
                for r in csv.DictReader(open(f)) if r["Counter_Name"] == c]
        row[c.lower() + "_gb_per_launch"] = round(sum(vals) / len(vals) * 1024 / 1e9, 4) if vals else None
    row["fetch_per_alg"] = round(row["fetch_size_gb_per_launch"] / t["alg_read_gb"], 3)
    row["write_per_alg"] = round(row["write_size_gb_per_launch"] / t["alg_write_gb"], 3)
    out[{0: "coop_unaligned", 1: "coop_aligned", 2: "stream_16B_per_lane", 3: "coop_unaligned_nt", 4: "coop_unaligned_read"}[m]] = row
json.dump(out, open("gpurun_out/copycal/summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
