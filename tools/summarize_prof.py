"""Summarise a tools/profile.sh output directory: per-kernel average duration (kernel trace) and the PMC
counters averaged per dispatch of each kernel.  Beside rocprof's average over every launch, the median and the mean
over the LAST `--timed N` launches (default 20: the bench's timed steps come last; the average includes the cold
warm-up launches) are computed from the per-dispatch trace."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d, timed=20):
    rows = []
    for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    print("== kernel stats (%s)" % d)
    for r in rows:
        print("  %-70s calls=%-4s avg_us=%.1f total_pct=%s" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3,
                                                               r.get("Percentage", "")))
    durs = defaultdict(list)
    for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            durs[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    for k, v in durs.items():
        if len(v) < 2 or not any(s in k for s in ("aes_gcm", "chacha")):
            continue
        v.sort()
        ds = sorted(x[1] for x in v)
        last = [x[1] for x in v[-timed:]]
        print("  %-70s median_us=%.1f last%d_avg_us=%.1f" % (k[:70], ds[len(ds) // 2] / 1e3, len(last),
                                                             sum(last) / len(last) / 1e3))
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "pmc*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        if not any(s in k for s in ("aes_gcm", "chacha", "ttab")):
            continue
        print("== counters per dispatch:", k[:90])
        for c, v in sorted(cs.items()):
            print("  %-24s %.4g  (n=%d)" % (c, sum(v) / len(v), len(v)))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[3]) if len(sys.argv) > 3 and sys.argv[2] == "--timed" else 20)
