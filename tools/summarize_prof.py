"""Summarise a tools/profile.sh output directory: per-kernel average duration (kernel trace) and the PMC
counters averaged per dispatch of each kernel."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d):
    rows = []
    for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    print("== kernel stats (%s)" % d)
    for r in rows:
        print("  %-70s calls=%-4s avg_us=%.1f total_pct=%s" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3,
                                                               r.get("Percentage", "")))
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
    main(sys.argv[1])
