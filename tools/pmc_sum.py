"""Average PMC counters per dispatch for kernels matching a substring: python tools/pmc_sum.py <dir> [substr]"""
import csv, glob, os, sys
from collections import defaultdict
d = sys.argv[1]; sub = sys.argv[2] if len(sys.argv) > 2 else "aes_gcm_quad_kernel"
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    if sub not in k: continue
    print("==", k[:100])
    for c, v in sorted(cs.items()):
        print("  %-28s %.4g" % (c, sum(v) / len(v)))
