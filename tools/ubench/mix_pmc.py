"""Pipe fractions per kernel of tools/ubench/mix from its PMC passes (run_mix.sh).

LDS busy   = SQ_LDS_IDX_ACTIVE / (CUs x cycles)             (LDS-array cycles; ds_read_b32 = 2, ds_read_b128 = 4)
VALU busy  = SQ_INSTS_VALU x 4 / (SIMDs x cycles)           (a wave64 VALU instruction holds its SIMD's issue 4 cycles)
cycles     = GRBM_GUI_ACTIVE / 8                            (the counter sums the 8 XCDs)
wait / issue-stall / active = SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES (disjoint)
"""
import csv, glob, os, re, sys
from collections import defaultdict

CUS = 256
d = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "pmc*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
print("%-44s %6s %6s %6s %6s %6s %7s %7s" % ("kernel", "LDS", "VALU", "sum", "wait", "istall", "VALU/wb", "LDSc/wb"))
for k in sorted(acc):
    c = {n: sum(v) / len(v) for n, v in acc[k].items()}
    if "GRBM_GUI_ACTIVE" not in c or "SQ_LDS_IDX_ACTIVE" not in c:
        continue
    cyc = c["GRBM_GUI_ACTIVE"] / 8
    lds = c["SQ_LDS_IDX_ACTIVE"] / (CUS * cyc)
    valu = c["SQ_INSTS_VALU"] * 4 / (4 * CUS * cyc)
    wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    m = re.match(r"void (\w+)<(.*?)>", k)
    name = (m.group(1) + "<" + m.group(2) + ">") if m else k[:44]
    print("%-44s %6.3f %6.3f %6.3f %6.3f %6.3f %7s %7s" % (name[:44], lds, valu, lds + valu, c.get("SQ_WAIT_ANY", 0) / wc,
                                                    c.get("SQ_WAIT_INST_ANY", 0) / wc if "SQ_WAIT_INST_ANY" in c else float("nan"), "", ""))
