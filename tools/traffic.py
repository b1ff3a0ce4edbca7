"""HBM traffic per launch of the seal kernel from a tools/profile.sh run (PMC FETCH_SIZE / WRITE_SIZE, KiB units),
written to profiles/traffic.json for bench.py's roofline.traffic.

    python tools/traffic.py gpurun_out/<prof dir> <workload key, e.g. aes128gcm/1200/1> [profiles/traffic.json]

FETCH_SIZE / WRITE_SIZE are the L2's memory-side request counters (MI355X_MICROARCH.md, HBM/rocprofv3), KiB x 1024.
The guide's x2 read correction is calibrated for 16-B-per-lane coalesced streams, and tells to calibrate other
patterns on a known byte count: tools/ubench/copy_pattern.hip moves exactly 1200 B in + 1200 B out per packet with
this kernel's cooperative 64-B chunks at +21 offsets and nt stores, and its FETCH_SIZE reads 1.184x the true bytes
(profiles/r02_copy_pattern_calibration.json, "coop_unaligned_nt"; loads alone: 1.174x), so fetch = FETCH_SIZE / 1.184.
WRITE_SIZE is taken as counted: the same copy reports 1.48x for writes whose 64-B chunks straddle 64-B segments, and
those partial-segment writes are real memory transactions (the aligned variant of the copy reports 1.115x).
Since the kernels' payload stores became nt, the seal kernel's FETCH_SIZE fell 42 % (1.54 -> 0.89 GiB raw per launch)
while the copy's did not move: the calibrated read figure then sits BELOW the algorithmic read bytes, so for this
kernel it is a lower bound and the write side (taken as counted) is the informative one ("note" in the output).
"""
import csv
import glob
import json
import os
import sys


def main(d, key, out="profiles/traffic.json"):
    acc = {}
    for f in glob.glob(os.path.join(d, "pmc*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if not (("aes_gcm_kernel<true" in name) or ("chacha_kernel<true" in name)):
                continue
            acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    fetch_raw = sum(acc["FETCH_SIZE"]) / len(acc["FETCH_SIZE"]) * 1024
    write = sum(acc["WRITE_SIZE"]) / len(acc["WRITE_SIZE"]) * 1024
    cal = json.load(open("profiles/r02_copy_pattern_calibration.json"))["coop_unaligned_nt"]["fetch_per_alg"]
    fetch = fetch_raw / cal
    db = json.load(open(out)) if os.path.exists(out) else {}
    db[key] = {"fetch_bytes": round(fetch), "fetch_size_raw_bytes": round(fetch_raw), "fetch_calibration": cal,
               "write_bytes": round(write), "traffic_bytes": round(fetch + write),
               "note": "calibrated fetch is below the algorithmic reads for the nt-store kernel: a lower bound",
               "source": os.path.basename(os.path.normpath(d)) + " (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, seal kernel;"
                         " fetch / " + str(cal) + " per the copy_pattern calibration)"}
    json.dump(db, open(out, "w"), indent=1, sort_keys=True)
    print(key, db[key])


if __name__ == "__main__":
    main(*sys.argv[1:])
