"""HBM traffic per launch of the seal kernel from a tools/profile.sh run (PMC FETCH_SIZE / WRITE_SIZE, KiB units),
written to profiles/traffic.json for bench.py's roofline.traffic.

    python tools/traffic.py gpurun_out/<prof dir> <workload key, e.g. aes128gcm/1200/1> [profiles/traffic.json]

FETCH_SIZE / WRITE_SIZE are the L2's memory-side request counters (MI355X_MICROARCH.md, HBM/rocprofv3): the bytes
are reported as counted (KiB x 1024), without the x2 streaming-read correction the guide calibrates for 16-B-per-lane
coalesced streams -- this kernel's 64-B per-packet chunks are not that pattern, so the raw count is the one stated.
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
    fetch = sum(acc["FETCH_SIZE"]) / len(acc["FETCH_SIZE"]) * 1024
    write = sum(acc["WRITE_SIZE"]) / len(acc["WRITE_SIZE"]) * 1024
    db = json.load(open(out)) if os.path.exists(out) else {}
    db[key] = {"fetch_bytes": round(fetch), "write_bytes": round(write), "traffic_bytes": round(fetch + write),
               "source": os.path.basename(os.path.normpath(d)) + " (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, seal kernel)"}
    json.dump(db, open(out, "w"), indent=1, sort_keys=True)
    print(key, db[key])


if __name__ == "__main__":
    main(*sys.argv[1:])
