"""HBM traffic per launch of the seal kernel from a tools/profile.sh run (PMC FETCH_SIZE / WRITE_SIZE, KiB units),
written to profiles/traffic.json for bench.py's roofline.traffic.

    python tools/traffic.py gpurun_out/<prof dir> <workload key, e.g. aes128gcm/1200/1> <packets> [profiles/traffic.json]

A key "rx:<suite>/<pt>/<keys>" takes the fused receive kernel (aes_gcm_quad_rx_kernel, one launch per call) instead,
with the receive path's algorithmic bytes (bench.rx_bytes_per_packet).

FETCH_SIZE / WRITE_SIZE are the L2's memory-side request counters (MI355X_MICROARCH.md, HBM/rocprofv3), KiB x 1024.
Reads follow the guide's rule: on gfx950 FETCH_SIZE reports half of a wide streaming read, so the read figure is
FETCH_SIZE x 2 (the raw count is kept beside it).  WRITE_SIZE is taken as counted.  The algorithmic bytes
(bench.seal_bytes_per_packet: read AAD + payload + descriptor, write ciphertext + tag + mask) go beside them, with
the ratios; traffic_bytes = reads x 2 + writes.
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(d, key, packets, out="profiles/traffic.json"):
    packets = int(packets)
    acc = {}
    rx = key.startswith("rx:")
    kernels = ("aes_gcm_quad_rx_kernel",) if rx else ("aes_gcm_quad_kernel<true", "chacha_kernel<true",
                                                      "aes_gcm_wave_kernel<true")
    for f in glob.glob(os.path.join(d, "pmc*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if not any(k in name for k in kernels):
                continue
            acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    fetch_raw = sum(acc["FETCH_SIZE"]) / len(acc["FETCH_SIZE"]) * 1024
    write = sum(acc["WRITE_SIZE"]) / len(acc["WRITE_SIZE"]) * 1024
    suite, pt, _ = key.split(":")[-1].split("/")
    pt = int(pt)
    aad = 21
    if rx:  # rx descriptor + header + CT + tag read; first byte + PN, descriptor out, plaintext, status written
        alg_read, alg_write = packets * (24 + aad + pt + 16), packets * (5 + 24 + pt + 1)
    else:
        alg_read, alg_write = packets * (aad + pt + 24), packets * (pt + 16 + 5)
    db = json.load(open(out)) if os.path.exists(out) else {}
    db[key] = {"fetch_size_raw_bytes": round(fetch_raw), "read_bytes": round(2 * fetch_raw), "write_bytes": round(write),
               "traffic_bytes": round(2 * fetch_raw + write), "alg_read_bytes": alg_read, "alg_write_bytes": alg_write,
               "read_per_alg": round(2 * fetch_raw / alg_read, 3), "write_per_alg": round(write / alg_write, 3),
               "source": os.path.basename(os.path.normpath(d)) + " (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, "
                         + ("fused receive" if rx else "seal") + " kernel, mean over its launches; reads = FETCH_SIZE"
                         " x 2 per MI355X_MICROARCH.md)"}
    json.dump(db, open(out, "w"), indent=1, sort_keys=True)
    print(key, db[key])


if __name__ == "__main__":
    main(*sys.argv[1:])
