"""Pinned host <-> HBM copy rates (the e2e / C5 path's ceiling): one direction, both directions at once, and both
directions with the copies split over 2 or 4 streams per direction.  usage: python tools/ubench/pcie.py"""
import json
import time

import torch


def rate(fn, nbytes, reps=6):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return nbytes * reps / (time.perf_counter() - t) / 1e9


def main():
    mb = 512
    n = mb << 20
    h_in = torch.empty(n, dtype=torch.uint8).pin_memory()
    h_out = torch.empty(n, dtype=torch.uint8).pin_memory()
    d_a = torch.empty(n, dtype=torch.uint8, device="cuda")
    d_b = torch.empty(n, dtype=torch.uint8, device="cuda")
    res = {}
    for k in (1, 2, 4):
        hs = [torch.cuda.Stream() for _ in range(k)]
        ds = [torch.cuda.Stream() for _ in range(k)]
        part = n // k

        def h2d():
            for i, s in enumerate(hs):
                with torch.cuda.stream(s):
                    d_a[i * part:(i + 1) * part].copy_(h_in[i * part:(i + 1) * part], non_blocking=True)

        def d2h():
            for i, s in enumerate(ds):
                with torch.cuda.stream(s):
                    h_out[i * part:(i + 1) * part].copy_(d_b[i * part:(i + 1) * part], non_blocking=True)

        def both():
            h2d()
            d2h()

        res[f"h2d_{k}streams_GBps"] = round(rate(h2d, n), 1)
        res[f"d2h_{k}streams_GBps"] = round(rate(d2h, n), 1)
        res[f"bidir_{k}streams_each_GBps"] = round(rate(both, 2 * n), 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
