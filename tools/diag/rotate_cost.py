"""Where the C5 rotation's host time goes: qpp_key_update_batch, qpp_key_free_batch and the descriptor key-slot
rewrite of a 2 Mi-packet batch, for 4096 AES-128 keys (bench.py --mode e2e --keys 4096 --rotate)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "s2n-quic_amd"))
import qpp  # noqa: E402

ctx = qpp.Context(0)
rng = np.random.default_rng(1)
keys = [ctx.key(1, rng.integers(0, 256, 32, dtype=np.uint8).tobytes()) for _ in range(4096)]
n = 2 << 20
descs = np.zeros(n, dtype=qpp.PKT_DTYPE)
conn = rng.integers(0, 4096, n).astype(np.int64)
t = {"update": 0.0, "free": 0.0, "slots": 0.0, "rewrite": 0.0}
for it in range(6):
    t0 = time.perf_counter()
    new = ctx.update_keys(keys)
    t1 = time.perf_counter()
    ctx.free_keys(keys)
    t2 = time.perf_counter()
    keys = new
    slots = np.array([k.slot for k in keys], dtype=np.uint32)
    t3 = time.perf_counter()
    descs["key_idx"] = slots[conn]
    t4 = time.perf_counter()
    if it >= 2:
        for k, v in zip(t, (t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
            t[k] += v
print({k: round(v / 4 * 1e3, 3) for k, v in t.items()}, "ms per rotation")
