"""Where a 4096-key rotation step (BASELINE configs[4], bench.py --mode e2e --rotate) spends its time: the C call
qpp_key_update_batch, the Python handle objects, qpp_key_slot_batch and qpp_key_free_batch, timed separately."""
import ctypes
import sys
import time

import numpy as np

sys.path.insert(0, "s2n-quic_amd")
import qpp
from qpp import lib, vp

ctx = qpp.Context(0)
rng = np.random.default_rng(3)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
keys = [ctx.key(1, rng.integers(0, 256, 32, dtype=np.uint8).tobytes()) for _ in range(n)]
ctx.synchronize()
slots = np.zeros(n, dtype=np.uint32)
acc = {"update_c": 0.0, "slots_c": 0.0, "py_objs": 0.0, "free_c": 0.0}
steps = 12
for s in range(steps):
    t0 = time.perf_counter()
    arr_in = (vp * n)(*[k.handle for k in keys])
    arr = (vp * n)()
    rc = lib().qpp_key_update_batch(arr_in, n, arr)
    assert rc == 0
    t1 = time.perf_counter()
    lib().qpp_key_slot_batch(arr, n, slots.ctypes.data)
    t2 = time.perf_counter()
    new = [qpp.Key(ctx, arr[i]) for i in range(n)]
    t3 = time.perf_counter()
    ctx.free_keys(keys)
    t4 = time.perf_counter()
    keys = new
    if s >= 2:
        acc["update_c"] += t1 - t0
        acc["slots_c"] += t2 - t1
        acc["py_objs"] += t3 - t2
        acc["free_c"] += t4 - t3
print({k: round(1e3 * v / (steps - 2), 3) for k, v in acc.items()}, "ms per step,", n, "keys", flush=True)
ctx.synchronize()
