"""Diagnostics for the persistent txq server: mismatching packets per flush, with the ring region reused or not."""
import sys
import numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, "s2n-quic_amd")
import _oracle as orc
import qpp
from test_gpu_txq_server import _fill, STRIDE

ctx = qpp.Context(0)
rng = np.random.default_rng(71)
k = ctx.key(1, rng.integers(0, 256, 32, dtype=np.uint8).tobytes())
for reuse in (True, False):
    q = qpp.TxQueue(ctx, 64 * STRIDE * 8, 64, persistent=True)
    largest = 1000
    for f in range(8):
        base = 0 if reuse else f * 64 * STRIDE
        want = _fill(q, rng, [k], 64, largest + 1, largest, base=base, sizes=(1000, 1200))
        q.flush()
        bad = [i for i, (o, p) in enumerate(want) if q.ring[o:o + len(p)].tobytes() != p]
        first = []
        for i in bad[:3]:
            o, p = want[i]
            got = q.ring[o:o + len(p)].tobytes()
            d = [j for j in range(len(p)) if got[j] != p[j]]
            first.append((i, len(p), d[0], d[-1], len(d)))
        print("reuse", reuse, "flush", f, "bad", len(bad), first, q.info(), flush=True)
        largest += 64
    q.close()
# launched path for comparison
q = qpp.TxQueue(ctx, 64 * STRIDE, 64)
want = _fill(q, rng, [k], 64, 5001, 5000, sizes=(1000, 1200))
q.flush()
print("launched bad", sum(q.ring[o:o + len(p)].tobytes() != p for o, p in want))
