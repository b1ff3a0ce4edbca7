"""Per-packet trait-API latency (Key::encrypt / decrypt through qpp_seal / qpp_open), median over 300 calls."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "s2n-quic_amd"))
import numpy as np
import qpp
ctx = qpp.Context(0)
hdr = bytes([0x43]) + bytes(20)
pt = bytes(np.random.default_rng(1).integers(0, 256, 1200, dtype=np.uint8))
for suite in (1, 3):
    k = ctx.key(suite, bytes(qpp.HASH_LEN[suite]))
    ts, to = [], []
    for i in range(300):
        t0 = time.perf_counter(); ct = k.encrypt(i, hdr, pt); t1 = time.perf_counter()
        assert k.decrypt(i, hdr, ct) == pt
        t2 = time.perf_counter()
        ts.append(t1 - t0); to.append(t2 - t1)
    print(f"suite {suite}: encrypt {1e6 * np.median(ts):.1f} us, decrypt {1e6 * np.median(to):.1f} us (1200 B, median of 300)")
