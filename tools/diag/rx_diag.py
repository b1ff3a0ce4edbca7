"""Where the fused receive kernel and the multi-launch path differ (tests/test_gpu_rx_fused.py's first case)."""
import os
import sys

import numpy as np

sys.path.insert(0, "tests"); sys.path.insert(0, "s2n-quic_amd")
import qpp
from test_gpu_rx_fused import _batch


class MP:
    def setenv(self, k, v):
        os.environ[k] = v


ctx = qpp.Context(0)
from test_gpu_rx_fused import _run
rng = np.random.default_rng(41)
ctx.set_burst_max(0)
k0 = ctx.key(1, rng.integers(0, 256, 32, dtype=np.uint8).tobytes())
k1 = k0.derive_next_key()
mats = [(1, *k0.material()), (1, *k1.material())]
slots = [k0.slot, k1.slot]
n = 3000
rx, orx, arena = _batch(rng, mats, slots, n)
k1.free()
a_f, o_f, s_f = _run(ctx, rx, arena, MP(), fused=True)
a_2, o_2, s_2 = _run(ctx, rx, arena, MP(), fused=False)
print("status equal", (s_f == s_2).all(), "descs equal", (o_f.view(np.uint8) == o_2.view(np.uint8)).all())
bad = np.nonzero(a_f != a_2)[0]
print("differing bytes", len(bad))
offs = rx["off"].astype(np.int64)
pk = np.searchsorted(offs, bad, side="right") - 1
for p in np.unique(pk)[:12]:
    o, ln, hl = int(rx[p]["off"]), int(rx[p]["len"]), int(rx[p]["header_len"])
    b = bad[pk == p] - o
    print("pkt", p, "len", ln, "hdr", hl, "aad", int(o_2[p]["aad_len"]), "status f/2", s_f[p], s_2[p],
          "key f/2", o_f[p]["key_idx"], o_2[p]["key_idx"], "flags", o_f[p]["flags"], o_2[p]["flags"],
          "bytes", b.min(), b.max(), len(b))
print("packets differing", len(np.unique(pk)))
