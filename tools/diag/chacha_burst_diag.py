"""Which packets of the ragged ChaCha batch differ between the burst kernel and the oracle (diagnostic)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "s2n-quic_amd")]
import qpp, _oracle as orc
from test_gpu_parity import _keys, _ragged_batch, _run_seal, _oracle_keys_for
ctx = qpp.Context(0)
ctx.set_burst_max(1 << 30)
keys, okeys = _keys(ctx, [3], seed=1 * 31 + 3)
slots = [k.slot for k in keys]
descs, arena = _ragged_batch(2048, slots, seed=7 + 1)
got, masks, st = _run_seal(ctx, descs, arena, 0)
want = arena.copy()
orc.seal_batch(okeys, _oracle_keys_for(okeys, descs, slots), want, 0)
bad = 0
for i, d in enumerate(descs):
    o, a, p = int(d["off"]), int(d["aad_len"]), int(d["pt_len"])
    ct_bad = (got[o + a:o + a + p] != want[o + a:o + a + p]).sum()
    tag_bad = (got[o + a + p:o + a + p + 16] != want[o + a + p:o + a + p + 16]).sum()
    if ct_bad or tag_bad:
        bad += 1
        m = (a + 15) // 16 + (p + 15) // 16 + 1
        print(f"pkt {i}: aad {a} pt {p} m {m} K {(m + 63) // 64} pad {64 * ((m + 63) // 64) - m} ct_bad {ct_bad} tag_bad {tag_bad}")
print("bad packets", bad, "of", len(descs))
