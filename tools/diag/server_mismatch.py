"""Replays tests/test_gpu_txq_server.py::test_server_bursts_bit_exact and, for every packet the persistent server
sealed differently from the oracle, tells which input it looks like it was sealed from: another packet's
descriptor of this or the previous flush (pn / offset), stale ring bytes, or neither; also the launched path."""
import os
import sys

import numpy as np

sys.path.insert(0, "s2n-quic_amd")
sys.path.insert(0, "tests")
os.environ["QPP_TXQ_SERVER_IDLE_MS"] = "4000"
import _oracle as orc  # noqa: E402
import qpp  # noqa: E402
from test_gpu_txq_server import STRIDE, _fill  # noqa: E402

persistent = "--launch" not in sys.argv
ctx = qpp.Context(0)
rng = np.random.default_rng(71)
k = ctx.key(1, rng.integers(0, 256, 32, dtype=np.uint8).tobytes())
kk, iv, hp = k.material()
q = qpp.TxQueue(ctx, 64 * STRIDE, 64, persistent=persistent)
largest = int(rng.integers(0, 2**40))
bad_total = 0
prev = None
for f in range(30):
    pn0 = largest + 1 + 64 * f
    want = _fill(q, rng, [k], 64, pn0, largest + 64 * f, sizes=(1000, 1200))
    plain = [q.ring[off:off + len(p)].tobytes() for off, p in want]  # header || pn || payload || (tag space)
    q.flush()
    bad = []
    for i, (off, p) in enumerate(want):
        got = q.ring[off:off + len(p)].tobytes()
        if got != p:
            first = next(j for j in range(len(p)) if got[j] != p[j])
            bad.append((i, first, len(p)))
    if bad:
        bad_total += len(bad)
        print(f"flush {f}: {len(bad)} packets differ: " + ", ".join(f"#{i} from byte {b} (len {n})" for i, b, n in bad[:12]))
        i, _, n = bad[0]
        off, p = want[i]
        got = q.ring[off:off + n].tobytes()
        # which pn was it sealed with?  try the pns of this flush and the previous one, header/payload as pushed
        hdr = plain[i][:17]
        pn_len = (hdr[0] & 3) + 1
        pay = plain[i][17 + pn_len:n - 16]
        for cand in list(range(pn0 - 64, pn0 + 64)):
            _, c = orc.protect_packet(1, kk, iv, hp, cand, hdr, pn_len, pay)
            if c[17 + pn_len:] == got[17 + pn_len:]:
                print(f"   packet #{i}: payload sealed with pn {cand} (want {pn0 + i}, delta {cand - pn0 - i})")
                break
        else:
            print(f"   packet #{i}: no pn in [{pn0 - 64}, {pn0 + 64}) reproduces it; got[17:40]={got[17:40].hex()} want={p[17:40].hex()}")
            print(f"   plain[17:40]={plain[i][17:40].hex()}")
print("served/launched/starts", q.info(), "bad packets", bad_total)
q.close()
k.free()
ctx.close()
