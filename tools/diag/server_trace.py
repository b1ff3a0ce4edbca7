"""Phase stamps of the persistent txq server (build with -DQPP_TXS_TRACE=1, e.g. tools/build_ab.sh sT
-DQPP_TXS_TRACE=1; run with QPP_LIB=ab/sT.so): median microseconds of each step of a 64 x 1200 B flush, from the
host's doorbell write to its return from qpp_txq_flush.  argv: [burst packets (64)] [payload bytes (1200)]."""
import ctypes
import sys
import time

import numpy as np

sys.path.insert(0, "s2n-quic_amd")
import qpp

ctx = qpp.Context(0)
rng = np.random.default_rng(9)
k = ctx.key(1, rng.integers(0, 256, 32, dtype=np.uint8).tobytes())
burst = int(sys.argv[1]) if len(sys.argv) > 1 else 64
pt = int(sys.argv[2]) if len(sys.argv) > 2 else 1200
stride = (21 + pt + 16 + 63) // 64 * 64
q = qpp.TxQueue(ctx, burst * stride, burst, persistent=True)
q.ring[:] = rng.integers(0, 256, q.ring.size, dtype=np.uint8)
proto = np.zeros(burst, dtype=qpp.PKT_DTYPE)
proto["key_idx"] = k.slot
proto["off"] = np.arange(burst) * stride
proto["aad_len"], proto["pt_len"], proto["pn_len"] = 21, pt, 4
# the mailbox: qpp_txq is opaque; read it through qpp_txq_server_time's neighbour fields via a raw pointer walk is not
# possible from Python, so the stamps are fetched with ctypes from the library's debug accessor
lib = qpp.lib()
rows = []
for i in range(600):
    d = proto.copy()
    d["pn"] = (1 << 20) + i * burst + np.arange(burst, dtype=np.uint64)
    q.push_descs(d)
    t0 = time.perf_counter()
    q.flush()
    t1 = time.perf_counter()
    st = (ctypes.c_uint64 * 12)()
    lib.qpp_txq_server_stamps(q.handle, st)
    if i >= 100:
        lo = st[0] & 0xffffffff
        rows.append([(t1 - t0) * 1e6] + [(st[j] - st[0]) / 100.0 for j in range(1, 6)] +
                    [st[6] / max(1.0, (st[4] - st[1]) / 100.0)] + [((st[j] - lo) & 0xffffffff) / 100.0 for j in range(7, 12)])
a = np.median(np.array(rows), axis=0)
print(f"{burst} x {pt} B: ", end="")
print("median us: host flush %.1f | from doorbell seen: broadcast %.2f item+desc %.2f packets %.2f arrive %.2f done %.2f"
      " | shader clock %.0f MHz | wave 0 packet: start %.2f block in %.2f passes %.2f tree %.2f hp %.2f" % tuple(a))
