"""Connection-indexed host batches (QPP_KEY_BY_CONN + qpp_ctx_set_conn_keys), on the GPU.

The transport's packets belong to a connection, whose KeySet holds the current key
(quic/s2n-quic-core/src/crypto/application/keyset.rs:75-96: a key update swaps the key behind the connection, the
queued packets do not change).  With QPP_KEY_BY_CONN the descriptors name connections and the device resolves them
through the table; bar: bit-exact with the same batch naming the slots directly, the table swap ordered between
batches (a batch in flight keeps the keys it was submitted with), and an index past the table refused.
"""
import numpy as np
import pytest

import qpp

pytestmark = pytest.mark.gpu

N_CONN = 64
N = 8192
PT = 600


def _seal(ctx, descs, arena, flags):
    host = ctx.host_alloc(arena.nbytes)
    host[:] = arena
    masks = ctx.host_alloc(5 * len(descs))
    st = ctx.host_alloc(len(descs)).view(np.int8)
    st[:] = 77
    t = ctx.host_submit(descs, host, masks, st, flags | qpp.HP_MASK_OUT, qpp.OP_SEAL)
    return t, host, masks, st


def test_conn_keys_equal_direct_slots_and_swap_between_batches():
    ctx = qpp.Context(0)
    try:
        rng = np.random.default_rng(0xC0)
        keys = [ctx.key(1, rng.integers(0, 256, 32, dtype=np.uint8).tobytes()) for _ in range(N_CONN)]
        m1 = np.array([k.slot for k in keys], dtype=np.uint32)
        new = ctx.update_keys(keys[:N_CONN // 2])  # a key update on half the connections
        m2 = m1.copy()
        m2[:N_CONN // 2] = [k.slot for k in new]
        descs, arena = qpp.make_batch(N, PT, list(range(N_CONN)), seed=0xC1)  # key_idx = connection index
        conn = descs["key_idx"].copy()
        descs["key_idx"][17] = N_CONN + 5  # past the table: refused
        # references: the same packets naming the slots directly
        refs = []
        for m in (m1, m2):
            d = descs.copy()
            d["key_idx"] = np.where(conn < N_CONN, m[np.minimum(conn, N_CONN - 1)], 0xffffffff)
            d["key_idx"][17] = 0xffffffff
            t, host, masks, st = _seal(ctx, d, arena, 0)
            ctx.host_wait(t)
            refs.append((host.copy(), masks.copy(), st.copy()))
        # connection-indexed: X through table m1, then the swap, then Y through m2, both in flight together
        ctx.set_conn_keys(m1)
        tx = _seal(ctx, descs, arena, qpp.KEY_BY_CONN)
        ctx.set_conn_keys(m2)
        ty = _seal(ctx, descs, arena, qpp.KEY_BY_CONN)
        for (t, host, masks, st), (rh, rm, rs) in zip((tx, ty), refs):
            ctx.host_wait(t)
            assert (st == rs).all() and st[17] == qpp.INTERNAL_ERROR and (np.delete(st, 17) == 0).all()
            assert (host == rh).all()
            assert (masks.reshape(-1, 5)[st == 0] == rm.reshape(-1, 5)[st == 0]).all()
        stride = arena.size // N
        assert (tx[1][17 * stride:18 * stride] == arena[17 * stride:18 * stride]).all()  # refused: untouched
        assert not (tx[1] == ty[1]).all()  # the two tables sealed with different keys
        c2 = qpp.Context(0)  # no table set: a connection-indexed batch is refused before anything is queued
        try:
            with pytest.raises(qpp.QppError):
                c2.host_submit(descs[:4], arena[:4 * stride].copy(), None, np.zeros(4, np.int8), qpp.KEY_BY_CONN,
                               qpp.OP_SEAL)
        finally:
            c2.close()
    finally:
        ctx.close()
