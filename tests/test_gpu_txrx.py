"""Transmit and receive in one context at the same time, as one endpoint event loop drives them
(quic/s2n-quic-core/src/io/event_loop.rs:39-165: receive, then transmit, every wakeup, one task).

A resident transmit-queue server (qpp_txq_create_persistent; burst.hip txq_server_kernel, 16 CUs) keeps running while
full-chip batches and the fused receive launch run on the context's stream: the batch kernels size their grids to the
CUs the server leaves (cu_avail) and the cooperative receive launch needs all its workgroups resident at once
(quad.hip aes_gcm_quad_rx_kernel).  Bar: every GSO flush, every packet of the 1 Mi x 1200 B seal / open batch and
every packet of the 64-key receive batch bit-exact against the oracle (fastcheck for the full batch), no receive
barrier timeout (qpp_ctx_rx_timeouts), and the server never restarted in between (it was resident throughout).
"""
import time

import numpy as np
import pytest

import _oracle as orc
import qpp

pytestmark = pytest.mark.gpu

STRIDE = 1280


def _fill(q, rng, keys, n, pn0, largest):
    """n packets pushed into the ring at i * STRIDE (key i % len(keys)); returns [(off, protected)] from the oracle"""
    want = []
    for i in range(n):
        k = keys[i % len(keys)]
        pn = pn0 + i
        trunc, pn_len = qpp.pn_truncate(pn, largest)
        header = bytes([0x40 | (pn_len - 1)]) + rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
        payload = rng.integers(0, 256, int(rng.integers(1000, 1200)), dtype=np.uint8).tobytes()
        pkt = header + trunc.to_bytes(pn_len, "big") + payload
        off = i * STRIDE
        q.ring[off:off + len(pkt)] = np.frombuffer(pkt, dtype=np.uint8)
        q.push(k, pn, off, len(header), pn_len, len(payload))
        kk, iv, hp = k.material()
        want.append((off, orc.protect_packet(k.suite, kk, iv, hp, pn, header, pn_len, payload)[1]))
    return want


def _check(q, want):
    for off, p in want:
        assert q.ring[off:off + len(p)].tobytes() == p


def _rx_batch(rng, mats, slots, n):
    """n short-header packets of random connections and key phases, PN truncated against largest; some tampered"""
    chunks, rx, orx = [], [], []
    off = 0
    for i in range(n):
        c = int(rng.integers(0, len(slots)))
        largest = int(rng.integers(0, 2**40))
        pn = largest + int(rng.integers(0, 300))
        _, _, pn_len = orc.truncate_pn(pn, largest)
        phase = int(rng.integers(0, 2))
        header = bytes([0x40 | (phase << 2) | (pn_len - 1)]) + rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
        payload = rng.integers(0, 256, int(rng.integers(1, 1400)), dtype=np.uint8).tobytes()
        suite, k, iv, hp = mats[2 * c + phase]
        _, pkt = orc.protect_packet(suite, k, iv, hp, pn, header, pn_len, payload)
        pkt = bytearray(pkt)
        if i % 23 == 5:
            pkt[-1 - i % 16] ^= 0x04  # tampered -> DECRYPT_ERROR
        chunks.append(bytes(pkt) + bytes(int(rng.integers(0, 5))))
        rx.append((largest, slots[c], off, len(header), len(pkt)))
        orx.append((largest, (2 * c, 2 * c + 1), off, len(header), len(pkt)))
        off += len(chunks[-1])
    arena = np.frombuffer(b"".join(chunks) + bytes(64), dtype=np.uint8).copy()
    return np.array(rx, dtype=qpp.RX_DTYPE), np.array(orx, dtype=qpp.RX_DTYPE), arena


def test_tx_and_rx_with_resident_server(monkeypatch):
    monkeypatch.setenv("QPP_TXQ_SERVER_IDLE_MS", "30000")  # resident for the whole test unless something stops it
    rng = np.random.default_rng(4040)
    ctx = qpp.Context(0)
    q = None
    try:
        ctx.set_aes_kernel(qpp.AES_KERNEL_QUAD)  # the receive batch takes the fused launch at test size
        # 32 connections with both key phases live: 64 AES-128 packet keys
        pairs = []
        for _ in range(32):
            k0 = ctx.key(1, rng.integers(0, 256, 32, dtype=np.uint8).tobytes())
            pairs.append((k0, k0.derive_next_key()))
        keys = [k for p in pairs for k in p]
        mats = [(1, *k.material()) for k in keys]
        okeys = orc.make_keys(mats)
        slots = [k.slot for k in keys]

        # the throughput batch: BASELINE configs[2] size over the 64 keys
        n, pt = 1 << 20, 1200
        descs, arena = qpp.make_batch(n, pt, slots, seed=0x5eed0404)
        d_desc, d_arena, d_mask, d_status = ctx.alloc(descs.nbytes), ctx.alloc(arena.nbytes), ctx.alloc(5 * n), ctx.alloc(n)
        d_desc.upload(descs)
        # the receive batch
        nrx = 6000
        rx, orx, rx_arena = _rx_batch(rng, mats, [(p[0].slot, p[1].slot) for p in pairs], nrx)
        d_rx, d_rxa = ctx.alloc(rx.nbytes), ctx.alloc(rx_arena.nbytes)
        d_out, d_rst = ctx.alloc(nrx * qpp.PKT_DTYPE.itemsize), ctx.alloc(nrx)
        d_rx.upload(rx)
        # warm-up: the plan and receive scratch grow to these sizes now
        d_arena.upload(arena)
        ctx.seal_batch(d_desc, n, d_arena, d_mask, d_status, qpp.HP_MASK_OUT)
        d_rxa.upload(rx_arena)
        ctx.unprotect_open_batch(d_rx, nrx, d_rxa, d_out, d_rst)
        ctx.sync()
        d_arena.upload(arena)
        d_rxa.upload(rx_arena)
        d_rst.upload(np.full(nrx, 99, dtype=np.int8))
        d_status.upload(np.full(n, 99, dtype=np.int8))

        q = qpp.TxQueue(ctx, 64 * STRIDE, 64, persistent=True)
        largest = int(rng.integers(0, 2**40))
        pn = largest + 1

        def flush():
            nonlocal pn, largest
            want = _fill(q, rng, keys[:8], 64, pn, largest)
            q.flush()
            _check(q, want)
            pn += 64
            largest += 64

        flush()  # the server is resident from here on
        starts = q.info()[2]
        trail = []  # (step, server launches so far, seconds since the first flush)
        t_0 = time.perf_counter()
        note = lambda what: trail.append((what, q.info()[2], round(time.perf_counter() - t_0, 3)))
        ctx.seal_batch(d_desc, n, d_arena, d_mask, d_status, qpp.HP_MASK_OUT)  # asynchronous: runs beside the flushes
        note("seal_batch")
        flush()
        note("flush 2")
        ctx.unprotect_open_batch(d_rx, nrx, d_rxa, d_out, d_rst)  # same stream: after the seal
        note("unprotect_open_batch")
        flush()
        note("flush 3")
        ctx.sync()
        flush()
        note("flush 4")
        # the same server launch sealed every flush beside the batches (checked before the slow oracle work below: a
        # queue idle for a quarter of QPP_TXQ_SERVER_IDLE_MS restarts its server on the next flush, by design)
        served, launched, starts_now = q.info()
        assert launched == 0 and starts_now == starts, f"the server was stopped while the batches ran: {trail}"
        sealed, masks = d_arena.download(), d_mask.download()
        assert (d_status.download(dtype=np.int8) == 0).all()
        assert orc.check_full_seal(okeys, slots, descs, arena, sealed, masks, qpp.HP_MASK_OUT) == n  # every packet
        ctx.open_batch(d_desc, n, d_arena, d_status)
        flush()
        ctx.sync()
        assert (d_status.download(dtype=np.int8) == 0).all()
        v, a = d_arena.download().reshape(n, -1), arena.reshape(n, -1)
        assert (v[:, 21:21 + pt] == a[:, 21:21 + pt]).all()

        got_arena, got_st = d_rxa.download(), d_rst.download(dtype=np.int8)
        want_arena = rx_arena.copy()
        want_out, want_st = orc.unprotect_open_batch(okeys, orx, want_arena)
        want_st = np.array(want_st, dtype=np.int8)
        assert (got_st == want_st).all()
        assert (got_st == 0).sum() > nrx * 3 // 4 and (got_st == qpp.DECRYPT_ERROR).any()
        assert (got_arena[:-64] == want_arena[:-64]).all()
        out = d_out.download(dtype=qpp.PKT_DTYPE)
        for f in ("pn", "aad_len", "pt_len", "pn_len", "off"):
            assert (out[f] == want_out[f]).all(), f

        assert ctx.rx_timeouts() == 0
        assert q.info()[1] == 0  # every flush served by the resident kernel
        for b in (d_desc, d_arena, d_mask, d_status, d_rx, d_rxa, d_out, d_rst):
            b.free()
        ctx.free_keys(keys)
    finally:
        if q is not None:
            q.close()
        ctx.close()


def test_frees_with_resident_server_return_quickly(monkeypatch):
    """hipFree waits for every stream of the device, a resident server's too: a free (and a plan growth, which frees
    the old plan) while a persistent queue is live is parked instead (api.cpp release) -- the call returns in
    milliseconds, not after the server's idle time, and the server stays resident for the next flushes, bit-exact"""
    monkeypatch.setenv("QPP_TXQ_SERVER_IDLE_MS", "30000")
    rng = np.random.default_rng(4041)
    ctx = qpp.Context(0)
    q = None
    try:
        k = ctx.key(1, rng.integers(0, 256, 32, dtype=np.uint8).tobytes())
        q = qpp.TxQueue(ctx, 64 * STRIDE, 64, persistent=True)
        want = _fill(q, rng, [k], 64, 1001, 1000)
        q.flush()
        _check(q, want)
        buf = ctx.alloc(1 << 20)
        t0 = time.perf_counter()
        buf.free()
        assert time.perf_counter() - t0 < 0.5
        # a batch larger than any before on this stream: its plan grows (the old one is freed)
        ctx.set_aes_kernel(qpp.AES_KERNEL_QUAD)
        k2 = ctx.key(1, rng.integers(0, 256, 32, dtype=np.uint8).tobytes())  # two keys: a planned batch
        want = _fill(q, rng, [k], 64, 1065, 1064)
        q.flush()
        _check(q, want)
        descs, arena = qpp.make_batch(100000, 200, [k.slot, k2.slot], seed=5)
        d_desc, d_arena, d_status = ctx.alloc(descs.nbytes), ctx.alloc(arena.nbytes), ctx.alloc(100000)
        d_desc.upload(descs)
        d_arena.upload(arena)
        t0 = time.perf_counter()
        ctx.seal_batch(d_desc, 100000, d_arena, None, d_status, 0)
        ctx.sync()
        assert time.perf_counter() - t0 < 0.5
        assert (d_status.download(dtype=np.int8) == 0).all()
        want = _fill(q, rng, [k, k2], 64, 1129, 1128)
        q.flush()
        _check(q, want)
        served, launched, starts = q.info()
        assert (served, launched, starts) == (3, 0, 1)  # one server launch: the frees did not stop it
        for b in (d_desc, d_arena, d_status):
            b.free()
        k.free()
        k2.free()
    finally:
        if q is not None:
            q.close()
        ctx.close()
