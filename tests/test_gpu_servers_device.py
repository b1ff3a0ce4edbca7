"""Resident server kernels accounted per DEVICE, not per context.

The reference's keys are independent `Send` objects any endpoint task may own (quic/s2n-quic-core/src/crypto/key.rs:8),
and one endpoint event loop drives receive and transmit together (quic/s2n-quic-core/src/io/event_loop.rs:39-165).  So
several contexts of one process -- each with its own packet server (qpp_seal / qpp_open / qpp_hp_mask) and maybe a
persistent transmit queue -- share the GPU while fused receives run.  api.cpp's device registry (DevServers) keeps:
  * the fused receive's grid sized for the CUs every context's resident servers leave (its grid barriers need every
    workgroup resident), fused receives of the device one after another, and a server launch behind the latest fused
    receive (a server starting while the receive's workgroups are dispatched would take CUs its grid counted on);
  * at most GPU_MAX_HW_QUEUES (4) resident servers per device: past that a context's per-packet call is launched and a
    transmit-queue flush takes the launched path (never queued behind a resident kernel's hardware queue).
Bar: every byte bit-exact against the oracle, no receive barrier timeout in any context, every call returns promptly.
"""
import time

import numpy as np
import pytest

import _oracle as orc
import qpp

pytestmark = pytest.mark.gpu

STRIDE = 1280


def _rx_batch(rng, mats, slots, n):
    """n short-header packets of random connections and key phases (a few tampered): rx descriptors, oracle rx, arena"""
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
        if i % 29 == 3:
            pkt[-1 - i % 16] ^= 0x08  # tampered -> DECRYPT_ERROR
        chunks.append(bytes(pkt) + bytes(int(rng.integers(0, 5))))
        rx.append((largest, slots[c], off, len(header), len(pkt)))
        orx.append((largest, (2 * c, 2 * c + 1), off, len(header), len(pkt)))
        off += len(chunks[-1])
    arena = np.frombuffer(b"".join(chunks) + bytes(64), dtype=np.uint8).copy()
    return np.array(rx, dtype=qpp.RX_DTYPE), np.array(orx, dtype=qpp.RX_DTYPE), arena


class _Receiver:
    """a context with 32 connections x 2 key phases (64 AES-128 packet keys) and one receive batch, re-armed per run"""

    def __init__(self, ctx, rng, nrx):
        ctx.set_aes_kernel(qpp.AES_KERNEL_QUAD)  # the fused launch at this batch size
        pairs = []
        for _ in range(32):
            k0 = ctx.key(1, rng.integers(0, 256, 32, dtype=np.uint8).tobytes())
            pairs.append((k0, k0.derive_next_key()))
        self.keys = [k for p in pairs for k in p]
        mats = [(1, *k.material()) for k in self.keys]
        self.okeys = orc.make_keys(mats)
        self.rx, self.orx, self.arena = _rx_batch(rng, mats, [(p[0].slot, p[1].slot) for p in pairs], nrx)
        self.ctx, self.n = ctx, nrx
        self.d_rx, self.d_arena = ctx.alloc(self.rx.nbytes), ctx.alloc(self.arena.nbytes)
        self.d_out, self.d_st = ctx.alloc(nrx * qpp.PKT_DTYPE.itemsize), ctx.alloc(nrx)
        self.d_rx.upload(self.rx)
        want_arena = self.arena.copy()
        self.want_out, want_st = orc.unprotect_open_batch(self.okeys, self.orx, want_arena)
        self.want_st, self.want_arena = np.array(want_st, dtype=np.int8), want_arena

    def arm(self, stream=None):
        self.d_arena.upload(self.arena, stream)
        self.d_st.upload(np.full(self.n, 99, dtype=np.int8), stream)

    def run(self, stream=None):
        self.ctx.unprotect_open_batch(self.d_rx, self.n, self.d_arena, self.d_out, self.d_st, stream=stream)

    def check(self):
        got_st = self.d_st.download(dtype=np.int8)
        assert (got_st == self.want_st).all()
        assert (got_st == qpp.DECRYPT_ERROR).any() and (got_st == 0).sum() > self.n * 3 // 4
        assert (self.d_arena.download()[:-64] == self.want_arena[:-64]).all()
        out = self.d_out.download(dtype=qpp.PKT_DTYPE)
        for f in ("pn", "aad_len", "pt_len", "pn_len", "off"):
            assert (out[f] == self.want_out[f]).all(), f


def _seal_one(rng, k, suite):
    kk, iv, _ = k.material()
    pn = int(rng.integers(0, 2**40))
    header = rng.integers(0, 256, 21, dtype=np.uint8).tobytes()
    payload = rng.integers(0, 256, int(rng.integers(0, 1400)), dtype=np.uint8).tobytes()
    want = b"".join(orc.seal(suite, kk, orc.nonce(iv, pn), header, payload))
    t0 = time.perf_counter()
    got = k.encrypt(pn, header, payload)
    dt = time.perf_counter() - t0
    assert got == want
    return dt


def test_five_contexts_servers_txq_and_fused_receive(monkeypatch):
    """Five contexts make interleaved per-packet seals (five packet servers: more than the device's 4 server slots),
    context A's persistent transmit queue flushes between them and context B runs 64-key fused receives: every byte
    matches the oracle, no receive barrier timed out anywhere, and no call stalls"""
    monkeypatch.setenv("QPP_TXQ_SERVER_IDLE_MS", "30000")
    rng = np.random.default_rng(5050)
    ctxs = [qpp.Context(0) for _ in range(5)]
    q = None
    try:
        suites = [1, 2, 3, 1, 2]
        pkeys = [c.key(s, rng.integers(0, 256, qpp.HASH_LEN[s], dtype=np.uint8).tobytes())
                 for c, s in zip(ctxs, suites)]
        recv = _Receiver(ctxs[1], rng, 6000)
        ka = ctxs[0].key(1, rng.integers(0, 256, 32, dtype=np.uint8).tobytes())
        q = qpp.TxQueue(ctxs[0], 64 * STRIDE, 64, persistent=True)
        pn_tx = 1000

        def flush():
            nonlocal pn_tx
            want = []
            for i in range(64):
                header = bytes([0x43]) + rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
                payload = rng.integers(0, 256, int(rng.integers(1000, 1200)), dtype=np.uint8).tobytes()
                trunc, pn_len = qpp.pn_truncate(pn_tx + i, pn_tx - 1)
                pkt = header + trunc.to_bytes(pn_len, "big") + payload
                q.ring[i * STRIDE:i * STRIDE + len(pkt)] = np.frombuffer(pkt, dtype=np.uint8)
                q.push(ka, pn_tx + i, i * STRIDE, len(header), pn_len, len(payload))
                kk, iv, hp = ka.material()
                want.append((i * STRIDE, orc.protect_packet(1, kk, iv, hp, pn_tx + i, header, pn_len, payload)[1]))
            t0 = time.perf_counter()
            q.flush()
            dt = time.perf_counter() - t0
            for off, p in want:
                assert q.ring[off:off + len(p)].tobytes() == p
            pn_tx += 64
            return dt

        times = []
        for rnd in range(6):
            recv.arm()
            recv.run()  # asynchronous on context B's stream
            for i, (k, s) in enumerate(zip(pkeys, suites)):
                times.append(_seal_one(rng, k, s))
                if i == 2:
                    times.append(flush())
            ctxs[1].sync()
            recv.check()
        for c in ctxs:
            assert c.rx_timeouts() == 0
        # every call returned promptly (no server launch queued behind another's hardware queue: that stalled for the
        # resident server's idle time, 30 s here); the bar is generous for a shared box, the median is printed
        times.sort()
        print(f"per-call latency: median {1e6 * times[len(times) // 2]:.0f} us, max {1e6 * times[-1]:.0f} us")
        assert times[-1] < 0.25, times[-5:]
        served = [c.packet_server_info()[0] for c in ctxs]
        assert sum(1 for x in served if x) >= 1  # some contexts' calls went through a packet server ...
        assert q.info()[0] + q.info()[1] == 6  # ... and every flush was sealed (served or launched)
        recv_keys = recv.keys
        ctxs[1].free_keys(recv_keys)
    finally:
        if q is not None:
            q.close()
        for c in ctxs:
            c.close()


def test_packet_server_start_behind_queued_fused_receive():
    """a fused receive queued behind a long seal, then a per-packet open that starts the context's packet
    server: the server's launch waits for the receive, whose grid did not count its CUs -- no barrier timeout"""
    rng = np.random.default_rng(5051)
    ctx = qpp.Context(0)
    try:
        recv = _Receiver(ctx, rng, 6000)
        n = 1 << 20
        descs, arena = qpp.make_batch(n, 1200, [recv.keys[0].slot, recv.keys[1].slot], seed=77)
        d_desc, d_arena, d_status = ctx.alloc(descs.nbytes), ctx.alloc(arena.nbytes), ctx.alloc(n)
        d_desc.upload(descs)
        d_arena.upload(arena)
        for rep in range(3):
            recv.arm()
            ctx.seal_batch(d_desc, n, d_arena, None, d_status)  # ~1 ms of device work ahead of the receive
            recv.run()
            k = recv.keys[(2 * rep) % len(recv.keys)]
            kk, iv, _ = k.material()
            pn = 1234 + rep
            header = bytes([0x40]) + rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
            payload = rng.integers(0, 256, 700, dtype=np.uint8).tobytes()
            sealed = b"".join(orc.seal(1, kk, orc.nonce(iv, pn), header, payload))
            assert k.decrypt(pn, header, sealed) == payload  # (starts the packet server on the first round)
            ctx.sync()
            recv.check()
            assert (d_status.download(dtype=np.int8) == 0).all()
            if rep == 0:
                ctx.set_packet_server(False)  # next rounds: the server is started afresh by the call
                ctx.set_packet_server(True)
        assert ctx.rx_timeouts() == 0
        assert ctx.packet_server_info()[0] >= 3
    finally:
        ctx.close()


def test_two_fused_receives_on_two_streams():
    """two fused receives of one context on two streams at once -- they run one after another (device
    registry), each with every workgroup resident: both bit-exact, no barrier timeout"""
    rng = np.random.default_rng(5052)
    ctx = qpp.Context(0)
    try:
        a = _Receiver(ctx, rng, 9000)
        b = _Receiver(ctx, rng, 7000)
        s1, s2 = ctx.new_stream(), ctx.new_stream()
        for rep in range(3):
            a.arm(s1)
            b.arm(s2)
            a.run(s1)
            b.run(s2)
            ctx.sync(s1)
            ctx.sync(s2)
            a.check()
            b.check()
        assert ctx.rx_timeouts() == 0
    finally:
        ctx.close()


def test_other_context_frees_and_syncs_do_not_wait_for_a_resident_server(monkeypatch):
    """hipFree / hipHostFree / hipDeviceSynchronize wait for every stream of the device, another context's resident
    server too (tools/diag/free_sync.hip: 1950 ms beside a 2-s kernel), and a context cannot stop another's servers.
    Context B keeps a persistent transmit queue and a packet server resident (20 s idle); context A allocates and frees
    device and pinned memory, grows its key table, synchronizes and closes: every call returns at once, and B's server
    was never restarted (its flushes before and after stay bit-exact on one server launch)."""
    monkeypatch.setenv("QPP_TXQ_SERVER_IDLE_MS", "20000")
    rng = np.random.default_rng(5053)
    b = qpp.Context(0)
    q = None
    try:
        kb = b.key(1, rng.integers(0, 256, 32, dtype=np.uint8).tobytes())
        q = qpp.TxQueue(b, 64 * STRIDE, 64, persistent=True)
        pn = [5000]

        def flush():
            want = []
            for i in range(64):
                header = bytes([0x43]) + rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
                payload = rng.integers(0, 256, 1100, dtype=np.uint8).tobytes()
                trunc, pn_len = qpp.pn_truncate(pn[0] + i, pn[0] - 1)
                pkt = header + trunc.to_bytes(pn_len, "big") + payload
                q.ring[i * STRIDE:i * STRIDE + len(pkt)] = np.frombuffer(pkt, dtype=np.uint8)
                q.push(kb, pn[0] + i, i * STRIDE, len(header), pn_len, len(payload))
                kk, iv, hp = kb.material()
                want.append((i * STRIDE, orc.protect_packet(1, kk, iv, hp, pn[0] + i, header, pn_len, payload)[1]))
            q.flush()
            for off, p in want:
                assert q.ring[off:off + len(p)].tobytes() == p
            pn[0] += 64

        flush()
        _seal_one(rng, kb, 1)  # B's packet server is resident too
        assert q.info()[2] == 1

        a = qpp.Context(0)
        times = {}

        def timed(name, f):
            t0 = time.perf_counter()
            r = f()
            times[name] = time.perf_counter() - t0
            return r

        d = timed("dev_alloc", lambda: a.alloc(1 << 24))
        d.upload(np.arange(1 << 24, dtype=np.uint64).astype(np.uint8))
        timed("dev_free", d.free)
        h = timed("host_alloc", lambda: a.host_alloc(1 << 20))
        timed("host_free", lambda: a.host_free(h))
        keys = timed("key_table_growth", lambda: [a.key(2, rng.integers(0, 256, 48, dtype=np.uint8).tobytes())
                                                  for _ in range(80)])  # past the 64-slot table: grow_keys
        descs, arena = qpp.make_batch(4096, 1200, [k.slot for k in keys], seed=9)
        da, dd, ds = a.alloc(arena.nbytes), a.alloc(descs.nbytes), a.alloc(4096)
        da.upload(arena)
        dd.upload(descs)
        a.seal_batch(dd, 4096, da, None, ds)
        timed("synchronize", a.synchronize)
        assert (ds.download(dtype=np.int8) == 0).all()
        _seal_one(rng, keys[0], 2)  # A's own packet server: stopped by its close below
        timed("close", a.close)
        print({k: round(1e3 * v, 2) for k, v in times.items()}, "ms")
        for name, dt in times.items():
            assert dt < 2.0, (name, dt)  # (the 20-s idle server of B would hold each for 20 s)

        flush()
        _seal_one(rng, kb, 1)
        served, launched, starts = q.info()
        assert (served, launched, starts) == (2, 0, 1)  # one server launch for both flushes: never stopped
        assert q.server_refused() == 0
    finally:
        if q is not None:
            q.close()
        b.close()
