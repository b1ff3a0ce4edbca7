"""Contexts driven from several host threads at once.

The reference's keys are `Send` objects that any endpoint task may own (quic/s2n-quic-core/src/crypto/key.rs:8), and
a server process runs one endpoint event loop per thread (quic/s2n-quic-core/src/io/event_loop.rs:39-165): so several
contexts of one process call the library concurrently.  ctypes releases the GIL for every library call, so the three
threads below really overlap inside api.cpp: per-packet seals through a packet server with device and pinned frees in
between (the parked-free path, api.cpp release), persistent transmit-queue flushes with key-table growth (a server
stop, a table move, the old table released), and 64-key fused receives with context synchronizes (the device
registry's lock: receive grids, server slots, server starts behind the latest receive).
Bar: every byte bit-exact, no receive barrier timeout, no thread stuck (each finishes within its budget).
"""
import threading
import time

import numpy as np
import pytest

import _oracle as orc
import qpp
from test_gpu_servers_device import STRIDE, _Receiver, _seal_one

pytestmark = pytest.mark.gpu

RUN_S = 4.0


def test_three_threads_three_contexts(monkeypatch):
    monkeypatch.setenv("QPP_TXQ_SERVER_IDLE_MS", "2000")
    errors, counts = [], {}
    stop = time.perf_counter() + RUN_S

    def guarded(name, fn):
        def run():
            try:
                counts[name] = fn()
            except BaseException as e:  # (reported below, with the thread's name)
                errors.append((name, repr(e)))
        return run

    def per_packet():
        rng = np.random.default_rng(6001)
        ctx = qpp.Context(0)
        n = 0
        try:
            keys = [ctx.key(s, rng.integers(0, 256, qpp.HASH_LEN[s], dtype=np.uint8).tobytes()) for s in (1, 2, 3)]
            while time.perf_counter() < stop:
                k = keys[n % 3]
                _seal_one(rng, k, k.suite)
                n += 1
                if n % 40 == 0:  # frees while servers of the device are resident (own and the other contexts')
                    b = ctx.alloc(1 << 20)
                    b.upload(np.full(1 << 20, n & 0xff, dtype=np.uint8))
                    b.free()
                    h = ctx.host_alloc(1 << 16)
                    h[:] = n & 0xff
                    ctx.host_free(h)
        finally:
            ctx.close()
        return n

    def flusher():
        rng = np.random.default_rng(6002)
        ctx = qpp.Context(0)
        q = None
        n = 0
        try:
            k = ctx.key(1, rng.integers(0, 256, 32, dtype=np.uint8).tobytes())
            q = qpp.TxQueue(ctx, 64 * STRIDE, 64, persistent=True)
            more = []
            pn = 1000
            while time.perf_counter() < stop:
                want = []
                for i in range(64):
                    header = bytes([0x43]) + rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
                    payload = rng.integers(0, 256, int(rng.integers(100, 1200)), dtype=np.uint8).tobytes()
                    trunc, pn_len = qpp.pn_truncate(pn + i, pn - 1)
                    pkt = header + trunc.to_bytes(pn_len, "big") + payload
                    q.ring[i * STRIDE:i * STRIDE + len(pkt)] = np.frombuffer(pkt, dtype=np.uint8)
                    q.push(k, pn + i, i * STRIDE, len(header), pn_len, len(payload))
                    kk, iv, hp = k.material()
                    want.append((i * STRIDE, orc.protect_packet(1, kk, iv, hp, pn + i, header, pn_len, payload)[1]))
                q.flush()
                for off, p in want:
                    assert q.ring[off:off + len(p)].tobytes() == p
                pn += 64
                n += 1
                if n % 15 == 0 and len(more) < 300:  # grow the key table (64 -> 128 -> 256 ... slots)
                    more += [ctx.key(1, rng.integers(0, 256, 32, dtype=np.uint8).tobytes()) for _ in range(70)]
            assert q.server_refused() == 0
        finally:
            if q is not None:
                q.close()
            ctx.close()
        return n

    def receiver():
        rng = np.random.default_rng(6003)
        ctx = qpp.Context(0)
        n = 0
        try:
            recv = _Receiver(ctx, rng, 3000)
            while time.perf_counter() < stop:
                recv.arm()
                recv.run()
                ctx.sync()
                recv.check()
                n += 1
                if n % 5 == 0:
                    ctx.synchronize()
            assert ctx.rx_timeouts() == 0
        finally:
            ctx.close()
        return n

    threads = [threading.Thread(target=guarded(f.__name__, f), name=f.__name__, daemon=True)
               for f in (per_packet, flusher, receiver)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=RUN_S + 60)
    stuck = [t.name for t in threads if t.is_alive()]
    assert not stuck, f"threads still running: {stuck}"
    assert not errors, errors
    print("calls per thread:", counts)
    assert all(counts.get(name, 0) > 3 for name in ("per_packet", "flusher", "receiver")), counts
