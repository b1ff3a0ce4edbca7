"""Per-packet Key::encrypt / Key::decrypt (crypto/src/cipher_suite.rs:86-160, the packet_protection.rs trait face)
through the context's packet server (api.cpp packet_server_run; burst.hip txq_server_kernel, kTxsPktNoHp /
kTxsPktOpen items): bit-exact against the oracle and against the launched path, for every suite, header and payload
lengths from empty to the server's 16 KiB ring, tampered tags, keys spread over the server's workgroups, the server
stopped and restarted between calls, FIPS seals and long packets on the launched path."""
import time

import numpy as np
import pytest

import _oracle as orc
import qpp

pytestmark = pytest.mark.gpu

SUITES = (1, 2, 3)  # AES-128-GCM, AES-256-GCM, ChaCha20-Poly1305


def _lengths(rng):
    return [0, 1, 15, 16, 17, 63, 64, 65, 1000, 1184, 1200, 1452, 4096, 16384 - 64 - 16] + \
        [int(x) for x in rng.integers(0, 3000, 10)]


@pytest.mark.parametrize("suite", SUITES)
def test_server_seal_open_bit_exact(suite):
    rng = np.random.default_rng(7100 + suite)
    ctx = qpp.Context(0)
    try:
        keys = [ctx.key(suite, rng.integers(0, 256, qpp.HASH_LEN[suite], dtype=np.uint8).tobytes())
                for _ in range(6)]  # slots over all 4 server workgroups, two sharing one (key switches in its LDS)
        for i, ln in enumerate(_lengths(rng)):
            k = keys[i % len(keys)]
            kk, iv, _ = k.material()
            pn = int(rng.integers(0, 2**62))
            header = rng.integers(0, 256, int(rng.integers(1, 64)), dtype=np.uint8).tobytes()
            payload = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
            want = b"".join(orc.seal(suite, kk, orc.nonce(iv, pn), header, payload))
            got = k.encrypt(pn, header, payload)
            assert got == want, (suite, ln)
            assert k.decrypt(pn, header, got) == payload
            bad = bytearray(got)
            bad[int(rng.integers(0, len(bad)))] ^= 0x10
            with pytest.raises(qpp.DecryptError):
                k.decrypt(pn, header, bytes(bad))
        served, starts = ctx.packet_server_info()
        assert served >= 3 * len(_lengths(rng)) and starts >= 1
    finally:
        ctx.close()


def test_server_matches_launched_path():
    rng = np.random.default_rng(7200)
    on, off = qpp.Context(0), qpp.Context(0)
    try:
        off.set_packet_server(False)
        for suite in SUITES:
            secret = rng.integers(0, 256, qpp.HASH_LEN[suite], dtype=np.uint8).tobytes()
            a, b = on.key(suite, secret), off.key(suite, secret)
            for ln in (0, 5, 300, 1200, 3000):
                pn = int(rng.integers(0, 2**40))
                header = rng.integers(0, 256, 21, dtype=np.uint8).tobytes()
                payload = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
                ct = a.encrypt(pn, header, payload)
                assert ct == b.encrypt(pn, header, payload)
                assert a.decrypt(pn, header, ct) == b.decrypt(pn, header, ct) == payload
        assert on.packet_server_info()[0] > 0 and off.packet_server_info() == (0, 0)
    finally:
        on.close()
        off.close()


def test_server_restarts_and_long_packets(monkeypatch):
    """the server leaves on its idle time, or is switched off and on; the next call restarts it.  A packet over the
    ring (16 KiB) and a FIPS seal take the launched path, identical bytes."""
    monkeypatch.setenv("QPP_TXQ_SERVER_IDLE_MS", "20")
    rng = np.random.default_rng(7300)
    ctx = qpp.Context(0)
    try:
        k = ctx.key(1, rng.integers(0, 256, 32, dtype=np.uint8).tobytes())
        kk, iv, _ = k.material()
        header = bytes(21)

        def one(pn, ln):
            payload = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
            ct = k.encrypt(pn, header, payload)
            assert ct == b"".join(orc.seal(1, kk, orc.nonce(iv, pn), header, payload))
            assert k.decrypt(pn, header, ct) == payload

        one(1, 1200)
        s0 = ctx.packet_server_info()[1]
        time.sleep(0.1)  # past the idle time: the server left
        one(2, 1200)
        assert ctx.packet_server_info()[1] >= s0 + 1
        ctx.set_packet_server(False)  # stopped ...
        ctx.set_packet_server(True)
        one(3, 1200)  # ... and started again by the next call
        assert ctx.packet_server_info()[1] >= s0 + 2
        served = ctx.packet_server_info()[0]
        one(4, 20000)  # over the ring: launched
        assert ctx.packet_server_info()[0] == served
        ctx.set_fips(True)
        f = ctx.key(1, rng.integers(0, 256, 32, dtype=np.uint8).tobytes())
        fk, fiv, _ = f.material()
        payload = bytes(range(200))
        assert f.encrypt(10, header, payload) == b"".join(orc.seal(1, fk, orc.nonce(fiv, 10), header, payload))
        assert ctx.packet_server_info()[0] == served  # FIPS seal: launched (nonce-order gate)
        with pytest.raises(qpp.QppError):
            f.encrypt(10, header, payload)  # the same packet number again: refused
    finally:
        ctx.close()


def test_device_free_keeps_the_server(monkeypatch):
    """device and pinned frees leave the packet server resident (one launch for every call): hipFree / hipHostFree
    would wait for it, so a buffer freed while a server of the device is resident is parked and freed by the next
    synchronize that finds none (api.cpp release)"""
    monkeypatch.setenv("QPP_TXQ_SERVER_IDLE_MS", "10000")
    rng = np.random.default_rng(7301)
    ctx = qpp.Context(0)
    try:
        k = ctx.key(1, rng.integers(0, 256, 32, dtype=np.uint8).tobytes())
        kk, iv, _ = k.material()
        header = bytes(21)

        def one(pn):
            payload = rng.integers(0, 256, 700, dtype=np.uint8).tobytes()
            assert k.encrypt(pn, header, payload) == b"".join(orc.seal(1, kk, orc.nonce(iv, pn), header, payload))

        one(1)
        starts = ctx.packet_server_info()[1]
        for i in range(5):
            b = ctx.alloc(1 << 20)
            b.upload(np.full(1 << 20, i, dtype=np.uint8))
            b.free()
            one(2 + i)
            h = ctx.host_alloc(1 << 16)
            h[:] = i
            ctx.host_free(h)
            one(20 + i)
        assert ctx.packet_server_info()[1] == starts
        ctx.synchronize()  # stops the server, frees what was parked
        one(40)
        assert ctx.packet_server_info()[1] == starts + 1
    finally:
        ctx.close()


@pytest.mark.parametrize("suite", SUITES)
def test_server_header_protection_masks(suite):
    """HeaderKey::*_header_protection_mask (header_key.rs:52-56) of packet keys and header-key-only records through the
    server's mask items, interleaved with seals of the same packet key (the mask's key words are cached apart from the
    packet key's in the workgroup's LDS): every mask and every seal bit-exact"""
    rng = np.random.default_rng(7400 + suite)
    ctx = qpp.Context(0)
    try:
        k = ctx.key(suite, rng.integers(0, 256, qpp.HASH_LEN[suite], dtype=np.uint8).tobytes())
        kk, iv, hp = k.material()
        hp2 = rng.integers(0, 256, len(hp), dtype=np.uint8).tobytes()
        hk = ctx.header_key(suite, hp=hp2)
        calls0 = ctx.packet_server_info()[0]
        for i in range(24):
            sample = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
            assert k.header_protection_mask(sample) == orc.hp_mask(suite, hp, sample)[:5]
            assert hk.header_protection_mask(sample) == orc.hp_mask(suite, hp2, sample)[:5]
            payload = rng.integers(0, 256, int(rng.integers(0, 1500)), dtype=np.uint8).tobytes()
            header = rng.integers(0, 256, 21, dtype=np.uint8).tobytes()
            assert k.encrypt(i, header, payload) == b"".join(orc.seal(suite, kk, orc.nonce(iv, i), header, payload))
        assert ctx.packet_server_info()[0] - calls0 == 3 * 24
        hk.free()
    finally:
        ctx.close()


def test_parked_bound_stops_own_server(monkeypatch):
    """past the parked-memory bound (QPP_PARKED_MAX_MB, here 1 MiB) a free stops the context's own servers and frees
    at once (no other context's server is resident): it returns promptly, the bytes stay right, the next call
    restarts the server"""
    import subprocess
    import sys
    code = r'''
import time, numpy as np, qpp, _oracle as orc
rng = np.random.default_rng(7302)
ctx = qpp.Context(0)
k = ctx.key(1, rng.integers(0, 256, 32, dtype=np.uint8).tobytes())
kk, iv, _ = k.material()
def one(pn):
    payload = rng.integers(0, 256, 700, dtype=np.uint8).tobytes()
    assert k.encrypt(pn, bytes(21), payload) == b"".join(orc.seal(1, kk, orc.nonce(iv, pn), bytes(21), payload))
one(1)
s0 = ctx.packet_server_info()[1]
small = ctx.alloc(1 << 16)
small.free()  # under the bound: parked, the server stays
one(2)
assert ctx.packet_server_info()[1] == s0
big = ctx.alloc(4 << 20)
t0 = time.perf_counter()
big.free()  # over the bound: own server stopped, freed now
dt = time.perf_counter() - t0
assert dt < 1.0, dt
one(3)
assert ctx.packet_server_info()[1] == s0 + 1
ctx.close()
print("ok", round(dt * 1e3, 2), "ms")
'''
    import os
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, QPP_PARKED_MAX_MB="1", QPP_TXQ_SERVER_IDLE_MS="10000",
               PYTHONPATH=os.pathsep.join([here, os.path.join(os.path.dirname(here), "s2n-quic_amd")]))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=100, cwd=here)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok" in r.stdout


def test_free_past_bound_evicts_other_contexts_fed_server():
    """past the parked-memory bound (QPP_PARKED_MAX_MB=1) a free of context A must not wait for context
    B's resident server while a thread keeps feeding it (hipFree waits for every stream of the device: it would wait
    for B's idle exit, i.e. for ever).  Every A free (device and pinned, 4 MiB each: over the bound every time) returns
    in < 1 s; every B flush (64 x 100-1200 B, AES-128, persistent server) is bit-exact; the evictions are counted and
    B's server is relaunched after them.  Runs in a child process (the bound is read once per process)."""
    import os
    import subprocess
    import sys
    code = r'''
import threading, time, numpy as np, qpp, _oracle as orc
STRIDE = 1536
rng = np.random.default_rng(7303)
stop = time.perf_counter() + 4.0
errs, flushes = [], [0]
started = threading.Event()
def feeder():
    try:
        ctx = qpp.Context(0)
        k = ctx.key(1, rng.integers(0, 256, 32, dtype=np.uint8).tobytes())
        kk, iv, hp = k.material()
        q = qpp.TxQueue(ctx, 64 * STRIDE, 64, persistent=True)
        pn = 5000
        while time.perf_counter() < stop:
            want = []
            for i in range(64):
                header = bytes([0x43]) + rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
                payload = rng.integers(0, 256, int(rng.integers(100, 1200)), dtype=np.uint8).tobytes()
                trunc, pn_len = qpp.pn_truncate(pn + i, pn - 1)
                pkt = header + trunc.to_bytes(pn_len, "big") + payload
                q.ring[i * STRIDE:i * STRIDE + len(pkt)] = np.frombuffer(pkt, dtype=np.uint8)
                q.push(k, pn + i, i * STRIDE, len(header), pn_len, len(payload))
                want.append((i * STRIDE, orc.protect_packet(1, kk, iv, hp, pn + i, header, pn_len, payload)[1]))
            q.flush()
            for off, p in want:
                assert q.ring[off:off + len(p)].tobytes() == p, ("flush", flushes[0])
            pn += 64
            flushes[0] += 1
            started.set()
        info = q.info()
        assert q.server_refused() == 0
        q.close()
        ctx.close()
        flushes.append(info)
    except BaseException as e:
        errs.append(repr(e))
        started.set()
t = threading.Thread(target=feeder, daemon=True)
t.start()
started.wait(60)
a = qpp.Context(0)
e0 = qpp.server_evictions(0)
worst, n = 0.0, 0
while time.perf_counter() < stop - 0.5 and not errs:
    b = a.alloc(4 << 20)
    b.upload(np.full(4 << 20, n & 0xff, dtype=np.uint8))
    t0 = time.perf_counter(); b.free(); worst = max(worst, time.perf_counter() - t0)
    h = a.host_alloc(4 << 20)
    h[:] = n & 0xff
    t0 = time.perf_counter(); a.host_free(h); worst = max(worst, time.perf_counter() - t0)
    n += 1
    time.sleep(0.05)
t.join(60)
assert not t.is_alive(), "feeder stuck"
assert not errs, errs
e1 = qpp.server_evictions(0)
a.close()
assert worst < 1.0, worst
assert e1[0] > e0[0], (e0, e1)
srv, launched, starts = flushes[-1]
assert srv > 0 and starts >= 2, flushes[-1]
print("ok frees", n, "worst_ms", round(worst * 1e3, 2), "flushes", flushes[0], "server", srv, "launched", launched,
      "starts", starts, "evictions", e1[0] - e0[0], "oneshots", e1[1] - e0[1])
'''
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, QPP_PARKED_MAX_MB="1", QPP_TXQ_SERVER_IDLE_MS="20000",
               PYTHONPATH=os.pathsep.join([here, os.path.join(os.path.dirname(here), "s2n-quic_amd")]))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=110, cwd=here)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok" in r.stdout
