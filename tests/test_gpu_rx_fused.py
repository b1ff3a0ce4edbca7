"""The fused receive kernel (quad.hip aes_gcm_quad_rx_kernel: unprotect -> PN expand -> key-phase choice -> group by
key -> open, ONE cooperative launch for any mix of live AES keys of both sizes, plus one ChaCha20 launch behind it on
the same stream when ChaCha20 keys are live) against the multi-launch path (unprotect_kernel + plan + open,
QPP_RX_FUSED=0) and against the oracle (orc_unprotect_open_batch).

The batch is what a receiver sees during a key update (quic/s2n-quic-core/src/crypto/application/keyset.rs:113-143):
short headers of both key phases and long headers, PNs truncated against the largest acknowledged PN, tampered tags,
packets too short for the HP sample.  The phase-1 key has already been dropped, so its packets are refused
(INTERNAL_ERROR) with their header unprotected and their payload untouched.  Bar: the two paths equal bit for bit
(arena, descriptors out, status), and every packet the oracle opens is bit-exact with it.
"""
import numpy as np
import pytest

import _oracle as orc
import qpp

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = qpp.Context(0)
    yield c
    c.close()


def _batch(rng, okeys_mat, slots, n):
    chunks, rx, orx = [], [], []
    off = 0
    for i in range(n):
        largest = int(rng.integers(0, 2**62 - 2**20)) if i % 3 else int(rng.integers(0, 300))
        pn = largest + int(rng.integers(0, 400))
        _, _, pn_len = orc.truncate_pn(pn, largest)
        pn_len = min(4, pn_len + int(rng.integers(0, 2)))
        long_hdr = i % 5 == 0
        phase = 0 if long_hdr else int(i % 4 == 1)
        if long_hdr:
            first = 0xc0 | (int(rng.integers(0, 4)) << 4) | (pn_len - 1)
            rest = rng.integers(0, 256, int(rng.integers(6, 40)), dtype=np.uint8).tobytes()
        else:
            first = 0x40 | (phase << 2) | (pn_len - 1)
            rest = rng.integers(0, 256, int(rng.integers(0, 21)), dtype=np.uint8).tobytes()
        header = bytes([first]) + rest
        pt = int(rng.integers(max(0, 4 - pn_len), 1400)) if i % 7 else max(0, 4 - pn_len)
        payload = rng.integers(0, 256, pt, dtype=np.uint8).tobytes()
        suite, k, iv, hp = okeys_mat[phase]
        rc, pkt = orc.protect_packet(suite, k, iv, hp, pn, header, pn_len, payload)
        assert rc == 0
        pkt = bytearray(pkt)
        if i % 11 == 3:
            pkt[-1 - i % 16] ^= 0x20  # tampered -> DECRYPT_ERROR
        length = len(pkt)
        if i % 13 == 5:
            length = len(header) + 19  # no room for the sample -> DECODE_ERROR
            pkt = pkt[:length]
        chunks.append(bytes(pkt) + bytes(int(rng.integers(0, 7))))
        rx.append((largest, (slots[0], slots[1]), off, len(header), length))
        orx.append((largest, (0, 1), off, len(header), length))
        off += len(chunks[-1])
    arena = np.frombuffer(b"".join(chunks) + bytes(64), dtype=np.uint8).copy()
    return np.array(rx, dtype=qpp.RX_DTYPE), np.array(orx, dtype=qpp.RX_DTYPE), arena


def _run(ctx, rx, arena, monkeypatch, fused):
    monkeypatch.setenv("QPP_RX_FUSED", "1" if fused else "0")
    n = len(rx)
    d_rx, d_arena = ctx.alloc(rx.nbytes), ctx.alloc(arena.nbytes)
    d_out, d_status = ctx.alloc(n * qpp.PKT_DTYPE.itemsize), ctx.alloc(n)
    d_rx.upload(rx)
    d_arena.upload(arena)
    d_status.upload(np.full(n, 99, dtype=np.int8))
    ctx.unprotect_open_batch(d_rx, n, d_arena, d_out, d_status)
    ctx.sync()
    out = d_arena.download(), d_out.download(dtype=qpp.PKT_DTYPE), d_status.download(dtype=np.int8)
    for b in (d_rx, d_arena, d_out, d_status):
        b.free()
    return out


@pytest.mark.parametrize("suite", [1, 2])
def test_fused_rx_equals_two_launch_path_and_oracle(ctx, suite, monkeypatch):
    rng = np.random.default_rng(40 + suite)
    ctx.set_burst_max(0)  # quad-kernel batches at test size (the fused path is the quad kernel's)
    try:
        k0 = ctx.key(suite, rng.integers(0, 256, qpp.HASH_LEN[suite], dtype=np.uint8).tobytes())
        k1 = k0.derive_next_key()
        mats = [(suite, *k0.material()), (suite, *k1.material())]
        slots = [k0.slot, k1.slot]
        n = 3000
        rx, orx, arena = _batch(rng, mats, slots, n)
        k1.free()  # the old phase's key is gone: k0 is the context's only live packet key -> the fused kernel
        a_f, o_f, s_f = _run(ctx, rx, arena, monkeypatch, fused=True)
        a_2, o_2, s_2 = _run(ctx, rx, arena, monkeypatch, fused=False)
        assert (s_f == s_2).all(), "status differs between the fused and the two-launch path"
        assert (a_f == a_2).all(), "arena differs between the fused and the two-launch path"
        assert (o_f.view(np.uint8) == o_2.view(np.uint8)).all(), "descriptors differ"

        want_arena = arena.copy()
        want_out, want_st = orc.unprotect_open_batch(orc.make_keys(mats), orx, want_arena)
        want_st = np.array(want_st, dtype=np.int8)
        phase1 = (want_out["key_idx"] == 1) & (want_st != qpp.DECODE_ERROR)
        assert phase1.sum() > 100 and (s_f[phase1] == qpp.INTERNAL_ERROR).all()
        assert (s_f[~phase1] == want_st[~phase1]).all()
        assert (s_f == 0).sum() > n // 2 and (s_f == qpp.DECRYPT_ERROR).any() and (s_f == qpp.DECODE_ERROR).any()
        for f in ("pn", "aad_len", "pt_len", "pn_len", "flags", "off"):
            assert (o_f[f] == want_out[f]).all(), f
        assert (o_f["key_idx"] == np.where(want_out["key_idx"] == 1, slots[1], slots[0])).all()
        for i in range(n):
            o, ln, aad = int(rx[i]["off"]), int(rx[i]["len"]), int(want_out[i]["aad_len"])
            if phase1[i]:  # header unprotected as the oracle did, payload || tag as received
                assert (a_f[o:o + aad] == want_arena[o:o + aad]).all()
                assert (a_f[o + aad:o + ln] == arena[o + aad:o + ln]).all()
            else:
                assert (a_f[o:o + ln] == want_arena[o:o + ln]).all(), i
        k0.free()
    finally:
        ctx.set_burst_max(16384)


@pytest.mark.parametrize("suite", [1, 2])
def test_fused_rx_local_and_planned_slices(ctx, suite, monkeypatch):
    """Local slices beside planned ones in one launch: the first half of the batch is one connection's phase-0 packets
    only (some tampered), so every workgroup slice there has one key and opens itself right after phase A; the second
    half mixes both live phases (a key update in progress) and long headers, so those slices go through the global
    plan (counts, scan, scatter) -- and the last slice can be either.  Bit-exact with the multi-launch path and the
    oracle; no barrier timeout."""
    rng = np.random.default_rng(140 + suite)
    ctx.set_burst_max(0)
    try:
        k0 = ctx.key(suite, rng.integers(0, 256, qpp.HASH_LEN[suite], dtype=np.uint8).tobytes())
        k1 = k0.derive_next_key()
        mats = [(suite, *k0.material()), (suite, *k1.material())]
        n = 6000
        chunks, rx, orx = [], [], []
        off = 0
        for i in range(n):
            largest = int(rng.integers(0, 2**40))
            pn = largest + int(rng.integers(0, 300))
            _, _, pn_len = orc.truncate_pn(pn, largest)
            uniform = i < n // 2
            phase = 0 if uniform else int(rng.integers(0, 2))
            if not uniform and i % 5 == 0:
                first = 0xc0 | (int(rng.integers(0, 4)) << 4) | (pn_len - 1)
                header = bytes([first]) + rng.integers(0, 256, int(rng.integers(6, 40)), dtype=np.uint8).tobytes()
                phase = 0
            else:
                header = bytes([0x40 | (phase << 2) | (pn_len - 1)]) + rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
            payload = rng.integers(0, 256, int(rng.integers(4, 1400)), dtype=np.uint8).tobytes()
            _, k, iv, hp = mats[phase]
            rc, pkt = orc.protect_packet(suite, k, iv, hp, pn, header, pn_len, payload)
            assert rc == 0
            pkt = bytearray(pkt)
            if i % 23 == 6:
                pkt[-1 - i % 16] ^= 0x04  # tampered -> DECRYPT_ERROR (still a local slice's packet)
            chunks.append(bytes(pkt) + bytes(int(rng.integers(0, 5))))
            rx.append((largest, (k0.slot, k1.slot), off, len(header), len(pkt)))
            orx.append((largest, (0, 1), off, len(header), len(pkt)))
            off += len(chunks[-1])
        rx, orx = np.array(rx, dtype=qpp.RX_DTYPE), np.array(orx, dtype=qpp.RX_DTYPE)
        arena = np.frombuffer(b"".join(chunks) + bytes(64), dtype=np.uint8).copy()
        t0 = ctx.rx_timeouts()
        a_f, o_f, s_f = _run(ctx, rx, arena, monkeypatch, fused=True)
        a_2, o_2, s_2 = _run(ctx, rx, arena, monkeypatch, fused=False)
        assert ctx.rx_timeouts() == t0
        assert (s_f == s_2).all(), "status differs between the fused and the multi-launch path"
        assert (a_f == a_2).all(), "arena differs between the fused and the multi-launch path"
        assert (o_f.view(np.uint8) == o_2.view(np.uint8)).all(), "descriptors differ"
        want_arena = arena.copy()
        want_out, want_st = orc.unprotect_open_batch(orc.make_keys(mats), orx, want_arena)
        want_st = np.array(want_st, dtype=np.int8)
        assert (s_f == want_st).all()
        assert (s_f == 0).sum() > n * 9 // 10 and (s_f == qpp.DECRYPT_ERROR).sum() > 100
        assert (a_f == want_arena).all()
        k1.free()
        k0.free()
    finally:
        ctx.set_burst_max(16384)


@pytest.mark.parametrize("suite", [1, 2])
def test_fused_rx_many_keys(suite, monkeypatch):
    """64 live packet keys (32 connections, both key phases live: a key update in progress everywhere), 4 more
    connections whose phase-1 key is already dropped, packets of all of them interleaved at random in one GRO batch:
    one fused launch (in-kernel group-by on the phase-chosen key) equals the multi-launch path bit for bit and the
    oracle on every packet (refused phase-1 packets of the 4 connections: INTERNAL_ERROR, payload untouched)."""
    rng = np.random.default_rng(90 + suite)
    ctx = qpp.Context(0)
    ctx.set_burst_max(0)
    ctx.set_aes_kernel(qpp.AES_KERNEL_QUAD)  # the throughput kernel's regime at test size (fused path's condition)
    try:
        pairs = []
        for c in range(36):
            k0 = ctx.key(suite, rng.integers(0, 256, qpp.HASH_LEN[suite], dtype=np.uint8).tobytes())
            pairs.append((k0, k0.derive_next_key()))
        mats = [(suite, *k.material()) for pair in pairs for k in pair]
        slots = [(p[0].slot, p[1].slot) for p in pairs]  # (a freed key's handle has no slot any more)
        for c in range(32, 36):
            pairs[c][1].free()
        n = 6000
        chunks, rx, orx = [], [], []
        off = 0
        for i in range(n):
            c = int(rng.integers(0, 36))
            largest = int(rng.integers(0, 2**40))
            pn = largest + int(rng.integers(0, 300))
            _, _, pn_len = orc.truncate_pn(pn, largest)
            phase = int(rng.integers(0, 2))
            header = bytes([0x40 | (phase << 2) | (pn_len - 1)]) + rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
            payload = rng.integers(0, 256, int(rng.integers(1, 1400)), dtype=np.uint8).tobytes()
            _, k, iv, hp = mats[2 * c + phase]
            rc, pkt = orc.protect_packet(suite, k, iv, hp, pn, header, pn_len, payload)
            pkt = bytearray(pkt)
            if i % 19 == 4:
                pkt[-1 - i % 16] ^= 0x01  # tampered -> DECRYPT_ERROR
            chunks.append(bytes(pkt) + bytes(int(rng.integers(0, 5))))
            rx.append((largest, slots[c], off, len(header), len(pkt)))
            orx.append((largest, (2 * c, 2 * c + 1), off, len(header), len(pkt)))
            off += len(chunks[-1])
        rx = np.array(rx, dtype=qpp.RX_DTYPE)
        orx = np.array(orx, dtype=qpp.RX_DTYPE)
        arena = np.frombuffer(b"".join(chunks) + bytes(64), dtype=np.uint8).copy()
        a_f, o_f, s_f = _run(ctx, rx, arena, monkeypatch, fused=True)
        a_2, o_2, s_2 = _run(ctx, rx, arena, monkeypatch, fused=False)
        assert (s_f == s_2).all(), "status differs between the fused and the multi-launch path"
        assert (a_f == a_2).all(), "arena differs between the fused and the multi-launch path"
        assert (o_f.view(np.uint8) == o_2.view(np.uint8)).all(), "descriptors differ"
        want_arena = arena.copy()
        want_out, want_st = orc.unprotect_open_batch(orc.make_keys(mats), orx, want_arena)
        want_st = np.array(want_st, dtype=np.int8)
        dropped = np.isin(want_out["key_idx"], [2 * c + 1 for c in range(32, 36)])
        assert dropped.sum() > 100 and (s_f[dropped] == qpp.INTERNAL_ERROR).all()
        assert (s_f[~dropped] == want_st[~dropped]).all()
        assert (s_f == 0).sum() > n * 3 // 4 and (s_f == qpp.DECRYPT_ERROR).any()
        for i in np.nonzero(~dropped)[0]:
            o, ln = int(rx[i]["off"]), int(rx[i]["len"])
            assert (a_f[o:o + ln] == want_arena[o:o + ln]).all(), i
    finally:
        ctx.close()


def test_fused_chacha_rx_many_keys(monkeypatch):
    """No AES record live: the ChaCha lane kernel unprotects and opens in one launch whatever the key mix (per-lane
    keys).  Three connections, each with both key phases; connection 1 has dropped its phase-1 key (its phase-1
    packets are refused), and some packets name a freed header-key slot (refused before any byte is touched).  The
    fused launch equals the two-launch path bit for bit and the oracle on every packet it opens."""
    rng = np.random.default_rng(77)
    ctx = qpp.Context(0)  # a context of its own: no AES key may be live
    ctx.set_burst_max(0)
    try:
        conns = []
        for _ in range(3):
            k0 = ctx.key(3, rng.integers(0, 256, 32, dtype=np.uint8).tobytes())
            conns.append((k0, k0.derive_next_key()))
        gone = ctx.key(3, rng.integers(0, 256, 32, dtype=np.uint8).tobytes())
        gone_slot = gone.slot
        mats = [(3, *k.material()) for pair in conns for k in pair]
        n = 4000
        chunks, rx, orx = [], [], []
        off = 0
        for i in range(n):
            c = int(rng.integers(0, 3))
            largest = int(rng.integers(0, 2**40))
            pn = largest + int(rng.integers(0, 300))
            _, _, pn_len = orc.truncate_pn(pn, largest)
            phase = int(rng.integers(0, 2))
            header = bytes([0x40 | (phase << 2) | (pn_len - 1)]) + rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
            payload = rng.integers(0, 256, int(rng.integers(1, 1400)), dtype=np.uint8).tobytes()
            _, k, iv, hp = mats[2 * c + phase]
            rc, pkt = orc.protect_packet(3, k, iv, hp, pn, header, pn_len, payload)
            pkt = bytearray(pkt)
            if i % 17 == 4:
                pkt[-3] ^= 1  # tampered tag
            chunks.append(bytes(pkt) + bytes(int(rng.integers(0, 5))))
            slots = (conns[c][0].slot, conns[c][1].slot)
            if i % 29 == 7:
                slots = (gone_slot, slots[1])  # a header-key slot that was freed
            rx.append((largest, slots, off, len(header), len(pkt)))
            orx.append((largest, (2 * c, 2 * c + 1), off, len(header), len(pkt)))
            off += len(chunks[-1])
        arena = np.frombuffer(b"".join(chunks) + bytes(64), dtype=np.uint8).copy()
        rx, orx = np.array(rx, dtype=qpp.RX_DTYPE), np.array(orx, dtype=qpp.RX_DTYPE)
        gone.free()
        conns[1][1].free()  # connection 1 dropped its phase-1 key
        a_f, o_f, s_f = _run(ctx, rx, arena, monkeypatch, fused=True)
        a_2, o_2, s_2 = _run(ctx, rx, arena, monkeypatch, fused=False)
        assert (s_f == s_2).all() and (a_f == a_2).all() and (o_f.view(np.uint8) == o_2.view(np.uint8)).all()
        want_arena = arena.copy()
        want_out, want_st = orc.unprotect_open_batch(orc.make_keys(mats), orx, want_arena)
        want_st = np.array(want_st, dtype=np.int8)
        freed_hdr = np.arange(n) % 29 == 7
        dropped = ~freed_hdr & (want_out["key_idx"] == 3)  # connection 1, phase 1
        assert freed_hdr.sum() > 100 and dropped.sum() > 300
        assert (s_f[freed_hdr | dropped] == qpp.INTERNAL_ERROR).all()
        ok = ~(freed_hdr | dropped)
        assert (s_f[ok] == want_st[ok]).all() and (s_f == qpp.DECRYPT_ERROR).any() and (s_f == 0).sum() > n // 2
        for i in np.flatnonzero(ok | freed_hdr):
            o, ln = int(rx[i]["off"]), int(rx[i]["len"])
            src = arena if freed_hdr[i] else want_arena  # a freed header key: nothing touched
            assert (a_f[o:o + ln] == src[o:o + ln]).all(), i
        for f in ("pn", "aad_len", "pt_len", "pn_len", "off"):
            assert (o_f[f][ok] == want_out[f][ok]).all(), f
        for k0, k1 in conns:
            k0.free()
            if k1.handle:
                k1.free()
    finally:
        ctx.close()


@pytest.mark.parametrize("only_aes", [False, True])
def test_fused_rx_mixed_suites(monkeypatch, only_aes):
    """A server whose clients negotiated all three suites (cipher_suite/negotiated.rs:15-125): 18 connections, 6 per
    suite, both key phases live, one connection per suite with its phase-1 key dropped; one GRO batch of their packets
    at random.  The fused path (one cooperative launch for the AES packets of both sizes, the ChaCha20 packets opened by
    one more launch on the stream) equals the multi-launch path bit for bit and the oracle on every packet.  With
    QPP_ONLY_AES both paths leave the ChaCha20 packets' status alone (header unprotected, payload untouched); a packet
    whose chosen key was dropped is INTERNAL_ERROR either way."""
    rng = np.random.default_rng(120 + only_aes)
    ctx = qpp.Context(0)
    ctx.set_burst_max(0)
    ctx.set_aes_kernel(qpp.AES_KERNEL_QUAD)  # the quad regime at test size (the fused path's condition)
    try:
        suites = [1, 2, 3] * 6
        pairs = []
        for s_ in suites:
            k0 = ctx.key(s_, rng.integers(0, 256, qpp.HASH_LEN[s_], dtype=np.uint8).tobytes())
            pairs.append((k0, k0.derive_next_key()))
        mats = [(k.suite, *k.material()) for pair in pairs for k in pair]
        slots = [(p[0].slot, p[1].slot) for p in pairs]
        dropped_conn = [0, 1, 2]  # one connection of each suite dropped its phase-1 key
        for c in dropped_conn:
            pairs[c][1].free()
        n = 6000
        chunks, rx, orx = [], [], []
        off = 0
        for i in range(n):
            c = int(rng.integers(0, len(pairs)))
            largest = int(rng.integers(0, 2**40))
            pn = largest + int(rng.integers(0, 300))
            _, _, pn_len = orc.truncate_pn(pn, largest)
            phase = int(rng.integers(0, 2))
            header = bytes([0x40 | (phase << 2) | (pn_len - 1)]) + rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
            payload = rng.integers(0, 256, int(rng.integers(1, 1400)), dtype=np.uint8).tobytes()
            s_, k, iv, hp = mats[2 * c + phase]
            _, pkt = orc.protect_packet(s_, k, iv, hp, pn, header, pn_len, payload)
            pkt = bytearray(pkt)
            if i % 19 == 4:
                pkt[-1 - i % 16] ^= 0x01  # tampered -> DECRYPT_ERROR
            chunks.append(bytes(pkt) + bytes(int(rng.integers(0, 5))))
            rx.append((largest, slots[c], off, len(header), len(pkt)))
            orx.append((largest, (2 * c, 2 * c + 1), off, len(header), len(pkt)))
            off += len(chunks[-1])
        rx = np.array(rx, dtype=qpp.RX_DTYPE)
        orx = np.array(orx, dtype=qpp.RX_DTYPE)
        arena = np.frombuffer(b"".join(chunks) + bytes(64), dtype=np.uint8).copy()
        flags = qpp.ONLY_AES if only_aes else 0

        def run(fused):
            monkeypatch.setenv("QPP_RX_FUSED", "1" if fused else "0")
            d_rx, d_arena = ctx.alloc(rx.nbytes), ctx.alloc(arena.nbytes)
            d_out, d_status = ctx.alloc(n * qpp.PKT_DTYPE.itemsize), ctx.alloc(n)
            d_rx.upload(rx)
            d_arena.upload(arena)
            d_status.upload(np.full(n, 99, dtype=np.int8))
            ctx.unprotect_open_batch(d_rx, n, d_arena, d_out, d_status, flags)
            ctx.sync()
            out = d_arena.download(), d_out.download(dtype=qpp.PKT_DTYPE), d_status.download(dtype=np.int8)
            for b in (d_rx, d_arena, d_out, d_status):
                b.free()
            return out

        a_f, o_f, s_f = run(True)
        a_2, o_2, s_2 = run(False)
        assert (s_f == s_2).all(), "status differs between the fused and the multi-launch path"
        assert (a_f == a_2).all(), "arena differs between the fused and the multi-launch path"
        assert (o_f.view(np.uint8) == o_2.view(np.uint8)).all(), "descriptors differ"
        assert ctx.rx_timeouts() == 0
        want_arena = arena.copy()
        want_out, want_st = orc.unprotect_open_batch(orc.make_keys(mats), orx, want_arena)
        want_st = np.array(want_st, dtype=np.int8)
        conn = want_out["key_idx"] // 2
        dropped = np.isin(want_out["key_idx"], [2 * c + 1 for c in dropped_conn])
        chacha = np.array([suites[c] == 3 for c in conn])
        # QPP_ONLY_AES: neither path opens a ChaCha20 packet (a dropped key is refused whatever the flags)
        untouched = chacha & only_aes & ~dropped
        assert dropped.sum() > 50 and (s_f[dropped] == qpp.INTERNAL_ERROR).all()
        ok = ~dropped & ~untouched
        assert (s_f[ok] == want_st[ok]).all()
        assert (s_f[untouched] == 99).all()
        for suite_ in (1, 2, 3):
            sel = ok & (np.array([suites[c] for c in conn]) == suite_)
            if only_aes and suite_ == 3:
                continue
            assert (s_f[sel] == 0).sum() > 1000 // 3, suite_
        assert (s_f == qpp.DECRYPT_ERROR).any()
        for i in np.flatnonzero(ok):
            o, ln = int(rx[i]["off"]), int(rx[i]["len"])
            assert (a_f[o:o + ln] == want_arena[o:o + ln]).all(), i
        for i in np.flatnonzero(untouched):
            o, ln, aad = int(rx[i]["off"]), int(rx[i]["len"]), int(want_out[i]["aad_len"])
            assert (a_f[o:o + aad] == want_arena[o:o + aad]).all() and (a_f[o + aad:o + ln] == arena[o + aad:o + ln]).all()
    finally:
        ctx.close()
