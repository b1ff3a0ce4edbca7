"""GPU tests of the boundary's ownership and asynchrony rules (include/qpp.h "Asynchrony"), through the C ABI.

* (Key, HeaderKey) are independently owned, as TLS_*::new returns them (quic/s2n-quic-crypto/src/negotiated.rs:95-134):
  the header key keeps working after the packet keys it was born with are rotated away and freed
  (KeySet::rotate_phase, quic/s2n-quic-core/src/crypto/application/keyset.rs:75-96; ApplicationSpace keeps its
  header key, quic/s2n-quic-transport/src/space/application.rs:70).
* Freeing a key while batches that use it are in flight is safe: the zeroization is stream-ordered and the slot is
  only reused afterwards.
* Two streams of one context run batches concurrently (per-stream plan scratch).
* Batched derive_next_key (qpp_key_update_batch) equals the per-key chain.
* A descriptor naming a slot outside the key table, a freed slot or a header-key slot is refused (INTERNAL_ERROR).
* The host pipeline (qpp_host_batch_*) seals / opens packets that start and end in host memory.
Every output is compared bit-exactly with the oracle (tests/_oracle.py over oracle/qpp_oracle.c).
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


def _secret(rng, suite):
    return rng.integers(0, 256, qpp.HASH_LEN[suite], dtype=np.uint8).tobytes()


def _oracle_seal(materials, descs, arena, flags):
    """oracle seal; materials: {slot: (suite, key, iv, hp)} for every slot the descriptors name"""
    slots = sorted(materials)
    okeys = orc.make_keys([materials[s] for s in slots])
    remap = {s: i for i, s in enumerate(slots)}
    d = descs.copy()
    d["key_idx"] = [remap[int(s)] for s in descs["key_idx"]]
    want = arena.copy()
    masks = orc.seal_batch(okeys, d, want, flags)
    return want, masks


def _mat(keys):
    return {k.slot: (k.suite, *k.material()) for k in keys}


def _sample(descs, arena, pick):
    """packets `pick` of a fixed-stride batch, re-based into their own small arena"""
    stride = arena.size // len(descs)
    sub = descs[pick].copy()
    sub["off"] = np.arange(len(pick)) * stride
    return sub, np.concatenate([arena[i * stride:(i + 1) * stride] for i in pick])


def _gather(buf, pick, stride):
    return np.concatenate([buf[i * stride:(i + 1) * stride] for i in pick])


@pytest.mark.parametrize("suite", [1, 2, 3])
def test_header_key_outlives_rotated_packet_keys(ctx, suite):
    """The shim pattern of INTEGRATION.md §2: (key, header key) from one secret; the key is updated twice and the
    old keys are freed (KeySet::rotate_phase); the header key's masks stay those of the original secret."""
    rng = np.random.default_rng(100 + suite)
    secret = _secret(rng, suite)
    key, hk = ctx.key_pair(suite, secret)
    _, _, hp = orc.derive(suite, secret)
    samples = [rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in range(8)]
    want = [orc.hp_mask(suite, hp, s) for s in samples]
    assert [hk.header_protection_mask(s) for s in samples] == want
    k1 = key.derive_next_key()
    key.free()
    k2 = k1.derive_next_key()
    k1.free()
    # churn the key table so that the freed slots are reused by unrelated keys
    others = [ctx.key(suite, _secret(rng, suite)) for _ in range(6)]
    ctx.sync()
    assert [hk.sealing_header_protection_mask(s) for s in samples] == want
    assert [hk.opening_header_protection_mask(s) for s in samples] == want
    assert hk.sample_len() == 16 and hk.suite == suite
    # the rotated key protects with the same header key (RFC 9001 §6) and seals with the twice-updated secret
    s2 = orc.update_secret(suite, orc.update_secret(suite, secret))
    k_want, iv_want, _ = orc.derive(suite, s2)
    assert k2.material() == (k_want, iv_want, hp)
    # the header key's slot serves qpp_hp_mask_batch descriptors (receive side: sample at aad_len + 4)
    n = 64
    arena = rng.integers(0, 256, n * 64, dtype=np.uint8)
    descs = np.zeros(n, dtype=qpp.PKT_DTYPE)
    descs["off"] = np.arange(n) * 64
    descs["aad_len"] = 7
    descs["key_idx"] = hk.slot
    d_desc, d_arena, d_mask = ctx.alloc(descs.nbytes), ctx.alloc(arena.nbytes), ctx.alloc(5 * n)
    d_desc.upload(descs)
    d_arena.upload(arena)
    ctx.hp_mask_batch(d_desc, n, d_arena, d_mask)
    got = d_mask.download().tobytes()
    for i in range(n):
        s = 64 * i + 7 + 4
        assert got[5 * i:5 * i + 5] == orc.hp_mask(suite, hp, arena[s:s + 16].tobytes())
    for b in (d_desc, d_arena, d_mask):
        b.free()
    hk.free()
    k2.free()
    for k in others:
        k.free()


def test_initial_keys_pair(ctx, rfc):
    H = bytes.fromhex
    sealer, opener, hs, ho = ctx.initial_keys_pair(qpp.ENDPOINT_CLIENT, H(rfc["dcid"]))
    sealer.free()
    opener.free()
    # InitialHeaderKey: the client seals with the client hp (A.2 mask) and opens with the server hp (A.3 mask)
    assert hs.header_protection_mask(H(rfc["a2"]["sample"])).hex() == rfc["a2"]["mask"]
    assert ho.header_protection_mask(H(rfc["a3"]["sample"])).hex() == rfc["a3"]["mask"]
    hs.free()
    ho.free()


def test_free_while_in_flight_is_stream_ordered(ctx):
    """Batches are enqueued on a side stream; their keys are freed right after the enqueue (no sync), new keys are
    installed and used on the context stream at once.  The side batches still seal with the old keys, bit-exactly;
    the freed slots are reused only after the side stream is done."""
    rng = np.random.default_rng(7)
    keys = [ctx.key(s, _secret(rng, s)) for s in (1, 2, 3, 1)]
    old_mat = _mat(keys)
    old_slots = set(old_mat)
    n = 1 << 19
    descs, arena = qpp.make_batch(n, 1200, [k.slot for k in keys], seed=70)
    stride = arena.size // n
    pick = np.sort(rng.choice(n, 1500, replace=False))
    pick[-1] = n - 1  # the very last packet of the batch
    sub_d, sub_a = _sample(descs, arena, pick)
    want, want_masks = _oracle_seal(old_mat, sub_d, sub_a, qpp.HP_MASK_OUT)
    side = ctx.new_stream()
    bufs = [ctx.alloc(descs.nbytes), ctx.alloc(arena.nbytes), ctx.alloc(5 * n), ctx.alloc(n)]
    d_desc, d_arena, d_mask, d_st = bufs
    d_desc.upload(descs)
    delay = ctx.alloc(arena.nbytes)  # a few ms of queued work in front of the checked batch
    delay.upload(arena)
    d_arena.upload(arena)
    for _ in range(4):
        ctx.seal_batch(d_desc, n, delay, d_mask, d_st, qpp.HP_MASK_OUT, stream=side)
    ctx.seal_batch(d_desc, n, d_arena, d_mask, d_st, qpp.HP_MASK_OUT, stream=side)
    for k in keys:
        k.free()
    fresh = [ctx.key(s, _secret(rng, s)) for s in (1, 3)]
    assert not ({k.slot for k in fresh} & old_slots), "a retired slot was reused while the side stream ran"
    # use the fresh keys at once on the context stream (their install is ordered before this launch)
    n2 = 4096
    d2, a2 = qpp.make_batch(n2, 333, [k.slot for k in fresh], seed=71)
    want2, masks2 = _oracle_seal(_mat(fresh), d2, a2, qpp.HP_MASK_OUT)
    b2 = [ctx.alloc(d2.nbytes), ctx.alloc(a2.nbytes), ctx.alloc(5 * n2), ctx.alloc(n2)]
    b2[0].upload(d2)
    b2[1].upload(a2)
    ctx.seal_batch(b2[0], n2, b2[1], b2[2], b2[3], qpp.HP_MASK_OUT)
    ctx.sync()
    assert (b2[1].download() == want2).all() and b2[2].download().tobytes() == masks2
    ctx.sync(side)
    got, masks, st = d_arena.download(), d_mask.download(), d_st.download(dtype=np.int8)
    assert (st == 0).all()
    assert (_gather(got, pick, stride) == want).all()
    assert np.concatenate([masks[5 * i:5 * i + 5] for i in pick]).tobytes() == want_masks
    # now (whole device idle: the retirements ran too) the retired slots are reusable
    ctx.synchronize()
    more = [ctx.key(1, _secret(rng, 1)) for _ in range(4)]
    assert {k.slot for k in more} <= old_slots
    assert ctx.key_slots()[2] == 0
    ctx.stream_destroy(side)
    for b in bufs + b2 + [delay]:
        b.free()
    for k in fresh + more:
        k.free()


def test_two_streams_of_one_context(ctx):
    """Lane-kernel batches (with their plans) on two streams at once, interleaved without syncs: each stream's plan
    scratch is its own, so both results are bit-exact."""
    rng = np.random.default_rng(8)
    ka = [ctx.key(s, _secret(rng, s)) for s in (1, 2, 1, 2, 3)]
    kb = [ctx.key(s, _secret(rng, s)) for s in (2, 1, 3)]
    s1, s2 = ctx.new_stream(), ctx.new_stream()
    runs = []
    for keys, stream, seed, pt in ((ka, s1, 81, 300), (kb, s2, 82, 700)):
        n = 40000
        descs, arena = qpp.make_batch(n, pt, [k.slot for k in keys], seed=seed)
        bufs = [ctx.alloc(descs.nbytes), ctx.alloc(arena.nbytes), ctx.alloc(5 * n), ctx.alloc(n)]
        bufs[0].upload(descs)
        bufs[1].upload(arena)
        runs.append((keys, stream, descs, arena, bufs))
    for _ in range(3):  # seal, open, seal again on both streams, interleaved: the last seal is checked
        for keys, stream, descs, arena, b in runs:
            ctx.seal_batch(b[0], len(descs), b[1], b[2], b[3], qpp.HP_MASK_OUT, stream=stream)
        for keys, stream, descs, arena, b in runs:
            ctx.open_batch(b[0], len(descs), b[1], b[3], 0, stream=stream)
    for keys, stream, descs, arena, b in runs:
        ctx.seal_batch(b[0], len(descs), b[1], b[2], b[3], qpp.HP_MASK_OUT, stream=stream)
    for keys, stream, descs, arena, b in runs:
        ctx.sync(stream)
        got = b[1].download()
        # after seal/open round trips the payload is the plaintext again; the tag bytes were overwritten in place
        # by each seal with the same value, so the arena equals one oracle seal of the original
        want, masks = _oracle_seal(_mat(keys), descs, arena, qpp.HP_MASK_OUT)
        assert (b[3].download(dtype=np.int8) == 0).all()
        assert (got == want).all()
        assert b[2].download().tobytes() == masks
        for x in b:
            x.free()
    ctx.stream_destroy(s1)
    ctx.stream_destroy(s2)
    for k in ka + kb:
        k.free()


def test_key_update_batch_matches_chain(ctx):
    rng = np.random.default_rng(9)
    suites = [1, 2, 3] * 100
    keys = [ctx.key(s, _secret(rng, s)) for s in suites]
    nxt = ctx.update_keys(keys)
    for k, u in zip(keys[::17], nxt[::17]):
        ref = k.derive_next_key()
        assert u.material() == ref.material() and u.suite == k.suite
        assert u.material()[2] == k.material()[2]  # the header key is carried over
        ref.free()
    slots2 = np.zeros(len(nxt), dtype=np.uint32)
    nxt2 = ctx.update_keys(nxt, slots_out=slots2)  # a second rotation from device-made keys
    assert list(slots2) == [k.slot for k in nxt2]  # qpp_key_slot_batch
    for k in keys:
        k.free()
    descs, arena = qpp.make_batch(6000, 500, [k.slot for k in nxt2], seed=91)
    d = [ctx.alloc(descs.nbytes), ctx.alloc(arena.nbytes), ctx.alloc(5 * 6000), ctx.alloc(6000)]
    d[0].upload(descs)
    d[1].upload(arena)
    ctx.seal_batch(d[0], 6000, d[1], d[2], d[3], qpp.HP_MASK_OUT)
    ctx.sync()
    want, masks = _oracle_seal(_mat(nxt2), descs, arena, qpp.HP_MASK_OUT)
    assert (d[3].download(dtype=np.int8) == 0).all()
    assert (d[1].download() == want).all() and d[2].download().tobytes() == masks
    for x in d:
        x.free()
    for k in nxt + nxt2:
        k.free()


@pytest.mark.parametrize("kernel", ["burst", "quad"])
def test_bad_slots_are_refused(ctx, kernel):
    """key_idx outside the table, of a freed key or of a header key: INTERNAL_ERROR, the packet untouched, every other
    packet of the batch bit-exact (the kernels never dereference a slot outside the table)."""
    rng = np.random.default_rng(10)
    ctx.set_burst_max(1 << 30 if kernel == "burst" else 0)
    try:
        keys = [ctx.key(s, _secret(rng, s)) for s in (1, 2, 3)]
        gone = ctx.key(1, _secret(rng, 1))
        hk = ctx.header_key(3, _secret(rng, 3))
        n = 3000
        descs, arena = qpp.make_batch(n, 200, [k.slot for k in keys], seed=12)
        bad = np.zeros(n, bool)
        bad[5::97] = True
        cap = ctx.key_slots()[0]
        descs["key_idx"][5::97] = np.resize(np.array([cap, cap + 12345, 2**32 - 1, gone.slot, hk.slot],
                                                     dtype=np.uint32), bad.sum())
        good_mat = _mat(keys)
        gone.free()
        ctx.synchronize()  # the retirement has run: the slot is zero (using a freed key is the caller's bug)
        d = [ctx.alloc(descs.nbytes), ctx.alloc(arena.nbytes), ctx.alloc(5 * n), ctx.alloc(n)]
        d[0].upload(descs)
        d[1].upload(arena)
        ctx.seal_batch(d[0], n, d[1], d[2], d[3], qpp.HP_MASK_OUT)
        ctx.sync()
        st, got = d[3].download(dtype=np.int8), d[1].download()
        assert (st[bad] == qpp.INTERNAL_ERROR).all() and (st[~bad] == 0).all()
        stride = arena.size // n
        ok = np.nonzero(~bad)[0]
        sub_d, sub_a = _sample(descs, arena, ok)
        want, _ = _oracle_seal(good_mat, sub_d, sub_a, 0)
        assert (_gather(got, ok, stride) == want).all()
        assert (_gather(got, np.nonzero(bad)[0], stride) == _gather(arena, np.nonzero(bad)[0], stride)).all()
        # receive side: a key slot outside the table is refused before any key is read
        rx = np.zeros(4, dtype=qpp.RX_DTYPE)
        rx["off"] = np.arange(4) * 256
        rx["header_len"] = 9
        rx["len"] = 200
        rx["key_idx"][:, 0] = [keys[0].slot, cap + 7, keys[0].slot, 2**31]
        rx["key_idx"][:, 1] = [keys[0].slot, keys[0].slot, cap, keys[0].slot]
        ra = rng.integers(0, 256, 1024, dtype=np.uint8)
        r = [ctx.alloc(rx.nbytes), ctx.alloc(ra.nbytes), ctx.alloc(4 * 24), ctx.alloc(4)]
        r[0].upload(rx)
        r[1].upload(ra)
        ctx.unprotect_open_batch(r[0], 4, r[1], r[2], r[3])
        ctx.sync()
        rst = r[3].download(dtype=np.int8)
        assert list(rst[1:]) == [qpp.INTERNAL_ERROR] * 3 and rst[0] == qpp.DECRYPT_ERROR  # random bytes: bad tag
        for x in d + r:
            x.free()
        hk.free()
        for k in keys:
            k.free()
    finally:
        ctx.set_burst_max(16384)


@pytest.mark.parametrize("ops", ["seal_then_open", "round_trip"])
def test_host_pipeline(ctx, ops):
    """Packets start and end in pinned host memory: chunked H2D -> seal and/or open -> D2H over a small ring (many
    chunks per batch), checked against the oracle on a sample and by the full round trip."""
    rng = np.random.default_rng(11)
    keys = [ctx.key(s, _secret(rng, s)) for s in (1, 2, 3, 1, 2)]
    ctx.set_host_pipe(12000, 16 << 20, 3)  # 12000 packets / 16 MiB per chunk, 3 chunk buffers
    try:
        n, pt = 100000, 1200
        descs, arena = qpp.make_batch(n, pt, [k.slot for k in keys], seed=13)
        stride = arena.size // n
        host = ctx.host_alloc(arena.nbytes)
        host[:] = arena
        masks = np.zeros(5 * n, np.uint8)
        st = np.full(n, 77, np.int8)
        pick = np.sort(rng.choice(n, 1200, replace=False))
        sub_d, sub_a = _sample(descs, arena, pick)
        want, want_masks = _oracle_seal(_mat(keys), sub_d, sub_a, qpp.HP_MASK_OUT)
        body = np.s_[:, 21:21 + pt]
        if ops == "seal_then_open":
            t = ctx.host_submit(descs, host, masks, st, qpp.HP_MASK_OUT, qpp.OP_SEAL)
            ctx.host_wait(t)
            assert (st == 0).all()
            assert (_gather(host, pick, stride) == want).all()
            assert np.concatenate([masks[5 * i:5 * i + 5] for i in pick]).tobytes() == want_masks
            sealed = host.copy()
            st[:] = 77
            t = ctx.host_submit(descs, host, None, st, 0, qpp.OP_OPEN)
            assert ctx.host_done(t) in (False, True)
            ctx.host_wait(t)
            assert (st == 0).all()
            assert (host.reshape(n, stride)[body] == arena.reshape(n, stride)[body]).all()
            assert (host.reshape(n, stride)[:, 21 + pt:21 + pt + 16] == sealed.reshape(n, stride)[:, 21 + pt:21 + pt + 16]).all()
        else:
            t = ctx.host_submit(descs, host, masks, st, qpp.HP_MASK_OUT, qpp.OP_SEAL | qpp.OP_OPEN)
            ctx.host_wait(t)
            assert (st == 0).all()
            assert np.concatenate([masks[5 * i:5 * i + 5] for i in pick]).tobytes() == want_masks
            assert (host.reshape(n, stride)[body] == arena.reshape(n, stride)[body]).all()
            # the tag written by the seal stays behind: it is the oracle's
            tags = _gather(host, pick, stride).reshape(len(pick), stride)[:, 21 + pt:21 + pt + 16]
            assert (tags == want.reshape(len(pick), stride)[:, 21 + pt:21 + pt + 16]).all()
        # descriptors out of arena order are refused
        bad = descs[:10][::-1].copy()
        with pytest.raises(qpp.QppError):
            ctx.host_submit(bad, host, None, st, 0, qpp.OP_SEAL)
        ctx.host_free(host)
    finally:
        ctx.set_host_pipe(65536, 96 << 20, 4)
        for k in keys:
            k.free()


@pytest.mark.parametrize("suite", [1, 2])
def test_single_live_key_batches_run_without_a_plan(suite):
    """With exactly one live packet key (an AES one) the quad kernel runs without the plan launches
    (api.cpp single_aes_slot); packets naming any other slot are still refused with INTERNAL_ERROR and left untouched,
    the rest are bit-exact, and open round-trips."""
    c = qpp.Context(0)
    try:
        c.set_burst_max(0)  # the quad kernel, not the wave-per-packet one
        rng = np.random.default_rng(70 + suite)
        k = c.key(suite, _secret(rng, suite))
        n = 4096
        descs, arena = qpp.make_batch(n, 600, [k.slot], seed=71 + suite)
        bad = np.zeros(n, bool)
        bad[3::53] = True
        descs["key_idx"][bad] = k.slot + 1  # not a live slot
        d = [c.alloc(descs.nbytes), c.alloc(arena.nbytes), c.alloc(5 * n), c.alloc(n)]
        d[0].upload(descs)
        d[1].upload(arena)
        c.seal_batch(d[0], n, d[1], d[2], d[3], qpp.HP_MASK_OUT)
        c.sync()
        st, got = d[3].download(dtype=np.int8), d[1].download()
        assert (st[bad] == qpp.INTERNAL_ERROR).all() and (st[~bad] == 0).all()
        stride = arena.size // n
        ok = np.nonzero(~bad)[0][::7]
        sub_d, sub_a = _sample(descs, arena, ok)
        want, _ = _oracle_seal(_mat([k]), sub_d, sub_a, 0)
        assert (_gather(got, ok, stride) == want).all()
        assert (_gather(got, np.nonzero(bad)[0], stride) == _gather(arena, np.nonzero(bad)[0], stride)).all()
        c.open_batch(d[0], n, d[1], d[3], 0)
        c.sync()
        st2, back = d[3].download(dtype=np.int8), d[1].download()
        assert (st2[~bad] == 0).all()
        for i in np.nonzero(~bad)[0][::11]:  # the payloads are the plaintext again (the tags stay sealed ones)
            a = int(descs["off"][i]) + int(descs["aad_len"][i])
            b = a + int(descs["pt_len"][i])
            assert (back[a:b] == arena[a:b]).all()
        k.free()
    finally:
        c.close()


def test_ctx_synchronize_covers_copy_only_streams(ctx):
    """qpp_ctx_synchronize waits for a stream that carried only copies / memsets / event records: a d2h on a
    qpp_stream_create stream, then qpp_ctx_synchronize, then the host bytes -- no per-stream sync in between (raw C-ABI
    calls, not the Python wrapper's upload/download, which synchronize their own stream)."""
    import ctypes
    L = qpp.lib()
    nbytes = 256 << 20  # large enough that the copies are still running when the calls return
    d = ctx.alloc(nbytes)
    h = ctx.host_alloc(nbytes)
    h[:] = 0
    st = ctx.new_stream()
    ev = ctx.event()
    for rnd, val in enumerate((0x5a, 0xc3)):
        assert L.qpp_memset_d(ctx.handle, d.ptr, val, nbytes, st) == 0
        assert L.qpp_memcpy_d2h(ctx.handle, h.ctypes.data, d.ptr, nbytes, st) == 0
        assert L.qpp_event_record(ctx.handle, ev, st) == 0
        assert L.qpp_ctx_synchronize(ctx.handle) == 0
        assert (h[::4093] == val).all() and h[-1] == val, rnd
    ctx.stream_destroy(st)
    # a destroyed stream leaves the context's set: synchronize still works
    assert L.qpp_ctx_synchronize(ctx.handle) == 0
    ctx.host_free(h)
    d.free()
