"""FIPS mode on the GPU: the sealing nonce-order gate (csrc/fips.hip) against the oracle's restatement of aws-lc's
TLS 1.3 AEAD check (oracle/qpp_oracle.c orc_fips_seal_ok).

The reference's `fips` feature backs AES keys with aws-lc-rs TlsRecordSealingKey (quic/s2n-quic-crypto/src/aead/
fips.rs:13-60, cipher_suite/ring.rs:13-31, no FIPS ChaCha: ring.rs:116-121).  aws-lc is not vendored and the reference
holds no vectors for the rule, so parity here is against the restatement only ("parity unpinned").  Bar: the same
packets refused (status INTERNAL_ERROR, bytes untouched) and every other packet bit-exact, across batches (the state
carries over), on every AES kernel path, the one-packet trait call and the transmit queue.
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


@pytest.fixture(params=["burst", "quad", "wave"])
def path(request, ctx):
    ctx.set_burst_max(1 << 30 if request.param == "burst" else 0)
    ctx.set_aes_kernel({"burst": qpp.AES_KERNEL_AUTO, "quad": qpp.AES_KERNEL_QUAD,
                        "wave": qpp.AES_KERNEL_WAVE}[request.param])
    yield request.param
    ctx.set_burst_max(16384)
    ctx.set_aes_kernel(qpp.AES_KERNEL_AUTO)


def _keys(ctx, suites, seed, fips=True):
    rng = np.random.default_rng(seed)
    ctx.set_fips(fips)
    keys = [ctx.key(s, rng.integers(0, 256, qpp.HASH_LEN[s], dtype=np.uint8).tobytes()) for s in suites]
    ctx.set_fips(False)
    okeys = orc.make_keys([(k.suite, *k.material()) for k in keys])
    return keys, okeys


def _pns(rng, n, start):
    """mostly increasing packet numbers with repeats, steps back, jumps and the XOR quirk (given = pn ^ pn_first)"""
    pn, out = start, []
    for _ in range(n):
        r = rng.random()
        if r < 0.70:
            pn += 1
        elif r < 0.80:
            pn += int(rng.integers(2, 40))
        elif r < 0.88:
            pass  # a repeat
        else:
            pn = max(0, pn - int(rng.integers(1, 30)))
        out.append(pn)
    return out


def _batch(rng, slots, pns_by_key, n, max_len=1300):
    descs = np.zeros(n, dtype=qpp.PKT_DTYPE)
    pt = rng.integers(4, max_len, n)
    aad = rng.integers(17, 30, n)
    sizes = aad + pt + 16
    offs = np.concatenate([[0], np.cumsum(sizes + 3)[:-1]])
    arena = rng.integers(0, 256, int(offs[-1] + sizes[-1] + 64), dtype=np.uint8)
    which = rng.integers(0, len(slots), n)
    cursor = [0] * len(slots)
    for i in range(n):
        k = int(which[i])
        descs[i]["pn"] = pns_by_key[k][cursor[k]]
        cursor[k] += 1
        descs[i]["key_idx"] = slots[k]
    descs["off"], descs["aad_len"], descs["pt_len"], descs["pn_len"] = offs, aad, pt, 4
    return descs, arena


def _seal(ctx, descs, arena, flags):
    n = len(descs)
    d_desc, d_arena, d_mask, d_status = ctx.alloc(descs.nbytes), ctx.alloc(arena.nbytes), ctx.alloc(5 * n), ctx.alloc(n)
    d_desc.upload(descs)
    d_arena.upload(arena)
    d_status.upload(np.full(n, 99, dtype=np.int8))
    ctx.seal_batch(d_desc, n, d_arena, d_mask, d_status, flags)
    ctx.sync()
    out = d_arena.download(), d_mask.download(), d_status.download(dtype=np.int8)
    for b in (d_desc, d_arena, d_mask, d_status):
        b.free()
    return out


def _oracle_descs(descs, slots):
    d = descs.copy()
    remap = {s: i for i, s in enumerate(slots)}
    d["key_idx"] = [remap[int(s)] for s in descs["key_idx"]]
    return d


def test_fips_flag_per_key(ctx):
    """keys created while FIPS mode is on seal in it (AES only, host- and device-derived); others keep their mode"""
    rng = np.random.default_rng(1)
    before = ctx.key(1, rng.integers(0, 256, 32, dtype=np.uint8).tobytes())
    keys, _ = _keys(ctx, [1, 2, 3], seed=2)
    assert [k.fips for k in keys] == [True, True, False] and not before.fips
    ctx.set_fips(True)
    derived = ctx.keys_batch(1, [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(3)], updates=1)
    nxt = ctx.update_keys([keys[0], keys[2]])
    ctx.set_fips(False)
    assert all(k.fips for k in derived) and nxt[0].fips and not nxt[1].fips
    for k in [before, *keys, *derived, *nxt]:
        k.free()


def test_fips_batches_match_the_sequential_rule(ctx, path):
    """three batches in a row over 2 FIPS AES keys, one non-FIPS AES key and a ChaCha key (never gated): the same
    packets are refused as by the sequential rule, refused packets stay untouched, the rest are bit-exact"""
    rng = np.random.default_rng(11)
    fkeys, fok = _keys(ctx, [1, 2], seed=5)
    pkeys, pok = _keys(ctx, [1, 3], seed=6, fips=False)
    keys = fkeys + pkeys
    okeys = orc.make_keys([(k.suite, *k.material()) for k in keys])
    slots = [k.slot for k in keys]
    fips = [k.fips for k in keys]
    assert fips == [True, True, False, False]
    states = orc.fips_states(len(keys))
    n = 2500
    starts = [int(rng.integers(0, 2**40)), 0, int(rng.integers(0, 2**30)), 7]
    pns = [_pns(rng, n, s) for s in starts]
    pos = [0] * len(keys)
    flags = qpp.HP_MASK_OUT | qpp.HP_APPLY
    refused_total = 0
    for batch in range(3):
        sub = [p[pos[i]:] for i, p in enumerate(pns)]
        descs, arena = _batch(rng, slots, sub, 700 + 300 * batch)
        for i in range(len(keys)):
            pos[i] += int((descs["key_idx"] == slots[i]).sum())
        got, masks, st = _seal(ctx, descs, arena, flags)
        want = arena.copy()
        want_masks, want_st = orc.seal_batch_fips(okeys, fips, states, _oracle_descs(descs, slots), want, flags)
        assert list(st) == want_st, f"batch {batch}: status differs"
        assert (got == want).all(), f"batch {batch}: arena differs"
        ok = np.array(want_st) == 0
        m = np.frombuffer(masks.tobytes(), dtype=np.uint8).reshape(-1, 5)
        wm = np.frombuffer(want_masks, dtype=np.uint8).reshape(-1, 5)
        assert (m[ok] == wm[ok]).all()
        refused = ~ok
        refused_total += int(refused.sum())
        # only FIPS keys refuse
        assert not np.isin(descs["key_idx"][refused], slots[2:]).any()
    assert refused_total > 50  # the pattern refuses repeats and steps back
    for k in keys:
        k.free()


def test_fips_one_key_lane_batch(ctx):
    """one live FIPS key: the plan-free single-key lane path with the gate in front (16 Ki packets, 1200 B)"""
    rng = np.random.default_rng(21)
    ctx.set_burst_max(0)
    try:
        keys, okeys = _keys(ctx, [1], seed=22)
        n = 16384
        # from pn 0: aws-lc takes the key's first nonce as sequence 0 and XORs it out (given = pn ^ pn_first), so a
        # run starting at 1000 would be refused wherever pn ^ 1000 steps back, not only at the planted repeats
        pns = list(range(n))
        for i in rng.integers(1, n, 40):  # a few repeats and steps back
            pns[i] = max(0, pns[i - 1] - int(rng.integers(0, 3)))
        descs = np.zeros(n, dtype=qpp.PKT_DTYPE)
        descs["pn"], descs["key_idx"] = pns, keys[0].slot
        descs["off"] = np.arange(n) * 1248
        descs["aad_len"], descs["pt_len"], descs["pn_len"] = 21, 1200, 4
        arena = rng.integers(0, 256, n * 1248 + 64, dtype=np.uint8)
        got, _, st = _seal(ctx, descs, arena, qpp.HP_MASK_OUT)
        want = arena.copy()
        _, want_st = orc.seal_batch_fips(okeys, [True], orc.fips_states(1), _oracle_descs(descs, [keys[0].slot]),
                                         want, qpp.HP_MASK_OUT)
        assert list(st) == want_st and 0 < want_st.count(3) <= 40
        assert (got == want).all()
        keys[0].free()
    finally:
        ctx.set_burst_max(16384)


def test_fips_per_packet_seal(ctx):
    """Key::encrypt in FIPS mode: INTERNAL_ERROR for a nonce that does not come after the last one, buffer untouched
    (the trait call fails); the key's first seal fixes the mask, so a later smaller pn can pass (aws-lc's XOR rule)"""
    keys, okeys = _keys(ctx, [2], seed=31)
    k = keys[0]
    kk, iv, hp = k.material()
    state = orc.fips_states(1)
    header = bytes(range(21))
    payload = bytes(range(100))
    for pn in [5, 6, 7, 8, 8, 100, 99, 101]:
        ok = orc.lib().orc_fips_seal_ok(state, orc._buf(orc.nonce(iv, pn)))
        if ok:
            ct, tag = orc.seal(2, kk, orc.nonce(iv, pn), header, payload)
            assert k.encrypt(pn, header, payload) == ct + tag
        else:
            with pytest.raises(qpp.QppError) as e:
                k.encrypt(pn, header, payload)
            assert e.value.code == qpp.INTERNAL_ERROR
    k.free()


@pytest.mark.parametrize("flush", ["zero_copy", "dma"])
def test_fips_txq_reports_refused_packets(ctx, flush, monkeypatch):
    """a txq flush with a refused packet (a repeated pn): the wait reports INTERNAL_ERROR once, the refused packet is
    left as pushed, the others equal crypto::encrypt + protect of the oracle"""
    monkeypatch.setenv("QPP_TXQ_ZC_MAX", "1024" if flush == "zero_copy" else "0")
    keys, okeys = _keys(ctx, [1], seed=41)
    k = keys[0]
    kk, iv, hp = k.material()
    q = qpp.TxQueue(ctx, 1 << 16, 64)
    rng = np.random.default_rng(42)
    off, layout = 0, []
    for pn in [40, 41, 41, 42]:
        header = bytes([0x40]) + rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
        payload = rng.integers(0, 256, 200, dtype=np.uint8).tobytes()
        pkt = header + (pn & 0xff).to_bytes(1, "big") + payload
        q.ring[off:off + len(pkt)] = np.frombuffer(pkt, dtype=np.uint8)
        q.push(k, pn, off, len(header), 1, len(payload))
        layout.append((off, pkt, pn, header, payload))
        off += len(pkt) + 16 + 8
    with pytest.raises(qpp.QppError) as e:
        q.flush()
    assert e.value.code == qpp.INTERNAL_ERROR
    for i, (o, pkt, pn, header, payload) in enumerate(layout):
        if i == 2:
            assert q.ring[o:o + len(pkt)].tobytes() == pkt  # untouched
        else:
            rc, protected = orc.protect_packet(1, kk, iv, hp, pn, header, 1, payload)
            assert q.ring[o:o + len(protected)].tobytes() == protected
    # the next flush is clean again
    o = off
    header = bytes([0x40]) + bytes(16)
    payload = bytes(64)
    q.ring[o:o + 17 + 1 + 64] = np.frombuffer(header + bytes([43]) + payload, dtype=np.uint8)
    q.push(k, 43, o, 17, 1, 64)
    q.flush()
    q.close()
    k.free()
