"""GPU parity: the HIP path (through the C ABI in libqpp.so) against the oracle and the golden vectors.

Bar: bit-exact ciphertext, tag, header-protection mask and status for every packet (integer work).
Mirrors the reference's tests (quic/s2n-quic-crypto/src/{initial.rs:142-241, retry.rs:55-64,
one_rtt.rs:79-114}; quic/s2n-quic-core/src/crypto/tls/testing.rs:612-681 seal_open/protect_unprotect)
and adds batch cases: ragged lengths, mixed keys and suites, tampered tags, full-size round trips.
"""
import numpy as np
import pytest

import _oracle as orc
import qpp
from conftest import load_golden

pytestmark = pytest.mark.gpu
H = bytes.fromhex


@pytest.fixture(scope="module")
def ctx():
    c = qpp.Context(0)
    yield c
    c.close()


@pytest.fixture(params=["burst", "quad", "wave"])
def path(request, ctx):
    """AES-GCM kernel path: wave per packet (small batches), the quad kernel (four lanes per packet, one workgroup per
    CU over a key-sorted slice),
    or lane per packet with one key per 64-packet wave (many keys); same outputs."""
    ctx.set_burst_max(1 << 30 if request.param == "burst" else 0)
    ctx.set_aes_kernel({"burst": qpp.AES_KERNEL_AUTO, "quad": qpp.AES_KERNEL_QUAD,
                        "wave": qpp.AES_KERNEL_WAVE}[request.param])
    yield request.param
    ctx.set_burst_max(16384)
    ctx.set_aes_kernel(qpp.AES_KERNEL_AUTO)


# ------------------------------------------------------------------ RFC 9001 Appendix A through the trait mirror

def test_initial_keys_and_a2_seal(ctx, rfc):
    sealer, opener = ctx.initial_keys(qpp.ENDPOINT_CLIENT, H(rfc["dcid"]))
    assert sealer.material() == (H(rfc["client"]["key"]), H(rfc["client"]["iv"]), H(rfc["client"]["hp"]))
    assert opener.material() == (H(rfc["server"]["key"]), H(rfc["server"]["iv"]), H(rfc["server"]["hp"]))
    a2 = rfc["a2"]
    payload = H(a2["payload_prefix"]) + bytes(a2["padded_payload_len"] - len(H(a2["payload_prefix"])))
    header = H(a2["header"])
    sealed = sealer.encrypt(a2["pn"], header, payload)
    prot = H(a2["protected_packet"])
    assert sealed == prot[len(header):]
    hdr_len = len(header) - a2["pn_len"]
    sample = sealed[4 - a2["pn_len"]:20 - a2["pn_len"]]
    assert sample.hex() == a2["sample"]
    assert sealer.header_protection_mask(sample).hex() == a2["mask"]
    # the server opens it (rfc_example_server_test)
    _, server_opener = ctx.initial_keys(qpp.ENDPOINT_SERVER, H(rfc["dcid"]))
    assert server_opener.decrypt(a2["pn"], header, sealed) == payload
    for k in (sealer, opener, server_opener):
        k.free()


def test_a3_server_initial(ctx, rfc):
    sealer, _ = ctx.initial_keys(qpp.ENDPOINT_SERVER, H(rfc["dcid"]))
    a3 = rfc["a3"]
    header = H(a3["header"])
    sealed = sealer.encrypt(a3["pn"], header, H(a3["payload"]))
    assert sealed == H(a3["protected_packet"])[len(header):]
    assert sealer.header_protection_mask(H(a3["sample"])).hex() == a3["mask"]


def test_a4_retry_tag(ctx, rfc):
    a4 = rfc["a4"]
    k = ctx.raw_key(1, H(a4["key"]), H(a4["nonce"]), bytes(16))  # pn 0: nonce == iv
    assert k.encrypt(0, H(a4["pseudo_packet"]), b"").hex() == a4["tag"]
    with pytest.raises(qpp.DecryptError):
        k.decrypt(0, H(a4["pseudo_packet"]), H("00112233445566778899aabbccddeeff"))
    assert k.decrypt(0, H(a4["pseudo_packet"]), H(a4["tag"])) == b""


def test_a5_chacha_and_key_update(ctx, rfc):
    a5 = rfc["a5"]
    k = ctx.key(3, H(a5["secret"]))
    assert k.material() == (H(a5["key"]), H(a5["iv"]), H(a5["hp"]))
    sealed = k.encrypt(a5["pn"], H(a5["header"]), H(a5["plaintext"]))
    assert sealed.hex() == a5["ciphertext"]
    assert k.header_protection_mask(H(a5["sample"])).hex() == a5["mask"]
    nxt = k.derive_next_key()
    ref = ctx.key(3, H(a5["ku_secret"]))
    assert nxt.material()[:2] == ref.material()[:2]
    assert nxt.material()[2] == k.material()[2]  # HP key is not updated (RFC 9001 §6)
    assert nxt.encrypt(0, b"", bytes(32)) == ref.encrypt(0, b"", bytes(32))  # test_key_update
    bad = ctx.key(3, bytes(32)).derive_next_key()
    assert bad.encrypt(0, b"", bytes(32)) != ref.encrypt(0, b"", bytes(32))


def test_limits_and_lengths(ctx):
    for suite, conf, integ in ((1, 2**23, 2**52), (2, 2**23, 2**52), (3, 2**62, 2**36)):
        k = ctx.key(suite, bytes(qpp.HASH_LEN[suite]))
        assert (k.tag_len(), k.sample_len()) == (16, 16)
        assert (k.aead_confidentiality_limit(), k.aead_integrity_limit()) == (conf, integ)
    with pytest.raises(qpp.QppError) as e:
        ctx.key(9, bytes(32))
    assert e.value.code == qpp.UNSUPPORTED


# ------------------------------------------------------------------ golden fixtures through the per-packet API

@pytest.mark.parametrize("name,suite", [("aead_aes128gcm.json", 1), ("aead_aes256gcm.json", 2),
                                        ("aead_chacha20poly1305.json", 3), ("gcm_spec_aes256.json", 2)])
def test_aead_fixtures(ctx, name, suite, path):
    for c in load_golden(name)["cases"]:
        k = ctx.raw_key(suite, H(c["key"]), H(c["iv"]), bytes(qpp.KEY_LEN[suite]))
        sealed = k.encrypt(c["pn"], H(c["aad"]), H(c["pt"]))
        assert sealed.hex() == c["ct"] + c["tag"], len(H(c["pt"]))
        assert k.decrypt(c["pn"], H(c["aad"]), sealed) == H(c["pt"])
        bad = bytearray(sealed)
        bad[len(bad) // 2] ^= 0x80
        with pytest.raises(qpp.DecryptError):
            k.decrypt(c["pn"], H(c["aad"]), bytes(bad))
        k.free()


def test_gcm_spec_aes256_batches(ctx, path):
    """The GCM specification's AES-256 test cases 13-16 (tests/golden/gcm_spec_aes256.json: the published vectors, the
    reference holds none for AES-256) through the batch kernels: 512 copies of each case in one 2048-packet batch over
    the two raw keys they use, sealed and opened on every AES kernel path, every packet's ciphertext and tag compared."""
    cases = load_golden("gcm_spec_aes256.json")["cases"]
    keys = {}
    for c in cases:
        if (c["key"], c["iv"]) not in keys:
            keys[(c["key"], c["iv"])] = ctx.raw_key(2, H(c["key"]), H(c["iv"]), bytes(32))
    reps, n = 512, 512 * len(cases)
    sizes = [len(H(c["aad"])) + len(H(c["pt"])) + 16 for c in cases]
    stride = (max(sizes) + 15) // 16 * 16
    descs = np.zeros(n, dtype=qpp.PKT_DTYPE)
    arena = np.zeros(n * stride, dtype=np.uint8)
    want = arena.copy()
    for i in range(n):
        c = cases[i % len(cases)]
        aad, pt = H(c["aad"]), H(c["pt"])
        o = i * stride
        descs[i] = (0, keys[(c["key"], c["iv"])].slot, o, len(aad), len(pt), 1, 0, 0)
        arena[o:o + len(aad) + len(pt)] = np.frombuffer(aad + pt, np.uint8)
        want[o:o + len(aad) + len(pt) + 16] = np.frombuffer(aad + H(c["ct"] + c["tag"]), np.uint8)
    got, _, st = _run_seal(ctx, descs, arena, 0)
    assert (st == 0).all()
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"first mismatch at arena byte {bad[:8]}"
    opened, st = _run_open(ctx, descs, want)
    plain = want.copy()  # the open leaves the tag in place and the plaintext where the ciphertext was
    for i in range(n):
        c = cases[i % len(cases)]
        a, p = len(H(c["aad"])), len(H(c["pt"]))
        plain[i * stride + a:i * stride + a + p] = arena[i * stride + a:i * stride + a + p]
    assert (st == 0).all() and (opened == plain).all()
    for k in keys.values():
        k.free()


def test_short_open_is_decrypt_error(ctx):
    k = ctx.key(1, bytes(32))
    with pytest.raises(qpp.DecryptError):
        k.decrypt(1, b"", bytes(15))


def test_hp_fixtures(ctx):
    for c in load_golden("hp_masks.json")["cases"]:
        k = ctx.raw_key(c["suite"], bytes(qpp.KEY_LEN[c["suite"]]), bytes(12), H(c["hp"]))
        assert k.header_protection_mask(H(c["sample"])).hex() == c["mask"]
        k.free()


def test_kdf_chains(ctx):
    for ch in load_golden("kdf_chains.json")["chains"]:
        k = ctx.key(ch["suite"], H(ch["secret"]))
        hp0 = H(ch["steps"][0]["hp"])
        for step in ch["steps"]:
            key, iv, hp = k.material()
            assert (key, iv) == (H(step["key"]), H(step["iv"]))
            assert hp == hp0  # carried over by every update
            k = k.derive_next_key()


def test_seal_scatter(ctx):
    # seal_in_place_scatter: inline || extra sealed as one message
    k = ctx.key(2, bytes(range(48)))
    inline, extra = bytes(range(100)), bytes(range(37))
    ct_in, ct_extra_tag = k.encrypt_scatter(77, b"\x41hdr", inline, extra)
    whole = k.encrypt(77, b"\x41hdr", inline + extra)
    assert ct_in + ct_extra_tag == whole


# ------------------------------------------------------------------ batches vs the oracle

def _keys(ctx, specs, seed):
    rng = np.random.default_rng(seed)
    keys, orc_keys = [], []
    for suite in specs:
        k = ctx.key(suite, rng.integers(0, 256, qpp.HASH_LEN[suite], dtype=np.uint8).tobytes())
        keys.append(k)
        kk, iv, hp = k.material()
        orc_keys.append((suite, kk, iv, hp))
    return keys, orc.make_keys(orc_keys)


def _ragged_batch(n, slots, seed, max_len=1500):
    rng = np.random.default_rng(seed)
    pt = rng.integers(0, max_len + 1, n).astype(np.int64)
    pt[:8] = [0, 1, 15, 16, 17, 31, 32, 33]
    aad = rng.choice([0, 1, 5, 6, 16, 21, 22, 45], n).astype(np.int64)
    pn_len = rng.integers(1, 5, n)
    aad = np.maximum(aad, pn_len)  # the header holds the PN bytes
    pt = np.maximum(pt, 4 - pn_len + 0)  # sample must fit (encoding.rs:179-186 pads to ensure it)
    sizes = aad + pt + 16
    offs = np.concatenate([[0], np.cumsum(sizes + rng.integers(0, 9, n))[:-1]]).astype(np.int64)
    arena = rng.integers(0, 256, int(offs[-1] + sizes[-1] + 64), dtype=np.uint8)
    descs = np.zeros(n, dtype=qpp.PKT_DTYPE)
    descs["pn"] = rng.integers(0, 2**62, n, dtype=np.uint64)
    descs["key_idx"] = np.asarray(slots, dtype=np.uint32)[rng.integers(0, len(slots), n)]
    descs["off"] = offs
    descs["aad_len"] = aad
    descs["pt_len"] = pt
    descs["pn_len"] = pn_len
    return descs, arena


def _run_seal(ctx, descs, arena, flags):
    n = len(descs)
    d_desc, d_arena = ctx.alloc(descs.nbytes), ctx.alloc(arena.nbytes)
    d_mask, d_status = ctx.alloc(5 * n), ctx.alloc(n)
    d_desc.upload(descs)
    d_arena.upload(arena)
    ctx.seal_batch(d_desc, n, d_arena, d_mask, d_status, flags)
    ctx.sync()
    out = d_arena.download(), d_mask.download(), d_status.download(dtype=np.int8)
    for b in (d_desc, d_arena, d_mask, d_status):
        b.free()
    return out


def _run_open(ctx, descs, arena):
    n = len(descs)
    d_desc, d_arena, d_status = ctx.alloc(descs.nbytes), ctx.alloc(arena.nbytes), ctx.alloc(n)
    d_desc.upload(descs)
    d_arena.upload(arena)
    ctx.open_batch(d_desc, n, d_arena, d_status)
    ctx.sync()
    out = d_arena.download(), d_status.download(dtype=np.int8)
    for b in (d_desc, d_arena, d_status):
        b.free()
    return out


def _oracle_keys_for(keys_orc, descs, slots):
    """oracle keys are indexed 0..K-1; map device slots to oracle indices"""
    remap = {s: i for i, s in enumerate(slots)}
    d = descs.copy()
    d["key_idx"] = [remap[int(s)] for s in descs["key_idx"]]
    return d


@pytest.mark.parametrize("specs", [[1], [2], [3], [1, 1, 2, 3, 3, 2, 1, 3]], ids=["aes128", "aes256", "chacha", "mixed"])
def test_batch_seal_open_ragged(ctx, specs, path):
    keys, okeys = _keys(ctx, specs, seed=len(specs) * 31 + specs[0])
    slots = [k.slot for k in keys]
    descs, arena = _ragged_batch(2048, slots, seed=7 + len(specs))
    flags = qpp.HP_MASK_OUT | qpp.HP_APPLY
    got_arena, got_masks, got_status = _run_seal(ctx, descs, arena, flags)
    want_arena = arena.copy()
    want_masks = orc.seal_batch(okeys, _oracle_keys_for(okeys, descs, slots), want_arena, flags)
    assert (got_status == 0).all()
    assert got_masks.tobytes() == want_masks
    bad = np.nonzero(got_arena != want_arena)[0]
    assert bad.size == 0, f"first mismatch at arena byte {bad[:8]}"

    # open needs the unprotected header: seal again without HP to get the AAD the receiver uses
    sealed_arena, _, _ = _run_seal(ctx, descs, arena, 0)
    tampered = np.zeros(len(descs), bool)
    tampered[::97] = True
    ct = sealed_arena.copy()
    for i in np.nonzero(tampered)[0]:
        d = descs[i]
        ct[int(d["off"]) + int(d["aad_len"]) + int(d["pt_len"]) + (i % 16)] ^= 1 << (i % 8)
    got_pt, st = _run_open(ctx, descs, ct)
    want_pt = ct.copy()
    want_st = orc.open_batch(okeys, _oracle_keys_for(okeys, descs, slots), want_pt)
    assert list(st) == want_st
    assert (st[tampered] == qpp.DECRYPT_ERROR).all() and (st[~tampered] == 0).all()
    assert (got_pt == want_pt).all()
    # round trip: untampered payloads are the original plaintext again
    for i in np.nonzero(~tampered)[0][:200]:
        d = descs[i]
        a, b = int(d["off"]) + int(d["aad_len"]), int(d["off"]) + int(d["aad_len"]) + int(d["pt_len"])
        assert (got_pt[a:b] == arena[a:b]).all()
    for k in keys:
        k.free()


@pytest.mark.parametrize("flags", [0, qpp.HP_MASK_OUT | qpp.HP_APPLY], ids=["nohp", "hp"])
def test_jumbo_and_edges(ctx, path, flags):
    """C4's 8000-B jumbo payload next to empty, 1-B, 4-B and near-64 KiB ones, with and without header protection
    (pn_len 4: the sample of an empty payload is the tag, payload.rs:151-169)."""
    keys, okeys = _keys(ctx, [1, 2, 3], seed=99)
    slots = [k.slot for k in keys]
    lens = [0, 1, 4, 8000, 8000, 1452, 300, 65535 - 100]
    n = len(lens) * 3
    descs = np.zeros(n, dtype=qpp.PKT_DTYPE)
    off = 0
    for i in range(n):
        L = lens[i % len(lens)]
        descs[i] = (2**32 + 7 * i if i % 2 else i, slots[i // len(lens)], off, 21, L, 4, 0, 0)
        off += 21 + L + 16 + 3
    arena = np.random.default_rng(5).integers(0, 256, off + 64, dtype=np.uint8)
    got, masks, st = _run_seal(ctx, descs, arena, flags)
    want = arena.copy()
    want_masks = orc.seal_batch(okeys, _oracle_keys_for(okeys, descs, slots), want, flags)
    assert (st == 0).all() and (got == want).all()
    if flags:
        assert masks.tobytes() == want_masks


def test_hp_mask_batch_receive_side(ctx):
    keys, okeys = _keys(ctx, [1, 3, 2], seed=3)
    slots = [k.slot for k in keys]
    descs, arena = _ragged_batch(512, slots, seed=11)
    descs["pt_len"] = np.maximum(descs["pt_len"], 20)
    descs["aad_len"] = np.maximum(descs["aad_len"], 4)
    descs["off"] = np.arange(512) * 1600
    arena = np.random.default_rng(2).integers(0, 256, 512 * 1600, dtype=np.uint8)
    recv = descs.copy()
    recv["pn_len"] = 0  # receive side: sample at header_len + 4
    d_desc, d_arena, d_mask = ctx.alloc(recv.nbytes), ctx.alloc(arena.nbytes), ctx.alloc(5 * 512)
    d_desc.upload(recv)
    d_arena.upload(arena)
    ctx.hp_mask_batch(d_desc, 512, d_arena, d_mask)
    got = d_mask.download().tobytes()
    for i in range(512):
        d = recv[i]
        k = okeys[slots.index(int(d["key_idx"]))]
        s = int(d["off"]) + int(d["aad_len"]) + 4
        want = orc.hp_mask(k.suite, bytes(k.hp)[:qpp.KEY_LEN[k.suite]], arena[s:s + 16].tobytes())
        assert got[5 * i:5 * i + 5] == want


@pytest.mark.parametrize("suite", [1, 2, 3, 0], ids=["aes128", "aes256", "chacha", "mixed"])
def test_full_size_round_trip(ctx, suite):
    """BASELINE configs 2/3 size (1 Mi x 1200 B): a seeded sample of sealed packets is bit-exact against the oracle and
    every packet against the full-size checker; the open of every packet (a tampered subset among them) is compared
    with the expected arena byte for byte.  mixed: 66 keys of all three suites in ONE batch (negotiated.rs:15-30; the
    single both-sizes AES launch and the plan-selected ChaCha20 packets)."""
    n, pt_len = 1 << 20, 1200
    keys, okeys = _keys(ctx, ([suite] * (1 if suite == 1 else 64)) if suite else [1, 2, 3] * 22, seed=suite)
    slots = [k.slot for k in keys]
    descs, arena = qpp.make_batch(n, pt_len, slots, seed=0x5eed0002, pn_base=(2**32 if suite == 2 else 0))
    d_desc, d_arena, d_mask, d_status = ctx.alloc(descs.nbytes), ctx.alloc(arena.nbytes), ctx.alloc(5 * n), ctx.alloc(n)
    d_desc.upload(descs)
    d_arena.upload(arena)
    ctx.seal_batch(d_desc, n, d_arena, d_mask, d_status, qpp.HP_MASK_OUT)
    sealed = d_arena.download()
    masks = d_mask.download()
    stride = arena.size // n
    rng = np.random.default_rng(suite)
    pick = np.sort(rng.choice(n, 1500, replace=False))
    sub_descs = descs[pick].copy()
    sub_arena = np.concatenate([arena[i * stride:(i + 1) * stride] for i in pick])
    sub_descs["off"] = np.arange(len(pick)) * stride
    sub_want = sub_arena.copy()
    want_masks = orc.seal_batch(okeys, _oracle_keys_for(okeys, sub_descs, slots), sub_want, qpp.HP_MASK_OUT)
    sub_got = np.concatenate([sealed[i * stride:(i + 1) * stride] for i in pick])
    assert (sub_got == sub_want).all()
    assert np.concatenate([masks[5 * i:5 * i + 5] for i in pick]).tobytes() == want_masks
    # and EVERY packet (ciphertext, tag, mask) against the full-size checker (oracle/fastcheck.c)
    assert orc.check_full_seal(okeys, slots, descs, arena, sealed, masks, qpp.HP_MASK_OUT) == n
    # open EVERY packet and compare the whole arena byte for byte (only the round trip and the status were
    # checked at this size): one packet in 997 tampered -- a ciphertext bit or a tag bit -- must come back
    # DECRYPT_ERROR with its payload zeroed (aead/default.rs:65-93: no unauthenticated plaintext), every other one
    # with its plaintext; headers and tags are left as they were
    bad = np.arange(3, n, 997)
    tampered = sealed.copy().reshape(n, stride)
    for j, i in enumerate(bad):
        col = 21 + int(i % pt_len) if j % 2 == 0 else 21 + pt_len + int(i % 16)
        tampered[i, col] ^= np.uint8(1 << (j % 8))
    d_arena.upload(tampered.reshape(-1))
    ctx.open_batch(d_desc, n, d_arena, d_status)
    st = d_status.download(dtype=np.int8)
    opened = d_arena.download().reshape(n, stride)
    want_st = np.zeros(n, dtype=np.int8)
    want_st[bad] = qpp.DECRYPT_ERROR
    assert (st == want_st).all()
    want = tampered.copy()
    a = arena.reshape(n, stride)
    want[:, 21:21 + pt_len] = a[:, 21:21 + pt_len]
    want[bad, 21:21 + pt_len] = 0
    assert (opened == want).all()
    # the oracle's open on a sample of the tampered packets and their neighbours: the same statuses and bytes
    pick = np.sort(np.concatenate([bad[:40], bad[:40] + 1]))
    sub_d = descs[pick].copy()
    sub_d["off"] = np.arange(len(pick)) * stride
    sub_a = np.concatenate([tampered[i] for i in pick])
    want_sub = orc.open_batch(okeys, _oracle_keys_for(okeys, sub_d, slots), sub_a)
    assert (np.array(want_sub, dtype=np.int8) == st[pick]).all()
    assert (sub_a.reshape(len(pick), stride) == opened[pick]).all()
    # a checksum of checksums over the ciphertext: identical across two runs (determinism)
    d_arena.upload(arena)
    ctx.seal_batch(d_desc, n, d_arena, d_mask, d_status, qpp.HP_MASK_OUT)
    assert (d_arena.download() == sealed).all()
    for b in (d_desc, d_arena, d_mask, d_status):
        b.free()
    for k in keys:
        k.free()


@pytest.mark.parametrize("kernel", ["quad", "wave"])
def test_full_size_many_keys(ctx, kernel):
    """1 Mi x 1200 B over 4096 AES keys (BASELINE configs[4]'s key count; 2048 AES-128 + 2048 AES-256, ~256 packets
    per key) through both throughput kernels: a seeded 2000-packet sample is bit-exact against the oracle (ciphertext,
    tag, mask) and every packet round-trips."""
    n, pt_len = 1 << 20, 1200
    rng = np.random.default_rng(77)
    batch = []
    for suite in (1, 2):
        batch += ctx.keys_batch(suite, [rng.integers(0, 256, qpp.HASH_LEN[suite], dtype=np.uint8).tobytes()
                                        for _ in range(2048)], 1)
    slots = [k.slot for k in batch]
    okeys = orc.make_keys([(k.suite, *k.material()) for k in batch])
    ctx.set_aes_kernel(qpp.AES_KERNEL_QUAD if kernel == "quad" else qpp.AES_KERNEL_WAVE)
    try:
        descs, arena = qpp.make_batch(n, pt_len, slots, seed=0x5eed0077)
        d_desc, d_arena, d_mask, d_status = (ctx.alloc(descs.nbytes), ctx.alloc(arena.nbytes), ctx.alloc(5 * n),
                                             ctx.alloc(n))
        d_desc.upload(descs)
        d_arena.upload(arena)
        ctx.seal_batch(d_desc, n, d_arena, d_mask, d_status, qpp.HP_MASK_OUT)
        sealed, masks = d_arena.download(), d_mask.download()
        assert (d_status.download(dtype=np.int8) == 0).all()
        stride = arena.size // n
        pick = np.sort(np.random.default_rng(78).choice(n, 2000, replace=False))
        sub_d = descs[pick].copy()
        sub_a = np.concatenate([arena[i * stride:(i + 1) * stride] for i in pick])
        sub_d["off"] = np.arange(len(pick)) * stride
        want = sub_a.copy()
        want_masks = orc.seal_batch(okeys, _oracle_keys_for(okeys, sub_d, slots), want, qpp.HP_MASK_OUT)
        assert (np.concatenate([sealed[i * stride:(i + 1) * stride] for i in pick]) == want).all()
        assert np.concatenate([masks[5 * i:5 * i + 5] for i in pick]).tobytes() == want_masks
        assert orc.check_full_seal(okeys, slots, descs, arena, sealed, masks, qpp.HP_MASK_OUT) == n  # every packet
        ctx.open_batch(d_desc, n, d_arena, d_status)
        assert (d_status.download(dtype=np.int8) == 0).all()
        v, a = d_arena.download().reshape(n, stride), arena.reshape(n, stride)
        assert (v[:, 21:21 + pt_len] == a[:, 21:21 + pt_len]).all()
        for b in (d_desc, d_arena, d_mask, d_status):
            b.free()
    finally:
        ctx.set_aes_kernel(qpp.AES_KERNEL_AUTO)
        ctx.free_keys(batch)


# ------------------------------------------------------------------ receive path: unprotect -> PN expand -> open

def _rx_batch(ctx, n, seed):
    """Protected packets as a peer sends them: short headers (key phase 0/1) and long headers, PN truncated
    against the receiver's largest acknowledged PN, some tampered tags and some too short for a sample."""
    rng = np.random.default_rng(seed)
    keys, orc_keys = [], []
    for suite in (1, 2, 3):
        k0 = ctx.key(suite, rng.integers(0, 256, qpp.HASH_LEN[suite], dtype=np.uint8).tobytes())
        k1 = k0.derive_next_key()  # KeySet crypto[1]: the next phase, same header key
        for k in (k0, k1):
            keys.append(k)
            orc_keys.append((suite, *k.material()))
    okeys = orc.make_keys(orc_keys)
    chunks, rx, orx, want_pn, want_payload = [], [], [], [], []
    off = 0
    for i in range(n):
        s = int(rng.integers(0, 3))  # suite index
        largest = int(rng.integers(0, 2**62 - 2**20)) if i % 3 else int(rng.integers(0, 300))
        pn = largest + int(rng.integers(0, 400))
        rc, _, pn_len = orc.truncate_pn(pn, largest)
        pn_len = min(4, pn_len + int(rng.integers(0, 2)))  # a sender may use a longer encoding
        long_hdr = i % 5 == 0
        phase = 0 if long_hdr else int(rng.integers(0, 2))
        if long_hdr:
            first = 0xc0 | (int(rng.integers(0, 4)) << 4) | (pn_len - 1)
            rest = rng.integers(0, 256, int(rng.integers(6, 40)), dtype=np.uint8).tobytes()
        else:
            first = 0x40 | (phase << 2) | (pn_len - 1)
            rest = rng.integers(0, 256, int(rng.integers(0, 21)), dtype=np.uint8).tobytes()
        header = bytes([first]) + rest
        pt = int(rng.integers(max(0, 4 - pn_len), 1400)) if i % 7 else max(0, 4 - pn_len)
        payload = rng.integers(0, 256, pt, dtype=np.uint8).tobytes()
        kk = orc_keys[2 * s + phase]
        rc, pkt = orc.protect_packet(kk[0], kk[1], kk[2], kk[3], pn, header, pn_len, payload)
        assert rc == 0
        pkt = bytearray(pkt)
        if i % 11 == 3:
            pkt[-1 - i % 16] ^= 0x20  # tampered tag / ciphertext -> DECRYPT_ERROR
        length = len(pkt)
        if i % 13 == 5:
            length = len(header) + 19  # no room for the 16-byte sample at header_len + 4 -> DECODE_ERROR
            pkt = pkt[:length]
        chunks.append(bytes(pkt) + bytes(int(rng.integers(0, 7))))
        rx.append((largest, (keys[2 * s].slot, keys[2 * s + 1].slot), off, len(header), length))
        orx.append((largest, (2 * s, 2 * s + 1), off, len(header), length))
        want_pn.append(pn)
        want_payload.append(payload)
        off += len(chunks[-1])
    arena = np.frombuffer(b"".join(chunks) + bytes(64), dtype=np.uint8).copy()
    return keys, okeys, np.array(rx, dtype=qpp.RX_DTYPE), np.array(orx, dtype=qpp.RX_DTYPE), arena, want_pn, want_payload


def test_unprotect_open_batch(ctx, path):
    n = 1500
    keys, okeys, rx, orx, arena, want_pn, want_payload = _rx_batch(ctx, n, seed=21)
    d_rx, d_arena = ctx.alloc(rx.nbytes), ctx.alloc(arena.nbytes)
    d_out, d_status = ctx.alloc(n * qpp.PKT_DTYPE.itemsize), ctx.alloc(n)
    d_rx.upload(rx)
    d_arena.upload(arena)
    ctx.unprotect_open_batch(d_rx, n, d_arena, d_out, d_status)
    ctx.sync()
    got_arena = d_arena.download()
    got_out = d_out.download(dtype=qpp.PKT_DTYPE)
    got_st = d_status.download(dtype=np.int8)
    want_arena = arena.copy()
    want_out, want_st = orc.unprotect_open_batch(okeys, orx, want_arena)
    assert list(got_st) == want_st
    assert (got_arena == want_arena).all()
    slot_of = [k.slot for k in keys]
    for f in ("pn", "aad_len", "pt_len", "pn_len", "flags", "off"):
        assert (got_out[f] == want_out[f]).all(), f
    assert [int(s) for s in got_out["key_idx"]] == [slot_of[int(k)] for k in want_out["key_idx"]]
    # every authentic packet decodes to the sender's packet number and plaintext
    ok = np.nonzero(got_st == 0)[0]
    assert len(ok) > n // 2 and (got_st[[i for i in range(n) if i % 13 == 5]] == qpp.DECODE_ERROR).all()
    for i in ok:
        d = got_out[i]
        assert int(d["pn"]) == want_pn[i]
        a = int(d["off"]) + int(d["aad_len"])
        assert got_arena[a:a + int(d["pt_len"])].tobytes() == want_payload[i]
    for b in (d_rx, d_arena, d_out, d_status):
        b.free()
    for k in keys:
        k.free()


# ------------------------------------------------------------------ device key schedule (key-update churn)

@pytest.mark.parametrize("suite", [1, 2, 3])
def test_key_new_batch_matches_host_chain(ctx, suite):
    rng = np.random.default_rng(40 + suite)
    hl = qpp.HASH_LEN[suite]
    secrets = [rng.integers(0, 256, hl, dtype=np.uint8).tobytes() for _ in range(300)]
    for updates in (0, 1, 3):
        batch = ctx.keys_batch(suite, secrets, updates)
        for i in range(0, 300, 37):
            k = ctx.key(suite, secrets[i])
            hp0 = k.material()[2]
            for _ in range(updates):
                k = k.derive_next_key()
            assert batch[i].material() == k.material()
            assert batch[i].material()[2] == hp0  # the header key is never updated
            # the oracle agrees on the whole chain
            s = secrets[i]
            for _ in range(updates):
                s = orc.update_secret(suite, s)
            key, iv, _ = orc.derive(suite, s)
            assert batch[i].material()[:2] == (key, iv)
            k.free()
        # the device-made records seal bit-exactly (round keys, H powers, nonce)
        slots = [k.slot for k in batch]
        descs, arena = qpp.make_batch(600, 700, slots, seed=77 + updates)
        okeys = orc.make_keys([(suite, *k.material()) for k in batch])
        got, masks, st = _run_seal(ctx, descs, arena, qpp.HP_MASK_OUT)
        want = arena.copy()
        want_masks = orc.seal_batch(okeys, _oracle_keys_for(okeys, descs, slots), want, qpp.HP_MASK_OUT)
        assert (st == 0).all() and (got == want).all() and masks.tobytes() == want_masks
        for k in batch:
            k.free()


def test_many_keys_small_batch(ctx, path):
    """3000 live keys (AES-128, AES-256 and ChaCha mixed) and 6000 short packets over them: the single-launch plan
    scans 3 key slots per thread (key table > 1024 slots) and empty keys share work-item starts; every packet is
    bit-exact against the oracle on both kernel paths."""
    rng = np.random.default_rng(91)
    batch = []
    for suite, count in ((1, 1200), (2, 900), (3, 900)):
        hl = qpp.HASH_LEN[suite]
        batch += ctx.keys_batch(suite, [rng.integers(0, 256, hl, dtype=np.uint8).tobytes() for _ in range(count)])
    slots = [k.slot for k in batch]
    used = [slots[i] for i in rng.choice(len(slots), 700, replace=False)]  # most keys get no packet at all
    descs, arena = _ragged_batch(6000, used, seed=92, max_len=300)
    okeys = orc.make_keys([(k.suite, *k.material()) for k in batch])
    flags = qpp.HP_MASK_OUT
    got, masks, st = _run_seal(ctx, descs, arena, flags)
    want = arena.copy()
    want_masks = orc.seal_batch(okeys, _oracle_keys_for(okeys, descs, slots), want, flags)
    assert (st == 0).all()
    assert masks.tobytes() == want_masks
    assert (got == want).all()
    for k in batch:
        k.free()


# ------------------------------------------------------------------ deferred transmit queue (the TX caller)

@pytest.mark.parametrize("flush", ["zero_copy", "dma"])
def test_txq_deferred_seal_matches_encode_packet(ctx, path, flush, monkeypatch):
    """Packets encoded into the queue's ring the way PacketEncoder::encode_packet lays them out
    (packet/encoding.rs:115-282: header, truncated PN, payload, tag room), pushed instead of sealed, then one
    flush: every packet equals crypto::encrypt + crypto::protect of the oracle.  zero_copy: the kernels work on
    the pinned ring in place with a host-built plan; dma: ring -> HBM -> ring around a device batch."""
    monkeypatch.setenv("QPP_TXQ_ZC_MAX", "1024" if flush == "zero_copy" else "0")
    rng = np.random.default_rng(8)
    keys = [ctx.key(s, rng.integers(0, 256, qpp.HASH_LEN[s], dtype=np.uint8).tobytes()) for s in (1, 2, 3)]
    q = qpp.TxQueue(ctx, 1 << 20, 1024)
    want, off = [], 0
    largest = int(rng.integers(0, 2**40))
    for i in range(600):
        k = keys[i % 3]
        pn = largest + 1 + i
        trunc, pn_len = qpp.pn_truncate(pn, largest)
        header = bytes([0x40 | (pn_len - 1)]) + rng.integers(0, 256, 16, dtype=np.uint8).tobytes()  # short header
        payload = rng.integers(0, 256, int(rng.integers(4, 1300)), dtype=np.uint8).tobytes()
        pkt = header + trunc.to_bytes(pn_len, "big") + payload
        q.ring[off:off + len(pkt)] = np.frombuffer(pkt, dtype=np.uint8)
        q.push(k, pn, off, len(header), pn_len, len(payload))
        suite, (kk, iv, hp) = k.suite, k.material()
        rc, protected = orc.protect_packet(suite, kk, iv, hp, pn, header, pn_len, payload)
        want.append((off, protected))
        off += len(protected) + int(rng.integers(0, 5))
    assert q.pending() == 600
    q.flush()
    assert q.pending() == 0
    for o, p in want:
        assert q.ring[o:o + len(p)].tobytes() == p
    # the sample must fit (encoding.rs:178-188 pads short payloads); the queue refuses instead of sealing
    with pytest.raises(qpp.QppError) as e:
        q.push(keys[0], 1, 0, 17, 1, 2)
    assert e.value.code == qpp.DECODE_ERROR
    with pytest.raises(qpp.QppError):
        q.push(keys[0], 1, (1 << 20) - 20, 17, 1, 100)  # does not fit the ring
    q.close()
    for k in keys:
        k.free()


@pytest.mark.parametrize("coalesce", [1, 3])
@pytest.mark.parametrize("flush", ["zero_copy", "dma"])
def test_txq_async_bursts_in_flight(ctx, flush, coalesce, monkeypatch):
    """GSO bursts flushed without waiting (qpp_txq_flush_async): 24 bursts of 64 packets, up to 8 in flight on the
    queue's streams, each in its own region of the ring; back-pressure reuses a slot only after its flush is over.
    Every packet equals crypto::encrypt + crypto::protect of the oracle once its ticket completes."""
    monkeypatch.setenv("QPP_TXQ_ZC_MAX", "1024" if flush == "zero_copy" else "0")
    rng = np.random.default_rng(18)
    keys = [ctx.key(s, rng.integers(0, 256, qpp.HASH_LEN[s], dtype=np.uint8).tobytes()) for s in (1, 2, 3, 1)]
    region, bursts, per = 96 << 10, 24, 64
    q = qpp.TxQueue(ctx, region * bursts, per * coalesce, in_flight=8)
    q.set_coalesce(coalesce)  # bursts held back and sent `coalesce` at a time (poll / wait send a held one at once)
    largest = int(rng.integers(0, 2**40))
    want, tickets, pn = [], [], largest + 1
    for b in range(bursts):
        off = b * region
        staged = np.zeros(per, dtype=qpp.PKT_DTYPE)  # odd bursts go in with one qpp_txq_push_descs call
        for i in range(per):
            k = keys[(b + i) % len(keys)]
            trunc, pn_len = qpp.pn_truncate(pn, largest)
            header = bytes([0x40 | (pn_len - 1)]) + rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
            payload = rng.integers(0, 256, int(rng.integers(4, 1400)), dtype=np.uint8).tobytes()
            pkt = header + trunc.to_bytes(pn_len, "big") + payload
            q.ring[off:off + len(pkt)] = np.frombuffer(pkt, dtype=np.uint8)
            if b % 2:
                staged[i] = (pn, k.slot, off, len(header) + pn_len, len(payload), pn_len, 0, 0)
            else:
                q.push(k, pn, off, len(header), pn_len, len(payload))
            suite, (kk, iv, hp) = k.suite, k.material()
            want.append((off, orc.protect_packet(suite, kk, iv, hp, pn, header, pn_len, payload)[1]))
            off += len(pkt) + 16
            pn += 1
        if b % 2:
            q.push_descs(staged)
        assert q.pending() == per
        tickets.append(q.flush_async())
        assert q.pending() == 0
    for t in tickets[::-1]:  # any order
        q.wait(t)
        assert q.poll(t)
    for o, p in want:
        assert q.ring[o:o + len(p)].tobytes() == p
    assert q.flush_async() == 0  # nothing pushed: ticket 0, complete
    q.close()
    for k in keys:
        k.free()


# ------------------------------------------------------------------ dc consumers

@pytest.mark.parametrize("name,suite", [("aead_aes128gcm.json", 1), ("aead_aes256gcm.json", 2),
                                        ("aead_chacha20poly1305.json", 3)])
def test_dc_application_fixtures(ctx, name, suite):
    """dc seal/open::Application (dc/s2n-quic-dc/src/crypto/awslc.rs:53-83,176-227) on the golden vectors:
    the dc nonce (crypto.rs:178-185 into_nonce, awslc.rs:364-370 xor iv) is the QUIC one, so the same CT || tag."""
    for c in load_golden(name)["cases"]:
        k = ctx.dc_key(suite, H(c["key"]), H(c["iv"]))
        pt, aad, want = H(c["pt"]), H(c["aad"]), H(c["ct"] + c["tag"])
        assert k.dc_encrypt(c["pn"], aad, None, pt + bytes(16)) == want
        cut = len(pt) // 3  # extra_payload: the tail of the message arrives separately
        assert k.dc_encrypt(c["pn"], aad, pt[cut:], pt[:cut] + bytes(len(pt) - cut + 16)) == want
        ct, tag = want[:-16], want[-16:]
        assert k.dc_decrypt(0, c["pn"], aad, ct, tag) == pt
        rc, buf = k.dc_decrypt_in_place(0, c["pn"], aad, ct, tag)
        assert rc == qpp.OK and buf == pt
        with pytest.raises(qpp.QppError) as e:  # ensure!(key_phase == Zero, RotationNotSupported)
            k.dc_decrypt(1, c["pn"], aad, ct, tag)
        assert e.value.code == qpp.ROTATION_NOT_SUPPORTED
        bad = bytearray(tag)
        bad[0] ^= 1
        with pytest.raises(qpp.DecryptError):
            k.dc_decrypt(0, c["pn"], aad, ct, bytes(bad))
        rc, buf = k.dc_decrypt_in_place(0, c["pn"], aad, ct, bytes(bad))
        assert rc == qpp.DECRYPT_ERROR and buf == bytes(len(ct))  # never releases unauthenticated plaintext
        rc, _ = k.dc_decrypt_in_place(0, c["pn"], aad, ct, tag[:15])
        assert rc == qpp.DECRYPT_ERROR
        k.free()


def test_dc_seal_capacity(ctx):
    k = ctx.dc_key(1, bytes(16), bytes(12))
    with pytest.raises(qpp.QppError) as e:  # payload_and_tag.len() >= tag_len + extra_in.len() (awslc.rs:65-67)
        k.dc_encrypt(1, b"h", bytes(10), bytes(20))
    assert e.value.code == qpp.INTERNAL_ERROR
    assert len(k.dc_encrypt(1, b"h", bytes(4), bytes(20))) == 20
    k.free()
