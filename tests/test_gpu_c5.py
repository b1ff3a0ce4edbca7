"""BASELINE configs[4] (C5) under parity, at one GPU's shard: key-update churn with 4 Ki rotating 1-RTT keys,
2 Mi x 1200 B packets (16 Mi / 8 GPUs), end to end through host memory (qpp_host_batch_*: chunked H2D -> seal / open
-> D2H).

Shape of the churn (quic/s2n-quic-core/src/crypto/application/keyset.rs:75-96 rotate_phase, cipher_suite.rs:68-83
update): the 4096 keys are built on the device by qpp_key_new_batch from 4096 secrets with 3 "quic ku" updates each;
batch A (first 1 Mi packets) is submitted; while it is in flight half the keys are rotated (qpp_key_update_batch)
and the OLD keys of that half are freed; batch B (second 1 Mi packets) names the new keys for that half.  Checks:
  * a seeded sample of 4096 packets of A and B (ciphertext, tag, HP mask) is bit-exact with the oracle, using the
    keys each packet was sealed with (A: all old keys, freed mid-flight; B: rotated or kept), and EVERY packet is
    bit-exact with the full-size checker (oracle/fastcheck.c, itself checked against the oracle);
  * every packet round-trips: A is opened with the old keys re-created from their material, B with its own keys;
    every status is OK and every payload equals the original plaintext.
"""
import numpy as np
import pytest

import _oracle as orc
import qpp

pytestmark = pytest.mark.gpu

N_KEYS = 4096
N = 2 << 20
PT = 1200


def test_c5_rotating_keys_end_to_end():
    ctx = qpp.Context(0)
    try:
        _run(ctx)
    finally:
        ctx.close()


def _run(ctx):
    rng = np.random.default_rng(0xC5)
    suite = qpp.SUITE_AES_128_GCM
    secrets = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(N_KEYS)]
    keys = ctx.keys_batch(suite, secrets, 3)  # device key schedule, 3 updates deep
    old_mat = [k.material() for k in keys]
    slots_old = np.array([k.slot for k in keys], dtype=np.uint32)
    # packets -> key index (which of the 4096 connections), spread like make_batch's splitmix
    descs, arena = qpp.make_batch(N, PT, list(range(N_KEYS)), seed=0xC5C5)
    conn = descs["key_idx"].astype(np.int64)  # connection id per packet
    descs["key_idx"] = slots_old[conn]
    half = N // 2
    host = ctx.host_alloc(arena.nbytes)
    host[:] = arena
    stride = arena.size // N
    masks = np.zeros(5 * N, np.uint8)
    st = np.full(N, 77, np.int8)
    dA, dB = descs[:half].copy(), descs[half:].copy()

    tA = ctx.host_submit(dA, host, masks[:5 * half], st[:half], qpp.HP_MASK_OUT, qpp.OP_SEAL)
    # while A is in flight: rotate connections [0, 2048), free their old keys
    rot = np.arange(N_KEYS // 2)
    new = ctx.update_keys([keys[i] for i in rot])
    for i in rot:
        keys[i].free()
        keys[i] = None
    new_mat = {int(i): k.material() for i, k in zip(rot, new)}
    slots_now = slots_old.copy()
    slots_now[rot] = [k.slot for k in new]
    dB["key_idx"] = slots_now[conn[half:]]
    tB = ctx.host_submit(dB, host, masks[5 * half:], st[half:], qpp.HP_MASK_OUT, qpp.OP_SEAL)
    assert not ctx.host_done(tB) or True
    ctx.host_wait(tA)
    ctx.host_wait(tB)
    assert (st == 0).all()

    # oracle on a seeded sample: A with the old keys, B with the rotated / kept ones
    pick = np.sort(rng.choice(N, 4096, replace=False))
    mats, kidx = [], []
    for i in pick:
        c = int(conn[i])
        m = new_mat[c] if (i >= half and c in new_mat) else old_mat[c]
        kidx.append(len(mats))
        mats.append((suite, *m))
    okeys = orc.make_keys(mats)
    sub = descs[pick].copy()
    sub["off"] = np.arange(len(pick)) * stride
    sub["key_idx"] = kidx
    sub_arena = np.concatenate([arena[i * stride:(i + 1) * stride] for i in pick])
    want_masks = orc.seal_batch(okeys, sub, sub_arena, qpp.HP_MASK_OUT)
    got = np.concatenate([host[i * stride:(i + 1) * stride] for i in pick])
    assert (got == sub_arena).all(), "ciphertext/tag differ from the oracle"
    assert np.concatenate([masks[5 * i:5 * i + 5] for i in pick]).tobytes() == want_masks

    # every packet against the full-size checker (oracle/fastcheck.c): oracle keys 0..4095 = the old keys,
    # 4096 + c = connection c's rotated key (batch B only)
    all_keys = orc.make_keys([(suite, *old_mat[c]) for c in range(N_KEYS)] +
                             [(suite, *new_mat[int(c)]) for c in rot])
    full = descs.copy()
    kk = conn.copy()
    rotated_b = (np.arange(N) >= half) & np.isin(conn, rot)
    kk[rotated_b] = N_KEYS + conn[rotated_b]
    full["key_idx"] = kk
    want_all = arena.copy()
    want_all_masks = orc.fast_seal_batch(all_keys, full, want_all, qpp.HP_MASK_OUT)
    assert (host == want_all).all(), "a packet differs from the full-size checker"
    assert (masks == want_all_masks).all()

    # full round trip: A with its (freed) old keys re-created from their material, B with its own keys
    recreated = {int(i): ctx.raw_key(suite, *old_mat[i]) for i in rot}
    slots_a = slots_old.copy()
    slots_a[rot] = [recreated[int(i)].slot for i in rot]
    dA["key_idx"] = slots_a[conn[:half]]
    st[:] = 77
    tA = ctx.host_submit(dA, host, None, st[:half], 0, qpp.OP_OPEN)
    tB = ctx.host_submit(dB, host, None, st[half:], 0, qpp.OP_OPEN)
    ctx.host_wait(tA)
    ctx.host_wait(tB)
    assert (st == 0).all()
    body = np.s_[:, 21:21 + PT]
    assert (host.reshape(N, stride)[body] == arena.reshape(N, stride)[body]).all()
    ctx.host_free(host)
    for k in list(recreated.values()) + new + [k for k in keys if k is not None]:
        k.free()
