"""A seeded random sequence of engine operations, as a busy endpoint issues them: seal and open batches of every size
class (one-wave burst, lane and wave-item kernels, ChaCha), over random mixes of the three suites, with and without
header protection, on two streams of one context; receive batches (unprotect -> PN expand -> open); GSO bursts through
the transmit queue's asynchronous flushes (its own streams); host-memory batches through the chunked H2D -> seal ->
D2H pipeline (re-chunked at random); all interleaved with key updates, frees, new keys and
device key batches while earlier work is still in flight, and with the kernel-choice knobs changed between batches.

Every batch is checked against the full-size checker (oracle/fastcheck.c, itself checked against the restatement in
tests/test_fastcheck.py) with the key material it was ENQUEUED with: the stream-ordered key retirement
(include/qpp.h) must keep freed and rotated keys valid for the work already queued.  Opened batches carry tampered
packets (DECRYPT_ERROR, payload zeroed).  Bit-exact on every byte, mask and status.
"""
import numpy as np
import pytest

import _oracle as orc
import qpp

pytestmark = pytest.mark.gpu

SIZES = [1, 7, 64, 300, 2000, 5000, 20000]


def _secret(rng, suite):
    return rng.integers(0, 256, qpp.HASH_LEN[suite], dtype=np.uint8).tobytes()


def _batch(rng, n, nkeys, hp):
    descs = np.zeros(n, dtype=qpp.PKT_DTYPE)
    pn_len = rng.integers(1, 5, n)
    aad = pn_len + rng.integers(0, 40, n)
    pt = rng.integers(4 if hp else 0, 1500, n)
    big = rng.random(n) < 0.01
    pt[big] = rng.integers(1500, 8000, int(big.sum()))
    size = aad + pt + 16
    descs["off"] = np.concatenate([[0], np.cumsum(size + rng.integers(0, 9, n))[:-1]])
    descs["pn"] = rng.integers(0, 2**62, n, dtype=np.uint64)
    descs["aad_len"], descs["pt_len"], descs["pn_len"] = aad, pt, pn_len
    which = rng.integers(0, nkeys, n)
    arena = rng.integers(0, 256, int(descs["off"][-1] + size[-1]) + 64, dtype=np.uint8)
    return descs, which, arena


class _Pending:
    def __init__(self, kind, bufs, want, want_masks, want_status, n, tag):
        self.kind, self.bufs, self.want, self.want_masks, self.want_status, self.n, self.tag = (
            kind, bufs, want, want_masks, want_status, n, tag)

    def check(self, ctx):
        d_desc, d_arena, d_mask, d_status = self.bufs
        ctx.synchronize()
        got = d_arena.download()
        st = d_status.download(dtype=np.int8)
        bad = np.flatnonzero(st != self.want_status)
        if len(bad):
            desc = d_desc.download(dtype=qpp.PKT_DTYPE)
            print("HISTORY", *HISTORY[-40:], sep="\n", flush=True)
            print("bad key slots", sorted(set(int(x) for x in desc["key_idx"][bad])), "batch slots",
                  sorted(set(int(x) for x in desc["key_idx"])), flush=True)
        assert not len(bad), f"{self.tag}: status of {len(bad)} packets, first {bad[:8].tolist()}: " \
                             f"got {st[bad[:8]].tolist()} want {self.want_status[bad[:8]].tolist()}"
        assert (got == self.want).all(), f"{self.tag}: arena bytes differ"
        if self.want_masks is not None:
            m = d_mask.download()[:5 * self.n]
            assert (m == self.want_masks).all(), f"{self.tag}: HP masks"
        for b in self.bufs:
            if b is not None:
                b.free()


HISTORY = []
TRACE = bool(__import__("os").environ.get("QPP_FUZZ_TRACE"))
SEEDS = [0xF022, 0xF023, 0xF024, 0xF025] + [0xF100 + i for i in range(int(__import__("os").environ.get("QPP_FUZZ_EXTRA", "8")))]


TXQ_REGIONS, TXQ_REGION = 8, 1 << 17


class _Check:
    """a deferred check: fn() asserts, then releases what it holds"""

    def __init__(self, fn):
        self.fn = fn

    def check(self, ctx):
        self.fn()


def _rx_op(ctx, rng, chosen, stream, tag):
    """a GRO batch of protected short-header packets (phase 0) -> qpp_unprotect_open_batch, some tampered"""
    n = int(rng.integers(1, 150))
    chunks, rx, orx, off = [], [], [], 0
    for i in range(n):
        j = int(rng.integers(0, len(chosen)))
        suite, k, iv, hp = chosen[j][1]
        largest = int(rng.integers(0, 2**40))
        pn = largest + int(rng.integers(0, 300))
        _, _, pn_len = orc.truncate_pn(pn, largest)
        header = bytes([0x40 | (pn_len - 1)]) + rng.integers(0, 256, int(rng.integers(0, 20)), dtype=np.uint8).tobytes()
        payload = rng.integers(0, 256, int(rng.integers(4, 1400)), dtype=np.uint8).tobytes()
        _, pkt = orc.protect_packet(suite, k, iv, hp, pn, header, pn_len, payload)
        pkt = bytearray(pkt)
        if rng.random() < 0.05:
            pkt[-1] ^= 4
        chunks.append(bytes(pkt) + bytes(int(rng.integers(0, 5))))
        slot = chosen[j][0].slot
        rx.append((largest, (slot, slot), off, len(header), len(pkt)))
        orx.append((largest, (j, j), off, len(header), len(pkt)))
        off += len(chunks[-1])
    arena = np.frombuffer(b"".join(chunks) + bytes(64), dtype=np.uint8).copy()
    rx, orx = np.array(rx, dtype=qpp.RX_DTYPE), np.array(orx, dtype=qpp.RX_DTYPE)
    want = arena.copy()
    want_out, want_st = orc.unprotect_open_batch(orc.make_keys([c[1] for c in chosen]), orx, want)
    bufs = [ctx.alloc(rx.nbytes), ctx.alloc(arena.nbytes), ctx.alloc(n * qpp.PKT_DTYPE.itemsize), ctx.alloc(n)]
    d_rx, d_arena, d_out, d_st = bufs
    d_rx.upload(rx)
    d_arena.upload(arena)
    d_st.upload(np.full(n, 0x55, dtype=np.uint8))
    ctx.unprotect_open_batch(d_rx, n, d_arena, d_out, d_st, stream=stream)

    def fn():
        ctx.synchronize()
        st = d_st.download(dtype=np.int8)
        assert list(st) == want_st, f"{tag}: status"
        assert (d_arena.download() == want).all(), f"{tag}: arena"
        out = d_out.download(dtype=qpp.PKT_DTYPE)
        for f in ("pn", "aad_len", "pt_len", "pn_len", "off"):
            assert (out[f] == want_out[f]).all(), f"{tag}: {f}"
        for b in bufs:
            b.free()
    return _Check(fn)


def _host_op(ctx, rng, chosen, tag):
    """a batch in pinned host memory through the host pipeline (chunked H2D -> seal + HP mask -> D2H)"""
    n = int(rng.choice([1, 50, 3000, 30000]))
    descs, which, arena = _batch(rng, n, len(chosen), True)
    descs["key_idx"] = np.array([c[0].slot for c in chosen], dtype=np.uint32)[which]
    odescs = descs.copy()
    odescs["key_idx"] = which
    want = arena.copy()
    want_masks = orc.fast_seal_batch(orc.make_keys([c[1] for c in chosen]), odescs, want, qpp.HP_MASK_OUT)
    host = ctx.host_alloc(arena.nbytes)
    host[:] = arena
    masks = np.zeros(5 * n, np.uint8)
    st = np.full(n, 0x55, np.int8)
    t = ctx.host_submit(descs, host, masks, st, qpp.HP_MASK_OUT, qpp.OP_SEAL)

    def fn():
        ctx.host_wait(t)
        assert (st == 0).all(), f"{tag}: status"
        assert (host == want).all(), f"{tag}: arena"
        assert (masks == want_masks).all(), f"{tag}: masks"
        ctx.host_free(host)
    return _Check(fn)


def _txq_op(txq, rng, chosen, region, tickets, tag):
    """one GSO-sized burst pushed into the transmit queue's ring region and flushed asynchronously"""
    base, off, expect = region * TXQ_REGION, 0, []
    for _ in range(int(rng.integers(1, 65))):
        j = int(rng.integers(0, len(chosen)))
        key, (suite, k, iv, hp) = chosen[j]
        pn = int(rng.integers(0, 2**40))
        pn_len = int(rng.integers(1, 5))
        header = bytes([0x40 | (pn_len - 1)]) + rng.integers(0, 256, int(rng.integers(0, 20)), dtype=np.uint8).tobytes()
        payload = rng.integers(0, 256, int(rng.integers(4, 1400)), dtype=np.uint8).tobytes()
        pkt = header + (pn & ((1 << (8 * pn_len)) - 1)).to_bytes(pn_len, "big") + payload
        if off + len(pkt) + 16 > TXQ_REGION:
            break
        o = base + off
        txq.ring[o:o + len(pkt)] = np.frombuffer(pkt, dtype=np.uint8)
        txq.push(key, pn, o, len(header), pn_len, len(payload))
        expect.append((o, orc.protect_packet(suite, k, iv, hp, pn, header, pn_len, payload)[1]))
        off += len(pkt) + 16 + int(rng.integers(0, 9))
    t = txq.flush_async()
    tickets[region] = t

    def fn():
        txq.wait(t)
        for o, prot in expect:
            assert txq.ring[o:o + len(prot)].tobytes() == prot, f"{tag}: packet at ring offset {o}"
    return _Check(fn)


@pytest.mark.parametrize("seed", SEEDS)
def test_random_operation_sequence(seed):
    rng = np.random.default_rng(seed)
    HISTORY.clear()
    ctx = qpp.Context(0)
    side = ctx.new_stream()
    keys = []  # [Key, (suite, key, iv, hp)] -- the material a batch is checked with is taken when it is enqueued

    def new_key():
        s = int(rng.choice([1, 2, 3]))
        k = ctx.key(s, _secret(rng, s))
        keys.append([k, (s, *k.material())])

    for _ in range(6):
        new_key()
    pending, counts = [], {"seal": 0, "open": 0, "update": 0, "free": 0, "rx": 0, "txq": 0, "host": 0}
    txq = qpp.TxQueue(ctx, TXQ_REGIONS * TXQ_REGION, 512, in_flight=4)
    txq_tickets, txq_next, txq_checks = [0] * TXQ_REGIONS, [0], [None] * TXQ_REGIONS
    knobs = [16384, qpp.AES_KERNEL_AUTO]
    try:
        for step in range(160):
            op = rng.choice(["seal", "open", "update", "free", "new", "knob", "check", "rx", "txq", "newbatch", "host"],
                            p=[0.26, 0.16, 0.10, 0.07, 0.05, 0.06, 0.05, 0.08, 0.08, 0.03, 0.06])
            HISTORY.append((step, str(op), [(k.slot, m[0]) for k, m in keys], ctx.key_slots(), tuple(knobs)))
            if TRACE:
                print(*HISTORY[-1], flush=True)
            if op in ("seal", "open"):
                if not keys:
                    new_key()
                pick = rng.choice(len(keys), int(rng.integers(1, len(keys) + 1)), replace=False)
                chosen = [keys[i] for i in pick]
                n = int(rng.choice(SIZES))
                hp = op == "seal" and rng.random() < 0.7
                flags = (qpp.HP_MASK_OUT | (qpp.HP_APPLY if rng.random() < 0.5 else 0)) if hp else 0
                descs, which, arena = _batch(rng, n, len(chosen), hp)
                descs["key_idx"] = np.array([c[0].slot for c in chosen], dtype=np.uint32)[which]
                okeys = orc.make_keys([c[1] for c in chosen])
                odescs = descs.copy()
                odescs["key_idx"] = which
                stream = side if rng.random() < 0.5 else None
                knob_tag = f"burst_max={knobs[0]} aes_kernel={knobs[1]} stream={'side' if stream else 'ctx'} " \
                           f"suites={sorted({c[1][0] for c in chosen})}"
                d_desc, d_arena, d_status = ctx.alloc(descs.nbytes), ctx.alloc(arena.nbytes), ctx.alloc(n)
                d_mask = ctx.alloc(5 * n) if op == "seal" else None
                d_desc.upload(descs)
                d_status.upload(np.full(n, 0x55, dtype=np.uint8))  # every status must be written by the engine
                if op == "seal":
                    want = arena.copy()
                    want_masks = orc.fast_seal_batch(okeys, odescs, want, flags)
                    d_arena.upload(arena)
                    ctx.seal_batch(d_desc, n, d_arena, d_mask, d_status, flags, stream=stream)
                    pending.append(_Pending("seal", (d_desc, d_arena, d_mask, d_status), want,
                                            want_masks if flags & qpp.HP_MASK_OUT else None,
                                            np.zeros(n, np.int8), n, f"step {step} seal n={n} flags={flags} {knob_tag}"))
                else:
                    sealed = arena.copy()
                    orc.fast_seal_batch(okeys, odescs, sealed, 0)
                    bad = rng.random(n) < 0.05
                    want = arena.copy()  # opened: plaintext back, tag left in place
                    for i in range(n):
                        o, a, p = int(descs["off"][i]), int(descs["aad_len"][i]), int(descs["pt_len"][i])
                        want[o + a + p:o + a + p + 16] = sealed[o + a + p:o + a + p + 16]
                        if bad[i]:
                            j = o + a + int(rng.integers(0, p + 16))
                            sealed[j] ^= 0x10
                            want[o + a:o + a + p] = 0  # no unauthenticated plaintext is released
                            if j >= o + a + p:
                                want[j] = sealed[j]  # the flipped tag byte stays as received
                    d_arena.upload(sealed)
                    ctx.open_batch(d_desc, n, d_arena, d_status, stream=stream)
                    pending.append(_Pending("open", (d_desc, d_arena, None, d_status), want, None,
                                            np.where(bad, qpp.DECRYPT_ERROR, qpp.OK).astype(np.int8), n,
                                            f"step {step} open n={n} {knob_tag}"))
                counts[op] += 1
            elif op == "rx" and keys:
                chosen = [keys[i] for i in rng.choice(len(keys), int(rng.integers(1, len(keys) + 1)), replace=False)]
                stream = side if rng.random() < 0.5 else None
                pending.append(_rx_op(ctx, rng, chosen, stream, f"step {step} rx"))
                counts["rx"] += 1
            elif op == "txq" and keys:
                chosen = [keys[i] for i in rng.choice(len(keys), int(rng.integers(1, len(keys) + 1)), replace=False)]
                region = txq_next[0] % TXQ_REGIONS
                txq_next[0] += 1
                prev = txq_checks[region]
                if prev is not None and prev in pending:  # the region's previous burst: checked before its bytes go
                    prev.check(ctx)
                    pending.remove(prev)
                txq_checks[region] = _txq_op(txq, rng, chosen, region, txq_tickets, f"step {step} txq")
                pending.append(txq_checks[region])
                counts["txq"] += 1
            elif op == "host" and keys:
                chosen = [keys[i] for i in rng.choice(len(keys), int(rng.integers(1, len(keys) + 1)), replace=False)]
                if rng.random() < 0.3:  # re-chunk the pipeline (small chunks: many chunks per batch)
                    ctx.set_host_pipe(int(rng.choice([64, 1000, 65536])), int(rng.choice([1, 4, 64])) << 20,
                                      int(rng.integers(2, 5)))
                pending.append(_host_op(ctx, rng, chosen, f"step {step} host"))
                counts["host"] += 1
            elif op == "newbatch" and len(keys) < 10:
                s_ = int(rng.choice([1, 2, 3]))
                made = ctx.keys_batch(s_, [_secret(rng, s_) for _ in range(int(rng.integers(1, 3)))],
                                      int(rng.integers(0, 3)))
                keys.extend([k, (s_, *k.material())] for k in made)
            elif op == "update" and keys:
                pick = sorted(rng.choice(len(keys), int(rng.integers(1, len(keys) + 1)), replace=False))
                nxt = ctx.update_keys([keys[i][0] for i in pick])
                for i, k in zip(pick, nxt):
                    keys[i][0].free()  # the old key goes at once: batches queued with it still use it
                    keys[i] = [k, (k.suite, *k.material())]
                counts["update"] += 1
            elif op == "free" and len(keys) > 1:
                k, _ = keys.pop(int(rng.integers(0, len(keys))))
                k.free()
                counts["free"] += 1
            elif op == "new" and len(keys) < 12:
                new_key()
            elif op == "knob":
                knobs[0] = int(rng.choice([0, 64, 16384]))
                knobs[1] = int(rng.choice([qpp.AES_KERNEL_AUTO, qpp.AES_KERNEL_QUAD, qpp.AES_KERNEL_WAVE]))
                ctx.set_burst_max(knobs[0])
                ctx.set_aes_kernel(knobs[1])
            elif op == "check":
                for p in pending:
                    p.check(ctx)
                pending = []
        for p in pending:
            p.check(ctx)
        # the coverage floor is a property of the default seeds (their op mix is pinned); a soak seed
        # (QPP_FUZZ_EXTRA > 8) is a random mix and only has to have run every kind of operation
        # (round 6: soak seed 0xF12A drew 5 receive operations, every data check green)
        lo = (20, 12, 5, 5, 5) if seed < 0xF108 else (0, 0, 0, 0, 0)
        assert counts["seal"] > lo[0] and counts["open"] > lo[1] and counts["update"] > lo[2] and \
            counts["rx"] > lo[3] and counts["txq"] > lo[4], counts
    finally:
        txq.close()
        for k, _ in keys:
            k.free()
        ctx.set_burst_max(16384)
        ctx.set_aes_kernel(qpp.AES_KERNEL_AUTO)
        ctx.close()


@pytest.mark.parametrize("seed", [0xF1F5, 0xF1F6])
def test_random_fips_sequence(seed):
    """FIPS mode under churn (aead/fips.rs:13-60): AES keys created with the mode on refuse seals whose nonce does not
    come after the key's previous one (aws-lc's TLS 1.3 rule, state carried across batches), ChaCha keys never do.
    Random seal batches (one stream: the rule is defined in submission order) over random key subsets, packet numbers
    mostly increasing with repeats and steps back, interleaved with key updates (fresh FIPS state), frees, new keys and
    kernel-path flips; statuses, refused-untouched bytes and sealed bytes against orc_seal_batch_fips."""
    rng = np.random.default_rng(seed)
    ctx = qpp.Context(0)
    ctx.set_fips(True)
    keys = []  # [Key, material, OrcFipsState (the oracle's copy of the key's device state), next pn]

    def add(k):
        keys.append([k, (k.suite, *k.material()), orc.fips_states(1)[0], int(rng.integers(0, 2**30))])

    try:
        for _ in range(4):
            s = int(rng.choice([1, 2, 3]))
            add(ctx.key(s, _secret(rng, s)))
        refused = 0
        for step in range(70):
            op = rng.choice(["seal", "update", "free", "new", "knob"], p=[0.6, 0.12, 0.08, 0.1, 0.1])
            if op == "seal" and keys:
                pick = rng.choice(len(keys), int(rng.integers(1, len(keys) + 1)), replace=False)
                chosen = [keys[i] for i in pick]
                n = int(rng.integers(1, 300))
                descs = np.zeros(n, dtype=qpp.PKT_DTYPE)
                pn_len = rng.integers(1, 5, n)
                aad = pn_len + rng.integers(0, 30, n)
                pt = rng.integers(4, 600, n)
                size = aad + pt + 16
                descs["off"] = np.concatenate([[0], np.cumsum(size + 3)[:-1]])
                descs["aad_len"], descs["pt_len"], descs["pn_len"] = aad, pt, pn_len
                which = rng.integers(0, len(chosen), n)
                for i in range(n):
                    c = chosen[int(which[i])]
                    r = rng.random()
                    c[3] = c[3] + 1 if r < 0.8 else c[3] if r < 0.9 else max(0, c[3] - int(rng.integers(1, 5)))
                    descs[i]["pn"] = c[3]
                descs["key_idx"] = np.array([c[0].slot for c in chosen], dtype=np.uint32)[which]
                arena = rng.integers(0, 256, int(descs["off"][-1] + size[-1]) + 64, dtype=np.uint8)
                odescs = descs.copy()
                odescs["key_idx"] = which
                states = orc.fips_states(len(chosen))
                for j, c in enumerate(chosen):
                    states[j] = c[2]
                want = arena.copy()
                flags = qpp.HP_MASK_OUT | qpp.HP_APPLY
                want_masks, want_st = orc.seal_batch_fips(orc.make_keys([c[1] for c in chosen]),
                                                          [bool(c[0].fips) for c in chosen], states, odescs, want,
                                                          flags)
                for j, c in enumerate(chosen):
                    c[2] = states[j]
                d_desc, d_arena, d_mask, d_st = ctx.alloc(descs.nbytes), ctx.alloc(arena.nbytes), ctx.alloc(5 * n), \
                    ctx.alloc(n)
                d_desc.upload(descs)
                d_arena.upload(arena)
                d_st.upload(np.full(n, 0x55, dtype=np.uint8))
                ctx.seal_batch(d_desc, n, d_arena, d_mask, d_st, flags)
                ctx.sync()
                st = d_st.download(dtype=np.int8)
                assert list(st) == want_st, f"step {step}: FIPS statuses"
                assert (d_arena.download() == want).all(), f"step {step}: arena"
                ok = np.array(want_st) == 0
                m = d_mask.download().reshape(-1, 5)[ok]
                assert (m == np.frombuffer(want_masks, dtype=np.uint8).reshape(-1, 5)[ok]).all()
                refused += int((~ok).sum())
                for b in (d_desc, d_arena, d_mask, d_st):
                    b.free()
            elif op == "update" and keys:
                pick = sorted(rng.choice(len(keys), int(rng.integers(1, len(keys) + 1)), replace=False))
                nxt = ctx.update_keys([keys[i][0] for i in pick])
                for i, k in zip(pick, nxt):
                    keys[i][0].free()
                    pn = keys[i][3]
                    keys[i] = [k, (k.suite, *k.material()), orc.fips_states(1)[0], pn]  # a new key: a fresh state
            elif op == "free" and len(keys) > 1:
                keys.pop(int(rng.integers(0, len(keys))))[0].free()
            elif op == "new" and len(keys) < 8:
                s = int(rng.choice([1, 2, 3]))
                add(ctx.key(s, _secret(rng, s)))
            elif op == "knob":
                ctx.set_burst_max(int(rng.choice([0, 64, 16384])))
                ctx.set_aes_kernel(int(rng.choice([qpp.AES_KERNEL_AUTO, qpp.AES_KERNEL_QUAD, qpp.AES_KERNEL_WAVE])))
        assert refused > 20
    finally:
        for k in keys:
            k[0].free()
        ctx.close()
