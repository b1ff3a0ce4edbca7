"""Transmit-queue ordering rules with several flushes in flight, on the GPU.

* FIPS nonce order across streams: the gate state lives in the device key record, so the gates of two flushes that
  are in flight on different streams must run in submission order (api.cpp fips_gate: one context-wide event).  A pn
  repeated across two such flushes is refused in the second, exactly as the sequential rule (aws-lc's TLS 1.3 sealer,
  quic/s2n-quic-crypto/src/aead/fips.rs:13-60) refuses it -- parity against orc_fips_seal_ok.
* DMA path ownership: a flush copies only its own packets' bytes to HBM and back (runs of adjacent packets), never the
  ring between them -- those bytes belong to the transport or to another flush in flight.
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


def _packet(rng, pn, largest, payload_len):
    trunc, pn_len = qpp.pn_truncate(pn, largest)
    header = bytes([0x40 | (pn_len - 1)]) + rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
    payload = rng.integers(0, 256, payload_len, dtype=np.uint8).tobytes()
    return header, pn_len, header + trunc.to_bytes(pn_len, "big") + payload, payload


@pytest.mark.parametrize("flush", ["zero_copy", "dma"])
def test_fips_gates_of_flushes_in_flight_run_in_submission_order(ctx, flush, monkeypatch):
    """flush A (pns 100..103) and flush B (pns 103, 104: 103 repeated) in flight at once on two streams: B's 103 is
    refused (B's wait reports INTERNAL_ERROR, its bytes stay as pushed), everything else equals the oracle"""
    monkeypatch.setenv("QPP_TXQ_ZC_MAX", "1024" if flush == "zero_copy" else "0")
    rng = np.random.default_rng(51)
    ctx.set_fips(True)
    k = ctx.key(1, rng.integers(0, 256, 32, dtype=np.uint8).tobytes())
    ctx.set_fips(False)
    assert k.fips
    kk, iv, hp = k.material()
    q = qpp.TxQueue(ctx, 1 << 18, 64, in_flight=2)
    state = orc.fips_states(1)
    off, tickets, layout = 0, [], []
    for burst in ([100, 101, 102, 103], [103, 104]):
        for pn in burst:
            header, pn_len, pkt, payload = _packet(rng, pn, 99, 900)
            q.ring[off:off + len(pkt)] = np.frombuffer(pkt, dtype=np.uint8)
            q.push(k, pn, off, len(header), pn_len, len(payload))
            ok = bool(orc.lib().orc_fips_seal_ok(state, orc._buf(orc.nonce(iv, pn))))
            layout.append((off, pkt, ok, orc.protect_packet(1, kk, iv, hp, pn, header, pn_len, payload)[1]))
            off += len(pkt) + 16 + 40
        tickets.append(q.flush_async())  # A is still in flight when B goes out
    assert [x[2] for x in layout] == [True, True, True, True, False, True]
    q.wait(tickets[0])
    with pytest.raises(qpp.QppError) as e:
        q.wait(tickets[1])
    assert e.value.code == qpp.INTERNAL_ERROR
    for o, pkt, ok, protected in layout:
        got = q.ring[o:o + len(protected)].tobytes()
        assert got == protected if ok else got[:len(pkt)] == pkt
    q.close()
    k.free()


def test_txq_dma_flush_copies_only_its_packets(ctx, monkeypatch):
    """two DMA-path flushes in flight with interleaved packets (A at even slots, B at odd slots of the ring) and the
    transport writing the gaps between packets while both are in flight: every packet equals the oracle, and every
    gap byte holds what the transport last wrote (a copy of a flush's whole [lo, hi) span would put stale bytes back)"""
    monkeypatch.setenv("QPP_TXQ_ZC_MAX", "0")
    rng = np.random.default_rng(52)
    keys = [ctx.key(s, rng.integers(0, 256, qpp.HASH_LEN[s], dtype=np.uint8).tobytes()) for s in (1, 3)]
    stride, per = 1536, 48
    q = qpp.TxQueue(ctx, stride * 2 * per + 4096, per, in_flight=2)
    q.ring[:] = 0xa5
    largest = int(rng.integers(0, 2**40))
    want, gaps, tickets, pn = [], [], [], largest + 1
    for side in (0, 1):  # flush A: slots 0, 2, 4, ...; flush B: slots 1, 3, 5, ...
        for i in range(per):
            k = keys[i % 2]
            off = (2 * i + side) * stride
            header, pn_len, pkt, payload = _packet(rng, pn, largest, int(rng.integers(200, 1300)))
            q.ring[off:off + len(pkt)] = np.frombuffer(pkt, dtype=np.uint8)
            q.push(k, pn, off, len(header), pn_len, len(payload))
            suite, (kk, iv, hp) = k.suite, k.material()
            protected = orc.protect_packet(suite, kk, iv, hp, pn, header, pn_len, payload)[1]
            want.append((off, protected))
            gaps.append((off + len(protected), off + stride))
            pn += 1
        tickets.append(q.flush_async())
        # the transport writes the gaps (bytes no flush owns) while the flushes are in flight
        for lo, hi in gaps:
            q.ring[lo:hi] = 0x3c + side
    for t in tickets:
        q.wait(t)
    for o, p in want:
        assert q.ring[o:o + len(p)].tobytes() == p
    for lo, hi in gaps:
        assert (q.ring[lo:hi] == 0x3d).all(), f"gap [{lo}, {hi}) overwritten"
    q.close()
    for k in keys:
        k.free()


def test_fips_seal_batch_needs_status(ctx):
    """with a FIPS key live, a seal batch without a status array is refused (it could not report refused packets)"""
    rng = np.random.default_rng(53)
    ctx.set_fips(True)
    k = ctx.key(1, rng.integers(0, 256, 32, dtype=np.uint8).tobytes())
    ctx.set_fips(False)
    descs, arena = qpp.make_batch(4, 100, [k.slot], seed=53)
    d_desc, d_arena, d_status = ctx.alloc(descs.nbytes), ctx.alloc(arena.nbytes), ctx.alloc(4)
    d_desc.upload(descs)
    d_arena.upload(arena)
    with pytest.raises(qpp.QppError) as e:
        ctx.seal_batch(d_desc, 4, d_arena, None, None, 0)
    assert e.value.code == qpp.INTERNAL_ERROR
    ctx.seal_batch(d_desc, 4, d_arena, None, d_status, 0)  # with one it goes through
    ctx.sync()
    assert (d_status.download(dtype=np.int8) == 0).all()
    for b in (d_desc, d_arena, d_status):
        b.free()
    k.free()


def _apply_header_protection(buf, off, header_len, pn_len, mask):
    """crypto::protect -> apply_header_protection (quic/s2n-quic-core/src/crypto/header_crypto.rs:80-95) in place"""
    b0 = int(buf[off])
    buf[off] = b0 ^ (mask[0] & (0x0f if b0 & 0x80 else 0x1f))
    for i in range(pn_len):
        buf[off + header_len + i] ^= mask[1 + i]


@pytest.mark.parametrize("flush", ["zero_copy", "dma"])
def test_deferred_encode_packet_sequence(ctx, flush, monkeypatch):
    """PacketEncoder::encode_packet in deferred mode, call for call (packet/encoding.rs:240-279):
    header || truncated PN || inline payload written into the ring; Key::encrypt -> qpp_txq_push_scatter with the
    scatter::Buffer's `extra` tail on a third of the packets (scatter.rs:6-68); then crypto::protect, which
    encoding.rs:278 calls unconditionally, with the deferred HeaderKey whose mask is [0; 5] (the bytes do not change);
    then the flush.  Every packet equals crypto::encrypt + crypto::protect of the oracle over inline || extra."""
    monkeypatch.setenv("QPP_TXQ_ZC_MAX", "1024" if flush == "zero_copy" else "0")
    rng = np.random.default_rng(54)
    keys = [ctx.key(s, rng.integers(0, 256, qpp.HASH_LEN[s], dtype=np.uint8).tobytes()) for s in (1, 2, 3)]
    q = qpp.TxQueue(ctx, 1 << 20, 256)
    largest = int(rng.integers(0, 2**40))
    want, off = [], 0
    for i in range(200):
        k = keys[i % 3]
        pn = largest + 1 + i
        header, pn_len, pkt, inline = _packet(rng, pn, largest, int(rng.integers(4, 900)))
        extra = rng.integers(0, 256, int(rng.integers(1, 400)), dtype=np.uint8).tobytes() if i % 3 == 0 else b""
        q.ring[off:off + len(pkt)] = np.frombuffer(pkt, dtype=np.uint8)
        q.push_scatter(k, pn, off, len(header), pn_len, len(inline), extra)  # Key::encrypt (deferred)
        before = q.ring[off:off + len(header) + pn_len].copy()
        _apply_header_protection(q.ring, off, len(header), pn_len, bytes(5))  # crypto::protect, deferred HeaderKey
        assert (q.ring[off:off + len(header) + pn_len] == before).all()
        suite, (kk, iv, hp) = k.suite, k.material()
        rc, protected = orc.protect_packet(suite, kk, iv, hp, pn, header, pn_len, inline + extra)
        want.append((off, protected))
        off += len(protected) + int(rng.integers(0, 9))
    q.flush()
    for o, p in want:
        assert q.ring[o:o + len(p)].tobytes() == p
    # an extra tail that would not fit the ring is refused before anything is copied
    tail = q.ring[(1 << 20) - 64:].copy()
    with pytest.raises(qpp.QppError):
        q.push_scatter(keys[0], 1, (1 << 20) - 64, 17, 1, 8, bytes(100))
    assert (q.ring[(1 << 20) - 64:] == tail).all()
    q.close()
    for k in keys:
        k.free()
