"""The full-size batch checker (oracle/fastcheck.c, OpenSSL EVP on 16 threads) against the pinned restatement
(oracle/qpp_oracle.c): same ciphertext, tags, HP masks and applied masks on ragged mixed-suite batches, so the GPU
tests may compare every packet of a 1 Mi-packet batch with it."""
import numpy as np
import pytest

import _oracle as orc


def _ragged(rng, n, nkeys):
    pkts = np.zeros(n, dtype=[("pn", "<u8"), ("key_idx", "<u4"), ("off", "<u4"), ("aad_len", "<u2"),
                              ("pt_len", "<u2"), ("pn_len", "u1"), ("flags", "u1"), ("reserved", "<u2")])
    pt = rng.integers(0, 1500, n)
    pt[:40] = np.arange(40)  # every short length (the HP sample reaches into the tag below 20 - pn_len)
    pn_len = rng.integers(1, 5, n)
    aad = pn_len + rng.integers(1, 40, n)
    size = aad + pt + 16 + 3
    pkts["off"] = np.concatenate([[0], np.cumsum(size)[:-1]])
    pkts["pn"] = rng.integers(0, 2**62, n, dtype=np.uint64)
    pkts["key_idx"] = rng.integers(0, nkeys, n)
    pkts["aad_len"], pkts["pt_len"], pkts["pn_len"] = aad, pt, pn_len
    arena = rng.integers(0, 256, int(size.sum()) + 64, dtype=np.uint8)
    return pkts, arena


@pytest.mark.parametrize("flags", [0, 1, 3])
def test_fastcheck_equals_restatement(flags):
    rng = np.random.default_rng(900 + flags)
    keys = orc.make_keys([(s, rng.integers(0, 256, 32, dtype=np.uint8).tobytes()[:16 if s == 1 else 32],
                           rng.integers(0, 256, 12, dtype=np.uint8).tobytes(),
                           rng.integers(0, 256, 32, dtype=np.uint8).tobytes()[:16 if s == 1 else 32])
                          for s in [1, 2, 3, 1, 3, 2, 2, 1]])
    pkts, arena = _ragged(rng, 3000, 8)
    want = arena.copy()
    want_masks = orc.seal_batch(keys, pkts, want, flags)
    got = arena.copy()
    got_masks = orc.fast_seal_batch(keys, pkts, got, flags)
    assert (got == want).all()
    if flags & 1:
        assert got_masks.tobytes() == want_masks
