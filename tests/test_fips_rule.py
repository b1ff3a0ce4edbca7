"""CPU checks of FIPS mode's sealing nonce-order rule (no GPU).

The oracle restates aws-lc's TLS 1.3 AEAD check on the nonce bytes (oracle/qpp_oracle.c orc_fips_seal_ok; aws-lc-rs 1.12
TlsRecordSealingKey behind quic/s2n-quic-crypto/src/aead/fips.rs:13-60 — aws-lc is not vendored, so the rule is
"parity unpinned").  The GPU gate (csrc/fips.hip) computes the same decisions in parallel from a per-key prefix maximum
of given = pn ^ pn_first over batch order; these tests check that reformulation against the sequential oracle.
"""
import ctypes

import numpy as np

import _oracle as orc


def _sequential(iv, pns, state):
    return [orc.lib().orc_fips_seal_ok(state, orc._buf(orc.nonce(iv, p))) for p in pns]


def _prefix_max_form(pns, seen, mask, min_next):
    """the gate's formulation: refused iff given < min_next, given == 2^64-1 or given <= max of earlier givens"""
    if not seen and pns:
        mask = pns[0]
    out, best = [], None  # best = max(given + 1) over earlier packets (all of them, refused or not)
    for p in pns:
        g = p ^ mask
        v = 0 if g == 2**64 - 1 else g + 1
        ok = v != 0 and g >= min_next and (best is None or v > best)
        out.append(int(ok))
        best = v if best is None else max(best, v)
    top = max(min_next, best or 0)  # the gate's update: refused packets are never above it (fips.hip fips_tails)
    return out, mask, top


def test_first_seal_fixes_the_mask_and_xor_order():
    iv = bytes(range(12))
    st = orc.OrcFipsState()
    # 5 is the first (mask 5): 6 -> 3 ok, 7 -> 2 < 4 refused, 8 -> 13 ok, 8 again refused, 100 -> 97, 99 -> 102 ok
    # (aws-lc compares pn ^ pn_first, not pn), 101 -> 96 refused
    assert _sequential(iv, [5, 6, 7, 8, 8, 100, 99, 101], ctypes.byref(st)) == [1, 1, 0, 1, 0, 1, 1, 0]
    # the mask is the first nonce's low 8 bytes: iv[4:12] ^ pn_first, so the iv cancels from every given
    assert st.mask == int.from_bytes(iv[4:], "big") ^ 5 and st.min_next == 103


def test_prefix_max_reformulation_matches_the_sequential_rule():
    rng = np.random.default_rng(7)
    iv = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    for trial in range(200):
        n = int(rng.integers(1, 60))
        start = int(rng.integers(0, 2**62))
        pns = [int(x) for x in np.clip(start + np.cumsum(rng.integers(-3, 6, n)), 0, 2**62 - 1)]
        st = orc.OrcFipsState()
        iv_lo = int.from_bytes(iv[4:], "big")
        seen, mask, min_next = 0, 0, 0
        if trial % 3 == 0:  # a key that has sealed before: mask in pn terms, the oracle's in nonce terms
            seen, mask, min_next = 1, int(rng.integers(0, 2**62)), int(rng.integers(0, 2**62))
            st.seen, st.mask, st.min_next = 1, mask ^ iv_lo, min_next
        want = _sequential(iv, pns, ctypes.byref(st))
        got, mask2, top = _prefix_max_form(pns, seen, mask, min_next)
        assert got == want, (trial, pns)
        assert st.mask == mask2 ^ iv_lo and st.min_next == top
