"""Packet-number codec the receive path depends on, CPU only.

The oracle (oracle/qpp_oracle.c) is pinned by the reference's own vectors, then the engine's host helpers in
libqpp.so (qpp_pn_truncate / qpp_pn_expand, the same decode the unprotect kernel runs) are checked against it.
Mirrors quic/s2n-quic-core/src/packet/number/{mod.rs:111-162, tests.rs:108-200}.
"""
import random

import pytest

import _oracle as orc
import qpp

VARINT_MAX = (1 << 62) - 1


def rfc_decoder(largest_pn, truncated_pn, pn_nbits):
    """RFC 9000 A.3 pseudo-code, transliterated (tests.rs:108-159); None for a checked op that overflows."""
    expected_pn = largest_pn + 1
    pn_win = 1 << pn_nbits
    pn_hwin = pn_win // 2
    pn_mask = pn_win - 1
    candidate_pn = (expected_pn & ~pn_mask) | truncated_pn
    if expected_pn - pn_hwin >= 0 and candidate_pn <= expected_pn - pn_hwin and candidate_pn < (1 << 62) - pn_win:
        return candidate_pn + pn_win
    if expected_pn + pn_hwin < 1 << 64 and candidate_pn > expected_pn + pn_hwin and candidate_pn >= pn_win:
        return candidate_pn - pn_win
    return candidate_pn


def test_reference_vectors():
    # packet_decoding_example_test (mod.rs:151-162)
    assert orc.decode_pn(0xa82f30ea, 0x9b32, 16) == 0xa82f9b32
    assert orc.truncate_pn(0xa82f9b32, 0xa82f30ea) == (0, 0x9b32, 2)
    # packet_number_len_example_test (mod.rs:111-133): 16-bit and 24-bit encodings
    assert orc.truncate_pn(0xac5c02, 0xabe8bc)[2] == 2
    assert orc.truncate_pn(0xace8fe, 0xabe8bc)[2] == 3
    # truncation is impossible below the largest acknowledged PN or beyond 4 bytes
    assert orc.truncate_pn(5, 6)[0] == 1  # ORC_DECODE_ERROR
    assert orc.truncate_pn(1 << 40, 0)[0] == 1


def test_oracle_vs_rfc_pseudocode():
    # rfc_differential_test (tests.rs:176-200)
    rng = random.Random(7)
    for _ in range(20000):
        nbits = 8 * rng.randint(1, 4)
        largest = rng.choice([0, 1, rng.randrange(1 << 62), (1 << 62) - 1, rng.randrange(1 << 20)])
        trunc = rng.randrange(1 << nbits)
        assert orc.decode_pn(largest, trunc, nbits) == min(rfc_decoder(largest, trunc, nbits), VARINT_MAX)


def test_truncate_expand_round_trip():
    # truncate_expand_test (tests.rs:163-174)
    rng = random.Random(11)
    for _ in range(20000):
        largest = rng.randrange(1 << 62)
        pn = min(largest + rng.choice([0, 1, 2, rng.randrange(1 << 8), rng.randrange(1 << 16), rng.randrange(1 << 31)]),
                 VARINT_MAX)
        rc, t, n = orc.truncate_pn(pn, largest)
        if rc == 0:
            assert orc.decode_pn(largest, t, 8 * n) == pn


def test_engine_host_helpers_match_oracle():
    rng = random.Random(13)
    for _ in range(5000):
        largest = rng.randrange(1 << 62)
        pn = min(largest + rng.randrange(1 << rng.choice([4, 12, 20, 31, 33])), VARINT_MAX)
        rc, t, n = orc.truncate_pn(pn, largest)
        if rc:
            with pytest.raises(qpp.QppError):
                qpp.pn_truncate(pn, largest)
            continue
        assert qpp.pn_truncate(pn, largest) == (t, n)
        assert qpp.pn_expand(largest, t, n) == pn
        nbits = 8 * rng.randint(1, 4)
        tr = rng.randrange(1 << nbits)
        assert qpp.pn_expand(largest, tr, nbits // 8) == orc.decode_pn(largest, tr, nbits)
