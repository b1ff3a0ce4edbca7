"""Pins the oracle (oracle/qpp_oracle.c) before anything is checked against it.

Sources of truth, in order:
  1. RFC 9001 Appendix A vectors as held by the reference
     (quic/s2n-quic-core/src/crypto/{initial.rs,retry.rs}, quic/s2n-quic-crypto/src/one_rtt.rs,
     specs/www.rfc-editor.org/rfc/rfc9001.txt) -> tests/golden/rfc9001.json
  2. OpenSSL-generated fixtures (stand-in for aws-lc-rs, which is not vendored)
     -> tests/golden/{aead_*,hp_masks,kdf_chains}.json
Mirrors the reference tests:
  rfc_example_{client,server}_test   quic/s2n-quic-crypto/src/initial.rs:142-241
  {client,server}_initial_protection_test quic/s2n-quic-core/src/crypto/initial.rs:132-140,265-274
  test_tag_validation                 quic/s2n-quic-crypto/src/retry.rs:55-64
  test_key_update                     quic/s2n-quic-crypto/src/one_rtt.rs:79-114
  label tests                         quic/s2n-quic-core/src/crypto/label.rs:70-105
"""
import pytest

import _oracle as orc
from conftest import load_golden

H = bytes.fromhex


def test_initial_secrets(rfc):
    c, s = orc.initial_secrets(H(rfc["dcid"]))
    assert c.hex() == rfc["client_initial_secret"]
    assert s.hex() == rfc["server_initial_secret"]
    for side, secret in (("client", c), ("server", s)):
        key, iv, hp = orc.derive(1, secret)
        assert (key.hex(), iv.hex(), hp.hex()) == (rfc[side]["key"], rfc[side]["iv"], rfc[side]["hp"])


@pytest.mark.parametrize("label,length,expected", [
    ("client in", 32, "00200f746c73313320636c69656e7420696e00"),
    ("server in", 32, "00200f746c7331332073657276657220696e00"),
    ("quic key", 16, "00100e746c7331332071756963206b657900"),
    ("quic iv", 12, "000c0d746c733133207175696320697600"),
    ("quic hp", 16, "00100d746c733133207175696320687000"),
    ("quic ku", 16, "00100d746c7331332071756963206b7500"),
    ("quic key", 32, "00200e746c7331332071756963206b657900"),
    ("quic hp", 32, "00200d746c733133207175696320687000"),
    ("quic ku", 32, "00200d746c7331332071756963206b7500"),
    ("quic ku", 48, "00300d746c7331332071756963206b7500"),
])
def test_label_encoding(label, length, expected):
    # label.rs:57-68 HkdfLabel; checked through HKDF-Expand with the explicit info bytes
    import ctypes
    secret = bytes(range(32))
    info = H(expected)
    out = (ctypes.c_uint8 * length)()
    orc.lib().orc_hkdf_expand(ctypes.c_size_t(32), orc._buf(secret), orc._buf(info), ctypes.c_size_t(len(info)),
                              out, ctypes.c_size_t(length))
    assert bytes(out) == orc.expand_label(32, secret, label, length)


def _a2_plain(rfc):
    a2 = rfc["a2"]
    payload = H(a2["payload_prefix"]) + bytes(a2["padded_payload_len"] - len(H(a2["payload_prefix"])))
    return a2, payload


def test_a2_client_initial_protect_bitexact(rfc):
    a2, payload = _a2_plain(rfc)
    key, iv, hp = orc.derive(1, H(rfc["client_initial_secret"]))
    header = H(a2["header"])[:-a2["pn_len"]]
    rc, pkt = orc.protect_packet(1, key, iv, hp, a2["pn"], header, a2["pn_len"], payload)
    assert rc == 0
    assert pkt.hex() == a2["protected_packet"]
    assert pkt[len(header) + 4:len(header) + 20].hex() == a2["sample"]
    assert orc.hp_mask(1, hp, H(a2["sample"])).hex() == a2["mask"]


@pytest.mark.parametrize("which,secret", [("a2", "client_initial_secret"), ("a3", "server_initial_secret")])
def test_rfc_initial_unprotect(rfc, which, secret):
    v = rfc[which]
    key, iv, hp = orc.derive(1, H(rfc[secret]))
    pkt = H(v["protected_packet"])
    header_len = len(H(v["header"])) - v["pn_len"]
    rc, pn_len, out = orc.unprotect_packet(1, key, iv, hp, v["pn"], pkt, header_len)
    assert rc == 0 and pn_len == v["pn_len"]
    assert out[:header_len + pn_len].hex() == v["header"]
    body = out[header_len + pn_len:len(pkt) - 16]
    expect = H(v["payload_prefix"] if which == "a2" else v["payload"])
    assert body[:len(expect)] == expect
    assert body[len(expect):] == bytes(len(body) - len(expect))


def test_a3_server_initial_protect_bitexact(rfc):
    a3 = rfc["a3"]
    key, iv, hp = orc.derive(1, H(rfc["server_initial_secret"]))
    header = H(a3["header"])[:-a3["pn_len"]]
    rc, pkt = orc.protect_packet(1, key, iv, hp, a3["pn"], header, a3["pn_len"], H(a3["payload"]))
    assert rc == 0 and pkt.hex() == a3["protected_packet"]


def test_a4_retry_tag(rfc):
    a4 = rfc["a4"]
    ct, tag = orc.seal(1, H(a4["key"]), H(a4["nonce"]), H(a4["pseudo_packet"]), b"")
    assert ct == b"" and tag.hex() == a4["tag"]
    # validate() rejects a wrong tag (retry.rs:55-64)
    rc, _ = orc.open_(1, H(a4["key"]), H(a4["nonce"]), H(a4["pseudo_packet"]), H("00112233445566778899aabbccddeeff"))
    assert rc == 2
    rc, _ = orc.open_(1, H(a4["key"]), H(a4["nonce"]), H(a4["pseudo_packet"]), H(a4["tag"]))
    assert rc == 0


def test_a5_chacha_short_header(rfc):
    a5 = rfc["a5"]
    key, iv, hp = orc.derive(3, H(a5["secret"]))
    assert (key.hex(), iv.hex(), hp.hex()) == (a5["key"], a5["iv"], a5["hp"])
    assert orc.nonce(iv, a5["pn"]).hex() == a5["nonce"]
    header = H(a5["header"])[:-a5["pn_len"]]
    rc, pkt = orc.protect_packet(3, key, iv, hp, a5["pn"], header, a5["pn_len"], H(a5["plaintext"]))
    assert rc == 0 and pkt.hex() == a5["packet"]
    assert orc.hp_mask(3, hp, H(a5["sample"])).hex() == a5["mask"]
    rc, pn_len, out = orc.unprotect_packet(3, key, iv, hp, a5["pn"], pkt, len(header))
    assert rc == 0 and pn_len == 3 and out[4:5] == H(a5["plaintext"])


def test_a5_key_update(rfc):
    a5 = rfc["a5"]
    # absolute: "quic ku" output equals the RFC's ku value
    assert orc.update_secret(3, H(a5["secret"])).hex() == a5["ku_secret"]
    # relative, as test_key_update does: update(secret) seals like new(ku_secret)
    k1, iv1, _ = orc.derive(3, orc.update_secret(3, H(a5["secret"])))
    k2, iv2, _ = orc.derive(3, H(a5["ku_secret"]))
    assert orc.seal(3, k1, orc.nonce(iv1, 0), b"", bytes(32)) == orc.seal(3, k2, orc.nonce(iv2, 0), b"", bytes(32))
    k3, iv3, _ = orc.derive(3, orc.update_secret(3, bytes(32)))
    assert orc.seal(3, k3, orc.nonce(iv3, 0), b"", bytes(32)) != orc.seal(3, k2, orc.nonce(iv2, 0), b"", bytes(32))


@pytest.mark.parametrize("name,suite", [("aead_aes128gcm.json", 1), ("aead_aes256gcm.json", 2),
                                        ("aead_chacha20poly1305.json", 3), ("gcm_spec_aes256.json", 2)])
def test_aead_fixtures(name, suite):
    fx = load_golden(name)
    assert fx["suite"] == suite
    for c in fx["cases"]:
        key, iv, aad, pt = H(c["key"]), H(c["iv"]), H(c["aad"]), H(c["pt"])
        n = orc.nonce(iv, c["pn"])
        assert n.hex() == c["nonce"]
        ct, tag = orc.seal(suite, key, n, aad, pt)
        assert ct.hex() == c["ct"] and tag.hex() == c["tag"], len(pt)
        rc, out = orc.open_(suite, key, n, aad, ct + tag)
        assert rc == 0 and out == pt
        bad = bytearray(ct + tag)
        bad[-1 - (len(pt) % 16)] ^= 0x01
        rc, out = orc.open_(suite, key, n, aad, bytes(bad))
        assert rc == 2 and out == bytes(len(pt))  # unauthenticated plaintext never released


def test_open_short_input():
    # cipher_suite.rs:126-129 — fewer than 16 bytes is DECRYPT_ERROR
    for suite in (1, 2, 3):
        rc, _ = orc.open_(suite, bytes(32), bytes(12), b"", bytes(15))
        assert rc == 2


def test_hp_fixtures():
    for c in load_golden("hp_masks.json")["cases"]:
        assert orc.hp_mask(c["suite"], H(c["hp"]), H(c["sample"])).hex() == c["mask"]


def test_kdf_chains():
    for ch in load_golden("kdf_chains.json")["chains"]:
        suite = ch["suite"]
        secret = H(ch["secret"])
        for step in ch["steps"]:
            assert secret.hex() == step["secret"]
            key, iv, hp = orc.derive(suite, secret)
            assert (key.hex(), iv.hex(), hp.hex()) == (step["key"], step["iv"], step["hp"])
            secret = orc.update_secret(suite, secret)
