"""ctypes view of oracle/liboracle.so — the CHECKER (test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
SUITES = {"aes128gcm": 1, "aes256gcm": 2, "chacha20poly1305": 3}
KEY_LEN = {1: 16, 2: 32, 3: 32}
HASH_LEN = {1: 32, 2: 48, 3: 32}

_lib = None


class OrcPkt(ctypes.Structure):
    _fields_ = [("pn", ctypes.c_uint64), ("key_idx", ctypes.c_uint32), ("off", ctypes.c_uint32),
                ("aad_len", ctypes.c_uint16), ("pt_len", ctypes.c_uint16), ("pn_len", ctypes.c_uint8),
                ("flags", ctypes.c_uint8), ("reserved", ctypes.c_uint16)]


class OrcKey(ctypes.Structure):
    _fields_ = [("suite", ctypes.c_int), ("key", ctypes.c_uint8 * 32), ("iv", ctypes.c_uint8 * 12),
                ("hp", ctypes.c_uint8 * 32)]


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(ORACLE_DIR, "liboracle.so")
        if not os.path.exists(path):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR, "liboracle.so"])
        _lib = ctypes.CDLL(path)
    return _lib


def _buf(data, extra=0):
    b = (ctypes.c_uint8 * (len(data) + extra + 1))()
    ctypes.memmove(b, bytes(data), len(data))
    return b


def nonce(iv, pn):
    out = (ctypes.c_uint8 * 12)()
    lib().orc_nonce(_buf(iv), ctypes.c_uint64(pn), out)
    return bytes(out)


def seal(suite, key, nonce_, aad, pt):
    b = _buf(pt, 16)
    lib().orc_seal(suite, _buf(key), _buf(nonce_), _buf(aad), ctypes.c_size_t(len(aad)), b, ctypes.c_size_t(len(pt)))
    return bytes(b[:len(pt)]), bytes(b[len(pt):len(pt) + 16])


def open_(suite, key, nonce_, aad, ct_tag):
    b = _buf(ct_tag)
    rc = lib().orc_open(suite, _buf(key), _buf(nonce_), _buf(aad), ctypes.c_size_t(len(aad)), b,
                        ctypes.c_size_t(len(ct_tag)))
    return rc, bytes(b[:max(len(ct_tag) - 16, 0)])


def hp_mask(suite, hp, sample):
    out = (ctypes.c_uint8 * 5)()
    lib().orc_hp_mask(suite, _buf(hp), _buf(sample), out)
    return bytes(out)


def derive(suite, secret):
    k = (ctypes.c_uint8 * 32)()
    iv = (ctypes.c_uint8 * 12)()
    hp = (ctypes.c_uint8 * 32)()
    lib().orc_derive(suite, _buf(secret), k, iv, hp)
    kl = KEY_LEN[suite]
    return bytes(k[:kl]), bytes(iv), bytes(hp[:kl])


def update_secret(suite, secret):
    out = (ctypes.c_uint8 * 48)()
    lib().orc_update_secret(suite, _buf(secret), out)
    return bytes(out[:HASH_LEN[suite]])


def initial_secrets(dcid):
    c = (ctypes.c_uint8 * 32)()
    s = (ctypes.c_uint8 * 32)()
    lib().orc_initial_secrets(_buf(dcid), ctypes.c_size_t(len(dcid)), c, s)
    return bytes(c), bytes(s)


def expand_label(hash_len, secret, label, n):
    out = (ctypes.c_uint8 * n)()
    lib().orc_hkdf_expand_label(ctypes.c_size_t(hash_len), _buf(secret), label.encode(), out, ctypes.c_size_t(n))
    return bytes(out)


def protect_packet(suite, key, iv, hp, pn, header, pn_len, payload):
    """header excludes the PN bytes; pkt = header || pn(pn_len) || payload || tag."""
    pn_bytes = (pn & ((1 << (8 * pn_len)) - 1)).to_bytes(pn_len, "big")
    pkt = bytes(header) + pn_bytes + bytes(payload)
    b = _buf(pkt, 16)
    rc = lib().orc_protect_packet(suite, _buf(key), _buf(iv), _buf(hp), ctypes.c_uint64(pn), b,
                                  ctypes.c_size_t(len(header)), ctypes.c_size_t(pn_len), ctypes.c_size_t(len(payload)))
    return rc, bytes(b[:len(pkt) + 16])


def unprotect_packet(suite, key, iv, hp, full_pn, pkt, header_len):
    b = _buf(pkt)
    pn_len = ctypes.c_size_t(0)
    rc = lib().orc_unprotect_packet(suite, _buf(key), _buf(iv), _buf(hp), ctypes.c_uint64(full_pn), b,
                                    ctypes.c_size_t(header_len), ctypes.c_size_t(len(pkt)), ctypes.byref(pn_len))
    return rc, pn_len.value, bytes(b[:len(pkt)])


class OrcRx(ctypes.Structure):
    _fields_ = [("largest_pn", ctypes.c_uint64), ("key_idx", ctypes.c_uint32 * 2), ("off", ctypes.c_uint32),
                ("header_len", ctypes.c_uint16), ("len", ctypes.c_uint16)]


def decode_pn(largest, truncated, nbits):
    f = lib().orc_decode_packet_number
    f.restype = ctypes.c_uint64
    return f(ctypes.c_uint64(largest), ctypes.c_uint64(truncated), ctypes.c_uint(nbits))


def truncate_pn(pn, largest):
    t, n = ctypes.c_uint64(), ctypes.c_size_t()
    rc = lib().orc_truncate_packet_number(ctypes.c_uint64(pn), ctypes.c_uint64(largest), ctypes.byref(t), ctypes.byref(n))
    return rc, t.value, n.value


def unprotect_open_batch(keys, rx, arena):
    """keys: OrcKey array; rx: numpy array with qpp_rx_pkt layout; arena modified in place -> (descs, status)."""
    import numpy as np
    n = len(rx)
    out = np.zeros(n, dtype=[("pn", "<u8"), ("key_idx", "<u4"), ("off", "<u4"), ("aad_len", "<u2"),
                             ("pt_len", "<u2"), ("pn_len", "u1"), ("flags", "u1"), ("reserved", "<u2")])
    status = (ctypes.c_int8 * (n + 1))()
    lib().orc_unprotect_open_batch(keys, rx.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(n),
                                   arena.ctypes.data_as(ctypes.c_void_p), out.ctypes.data_as(ctypes.c_void_p), status)
    return out, list(status[:n])


def make_keys(keys):
    """keys: list of (suite, key, iv, hp) -> OrcKey array"""
    arr = (OrcKey * len(keys))()
    for i, (suite, k, iv, hp) in enumerate(keys):
        arr[i].suite = suite
        ctypes.memmove(arr[i].key, bytes(k), len(k))
        ctypes.memmove(arr[i].iv, bytes(iv), 12)
        ctypes.memmove(arr[i].hp, bytes(hp), len(hp))
    return arr


def seal_batch(keys, pkts, arena, flags=0):
    """keys: OrcKey array; pkts: numpy structured array with qpp_pkt layout; arena: numpy uint8 (modified)."""
    n = len(pkts)
    masks = (ctypes.c_uint8 * (5 * n + 1))()
    lib().orc_seal_batch(keys, pkts.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(n),
                         arena.ctypes.data_as(ctypes.c_void_p), masks, flags)
    return bytes(masks[:5 * n])


_fc = None


def fast_seal_batch(keys, pkts, arena, flags=0, threads=16):
    """seal_batch through oracle/libfastcheck.so (OpenSSL EVP on up to 16 threads; same semantics, checked against the
    restatement in tests/test_fastcheck.py): for comparing EVERY packet of a full-size GPU batch."""
    global _fc
    if _fc is None:
        path = os.path.join(ORACLE_DIR, "libfastcheck.so")
        if not os.path.exists(path):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR, "libfastcheck.so"])
        _fc = ctypes.CDLL(path)
    n = len(pkts)
    masks = np.zeros(5 * n + 1, dtype=np.uint8)
    ok = _fc.fc_seal_batch(keys, pkts.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(n),
                           arena.ctypes.data_as(ctypes.c_void_p), masks.ctypes.data_as(ctypes.c_void_p), flags,
                           threads)
    assert ok == 1, "OpenSSL refused a call in fc_seal_batch"
    return masks[:5 * n]


def check_full_seal(keys, slots, descs, arena_in, sealed, masks=None, flags=0):
    """every packet of a GPU-sealed batch against fast_seal_batch: keys = OrcKey array indexed like `slots` (device
    slots); returns the number of packets compared (asserts on the first mismatch, naming it)"""
    lut = np.full(int(max(slots)) + 1, -1, dtype=np.int64)
    lut[np.asarray(slots, dtype=np.int64)] = np.arange(len(slots))
    d = descs.copy()
    d["key_idx"] = lut[descs["key_idx"].astype(np.int64)]
    assert (d["key_idx"] >= 0).all()
    want = arena_in.copy()
    want_masks = fast_seal_batch(keys, d, want, flags)
    if not (sealed == want).all():
        bad = int(np.flatnonzero(sealed != want)[0])
        i = int(np.searchsorted(descs["off"].astype(np.int64), bad, side="right")) - 1
        raise AssertionError(f"sealed bytes differ from the checker, first at arena byte {bad} (packet ~{i})")
    if masks is not None and flags & 1:
        m = np.asarray(masks, dtype=np.uint8)[:5 * len(descs)]
        if not (m == want_masks).all():
            raise AssertionError(f"HP mask differs, first at packet {int(np.flatnonzero(m != want_masks)[0]) // 5}")
    return len(descs)


class OrcFipsState(ctypes.Structure):
    _fields_ = [("mask", ctypes.c_uint64), ("min_next", ctypes.c_uint64), ("seen", ctypes.c_int), ("pad", ctypes.c_int)]


def fips_states(nkeys):
    """per-key FIPS nonce-order state, kept across batches (orc_fips_seal_ok)"""
    return (OrcFipsState * max(nkeys, 1))()


def seal_batch_fips(keys, fips, states, pkts, arena, flags=0):
    """orc_seal_batch in batch order with aws-lc's TLS 1.3 nonce-order check on keys with fips[k]: returns (masks,
    status); refused packets stay untouched with status 3 (INTERNAL_ERROR)."""
    n = len(pkts)
    masks = (ctypes.c_uint8 * (5 * n + 1))()
    status = (ctypes.c_int8 * (n + 1))()
    on = (ctypes.c_uint8 * max(len(fips), 1))(*[1 if f else 0 for f in fips])
    lib().orc_seal_batch_fips(keys, on, states, pkts.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(n),
                              arena.ctypes.data_as(ctypes.c_void_p), masks, flags, status)
    return bytes(masks[:5 * n]), list(status[:n])


def open_batch(keys, pkts, arena):
    n = len(pkts)
    status = (ctypes.c_int8 * (n + 1))()
    lib().orc_open_batch(keys, pkts.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(n),
                         arena.ctypes.data_as(ctypes.c_void_p), status)
    return list(status[:n])
