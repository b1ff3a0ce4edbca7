"""Python view of libqpp.so (the C ABI in include/qpp.h), for the tests, bench.py and smoke().

The names mirror the reference's trait surface (quic/s2n-quic-core/src/crypto/key.rs:8-35,
header_crypto.rs:11-31, one_rtt.rs:11-14) the way a Rust shim over the same ABI would:
    Key.encrypt(pn, header, payload) -> sealed payload || tag          (Key::encrypt)
    Key.decrypt(pn, header, payload) -> plaintext, raises DecryptError  (Key::decrypt)
    Key.header_protection_mask(sample) -> 5 bytes                       (HeaderKey::*_mask)
    Key.derive_next_key()                                               (OneRttKey::derive_next_key)
plus the batch entry points over device buffers.

There is NO fallback: if libqpp.so or a gfx950 GPU is missing, Context() raises.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("QPP_LIB") or os.path.join(HERE, "libqpp.so")  # QPP_LIB: A/B builds

SUITE_AES_128_GCM = 1
SUITE_AES_256_GCM = 2
SUITE_CHACHA20_POLY1305 = 3
SUITE_NAMES = {1: "TLS_AES_128_GCM_SHA256", 2: "TLS_AES_256_GCM_SHA384", 3: "TLS_CHACHA20_POLY1305_SHA256"}
KEY_LEN = {1: 16, 2: 32, 3: 32}
HASH_LEN = {1: 32, 2: 48, 3: 32}

OK, DECODE_ERROR, DECRYPT_ERROR, INTERNAL_ERROR, UNSUPPORTED, DEVICE_ERROR = 0, 1, 2, 3, 4, 5
ROTATION_NOT_SUPPORTED = 6  # dc open::Error::RotationNotSupported
HP_MASK_OUT, HP_APPLY, ONLY_AES, ONLY_CHACHA = 0x1, 0x2, 0x10, 0x20
KEY_BY_CONN = 0x40  # host batches: key_idx = connection index (qpp_ctx_set_conn_keys)
AES_KERNEL_AUTO, AES_KERNEL_QUAD, AES_KERNEL_WAVE = 0, 1, 2
AES_KERNEL_LANE = AES_KERNEL_QUAD  # round-1..3 name of the quad selector (qpp.h)
ENDPOINT_CLIENT, ENDPOINT_SERVER = 0, 1

# qpp_pkt (24 bytes) as a numpy structured dtype
PKT_DTYPE = np.dtype([("pn", "<u8"), ("key_idx", "<u4"), ("off", "<u4"), ("aad_len", "<u2"), ("pt_len", "<u2"),
                      ("pn_len", "u1"), ("flags", "u1"), ("reserved", "<u2")])
assert PKT_DTYPE.itemsize == 24
PKT_SKIP = 0x1
BURST_MAX_DEFAULT = 16384  # kBurstMaxDefault (qpp_internal.h): larger AES batches run one lane per packet
WAVE_KERNEL_PACKETS_PER_KEY = 128  # kWaveKernelPacketsPerKey: fewer packets per live AES key take the wave-item kernel
# qpp_rx_pkt (24 bytes): one received, still protected packet
RX_DTYPE = np.dtype([("largest_pn", "<u8"), ("key_idx", "<u4", (2,)), ("off", "<u4"), ("header_len", "<u2"),
                     ("len", "<u2")])
assert RX_DTYPE.itemsize == 24

# every symbol include/qpp.h declares (tests/test_abi.py checks the library exports them all)
EXPORTS = [
    "qpp_abi_version", "qpp_ctx_create", "qpp_ctx_destroy", "qpp_ctx_stream", "qpp_ctx_synchronize",
    "qpp_ctx_last_error", "qpp_ctx_rx_timeouts", "qpp_key_new", "qpp_key_new_raw", "qpp_key_update", "qpp_key_free", "qpp_key_free_batch", "qpp_ctx_set_aes_kernel", "qpp_key_slot", "qpp_key_slot_batch",
    "qpp_key_suite", "qpp_tag_len", "qpp_sample_len", "qpp_confidentiality_limit", "qpp_integrity_limit",
    "qpp_key_material", "qpp_initial_keys", "qpp_seal", "qpp_seal_scatter", "qpp_open", "qpp_hp_mask",
    "qpp_seal_batch", "qpp_open_batch", "qpp_hp_mask_batch", "qpp_dev_alloc", "qpp_dev_free", "qpp_host_alloc",
    "qpp_host_free", "qpp_memcpy_h2d", "qpp_memcpy_d2h", "qpp_memset_d", "qpp_stream_create",
    "qpp_stream_destroy", "qpp_stream_synchronize", "qpp_event_create", "qpp_event_destroy", "qpp_event_record",
    "qpp_event_elapsed_ms", "qpp_stream_wait_event", "qpp_unprotect_open_batch", "qpp_pn_truncate", "qpp_pn_expand",
    "qpp_key_new_batch", "qpp_txq_create", "qpp_txq_destroy", "qpp_txq_ring", "qpp_txq_push", "qpp_txq_flush",
    "qpp_txq_create_async", "qpp_txq_flush_async", "qpp_txq_poll", "qpp_txq_wait", "qpp_txq_push_descs", "qpp_txq_set_coalesce", "qpp_txq_push_scatter",
    "qpp_txq_create_persistent", "qpp_txq_info", "qpp_txq_server_time", "qpp_txq_server_refused", "qpp_ctx_set_conn_keys",
    "qpp_txq_server_stamps",
    "qpp_txq_pending", "qpp_memcpy_d2d", "qpp_ctx_set_burst_max", "qpp_dc_key_new", "qpp_dc_seal", "qpp_dc_open",
    "qpp_dc_open_in_place", "qpp_ctx_key_slots", "qpp_key_new_pair", "qpp_key_update_batch", "qpp_initial_keys_pair",
    "qpp_header_key_new", "qpp_header_key_new_raw", "qpp_header_key_free", "qpp_header_key_slot",
    "qpp_header_key_suite", "qpp_header_key_sample_len", "qpp_header_key_mask", "qpp_host_batch_submit",
    "qpp_host_batch_query", "qpp_host_batch_wait", "qpp_ctx_set_host_pipe", "qpp_ctx_set_fips", "qpp_key_fips",
    "qpp_ctx_set_packet_server", "qpp_ctx_packet_server_info", "qpp_dev_server_evictions",
]
OP_SEAL, OP_OPEN = 0x1, 0x2


class QppError(RuntimeError):
    def __init__(self, code, what=""):
        self.code = code
        names = {1: "DECODE_ERROR", 2: "DECRYPT_ERROR", 3: "INTERNAL_ERROR", 4: "UNSUPPORTED", 5: "DEVICE_ERROR",
                 6: "ROTATION_NOT_SUPPORTED"}
        super().__init__(f"{names.get(code, code)} {what}".strip())


class DecryptError(QppError):
    """packet_protection::Error::DECRYPT_ERROR"""


_lib = None
vp, u8p, sz, u32, u64 = ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint8), ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint64


_LATER = {"qpp_txq_server_refused", "qpp_dev_server_evictions"}  # entry points added in rounds 5, 6


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise QppError(DEVICE_ERROR, f"{LIB_PATH} is not built (run __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        sig = {
            "qpp_abi_version": (ctypes.c_int, []),
            "qpp_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(vp)]),
            "qpp_ctx_destroy": (None, [vp]),
            "qpp_ctx_stream": (vp, [vp]),
            "qpp_ctx_synchronize": (ctypes.c_int, [vp]),
            "qpp_ctx_last_error": (ctypes.c_char_p, [vp]),
            "qpp_ctx_rx_timeouts": (ctypes.c_int, [vp, ctypes.POINTER(u64)]),
            "qpp_key_new": (ctypes.c_int, [vp, ctypes.c_int, vp, sz, ctypes.POINTER(vp)]),
            "qpp_key_new_raw": (ctypes.c_int, [vp, ctypes.c_int, vp, sz, vp, vp, sz, ctypes.POINTER(vp)]),
            "qpp_key_update": (ctypes.c_int, [vp, ctypes.POINTER(vp)]),
            "qpp_key_free": (None, [vp]),
            "qpp_key_free_batch": (None, [vp, sz]),
            "qpp_ctx_set_aes_kernel": (ctypes.c_int, [vp, ctypes.c_int]),
            "qpp_ctx_set_fips": (ctypes.c_int, [vp, ctypes.c_int]),
            "qpp_key_fips": (ctypes.c_int, [vp]),
            "qpp_key_slot": (u32, [vp]),
            "qpp_key_slot_batch": (None, [vp, sz, vp]),
            "qpp_key_suite": (ctypes.c_int, [vp]),
            "qpp_tag_len": (sz, [vp]),
            "qpp_sample_len": (sz, [vp]),
            "qpp_confidentiality_limit": (u64, [vp]),
            "qpp_integrity_limit": (u64, [vp]),
            "qpp_key_material": (ctypes.c_int, [vp, vp, vp, vp]),
            "qpp_initial_keys": (ctypes.c_int, [vp, ctypes.c_int, vp, sz, ctypes.POINTER(vp), ctypes.POINTER(vp)]),
            "qpp_seal": (ctypes.c_int, [vp, u64, vp, sz, vp, sz, sz]),
            "qpp_seal_scatter": (ctypes.c_int, [vp, u64, vp, sz, vp, sz, vp, sz, vp]),
            "qpp_open": (ctypes.c_int, [vp, u64, vp, sz, vp, sz]),
            "qpp_hp_mask": (ctypes.c_int, [vp, vp, sz, vp]),
            "qpp_seal_batch": (ctypes.c_int, [vp, vp, sz, vp, vp, vp, u32, vp]),
            "qpp_open_batch": (ctypes.c_int, [vp, vp, sz, vp, vp, u32, vp]),
            "qpp_hp_mask_batch": (ctypes.c_int, [vp, vp, sz, vp, vp, vp]),
            "qpp_dev_alloc": (ctypes.c_int, [vp, sz, ctypes.POINTER(vp)]),
            "qpp_dev_free": (None, [vp, vp]),
            "qpp_host_alloc": (ctypes.c_int, [vp, sz, ctypes.POINTER(vp)]),
            "qpp_host_free": (None, [vp, vp]),
            "qpp_memcpy_h2d": (ctypes.c_int, [vp, vp, vp, sz, vp]),
            "qpp_memcpy_d2h": (ctypes.c_int, [vp, vp, vp, sz, vp]),
            "qpp_memset_d": (ctypes.c_int, [vp, vp, ctypes.c_int, sz, vp]),
            "qpp_stream_create": (ctypes.c_int, [vp, ctypes.POINTER(vp)]),
            "qpp_stream_destroy": (None, [vp, vp]),
            "qpp_stream_synchronize": (ctypes.c_int, [vp, vp]),
            "qpp_event_create": (ctypes.c_int, [vp, ctypes.POINTER(vp)]),
            "qpp_event_destroy": (None, [vp, vp]),
            "qpp_event_record": (ctypes.c_int, [vp, vp, vp]),
            "qpp_event_elapsed_ms": (ctypes.c_int, [vp, vp, vp, ctypes.POINTER(ctypes.c_float)]),
            "qpp_stream_wait_event": (ctypes.c_int, [vp, vp, vp]),
            "qpp_unprotect_open_batch": (ctypes.c_int, [vp, vp, sz, vp, vp, vp, u32, vp]),
            "qpp_pn_truncate": (ctypes.c_int, [u64, u64, ctypes.POINTER(u64), ctypes.POINTER(sz)]),
            "qpp_pn_expand": (u64, [u64, u64, sz]),
            "qpp_key_new_batch": (ctypes.c_int, [vp, ctypes.c_int, vp, sz, u32, ctypes.POINTER(vp)]),
            "qpp_txq_create": (ctypes.c_int, [vp, sz, sz, ctypes.POINTER(vp)]),
            "qpp_txq_destroy": (None, [vp]),
            "qpp_txq_ring": (vp, [vp]),
            "qpp_txq_push": (ctypes.c_int, [vp, vp, u64, sz, sz, sz, sz]),
            "qpp_txq_flush": (ctypes.c_int, [vp]),
            "qpp_txq_create_async": (ctypes.c_int, [vp, sz, sz, sz, ctypes.POINTER(vp)]),
            "qpp_txq_flush_async": (ctypes.c_int, [vp, ctypes.POINTER(u64)]),
            "qpp_txq_poll": (ctypes.c_int, [vp, u64, ctypes.POINTER(ctypes.c_int)]),
            "qpp_txq_wait": (ctypes.c_int, [vp, u64]),
            "qpp_txq_push_descs": (ctypes.c_int, [vp, vp, sz]),
            "qpp_txq_push_scatter": (ctypes.c_int, [vp, vp, u64, sz, sz, sz, sz, vp, sz]),
            "qpp_txq_create_persistent": (ctypes.c_int, [vp, sz, sz, ctypes.POINTER(vp)]),
            "qpp_txq_info": (ctypes.c_int, [vp, ctypes.POINTER(u64), ctypes.POINTER(u64), ctypes.POINTER(u64)]),
            "qpp_txq_server_time": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_double)]),
            "qpp_txq_server_refused": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_uint64)]),
            "qpp_dev_server_evictions": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(u64), ctypes.POINTER(u64)]),
            "qpp_ctx_set_conn_keys": (ctypes.c_int, [vp, vp, sz]),
            "qpp_txq_server_stamps": (ctypes.c_int, [vp, vp]),
            "qpp_txq_set_coalesce": (ctypes.c_int, [vp, sz]),
            "qpp_txq_pending": (sz, [vp]),
            "qpp_memcpy_d2d": (ctypes.c_int, [vp, vp, vp, sz, vp]),
            "qpp_ctx_set_burst_max": (ctypes.c_int, [vp, sz]),
            "qpp_ctx_set_packet_server": (ctypes.c_int, [vp, ctypes.c_int]),
            "qpp_ctx_packet_server_info": (ctypes.c_int, [vp, ctypes.POINTER(u64), ctypes.POINTER(u64)]),
            "qpp_dc_key_new": (ctypes.c_int, [vp, ctypes.c_int, vp, sz, vp, ctypes.POINTER(vp)]),
            "qpp_dc_seal": (ctypes.c_int, [vp, u64, vp, sz, vp, sz, vp, sz]),
            "qpp_dc_open": (ctypes.c_int, [vp, ctypes.c_int, u64, vp, sz, vp, vp, sz, vp, sz]),
            "qpp_dc_open_in_place": (ctypes.c_int, [vp, ctypes.c_int, u64, vp, sz, vp, sz, vp, sz]),
            "qpp_ctx_key_slots": (ctypes.c_int, [vp, ctypes.POINTER(u32), ctypes.POINTER(u32), ctypes.POINTER(u32)]),
            "qpp_key_new_pair": (ctypes.c_int, [vp, ctypes.c_int, vp, sz, ctypes.POINTER(vp), ctypes.POINTER(vp)]),
            "qpp_key_update_batch": (ctypes.c_int, [vp, sz, vp]),
            "qpp_initial_keys_pair": (ctypes.c_int, [vp, ctypes.c_int, vp, sz] + [ctypes.POINTER(vp)] * 4),
            "qpp_header_key_new": (ctypes.c_int, [vp, ctypes.c_int, vp, sz, ctypes.POINTER(vp)]),
            "qpp_header_key_new_raw": (ctypes.c_int, [vp, ctypes.c_int, vp, sz, ctypes.POINTER(vp)]),
            "qpp_header_key_free": (None, [vp]),
            "qpp_header_key_slot": (u32, [vp]),
            "qpp_header_key_suite": (ctypes.c_int, [vp]),
            "qpp_header_key_sample_len": (sz, [vp]),
            "qpp_header_key_mask": (ctypes.c_int, [vp, vp, sz, vp]),
            "qpp_host_batch_submit": (ctypes.c_int, [vp, vp, sz, vp, vp, vp, u32, u32, ctypes.POINTER(u64)]),
            "qpp_host_batch_query": (ctypes.c_int, [vp, u64, ctypes.POINTER(ctypes.c_int)]),
            "qpp_host_batch_wait": (ctypes.c_int, [vp, u64]),
            "qpp_ctx_set_host_pipe": (ctypes.c_int, [vp, sz, sz, sz]),
        }
        assert set(sig) == set(EXPORTS)
        for name, (res, args) in sig.items():
            if name in _LATER and not hasattr(L, name) and os.environ.get("QPP_LIB"):
                continue  # (an earlier build loaded for a same-box A/B: it predates this entry point)
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _bytes_ptr(b):
    buf = ctypes.create_string_buffer(bytes(b), max(len(b), 1))
    return buf


class DeviceBuffer:
    """Raw device allocation owned by a Context."""

    def __init__(self, ctx, nbytes):
        self.ctx, self.nbytes = ctx, int(nbytes)
        p = vp()
        ctx._check(lib().qpp_dev_alloc(ctx.handle, self.nbytes, ctypes.byref(p)), "dev_alloc")
        self.ptr = p.value
        ctx._bufs.append(self)

    def upload(self, arr, stream=None, offset=0):
        a = np.ascontiguousarray(arr)
        assert offset + a.nbytes <= self.nbytes
        self.ctx._check(lib().qpp_memcpy_h2d(self.ctx.handle, self.ptr + offset, a.ctypes.data, a.nbytes, stream), "h2d")
        self.ctx.sync(stream)

    def download(self, nbytes=None, stream=None, dtype=np.uint8, offset=0):
        nbytes = self.nbytes - offset if nbytes is None else nbytes
        out = np.empty(nbytes, dtype=np.uint8)
        self.ctx._check(lib().qpp_memcpy_d2h(self.ctx.handle, out.ctypes.data, self.ptr + offset, nbytes, stream), "d2h")
        self.ctx.sync(stream)
        return out.view(dtype)

    def free(self):
        if self.ptr:
            if self.ctx.handle:
                lib().qpp_dev_free(self.ctx.handle, self.ptr)
            self.ptr = None
        try:  # (a long-lived context that makes temporary buffers does not keep them listed)
            self.ctx._bufs.remove(self)
        except ValueError:
            pass


class Context:
    """One MI355X (qpp_ctx): device key table, default stream, batch entry points."""

    def __init__(self, device=0):
        h = vp()
        rc = lib().qpp_ctx_create(int(device), ctypes.byref(h))
        if rc != OK:
            raise QppError(rc, f"qpp_ctx_create(device={device}): no usable gfx950 GPU (no CPU fallback exists)")
        self.handle = h.value
        self.device = device
        # what this wrapper handed out, released in order by close(): device work drained first, then events,
        # streams, device buffers and pinned host memory, and the context last -- nothing is left for the HIP
        # runtime's (or a profiler's) process-exit teardown to destroy behind a context that no longer exists
        self._bufs, self._events, self._streams, self._host = [], [], [], {}

    def close(self):
        if not self.handle:
            return
        h = self.handle
        lib().qpp_ctx_synchronize(h)
        for e in self._events:
            lib().qpp_event_destroy(h, e)
        for s in self._streams:
            lib().qpp_stream_destroy(h, s)
        for b in list(self._bufs):
            b.free()
        for p in self._host:
            lib().qpp_host_free(h, p)
        self._bufs, self._events, self._streams, self._host = [], [], [], {}
        lib().qpp_ctx_destroy(h)
        self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc, what):
        if rc != OK:
            err = lib().qpp_ctx_last_error(self.handle)
            raise QppError(rc, f"{what}: {err.decode() if err else ''}")

    @property
    def stream(self):
        return lib().qpp_ctx_stream(self.handle)

    def set_burst_max(self, max_packets):
        """AES batches of <= max_packets run one wave per packet (burst kernel); 0 = always lane per packet."""
        self._check(lib().qpp_ctx_set_burst_max(self.handle, int(max_packets)), "set_burst_max")

    def set_packet_server(self, on=True):
        """Per-packet seal / open through the context's resident packet server (default on) or one launch per call."""
        self._check(lib().qpp_ctx_set_packet_server(self.handle, int(bool(on))), "set_packet_server")

    def packet_server_info(self):
        """(per-packet calls the packet server took, its kernel launches)"""
        calls, starts = ctypes.c_uint64(), ctypes.c_uint64()
        self._check(lib().qpp_ctx_packet_server_info(self.handle, ctypes.byref(calls), ctypes.byref(starts)),
                    "packet_server_info")
        return calls.value, starts.value

    def set_aes_kernel(self, kernel):
        """AES_KERNEL_AUTO / _QUAD / _WAVE for batches above burst_max (identical outputs; A/B and tests)."""
        self._check(lib().qpp_ctx_set_aes_kernel(self.handle, int(kernel)), "set_aes_kernel")

    def set_fips(self, on=True):
        """FIPS mode (the s2n-quic-crypto `fips` feature): AES packet keys created from now on seal with aws-lc's TLS 1.3
        nonce-order rule (qpp.h qpp_ctx_set_fips); refused packets get status INTERNAL_ERROR and stay untouched."""
        self._check(lib().qpp_ctx_set_fips(self.handle, 1 if on else 0), "set_fips")

    def sync(self, stream=None):
        self._check(lib().qpp_stream_synchronize(self.handle, stream), "sync")

    # keys
    def key(self, suite, secret):
        h = vp()
        rc = lib().qpp_key_new(self.handle, suite, _bytes_ptr(secret), len(secret), ctypes.byref(h))
        if rc != OK:
            raise QppError(rc, "qpp_key_new")
        return Key(self, h.value)

    def key_pair(self, suite, secret):
        """TLS_*::new(secret) -> (Key, HeaderKey), independently owned (qpp_key_new_pair)."""
        k, h = vp(), vp()
        rc = lib().qpp_key_new_pair(self.handle, suite, _bytes_ptr(secret), len(secret), ctypes.byref(k),
                                    ctypes.byref(h))
        if rc != OK:
            raise QppError(rc, "qpp_key_new_pair")
        return Key(self, k.value), HeaderKey(self, h.value)

    def header_key(self, suite, secret=None, hp=None):
        """HeaderKey::new(secret, "quic hp") or from the raw header-protection key."""
        h = vp()
        if hp is not None:
            rc = lib().qpp_header_key_new_raw(self.handle, suite, _bytes_ptr(hp), len(hp), ctypes.byref(h))
        else:
            rc = lib().qpp_header_key_new(self.handle, suite, _bytes_ptr(secret), len(secret), ctypes.byref(h))
        if rc != OK:
            raise QppError(rc, "qpp_header_key_new")
        return HeaderKey(self, h.value)

    def update_keys(self, keys, slots_out=None):
        """qpp_key_update_batch: [k.derive_next_key() for k in keys] in one device pass per suite.  slots_out (a
        uint32 numpy array of len(keys)) receives the new keys' slots (qpp_key_slot_batch, one call)."""
        n = len(keys)
        arr_in = (vp * max(n, 1))(*[k.handle for k in keys])
        arr = (vp * max(n, 1))()
        rc = lib().qpp_key_update_batch(arr_in, n, arr)
        if rc != OK:
            raise QppError(rc, "qpp_key_update_batch")
        if slots_out is not None:
            assert slots_out.dtype == np.uint32 and slots_out.size >= n and slots_out.flags["C_CONTIGUOUS"]
            lib().qpp_key_slot_batch(arr, n, slots_out.ctypes.data)
        return [Key(self, arr[i]) for i in range(n)]

    def free_keys(self, keys):
        """qpp_key_free_batch: frees every key of the list (the old keys of a rotation) in one call."""
        live = [k for k in keys if k.handle]
        arr = (vp * max(len(live), 1))(*[k.handle for k in live])
        lib().qpp_key_free_batch(arr, len(live))
        for k in live:
            k.handle = None

    def key_slots(self):
        """(capacity, high-water slot, retired-not-yet-reusable) of the device key table."""
        c, h, r = u32(), u32(), u32()
        self._check(lib().qpp_ctx_key_slots(self.handle, ctypes.byref(c), ctypes.byref(h), ctypes.byref(r)), "slots")
        return c.value, h.value, r.value

    def set_host_pipe(self, chunk_packets, chunk_bytes, slots):
        self._check(lib().qpp_ctx_set_host_pipe(self.handle, chunk_packets, chunk_bytes, slots), "set_host_pipe")

    def set_conn_keys(self, slots):
        """qpp_ctx_set_conn_keys: slots[c] = the current key slot of connection c (QPP_KEY_BY_CONN host batches)"""
        slots = np.ascontiguousarray(slots, dtype=np.uint32)
        self._check(lib().qpp_ctx_set_conn_keys(self.handle, slots.ctypes.data, len(slots)), "set_conn_keys")

    def host_submit(self, descs, arena, masks=None, status=None, flags=0, ops=OP_SEAL | OP_OPEN):
        """qpp_host_batch_submit over host numpy arrays (arena ideally from host_alloc); returns the ticket.
        The arrays must stay alive and untouched until host_wait(ticket)."""
        t = u64()
        self._check(lib().qpp_host_batch_submit(self.handle, descs.ctypes.data, len(descs), arena.ctypes.data,
                                                None if masks is None else masks.ctypes.data,
                                                None if status is None else status.ctypes.data, flags, ops,
                                                ctypes.byref(t)), "host_batch_submit")
        return t.value

    def host_done(self, ticket):
        d = ctypes.c_int()
        self._check(lib().qpp_host_batch_query(self.handle, ticket, ctypes.byref(d)), "host_batch_query")
        return bool(d.value)

    def host_wait(self, ticket):
        self._check(lib().qpp_host_batch_wait(self.handle, ticket), "host_batch_wait")

    def keys_batch(self, suite, secrets, updates=0):
        """qpp_key_new_batch: every secret -> `updates` x derive_next_key, derived on the GPU in one pass."""
        secrets = [bytes(x) for x in secrets]
        n = len(secrets)
        arr = (vp * max(n, 1))()
        rc = lib().qpp_key_new_batch(self.handle, suite, _bytes_ptr(b"".join(secrets)), n, updates, arr)
        if rc != OK:
            raise QppError(rc, "qpp_key_new_batch")
        return [Key(self, arr[i]) for i in range(n)]

    def raw_key(self, suite, key, iv, hp):
        h = vp()
        rc = lib().qpp_key_new_raw(self.handle, suite, _bytes_ptr(key), len(key), _bytes_ptr(iv), _bytes_ptr(hp),
                                   len(hp), ctypes.byref(h))
        if rc != OK:
            raise QppError(rc, "qpp_key_new_raw")
        return Key(self, h.value)

    def dc_key(self, suite, key, iv):
        """dc seal/open::Application::new(key, iv, algorithm) (dc/s2n-quic-dc/src/crypto/awslc.rs:24-33)"""
        h = vp()
        rc = lib().qpp_dc_key_new(self.handle, suite, _bytes_ptr(key), len(key), _bytes_ptr(iv), ctypes.byref(h))
        if rc != OK:
            raise QppError(rc, "qpp_dc_key_new")
        return DcKey(self, h.value)

    def initial_keys_pair(self, endpoint, dcid):
        """InitialKey::new_* -> (sealer, opener, header sealer, header opener)"""
        hs = [vp() for _ in range(4)]
        rc = lib().qpp_initial_keys_pair(self.handle, endpoint, _bytes_ptr(dcid), len(dcid), *[ctypes.byref(h) for h in hs])
        if rc != OK:
            raise QppError(rc, "qpp_initial_keys_pair")
        return Key(self, hs[0].value), Key(self, hs[1].value), HeaderKey(self, hs[2].value), HeaderKey(self, hs[3].value)

    def initial_keys(self, endpoint, dcid):
        s, o = vp(), vp()
        rc = lib().qpp_initial_keys(self.handle, endpoint, _bytes_ptr(dcid), len(dcid), ctypes.byref(s), ctypes.byref(o))
        if rc != OK:
            raise QppError(rc, "qpp_initial_keys")
        return Key(self, s.value), Key(self, o.value)

    def alloc(self, nbytes):
        return DeviceBuffer(self, nbytes)

    # batches (device pointers)
    def seal_batch(self, descs, n, arena, masks=None, status=None, flags=0, stream=None):
        self._check(lib().qpp_seal_batch(self.handle, _ptr(descs), n, _ptr(arena), _ptr(masks), _ptr(status), flags,
                                         stream), "seal_batch")

    def open_batch(self, descs, n, arena, status, flags=0, stream=None):
        self._check(lib().qpp_open_batch(self.handle, _ptr(descs), n, _ptr(arena), _ptr(status), flags, stream),
                    "open_batch")

    def unprotect_open_batch(self, rx, n, arena, descs_out, status, flags=0, stream=None):
        """Receive path: remove HP, expand the PN, pick the key by key phase, open (qpp_unprotect_open_batch)."""
        self._check(lib().qpp_unprotect_open_batch(self.handle, _ptr(rx), n, _ptr(arena), _ptr(descs_out), _ptr(status),
                                                   flags, stream), "unprotect_open_batch")

    def hp_mask_batch(self, descs, n, arena, masks, stream=None):
        self._check(lib().qpp_hp_mask_batch(self.handle, _ptr(descs), n, _ptr(arena), _ptr(masks), stream),
                    "hp_mask_batch")

    # timing on a stream (HIP events)
    def event(self):
        e = vp()
        self._check(lib().qpp_event_create(self.handle, ctypes.byref(e)), "event")
        self._events.append(e.value)
        return e.value

    def event_destroy(self, ev):
        if ev in self._events:
            self._events.remove(ev)
            lib().qpp_event_destroy(self.handle, ev)

    def record(self, ev, stream=None):
        self._check(lib().qpp_event_record(self.handle, ev, stream), "record")

    def new_stream(self):
        st = vp()
        self._check(lib().qpp_stream_create(self.handle, ctypes.byref(st)), "stream")
        self._streams.append(st.value)
        return st.value

    def stream_destroy(self, stream):
        if stream in self._streams:
            self._streams.remove(stream)
        lib().qpp_stream_destroy(self.handle, stream)

    def rx_timeouts(self):
        """fused-receive workgroups that left on a grid-barrier timeout since creation (qpp_ctx_rx_timeouts)"""
        c = u64()
        self._check(lib().qpp_ctx_rx_timeouts(self.handle, ctypes.byref(c)), "rx_timeouts")
        return c.value

    def synchronize(self):
        """qpp_ctx_synchronize: every stream of this context (key installs and retirements included), not the device"""
        self._check(lib().qpp_ctx_synchronize(self.handle), "synchronize")

    def wait(self, stream, ev):
        self._check(lib().qpp_stream_wait_event(self.handle, stream, ev), "wait_event")

    def host_alloc(self, nbytes):
        """pinned host memory as a numpy uint8 array (host_free it, or close() releases it: no view may outlive either)"""
        p = vp()
        self._check(lib().qpp_host_alloc(self.handle, int(nbytes), ctypes.byref(p)), "host_alloc")
        self._host[p.value] = int(nbytes)
        return np.ctypeslib.as_array((ctypes.c_uint8 * int(nbytes)).from_address(p.value))

    def host_free(self, arr):
        """release a host_alloc array (no view of it may be used afterwards)"""
        p = arr.ctypes.data
        self._host.pop(p, None)
        lib().qpp_host_free(self.handle, p)

    def elapsed_ms(self, e0, e1):
        ms = ctypes.c_float()
        self._check(lib().qpp_event_elapsed_ms(self.handle, e0, e1, ctypes.byref(ms)), "elapsed")
        return ms.value


def _ptr(x):
    if x is None:
        return None
    if isinstance(x, DeviceBuffer):
        return x.ptr
    return int(x)


class Key:
    """One direction's packet key + header key (TLS_*::new -> (Self, HeaderKey))."""

    def __init__(self, ctx, handle):
        self.ctx, self.handle = ctx, handle

    def free(self):
        if self.handle:
            lib().qpp_key_free(self.handle)
            self.handle = None

    @property
    def slot(self):
        return lib().qpp_key_slot(self.handle)

    @property
    def suite(self):
        return lib().qpp_key_suite(self.handle)

    @property
    def fips(self):
        """True when the key seals in FIPS mode (Context.set_fips was on when it was created; AES suites only)."""
        return bool(lib().qpp_key_fips(self.handle))

    def tag_len(self):
        return lib().qpp_tag_len(self.handle)

    def sample_len(self):
        return lib().qpp_sample_len(self.handle)

    def aead_confidentiality_limit(self):
        return lib().qpp_confidentiality_limit(self.handle)

    def aead_integrity_limit(self):
        return lib().qpp_integrity_limit(self.handle)

    def material(self):
        kl = KEY_LEN[self.suite]
        k, iv, hp = (ctypes.c_uint8 * 32)(), (ctypes.c_uint8 * 12)(), (ctypes.c_uint8 * 32)()
        lib().qpp_key_material(self.handle, k, iv, hp)
        return bytes(k[:kl]), bytes(iv), bytes(hp[:kl])

    def derive_next_key(self):
        h = vp()
        rc = lib().qpp_key_update(self.handle, ctypes.byref(h))
        if rc != OK:
            raise QppError(rc, "qpp_key_update")
        return Key(self.ctx, h.value)

    def encrypt(self, pn, header, payload):
        buf = ctypes.create_string_buffer(bytes(payload) + bytes(16), len(payload) + 16)
        rc = lib().qpp_seal(self.handle, pn, _bytes_ptr(header), len(header), buf, len(payload), len(payload) + 16)
        if rc != OK:
            raise QppError(rc, "qpp_seal")
        return buf.raw

    def encrypt_scatter(self, pn, header, inline, extra):
        io = ctypes.create_string_buffer(bytes(inline), max(len(inline), 1))
        out = ctypes.create_string_buffer(len(extra) + 16)
        rc = lib().qpp_seal_scatter(self.handle, pn, _bytes_ptr(header), len(header), io, len(inline),
                                    _bytes_ptr(extra), len(extra), out)
        if rc != OK:
            raise QppError(rc, "qpp_seal_scatter")
        return io.raw[:len(inline)], out.raw

    def decrypt(self, pn, header, payload):
        buf = ctypes.create_string_buffer(bytes(payload), max(len(payload), 1))
        rc = lib().qpp_open(self.handle, pn, _bytes_ptr(header), len(header), buf, len(payload))
        if rc == DECRYPT_ERROR:
            raise DecryptError(rc, "qpp_open")
        if rc != OK:
            raise QppError(rc, "qpp_open")
        return buf.raw[:len(payload) - 16]

    def header_protection_mask(self, sample):
        out = (ctypes.c_uint8 * 5)()
        rc = lib().qpp_hp_mask(self.handle, _bytes_ptr(sample), len(sample), out)
        if rc != OK:
            raise QppError(rc, "qpp_hp_mask")
        return bytes(out)


class HeaderKey:
    """HeaderKey (header_key.rs:7-63): owned independently of the packet keys it was born with."""

    def __init__(self, ctx, handle):
        self.ctx, self.handle = ctx, handle

    def free(self):
        if self.handle:
            lib().qpp_header_key_free(self.handle)
            self.handle = None

    @property
    def slot(self):
        return lib().qpp_header_key_slot(self.handle)

    @property
    def suite(self):
        return lib().qpp_header_key_suite(self.handle)

    def sample_len(self):
        return lib().qpp_header_key_sample_len(self.handle)

    def header_protection_mask(self, sample):
        out = (ctypes.c_uint8 * 5)()
        rc = lib().qpp_header_key_mask(self.handle, _bytes_ptr(sample), len(sample), out)
        if rc != OK:
            raise QppError(rc, "qpp_header_key_mask")
        return bytes(out)

    sealing_header_protection_mask = header_protection_mask
    opening_header_protection_mask = header_protection_mask


# ------------------------------------------------------------------ synthetic batches (bench + tests)

class DcKey(Key):
    """dc/s2n-quic-dc crypto::{seal,open}::Application over the same engine (crypto/awslc.rs:40-83,168-227)."""

    def dc_encrypt(self, pn, header, extra_payload, payload_and_tag):
        """seal::Application::encrypt: returns the sealed payload_and_tag buffer"""
        extra = bytes(extra_payload or b"")
        buf = ctypes.create_string_buffer(bytes(payload_and_tag), max(len(payload_and_tag), 1))
        rc = lib().qpp_dc_seal(self.handle, pn, _bytes_ptr(header), len(header), _bytes_ptr(extra), len(extra), buf,
                               len(payload_and_tag))
        if rc != OK:
            raise QppError(rc, "qpp_dc_seal")
        return buf.raw[:len(payload_and_tag)]

    def dc_decrypt(self, key_phase, pn, header, payload_in, tag):
        """open::Application::decrypt (separate input, tag and output)"""
        out = ctypes.create_string_buffer(max(len(payload_in), 1))
        rc = lib().qpp_dc_open(self.handle, key_phase, pn, _bytes_ptr(header), len(header), _bytes_ptr(payload_in),
                               _bytes_ptr(tag), len(tag), out, len(payload_in))
        if rc == DECRYPT_ERROR:
            raise DecryptError(rc, "qpp_dc_open")
        if rc != OK:
            raise QppError(rc, "qpp_dc_open")
        return out.raw[:len(payload_in)]

    def dc_decrypt_in_place(self, key_phase, pn, header, payload, tag):
        """open::Application::decrypt_in_place; returns (status, buffer after the call)"""
        buf = ctypes.create_string_buffer(bytes(payload), max(len(payload), 1))
        rc = lib().qpp_dc_open_in_place(self.handle, key_phase, pn, _bytes_ptr(header), len(header), buf,
                                        len(payload), _bytes_ptr(tag), len(tag))
        return rc, buf.raw[:len(payload)]


def xoshiro_bytes(seed, n):
    """Deterministic synthetic payload bytes (numpy PCG64 seeded from `seed`)."""
    return np.random.Generator(np.random.PCG64(seed)).integers(0, 256, size=n, dtype=np.uint8)


def make_batch(n, pt_len, key_slots, seed, aad_len=21, pn_len=4, pn_base=0, stride=None, mixed=True, run=1):
    """Packets back to back in an arena: [AAD aad_len | payload pt_len | tag 16] per `stride` bytes.

    AAD = 1-RTT short header 0x43 || DCID(16) || PN(4).  key_idx = splitmix64(i // run) % len(key_slots)
    when mixed (run > 1: runs of `run` consecutive packets of one connection, a GSO burst), else key_slots[0].
    Returns (descs, arena).
    """
    stride = stride or ((aad_len + pt_len + 16 + 15) // 16) * 16
    if n * stride > 1 << 32:
        raise ValueError(f"{n} x {stride} B exceeds the 4 GiB arena window of one batch (qpp_pkt.off is 32-bit); "
                         "split the batch")
    arena = xoshiro_bytes(seed, n * stride)
    descs = np.zeros(n, dtype=PKT_DTYPE)
    idx = np.arange(n, dtype=np.uint64)
    descs["pn"] = (np.uint64(pn_base) + idx) & np.uint64((1 << 62) - 1)
    descs["off"] = (idx * np.uint64(stride)).astype(np.uint32)
    descs["aad_len"] = aad_len
    descs["pt_len"] = pt_len
    descs["pn_len"] = pn_len
    slots = np.asarray(key_slots, dtype=np.uint32)
    if mixed and len(slots) > 1:
        z = (idx // np.uint64(max(1, run)) + np.uint64(0x9E3779B97F4A7C15)) * np.uint64(1)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
        descs["key_idx"] = slots[(z % np.uint64(len(slots))).astype(np.int64)]
    else:
        descs["key_idx"] = slots[0]
    if aad_len >= 1:
        arena.reshape(n, stride)[:, 0] = 0x43
    return descs, arena


def server_evictions(device=0):
    """qpp_dev_server_evictions: (frees past the parked bound that evicted the device's resident servers, one-shot server
    launches that finished a posted flush while every server slot was taken)"""
    a, b = u64(), u64()
    rc = lib().qpp_dev_server_evictions(device, ctypes.byref(a), ctypes.byref(b))
    if rc != OK:
        raise QppError(rc, "qpp_dev_server_evictions")
    return a.value, b.value


def pn_truncate(pn, largest_acked):
    """PacketNumber::truncate -> (truncated, pn_len); raises QppError(DECODE_ERROR) when it cannot be encoded."""
    t, ln = u64(), sz()
    rc = lib().qpp_pn_truncate(pn, largest_acked, ctypes.byref(t), ctypes.byref(ln))
    if rc != OK:
        raise QppError(rc, "pn_truncate")
    return t.value, ln.value


def pn_expand(largest_acked, truncated, pn_len):
    """TruncatedPacketNumber::expand (RFC 9000 A.3)."""
    return lib().qpp_pn_expand(largest_acked, truncated, pn_len)


class TxQueue:
    """qpp_txq: deferred Key::encrypt + header protection over a pinned ring (the GSO segment buffer)."""

    def __init__(self, ctx, ring_bytes, max_packets, in_flight=1, persistent=False):
        """persistent: qpp_txq_create_persistent (one flush in flight, posted to a resident server kernel)"""
        h = vp()
        if persistent:
            rc = lib().qpp_txq_create_persistent(ctx.handle, ring_bytes, max_packets, ctypes.byref(h))
        else:
            rc = lib().qpp_txq_create_async(ctx.handle, ring_bytes, max_packets, in_flight, ctypes.byref(h))
        if rc != OK:
            raise QppError(rc, "qpp_txq_create")
        self.handle, self.ctx = h.value, ctx
        self.ring = np.ctypeslib.as_array((ctypes.c_uint8 * ring_bytes).from_address(lib().qpp_txq_ring(self.handle)))

    def push(self, key, pn, off, header_len, pn_len, payload_len):
        rc = lib().qpp_txq_push(self.handle, key.handle, pn, off, header_len, pn_len, payload_len)
        if rc != OK:
            raise QppError(rc, "qpp_txq_push")

    def flush(self):
        rc = lib().qpp_txq_flush(self.handle)
        if rc != OK:
            raise QppError(rc, "qpp_txq_flush")

    def push_scatter(self, key, pn, off, header_len, pn_len, inline_len, extra=b""):
        """qpp_txq_push_scatter: the inline plaintext is in the ring; `extra` (scatter::Buffer's tail) is copied after it"""
        buf = (ctypes.c_uint8 * max(1, len(extra))).from_buffer_copy(bytes(extra) or b"\0")
        rc = lib().qpp_txq_push_scatter(self.handle, key.handle, pn, off, header_len, pn_len, inline_len,
                                        ctypes.cast(buf, vp) if extra else None, len(extra))
        if rc != OK:
            raise QppError(rc, "qpp_txq_push_scatter")

    def info(self):
        """qpp_txq_info: (flushes sealed by the persistent server, flushes launched, server launches)"""
        a, b, c = u64(), u64(), u64()
        rc = lib().qpp_txq_info(self.handle, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
        if rc != OK:
            raise QppError(rc, "qpp_txq_info")
        return a.value, b.value, c.value

    def server_refused(self):
        """qpp_txq_server_refused: descriptors the server refused as lying outside the ring (always 0)"""
        c = ctypes.c_uint64()
        rc = lib().qpp_txq_server_refused(self.handle, ctypes.byref(c))
        if rc != OK:
            raise QppError(rc, "qpp_txq_server_refused")
        return c.value

    def server_time_us(self):
        """qpp_txq_server_time: doorbell seen -> completion of the last posted flush, on the server's clock"""
        t = ctypes.c_double()
        rc = lib().qpp_txq_server_time(self.handle, ctypes.byref(t))
        if rc != OK:
            raise QppError(rc, "qpp_txq_server_time")
        return t.value

    def push_descs(self, descs):
        """qpp_txq_push_descs: a PKT_DTYPE array of ready descriptors in one call"""
        descs = np.ascontiguousarray(descs, dtype=PKT_DTYPE)
        rc = lib().qpp_txq_push_descs(self.handle, descs.ctypes.data, len(descs))
        if rc != OK:
            raise QppError(rc, "qpp_txq_push_descs")

    def set_coalesce(self, bursts):
        rc = lib().qpp_txq_set_coalesce(self.handle, bursts)
        if rc != OK:
            raise QppError(rc, "qpp_txq_set_coalesce")

    def flush_async(self):
        """qpp_txq_flush_async -> ticket (the pushed packets' ring bytes belong to the engine until it completes)"""
        t = u64()
        rc = lib().qpp_txq_flush_async(self.handle, ctypes.byref(t))
        if rc != OK:
            raise QppError(rc, "qpp_txq_flush_async")
        return t.value

    def poll(self, ticket):
        d = ctypes.c_int()
        rc = lib().qpp_txq_poll(self.handle, ticket, ctypes.byref(d))
        if rc != OK:
            raise QppError(rc, "qpp_txq_poll")
        return bool(d.value)

    def wait(self, ticket):
        rc = lib().qpp_txq_wait(self.handle, ticket)
        if rc != OK:
            raise QppError(rc, "qpp_txq_wait")

    def pending(self):
        return lib().qpp_txq_pending(self.handle)

    def close(self):
        if self.handle:
            self.ring = None
            lib().qpp_txq_destroy(self.handle)
            self.handle = None
