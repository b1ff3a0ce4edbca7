"""CPU checks of the drop-in boundary: libqpp.so loads, exports every function include/qpp.h declares,
the Python view binds exactly that set, struct layouts agree, and with no GPU the engine refuses to run
(QPP_DEVICE_ERROR) instead of falling back to the CPU."""
import ctypes
import os
import re

import numpy as np
import pytest

import qpp
import _oracle as orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "qpp.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(qpp_\w+)\s*\(", src)))


def test_header_matches_binding():
    assert declared_functions() == sorted(qpp.EXPORTS)


def test_library_exports_every_symbol():
    L = ctypes.CDLL(qpp.LIB_PATH)
    for name in declared_functions():
        assert hasattr(L, name), name
    assert qpp.lib().qpp_abi_version() == 2


def test_pkt_layout_matches_oracle():
    assert qpp.PKT_DTYPE.itemsize == ctypes.sizeof(orc.OrcPkt) == 24
    for name, off in (("pn", 0), ("key_idx", 8), ("off", 12), ("aad_len", 16), ("pt_len", 18), ("pn_len", 20)):
        assert qpp.PKT_DTYPE.fields[name][1] == getattr(orc.OrcPkt, name).offset


def test_no_cpu_fallback_without_gpu():
    import subprocess
    import sys
    # probe in a child so this process never initialises HIP
    code = ("import sys; sys.path.insert(0, %r); import qpp\n"
            "try:\n    qpp.Context(0)\nexcept qpp.QppError as e:\n    print('ERR', e.code)\nelse:\n    print('GPU')\n"
            % os.path.join(ROOT, "s2n-quic_amd"))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120).stdout
    if "GPU" in out:
        pytest.skip("a GPU is present: covered by the -m gpu tests")
    assert "ERR 5" in out


def test_synthetic_batch_layout():
    descs, arena = qpp.make_batch(64, 1200, [3, 7], seed=1)
    assert arena.size == 64 * 1248 and descs["off"][1] == 1248
    assert set(np.unique(descs["key_idx"])) <= {3, 7} and len(np.unique(descs["key_idx"])) == 2
    assert (arena.reshape(64, 1248)[:, 0] == 0x43).all()
    assert descs["pn"][5] == 5


def test_batch_arena_window_is_4gib():
    # qpp_pkt.off is 32-bit: one batch addresses a 4 GiB arena window (include/qpp.h); larger sets are split
    with pytest.raises(ValueError):
        qpp.make_batch(4 << 20, 1200, [0], seed=1)
