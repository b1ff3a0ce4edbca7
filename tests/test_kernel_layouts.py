"""CPU checks of properties the GPU kernels rely on but cannot assert at run time:

* the LDS bank-conflict freedom of the staging layouts (MI355X_MICROARCH.md §LDS: ds_read_b128 is served in four
  16-lane groups over 64 banks, ds_write_b128 in 8-lane groups over 32 banks; a 16-B slot covers 4 banks), for the
  ChaCha20-Poly1305 pair stage (csrc/chacha.hip) and the AES-GCM Stage<4> (csrc/device_common.h);
* that the build's kernel-resource check (csrc/check_resources.py) rejects static LDS in the AES-GCM kernels (they
  reserve all 160 KiB dynamically) and scratch in their default variants.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

READ_B128_GROUPS = [[0, 1, 2, 3, 12, 13, 14, 15] + list(range(20, 28)),
                    list(range(4, 12)) + [16, 17, 18, 19, 28, 29, 30, 31]]
READ_B128_GROUPS += [[x + 32 for x in g] for g in READ_B128_GROUPS]
WRITE_B128_GROUPS = [list(range(8 * t, 8 * t + 8)) for t in range(8)]


def _chacha_slot(p, j):  # chacha.hip: stage slot of packet p's block j of the pair
    return 64 * (p // 8) + 8 * (p % 8) + ((j + p + (p >> 4)) & 7)


def test_chacha_pair_stage_is_conflict_free():
    for j in range(8):
        for g in READ_B128_GROUPS:  # owner reads: 16 distinct bank quads of 64 banks
            assert len({_chacha_slot(p, j) % 16 for p in g}) == 16, (j, g)
        for g in WRITE_B128_GROUPS:  # owner writes: 8 distinct bank quads of 32 banks
            assert len({_chacha_slot(p, j) % 8 for p in g}) == 8, (j, g)


def test_chacha_pair_stage_lane_linear_roles():
    # pair instruction i, lane l: packet 8 i + l / 8, block lj(i) lands at / is read from slot 64 i + l, and the 8
    # lanes of a packet cover its 8 blocks (128 contiguous bytes)
    for i in range(8):
        for q in range(8):
            blocks = set()
            for l in range(8 * q, 8 * q + 8):
                p = 8 * i + l // 8
                lj = ((l & 7) - (l // 8 + (i >> 1))) & 7
                assert _chacha_slot(p, lj) == 64 * i + l
                blocks.add(lj)
            assert blocks == set(range(8))


def test_aes_stage4_is_conflict_free():
    nb, ppi = 4, 16  # Stage<4>: own(k) of lane p, coop(i) of lane l

    def rho(p):
        return ((p >> 1) + (p >> 4)) & 3

    def own(p, k):
        return 64 * (p // ppi) + nb * (p % ppi) + ((k + rho(p)) % nb)

    for k in range(nb):
        for g in READ_B128_GROUPS:
            assert len({own(p, k) % 16 for p in g}) == 16, (k, g)
        for g in WRITE_B128_GROUPS:
            assert len({own(p, k) % 8 for p in g}) == 8, (k, g)
    # the cooperative role of lane l in instruction i: packet ppi i + l / nb, chunk coop_chunk, at slot 64 i + l
    for i in range(nb):
        for l in range(64):
            p = ppi * i + l // nb
            k = ((l % nb) + nb - rho(p) % nb) % nb
            assert own(p, k) == 64 * i + l


def _check(text):
    return subprocess.run([sys.executable, os.path.join(ROOT, "s2n-quic_amd", "csrc", "check_resources.py"), text],
                          capture_output=True, text=True)


def test_resource_check_rejects_static_lds_and_scratch(tmp_path):
    name = "_ZN3qpp12_GLOBAL__N_119aes_gcm_quad_kernelILb1ELi10EEEvPKNS_6DevKeyE"
    ok = tmp_path / "ok.res"
    ok.write_text(f"x: remark: Function Name: {name}\nx: remark:     ScratchSize [bytes/lane]: 0\n"
                  "x: remark:     LDS Size [bytes/block]: 0\n")
    assert _check(str(ok)).returncode == 0
    lds = tmp_path / "lds.res"
    lds.write_text(f"x: remark: Function Name: {name}\nx: remark:     LDS Size [bytes/block]: 32768\n")
    r = _check(str(lds))
    assert r.returncode != 0 and "static LDS" in r.stderr
    scr = tmp_path / "scr.res"
    # (up to 32 B/lane -- a few per-packet spills outside the group loop -- is tolerated; more is refused)
    scr.write_text(f"x: remark: Function Name: {name}\nx: remark:     ScratchSize [bytes/lane]: 48\n")
    r = _check(str(scr))
    assert r.returncode != 0 and "scratch" in r.stderr
    # a kernel outside the no-spill set (AES-256) may use scratch; it may not add static LDS either
    other = tmp_path / "other.res"
    other.write_text("x: remark: Function Name: _ZN3qpp12_GLOBAL__N_119aes_gcm_quad_kernelILb1ELi14EEEvPKNS_6DevKeyE\n"
                     "x: remark:     ScratchSize [bytes/lane]: 52\n")
    assert _check(str(other)).returncode == 0
