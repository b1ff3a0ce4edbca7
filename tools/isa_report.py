"""Per-kernel ISA report for quad.hip / aes_gcm.hip / chacha.hip: the largest loop's instruction mix (where the time goes).
usage: python tools/isa_report.py [source.hip] [kernel-substring ...]"""
import collections
import os
import re
import subprocess
import sys
import tempfile

SRC = sys.argv[1] if len(sys.argv) > 1 else "s2n-quic_amd/csrc/quad.hip"
PATS = sys.argv[2:] or ["aes_gcm_quad_kernel"]
tmp = tempfile.mkdtemp()
subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-munsafe-fp-atomics", "-c", os.path.abspath(SRC),
                       "-o", os.path.join(tmp, "x.o"), "-save-temps"], cwd=tmp, stderr=subprocess.DEVNULL)
asm = [f for f in os.listdir(tmp) if f.endswith("gfx950.s")][0]
src = open(os.path.join(tmp, asm)).read()
for m in re.finditer(r"^(_Z\S+):\s*;\s*@", src, re.M):
    name = m.group(1)
    if not any(p in name for p in PATS):
        continue
    body = src[m.end():src.index("s_endpgm", m.end())]
    blocks, cur = [], None
    for l in body.split("\n"):
        l = l.strip()
        mm = re.match(r"^(\.LBB\d+_\d+):", l)
        if mm:
            cur = [mm.group(1), []]
            blocks.append(cur)
            continue
        if cur is None:
            cur = ["entry", []]
            blocks.append(cur)
        if l and not l.startswith((";", ".")):
            cur[1].append(l)
    idx = {b[0]: k for k, b in enumerate(blocks)}
    best = None
    for k, (lab, ins) in enumerate(blocks):
        for s in ins:
            mm = re.match(r"s_(?:cbranch_\w+|branch) (\.LBB\d+_\d+)", s)
            if mm and idx.get(mm.group(1), 1e9) <= k:
                loop = blocks[idx[mm.group(1)]:k + 1]
                n = sum(len(x[1]) for x in loop)
                # innermost big loop: fewest blocks among loops with > 60% of the max size
                best = loop if best is None or n > sum(len(x[1]) for x in best) else best
    if not best:
        continue
    c = collections.Counter(s.split()[0] for x in best for s in x[1])
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    print(f"{name[:90]}\n   loop insts={sum(c.values())} blocks={len(best)} VALU={valu} ds_read_b32={c['ds_read_b32']} "
          f"ds_read2={c['ds_read2_b32']} ds_read_b128={c['ds_read_b128']} s_waitcnt={c['s_waitcnt']} "
          f"global_load={c['global_load_dwordx4'] + c['global_load_dword']} global_store={c['global_store_dwordx4']} "
          f"readlane={c['v_readlane_b32']} s_load={sum(v for k, v in c.items() if k.startswith('s_load'))}")
