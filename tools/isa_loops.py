"""Every loop (back edge) of one kernel with its instruction mix, and the opcode histogram of the loop chosen with
--pick (default: the loop with the most ds_read_b32, i.e. the CTR group loop of the AES kernel).
usage: python tools/isa_loops.py [source.hip] kernel-substring [--pick K] [-D MACRO ...]"""
import collections
import os
import re
import subprocess
import sys
import tempfile

args = sys.argv[1:]
defs = [a for a in args if a.startswith("-D")]
args = [a for a in args if not a.startswith("-D")]
pick = None
if "--pick" in args:
    i = args.index("--pick")
    pick = int(args[i + 1])
    del args[i:i + 2]
SRC = args[0] if args else "s2n-quic_amd/csrc/aes_gcm.hip"
PAT = args[1] if len(args) > 1 else "aes_gcm_kernelILb1ELi4ELi512ELi10E"
tmp = tempfile.mkdtemp()
subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", *defs, "-c",
                       os.path.abspath(SRC), "-o", os.path.join(tmp, "x.o"), "-save-temps"], cwd=tmp,
                      stderr=subprocess.DEVNULL)
asm = [f for f in os.listdir(tmp) if f.endswith("gfx950.s")][0]
src = open(os.path.join(tmp, asm)).read()
for m in re.finditer(r"^(_Z\S+):\s*;\s*@", src, re.M):
    name = m.group(1)
    if PAT not in name:
        continue
    tail = src[m.end():]
    meta = re.search(r"; NumVgprs: (\d+).*?; ScratchSize: (\d+)", tail, re.S)
    body = tail[:tail.index("s_endpgm")]
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
    loops = []
    for k, (lab, ins) in enumerate(blocks):
        for s in ins:
            mm = re.match(r"s_(?:cbranch_\w+|branch) (\.LBB\d+_\d+)", s)
            if mm and idx.get(mm.group(1), 1e9) <= k:
                loops.append(blocks[idx[mm.group(1)]:k + 1])
    print(name[:100], "vgprs/scratch", meta.groups() if meta else "?")
    hists = []
    for n, lp in enumerate(loops):
        c = collections.Counter(s.split()[0] for x in lp for s in x[1])
        hists.append(c)
        valu = sum(v for k, v in c.items() if k.startswith("v_"))
        print(f"  loop {n}: insts={sum(c.values())} blocks={len(lp)} VALU={valu} ds_read_b32={c['ds_read_b32']} "
              f"ds_read_b128={c['ds_read_b128']} ds_write_b128={c['ds_write_b128']} s_waitcnt={c['s_waitcnt']} "
              f"SALU={sum(v for k, v in c.items() if k.startswith('s_'))}")
    if not hists:
        continue
    k = pick if pick is not None else max(range(len(hists)), key=lambda i: hists[i]["ds_read_b32"])
    print(f"  -- loop {k} opcode histogram")
    for op, v in hists[k].most_common(40):
        print(f"     {op:28s} {v}")
