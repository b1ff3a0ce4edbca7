"""Hot-loop census of one kernel in a hipcc -save-temps .s: the innermost backward-branch loops between 2000 and 8000
instructions, with their VALU / LDS / scratch / readlane counts.  usage: python3 isa_hot.py FILE.s SYMBOL_SUBSTR"""
import re
import sys
from collections import Counter

txt = open(sys.argv[1]).read()
name = [m.group(1) for m in re.finditer(r'^(\S+):', txt, re.M) if sys.argv[2] in m.group(1) and not m.group(1).startswith('.')][0]
i = txt.index(name + ':')
lines = txt[i:txt.index('.Lfunc_end', i)].split('\n')
labels = {m.group(1): n for n, l in enumerate(lines) for m in [re.match(r'^(\.LBB\d+_\d+):', l)] if m}
seen = set()
for n, l in enumerate(lines):
    m = re.search(r's_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)', l)
    if not (m and m.group(1) in labels and labels[m.group(1)] < n):
        continue
    a = labels[m.group(1)]
    ins = [x.strip().split()[0] for x in lines[a:n] if x.strip() and not x.strip().startswith(('.', ';')) and not x.strip().endswith(':')]
    if not 2000 <= len(ins) <= 8000 or a in seen:
        continue
    seen.add(a)
    c = Counter(ins)
    print(f'loop @{a}: instr {len(ins)} valu {sum(v for k, v in c.items() if k.startswith("v_"))} '
          f'ds {sum(v for k, v in c.items() if k.startswith("ds_"))} scratch {sum(v for k, v in c.items() if "scratch" in k)} '
          f'readlane {c["v_readlane_b32"]} vmem {sum(v for k, v in c.items() if k.startswith(("global_", "buffer_")))}')
