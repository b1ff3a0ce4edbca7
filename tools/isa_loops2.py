"""Per-loop instruction census of one kernel in a hipcc -save-temps .s file: python3 isa_loops2.py FILE.s SYMBOL_SUBSTR"""
import re
import sys
from collections import Counter

txt = open(sys.argv[1]).read()
name = [m.group(1) for m in re.finditer(r'^(\S+):', txt, re.M) if sys.argv[2] in m.group(1) and not m.group(1).startswith('.')][0]
i = txt.index(name + ':')
j = txt.index('.Lfunc_end', i)
body = txt[i:j].split('\n')
labels = {}
for n, l in enumerate(body):
    m = re.match(r'^(\.LBB\d+_\d+):', l)
    if m:
        labels[m.group(1)] = n
print(name)
for n, l in enumerate(body):
    m = re.search(r's_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)', l)
    if m and m.group(1) in labels and labels[m.group(1)] < n:
        seg = body[labels[m.group(1)]:n]
        ins = [x.strip().split()[0] for x in seg if x.strip() and not x.strip().startswith(('.', ';')) and not x.strip().endswith(':')]
        c = Counter(ins)
        valu = sum(v for k, v in c.items() if k.startswith('v_'))
        print('loop', m.group(1), 'instr', len(ins), 'valu', valu, 'accvgpr', sum(v for k, v in c.items() if 'accvgpr' in k),
              'ds', sum(v for k, v in c.items() if k.startswith('ds_')), 'salu', sum(v for k, v in c.items() if k.startswith('s_')))
        print('   ', c.most_common(14))
