import re,sys
from collections import defaultdict
s=open(sys.argv[1]).read().split('\n')
starts=[i for i,l in enumerate(s) if re.match(r'_Z\w+:',l)]
starts.append(len(s))
for a,b in zip(starts,starts[1:]):
    lines=s[a:b]; name=lines[0].split(':')[0]
    cur=None; cnt=defaultdict(list)
    for i,l in enumerate(lines):
        if re.match(r'(\.LBB\d+_\d+:|; %bb\.\d+:)',l):
            ctx=l+' '+(lines[i+1] if i+1<len(lines) else '')
            m=re.search(r'\.LBB(\d+_\d+):.*Loop Header: Depth=1',l)
            if m: cur='BB'+m.group(1)
            else:
                m=re.search(r'Header=(BB\d+_\d+) Depth=',ctx)
                cur=m.group(1) if m else None
                # nested headers: depth>1 headers keep outer via their comment
                if not m and 'Loop Header: Depth=' in l:
                    m2=re.search(r'Header=(BB\d+_\d+) Depth=1',ctx); cur=m2.group(1) if m2 else cur
            continue
        if cur and l.startswith('\t') and not l.strip().startswith((';','.')):
            cnt[cur].append(l.split()[0])
    if not cnt: print(name[:50],'no loop'); continue
    h=max(cnt,key=lambda k:len(cnt[k])); ins=cnt[h]
    c=lambda p: sum(1 for x in ins if x==p)
    print("%-52s valu %4d b32 %4d b128 %3d waitcnt %3d salu %3d smem %2d scratch %d" % (name[:52], sum(1 for x in ins if x.startswith('v_')), c('ds_read_b32'), c('ds_read_b128'), c('s_waitcnt'), sum(1 for x in ins if x.startswith('s_') and x not in('s_waitcnt','s_nop')), sum(1 for x in ins if x.startswith('s_load')), sum(1 for x in ins if 'scratch' in x)))
