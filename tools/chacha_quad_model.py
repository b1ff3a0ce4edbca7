"""Lane-level model of the wave-per-packet ChaCha20 keystream by quads (csrc/chacha_wave.h chacha_row_quad and the
pass loop of chacha_wave_packet): DPP quad_perm semantics (lane l reads lane 4 (l / 4) + sel[l % 4]), the column /
diagonal split, the 4 x 4 transpose and the realignment by delta, checked against the RFC 8439 block function for
random AAD / payload lengths (every data block of every pass, and the Poly1305 key block).  Run: python3 tools/chacha_quad_model.py"""
import random
M=0xffffffff
def rotl(x,n): return ((x<<n)|(x>>(32-n)))&M
def qr(a,b,c,d):
    a=(a+b)&M; d^=a; d=rotl(d,16); c=(c+d)&M; b^=c; b=rotl(b,12)
    a=(a+b)&M; d^=a; d=rotl(d,8); c=(c+d)&M; b^=c; b=rotl(b,7)
    return a,b,c,d
C=[0x61707865,0x3320646e,0x79622d32,0x6b206574]
def block(k,ctr,n):
    x=C+k+[ctr]+n; inp=list(x)
    for _ in range(10):
        for (i,j,l,m) in [(0,4,8,12),(1,5,9,13),(2,6,10,14),(3,7,11,15),(0,5,10,15),(1,6,11,12),(2,7,8,13),(3,4,9,14)]:
            x[i],x[j],x[l],x[m]=qr(x[i],x[j],x[l],x[m])
    return [(x[i]+inp[i])&M for i in range(16)]
def perm(vals, sel):  # vals per lane (64), lane l reads 4*(l//4)+sel[l%4]
    return [vals[4*(l//4)+sel[l%4]] for l in range(64)]
R1=[1,2,3,0]; R2=[2,3,0,1]; R3=[3,0,1,2]
def row_quad(k, cbs, n):  # cbs: per lane counter (equal within quad)
    S=[l&3 for l in range(64)]
    a0=[C[s] for s in S]; b0=[k[s] for s in S]; c0=[k[4+s] for s in S]; d0=[[cbs[l],n[0],n[1],n[2]][S[l]] for l in range(64)]
    a,b,c,d=list(a0),list(b0),list(c0),list(d0)
    for _ in range(10):
        for l in range(64): a[l],b[l],c[l],d[l]=qr(a[l],b[l],c[l],d[l])
        b=perm(b,R1); c=perm(c,R2); d=perm(d,R3)
        for l in range(64): a[l],b[l],c[l],d[l]=qr(a[l],b[l],c[l],d[l])
        b=perm(b,R3); c=perm(c,R2); d=perm(d,R1)
    w=[[ (a[l]+a0[l])&M, (b[l]+b0[l])&M, (c[l]+c0[l])&M, (d[l]+d0[l])&M] for l in range(64)]
    r0=[w[l][S[l]] for l in range(64)]
    r1=perm([w[l][(S[l]-1)&3] for l in range(64)],R1)
    r2=perm([w[l][(S[l]-2)&3] for l in range(64)],R2)
    r3=perm([w[l][(S[l]-3)&3] for l in range(64)],R3)
    rs=[r0,r1,r2,r3]
    return [[rs[(t-S[l])&3][l] for t in range(4)] for l in range(64)]
random.seed(1)
k=[random.getrandbits(32) for _ in range(8)]; n=[random.getrandbits(32) for _ in range(3)]
for trial in range(12):
    aad=random.randint(1,80); ln=random.randint(0,3000)
    a=(aad+15)//16; c=(ln+15)//16; m=a+c+1; K=(m+63)//64; pad=64*K-m
    delta=(pad+a)&3
    prev=[[0]*4]*64
    for kk in range(K):
        base_b=64*kk-pad-a+delta
        cbs=[max(1+(base_b>>2)+(l>>2),0) for l in range(64)]
        row=row_quad(k,cbs,n)
        for l in range(64):
            i=l+64*kk-pad
            if a<=i<a+c:
                b=i-a
                src=(l-delta)&63
                kq = row[src] if (delta==0 or l>=delta) else prev[src]
                ref=block(k,1+(b>>2),n)[4*(b&3):4*(b&3)+4]
                assert kq==ref,(trial,kk,l,delta)
        if kk==0:
            j0=-(base_b>>2)-1
            pk = (row[4*j0]+row[4*j0+1]) if 0<=j0<16 else None
            if pk is None:
                r0=row_quad(k,[0]*64,n); pk=r0[0]+r0[1]
            assert pk==block(k,0,n)[:8],(trial,'pk')
        prev=row
    print('ok',aad,ln,K,pad,delta)
