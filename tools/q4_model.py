# python model of AesQ4 (device_common.h) to check the lane convention
import os
SBOX=[0]*256
p=q=1
# generate sbox
def rotl8(x,s): return ((x<<s)|(x>>(8-s)))&0xff
while True:
    p = p ^ ((p<<1)&0xff) ^ (0x1b if p&0x80 else 0)
    q ^= q<<1; q ^= q<<2; q ^= q<<4; q &= 0xff
    if q & 0x80: q ^= 0x09
    SBOX[p] = q ^ rotl8(q,1) ^ rotl8(q,2) ^ rotl8(q,3) ^ rotl8(q,4) ^ 0x63
    if p == 1: break
SBOX[0]=0x63
def xt(s): return ((s<<1) ^ (0x1b if s&0x80 else 0)) & 0xff
M=0xffffffff
def rotl(x,n): n%=32; return ((x<<n)|(x>>(32-n)))&M if n else x
T0=[ (xt(s)) | (s<<8) | (s<<16) | ((xt(s)^s)<<24) for s in SBOX]
lds={}
for x in range(256):
    for slot in range(32):
        m=slot>>3
        lds[65536+256*x+4*slot]=rotl(T0[x],8*m)
def perm(src0,src1,sel):
    b=[(src1>>(8*i))&0xff for i in range(4)]+[(src0>>(8*i))&0xff for i in range(4)]
    out=0
    for i in range(4):
        s=(sel>>(8*i))&0xff
        if s<8: v=b[s]
        elif s==12: v=0
        elif s>=13: v=0xff
        else: raise Exception('sign sel')
        out|=v<<(8*i)
    return out
def alignbit(a,b,s): return (((a<<32)|b)>>(s&31))&M
class Q4:
    def __init__(s,tid):
        l=tid&7; q=(tid>>3)&3; s.q=q
        s.lw=0
        for m in range(4): s.lw|=(4+32*m+4*l)<<(8*m)
        s.sel=[0x0c0c0000|((4+((k+q)&3))<<8)|((k+q)&3) for k in range(4)]
        s.selx=0x0c0c0400|((3+q)&3)
        s.sh=(32-8*q)&31
        s.flo=0x0c0c0000|((4+((2+q)&3))<<8)|((1+q)&3)
        s.fhi=((4+q)<<24)|(((3+q)&3)<<16)|0x0c0c
    def rot(s,x): return alignbit(x,x,s.sh)
    def look(s,K,w):
        a=(perm(w,s.lw,s.sel[K])+65532)
        return lds[a]
    def lookx(s,w): return lds[perm(w,s.lw,s.selx)+65532]
    def col(s,a,b,c,d,kr): return s.look(0,a)^s.look(1,b)^s.look(2,c)^s.look(3,d)^kr
    def fin(s,l0,l1,l2,l3,k): return perm(l1,l0,s.flo)^perm(l3,l2,s.fhi)^k
    def last(s,a,b,c,d,k): return s.fin(s.look(0,a),s.look(1,b),s.look(2,c),s.look(3,d),k)
    def encrypt(s,inp,rk,NR):
        st=[s.rot(inp[i]^rk[i]) for i in range(4)]
        for r in range(1,NR):
            kr=[s.rot(rk[4*r+c]) for c in range(4)]
            st=[s.col(st[c],st[(c+1)%4],st[(c+2)%4],st[(c+3)%4],kr[c]) for c in range(4)]
        k=rk[4*NR:]
        return [s.last(st[c],st[(c+1)%4],st[(c+2)%4],st[(c+3)%4],k[c]) for c in range(4)]
# natural reference AES via T-tables (little-endian words: byte i of word = state byte 4c+i)
def aes_ref(inp,rk,NR):
    st=[inp[i]^rk[i] for i in range(4)]
    for r in range(1,NR):
        st=[T0[st[c]&0xff]^rotl(T0[(st[(c+1)%4]>>8)&0xff],8)^rotl(T0[(st[(c+2)%4]>>16)&0xff],16)^rotl(T0[(st[(c+3)%4]>>24)&0xff],24)^rk[4*r+c] for c in range(4)]
    return [ (SBOX[st[c]&0xff] | (SBOX[(st[(c+1)%4]>>8)&0xff]<<8) | (SBOX[(st[(c+2)%4]>>16)&0xff]<<16) | (SBOX[(st[(c+3)%4]>>24)&0xff]<<24)) ^ rk[4*NR+c] for c in range(4)]
def expand128(key):
    w=[int.from_bytes(key[4*i:4*i+4],'little') for i in range(4)]
    rcon=1
    for i in range(4,44):
        t=w[i-1]
        if i%4==0:
            t=rotl(t,24)  # RotWord on little-endian word = rotr 8
            t=SBOX[t&0xff]|(SBOX[(t>>8)&0xff]<<8)|(SBOX[(t>>16)&0xff]<<16)|(SBOX[t>>24]<<24)
            t^=rcon; rcon=xt(rcon)
        w.append(w[i-4]^t)
    return w
key=bytes.fromhex('000102030405060708090a0b0c0d0e0f'); pt=bytes.fromhex('00112233445566778899aabbccddeeff')
rk=expand128(key)
inp=[int.from_bytes(pt[4*i:4*i+4],'little') for i in range(4)]
ref=aes_ref(inp,rk,10)
print('ref', b''.join(x.to_bytes(4,'little') for x in ref).hex(), '(FIPS-197: 69c4e0d86a7b0430d8cdb78070b4c55a)')
for tid in range(32):
    a=Q4(tid); out=a.encrypt(inp,rk,10)
    if out!=ref: print('lane',tid,'q',a.q,'BAD',b''.join(x.to_bytes(4,'little') for x in out).hex())
print('encrypt lanes checked')
import random
def bswap(x): return int.from_bytes(x.to_bytes(4,'little'),'big')
class Page:
    def build(s,a,rk,n0,n1,n2,pg):
        s0=a.rot(n0^rk[0]); s1=a.rot(n1^rk[1]); s2=a.rot(n2^rk[2]); s3=a.rot(bswap((pg<<8)&M)^rk[3])
        s.k0=a.look(0,s0)^a.look(1,s1)^a.look(2,s2)^a.rot(rk[4])
        s.k1=a.col(s1,s2,s3,s0,a.rot(rk[5])); s.k2=a.col(s2,s3,s0,s1,a.rot(rk[6])); s.k3=a.col(s3,s0,s1,s2,a.rot(rk[7]))
        k1,k2,k3=s.k1,s.k2,s.k3
        s.l0=a.look(1,k1)^a.look(2,k2)^a.look(3,k3)^a.rot(rk[8])
        s.l1=a.look(0,k1)^a.look(1,k2)^a.look(2,k3)^a.rot(rk[9])
        s.l2=a.look(0,k2)^a.look(1,k3)^a.look(3,k1)^a.rot(rk[10])
        s.l3=a.look(0,k3)^a.look(2,k1)^a.look(3,k2)^a.rot(rk[11])
        s.x3=rk[3]>>24
    def two(s,a,c):
        u0=s.k0^a.lookx(c^s.x3)
        return [s.l0^a.look(0,u0), s.l1^a.look(3,u0), s.l2^a.look(2,u0), s.l3^a.look(1,u0)]
def ks_q4(a,pg,rk,c,NR):
    st=pg.two(a,c)
    for r in range(3,NR):
        kr=[a.rot(rk[4*r+i]) for i in range(4)]
        st=[a.col(st[cc],st[(cc+1)%4],st[(cc+2)%4],st[(cc+3)%4],kr[cc]) for cc in range(4)]
    k=rk[4*NR:]
    return [a.last(st[cc],st[(cc+1)%4],st[(cc+2)%4],st[(cc+3)%4],k[cc]) for cc in range(4)]
random.seed(1)
for trial in range(3):
    key=bytes(random.randrange(256) for _ in range(16)); rk=expand128(key)
    n=[random.getrandbits(32) for _ in range(3)]
    for tid in [0,5,9,17,26,31]:
        a=Q4(tid); pg=Page()
        for page in [0,3]:
            pg.build(a,rk,n[0],n[1],n[2],page)
            for c in [page*256+1, page*256+77, page*256+255]:
                want=aes_ref([n[0],n[1],n[2],bswap(c)],rk,10)
                got=ks_q4(a,pg,rk,c,10)
                assert got==want,(tid,c)
print('ctr page ok')
