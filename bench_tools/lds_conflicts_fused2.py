#!/usr/bin/env python3
"""lds_conflicts_fused2.py -- bank-conflict model of k_stream_fused2's S/C region accesses (stream_fused2.hpp):
the compute lanes' region read / write (layers 4 c0 + g, G = 3) and the rounds' C reads per target item,
for the plain layout (row of layer z at 64 z) and the round-6 swizzle f2_rz.  Extra LDS cycles per
tile and CU for the BASELINE pattern {0,4,8,12}."""
G64=[list(range(0,32)), list(range(32,64))]           # ds_read_b64 lane groups
W16=[list(range(i,i+16)) for i in range(0,64,16)]     # ds_write_b64 groups (4 x 16 contiguous)
def wt(y): return 1 << (2*(3-y))
def cyc(addrs, groups, width=8):
    tot=0
    for g in groups:
        banks={}
        for l in g:
            if l not in addrs: continue
            a=addrs[l]
            for b in range(a//4, (a+width)//4):
                banks.setdefault(b%64,set()).add(a)
        tot += max((len(v) for v in banks.values()), default=1)-1
    return tot
def rz_plain(z): return z*64
def rz_sw(z): return ((z & ~3) | ((z ^ (z>>2) ^ (z>>4) ^ (z>>6)) & 3))*64
def compute_region(rz):
    # 8 compute waves: lane (c0, p), layers z = 4 c0 + g (G = 3), 16 reads and 16 writes
    ex_r=ex_w=0
    for w in range(8):
        for g in range(4):
            addrs={}
            for l in range(64):
                c0=(w*64+l)>>3; p=l&7
                addrs[l]=rz(4*c0+g)+8*p
            ex_r+=cyc(addrs,G64); ex_w+=cyc(addrs,W16)
    return ex_r*4, ex_w*4   # x 4 rows
def targets(Y, xe, L):
    esec=[1 if xe[y] is not None else 0 for y in range(4)]
    others=[y for y in (3,2,1,0) if y!=Y and esec[y]]
    no=len(others); n4=4-sum(esec)
    res=[]
    subs=[m for m in range(1<<no) if bin(m).count('1')==L-1]
    per=3**(no-(L-1))*4**n4
    for sub in subs:
        for v0 in range(per):
            v=v0; zb=0; o=0
            for yy in (3,2,1,0):
                if yy==Y: continue
                if esec[yy]:
                    if (sub>>o)&1: d=xe[yy]
                    else:
                        u=v%3; v//=3; d=u+(1 if u>=xe[yy] else 0)
                    o+=1
                else:
                    d=v&3; v>>=2
                zb+=d*wt(yy)
            res.append(zb)
    return res
def rounds(rz, xe):
    ex=0; n=0
    for Y in range(4):
        if xe[Y] is None: continue
        for L in range(1,5):
            t=targets(Y,xe,L)
            items=[(ci, d8) for ci in range(len(t)) for d8 in range(8)]
            for i0 in range(0,len(items),64):
                chunk=items[i0:i0+64]
                for X in list(range(4)):
                    addrs={}
                    for l,(ci,d8) in enumerate(chunk):
                        z=t[ci]+X*wt(Y)
                        addrs[l]=rz(z)+8*d8
                    e=cyc(addrs,G64); ex+=e; n+=1
    return ex, n
xe=[0,0,0,0]
print("compute region (read, write) extra cycles / tile / CU: plain", compute_region(rz_plain), "swizzled", compute_region(rz_sw))
print("rounds extra cycles / tile / CU (3 reads + 1 atomic per item pass): plain", rounds(rz_plain,xe), "swizzled", rounds(rz_sw,xe))
