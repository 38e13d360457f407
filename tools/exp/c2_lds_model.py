#!/usr/bin/env python3
# r06: the LDS bank model of firI8MfmaKernel (C2) plane accesses, the r05 layout against the r06 swizzle.
# LDS bank model (MI355X_MICROARCH.md LDS table) of firI8MfmaKernel's plane accesses: split writes
# (ds_write_b128, 8 groups of 8 contiguous lanes, bank (a/4) mod 32) and A-fragment reads (ds_read_b128,
# 4 groups of 16, bank (a/4) mod 64). Extra cycles per instruction = sum over groups of (max distinct
# addresses on one bank - 1).
RG=[[0,1,2,3,12,13,14,15,20,21,22,23,24,25,26,27],[4,5,6,7,8,9,10,11,16,17,18,19,28,29,30,31],
    [32,33,34,35,44,45,46,47,52,53,54,55,56,57,58,59],[36,37,38,39,40,41,42,43,48,49,50,51,60,61,62,63]]
def cost(addrs, groups, nb):
    extra=0
    for g in groups:
        banks={}
        for l in g:
            a=addrs[l]
            for w in range(4):
                banks.setdefault((a//4+w)%nb,set()).add(a//4+w)
        extra+=max(len(v) for v in banks.values())-1
    return extra
def run(unit, P, S=5, nthreads=256, kGroups=None):
    wr=0; nw=0
    G=kGroups
    for u0 in range(0, G, nthreads):
        for wv in range(4):
            addrs={}
            for l in range(64):
                g=u0+wv*64+l
                addrs[l]=16*unit(g>>2,g&3) if g<G else 16*unit(0,0)
            wr+=cost(addrs,[list(range(8*k,8*k+8)) for k in range(8)],32); nw+=1
    rd=0; nr=0
    for tile in range(8):
        for s in range(S):
            for u in range(2):
                addrs={}
                for l in range(64):
                    row=l&31; half=l>>5
                    b0=tile*16+(row&15)
                    addrs[l]=(row>>4)*P+16*unit(b0+s,2*u+half)
                rd+=cost(addrs,RG,64); nr+=1
    return wr/nw, rd/nr
S=5; kWin=8*512+32*S; kGroups=(kWin)//8
blocks=kGroups//4+8
old=lambda b,q:5*b+q
Pold=(80*blocks+255)//256*256
new=lambda b,q:4*b+(q^((b>>2)&3))
Pnew=(64*blocks+255)//256*256
print('old: extra cycles per write, per read', run(old,Pold,S,kGroups=kGroups))
print('new:', run(new,Pnew,S,kGroups=kGroups))
