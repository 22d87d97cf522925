"""LDS bank model of the split exchanges of hsfft_pass_r8.h's r8::exchange (measurement aid):
ds_write_b64 as 4 groups of 16 lanes over 32 banks, ds_read_b64 as 2 groups of 32 lanes over 64
banks; prints cycles per store / load instruction for the first passes' exchanges with the
identity slot map, padding variants and one-bit XOR swizzles.  Round 3 (third session): the
model's best swizzle for the second exchange (8 -> 4 cycles per store) was built bit-exact and
measured 4 % SLOWER on c2 and c5 (profiles/r03c_*_sw2_ab*.txt) -- the model does not predict time.
"""
# LDS bank model of the split exchanges (ds_write_b64: 4 groups of 16 lanes over 32 banks;
# ds_read_b64: 2 groups of 32 lanes over 64 banks), as described in hsfft_pass_r8.h
from collections import defaultdict
def cycles(addrs, lanes_per, nbanks):
    tot = 0
    for g0 in range(0, 64, lanes_per):
        banks = defaultdict(set)
        for a in addrs[g0:g0+lanes_per]:
            if a is None: continue
            for d in (2*a, 2*a+1):
                banks[d % nbanks].add(d)
        tot += max((len(s) for s in banks.values()), default=0)
    return tot
def exch(P, TPG, G, R, LLOC, R2, slot, waves=None):
    NB, NB2, L2 = 8//R, 8//R2, LLOC*R
    S2 = P // (L2*R2)
    nthr = TPG*G
    wc = rc = 0; nw = nr = 0
    for w in range(nthr//64):
        tids = range(w*64, w*64+64)
        for c in range(NB):
            for jj in range(R):
                ad = []
                for t in tids:
                    g, jt = t % G, t // G
                    b = c*TPG + jt; kloc = b & (LLOC-1); ml = b // LLOC
                    ad.append(slot(ml*LLOC*R + kloc + jj*LLOC)*G + g)
                wc += cycles(ad, 16, 32); nw += 1
        for c in range(NB2):
            for i in range(R2):
                ad = []
                for t in tids:
                    g, jt = t % G, t // G
                    b = c*TPG + jt; kloc = b & (L2-1); ml = b // L2
                    ad.append(slot((ml + i*S2)*L2 + kloc)*G + g)
                rc += cycles(ad, 32, 64); nr += 1
    return wc/nw, rc/nr
ident = lambda p: p
for name, P, TPG, G, shapes in [("c2 pass A <4,3,2>", 2048, 256, 2, [(4,1,8),(8,4,8),(8,32,8)]),
                                 ("c5 pass A <8,3,1>", 4096, 512, 1, [(8,1,8),(8,8,8),(8,64,8)])]:
    for (R, LLOC, R2) in shapes:
        print(name, f"R={R} LLOC={LLOC}", "identity: write %.2f read %.2f cycles/instr" % exch(P, TPG, G, R, LLOC, R2, ident))
        for sh in (5, 4, 3, 6):
            pad = lambda p, sh=sh: p + (p >> sh)
            print("    pad 1 per %d: write %.2f read %.2f" % ((1 << sh,) + exch(P, TPG, G, R, LLOC, R2, pad)))
print("---- XOR one bit: p ^ (((p >> s) & 1) << t)")
for name, P, TPG, G, (R, LLOC, R2) in [("c2 A exch2", 2048, 256, 2, (8,4,8)), ("c2 A exch3", 2048, 256, 2, (8,32,8)),
                                       ("c5 A exch2", 4096, 512, 1, (8,8,8)), ("c5 A exch3", 4096, 512, 1, (8,64,8))]:
    best = []
    for s in range(3, 11):
        for t in range(0, 6):
            f = lambda p, s=s, t=t: p ^ (((p >> s) & 1) << t)
            w, r = exch(P, TPG, G, R, LLOC, R2, f)
            best.append((w + r, w, r, s, t))
    best.sort()
    print(name, "identity", exch(P, TPG, G, R, LLOC, R2, ident), "best", best[:4])
print("---- walk2 lo tile (split, P=512, G=8)")
for (R, LLOC, R2) in [(8,1,8),(8,8,8)]:
    print((R,LLOC,R2), "identity", exch(512, 64, 8, R, LLOC, R2, ident))
print("---- existing LLOC==1 swizzle")
def cur(R, G):
    lg = {1:0,2:1,4:2,8:3}[G]; k = R.bit_length()-1; s = max(4-lg, k)
    return lambda p: p ^ (((p >> s) & ((1<<k)-1)))
for name, P, TPG, G, R in [("c2 A", 2048, 256, 2, 4), ("c5 A", 4096, 512, 1, 8), ("walk2 lo", 512, 64, 8, 8)]:
    print(name, exch(P, TPG, G, R, 1, 8, cur(R, G)))
