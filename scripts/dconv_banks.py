# Search of the XOR swizzles of conv_direct.h: every tap of every fragment
# read of a v_mfma_f32_32x32x16_bf16 A operand from the halo patch must be
# conflict-free under the ds_read_b128 lane grouping (4 LDS cycles).
import itertools
G = [list(range(0,4))+list(range(12,16))+list(range(20,28)),
     list(range(4,12))+list(range(16,20))+list(range(28,32))]
G += [[l+32 for l in g] for g in G]
def cycles(addr):
    tot = 0
    for g in G:
        cnt = {}
        for l in g:
            s = (addr[l] // 16) % 16
            cnt[s] = cnt.get(s, 0) + 1
        tot += max(cnt.values())
    return tot
def conv_lanes(OW, R, ky, kx, pb):
    out=[]
    for l in range(64):
        q = pb + (l & 31); oy, ox = q // OW, q % OW
        y = 2*oy + ky; ixp = 2*ox + kx
        x = ixp//2 if ixp % 2 == 0 else (OW+1) + (ixp-1)//2
        out.append((y, x, l >> 5))
    return out
def tconv_lanes(WA, R, ty, tx, pb):
    out=[]
    for l in range(64):
        q = pb + (l & 31); a, b = q // WA, q % WA
        out.append((a + ty, b + tx, l >> 5))   # ty,tx in 0..2 (row/col offsets incl ea/eb)
    return out
def worst(CA, PCp, f, lanes_fn, geo, R, taps, nfr):
    P = 2*CA; nch = CA//8; w = 0
    for (ty, tx) in taps:
        for fr in range(nfr):
            for c0 in range(0, nch, 2):
                L = lanes_fn(geo, R, ty, tx, 32*fr)
                addr = [((y*PCp + x)*P + 16*((c0+g) ^ f(y, x)) ) for (y, x, g) in L]
                w = max(w, cycles(addr))
    return w
def search(name, CA, geo, R, mode):
    nch = CA//8
    if mode == 'conv':
        PC = 2*geo + 2; taps = [(ky, kx) for ky in range(4) for kx in range(4)]; fn = conv_lanes; M = R*geo
    else:
        PC = geo + 2; taps = [(ty, tx) for ty in range(3) for tx in range(3)]; fn = tconv_lanes; M = R*geo
    nfr = M // 32
    best = None
    for PCp in range(PC, PC + 17):
        for al in range(0, 16):
            for be in range(0, 3):
                for m in (1, 3, 7, 15):
                    if m >= nch: continue
                    f = lambda y, x, al=al, be=be, m=m: ((x + al*y) >> be) & m
                    w = worst(CA, PCp, f, fn, geo, R, taps, nfr)
                    cand = (w, PCp - PC, al, be, m)
                    if best is None or cand < best: best = cand
                    if w == 4 and PCp == PC: break
    print(name, "CA", CA, "geo", geo, "R", R, "->", best)
search("S1 conv", 32, 32, 4, 'conv')
search("S2 conv", 64, 16, 8, 'conv')
search("S3 conv", 128, 8, 8, 'conv')
search("T1 tconv", 256, 8, 8, 'tconv')
search("T2 tconv", 128, 16, 4, 'tconv')
search("T3 tconv", 64, 32, 2, 'tconv')
