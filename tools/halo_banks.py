"""Bank-conflict check of conv_halo's B-fragment ds_read_b128 reads for the stride-2 column-split halo
(stride-2 forward). Prints, per output width, the layouts (half width, row pitch) whose worst
lane group hits each 16-B bank slot once (cost 1 = conflict-free) for every tap shift and fragment.
usage: python tools/halo_banks.py"""
import itertools
G = [[*range(0,4),*range(12,16),*range(20,28)], [*range(4,12),*range(16,20),*range(28,32)],
     [*range(32,36),*range(44,48),*range(52,60)], [*range(36,44),*range(48,52),*range(60,64)]]
def hswz(r): return ((r>>1)&3)<<1
def cost(rows_of_col, toffs, swz=hswz):
    worst = 1
    for toff in toffs:
        for ks in range(2):
            for grp in G:
                slots = {}
                for l in grp:
                    j = l & 15; g = l >> 4
                    row = rows_of_col[j] + toff
                    chunk = (ks*4 + (g & 1) + 0) ^ swz(row)   # g in 0..3 -> chunk ks*4+g
                    chunk = (ks*4 + g) ^ swz(row)
                    slot = ((row & 1)*8 + chunk) % 16
                    slots.setdefault(slot, set()).add(row*8+chunk)
                worst = max(worst, max(len(v) for v in slots.values()))
    return worst
def s2_rows(Q, P2, HW, perm, frag0=0):
    # output pixel index t (within tile) -> (y, x), halo row base = 2y*P2 + x
    out = []
    for j in range(16):
        t = frag0 + perm[j]
        y, x = divmod(t, Q)
        out.append(2*y*P2 + x)
    return out
def s2_toffs(P2, HW):
    return [r*P2 + (s&1)*HW + (s>>1) for r in range(3) for s in range(3)]
if __name__ == "__main__":
    for Q in (16, 8, 4):
        best = []
        for HW in range(Q+1, Q+9):
            for extra in range(0, 8):
                P2 = 2*HW + extra
                for perm in ([*range(16)],
                             [8,9,10,11,0,1,2,3,4,5,6,7,12,13,14,15],
                             [4,5,6,7,0,1,2,3,8,9,10,11,12,13,14,15],
                             [12,13,14,15,0,1,2,3,4,5,6,7,8,9,10,11]):
                    c = max(cost(s2_rows(Q, P2, HW, perm, f0), s2_toffs(P2, HW)) for f0 in range(0, 64, 16))
                    best.append((c, P2 - 2*HW, HW, P2, perm[:8]))
        best.sort()
        print(Q, best[:4])

def gen_rows(Q, P2, hb, rows, perm, frag0):
    out = []
    for j in range(16):
        t = frag0 + perm[j]
        i, rem = divmod(t, rows*Q)
        y, x = divmod(rem, Q)
        out.append(i*hb + 2*y*P2 + x)
    return out
def check_geom(H, Q, BN):
    # H: output rows per image; choose rows/imgs as conv_halo does
    hw = H*Q
    if hw >= BN: rows, imgs = BN//Q, 1
    else: rows, imgs = H, BN//hw
    res = []
    for HW in range(Q+1, Q+6):
        for extra in (0, 2, 4):
            P2 = 2*HW + extra
            for hpad in range(0, 8):
                hb = (2*rows+1)*P2 + hpad
                c = max(cost(gen_rows(Q, P2, hb, rows, list(range(16)), f0), s2_toffs(P2, HW)) for f0 in range(0, BN, 16))
                res.append((c, (2*rows+1)*P2*imgs + hpad*imgs, HW, P2, hb))
    res.sort()
    return rows, imgs, res[:3]
print("--- identity perm, generic tiles")
for (H, Q, BN) in [(16,16,128),(16,16,256),(8,8,128),(8,8,64),(4,4,128),(4,4,64),(112,112,128),(56,56,128),(28,28,128),(14,14,128),(7,7,49)]:
    try:
        print(H, Q, BN, check_geom(H, Q, BN))
    except Exception as e:
        print(H,Q,BN,"err",e)
