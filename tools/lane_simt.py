"""Diagnostic: SIMT cost model of the lane-per-page LZ4 decoder on the bench pages.

Parses the oracle LZ4 encodings of pagegen pages into (literal, match, offset) sequences and reports
sequences per page, lane utilization of 64-page waves, the per-iteration copy-step units (1 + the
slowest lane's extra 16-byte steps), far-match loads per iteration and far fractions per ring size.
CPU only:  python tools/lane_simt.py
"""
import numpy as np, sys
sys.path.insert(0, '.')
from oracle import oracle as O
def seqs(c):
    ip = 0; out = []; op = 0
    L = len(c)
    while True:
        t = c[ip]; ip += 1
        lit = t >> 4
        if lit == 15:
            while True:
                b = c[ip]; ip += 1; lit += b
                if b != 255: break
        ip += lit
        if ip >= L: out.append((lit, 0, 0, ip)); break
        off = c[ip] | c[ip+1] << 8; ip += 2
        ml = t & 15
        if ml == 15:
            while True:
                b = c[ip]; ip += 1; ml += b
                if b != 255: break
        ml += 4
        out.append((lit, ml, off, ip)); op += lit + ml
    return out
n = 640   # pages (10 waves)
pages = O.pagegen(n, 16384)
S = [seqs(O.lz4_compress(pages[i].tobytes())) for i in range(n)]
ns = np.array([len(s) for s in S])
print("seq/page mean", ns.mean(), "min", ns.min(), "max", ns.max())
# wave rounds: 64 lanes, time = max seq count
W = ns.reshape(-1, 64)
print("lane utilization (sum/ (64*max))", (W.sum(1) / (64 * W.max(1))).mean())
# per-iteration chunk costs: for each wave, iteration j, lanes active -> cost units
for R in (192, 256):
    tot_it = 0; tot_units = 0; tot_far_serial = 0; tot_far_grp = 0; lane_units = 0
    for w in range(W.shape[0]):
        lanes = S[w*64:(w+1)*64]
        m = max(len(l) for l in lanes)
        for j in range(m):
            mx_l = 0; mx_m = 0; mx_far = 0; mx_fg = 0
            for l in lanes:
                if j < len(l):
                    lit, ml, off, _ = l[j]
                    cl = max(0, (lit + 1 + 15) // 16 - 1) if lit > 14 else 0
                    cm = max(0, (ml - 1) // 16) if off >= 16 else 0
                    mx_l = max(mx_l, cl); mx_m = max(mx_m, cm)
                    if off > R - 32:
                        mx_far = max(mx_far, (ml + 15)//16); mx_fg = max(mx_fg, (ml + 63)//64)
                    lane_units += 1 + cl + cm
            tot_it += 1; tot_units += 1 + mx_l + mx_m; tot_far_serial += mx_far; tot_far_grp += mx_fg
    print(f"ring {R}: wave iterations {tot_it}, iteration cost units (1 + max chunk loops) {tot_units/tot_it:.2f}, far load waits/iter serial {tot_far_serial/tot_it:.2f} grouped {tot_far_grp/tot_it:.2f}, balanced units/lane-iter {lane_units/(64*tot_it):.2f}")
allm = [x for s in S for x in s]
ml = np.array([x[1] for x in allm]); off = np.array([x[2] for x in allm]); lit = np.array([x[0] for x in allm])
print("ml>16", (ml>16).mean(), "ml>32", (ml>32).mean(), "ml>64", (ml>64).mean(), "lit>12", (lit>12).mean())
for R in (128,192,256,512,1024):
    print("far frac ring", R, (off > R-32).mean())
