"""Diagnostic: SIMT / memory model of the quad-per-page chunked LZ4 decoder (lz4_decode_quad.hip,
DESIGN.md 3.1e) on the bench pages, next to the lane-per-page model of tools/lane_simt.py.

Parses the oracle LZ4 encodings of pagegen pages into sequences, replays the kernel's chunking rules
(kQN records, kQF far entries, an output budget of H - 192 bytes, breakers for long far matches and
oversize fields) for each ring size H, and reports per 16 KiB page: chunks, breakers, far entries
(64-byte HBM requests), line writes, stream windows; and per 16-page wave: the SIMT iteration counts
of stage 1 (parse) and stage 3 (copy steps), i.e. the max over the wave's 16 pages per chunk.  The
last column turns those counts into ms per 1M pages with per-iteration costs (cycles) given on the
command line, calibrated against a measured run.

CPU only:  python tools/quad_model.py [pages] [c_parse] [c_step] [c_chunk] [waves_per_cu]
"""
import sys

import numpy as np

sys.path.insert(0, '.')
from oracle import oracle as O  # noqa: E402


def seqs(c):
    """(lit, ml, off) per sequence (ml = 0: the terminal literal run) of an LZ4 block."""
    ip, out, L = 0, [], len(c)
    while True:
        t = c[ip]
        ip += 1
        lit = t >> 4
        if lit == 15:
            while True:
                b = c[ip]
                ip += 1
                lit += b
                if b != 255:
                    break
        ip += lit
        if ip >= L:
            out.append((lit, 0, 0))
            break
        off = c[ip] | c[ip + 1] << 8
        ip += 2
        ml = t & 15
        if ml == 15:
            while True:
                b = c[ip]
                ip += 1
                ml += b
                if b != 255:
                    break
        out.append((lit, ml + 4, off))
    return out


def steps(d, n):
    """copy steps of <= 32 bytes (qword-aligned: 32 - (d & 7)) for n bytes from output position d"""
    k = 0
    while n > 0:
        s = min(n, 32 - (d & 7))
        d += s
        n -= s
        k += 1
    return k, d


def chunks(S, H, N=32, F=8, far_max_ml=42):
    """per page: list of chunks, each (records, far entries, copy steps); breakers counted apart"""
    budget, far_off = H - 192, H - 32
    out, i, d, brk = [], 0, 0, 0
    while i < len(S):
        nrec = nfar = st = 0
        d0 = d
        while i < len(S) and nrec < N:
            lit, ml, off = S[i]
            far = ml > 0 and off > far_off
            fits = lit <= 255 and ml <= 258 and (d + lit + ml - d0) <= budget and not (far and (ml > far_max_ml or nfar == F))
            if not fits:
                if nrec == 0:   # breaker: the slow path takes this one sequence
                    brk += 1
                    d += lit + ml
                    i += 1
                break
            k1, d = steps(d, lit)
            k2, d = steps(d, ml)
            st += k1 + k2
            nfar += far
            nrec += 1
            i += 1
        if nrec:
            out.append((nrec, nfar, st))
    return out, brk


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 640
    c_parse = float(sys.argv[2]) if len(sys.argv) > 2 else 220.0   # cycles per stage-1 wave iteration
    c_step = float(sys.argv[3]) if len(sys.argv) > 3 else 180.0    # cycles per stage-3 copy step
    c_chunk = float(sys.argv[4]) if len(sys.argv) > 4 else 2500.0  # fixed cycles per chunk (stage 2 wait, flush)
    wpc = float(sys.argv[5]) if len(sys.argv) > 5 else 5.0          # resident waves per CU
    pages = O.pagegen(n, 16384)
    S = [seqs(O.lz4_compress(pages[i].tobytes())) for i in range(n)]
    print(f"{n} pages, {np.mean([len(s) for s in S]):.1f} sequences per page")
    for H, F in ((512, 6), (512, 8), (1024, 6), (1024, 8), (2048, 8)):
        per = [chunks(s, H, F=F) for s in S]
        nch = np.array([len(c) for c, _ in per])
        brk = np.array([b for _, b in per])
        far = np.array([sum(x[1] for x in c) for c, _ in per])
        # 16-page waves: chunk k of the wave's pages run together; SIMT cost = max over the 16 pages
        it_parse = it_step = n_chunks = 0
        for w in range(0, n - 15, 16):
            wc = [per[p][0] for p in range(w, w + 16)]
            m = max(len(c) for c in wc)
            for k in range(m):
                recs = [c[k][0] if k < len(c) else 0 for c in wc]
                stp = [c[k][2] if k < len(c) else 0 for c in wc]
                it_parse += max(recs)
                it_step += max(stp)
                n_chunks += 1
        waves = n // 16
        lds = 16 * (H + 288 + 32 * 4 + F * 4 + F * 64)
        wcu = min(wpc, (160 * 1024) // lds)
        cyc = (it_parse * c_parse + it_step * c_step + n_chunks * c_chunk) / waves   # per wave of 16 pages
        # waves of 16 pages per CU over 1M pages; wcu of them in flight, latency-bound (no issue limit)
        ms = cyc * ((1 << 20) / 16 / 256 / wcu) / 2.1e9 * 1e3
        print(f"H {H:5d} F {F}: LDS/wave {lds / 1024:5.1f} KiB ({int((160 * 1024) // lds)} waves/CU); per page: "
              f"chunks {nch.mean():5.1f}, breakers {brk.mean():4.2f}, far entries {far.mean():6.1f} "
              f"({far.mean() / len(S[0]) * 100:4.1f} % of sequences), 64-B line writes 256; per wave chunk: "
              f"parse iterations {it_parse / n_chunks:5.1f}, copy steps {it_step / n_chunks:5.1f}; "
              f"model {ms:6.2f} ms / 1M pages at {wcu:.0f} waves/CU")


if __name__ == "__main__":
    main()
