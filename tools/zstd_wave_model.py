"""CPU model of the device zstd block parse as it runs on the GPU
(rcdc_zstd.hip rcdc_zstd_block_kernel, NARROW tables): wave steps of 64
positions, the table read before the step's inserts, the last offsets checked
at every position, the lazy rule, selection in lane order, and the step's
positions inserted afterwards except those inside the matches taken.  The
block coder is tests/zstd_model.py's.  Test infrastructure for exploring
parse variants before building them; not the device path.

  python tools/zstd_wave_model.py [--hl 12] [--kinds csv,code,text] [--kib 512]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import zstd_model as zm  # noqa: E402

M64 = (1 << 64) - 1


def zhash(k, hl):
    return ((k * 0x9E3779B97F4A7C15) & M64) >> (64 - hl)


def parse(blk, hl=12, key=6, repchk=True, rep1=True, insall=False, ins_sel=True, lazy_rep=True,
          phases=1, rep2=False, ins_end=False, rep_longer=False):
    n = len(blk)
    b = np.frombuffer(blk, np.uint8)
    tab = [None] * (1 << hl)
    anchor, base, ilimit = 0, 0, n - 8
    r0 = r1 = r2 = 0
    seqs = []

    def ext(a, c, mx):
        m = 0
        while m < mx and b[a + m] == b[c + m]:
            m += 1
        return m

    def extb(a, c, mx):
        m = 0
        while m < mx and b[a - 1 - m] == b[c - 1 - m]:
            m += 1
        return m

    while base <= ilimit:
        stride = min(1 + ((base - anchor) >> 8), 32)
        P = [base + l * stride for l in range(64)]
        act = [p <= ilimit for p in P]
        C = [None] * 64
        H = [None] * 64
        isrep = [False] * 64
        ok = [False] * 64
        FL = [0] * 64
        BL = [0] * 64
        lp = 64 // phases
        for l in range(64):
            if not act[l]:
                continue
            p = P[l]
            w = blk[p:p + 4]
            k = int.from_bytes(blk[p:p + key], "little")
            H[l] = h = zhash(k, hl)
            if phases > 1 and l % lp == 0 and l:  # the earlier phases' positions are visible
                for q in range(l - lp, l):
                    if act[q]:
                        tab[H[q]] = P[q] & 0xFFFF
            e = tab[h]
            c = None
            if e is not None:
                c = (p & ~0xFFFF) | e
                if c >= p:
                    c = c - 0x10000 if c >= 0x10000 else None
            ct = c
            if ct is not None and blk[ct:ct + 4] != w:
                ct = None
            if repchk and r0 and p >= r0 and blk[p - r0:p - r0 + 4] == w:
                c, isrep[l] = p - r0, True
            elif repchk and rep1 and r1 and p >= r1 and blk[p - r1:p - r1 + 4] == w:
                c, isrep[l] = p - r1, True
            elif repchk and rep2 and r2 and p >= r2 and blk[p - r2:p - r2 + 4] == w:
                c, isrep[l] = p - r2, True
            if rep_longer and isrep[l] and ct is not None:
                # the longer of the table's and the last offset's match
                lt = ext(p + 4, ct + 4, min(16, n - p - 4))
                lr = ext(p + 4, c + 4, min(16, n - p - 4))
                if 4 + lt >= key and lt > lr + 1:
                    c, isrep[l] = ct, False
            C[l] = c
            if c is None:
                continue
            limf = n - p - 4
            fl = ext(p + 4, c + 4, min(16, limf))
            limb = min(p - anchor, c)
            bl = extb(p, c, min(16, limb))
            FL[l], BL[l] = fl, bl
            ok[l] = blk[c:c + 4] == w and (isrep[l] or 4 + fl >= key)
        tgt = list(range(64))
        for l in range(63):
            if stride == 1 and ok[l] and ok[l + 1]:
                if (FL[l] < 16 and FL[l + 1] > FL[l] + 1) or (lazy_rep and isrep[l + 1] and not isrep[l]):
                    tgt[l] = l + 1
        m = [l for l in range(64) if ok[l]]
        sel = set()
        ends = []
        covered = [False] * 64
        while m:
            j = tgt[m[0]]
            f = FL[j]
            pj, cj = P[j], C[j]
            ln = 4 + f
            if f == 16 and n - pj > 20:
                ln += ext(pj + 20, cj + 20, n - pj - 20)
            mb = min(pj - anchor, cj)
            bk = min(BL[j], mb)
            if BL[j] == 16 and mb > 16:
                bk += extb(pj - 16, cj - 16, mb - 16)
            pj, cj, ln = pj - bk, cj - bk, ln + bk
            off, ll = pj - cj, pj - anchor
            seqs.append((ll, ln, off))
            # repeat history as the device keeps it (offsets_to_values' rules)
            if ll:
                if off == r0:
                    pass
                elif off == r1:
                    r0, r1 = off, r0
                elif off == r2:
                    r0, r1, r2 = off, r0, r1
                else:
                    r0, r1, r2 = off, r0, r1
            else:
                if off == r1:
                    r0, r1 = off, r0
                elif off == r2:
                    r0, r1, r2 = off, r0, r1
                else:
                    r0, r1, r2 = off, r0, r1
            sel.add(j)
            for l in range(64):
                if P[l] > pj and P[l] < pj + ln:
                    covered[l] = True
            anchor = pj + ln
            m = [l for l in m if P[l] >= anchor]
            if ins_end and anchor - 2 > pj and anchor - 2 + key <= n:
                q = anchor - 2
                ends.append((zhash(int.from_bytes(blk[q:q + key], "little"), hl), q))
        for l in range(64):
            if act[l] and (insall or not covered[l] or (ins_sel and l in sel)):
                tab[H[l]] = P[l] & 0xFFFF
        for h, q in ends:
            tab[h] = q & 0xFFFF
        base = max(base + 64 * stride, anchor)
    return seqs


def size(data, bs=128 << 10, **kw):
    T = zm.tables()
    tot = 0
    for o in range(0, len(data), bs):
        blk = data[o:o + bs]
        seqs = parse(blk, **kw)
        out = zm.compressed_block_adaptive(T, blk, seqs, reps=True)
        tot += min(len(out), len(blk))
    return tot / len(data)


def kinds(kib):
    rng = np.random.default_rng(1)  # tools/zstd_prof.py's generators
    words = [bytes(rng.integers(97, 123, size=int(rng.integers(2, 9))).astype(np.uint8))
             for _ in range(400)]
    text = b" ".join(words[int(i)] for i in rng.integers(0, 400, kib << 10 >> 2))[:kib << 10]
    csv = b"".join(b"%08d,%s,%d,%s\n" % (i, words[i % 400], (i * 7919) % 100000,
                                         words[(i * 31) % 400]) for i in range(kib * 40))[:kib << 10]
    code = b"".join(b"    x_%d = foo(%s, %d) + bar[%d];\n" % (i % 97, words[i % 50], i,
                                                            (i * 13) % 1000)
                    for i in range(kib * 30))[:kib << 10]
    return {"text": text, "csv": csv, "code": code}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hl", type=int, default=12)
    ap.add_argument("--kinds", default="csv,code,text")
    ap.add_argument("--kib", type=int, default=512)
    ap.add_argument("--variant", default="", help="comma list of k=v parse() options")
    a = ap.parse_args()
    kw = {"hl": a.hl}
    for kv in a.variant.split(","):
        if kv:
            k, v = kv.split("=")
            kw[k] = int(v) if k in ("key", "phases") else bool(int(v))
    d = kinds(a.kib)
    for k in a.kinds.split(","):
        print(k, kw, round(size(d[k], **kw), 4), flush=True)


if __name__ == "__main__":
    main()
