"""CPU model of long-distance candidates for the device zstd parse: the
block parse of tools/zstd_wave_model.py (one wave, 64 positions per step, the
block's own LDS table, last-offset checks, the lazy rule), plus candidates
from earlier blocks of the same blob.  A pre-pass keeps, per block, a table
of 2^FH buckets holding the latest *sampled* position (content-defined: the
position's key hash has its low S bits zero, as zstd's long-distance matcher
samples with a rolling-hash mask), and a sampled position whose own table
misses probes the tables of the D previous blocks.  Blocks stay independent
(a wave per block); a far match needs the frame window, which is the blob
(single-segment frame).  Test infrastructure for exploring the design; not
the device path.

  python tools/zstd_ldm_model.py [--kib 2048] [--blob-kib 1024] [--fh 13] [--s 3] [--d 3]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import zstd_model as zm  # noqa: E402
from zstd_wave_model import kinds, zhash  # noqa: E402

M64 = (1 << 64) - 1
BS = 128 << 10


def far_tables(buf, o, n, key, fh, s):
    """The pre-pass: bucket -> latest sampled absolute position in [o, o+n-8]."""
    t = {}
    for p in range(o, o + n - 7):
        k = int.from_bytes(buf[p:p + key], "little")
        hv = (k * 0x9E3779B97F4A7C15) & M64
        if (hv >> 20) & ((1 << s) - 1):
            continue
        t[hv >> (64 - fh)] = p
    return t


def parse(buf, o, n, hl=12, key=6, fars=(), fh=13, s=3, lazy_rep=True, far_first=False, hints=(), fmap=None, mapg=4):
    """Sequences (ll, ml, offset) of the block [o, o+n) of buf; offsets may
    reach before o (into the blob's earlier blocks) through `fars`."""
    tab = [None] * (1 << hl)
    anchor, base, ilimit = o, o, o + n - 8
    end = o + n
    r0 = r1 = r2 = 0
    seqs = []
    nfar = 0

    def ext(a, c, mx):
        m = 0
        while m < mx and buf[a + m] == buf[c + m]:
            m += 1
        return m

    def extb(a, c, mx):
        m = 0
        while m < mx and buf[a - 1 - m] == buf[c - 1 - m]:
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
        for l in range(64):
            if not act[l]:
                continue
            p = P[l]
            w = buf[p:p + 4]
            k = int.from_bytes(buf[p:p + key], "little")
            H[l] = h = zhash(k, hl)
            e = tab[h]
            c = None
            if e is not None:
                rp = p - o
                cr = (rp & ~0xFFFF) | e
                if cr >= rp:
                    cr = cr - 0x10000 if cr >= 0x10000 else None
                c = None if cr is None else o + cr
            ct = c
            if ct is not None and buf[ct:ct + 4] != w:
                ct = c = None
            if ct is not None and 4 + ext(p + 4, ct + 4, min(16, end - p - 4)) < key:
                ct = c = None
            if fmap is not None and ct is None:
                off = fmap.get((p - o) >> mapg)
                if off and p - off >= 0 and buf[p - off:p - off + 4] == w and \
                        4 + ext(p + 4, p - off + 4, min(16, end - p - 4)) >= key:
                    c = p - off
            if fars and stride == 1 and (ct is None or far_first):
                hv = (k * 0x9E3779B97F4A7C15) & M64
                if not (hv >> 20) & ((1 << s) - 1):
                    fb = hv >> (64 - fh)
                    for t in fars:
                        q = t.get(fb)
                        if q is not None and buf[q:q + 4] == w and \
                                4 + ext(p + 4, q + 4, min(16, end - p - 4)) >= key:
                            if ct is None or ext(p, q, min(64, end - p)) > ext(p, ct, min(64, end - p)):
                                c = q
                            break
            if r0 and p - r0 >= 0 and buf[p - r0:p - r0 + 4] == w and p - r0 >= anchor - (1 << 30):
                c, isrep[l] = p - r0, True
            elif r1 and p >= r1 and buf[p - r1:p - r1 + 4] == w:
                c, isrep[l] = p - r1, True
            elif r2 and p >= r2 and buf[p - r2:p - r2 + 4] == w:
                c, isrep[l] = p - r2, True
            if c is None or (not isrep[l] and c == ct and ct is None):
                for hh in hints:
                    if p - hh >= 0 and buf[p - hh:p - hh + 4] == w and \
                            4 + ext(p + 4, p - hh + 4, min(16, end - p - 4)) >= key:
                        c = p - hh
                        break
            C[l] = c
            if c is None:
                continue
            fl = ext(p + 4, c + 4, min(16, end - p - 4))
            limb = min(p - anchor, 16)
            bl = extb(p, c, limb)
            FL[l], BL[l] = fl, bl
            ok[l] = buf[c:c + 4] == w and (isrep[l] or 4 + fl >= key)
        tgt = list(range(64))
        for l in range(63):
            if stride == 1 and ok[l] and ok[l + 1]:
                if (FL[l] < 16 and FL[l + 1] > FL[l] + 1) or (lazy_rep and isrep[l + 1] and not isrep[l]):
                    tgt[l] = l + 1
        m = [l for l in range(64) if ok[l]]
        sel = set()
        covered = [False] * 64
        while m:
            j = tgt[m[0]]
            f = FL[j]
            pj, cj = P[j], C[j]
            ln = 4 + f
            if f == 16 and end - pj > 20:
                ln += ext(pj + 20, cj + 20, end - pj - 20)
            mb = pj - anchor
            bk = min(BL[j], mb)
            if BL[j] == 16 and mb > 16:
                bk += extb(pj - 16, cj - 16, mb - 16)
            pj, cj, ln = pj - bk, cj - bk, ln + bk
            off, ll = pj - cj, pj - anchor
            if cj < o:
                nfar += 1
            seqs.append((ll, ln, off))
            if off != r0:
                if off == r1:
                    r0, r1 = off, r0
                else:
                    r0, r1, r2 = off, r0, r1
            sel.add(j)
            for l in range(64):
                if P[l] > pj and P[l] < pj + ln:
                    covered[l] = True
            anchor = pj + ln
            m = [l for l in m if P[l] >= anchor]
        for l in range(64):
            if act[l] and (not covered[l] or l in sel):
                tab[H[l]] = (P[l] - o) & 0xFFFF
        base = max(base + 64 * stride, anchor)
    return seqs, nfar


def block_hints(buf, o, n, tabs, key, fh, s, k, minlen=8):
    """Phase 2: the top-k offsets by matched bytes of the sampled positions of
    [o, o+n) found in the earlier blocks' tables."""
    from collections import Counter
    cnt = Counter()
    end = o + n
    for p in range(o, o + n - 7):
        kk = int.from_bytes(buf[p:p + key], "little")
        hv = (kk * 0x9E3779B97F4A7C15) & M64
        if (hv >> 20) & ((1 << s) - 1):
            continue
        fb = hv >> (64 - fh)
        for t in tabs:
            q = t.get(fb)
            if q is None:
                continue
            m = 0
            while m < 64 and p + m < end and buf[p + m] == buf[q + m]:
                m += 1
            if m >= minlen:
                cnt[p - q] += m
                break
    return [off for off, _ in cnt.most_common(k)]


def block_map(buf, o, n, tabs, key, fh, s, mapg):
    """Phase 2 as a map: per 2^mapg-byte group of [o, o+n), the offset of a
    sampled position's verified candidate in the earlier blocks' tables."""
    fm = {}
    end = o + n
    for p in range(o, o + n - 7):
        kk = int.from_bytes(buf[p:p + key], "little")
        hv = (kk * 0x9E3779B97F4A7C15) & M64
        if (hv >> 20) & ((1 << s) - 1):
            continue
        fb = hv >> (64 - fh)
        for t in tabs:
            q = t.get(fb)
            if q is not None and buf[q:q + 4] == buf[p:p + 4] and \
                    4 + sum(1 for _ in iter(lambda m=[0]: (m.__setitem__(0, m[0] + 1) or m[0]) <= min(16, end - p - 4) and buf[p + 3 + m[0]] == buf[q + 3 + m[0]], False)) >= key:
                fm[(p - o) >> mapg] = p - q
                break
    return fm


def size(data, blob, fh, s, d, key=6, hl=12, far_first=False, hint_k=0, mapg=0):
    T = zm.tables()
    tot = nfar = 0
    for bo in range(0, len(data), blob):
        buf = data[bo:bo + blob]
        tabs = []
        for o in range(0, len(buf), BS):
            n = min(BS, len(buf) - o)
            fars = tabs[::-1][:d] if d else ()
            hints = ()
            fmap = None
            if mapg:
                fmap, fars = block_map(buf, o, n, fars, key, fh, s, mapg), ()
            if hint_k:
                hints, fars = block_hints(buf, o, n, fars, key, fh, s, hint_k), ()
            seqs, nf = parse(buf, o, n, hl=hl, key=key, fars=fars, fh=fh, s=s, far_first=far_first,
                             hints=hints, fmap=fmap, mapg=mapg or 4)
            nfar += nf
            out = zm.compressed_block_adaptive(T, buf[o:o + n], seqs, reps=True)
            tot += min(len(out), n)
            if d:
                tabs.append(far_tables(buf, o, n, key, fh, s))
    return tot / len(data), nfar


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kib", type=int, default=2048)
    ap.add_argument("--blob-kib", type=int, default=1024)
    ap.add_argument("--fh", type=int, default=13)
    ap.add_argument("--s", type=int, default=3)
    ap.add_argument("--d", type=int, default=3)
    ap.add_argument("--key", type=int, default=6)
    ap.add_argument("--far-first", action="store_true")
    ap.add_argument("--map", type=int, default=0, help="phase-2 map of 2^MAP-byte groups")
    ap.add_argument("--hints", type=int, default=0, help="phase-2 hint offsets instead of probes")
    ap.add_argument("--kinds", default="csv,code,text")
    a = ap.parse_args()
    dk = kinds(a.kib)
    for k in a.kinds.split(","):
        r, nf = size(dk[k], a.blob_kib << 10, a.fh, a.s, a.d, key=a.key, far_first=a.far_first,
                     hint_k=a.hints, mapg=a.map)
        print(k, vars(a), round(r, 4), "far matches", nf, flush=True)


if __name__ == "__main__":
    main()
