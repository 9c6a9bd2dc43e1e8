"""A sequential Python model of the device block encoder (rcdc_zstd.hip) --
test infrastructure.  It codes given sequences with the library's own FSE
tables (rcdc_zstd_tables) exactly as rcdc_zstd_block_kernel's lane 0 does,
so the CPU suite checks the tables, the bitstream order and the section
headers against a standard decoder (oracle/zstd_ref.py) without a GPU.
"""
from __future__ import annotations

import ctypes

import numpy as np

TABLES_DTYPE = np.dtype([
    ("ll", [("find", "<i4"), ("nbits", "<u4")], (36,)),
    ("ml", [("find", "<i4"), ("nbits", "<u4")], (53,)),
    ("of", [("find", "<i4"), ("nbits", "<u4")], (32,)),
    ("llst", "<u2", (64,)), ("mlst", "<u2", (64,)), ("ofst", "<u2", (32,)),
    ("llcode", "u1", (64,)), ("mlcode", "u1", (128,)),
    ("llbits", "u1", (36,)), ("mlbits", "u1", (53,)), ("pad", "u1", (3,)),
])


def tables():
    from rustic_core_amd import _lib
    L = _lib.lib()
    n = L.rcdc_zstd_tables_size()
    assert n == TABLES_DTYPE.itemsize, (n, TABLES_DTYPE.itemsize)
    buf = ctypes.create_string_buffer(n)
    L.rcdc_zstd_tables(buf)
    return np.frombuffer(buf.raw, dtype=TABLES_DTYPE)[0]


class BitWriter:
    def __init__(self):
        self.acc = 0
        self.nb = 0
        self.out = bytearray()

    def add(self, v, bits):
        self.acc |= (int(v) & ((1 << int(bits)) - 1)) << self.nb
        self.nb += int(bits)

    def flush(self):
        while self.nb >= 8:
            self.out.append(self.acc & 0xFF)
            self.acc >>= 8
            self.nb -= 8


def _codes(T, ll, ml, off, is_value=False):
    mlb, ofv = ml - 3, (off if is_value else off + 3)
    llc = int(T["llcode"][ll]) if ll < 64 else ll.bit_length() - 1 + 19
    mlc = int(T["mlcode"][mlb]) if mlb < 128 else mlb.bit_length() - 1 + 36
    return llc, mlc, ofv.bit_length() - 1, mlb, ofv


def encode_sequences(T, seqs):
    """FSE bitstream of [(ll, ml, off)] (ZSTD_encodeSequences order)."""
    w = BitWriter()

    def init(tt, st, sym):
        find, nbits = int(tt[sym]["find"]), int(tt[sym]["nbits"])
        nbo = (nbits + (1 << 15)) >> 16
        v = (nbo << 16) - nbits
        return int(st[(v >> nbo) + find])

    def enc(state, tt, st, sym):
        find, nbits = int(tt[sym]["find"]), int(tt[sym]["nbits"])
        nbo = (state + nbits) >> 16
        w.add(state, nbo)
        return int(st[(state >> nbo) + find])

    ll, ml, off = seqs[-1]
    llc, mlc, ofc, mlb, ofv = _codes(T, ll, ml, off)
    sml = init(T["ml"], T["mlst"], mlc)
    sof = init(T["of"], T["ofst"], ofc)
    sll = init(T["ll"], T["llst"], llc)
    w.add(ll, T["llbits"][llc])
    w.add(mlb, T["mlbits"][mlc])
    w.flush()
    w.add(ofv, ofc)
    w.flush()
    for ll, ml, off in reversed(seqs[:-1]):
        llc, mlc, ofc, mlb, ofv = _codes(T, ll, ml, off)
        sof = enc(sof, T["of"], T["ofst"], ofc)
        sml = enc(sml, T["ml"], T["mlst"], mlc)
        w.flush()
        sll = enc(sll, T["ll"], T["llst"], llc)
        w.add(ll, T["llbits"][llc])
        w.flush()
        w.add(mlb, T["mlbits"][mlc])
        w.flush()
        w.add(ofv, ofc)
        w.flush()
    w.add(sml, 6)
    w.flush()
    w.add(sof, 5)
    w.flush()
    w.add(sll, 6)
    w.add(1, 1)
    w.flush()
    if w.nb:
        w.out.append(w.acc & 0xFF)
    return bytes(w.out)


def compressed_block(T, data: bytes, seqs):
    """Block content: raw literals section + sequences section."""
    lits = bytearray()
    pos = 0
    for ll, ml, off in seqs:
        lits += data[pos:pos + ll]
        pos += ll + ml
    lits += data[pos:]
    n = len(lits)
    if n < 32:
        lh = bytes([n << 3])
    elif n < 4096:
        lh = (1 << 2 | n << 4).to_bytes(2, "little")
    else:
        lh = (3 << 2 | n << 4).to_bytes(3, "little")
    k = len(seqs)
    if k == 0:
        sh = b"\x00"
    elif k < 128:
        sh = bytes([k, 0])
    elif k < 0x7F00:
        sh = bytes([(k >> 8) + 0x80, k & 0xFF, 0])
    else:
        sh = bytes([0xFF]) + (k - 0x7F00).to_bytes(2, "little") + b"\x00"
    return lh + bytes(lits) + sh + (encode_sequences(T, seqs) if k else b"")


def frame(blocks_, size):
    """A single-segment frame of (type, content, regenerated size) blocks."""
    if size < 256:
        hdr = bytes([0x20, size])
    elif size < 65536 + 256:
        hdr = bytes([0x60]) + (size - 256).to_bytes(2, "little")
    else:
        hdr = bytes([0xA0]) + size.to_bytes(4, "little")
    out = bytearray(b"\x28\xb5\x2f\xfd" + hdr)
    for i, (tpe, content, rsize) in enumerate(blocks_):
        last = i == len(blocks_) - 1
        bsize = rsize if tpe == 1 else len(content)
        out += (int(last) | tpe << 1 | bsize << 3).to_bytes(3, "little") + content
    return bytes(out)


def greedy_sequences(data: bytes, min_match: int = 4):
    """A plain greedy LZ parse (dictionary of last positions), for tests."""
    seqs, last, anchor, p, n = [], {}, 0, 0, len(data)
    while p + min_match <= n - 4:
        key = data[p:p + 4]
        c = last.get(key)
        last[key] = p
        if c is not None:
            m = 4
            while p + m < n and data[c + m] == data[p + m]:
                m += 1
            seqs.append((p - anchor, m, p - c))
            p += m
            anchor = p
        else:
            p += 1
    return seqs


# ---- Huffman-coded literals (RFC 8878 4.2), the device's algorithm ---------

HUF_MAX_BITS = 11


def huf_lengths(counts):
    """Code lengths (<= 11 bits, Kraft sum exactly 1) as the device builds
    them: Shannon lengths ceil(log2(total / count)) clamped to 11; while the
    Kraft sum exceeds 1, lengthen the shortest code below 11 (lowest symbol
    first); then, shortest codes first, shorten every code while the slack
    allows.  None if that cannot close the sum (never seen) or < 2 symbols."""
    M = HUF_MAX_BITS
    total = int(sum(counts))
    L = [0] * 256
    for s in range(256):
        c = int(counts[s])
        if c:
            q = -(-total // c)
            L[s] = min(M, max(1, (q - 1).bit_length()))
    syms = [s for s in range(256) if L[s]]
    if len(syms) < 2:
        return None
    K = sum(1 << (M - L[s]) for s in syms)
    while K > (1 << M):
        s = min((s for s in syms if L[s] < M), key=lambda s: (L[s], s))
        K -= 1 << (M - L[s] - 1)
        L[s] += 1
    for ln in range(1, M + 1):
        for s in syms:
            if L[s] == ln:
                while L[s] > 1 and K + (1 << (M - L[s])) <= (1 << M):
                    K += 1 << (M - L[s])
                    L[s] -= 1
    return L if K == (1 << M) else None


def huf_codes(L):
    """Canonical codes of the decoder's table (HUF_readDTableX1): weights
    ascending, symbols in order within a weight; the table log is the
    longest code (HUF_readStats wants >= 2 symbols of weight 1).  Returns
    (vals, nbits, weights)."""
    M = max(L)
    w = [M + 1 - l if l else 0 for l in L]
    cnt = [0] * (M + 2)
    for x in w:
        if x:
            cnt[x] += 1
    start, acc = [0] * (M + 2), 0
    for x in range(1, M + 1):
        start[x] = acc
        acc += cnt[x] << (x - 1)
    vals = [0] * 256
    for s in range(256):
        if w[s]:
            vals[s] = start[w[s]] >> (w[s] - 1)
            start[w[s]] += 1 << (w[s] - 1)
    return vals, L, w


def huf_literals_section(lits: bytes):
    """Compressed_Literals_Block with 4 streams and direct weights, or None
    (max symbol > 128, < 2 symbols, no gain)."""
    n = len(lits)
    counts = np.bincount(np.frombuffer(lits, np.uint8), minlength=256)
    maxsym = int(np.nonzero(counts)[0].max())
    if n < 64:
        return None
    L = huf_lengths(counts)
    if L is None:
        return None
    vals, nb, w = huf_codes(L)
    if maxsym <= 128:  # direct representation: 4-bit weights
        tree = bytes([127 + maxsym]) + bytes(
            (w[k] << 4 | (w[k + 1] if k + 1 < maxsym else 0)) for k in range(0, maxsym, 2))
    else:  # FSE-compressed weights
        fw = fse_compress_weights(w[:maxsym])
        if fw is None:
            return None
        tree = bytes([len(fw)]) + fw
    seg = (n + 3) // 4
    streams = []
    for k in range(4):
        part = lits[k * seg:min(n, (k + 1) * seg)]
        bw = BitWriter()
        for b in reversed(part):
            bw.add(vals[b], nb[b])
            bw.flush()
        bw.add(1, 1)
        bw.flush()
        if bw.nb:
            bw.out.append(bw.acc & 0xFF)
        streams.append(bytes(bw.out))
    jump = b"".join(len(s).to_bytes(2, "little") for s in streams[:3])
    comp = len(tree) + 6 + sum(len(s) for s in streams)
    if n < 1024:
        hdr = (2 | 1 << 2 | n << 4 | comp << 14).to_bytes(3, "little")
    elif n < 16384:
        hdr = (2 | 2 << 2 | n << 4 | comp << 18).to_bytes(4, "little")
    else:
        hdr = (2 | 3 << 2 | n << 4 | comp << 22).to_bytes(5, "little")
    return hdr + tree + jump + b"".join(streams)


def compressed_block_huf(T, data: bytes, seqs):
    """compressed_block with Huffman literals where they apply."""
    lits = bytearray()
    pos = 0
    for ll, ml, off in seqs:
        lits += data[pos:pos + ll]
        pos += ll + ml
    lits += data[pos:]
    sec = huf_literals_section(bytes(lits))
    raw = compressed_block(T, data, seqs)
    if sec is None:
        return raw
    n = len(lits)
    lh = 1 if n < 32 else 2 if n < 4096 else 3
    return sec + raw[lh + n:]


# ---- adaptive FSE tables for the sequences (FSE_Compressed mode, log 6) ---

FSE_ADAPT_LOG = 6
PREDEF_NORM = {
    "ll": ([4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1,
            1, 1, -1, -1, -1, -1], 6),
    "ml": ([1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
            1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1], 6),
    "of": ([1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1,
            -1], 5),
}


def fse_normalize(counts, tl=FSE_ADAPT_LOG):
    """Counts -> normalized counts summing to 2^tl, every present symbol >= 1
    (no low-probability -1 symbols): rounded shares, the difference taken
    from / given to the largest symbols (the device's rule)."""
    size = 1 << tl
    total = int(sum(counts))
    norm = [0] * len(counts)
    for s, c in enumerate(counts):
        if c:
            norm[s] = max(1, (int(c) * size + total // 2) // total)
    diff = size - sum(norm)
    big = max(range(len(counts)), key=lambda s: (norm[s], -s))
    if diff > 0:
        norm[big] += diff
    while diff < 0:  # take one from the current largest (lowest symbol on ties)
        big = max(range(len(counts)), key=lambda s: (norm[s], -s))
        norm[big] -= 1
        diff += 1
    return norm


def fse_write_ncount(norm, tl):
    """FSE_writeNCount (RFC 8878 4.1.1): the table description bytes."""
    bw = BitWriter()
    bw.add(tl - 5, 4)
    remaining = (1 << tl) + 1
    threshold = 1 << tl
    nbits = tl + 1
    s, n = 0, len(norm)
    prev0 = False
    while s < n and remaining > 1:
        if prev0:
            start = s
            while s < n and norm[s] == 0:
                s += 1
            while s >= start + 24:
                start += 24
                bw.add(0xFFFF, 16)
                bw.flush()
            while s >= start + 3:
                start += 3
                bw.add(3, 2)
            bw.add(s - start, 2)
            bw.flush()
        count = norm[s]
        s += 1
        mx = (2 * threshold - 1) - remaining
        remaining -= abs(count)
        count += 1
        if count >= threshold:
            count += mx
        bw.add(count, nbits - (1 if count < mx else 0))
        bw.flush()
        prev0 = count == 1
        while remaining < threshold:
            nbits -= 1
            threshold >>= 1
    assert remaining == 1
    if bw.nb:
        bw.out.append(bw.acc & 0xFF)
    return bytes(bw.out)


def fse_ctable(norm, tl):
    """FSE_buildCTable: (symbol transforms [(find, nbits)], state table)."""
    size, mask, step = 1 << tl, (1 << tl) - 1, (1 << tl >> 1) + (1 << tl >> 3) + 3
    sym, cumul, high = [0] * size, [0] * (len(norm) + 1), size - 1
    for u in range(1, len(norm) + 1):
        if norm[u - 1] == -1:
            cumul[u] = cumul[u - 1] + 1
            sym[high] = u - 1
            high -= 1
        else:
            cumul[u] = cumul[u - 1] + norm[u - 1]
    pos = 0
    for s, c in enumerate(norm):
        for _ in range(max(c, 0)):
            sym[pos] = s
            pos = (pos + step) & mask
            while pos > high:
                pos = (pos + step) & mask
    st = [0] * size
    cu = list(cumul)
    for u in range(size):
        st[cu[sym[u]]] = size + u
        cu[sym[u]] += 1
    tt, total = [], 0
    for c in norm:
        if c in (-1, 1):
            tt.append((total - 1, (tl << 16) - size))
            total += 1
        elif c > 1:
            mbo = tl - ((c - 1).bit_length() - 1)
            tt.append((total - c, (mbo << 16) - (c << mbo)))
            total += c
        else:
            tt.append((0, ((tl + 1) << 16) - size))
    return tt, st


def encode_sequences_tabs(tabs, seqs, T, values=False):
    """encode_sequences with per-stream tables tabs[name] = (tt, st, tl);
    values: seqs carry offset values (repeat codes) instead of offsets."""
    w = BitWriter()

    def init(name, sym):
        tt, st, _ = tabs[name]
        find, nbits = tt[sym]
        nbo = (nbits + (1 << 15)) >> 16
        v = (nbo << 16) - nbits
        return st[(v >> nbo) + find]

    def enc(name, state, sym):
        tt, st, _ = tabs[name]
        find, nbits = tt[sym]
        nbo = (state + nbits) >> 16
        w.add(state, nbo)
        return st[(state >> nbo) + find]

    ll, ml, off = seqs[-1]
    llc, mlc, ofc, mlb, ofv = _codes(T, ll, ml, off, values)
    sml, sof, sll = init("ml", mlc), init("of", ofc), init("ll", llc)
    w.add(ll, T["llbits"][llc])
    w.add(mlb, T["mlbits"][mlc])
    w.flush()
    w.add(ofv, ofc)
    w.flush()
    for ll, ml, off in reversed(seqs[:-1]):
        llc, mlc, ofc, mlb, ofv = _codes(T, ll, ml, off, values)
        sof = enc("of", sof, ofc)
        sml = enc("ml", sml, mlc)
        w.flush()
        sll = enc("ll", sll, llc)
        w.add(ll, T["llbits"][llc])
        w.flush()
        w.add(mlb, T["mlbits"][mlc])
        w.flush()
        w.add(ofv, ofc)
        w.flush()
    w.add(sml, tabs["ml"][2])
    w.flush()
    w.add(sof, tabs["of"][2])
    w.flush()
    w.add(sll, tabs["ll"][2])
    w.add(1, 1)
    w.flush()
    if w.nb:
        w.out.append(w.acc & 0xFF)
    return bytes(w.out)


def _cost_bits(counts, norm, tl):
    import math
    return sum(c * (tl - math.log2(norm[s])) for s, c in enumerate(counts) if c)


def sequences_section_adaptive(T, seqs, values=False):
    """Sequences section choosing, per stream, predefined or an adaptive
    log-6 table by estimated bits (the device's rule)."""
    k = len(seqs)
    codes = [_codes(T, *s, values) for s in seqs]
    hist = {"ll": [0] * 36, "ml": [0] * 53, "of": [0] * 32}
    for llc, mlc, ofc, _, _ in codes:
        hist["ll"][llc] += 1
        hist["ml"][mlc] += 1
        hist["of"][ofc] += 1
    modes, descs, tabs = {}, {}, {}
    for name in ("ll", "of", "ml"):
        pn, ptl = PREDEF_NORM[name]
        cnt = hist[name]
        pnorm = [abs(x) for x in pn] + [0] * (len(cnt) - len(pn))
        if any(c and not pnorm[s] for s, c in enumerate(cnt)):
            pcost = float("inf")
        else:
            pcost = _cost_bits(cnt, pnorm, ptl)
        an = fse_normalize(cnt)
        last = max(s for s in range(len(cnt)) if cnt[s])
        desc = fse_write_ncount(an[:last + 1], FSE_ADAPT_LOG)
        acost = _cost_bits(cnt, an, FSE_ADAPT_LOG) + 8 * len(desc)
        if acost < pcost:
            modes[name], descs[name] = 2, desc
            tt, st = fse_ctable(an[:last + 1], FSE_ADAPT_LOG)
            tabs[name] = (tt, st, FSE_ADAPT_LOG)
        else:
            modes[name], descs[name] = 0, b""
            tt, st = fse_ctable(pn, ptl)
            tabs[name] = (tt, st, ptl)
    if k < 128:
        sh = bytes([k])
    elif k < 0x7F00:
        sh = bytes([(k >> 8) + 0x80, k & 0xFF])
    else:
        sh = bytes([0xFF]) + (k - 0x7F00).to_bytes(2, "little")
    sh += bytes([modes["ll"] << 6 | modes["of"] << 4 | modes["ml"] << 2])
    return sh + descs["ll"] + descs["of"] + descs["ml"] + encode_sequences_tabs(tabs, seqs, T,
                                                                               values)


def compressed_block_adaptive(T, data: bytes, seqs, reps=False):
    """Huffman literals (where they apply) + adaptive sequences; reps: code
    offsets with block-local repeat codes (offsets_to_values)."""
    lits = bytearray()
    pos = 0
    for ll, ml, off in seqs:
        lits += data[pos:pos + ll]
        pos += ll + ml
    lits += data[pos:]
    sec = huf_literals_section(bytes(lits))
    if sec is None:
        n = len(lits)
        if n < 32:
            sec = bytes([n << 3]) + bytes(lits)
        elif n < 4096:
            sec = (1 << 2 | n << 4).to_bytes(2, "little") + bytes(lits)
        else:
            sec = (3 << 2 | n << 4).to_bytes(3, "little") + bytes(lits)
    if not seqs:
        return sec + b"\x00"
    if reps:
        return sec + sequences_section_adaptive(T, offsets_to_values(seqs), True)
    return sec + sequences_section_adaptive(T, seqs)


# ---- FSE-compressed Huffman weights (RFC 8878 4.2.1.2), for maxsym > 128 ---

def fse_compress_weights(weights):
    """Huffman weights (symbols 0 .. n-1) as an FSE stream of accuracy log 6
    with two interleaved states (FSE_compress_usingCTable order), NCount
    description first; None when < 2 distinct weights or >= 128 bytes."""
    n = len(weights)
    counts = [0] * 12
    for w in weights:
        counts[w] += 1
    if sum(1 for c in counts if c) < 2:
        return None
    tl = 6
    norm = fse_normalize(counts, tl)
    last = max(s for s in range(12) if counts[s])
    desc = fse_write_ncount(norm[:last + 1], tl)
    tt, st = fse_ctable(norm[:last + 1], tl)
    w = BitWriter()

    def init(sym):
        find, nbits = tt[sym]
        nbo = (nbits + (1 << 15)) >> 16
        v = (nbo << 16) - nbits
        return st[(v >> nbo) + find]

    def enc(state, sym):
        find, nbits = tt[sym]
        nbo = (state + nbits) >> 16
        w.add(state, nbo)
        return st[(state >> nbo) + find]

    ip = n
    if n & 1:
        s1 = init(weights[ip - 1])
        s2 = init(weights[ip - 2])
        s1 = enc(s1, weights[ip - 3])
        ip -= 3
        w.flush()
    else:
        s2 = init(weights[ip - 1])
        s1 = init(weights[ip - 2])
        ip -= 2
    rest = n - 2
    if rest & 2:
        s2 = enc(s2, weights[ip - 1])
        s1 = enc(s1, weights[ip - 2])
        ip -= 2
        w.flush()
    while ip > 0:
        s2 = enc(s2, weights[ip - 1])
        s1 = enc(s1, weights[ip - 2])
        s2 = enc(s2, weights[ip - 3])
        s1 = enc(s1, weights[ip - 4])
        ip -= 4
        w.flush()
    w.add(s2, tl)
    w.flush()
    w.add(s1, tl)
    w.add(1, 1)
    w.flush()
    if w.nb:
        w.out.append(w.acc & 0xFF)
    out = desc + bytes(w.out)
    return out if len(out) < 128 else None


# ---- repeat offsets (RFC 8878 3.1.2.5), block-local history ---------------

def offsets_to_values(seqs):
    """[(ll, ml, off)] -> [(ll, ml, offset_value)] with repeat codes where
    the offset is one of the repeat history entries set inside this block
    (entries inherited from earlier blocks are unknown to a block coded in
    parallel, so never referenced): the device's rule."""
    rep = [None, None, None]
    out = []
    for ll, ml, off in seqs:
        if ll > 0:
            if rep[0] == off:
                v = 1
            elif rep[1] == off:
                v, rep = 2, [rep[1], rep[0], rep[2]]
            elif rep[2] == off:
                v, rep = 3, [rep[2], rep[0], rep[1]]
            else:
                v, rep = off + 3, [off, rep[0], rep[1]]
        else:
            if rep[1] == off:
                v, rep = 1, [rep[1], rep[0], rep[2]]
            elif rep[2] == off:
                v, rep = 2, [rep[2], rep[0], rep[1]]
            elif rep[0] is not None and rep[0] - 1 == off:
                v, rep = 3, [off, rep[0], rep[1]]
            else:
                v, rep = off + 3, [off, rep[0], rep[1]]
        out.append((ll, ml, v))
    return out


def greedy_sequences_rep(data: bytes):
    """greedy_sequences with zstd_fast's repeat check first (the last offset
    at the current position)."""
    seqs, last, anchor, p, n = [], {}, 0, 0, len(data)
    rep = None
    while p + 8 <= n:
        if rep and p - rep >= 0 and data[p:p + 4] == data[p - rep:p - rep + 4]:
            m = 4
            while p + m < n and data[p + m] == data[p - rep + m]:
                m += 1
            seqs.append((p - anchor, m, rep))
            last[data[p:p + 4]] = p
            p += m
            anchor = p
            continue
        key = data[p:p + 4]
        c = last.get(key)
        last[key] = p
        if c is not None:
            m = 4
            while p + m < n and data[c + m] == data[p + m]:
                m += 1
            seqs.append((p - anchor, m, p - c))
            rep = p - c
            p += m
            anchor = p
        else:
            p += 1
    return seqs
