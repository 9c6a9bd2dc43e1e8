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


def _codes(T, ll, ml, off):
    mlb, ofv = ml - 3, off + 3
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
