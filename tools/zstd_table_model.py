"""CPU model of the zstd block parse's match-finder table (DESIGN.md 3f,
round 3): compressed size per kind when the LDS hash table keeps 2^HL
positions with K-byte keys, inserting every INS-th position, and a
zstd_dfast-like pair of tables; the block coder is tests/zstd_model.py's
(adaptive FSE, Huffman literals, repeat offsets).  Test infrastructure,
not the device path.

  python tools/zstd_table_model.py
"""
import os
import sys

import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tests')); sys.path.insert(0, ROOT)
import zstd_model as zm
rng = np.random.default_rng(0)
words = [bytes(rng.integers(97, 123, size=int(rng.integers(2, 9))).astype(np.uint8)) for _ in range(400)]
text = b" ".join(words[int(i)] for i in rng.integers(0, 400, 1 << 18))
csv = b"".join(b"%08d,%s,%d,%s\n" % (i, words[i % 400], (i * 7919) % 100000, words[(i * 31) % 400]) for i in range(40000))
code = b"".join(b"    x_%d = foo(%s, %d) + bar[%d];\n" % (i % 97, words[i % 50], i, (i * 13) % 1000) for i in range(40000))
T = zm.tables()

def parse(d, HL, key, ins, lazy=True):
    """greedy with a 2^HL table (one position per bucket, exact tag), lookup
    every position, insert positions p % ins == 0; backward extension."""
    n = len(d); tab = {}; seqs = []; anchor = 0; p = 0; mask = (1 << HL) - 1
    while p + 8 <= n:
        k = d[p:p + key]
        h = hash(k) & mask
        e = tab.get(h)
        c = None
        if e is not None and e[1] == k: c = e[0]
        if p % ins == 0: tab[h] = (p, k)
        if c is not None:
            m = key
            while p + m < n and d[c + m] == d[p + m]: m += 1
            b = 0
            while p - b > anchor and c - b > 0 and d[p - b - 1] == d[c - b - 1]: b += 1
            seqs.append((p - b - anchor, m + b, p - c))
            p += m; anchor = p
        else:
            p += 1
    return seqs

def size(data, HL, key, ins, bs=128 << 10):
    tot = 0
    for o in range(0, len(data), bs):
        blk = data[o:o + bs]
        seqs = parse(blk, HL, key, ins)
        try:
            b = zm.compressed_block_adaptive(T, blk, seqs, reps=True)
        except TypeError:
            b = zm.compressed_block_adaptive(T, blk, seqs)
        tot += min(len(b), len(blk))
    return tot / len(data)

def parse2(d, HA, kA, HB, kB, insB):
    n=len(d); ta={}; tb={}; seqs=[]; anchor=0; p=0; ma=(1<<HA)-1; mb=(1<<HB)-1
    while p + 8 <= n:
        c=None
        kb=d[p:p+kB]
        if len(kb)==kB:
            e=tb.get(hash(kb)&mb)
            if e is not None and e[1]==kb: c=e[0]
        ka=d[p:p+kA]; ha=hash(ka)&ma
        if c is None:
            e=ta.get(ha)
            if e is not None and e[1]==ka: c=e[0]
        ta[ha]=(p,ka)
        if p % insB == 0 and len(kb)==kB: tb[hash(kb)&mb]=(p,kb)
        if c is not None:
            m=0
            while p+m<n and d[c+m]==d[p+m]: m+=1
            b=0
            while p-b>anchor and c-b>0 and d[p-b-1]==d[c-b-1]: b+=1
            seqs.append((p-b-anchor, m+b, p-c)); 
            # insert a couple of positions inside the match (zstd fast inserts p+2 and end-2)
            q=p+2
            if q+kB<=n and q % insB == 0: tb[hash(d[q:q+kB])&mb]=(q,d[q:q+kB])
            p+=m; anchor=p
        else: p+=1
    return seqs
def size2(data, *a, bs=128<<10):
    tot=0
    for o in range(0,len(data),bs):
        blk=data[o:o+bs]; seqs=parse2(blk,*a)
        b = zm.compressed_block_adaptive(T, blk, seqs, reps=True)
        tot+=min(len(b),len(blk))
    return tot/len(data)

if __name__ == "__main__":
    for name, data in (("csv", csv[:512 << 10]), ("code", code[:512 << 10]), ("text", text[:512 << 10])):
        for HL, key, ins in [(11, 4, 1), (11, 4, 2), (11, 4, 4), (11, 6, 1), (11, 6, 2), (11, 6, 4), (12, 4, 1), (12, 6, 2), (12, 6, 4), (16, 6, 1), (20, 6, 1)]:
            print(name, HL, key, ins, round(size(data, HL, key, ins), 4), flush=True)
    for name, data in (("csv", csv[:512<<10]), ("code", code[:512<<10]), ("text", text[:512<<10])):
        for cfg in [(10,4,11,8,4), (10,4,12,8,4), (10,4,11,6,2), (10,4,11,8,2), (11,4,11,8,4), (10,4,11,6,4)]:
            print(name, cfg, round(size2(data, *cfg),4), flush=True)
