"""Craft inputs whose first cut falls in the min-zone [min, min+64).

The min-zone is where the reference's 63-byte prefill (V1, canonical) and a
full 64-byte prefill (variant A) disagree.  fp is
GF(2)-linear in the window bits, so flipping chosen bits of 3 bytes inside
the hashed window solves ``fp(window) & mask == 0`` exactly (Gaussian
elimination over GF(2)).  Used by the parity tests to exercise the device
min-zone path; the expected cuts always come from the oracle.
"""
import numpy as np

from oracle import oracle, pyref


def _fp(data, positions, poly):
    return pyref.fp(bytes(int(data[p]) for p in positions), poly)


def _solve(data, positions, free, mask, poly):
    """Flip bits of bytes at `free` so that fp(data[positions]) & mask == 0."""
    base = _fp(data, positions, poly) & mask
    cols = []
    for p in free:
        for bit in range(8):
            d = np.zeros_like(data)
            d[p] = 1 << bit
            cols.append(_fp(d, positions, poly) & mask)
    nbits = mask.bit_length()
    # rows: equations (bits of mask); unknowns: len(cols)
    rows = []
    for r in range(nbits):
        row = 0
        for j, c in enumerate(cols):
            if (c >> r) & 1:
                row |= 1 << j
        rows.append([row, (base >> r) & 1])
    # elimination
    piv_cols = []
    ri = 0
    n = len(cols)
    for c in range(n):
        sel = None
        for k in range(ri, len(rows)):
            if (rows[k][0] >> c) & 1:
                sel = k
                break
        if sel is None:
            continue
        rows[ri], rows[sel] = rows[sel], rows[ri]
        for k in range(len(rows)):
            if k != ri and (rows[k][0] >> c) & 1:
                rows[k][0] ^= rows[ri][0]
                rows[k][1] ^= rows[ri][1]
        piv_cols.append(c)
        ri += 1
    for k in range(ri, len(rows)):
        if rows[k][1]:
            return None  # inconsistent
    x = 0
    for k, c in enumerate(piv_cols):
        if rows[k][1]:
            x |= 1 << c
    out = data.copy()
    for j in range(n):
        if (x >> j) & 1:
            p = free[j // 8]
            out[p] ^= 1 << (j % 8)
    assert _fp(out, positions, poly) & mask == 0
    return out


def craft_zone_cases(min_size, avg, count=16, seed=1, poly=oracle.DEFAULT_POLY, n=None):
    rng = np.random.default_rng(seed)
    mask = avg - 1
    z = min_size
    n = n or (min_size + 3 * avg)
    out = []
    for i in range(count):
        data = rng.integers(0, 256, size=n, dtype=np.uint8)
        if i % 2 == 0:
            # V1 hit at z + k: window = b[z-64+k-1 .. z-1) ++ b[z .. z+k)
            k = int(rng.integers(0, 64))
            if k == 0:
                pos = list(range(z - 64, z - 1))
            else:
                pos = list(range(z - 65 + k, z - 1)) + list(range(z, z + k))
            free = [pos[3], pos[len(pos) // 2], pos[-2]]
        else:
            # variant-A hit at z: window = b[z-64 .. z); flip inside b[z-64..z-1)
            k = 0
            pos = list(range(z - 64, z))
            free = [pos[2], pos[30], pos[60]]
        res = _solve(data, pos, free, mask, poly)
        if res is not None:
            out.append((res, k))
    return out
