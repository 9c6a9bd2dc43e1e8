"""Pure-Python restatement of the Rabin64 chunker, for SMALL cross-checks only.

TEST INFRASTRUCTURE ONLY (see oracle/oracle.py).  Independent second
restatement of rustic_cdc 0.3.1 ``Rabin64`` (tables: SURVEY.md A.1; slide /
reset_and_prefill_window: A.2) and of ``ChunkIter::next``
(crates/core/src/chunker/rabin.rs:107-191), written from the closed form of
SURVEY.md section 8a instead of the ring-window state machine that
oracle/cdc_ref.c uses, so that the two restatements check each other.
"""


def degree(p: int) -> int:
    return p.bit_length() - 1


def modulo(p: int, m: int) -> int:
    dm = degree(m)
    while p and degree(p) >= dm:
        p ^= m << (degree(p) - dm)
    return p


def fp(window: bytes, poly: int) -> int:
    """fp(w) = sum w[i] x^(8(|w|-1-i)) mod P (direct long division)."""
    v = 0
    for b in window:
        v = modulo((v << 8) | b, poly)
    return v


def chunk_cuts(data: bytes, poly: int, min_size: int, avg: int, max_size: int,
               prefill64: bool = False):
    """Cut offsets from the section 8a closed form (O(n*64), small inputs only)."""
    mask = avg - 1
    n = len(data)
    s = 0
    cuts = []
    while s < n:
        if n - s < min_size:
            cuts.append(n)
            break
        z = s + min_size
        cut = None
        k = 0
        while True:
            L = z + k
            if L - s >= max_size:
                cut = L
                break
            if k < 64 and not prefill64:
                v = data[z - 64:z - 1] + data[z:L]   # byte z-1 never hashed (V1)
                h = fp(v[-64:], poly)
            else:
                h = fp(data[L - 64:L], poly)
            if h & mask == 0:
                cut = L
                break
            if L == n:
                cut = n
                break
            k += 1
        cuts.append(cut)
        s = cut
    return cuts
