#!/usr/bin/env python
"""CPU model of the walk kernel's hashing work (rcdc_walk.hip walk_next /
round_first), to split its lane-hashed bytes into what the reference hashes
and the overheads: per-lane warm-up, the part of a chunk's last round past
its cut, the partial last round of a piece that stops "open", and piece
boundaries.  Data: C3-shaped streams (bench.make_mixed's run layout, numpy
bytes); cut chains from the oracle (test infrastructure, this is a model).

  python tools/walk_model.py --streams 2 --mib 256 [--seg 1024] [--adaptive]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle  # noqa: E402

MIN, MAX = 512 << 10, 8 << 20
LANES = [64]  # lanes per round (--lanes)
SCHED = []  # per-lane segment of a search's first rounds (--sched), then --seg


def mixed(seed, n):
    rng = np.random.default_rng(seed)
    out = np.zeros(n, np.uint8)
    pos, runs = 0, []
    while pos < n:
        if rng.random() < 0.5:
            L = min(int(np.exp(rng.uniform(np.log(64 << 10), np.log(16 << 20)))), n - pos)
            runs.append((pos, L, False))
        else:
            L = min(int(np.exp(rng.uniform(np.log(4 << 10), np.log(16 << 20)))), n - pos)
            runs.append((pos, L, True))
        pos += L
    br = np.random.default_rng(seed + 77)
    for p, L, z in runs:
        if not z:
            out[p:p + L] = br.integers(0, 256, L, dtype=np.uint8)
    return out


def pieces(N, Lp=4 << 20, split=20):
    P = max(N // Lp, 1)
    nsplit = (P * split + 50) // 100
    Ls = max(Lp // 4 // MIN, 1) * MIN
    out = []
    for b in range(P):
        a, e = b * Lp, (b + 1) * Lp if b + 1 < P else N
        if b + nsplit < P:
            out.append((a, e))
        else:
            q = max((e - a) // Ls, 1)
            for k in range(q):
                out.append((a + k * Ls, a + (k + 1) * Ls if k + 1 < q else e))
    return out


def round_bytes(S, span, adaptive):
    """Lane-hashed bytes of the rounds that cover `span` positions from A
    (64 lanes x (S + 64)); adaptive: the last round shrinks its segment to
    the 64-byte units it needs."""
    nl = LANES[0]
    step = nl * S
    full, rest = divmod(span, step)
    b = full * nl * (S + 64)
    if rest:
        if adaptive:
            s2 = min(S, max(((rest + 63) // 64 + 63) // 64 * 64, 64))
            b += nl * (s2 + 64)
        else:
            b += nl * (S + 64)
    return b


def walk_piece(data, N, a, e, S, adaptive, hitpos):
    """Walker of piece [a, e): (lane bytes, searched-to-hit bytes, zones, kinds)."""
    end_slice = min(N, e + MAX + 1)
    cuts = a + oracle.chunk_cuts(data[a:end_slice]).astype(np.int64)
    if end_slice < N and len(cuts) and cuts[-1] == end_slice:
        cuts = cuts[:-1]  # slice-end artefact (never reached: the walk stops first)
    stop_scan = e + MIN + 64 if e < N else 1 << 62
    lane = zones = ideal = 0
    waste_hit = waste_open = 0
    s = a
    for c in cuts:
        c = int(c)
        if N - s <= MIN:
            break
        zones += 1
        if c - s < MIN + 64 and c < min(s + MAX, N):  # zone / zero-prefill cut
            s = c
            if s >= e:
                break
            continue
        q = s + MIN + 64
        A = (q - 1) & ~63
        limit = min(s + MAX, N)
        end = min(limit, stop_scan)
        if c < end and c < limit:  # a hit inside the searched range
            # rounds of SCHED[0], SCHED[1], ... then S bytes per lane
            pos, b, r = A, 0, 0
            while pos < c:
                sg = SCHED[r] if r < len(SCHED) else S
                pos += LANES[0] * sg
                b += LANES[0] * (sg + 64)
                r += 1
            lane += b
            ideal += c - q + 1
            waste_hit += b - (c - A) - r * LANES[0] * 64
            s = c
        else:
            span = end - A
            b = round_bytes(S, span, adaptive)
            lane += b
            ideal += end - q
            if end < limit:
                nl = LANES[0]
                waste_open += b - span - ((span + nl * S - 1) // (nl * S)) * nl * 64
                return lane, ideal, zones, waste_hit, waste_open, True
            s = c
        if s >= e:
            break
    return lane, ideal, zones, waste_hit, waste_open, False


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--seg", type=int, default=1024)
    ap.add_argument("--adaptive", action="store_true")
    ap.add_argument("--piece-mib", type=int, default=4)
    ap.add_argument("--split", type=int, default=20)
    ap.add_argument("--random", action="store_true", help="uniform random bytes (C4's files)")
    ap.add_argument("--lanes", type=int, default=64, help="lanes per round (one chain)")
    ap.add_argument("--sched", default="", help="comma list: segment of a search's first rounds")
    a = ap.parse_args()
    SCHED[:] = [int(x) for x in a.sched.split(",") if x]
    LANES[0] = a.lanes
    tot = {"lane": 0, "ideal_search": 0, "zones": 0, "waste_hit": 0, "waste_open": 0,
           "ref_hashed": 0, "warm": 0, "pieces": 0, "open": 0, "true_lane": 0}
    for j in range(a.streams):
        N = a.mib << 20
        data = (np.random.default_rng(4000 + j).integers(0, 256, N, dtype=np.uint8)
                if a.random else mixed(3000 + j, N))
        true = oracle.chunk_cuts(data).astype(np.int64)
        L = np.diff(np.concatenate([[0], true]))
        tot["ref_hashed"] += int(np.sum(L[L >= MIN] - MIN)) + 63 * int(np.count_nonzero(L >= MIN))
        # the true chain walked as one piece (no boundaries)
        lt, _, _, _, _, _ = walk_piece(data, N, 0, N, a.seg, a.adaptive, None)
        tot["true_lane"] += lt
        for (p0, p1) in pieces(N, a.piece_mib << 20, a.split):
            lane, ideal, zones, wh, wo, op = walk_piece(data, N, p0, p1, a.seg, a.adaptive, None)
            tot["lane"] += lane
            tot["ideal_search"] += ideal
            tot["zones"] += zones
            tot["waste_hit"] += wh
            tot["waste_open"] += wo
            tot["pieces"] += 1
            tot["open"] += op
    lane_z = tot["lane"] + tot["zones"] * 4096
    print({k: v for k, v in tot.items()})
    print(f"lane+zones / ref = {lane_z / tot['ref_hashed']:.4f}; true chain alone / ref = "
          f"{tot['true_lane'] / tot['ref_hashed']:.4f}; waste_hit {tot['waste_hit'] / tot['ref_hashed']:.4f}"
          f" waste_open {tot['waste_open'] / tot['ref_hashed']:.4f}")


if __name__ == "__main__":
    main()
