"""Per-piece trace of rcdc_walk_kernel (RCDC_WALK_TRACE=1): where the walk's
time goes on C3-shaped (mixed) and all-random 64 x 1 GiB batches.

usage: python tools/walk_trace.py [mixed|random|both|c4] [streams] [GiB per stream]
(c4: bench.py's C4 files -- `streams` files, log-uniform 4-256 MiB, random bytes)
Prints per batch: walk/chain time (HIP events), work counters, wave-slot
utilisation (sum of piece durations / (4096 wave slots x makespan)), the
active-piece timeline (how long fewer than 1024 / 256 pieces were in flight:
the tail), and the per-round time at full and at tail occupancy.
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["RCDC_WALK_TRACE"] = "1"

from bench import make_mixed  # noqa: E402
from oracle import oracle  # noqa: E402
from rustic_core_amd.chunker import Context  # noqa: E402
from rustic_core_amd.device import DevicePlan, pack_offsets  # noqa: E402

GiB = 1 << 30


def run(kind, nstreams, sgib):
    dev = torch.device("cuda", 0)
    sb = int(sgib * GiB)
    lens = np.full(nstreams, sb, np.uint64)
    if kind == "c4":  # bench.py C4: the first `nstreams` files, log-uniform 4-256 MiB
        from bench import c4_fill, c4_files
        sizes = c4_files(nstreams)
        files = sorted(range(nstreams), key=lambda f: -sizes[f])
        lens = np.array([sizes[f] for f in files], np.uint64)
    offs, alen = pack_offsets(lens)
    if kind == "c4":
        arena = torch.empty(alen, dtype=torch.uint8, device=dev)
        c4_fill(torch, arena, offs, files, sizes, dev)
    elif kind == "random":
        g = torch.Generator(device=dev)
        g.manual_seed(5)
        arena = torch.randint(0, 256, (alen,), dtype=torch.uint8, device=dev, generator=g)
    else:
        arena = torch.empty(alen, dtype=torch.uint8, device=dev)
        for j in range(nstreams):
            make_mixed(torch, arena, int(offs[j]), sb, np.random.default_rng(3000 + j), dev)
    ctx = Context.get(oracle.DEFAULT_POLY, oracle.DEFAULT_MIN, oracle.DEFAULT_AVG,
                      oracle.DEFAULT_MAX, device=0)
    plan = DevicePlan(ctx, offs, lens, alen)
    s = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(3):
        plan.run(arena.data_ptr(), s)
    torch.cuda.synchronize()
    plan.set_timing(True, 1)
    for _ in range(5):
        plan.run(arena.data_ptr(), s)
    torch.cuda.synchronize()
    plan.set_timing(False)
    runs, walk_ms, chain_ms = plan.kernel_times()
    st, tr, ct = plan.walk_stats(check_trace=True)
    cuts = plan.results()
    # reference slides (what rabin.rs:127-188 hashes): per chunk that is not the
    # short final one, 63 prefill bytes + (cut - (s + min))
    ref = 0
    for c in cuts:
        prev = np.concatenate([[0], c[:-1]]).astype(np.int64)
        L = c.astype(np.int64) - prev
        full = L >= oracle.DEFAULT_MIN
        ref += int(np.sum(L[full] - oracle.DEFAULT_MIN)) + 63 * int(np.count_nonzero(full))
    t0 = tr[:, 0].astype(np.int64)
    t1 = tr[:, 1].astype(np.int64)
    base = t0.min()
    a, b = (t0 - base) / 100.0, (t1 - base) / 100.0  # us (100 MHz wall clock)
    span = b.max()
    dur = b - a
    slots = 256 * 16
    ev = np.concatenate([np.stack([a, np.ones_like(a)], 1), np.stack([b, -np.ones_like(b)], 1)])
    ev = ev[np.argsort(ev[:, 0], kind="stable")]
    active = np.cumsum(ev[:, 1])
    tt = ev[:, 0]
    dt = np.diff(np.concatenate([tt, [span]]))
    below = {k: float(np.sum(dt[active < k])) for k in (4096, 2048, 1024, 256, 64)}
    rounds = tr[:, 2].astype(np.float64)
    rr = dur / np.maximum(rounds, 1)
    lane_bytes = st["round_bytes"] + st["zones"] * 64 * 64
    # list scheduling of the measured durations on 4096 slots: the queue's
    # own order vs longest-first (what a perfect cost-ordered queue would give)
    import heapq

    def makespan(durs):
        h = [0.0] * slots
        for x in durs:
            t = heapq.heappop(h)
            heapq.heappush(h, t + x)
        return max(h)
    q_order = np.argsort(a, kind="stable")
    sim_queue = makespan(dur[q_order])
    sim_lpt = makespan(np.sort(dur)[::-1])
    top = np.argsort(dur)[::-1][:8]
    longest = [{"unit": int(i), "start_us": round(float(a[i]), 1), "us": round(float(dur[i]), 1),
                "rounds": int(tr[i, 2]), "chunks": int(tr[i, 3])} for i in top]
    # the check kernel: per boundary (rows with t0 = 0 are first pieces)
    cv = ct[:, 0] > 0
    c0 = ct[cv, 0].astype(np.int64)
    c1 = ct[cv, 1].astype(np.int64)
    cb = c0.min()
    cdur = (c1 - c0) / 100.0
    crounds = ct[cv, 2].astype(np.int64)
    check = {
        "boundaries": int(cv.sum()), "span_us": float((c1.max() - cb) / 100.0),
        "us_p50_p90_p99_max": [float(np.percentile(cdur, q)) for q in (50, 90, 99)] + [float(cdur.max())],
        "with_gap_rounds": int(np.count_nonzero(crounds)),
        "us_p50_with_rounds": float(np.median(cdur[crounds > 0])) if np.any(crounds) else None,
        "us_p50_without_rounds": float(np.median(cdur[crounds == 0])),
        "rounds_max": int(crounds.max()),
        "last_start_us": float((c0.max() - cb) / 100.0),
        "walk_end_to_check_start_us": float((cb - (t1.max())) / 100.0),
    }
    out = {
        "kind": kind, "streams": nstreams, "gib_per_stream": sgib,
        "check": check,
        "sim_makespan_queue_order_us": round(sim_queue, 1),
        "sim_makespan_longest_first_us": round(sim_lpt, 1),
        "longest_pieces": longest,
        "walk_ms": walk_ms / runs, "chain_ms": chain_ms / runs,
        "stats": st, "pieces": int(len(tr)),
        "ref_slide_bytes": ref, "lane_slide_bytes": lane_bytes,
        "ref_over_lane": ref / max(lane_bytes, 1),
        "ref_tb_s_walk": ref / (walk_ms / runs / 1e3) / 1e12,
        "lane_tb_s_walk": lane_bytes / (walk_ms / runs / 1e3) / 1e12,
        "trace_span_us": float(span),
        "slot_utilisation": float(dur.sum() / (slots * span)),
        "us_with_active_below": below,
        "piece_us_p50_p90_max": [float(np.percentile(dur, 50)), float(np.percentile(dur, 90)),
                                 float(dur.max())],
        "us_per_round_median": float(np.median(rr[rounds > 4])) if np.any(rounds > 4) else None,
        "rounds_per_piece_mean": float(rounds.mean()),
        "last_piece_start_us": float(a.max()),
    }
    print(json.dumps(out), flush=True)
    if os.environ.get("WALK_TRACE_NPZ"):  # raw per-piece trace for offline analysis
        np.savez_compressed(os.environ["WALK_TRACE_NPZ"] + f"_{kind}.npz", trace=tr, check=ct,
                            lens=np.asarray(lens, np.uint64))
    plan.close()
    del arena
    torch.cuda.empty_cache()


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "both"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    g = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
    for k in (["mixed", "random"] if which == "both" else [which]):
        run(k, n, g)
