"""Randomised parity soak of the device chunker against the CPU oracle
(test infrastructure: the oracle is the checker).  Each case draws chunker
parameters, a batch of streams (lengths from empty to tens of MiB, data
kinds: random, zeros, runs of both, a small alphabet, a repeated block,
zero runs sized around min and max), a path (scan only, walk with random
piece sizes, the default choice), the tail helpers on or off, and serial or
pipelined runs; every cut list is diffed against oracle.chunk_many_cuts.
Prints one JSON line per minute and a summary; exits 1 on a mismatch, with
the case's seed to replay it.

  python tools/soak.py [seconds] [seed]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import oracle  # noqa: E402

KiB, MiB = 1 << 10, 1 << 20
POLYS = [oracle.DEFAULT_POLY, (1 << 40) | 0x1B, (1 << 56) | 0x95, 0x3DA3358B4DC173 ^ (1 << 20)]
# (min, avg, max): rustic's default, and smaller ones that put many chunks,
# zones and piece boundaries into every MiB (a bounded set: one context each)
PARAMS = [(512 * KiB, 1 * MiB, 8 * MiB), (4 * KiB, 8 * KiB, 64 * KiB), (8 * KiB, 16 * KiB, 64 * KiB),
          (16 * KiB, 64 * KiB, 256 * KiB), (64 * KiB, 256 * KiB, 1 * MiB), (64 * KiB, 64 * KiB, 128 * KiB),
          (128 * KiB, 1 * MiB, 2 * MiB), (256 * KiB, 512 * KiB, 4 * MiB)]


def gen(rng, n, kind, mn, mx):
    if kind == "random":
        return rng.integers(0, 256, n, dtype=np.uint8)
    if kind == "zeros":
        return np.zeros(n, np.uint8)
    if kind == "alphabet":  # low entropy: many candidate windows repeat
        return rng.choice(np.array([0, 1, 32, 255], np.uint8), n)
    if kind == "block":  # a repeated block: periodic windows
        b = rng.integers(0, 256, int(rng.integers(64, 8192)), dtype=np.uint8)
        return np.resize(b, n)
    # runs of random and zero bytes, zero runs sized around min / max
    out = np.zeros(n, np.uint8)
    p = 0
    while p < n:
        r = int(rng.integers(1, 4 * mn))
        out[p:p + r] = rng.integers(0, 256, min(r, n - p), dtype=np.uint8)
        p += r
        z = int(rng.choice([mn - 64, mn, mn + 1, mx - 1, mx, 2 * mx + 7, int(rng.integers(1, 3 * mx))]))
        p += max(z, 0)
    return out


def one_case(seed, torch):
    from rustic_core_amd.chunker import Context, check_rabin_params
    from rustic_core_amd.device import DevicePlan, pack_offsets
    rng = np.random.default_rng(seed)
    poly = POLYS[int(rng.integers(0, len(POLYS)))]
    mn, avg, mx = PARAMS[int(rng.integers(0, len(PARAMS)))]
    check_rabin_params(avg, mn, mx)
    nstreams = int(rng.integers(1, 48))
    lens = []
    for _ in range(nstreams):
        c = rng.random()
        lens.append(int(rng.integers(0, mn + 2)) if c < 0.2 else
                    int(rng.integers(mn, 4 * mx)) if c < 0.6 else
                    int(rng.integers(4 * mx, max(24 * MiB, 8 * mx))))
    while sum(lens) > 384 * MiB:
        lens.pop()
    kinds = ["random", "zeros", "alphabet", "block", "runs", "runs", "random"]
    bufs = [gen(rng, n, kinds[int(rng.integers(0, len(kinds)))], mn, mx) for n in lens]
    path = rng.choice(["default", "scan", "walk"])
    env = {"RCDC_WALK_HELP": str(int(rng.integers(0, 2)))}
    if path == "scan":
        env["RCDC_WALK_PIECE"] = "0"
    elif path == "walk":
        env["RCDC_WALK_PIECE"] = str(int(mn * int(rng.integers(2, 40))))
        env["RCDC_WALK_MIN_PIECES"] = "1"
    for k, v in env.items():
        os.environ[k] = v
    try:
        ctx = Context.get(poly, mn, avg, mx, device=0)
        offs, alen = pack_offsets(lens)
        host = np.zeros(alen, np.uint8)
        for o, b in zip(offs, bufs):
            host[int(o):int(o) + len(b)] = b
        dev = torch.from_numpy(host).to("cuda:0")
        plan = DevicePlan(ctx, offs, lens, alen)
        info = plan.info()
        pipelined = bool(rng.integers(0, 2))
        runs = 1
        if pipelined:
            plan.set_pipeline(True)
            runs = int(rng.integers(2, 4))
            for r in range(runs):
                if r == runs - 1:
                    plan.flush_next()
                plan.run(dev.data_ptr())
        else:
            plan.run(dev.data_ptr())
        got = plan.results()
        plan.close()
    finally:
        for k in env:
            os.environ.pop(k, None)
    want = oracle.chunk_many_cuts(host, [int(o) for o in offs], lens, poly, mn, avg, mx,
                                  nthreads=16)
    bad = [i for i in range(len(lens)) if not np.array_equal(got[i], want[i])]
    return {"seed": seed, "poly": hex(poly), "min": mn, "avg": avg, "max": mx,
            "streams": len(lens), "bytes": int(sum(lens)), "path": str(path),
            "walk_pieces": int(info.get("walk_pieces", 0)), "pipelined": pipelined,
            "env": env, "cuts": int(sum(len(w) for w in want)), "bad": bad}


def main():
    import torch
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 300
    seed0 = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    t0 = last = time.time()
    n = cuts = nbytes = walked = 0
    seed = seed0
    while time.time() - t0 < secs:
        r = one_case(seed, torch)
        n += 1
        cuts += r["cuts"]
        nbytes += r["bytes"]
        walked += r["walk_pieces"] > 0
        if r["bad"]:
            print(json.dumps({"MISMATCH": r}), flush=True)
            sys.exit(1)
        seed += 1
        if time.time() - last > 60:
            last = time.time()
            print(json.dumps({"cases": n, "walked": walked, "cuts": cuts,
                              "gib": round(nbytes / 2**30, 2)}), flush=True)
    print(json.dumps({"soak": "ok", "cases": n, "walked": walked, "cuts_diffed": cuts,
                      "gib": round(nbytes / 2**30, 2), "seeds": [seed0, seed - 1],
                      "seconds": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
