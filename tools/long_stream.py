"""Scan / resolve timing on long streams (C3 / C5 shapes), parity vs oracle.

usage: python tools/long_stream.py [GiB_per_stream] [n_streams] [case,case..]
Cases: random, zeros, mixed (random runs 64 KiB-16 MiB + zero runs 4 KiB-16 MiB).
"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from oracle import oracle
from rustic_core_amd.chunker import Context
from rustic_core_amd.device import DevicePlan, pack_offsets

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
ns = int(sys.argv[2]) if len(sys.argv) > 2 else 1
n = int(gib * (1 << 30))
ctx = Context.get(oracle.DEFAULT_POLY, oracle.DEFAULT_MIN, oracle.DEFAULT_AVG, oracle.DEFAULT_MAX, device=0)


def mixed(dev_arr, off, length, rng):
    pos = 0
    while pos < length:
        if rng.random() < 0.5:
            L = int(np.exp(rng.uniform(np.log(64 << 10), np.log(16 << 20))))
            L = min(L, length - pos)
            dev_arr[off + pos: off + pos + L] = torch.randint(0, 256, (L,), dtype=torch.uint8, device="cuda")
        else:
            L = int(np.exp(rng.uniform(np.log(4 << 10), np.log(16 << 20))))
            L = min(L, length - pos)
            dev_arr[off + pos: off + pos + L] = 0
        pos += L


cases = sys.argv[3].split(",") if len(sys.argv) > 3 else ["random", "zeros", "mixed"]
for case in cases:
    lens = [n] * ns
    offs, alen = pack_offsets(lens)
    arena = torch.zeros(alen, dtype=torch.uint8, device="cuda")
    rng = np.random.default_rng(3000)
    for i in range(ns):
        o = int(offs[i])
        if case == "random":
            arena[o:o + n] = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
        elif case == "mixed":
            mixed(arena, o, n, rng)
    plan = DevicePlan(ctx, offs, lens, alen)
    plan.run(arena.data_ptr()); torch.cuda.synchronize()
    plan.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(3):
        plan.run(arena.data_ptr())
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / 3
    runs, sms, rms = plan.kernel_times()
    plan.set_timing(False)
    got = plan.results()
    host = arena.cpu().numpy()
    bad = 0
    for i in range(ns):
        o = int(offs[i])
        exp = oracle.chunk_cuts(host[o:o + n])
        bad += not np.array_equal(got[i], exp)
    ncuts = sum(len(g) for g in got)
    print(f"{case:6s} {ns} x {gib} GiB: step {el*1e3:.2f} ms  scan {sms/runs:.2f} ms  resolve {rms/runs:.2f} ms "
          f"cuts {ncuts}  resolve/cut {rms/runs*1e3/max(ncuts,1):.2f} us  -> {ns*n/el/2**30:.1f} GiB/s  mismatches {bad}",
          flush=True)
    plan.close()
    del arena
    torch.cuda.empty_cache()
