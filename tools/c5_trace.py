"""Where a C5 step goes (one all-zero stream, bench.py --workload C5 at N = 1):
the walk and chain kernels' HIP-event times, pipelined and serial, and the
per-piece / per-boundary wall-clock traces (RCDC_WALK_TRACE=1) of the last
run: walk span, the check kernel's first-boundary delay (its prologue) and
per-boundary durations.

usage: python tools/c5_trace.py [GiB]   (default 12.5)
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["RCDC_WALK_TRACE"] = "1"

from oracle import oracle  # noqa: E402
from rustic_core_amd.chunker import Context  # noqa: E402
from rustic_core_amd.device import DevicePlan  # noqa: E402


def main():
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 12.5
    dev = torch.device("cuda", 0)
    n = int(gib * (1 << 30))
    arena = torch.zeros(n + 256, dtype=torch.uint8, device=dev)
    ctx = Context.get(oracle.DEFAULT_POLY, oracle.DEFAULT_MIN, oracle.DEFAULT_AVG,
                      oracle.DEFAULT_MAX, device=0)
    out = {}
    for mode in ("pipelined", "serial"):
        plan = DevicePlan(ctx, np.zeros(1, np.uint64), np.array([n], np.uint64), n + 256)
        plan.set_pipeline(mode == "pipelined")
        s = torch.cuda.current_stream(dev).cuda_stream
        for _ in range(20):
            plan.run(arena.data_ptr(), s)
        torch.cuda.synchronize()
        plan.set_timing(True, 1)
        steps = 50
        t0 = time.perf_counter()
        for i in range(steps):
            if mode == "pipelined" and i == steps - 1:
                plan.flush_next()
            plan.run(arena.data_ptr(), s)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        plan.set_timing(False)
        runs, walk_ms, chain_ms = plan.kernel_times()
        st, tr, ct = plan.walk_stats(check_trace=True)
        w0, w1 = tr[:, 0].astype(np.int64), tr[:, 1].astype(np.int64)
        cv = ct[:, 0] > 0
        c0, c1 = ct[cv, 0].astype(np.int64), ct[cv, 1].astype(np.int64)
        base = w0.min()
        cd = (c1 - c0) / 100.0
        out[mode] = {
            "ms_per_step": round(el / steps * 1e3, 4),
            "walk_us": round(walk_ms / runs * 1e3, 1), "chain_us": round(chain_ms / runs * 1e3, 1),
            "walk_trace_span_us": round((w1.max() - base) / 100.0, 1),
            "walk_piece_us_p50_max": [round(float(np.median((w1 - w0) / 100.0)), 2),
                                      round(float(((w1 - w0) / 100.0).max()), 2)],
            "check_first_start_after_walk_start_us": round((c0.min() - base) / 100.0, 1),
            "check_first_start_after_walk_end_us": round((c0.min() - w1.max()) / 100.0, 1),
            "check_span_us": round((c1.max() - c0.min()) / 100.0, 1),
            "check_boundary_us_p50_p99_max": [round(float(np.percentile(cd, q)), 2)
                                              for q in (50, 99, 100)],
            "boundaries": int(cv.sum()), "pieces": int(len(tr)),
            "chk_zones": st["chk_zones"], "chk_rounds": st["chk_rounds"], "zones": st["zones"],
        }
        plan.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
