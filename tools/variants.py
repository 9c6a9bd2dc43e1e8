"""A/B the scan-kernel variants (RCDC_SCAN_VARIANT) in one process, interleaved.

usage: python tools/variants.py [variants...]   (default 0 1 2 3)
Prints per-variant median scan-kernel time (HIP events) on the C2 workload
and checks every variant's cut lists against variant 0's.
"""
import os, sys, statistics
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from rustic_core_amd.chunker import Context
from rustic_core_amd.device import DevicePlan, pack_offsets

variants = [int(x) for x in sys.argv[1:]] or [0, 1, 2, 3]
n = int(os.environ.get("RCDC_STREAMS", "1024")); sb = int(os.environ.get("RCDC_STREAM_BYTES", str(1 << 20)))
lens = np.full(n, sb, np.uint64); offs, alen = pack_offsets(lens)
g = torch.Generator(device="cuda"); g.manual_seed(1000)
arena = torch.randint(0, 256, (alen,), dtype=torch.uint8, device="cuda", generator=g)
if os.environ.get("RCDC_ZEROS"):
    arena.zero_()
plans = {}
for v in variants:
    os.environ["RCDC_SCAN_VARIANT"] = str(v)
    ctx = Context(0x003DA3358B4DC173, 512 << 10, 1 << 20, 8 << 20, device=0)
    plans[v] = (ctx, DevicePlan(ctx, offs, lens, alen))
ref = None
for v, (ctx, p) in plans.items():
    p.run(arena.data_ptr()); r = p.results()
    if ref is None: ref = r
    ok = all(np.array_equal(a, b) for a, b in zip(r, ref))
    print(f"variant {v}: info {p.info()} parity_vs_first={ok}")
times = {v: [] for v in variants}
for rnd in range(5):
    for v, (ctx, p) in plans.items():
        p.set_timing(True)
        for _ in range(10):
            p.run(arena.data_ptr())
        torch.cuda.synchronize()
        runs, sms, rms = p.kernel_times()
        p.set_timing(False)
        times[v].append(sms / runs * 1e3)
hashed = n * max(sb - (512 << 10), 0)
for v in variants:
    med = statistics.median(times[v])
    print(f"variant {v}: scan median {med:.1f} us  min {min(times[v]):.1f}  -> {hashed/med/1e3:.0f} GB/s hashed")
