"""Wall time per C2 step with and without the per-step HIP timing events.

usage: python tools/step_gaps.py [steps]
Prints us/step for plan.run() back to back (timing off), with the scan /
resolve HIP events on (rcdc_plan_set_timing), and the event-measured kernel
times, so the inter-kernel gaps the events add can be read off.
"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from rustic_core_amd.chunker import Context
from rustic_core_amd.device import DevicePlan, pack_offsets

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
n, sb = 1024, 1 << 20
lens = np.full(n, sb, np.uint64); offs, alen = pack_offsets(lens)
g = torch.Generator(device="cuda"); g.manual_seed(1000)
arena = torch.randint(0, 256, (alen,), dtype=torch.uint8, device="cuda", generator=g)
ctx = Context.get(0x003DA3358B4DC173, 512 << 10, 1 << 20, 8 << 20, device=0)
plan = DevicePlan(ctx, offs, lens, alen)
ptr = arena.data_ptr()
sptr = torch.cuda.current_stream().cuda_stream
for _ in range(20):
    plan.run(ptr, sptr)
torch.cuda.synchronize()
for rep in range(3):
    for timing in (False, True):
        plan.set_timing(timing)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            plan.run(ptr, sptr)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        extra = ""
        if timing:
            runs, sms, rms = plan.kernel_times()
            extra = f"  scan {sms / runs * 1e3:.1f} us  resolve {rms / runs * 1e3:.1f} us"
        plan.set_timing(False)
        print(f"timing={int(timing)}: {el / steps * 1e6:.1f} us/step{extra}", flush=True)
