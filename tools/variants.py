"""A/B scan-kernel configurations in one process, interleaved.

usage: python tools/variants.py [spec...]      (default 41 30)
spec = CODE[:aALIGN][:sSEG]  e.g. 41  41:a128  30:a128:s2176
  CODE  rcdc_scan.hip launch_scan configuration (RCDC_SCAN_VARIANT)
  ALIGN lane-start alignment of the plan (RCDC_Q0_ALIGN)
  SEG   segment bytes (RCDC_SEG_BYTES)
Prints per-spec median / p10 / min scan-kernel time (HIP events) on the C2
workload (env RCDC_STREAMS, RCDC_STREAM_BYTES, RCDC_ZEROS, RCDC_ROUNDS) and
checks every spec's cut lists against the first one's.
"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from rustic_core_amd.chunker import Context
from rustic_core_amd.device import DevicePlan, pack_offsets

specs = sys.argv[1:] or ["41", "30"]
n = int(os.environ.get("RCDC_STREAMS", "1024")); sb = int(os.environ.get("RCDC_STREAM_BYTES", str(1 << 20)))
rounds = int(os.environ.get("RCDC_ROUNDS", "12"))
lens = np.full(n, sb, np.uint64); offs, alen = pack_offsets(lens)
g = torch.Generator(device="cuda"); g.manual_seed(1000)
arena = torch.randint(0, 256, (alen,), dtype=torch.uint8, device="cuda", generator=g)
if os.environ.get("RCDC_ZEROS"):
    arena.zero_()
plans = {}
for spec in specs:
    parts = spec.split(":")
    os.environ["RCDC_SCAN_VARIANT"] = parts[0]
    os.environ.pop("RCDC_Q0_ALIGN", None); os.environ.pop("RCDC_SEG_BYTES", None)
    for p in parts[1:]:
        if p[0] == "a": os.environ["RCDC_Q0_ALIGN"] = p[1:]
        if p[0] == "s": os.environ["RCDC_SEG_BYTES"] = p[1:]
    ctx = Context(0x003DA3358B4DC173, 512 << 10, 1 << 20, 8 << 20, device=0)
    plans[spec] = (ctx, DevicePlan(ctx, offs, lens, alen))
for k in ("RCDC_Q0_ALIGN", "RCDC_SEG_BYTES"):
    os.environ.pop(k, None)
ref = None
for spec, (ctx, p) in plans.items():
    p.run(arena.data_ptr()); r = p.results()
    if ref is None: ref = r
    ok = all(np.array_equal(a, b) for a, b in zip(r, ref))
    i = p.info()
    print(f"{spec:>16}: S {i['segment_bytes']} items {i['work_items']} parity_vs_first={ok}")
times = {s: [] for s in specs}
for rnd in range(rounds):
    for spec, (ctx, p) in plans.items():
        p.set_timing(True)
        for _ in range(10):
            p.run(arena.data_ptr())
        torch.cuda.synchronize()
        runs, sms, rms = p.kernel_times()
        p.set_timing(False)
        times[spec].append(sms / runs * 1e3)
hashed = sum(max(int(x) - (512 << 10), 0) for x in lens)
for spec in specs:
    t = np.array(times[spec])
    print(f"{spec:>16}: scan median {np.median(t):.1f} us  p10 {np.percentile(t, 10):.1f}  min {t.min():.1f}"
          f"  -> {hashed / np.median(t) / 1e3:.0f} GB/s hashed")
