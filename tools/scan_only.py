"""Runs only the C2 scan+resolve launches (for rocprofv3 PMC passes)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from rustic_core_amd.chunker import Context
from rustic_core_amd.device import DevicePlan, pack_offsets
n = int(os.environ.get("RCDC_STREAMS", "1024")); sb = 1 << 20
lens = np.full(n, sb, np.uint64); offs, alen = pack_offsets(lens)
g = torch.Generator(device="cuda"); g.manual_seed(1000)
arena = torch.randint(0, 256, (alen,), dtype=torch.uint8, device="cuda", generator=g)
if os.environ.get("RCDC_ZEROS"): arena.zero_()
ctx = Context.get(0x003DA3358B4DC173, 512 << 10, 1 << 20, 8 << 20, device=0)
plan = DevicePlan(ctx, offs, lens, alen)
for _ in range(int(os.environ.get("RCDC_REPS", "5"))):
    plan.run(arena.data_ptr())
torch.cuda.synchronize()
print("ok", plan.info())
