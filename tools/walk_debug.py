"""Small walk-path case with stage-by-stage sync (RCDC_DEBUG_SYNC)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("RCDC_DEBUG_SYNC", "1")
os.environ.setdefault("RCDC_WALK_PIECE", str(256 << 10))
os.environ.setdefault("RCDC_WALK_MIN_PIECES", "1")
import numpy as np, torch
from oracle import oracle
from rustic_core_amd.chunker import Context
from rustic_core_amd.device import DevicePlan, pack_offsets
mn, avg, mx = 8 << 10, 16 << 10, 64 << 10
n = int(sys.argv[1]) if len(sys.argv) > 1 else (1 << 20)
kind = sys.argv[2] if len(sys.argv) > 2 else "rand"
data = np.random.default_rng(1).integers(0, 256, n, dtype=np.uint8) if kind == "rand" else np.zeros(n, np.uint8)
ctx = Context.get(oracle.DEFAULT_POLY, mn, avg, mx, device=0)
offs, alen = pack_offsets([n])
host = np.zeros(alen, np.uint8); host[:n] = data
dev = torch.from_numpy(host).to("cuda:0")
plan = DevicePlan(ctx, offs, [n], alen)
print("info", plan.info(), flush=True)
plan.run(dev.data_ptr())
torch.cuda.synchronize()
print("ran", flush=True)
got = plan.results()[0]
exp = oracle.chunk_cuts(data, oracle.DEFAULT_POLY, mn, avg, mx)
print("cuts", len(got), len(exp), "equal", np.array_equal(got, exp), flush=True)
if not np.array_equal(got, exp):
    k = min(len(got), len(exp)); d = np.nonzero(got[:k] != exp[:k])[0]
    i = int(d[0]) if len(d) else k
    print("first diff", i, got[max(0,i-3):i+3], exp[max(0,i-3):i+3])
