"""Re-run one walk-path test case with RCDC_WALK_DUMP (piece lists, boundary
results) and print where the device cuts first differ from the oracle."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("RCDC_WALK_PIECE", str(256 << 10))
os.environ.setdefault("RCDC_WALK_MIN_PIECES", "1")
import numpy as np, torch
from oracle import oracle
from rustic_core_amd.chunker import Context
from rustic_core_amd.device import DevicePlan, pack_offsets
mn, avg, mx = 8 << 10, 16 << 10, 64 << 10
seed, n = int(sys.argv[1]), int(sys.argv[2])
data = np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8)
ctx = Context.get(oracle.DEFAULT_POLY, mn, avg, mx, device=0)
offs, alen = pack_offsets([n])
host = np.zeros(alen, np.uint8); host[:n] = data
dev = torch.from_numpy(host).to("cuda:0")
plan = DevicePlan(ctx, offs, [n], alen)
plan.run(dev.data_ptr()); torch.cuda.synchronize()
os.environ["RCDC_WALK_DUMP"] = "0"
got = plan.results()[0]
exp = oracle.chunk_cuts(data, oracle.DEFAULT_POLY, mn, avg, mx)
print("equal", np.array_equal(got, exp), len(got), len(exp), flush=True)
k = min(len(got), len(exp)); d = np.nonzero(got[:k] != exp[:k])[0]
if len(d) or len(got) != len(exp):
    i = int(d[0]) if len(d) else k
    print("first diff", i, got[max(0, i - 3):i + 3], exp[max(0, i - 3):i + 3])
