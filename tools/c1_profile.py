import cProfile, pstats, io, os, sys, time, tempfile
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np
import torch
torch.zeros(1).cuda()
from bench import stdrng_numpy
from rustic_core_amd import ChunkIter, ConfigFile
n = 256 << 20
data = stdrng_numpy(0x256, n)
path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "c1prof.bin")
open(path, "wb").write(data.tobytes())
cfg = ConfigFile.new(2, 0x003DA3358B4DC173)
def one():
    k = 0
    with open(path, "rb") as f:
        for c in ChunkIter.from_config(cfg, f, n):
            k += len(c)
    return k
one()
t0 = time.perf_counter(); one(); print("pass s", time.perf_counter() - t0, flush=True)
pr = cProfile.Profile(); pr.enable(); one(); pr.disable()
s = io.StringIO(); pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(25); print(s.getvalue())
