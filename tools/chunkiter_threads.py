"""Many ChunkIter.from_config iterators at once, one per worker thread (the
archiver's per-file parallelism, archiver.rs:195): T threads, each chunking
F in-memory files of M MiB; prints aggregate GiB/s and checks every file's
chunks concatenate back to its bytes.

  python tools/chunkiter_threads.py [--threads 16] [--files 4] [--mib 64]
"""
import argparse
import io
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rustic_core_amd import ChunkIter, ConfigFile  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--threads", type=int, default=16)
ap.add_argument("--files", type=int, default=4)
ap.add_argument("--mib", type=int, default=64)
ap.add_argument("--passes", type=int, default=3)
a = ap.parse_args()
cfg = ConfigFile.new(2, 0x003DA3358B4DC173)
rng = np.random.default_rng(1)
data = [rng.integers(0, 256, a.mib << 20, dtype=np.uint8).tobytes() for _ in range(a.threads)]


def work(t):
    ok, n = True, 0
    for _ in range(a.files):
        chunks = list(ChunkIter.from_config(cfg, io.BytesIO(data[t]), len(data[t])))
        ok &= sum(len(c) for c in chunks) == len(data[t])
        n += len(data[t])
    return ok, n


with ThreadPoolExecutor(a.threads) as pool:
    list(pool.map(work, range(a.threads)))  # warm
    t0 = time.perf_counter()
    for _ in range(a.passes):
        res = list(pool.map(work, range(a.threads)))
    el = time.perf_counter() - t0
tot = sum(n for _, n in res) * a.passes
print(json.dumps({"threads": a.threads, "files_per_thread": a.files, "mib": a.mib,
                  "gibs": round(tot / el / 2**30, 2), "all_ok": all(ok for ok, _ in res),
                  "block_pool": os.environ.get("RCDC_BLOCK_POOL", "32")}))
