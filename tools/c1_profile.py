"""Where C1's drop-in time goes (bench.py run_c1's file through
ChunkIter.from_config): wall time split into the file reads (_read_into),
the device feeds (_Stream.feed: H2D, chunking, cuts D2H) and the rest
(chunk copies, Python).  Prints one JSON line.

  python tools/c1_profile.py [--mib 256] [--passes 5]
"""
import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (the C1 input generator)
from rustic_core_amd import ChunkIter, ConfigFile, chunker  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--mib", type=int, default=256)
ap.add_argument("--passes", type=int, default=5)
a = ap.parse_args()
n = a.mib << 20
data = bench.stdrng_numpy(0x256, n)
fd, path = tempfile.mkstemp(prefix="rcdc_c1p_", dir=os.environ.get("TMPDIR", "/tmp"))
with os.fdopen(fd, "wb") as f:
    f.write(data.tobytes())
acc = {"read_s": 0.0, "feed_s": 0.0}
orig_read, orig_feed = chunker._read_into, chunker._Stream.feed


def t_read(*x, **k):
    t = time.perf_counter()
    try:
        return orig_read(*x, **k)
    finally:
        acc["read_s"] += time.perf_counter() - t


def t_feed(self, *x, **k):
    t = time.perf_counter()
    try:
        return orig_feed(self, *x, **k)
    finally:
        acc["feed_s"] += time.perf_counter() - t


chunker._read_into, chunker._Stream.feed = t_read, t_feed
cfg = ConfigFile.new(2, bench.POLY)
try:
    def one_pass():
        with open(path, "rb") as f:
            return sum(1 for _ in ChunkIter.from_config(cfg, f, n))
    one_pass()
    acc["read_s"] = acc["feed_s"] = 0.0
    t0 = time.perf_counter()
    for _ in range(a.passes):
        one_pass()
    wall = time.perf_counter() - t0
finally:
    os.unlink(path)
out = {"mib": a.mib, "passes": a.passes, "gibs": round(n * a.passes / wall / 2**30, 3),
       "wall_ms_per_pass": round(wall / a.passes * 1e3, 2),
       "read_ms_per_pass": round(acc["read_s"] / a.passes * 1e3, 2),
       "feed_ms_per_pass": round(acc["feed_s"] / a.passes * 1e3, 2)}
out["rest_ms_per_pass"] = round(out["wall_ms_per_pass"] - out["read_ms_per_pass"] - out["feed_ms_per_pass"], 2)
print(json.dumps(out))
