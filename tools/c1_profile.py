"""Where a C1 pass goes (one 256 MiB file through ChunkIter.from_config):
wall time per pass, and the time inside the reader thread's reads, the
device stream feeds and the chunk copies (wrapped in place; the sums
overlap: large files run as a pipe of reader, feeder and consumer threads).

  python tools/c1_profile.py [MiB] [passes]
"""
import os
import sys
import tempfile
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from rustic_core_amd import ChunkIter, ConfigFile  # noqa: E402
from rustic_core_amd import chunker  # noqa: E402

acc = {"read": 0.0, "read_n": 0, "feed": 0.0, "feed_n": 0, "take": 0.0, "take_n": 0}
lock = threading.Lock()


def wrap(obj, name, key):
    f = getattr(obj, name)

    def g(*a, **k):
        t = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            with lock:
                acc[key] += time.perf_counter() - t
                acc[key + "_n"] += 1
    setattr(obj, name, g)


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    passes = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    n = mib << 20
    data = np.random.default_rng(7).integers(0, 256, n, dtype=np.uint8)
    fd, path = tempfile.mkstemp(prefix="rcdc_c1p_", dir=os.environ.get("TMPDIR", "/tmp"))
    with os.fdopen(fd, "wb") as f:
        f.write(data.tobytes())
    cfg = ConfigFile.new(2, 0x003DA3358B4DC173)

    def one():
        k = 0
        with open(path, "rb") as f:
            for c in ChunkIter.from_config(cfg, f, n):
                k += len(c)
        assert k == n

    one()
    one()
    # the plain sequential read of the file alone (page cache, 16 MiB reads)
    buf = bytearray(16 << 20)
    t = time.perf_counter()
    for _ in range(passes):
        with open(path, "rb", buffering=0) as f:
            while f.readinto(buf):
                pass
    t_read = (time.perf_counter() - t) / passes
    wrap(chunker, "_read_into", "read")
    wrap(chunker._Stream, "feed", "feed")
    wrap(chunker.RabinChunkIter, "_take", "take")
    t = time.perf_counter()
    for _ in range(passes):
        one()
    el = (time.perf_counter() - t) / passes
    os.unlink(path)
    out = {"mib": mib, "ms_per_pass": round(el * 1e3, 2), "gibs": round(n / el / 2**30, 2),
           "plain_read_ms": round(t_read * 1e3, 2)}
    for k in ("read", "feed", "take"):
        out[k + "_ms_per_pass"] = round(acc[k] / passes * 1e3, 2)
        out[k + "_calls_per_pass"] = acc[k + "_n"] // passes
    print(out)


if __name__ == "__main__":
    main()
