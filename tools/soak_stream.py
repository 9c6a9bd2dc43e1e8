"""Randomised soak of the streaming drop-in paths against the CPU oracle
(test infrastructure: the oracle is the checker).  Each case draws chunker
parameters and 1-6 inputs (empty to 48 MiB: random, zeros, text, runs), and
runs them concurrently on threads sharing one context through:
  - ChunkIter.from_config over a reader: BytesIO, BufferedReader, a raw
    reader with short reads of random sizes, one that raises
    InterruptedError now and then (rabin.rs:173 retries), or a file on
    disk; the large-file pipe on or off, with 2-6 blocks;
  - rcdc_stream_feed directly (the _Stream wrapper) with random piece sizes.
Every chunk's bytes are compared with the oracle's cut list on the same
input.  Exits 1 on a mismatch with the case's seed.

  python tools/soak_stream.py [seconds] [seed]
"""
import io
import json
import os
import sys
import tempfile
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from oracle import oracle  # noqa: E402
from soak import POLYS  # noqa: E402
from soak_ingest import PARAMS, gen  # noqa: E402

KiB, MiB = 1 << 10, 1 << 20


class Short(io.RawIOBase):
    """readinto returns 1..k bytes; every `intr`-th call raises EINTR first."""

    def __init__(self, data, k, seed, intr=0):
        self._b, self._k = io.BytesIO(data), k
        self._r = np.random.default_rng(seed)
        self._intr, self._calls = intr, 0

    def readable(self):
        return True

    def readinto(self, mv):
        self._calls += 1
        if self._intr and self._calls % self._intr == 0:
            raise InterruptedError("EINTR")
        b = self._b.read(min(len(mv), int(self._r.integers(1, self._k + 1))))
        mv[:len(b)] = b
        return len(b)


def run_one(ctx, cfg, data, how, seed, tmp, errs):
    from rustic_core_amd import chunker
    try:
        want = oracle.chunk_cuts(data, *cfg)
        if how == "feed":
            st = chunker._Stream(ctx)
            rng = np.random.default_rng(seed)
            got, p = [], 0
            while p < data.size:
                k = min(int(rng.integers(1, 24 * MiB)), data.size - p)
                got.extend(st.feed(data[p:p + k], False).tolist())
                p += k
            got.extend(st.feed(np.zeros(0, np.uint8), True).tolist())
            st.close()
            if not np.array_equal(np.array(got, np.uint64), want):
                errs.append(("feed cuts", seed))
            return
        path = None
        if how == "file":
            path = os.path.join(tmp, f"f{seed}")
            with open(path, "wb") as fh:
                fh.write(data.tobytes())
            reader = open(path, "rb")
        elif how == "bytesio":
            reader = io.BytesIO(data.tobytes())
        elif how == "buffered":
            reader = io.BufferedReader(io.BytesIO(data.tobytes()))
        elif how == "short":
            reader = Short(data.tobytes(), int(np.random.default_rng(seed).integers(64 * KiB, 20 * MiB)),
                           seed)
        else:  # "intr"
            reader = Short(data.tobytes(), 8 * MiB, seed, intr=3)
        try:
            it = chunker.ChunkIter.from_config(cfg_file(cfg), reader, data.size)
            prev = 0
            for j, c in enumerate(it):
                if j >= len(want):
                    errs.append(("extra chunk", seed, how))
                    return
                e = int(want[j])
                if len(c) != e - prev or c != data[prev:e].tobytes():
                    errs.append(("chunk", seed, how, j))
                    return
                prev = e
            if prev != data.size or (data.size and j + 1 != len(want)):
                errs.append(("short", seed, how))
        finally:
            reader.close()
            if path:
                os.unlink(path)
    except BaseException as e:  # noqa: BLE001 (reported, the soak stops)
        errs.append(("raised", seed, how, repr(e)[:300]))


def cfg_file(cfg):
    from rustic_core_amd import ConfigFile
    poly, mn, avg, mx = cfg
    c = ConfigFile.new(2, poly)
    c.chunk_size_, c.chunk_min_size_, c.chunk_max_size_ = avg, mn, mx
    return c


def one_case(seed, tmp):
    from rustic_core_amd import chunker
    from rustic_core_amd.chunker import Context
    rng = np.random.default_rng(seed)
    poly = POLYS[int(rng.integers(0, len(POLYS)))]
    mn, avg, mx = PARAMS[int(rng.integers(0, len(PARAMS)))]
    cfg = (poly, mn, avg, mx)
    ctx = Context.get(poly, mn, avg, mx, device=0)
    chunker.PIPE_BLOCKS = int(rng.integers(2, 7))
    os.environ["RCDC_READ_AHEAD"] = str(int(rng.random() < 0.8))
    jobs = []
    for k in range(int(rng.integers(1, 7))):
        kind = ["random", "zeros", "text", "runs", "runs"][int(rng.integers(0, 5))]
        n = int(rng.choice([0, int(rng.integers(1, 64 * KiB)), int(rng.integers(64 * KiB, 4 * MiB)),
                            int(rng.integers(4 * MiB, 48 * MiB))]))
        how = ["feed", "file", "bytesio", "buffered", "short", "intr"][int(rng.integers(0, 6))]
        jobs.append((gen(rng, kind, n, []), how, seed * 10 + k))
    errs = []
    ts = [threading.Thread(target=run_one, args=(ctx, cfg, d, h, s, tmp, errs)) for d, h, s in jobs]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return {"seed": seed, "inputs": len(jobs), "bytes": int(sum(d.size for d, _, _ in jobs)),
            "hows": [h for _, h, _ in jobs], "errors": errs}


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 300
    seed0 = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    t0 = last = time.time()
    n = nbytes = inputs = 0
    seed = seed0
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as tmp:
        while time.time() - t0 < secs:
            r = one_case(seed, tmp)
            if r["errors"]:
                print(json.dumps({"MISMATCH": r}), flush=True)
                sys.exit(1)
            n += 1
            inputs += r["inputs"]
            nbytes += r["bytes"]
            seed += 1
            if time.time() - last > 30:
                last = time.time()
                print(json.dumps({"cases": n, "inputs": inputs, "gib": round(nbytes / 2**30, 2)}),
                      flush=True)
    print(json.dumps({"soak_stream": "ok", "cases": n, "inputs": inputs,
                      "gib": round(nbytes / 2**30, 2), "seeds": [seed0, seed - 1],
                      "seconds": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
