"""Randomised soak of the native ingest engine (rcdc_ingest_* through
ctypes) against the oracle and hashlib (test infrastructure: the checks of
tests/test_gpu_native_ingest.py _check_all).  Each case draws chunker
parameters, 2-12 files (empty to 40 MiB; random, zeros, text, runs, copies
and prefixes of earlier files), how each file goes in (rcdc_ingest_add,
add_stream with short reads and random piece sizes, or from a file on disk),
the engine shape (batch_bytes 1-64 MiB, depth, slots, streams, long-chunk
threshold, pack size and grow factor) and the zstd level (stored blobs,
0 = default, 1, 3, 7), and checks every cut, chunk id, pack id, pack header,
blob and dedup decision.  Exits 1 on a mismatch with the case's seed.

  python tools/soak_ingest.py [seconds] [seed]
"""
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

sys.path.insert(0, os.path.join(ROOT, "tools"))
from tests.test_gpu_native_ingest import KEY, _check_all  # noqa: E402
from tests.test_gpu_ingest_streams import ChoppyReader  # noqa: E402
from soak import POLYS  # noqa: E402

KiB, MiB = 1 << 10, 1 << 20
PARAMS = [(512 * KiB, 1 * MiB, 8 * MiB), (64 * KiB, 256 * KiB, 1 * MiB), (16 * KiB, 64 * KiB, 256 * KiB),
          (128 * KiB, 512 * KiB, 2 * MiB)]


def gen(rng, kind, n, earlier):
    if kind == "copy" and earlier:
        src = earlier[int(rng.integers(0, len(earlier)))]
        return src[:int(rng.integers(0, src.size + 1))].copy()
    if kind == "zeros":
        return np.zeros(n, np.uint8)
    if kind == "text":
        return np.resize(np.frombuffer(b"id,name,value\n17,alpha,3.25\n", np.uint8), n).copy()
    if kind == "runs":
        out = np.zeros(n, np.uint8)
        p = 0
        while p < n:
            k = int(rng.integers(4 * KiB, 3 * MiB))
            if rng.random() < 0.5:
                out[p:p + k] = rng.integers(0, 256, len(out[p:p + k]), dtype=np.uint8)
            p += k
        return out
    return rng.integers(0, 256, n, dtype=np.uint8)


def one_case(seed, tmp):
    from rustic_core_amd.chunker import Context
    from rustic_core_amd.native_ingest import NativeIngest
    rng = np.random.default_rng(seed)
    poly = POLYS[int(rng.integers(0, len(POLYS)))]
    mn, avg, mx = PARAMS[int(rng.integers(0, len(PARAMS)))]
    ctx = Context.get(poly, mn, avg, mx, device=0)
    files = []
    for _ in range(int(rng.integers(2, 13))):
        kind = ["random", "zeros", "text", "runs", "runs", "copy", "random"][int(rng.integers(0, 7))]
        n = int(rng.choice([0, int(rng.integers(1, 4 * KiB)), int(rng.integers(4 * KiB, 2 * MiB)),
                            int(rng.integers(2 * MiB, 40 * MiB))]))
        files.append(gen(rng, kind, n, files))
    batch = int(rng.choice([1, 2, 4, 8, 16, 64])) * MiB
    batch = max(batch, 2 * mx + 256)  # a stream piece may be up to a quarter batch; carries < max
    cfg = dict(batch_bytes=batch, depth=int(rng.integers(1, 5)), in_slots=int(rng.integers(2, 5)),
               out_slots=int(rng.integers(1, 4)), max_streams=int(rng.integers(1, 6)),
               long_chunk=int(rng.choice([256 * KiB, 1 * MiB, 2 * MiB, 64 * MiB])),
               pack_size=int(rng.choice([1, 4, 32])) * MiB,
               pack_grow_factor=int(rng.choice([0, 32])), hash_threads=int(rng.integers(1, 11)))
    level = [None, 0, 1, 3, 7][int(rng.integers(0, 5))]
    ing = NativeIngest(ctx, KEY, level=level, **cfg)
    how = []
    try:
        for i, f in enumerate(files):
            h = int(rng.integers(0, 3))
            how.append(h)
            if h == 0:
                ing.add(i, f)
            elif h == 1:
                piece = int(rng.integers(64 * KiB, max(batch // 4, 64 * KiB + 1)))
                assert ing.add_stream(i, ChoppyReader(f, seed * 100 + i), piece=piece,
                                      size_hint=int(rng.integers(0, 2 * f.size + 1))) == f.size
            else:
                p = os.path.join(tmp, f"s{seed}_{i}")
                with open(p, "wb") as fh:
                    fh.write(f.tobytes())
                ing.add_file(i, p)
                os.unlink(p)
        stats = ing.finish()
        _check_all(files, ing, stats, level, params=(poly, mn, avg, mx))
    finally:
        ing.close()
    return {"seed": seed, "files": len(files), "bytes": int(sum(f.size for f in files)),
            "batches": int(stats["batches"]), "packs": int(stats["packs"]), "level": level,
            "how": how, "cfg": cfg, "params": [hex(poly), mn, avg, mx]}


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 300
    seed0 = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    t0 = last = time.time()
    n = nbytes = packs = 0
    seed = seed0
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as tmp:
        while time.time() - t0 < secs:
            try:
                r = one_case(seed, tmp)
            except AssertionError as e:
                print(json.dumps({"MISMATCH": {"seed": seed, "error": repr(e)[:2000]}}), flush=True)
                sys.exit(1)
            n += 1
            nbytes += r["bytes"]
            packs += r["packs"]
            seed += 1
            if time.time() - last > 60:
                last = time.time()
                print(json.dumps({"cases": n, "packs": packs, "gib": round(nbytes / 2**30, 2)}),
                      flush=True)
    print(json.dumps({"soak_ingest": "ok", "cases": n, "packs": packs,
                      "gib": round(nbytes / 2**30, 2), "seeds": [seed0, seed - 1],
                      "seconds": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
