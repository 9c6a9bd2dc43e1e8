"""Randomised soak of the native ingest engine (rcdc_ingest_* through
ctypes) against the oracle and hashlib (test infrastructure: the checks of
tests/test_gpu_native_ingest.py _check_all).  Each case draws chunker
parameters, 2-12 files (empty to 40 MiB; random, zeros, text, runs, copies
and prefixes of earlier files), how each file goes in (rcdc_ingest_add,
add_stream with short reads and random piece sizes, or from a file on disk),
the engine shape (batch_bytes 1-64 MiB, depth, slots, streams, long-chunk
threshold, pack size and grow factor) and the zstd level (stored blobs,
0 = default, 1, 3, 7), and checks every cut, chunk id, pack id, pack header,
blob and dedup decision.  Some streams fail mid-way (their read raises: the
stream is aborted, its completed chunks stay packed, no file result), some
reservations are cancelled, and some cases run two engines over one shared
dedup set (MultiIngest: every new id packed exactly once across both).
Exits 1 on a mismatch with the case's seed.

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
from tests.test_gpu_native_ingest import KEY  # noqa: E402

# zstd levels drawn (None: stored blobs); SOAK_LEVELS="22,-5,4" replaces the
# list (the default keeps earlier seeds replayable)
LEVELS = [None, 0, 1, 3, 7] if not os.environ.get("SOAK_LEVELS") else \
    [None if x == "none" else int(x) for x in os.environ["SOAK_LEVELS"].split(",")]
from tests.test_gpu_ingest_streams import ChoppyReader, FailingReader  # noqa: E402
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


def _chunks(data, cuts):
    prev = 0
    for c in cuts:
        yield data[prev:int(c)]
        prev = int(c)


def check(events, engines, stats, level, params, ordered):
    """events: (tag, bytes, kind, fed) in add order; kind full / aborted /
    cancelled.  The checks of tests/test_gpu_native_ingest._check_all,
    with aborted streams' completed chunks in the replay (all the cuts of
    the fed prefix but the last) and, with two engines (ordered False),
    the packed ids compared as a set, each exactly once."""
    import hashlib
    from oracle import oracle, zstd_ref
    full = [(t, d) for t, d, k, _ in events if k == "full"]
    files = {}
    for e in engines:
        files.update(e.files)
    assert stats["files"] == len(full) == len(files), ("files", stats["files"], len(full), len(files))
    seen, new, by_id = set(), [], {}
    for t, d, k, fed in events:
        if k == "cancelled":
            continue
        if k == "full":
            cuts = oracle.chunk_cuts(d, *params)
            got_cuts, ids, nnew, ln = files[t]
            assert ln == d.size, ("len", t)
            assert np.array_equal(got_cuts, cuts), ("cuts", t)
            for j, c in enumerate(_chunks(d, cuts)):
                assert bytes(ids[j]) == hashlib.sha256(c.tobytes()).digest(), ("id", t, j)
        else:  # aborted: the fed prefix's final cuts
            cuts = oracle.chunk_cuts(d[:fed], *params)[:-1]
        for c in _chunks(d, cuts):
            h = hashlib.sha256(c.tobytes()).digest()
            by_id.setdefault(h, c)
            if h not in seen:
                seen.add(h)
                new.append(h)
    assert stats["new_blobs"] == len(new), ("new_blobs", stats["new_blobs"], len(new))
    packed = []
    for e in engines:
        assert [p["seq"] for p in e.packs] == list(range(len(e.packs))), "pack seq"
        for p in e.packs:
            data = p["data"]
            assert len(data) == p["size"] and hashlib.sha256(data).digest() == p["id"], "pack id"
            parsed = oracle.parse_pack(KEY, data)
            assert len(parsed) == len(p["blobs"]), "pack header"
            end = 0
            for (tpe, off, ln, ulen, bid), (id_, boff, blen, bulen, btype) in zip(parsed, p["blobs"]):
                assert off == boff and ln == blen and bytes(bid) == id_ and ulen == bulen, "blob entry"
                plain = oracle.open_(KEY, data[off:off + ln])
                raw = zstd_ref.decompress_stream(plain) if level is not None else plain  # decode_all
                assert hashlib.sha256(raw).digest() == id_, "blob bytes"
                end = off + ln
                packed.append(id_)
            assert end + p["header_len"] + 4 == p["size"], "pack size"
    if ordered:
        assert packed == new, "Packer::add order"
    else:
        assert len(packed) == len(set(packed)) and set(packed) == set(new), "packed once"


def one_case(seed, tmp):
    import ctypes
    from rustic_core_amd import _lib
    from rustic_core_amd.chunker import Context
    from rustic_core_amd.native_ingest import MultiIngest, NativeIngest
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
    levels = LEVELS
    level = levels[int(rng.integers(0, len(levels)))]
    multi = rng.random() < 0.2
    events = []
    if multi:
        m = MultiIngest([ctx, ctx], KEY, level=level, **cfg)
        engines = m.engines
        try:
            for i, f in enumerate(files):
                m.add(i, f)
                events.append((i, f, "full", f.size))
            stats = m.finish()
            check(events, engines, stats, level, (poly, mn, avg, mx), ordered=False)
        finally:
            m.close()
    else:
        ing = NativeIngest(ctx, KEY, level=level, **cfg)
        engines = [ing]
        try:
            for i, f in enumerate(files):
                h = int(rng.integers(0, 5))
                if h == 0 or h == 4:
                    ing.add(i, f)
                    events.append((i, f, "full", f.size))
                elif h == 1:
                    piece = int(rng.integers(64 * KiB, max(batch // 4, 64 * KiB + 1)))
                    if rng.random() < 0.25 and f.size > 1:  # the read fails mid-way
                        fail_at = int(rng.integers(1, f.size))
                        try:
                            ing.add_stream(i, FailingReader(f, seed * 100 + i, fail_at), piece=piece)
                            raise AssertionError("the failing read did not raise")
                        except OSError:
                            pass
                        events.append((i, f, "aborted", fail_at // piece * piece))
                    else:
                        assert ing.add_stream(i, ChoppyReader(f, seed * 100 + i), piece=piece,
                                              size_hint=int(rng.integers(0, 2 * f.size + 1))) == f.size
                        events.append((i, f, "full", f.size))
                elif h == 2:
                    p = os.path.join(tmp, f"s{seed}_{i}")
                    with open(p, "wb") as fh:
                        fh.write(f.tobytes())
                    ing.add_file(i, p)
                    os.unlink(p)
                    events.append((i, f, "full", f.size))
                else:  # a reservation whose read fails: cancelled
                    buf, t = ctypes.c_void_p(), ctypes.c_uint64()
                    n = min(f.size, batch)
                    assert _lib.lib().rcdc_ingest_reserve(ing._h, n, ctypes.byref(buf),
                                                          ctypes.byref(t)) == 0
                    ing.cancel(t.value)
                    events.append((i, f, "cancelled", 0))
            stats = ing.finish()
            check(events, engines, stats, level, (poly, mn, avg, mx), ordered=True)
        finally:
            ing.close()
    return {"seed": seed, "files": len(files), "bytes": int(sum(f.size for f in files)),
            "batches": int(stats["batches"]), "packs": int(stats["packs"]), "level": level,
            "multi": multi, "kinds": [e[2] for e in events], "cfg": cfg,
            "params": [hex(poly), mn, avg, mx]}


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 300
    seed0 = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    t0 = last = time.time()
    n = nbytes = packs = aborted = cancelled = multi = 0
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
            aborted += r["kinds"].count("aborted")
            cancelled += r["kinds"].count("cancelled")
            multi += r["multi"]
            seed += 1
            if time.time() - last > 60:
                last = time.time()
                print(json.dumps({"cases": n, "packs": packs, "gib": round(nbytes / 2**30, 2)}),
                      flush=True)
    print(json.dumps({"soak_ingest": "ok", "cases": n, "packs": packs, "aborted_streams": aborted,
                      "cancelled": cancelled, "two_engine_cases": multi,
                      "gib": round(nbytes / 2**30, 2), "seeds": [seed0, seed - 1],
                      "seconds": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
