"""Randomised soak of the device zstd encoder and frame checker
(rcdc_zstd_compress / rcdc_zstd_check) against two independent decoders
(test infrastructure: oracle/zstd_ref.py, libzstd through ctypes and
pyarrow's zstd).  Each case draws 1-48 blobs (edge lengths around 128 KiB
blocks and the 16-byte / 256-byte / 64 KiB thresholds, or random up to
6 MiB) of the test kinds (random, zeros, text, mixed, periodic, skewed,
binary), offsets in and out with random padding, and a level from the
repository range; every frame must decode to its blob with both decoders,
declare its content size, fit the bound, and pass the device frame check,
and a flipped byte in one frame must fail that check or decode to other
bytes.  Exits 1 on a mismatch with the case's seed.

  python tools/soak_zstd.py [seconds] [seed] [cases]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import zstd_ref as zr  # noqa: E402
from tests.test_gpu_zstd import _kinds  # noqa: E402

KiB, MiB = 1 << 10, 1 << 20
EDGE = [0, 1, 15, 16, 17, 255, 256, 257, 4095, 4096, 65535, 65536, 65537, 131071, 131072,
        131073, 262143, 262144, 262145]
KINDS = ["random", "zeros", "text", "mixed", "periodic", "skewed", "binary"]
LEVELS = [0, 1, 2, 3, 3, 3, 4, 5, 7, 9, 12, 19, 22, -1, -5]
GUARD = 0 if os.environ.get("SOAK_NO_GUARD") == "1" else 8 << 20  # (0: the bare layout)


def one_case(seed, torch):
    from rustic_core_amd.chunker import Context
    from rustic_core_amd.compress import (CHECK_OK, check_frames, compress_blobs, make_refs,
                                          zstd_bound)
    from oracle import oracle
    rng = np.random.default_rng(seed)
    ctx = Context.get(oracle.DEFAULT_POLY, oracle.DEFAULT_MIN, oracle.DEFAULT_AVG,
                      oracle.DEFAULT_MAX, device=0)
    level = LEVELS[int(rng.integers(0, len(LEVELS)))]
    datas = []
    for _ in range(int(rng.integers(1, 49))):
        n = EDGE[int(rng.integers(0, len(EDGE)))] if rng.random() < 0.4 else \
            int(rng.integers(0, 6 * MiB)) if rng.random() < 0.3 else int(rng.integers(0, 300 * KiB))
        datas.append(_kinds(rng, n, KINDS[int(rng.integers(0, len(KINDS)))]))
    offs, o = [], 0
    for d in datas:
        o += int(rng.integers(0, 64))
        offs.append(o)
        o += len(d)
    arena = np.zeros(o + 64, np.uint8)
    for a, d in zip(offs, datas):
        arena[a:a + len(d)] = np.frombuffer(d, np.uint8)
    oo, q = [], 0
    for d in datas:
        q += int(rng.integers(0, 64))
        oo.append(q)
        q += zstd_bound(len(d))
    lens = [len(d) for d in datas]
    # GUARD bytes before and after both buffers: an access past a blob or a
    # frame lands in them (and is reported) instead of faulting the device
    g_in = torch.full((GUARD + arena.size + GUARD,), 0x5C, dtype=torch.uint8, device="cuda:0")
    g_in[GUARD:GUARD + arena.size] = torch.from_numpy(arena).to("cuda:0")
    d_in = g_in[GUARD:]
    g_out = torch.full((GUARD + q + 64 + GUARD,), 0xA5, dtype=torch.uint8, device="cuda:0")
    d_out = g_out[GUARD:]
    ln = compress_blobs(ctx, d_in.data_ptr(), make_refs(offs, lens, oo), d_out.data_ptr(), level)
    torch.cuda.synchronize()
    gout = g_out.cpu().numpy()
    if not ((gout[:GUARD] == 0xA5).all() and (gout[GUARD + q + 64:] == 0xA5).all()):
        bad = np.nonzero(gout != 0xA5)[0]
        return {"seed": seed, "blobs": len(datas), "bytes": int(sum(lens)), "level": level,
                "frame_bytes": 0, "errors": [("written in a guard", int(bad.min()) - GUARD,
                                              int(bad.max()) - GUARD, q)]}
    st = check_frames(ctx, d_out.data_ptr(), oo, ln, d_in.data_ptr(), offs, lens)
    torch.cuda.synchronize()
    out = d_out[:q + 64].cpu().numpy()
    errs = []
    mask = np.ones(len(out), bool)
    for i, (a, n, d) in enumerate(zip(oo, ln, datas)):
        a, n = int(a), int(n)
        mask[a:a + n] = False
        fr = out[a:a + n].tobytes()
        if n > zstd_bound(len(d)) or zr.content_size(fr) != len(d) or zr.frame_size(fr) != n:
            errs.append(("frame header/size", i))
        elif zr.decompress(fr) != d or (len(d) and zr.decompress_pyarrow(fr, len(d)) != d):
            errs.append(("decode", i))
        if int(st[i]) != CHECK_OK:
            errs.append(("device check", i, int(st[i])))
    if not (out[mask] == 0xA5).all():
        errs.append(("written outside the frames",))
    # a corrupted frame: the device check rejects it, or it decodes to other bytes
    big = [i for i, d in enumerate(datas) if len(d) > 64]
    if big and not errs:
        i = big[int(rng.integers(0, len(big)))]
        a, n = int(oo[i]), int(ln[i])
        pos = a + int(rng.integers(0, n))
        out2 = d_out.clone()
        out2[pos] ^= 0x5A
        st2 = check_frames(ctx, out2.data_ptr(), [oo[i]], [ln[i]], d_in.data_ptr(), [offs[i]],
                           [lens[i]])
        if int(st2[0]) == CHECK_OK:
            fr = out2[a:a + n].cpu().numpy().tobytes()
            try:
                same = zr.decompress(fr) == datas[i]
            except Exception:  # noqa: BLE001 (libzstd rejects it: the device should have)
                same = False
            if not same:
                errs.append(("corrupted frame passed the device check", i, pos - a))
    return {"seed": seed, "blobs": len(datas), "bytes": int(sum(lens)), "level": level,
            "frame_bytes": int(np.sum(ln)), "errors": errs}


def main():
    import torch
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 300
    seed0 = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    ncase = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 62
    t0 = last = time.time()
    n = nbytes = blobs = 0
    seed = seed0
    while time.time() - t0 < secs and n < ncase:
        r = one_case(seed, torch)
        if r["errors"]:
            print(json.dumps({"MISMATCH": r}), flush=True)
            sys.exit(1)
        n += 1
        blobs += r["blobs"]
        nbytes += r["bytes"]
        seed += 1
        if time.time() - last > 30:
            last = time.time()
            print(json.dumps({"cases": n, "blobs": blobs, "gib": round(nbytes / 2**30, 2)}),
                  flush=True)
    print(json.dumps({"soak_zstd": "ok", "cases": n, "blobs": blobs,
                      "gib": round(nbytes / 2**30, 2), "seeds": [seed0, seed - 1],
                      "seconds": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
