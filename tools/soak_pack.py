"""Randomised soak of pack building on the device (rcdc_pack_build,
rcdc_pack_build_raw, rcdc_pack_build_raw_multi; rcdc_runtime.cpp) against
the oracle's pack writer (test infrastructure: oracle.pack_file /
parse_pack, pinned by rebuilding the reference's own pack file byte for
byte in tests/test_pack_oracle.py).  Each case draws a key, 1-1500 blobs
(edge lengths around the 16-byte block, chunk-like up to 1 MiB; data or
tree; a quarter with an uncompressed length, i.e. CompData / CompTree
header entries), cuts them into 1-60 packs of consecutive blobs, places the
packs at 1-, 16- or 4096-byte alignment in one output buffer, and builds
them one of three ways:
  - sealed: plaintext blobs at ragged input offsets, sealed by the device;
  - raw: blobs already sealed (by the oracle), copied (packer.rs add_raw);
  - multi: raw blobs spread over 2-4 device buffers.
Every pack must equal the oracle's bytes, every returned offset the blob's
place in its pack, parse_pack must read the header back, and nothing may be
written outside the packs.  Exits 1 on a mismatch with the case's seed.

  python tools/soak_pack.py [seconds] [seed] [cases]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import oracle  # noqa: E402

KiB, MiB = 1 << 10, 1 << 20
EDGE = [0, 1, 15, 16, 17, 31, 32, 33, 4095, 4096, 65536, 65537]


def one_case(seed, torch, ctx):
    from rustic_core_amd.pack import (build_packs, build_packs_multi, make_blobs, pack_layout)
    rng = np.random.default_rng(seed)
    key = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
    nb = int(rng.integers(1, 1501))
    lens = []
    for _ in range(nb):
        lens.append(EDGE[int(rng.integers(0, len(EDGE)))] if rng.random() < 0.3 else
                    int(rng.integers(0, 64 * KiB)) if rng.random() < 0.7 else
                    int(rng.integers(64 * KiB, MiB)))
        if sum(lens) > 48 * MiB:
            break
    nb = len(lens)
    mode = ["sealed", "raw", "multi"][int(rng.integers(0, 3))]
    datas = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in lens]
    types = [int(rng.integers(0, 2)) for _ in range(nb)]
    ids = rng.integers(0, 256, (nb, 32), dtype=np.uint8)
    nonces = rng.integers(0, 256, (nb, 16), dtype=np.uint8)
    ulens = [int(rng.integers(1, 1 << 24)) if rng.random() < 0.25 else 0 for _ in range(nb)]
    # consecutive groups
    npk = int(rng.integers(1, min(60, nb) + 1))
    cuts = sorted(set(int(x) for x in rng.choice(np.arange(1, nb), npk - 1, replace=False))) \
        if npk > 1 else []
    bounds = [0] + cuts + [nb]
    groups = [(bounds[k], bounds[k + 1] - bounds[k]) for k in range(len(bounds) - 1)]
    hn = rng.integers(0, 256, (len(groups), 16), dtype=np.uint8)
    align = int(rng.choice([1, 16, 4096]))
    if mode == "sealed":
        srcs = datas
    else:
        srcs = [oracle.seal(key, nonces[i].tobytes(), datas[i]) for i in range(nb)]
    nbuf = int(rng.integers(2, 5)) if mode == "multi" else 1
    which = [int(rng.integers(0, nbuf)) for _ in range(nb)]
    arenas, offs = [], [0] * nb
    for b in range(nbuf):
        o, mine = 0, []
        for i in range(nb):
            if which[i] != b:
                continue
            o += int(rng.integers(0, 48))
            offs[i] = o
            mine.append(i)
            o += len(srcs[i])
        a = np.zeros(o + 64, np.uint8)
        for i in mine:
            a[offs[i]:offs[i] + len(srcs[i])] = np.frombuffer(srcs[i], np.uint8)
        arenas.append(torch.from_numpy(a).to("cuda:0"))
    blobs = make_blobs(offs, [len(s) for s in srcs], ids, nonces, types=types, uncompressed=ulens)
    if mode == "multi":
        blobs["pad"] = which
    packs, total = pack_layout(blobs, groups, hn, align=align, raw=mode != "sealed")
    d_out = torch.full((total + 64,), 0xA5, dtype=torch.uint8, device="cuda:0")
    if mode == "multi":
        got_offs = build_packs_multi(ctx, key, [a.data_ptr() for a in arenas], blobs, packs,
                                     d_out.data_ptr(), total)
    else:
        got_offs = build_packs(ctx, key, arenas[0].data_ptr(), blobs, packs, d_out.data_ptr(), total,
                               raw=mode == "raw")
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    errs = []
    mask = np.ones(len(out), bool)
    for k, (b0, n) in enumerate(groups):
        p = packs[k]
        f = out[int(p["out_off"]):int(p["out_off"]) + int(p["size"])].tobytes()
        mask[int(p["out_off"]):int(p["out_off"]) + int(p["size"])] = False
        # the expected pack: sealed blobs back to back, the sealed header, its length
        body, header, off, exp_offs = [], b"", 0, []
        for i in range(b0, b0 + n):
            s = srcs[i] if mode != "sealed" else oracle.seal(key, nonces[i].tobytes(), datas[i])
            body.append(s)
            exp_offs.append(off)
            header += oracle.pack_header_entry(types[i], len(s), ids[i].tobytes(), ulens[i])
            off += len(s)
        sh = oracle.seal(key, hn[k].tobytes(), header)
        want = b"".join(body) + sh + len(sh).to_bytes(4, "little")
        if f != want:
            errs.append(("pack bytes", k, mode, len(f), len(want)))
            continue
        if [int(got_offs[i]) for i in range(b0, b0 + n)] != exp_offs:
            errs.append(("offsets", k, mode))
        if int(p["header_len"]) != len(sh):
            errs.append(("header_len", k, mode))
        parsed = oracle.parse_pack(key, f)
        if [(t, o, ln, u, bytes(b)) for t, o, ln, u, b in parsed] != \
                [(types[i], exp_offs[i - b0], len(body[i - b0]), ulens[i], ids[i].tobytes())
                 for i in range(b0, b0 + n)]:
            errs.append(("parse", k, mode))
    if not (out[mask] == 0xA5).all():
        errs.append(("written outside the packs", mode))
    return {"seed": seed, "blobs": nb, "packs": len(groups), "mode": mode,
            "bytes": int(sum(lens)), "errors": errs}


def main():
    import torch
    from rustic_core_amd.chunker import Context
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 300
    seed0 = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    ncase = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 62
    ctx = Context.get(oracle.DEFAULT_POLY, oracle.DEFAULT_MIN, oracle.DEFAULT_AVG,
                      oracle.DEFAULT_MAX, device=0)
    t0 = last = time.time()
    n = blobs = packs = nbytes = 0
    modes = {"sealed": 0, "raw": 0, "multi": 0}
    seed = seed0
    while time.time() - t0 < secs and n < ncase:
        r = one_case(seed, torch, ctx)
        if r["errors"]:
            print(json.dumps({"MISMATCH": r}), flush=True)
            sys.exit(1)
        n += 1
        blobs += r["blobs"]
        packs += r["packs"]
        nbytes += r["bytes"]
        modes[r["mode"]] += 1
        seed += 1
        if time.time() - last > 30:
            last = time.time()
            print(json.dumps({"cases": n, "blobs": blobs, "packs": packs}), flush=True)
    print(json.dumps({"soak_pack": "ok", "cases": n, "blobs": blobs, "packs": packs, "modes": modes,
                      "gib": round(nbytes / 2**30, 2), "seeds": [seed0, seed - 1],
                      "seconds": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
