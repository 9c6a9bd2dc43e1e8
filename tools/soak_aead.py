"""Randomised soak of device blob encryption (rcdc_aead_seal / rcdc_aead_open,
rcdc_aead.hip) against the C oracle (test infrastructure: oracle/crypto_ref.c,
pinned to FIPS-197, RFC 8439 and the reference's encrypted fixtures).  Each
case draws a key, 1-300 blobs (empty, around the 16-byte block and the
4096-block unit, chunk-like up to 2 MiB, now and then 8 MiB), nonces (random,
or with low words near a carry: ..ff), and ragged in and out padding.  Every
sealed blob must equal the oracle's bytes, nothing may be written outside the
sealed blobs, and opening a batch of sealed blobs -- intact, corrupted (bit
flips in nonce, ciphertext or tag; truncations; blobs under 32 and 16 bytes;
another key's blob) -- must give status 0 and the plaintext exactly where
the oracle's open succeeds, 1 where its MAC check fails and 2 under 16
bytes.  Exits 1 on a mismatch with the case's seed.

  python tools/soak_aead.py [seconds] [seed] [cases]
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
EDGE = [0, 1, 15, 16, 17, 31, 32, 33, 63, 64, 65, 4095, 4096, 65535, 65536, 65537,
        4096 * 16 - 1, 4096 * 16, 4096 * 16 + 1]


def draw_len(rng):
    r = rng.random()
    if r < 0.3:
        return EDGE[int(rng.integers(0, len(EDGE)))]
    if r < 0.95:
        return int(rng.integers(0, 2 * MiB))
    return 8 * MiB - int(rng.integers(0, 2))


def draw_nonce(rng):
    n = bytearray(rng.integers(0, 256, 16, dtype=np.uint8).tobytes())
    if rng.random() < 0.2:  # near a counter carry in the low 64 bits or all 128
        k = int(rng.integers(1, 17))
        n[16 - k:] = b"\xff" * k
        n[15] = (0x100 - int(rng.integers(1, 64))) & 0xFF
    return bytes(n)


def one_case(seed, torch):
    from rustic_core_amd.crypto import Key, make_refs, sealed_layout
    rng = np.random.default_rng(seed)
    key = Key(rng.integers(0, 256, 64, dtype=np.uint8).tobytes())
    nb = int(rng.integers(1, 301))
    lens = [draw_len(rng) for _ in range(nb)]
    while sum(lens) > 256 * MiB:
        lens.pop()
    nb = len(lens)
    datas = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in lens]
    nonces = [draw_nonce(rng) for _ in range(nb)]
    offs, o = [], 0
    for n in lens:
        o += int(rng.integers(0, 64))
        offs.append(o)
        o += n
    arena = np.zeros(o + 64, np.uint8)
    for a, d in zip(offs, datas):
        arena[a:a + len(d)] = np.frombuffer(d, np.uint8)
    oo, olen = sealed_layout(lens)
    d_in = torch.from_numpy(arena).to("cuda:0")
    d_out = torch.full((olen + 64,), 0xA5, dtype=torch.uint8, device="cuda:0")
    key.seal_blobs(d_in.data_ptr(), make_refs(offs, lens, oo, b"".join(nonces)), d_out.data_ptr())
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    errs = []
    sealed = []
    mask = np.ones(len(out), bool)
    for i, (a, n) in enumerate(zip(oo, lens)):
        s = out[int(a):int(a) + n + 32].tobytes()
        mask[int(a):int(a) + n + 32] = False
        sealed.append(s)
        if s != oracle.seal(key._key, nonces[i], datas[i]):
            errs.append(("seal", i, n))
    if not (out[mask] == 0xA5).all():
        errs.append(("written outside the sealed blobs",))
    if errs:
        return {"seed": seed, "blobs": nb, "bytes": int(sum(lens)), "errors": errs}
    # open: intact and corrupted
    other = Key(rng.integers(0, 256, 64, dtype=np.uint8).tobytes())
    blobs = []
    for i, s in enumerate(sealed):
        r = rng.random()
        b = bytearray(s)
        if r < 0.5:
            pass
        elif r < 0.8:
            for _ in range(int(rng.integers(1, 3))):
                b[int(rng.integers(0, len(b)))] ^= 1 << int(rng.integers(0, 8))
        elif r < 0.9:
            b = b[:int(rng.integers(0, len(b)))]
        elif r < 0.95:
            b = bytearray(oracle.seal(other._key, nonces[i], datas[i]))
        else:
            b = bytearray(rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8).tobytes())
        blobs.append(bytes(b))
    ioffs, o = [], 0
    for b in blobs:
        o += int(rng.integers(0, 64))
        ioffs.append(o)
        o += len(b)
    arena = np.zeros(o + 64, np.uint8)
    for a, b in zip(ioffs, blobs):
        arena[a:a + len(b)] = np.frombuffer(b, np.uint8)
    outs, p = [], 0
    for b in blobs:
        p += int(rng.integers(0, 4)) * 16
        outs.append(p)
        p = (p + max(len(b) - 32, 0) + 15) // 16 * 16
    d_in = torch.from_numpy(arena).to("cuda:0")
    d_pl = torch.full((p + 64,), 0x5A, dtype=torch.uint8, device="cuda:0")
    st = key.open_blobs(d_in.data_ptr(), make_refs(ioffs, [len(b) for b in blobs], outs),
                        d_pl.data_ptr())
    torch.cuda.synchronize()
    pl = d_pl.cpu().numpy()
    for i, b in enumerate(blobs):
        try:
            want, ws = oracle.open_(key._key, b), 0
        except oracle.MacMismatch:
            want, ws = None, 1
        except ValueError:  # under 32 bytes; 16-31 is a MAC failure (aespoly1305.rs:89-108)
            want, ws = None, 2 if len(b) < 16 else 1
        if int(st[i]) != ws:
            errs.append(("open status", i, len(b), int(st[i]), ws))
        elif ws == 0 and pl[outs[i]:outs[i] + len(b) - 32].tobytes() != want:
            errs.append(("open bytes", i, len(b)))
    return {"seed": seed, "blobs": nb, "bytes": int(sum(lens)), "errors": errs}


def main():
    import torch
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 300
    seed0 = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    ncase = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 62
    t0 = last = time.time()
    n = blobs = nbytes = 0
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
    print(json.dumps({"soak_aead": "ok", "cases": n, "blobs": blobs,
                      "gib": round(nbytes / 2**30, 2), "seeds": [seed0, seed - 1],
                      "seconds": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
