"""Randomised soak of the device frame checker (rcdc_zstd_check,
rcdc_zstd_dec.hip) on frames from libzstd and from this library's encoder,
intact and corrupted, against libzstd's verdict (test infrastructure:
oracle/zstd_ref.py is the checker).  Each case draws 1-40 blobs of the test
kinds (up to 1.5 MiB), a source per blob (libzstd at a level in [-7, 19] or
22 on small blobs, or the device encoder), and corrupts about half of the
frames: bit flips, byte and span overwrites, zeroed spans, truncation, bytes
appended, edits aimed at block headers and at the first bytes of a block's
literals / sequences sections, random garbage behind a good header, and
another frame's body behind this frame's header.  The device must accept
(status 0) exactly the frames libzstd's streaming decoder (rustic's
decode_all, window limit included) decodes to the blob; a wrong blob
length or byte must give status 1 or 2.  Exits 1 on a disagreement with the
case's seed.

  python tools/soak_zstd_check.py [seconds] [seed] [cases]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import zstd_ref as zr  # noqa: E402
from tests.test_gpu_zstd_check import _data  # noqa: E402

KiB, MiB = 1 << 10, 1 << 20
KINDS = ["random", "zeros", "text", "csv", "binary", "periodic", "mixed"]
MAGIC = b"\x28\xb5\x2f\xfd"


def block_spots(fr):
    """(block header offsets, block content offsets) of a frame, as far as
    its headers parse (RFC 8878 3.1.1.1-2)."""
    heads, bodies = [], []
    if len(fr) < 6 or fr[:4] != MAGIC:
        return heads, bodies
    fhd = fr[4]
    single, did, fcs = (fhd >> 5) & 1, fhd & 3, fhd >> 6
    pos = 5 + (0 if single else 1) + (0, 1, 2, 4)[did] + \
        ((1 if single else 0), 2, 4, 8)[fcs]
    while pos + 3 <= len(fr):
        h = int.from_bytes(fr[pos:pos + 3], "little")
        heads.append(pos)
        tpe, size = (h >> 1) & 3, h >> 3
        pos += 3
        if tpe == 2:
            bodies.append(pos)
        pos += 1 if tpe == 1 else size
        if h & 1:
            break
    return heads, bodies


def corrupt(rng, fr, other):
    g = bytearray(fr)
    how = int(rng.integers(0, 10))
    heads, bodies = block_spots(fr)
    if how == 0 and len(g) > 4:  # bit flips
        for _ in range(int(rng.integers(1, 4))):
            g[int(rng.integers(4, len(g)))] ^= 1 << int(rng.integers(0, 8))
    elif how == 1 and len(g) > 4:  # a byte
        g[int(rng.integers(4, len(g)))] = int(rng.integers(0, 256))
    elif how == 2 and len(g) > 5:  # a random span
        a = int(rng.integers(4, len(g)))
        k = min(int(rng.integers(1, 65)), len(g) - a)
        g[a:a + k] = rng.integers(0, 256, k, dtype=np.uint8).tobytes()
    elif how == 3 and len(g) > 5:  # a zeroed span
        a = int(rng.integers(4, len(g)))
        k = min(int(rng.integers(1, 257)), len(g) - a)
        g[a:a + k] = bytes(k)
    elif how == 4:  # truncated
        g = g[:int(rng.integers(0, len(g)))] if len(g) else g
    elif how == 5:  # bytes after the frame
        g += rng.integers(0, 256, int(rng.integers(1, 65)), dtype=np.uint8).tobytes()
    elif how == 6 and heads:  # a block header: size, type or last flag
        p = heads[int(rng.integers(0, len(heads)))]
        h = int.from_bytes(g[p:p + 3], "little")
        r = int(rng.integers(0, 3))
        if r == 0:
            h ^= 1
        elif r == 1:
            h = (h & ~6) | int(rng.integers(0, 4)) << 1
        else:
            h = (h & 7) | int(rng.integers(0, 1 << 21)) << 3
        g[p:p + 3] = (h & 0xFFFFFF).to_bytes(3, "little")
    elif how == 7 and bodies:  # the first bytes of a compressed block's sections
        p = bodies[int(rng.integers(0, len(bodies)))] + int(rng.integers(0, 8))
        if p < len(g):
            g[p] = int(rng.integers(0, 256)) if rng.random() < 0.5 else g[p] ^ (1 << int(rng.integers(0, 8)))
    elif how == 8 and heads:  # garbage behind a good header
        p = heads[0] + 3
        g[p:] = rng.integers(0, 256, max(len(g) - p, 0), dtype=np.uint8).tobytes()
    elif other:  # another frame's body behind this header
        h0, _ = block_spots(fr)
        h1, _ = block_spots(other)
        if h0 and h1:
            g = g[:h0[0]] + other[h1[0]:]
    return bytes(g)


def reserved_modes_bits(fr):
    """A compressed block whose Symbol_Compression_Modes byte has its
    reserved bits 1-0 set (RFC 8878 3.1.1.3.2.1: "must be all-zeroes";
    libzstd 1.5 rejects it, the 1.4.8 here decodes it)."""
    heads, bodies = block_spots(fr)
    for p in bodies:
        try:
            b0 = fr[p]
            lt, sf = b0 & 3, (b0 >> 2) & 3
            if lt < 2:  # raw / RLE literals
                if sf & 1 == 0:
                    hl, n = 1, b0 >> 3
                elif sf == 1:
                    hl, n = 2, (b0 >> 4) + (fr[p + 1] << 4)
                else:
                    hl, n = 3, (b0 >> 4) + (fr[p + 1] << 4) + (fr[p + 2] << 12)
                q = p + hl + (n if lt == 0 else 1)
            else:  # compressed / treeless: the compressed size
                v = int.from_bytes(fr[p:p + 5], "little")
                hl, bits = ((3, 10), (3, 10), (4, 14), (5, 18))[sf]
                q = p + hl + ((v >> (4 + bits)) & ((1 << bits) - 1))
            s0 = fr[q]
            if s0 == 0:
                continue
            q += 1 if s0 < 128 else 2 if s0 < 255 else 3
            if fr[q] & 3:
                return True
        except IndexError:
            return False
    return False


def libzstd_ok(frame, data):
    try:
        # decode_all's decoder: streaming, with libzstd's default window limit
        ok = zr.frame_size(frame) == len(frame) and zr.decompress_stream(frame) == data
    except zr.ZstdError:
        return False
    return ok and not reserved_modes_bits(frame)


def one_case(seed, torch, ctx):
    from rustic_core_amd.compress import check_frames, compress_blobs, frame_layout, make_refs
    rng = np.random.default_rng(seed)
    nb = int(rng.integers(1, 41))
    datas, srcs = [], []
    for _ in range(nb):
        n = int(rng.choice([0, int(rng.integers(1, 300)), int(rng.integers(300, 140 * KiB)),
                            int(rng.integers(140 * KiB, int(1.5 * MiB)))]))
        datas.append(_data(rng, n, KINDS[int(rng.integers(0, len(KINDS)))]))
        r = rng.random()
        srcs.append("device" if r < 0.3 else 22 if r < 0.35 and n < 200 * KiB else
                    int(rng.integers(-7, 20)))
    # the device frames in one call
    dev = [i for i, s in enumerate(srcs) if s == "device"]
    frames = [None] * nb
    if dev:
        lens = [len(datas[i]) for i in dev]
        offs, o = [], 0
        for i in dev:
            offs.append(o)
            o += len(datas[i])
        arr = np.zeros(o + 64, np.uint8)
        for a, i in zip(offs, dev):
            arr[a:a + len(datas[i])] = np.frombuffer(datas[i], np.uint8)
        f_offs, tot = frame_layout(lens)
        d_in = torch.from_numpy(arr).to("cuda:0")
        d_out = torch.zeros(tot + 64, dtype=torch.uint8, device="cuda:0")
        ln = compress_blobs(ctx, d_in.data_ptr(), make_refs(offs, lens, f_offs), d_out.data_ptr(),
                            int(rng.choice([0, 1, 3, 7, 22])))
        out = d_out.cpu().numpy()
        for j, i in enumerate(dev):
            frames[i] = out[int(f_offs[j]):int(f_offs[j]) + int(ln[j])].tobytes()
    for i, s in enumerate(srcs):
        if s != "device":
            frames[i] = zr.compress(datas[i], s)
    # corruptions, wrong blobs
    fs, ds, kinds = [], [], []
    for i in range(nb):
        f, d = frames[i], datas[i]
        r = rng.random()
        if r < 0.45:
            fs.append(f)
            ds.append(d)
            kinds.append("intact")
        elif r < 0.9:
            fs.append(corrupt(rng, f, frames[int(rng.integers(0, nb))]))
            ds.append(d)
            kinds.append("corrupt")
        else:  # the frame against another length or one changed byte
            e = bytearray(d)
            if e and rng.random() < 0.5:
                e[int(rng.integers(0, len(e)))] ^= 1 << int(rng.integers(0, 8))
            else:
                e = e[:-1] if e and rng.random() < 0.5 else e + b"x"
            fs.append(f)
            ds.append(bytes(e))
            kinds.append("wrong data")
    # ragged layouts, 4 readable bytes after each range (the ABI's promise)
    def lay(bufs):
        offs, o = [], 0
        for b in bufs:
            o += int(rng.integers(0, 32))
            offs.append(o)
            o += len(b)
        arr = np.full(o + 64, 0x77, np.uint8)
        for a, b in zip(offs, bufs):
            arr[a:a + len(b)] = np.frombuffer(b, np.uint8)
        return arr, offs
    farr, foffs = lay(fs)
    darr, doffs = lay(ds)
    d_f = torch.from_numpy(farr).to("cuda:0")
    d_d = torch.from_numpy(darr).to("cuda:0")
    st = check_frames(ctx, d_f.data_ptr(), foffs, [len(f) for f in fs], d_d.data_ptr(), doffs,
                      [len(d) for d in ds])
    torch.cuda.synchronize()
    errs = []
    for i, (f, d, k) in enumerate(zip(fs, ds, kinds)):
        want = libzstd_ok(f, d)
        got = int(st[i])
        if got not in (0, 1, 2) or (got == 0) != want:
            e = {"i": i, "kind": k, "src": str(srcs[i]), "status": got, "libzstd": want,
                 "frame_len": len(f), "data_len": len(d)}
            if len(f) <= 4096:  # small enough to replay on the host
                e["frame"], e["good"] = f.hex(), frames[i].hex()
            dump = os.environ.get("SOAK_DUMP")  # a directory: the frame, its source and the blob
            if dump:
                os.makedirs(dump, exist_ok=True)
                for tag, b in (("frame", f), ("good", frames[i]), ("data", d)):
                    with open(os.path.join(dump, f"s{seed}_{i}.{tag}"), "wb") as fh:
                        fh.write(b)
            errs.append(e)
    return {"seed": seed, "frames": nb, "bytes": int(sum(len(d) for d in datas)),
            "corrupt": kinds.count("corrupt"), "errors": errs}


def main():
    import torch
    from oracle import oracle
    from rustic_core_amd.chunker import Context
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 300
    seed0 = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    ncase = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 62
    ctx = Context.get(oracle.DEFAULT_POLY, oracle.DEFAULT_MIN, oracle.DEFAULT_AVG,
                      oracle.DEFAULT_MAX, device=0)
    t0 = last = time.time()
    n = frames = corrupt_n = nbytes = 0
    seed = seed0
    while time.time() - t0 < secs and n < ncase:
        r = one_case(seed, torch, ctx)
        if r["errors"]:
            print(json.dumps({"MISMATCH": r}), flush=True)
            sys.exit(1)
        n += 1
        frames += r["frames"]
        corrupt_n += r["corrupt"]
        nbytes += r["bytes"]
        seed += 1
        if time.time() - last > 30:
            last = time.time()
            print(json.dumps({"cases": n, "frames": frames, "corrupt": corrupt_n}), flush=True)
    print(json.dumps({"soak_zstd_check": "ok", "cases": n, "frames": frames, "corrupt": corrupt_n,
                      "gib": round(nbytes / 2**30, 2), "seeds": [seed0, seed - 1],
                      "seconds": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
