"""Device zstd throughput per data kind (rcdc_zstd_compress): 8 GiB of
chunk-sized blobs (0.5-8 MiB) of random bytes, zeros, C3-style mixed runs,
word text, CSV-like rows and code-like lines; GiB/s by HIP events, ratio, and a decode check
of a sample (and libzstd level 3's ratio on a 16 MiB piece of each kind).
Run under rocprofv3 --kernel-trace --stats for the per-kernel split."""
import argparse
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from oracle import zstd_ref as zr  # noqa: E402  (the checker)
from rustic_core_amd.chunker import Context  # noqa: E402
from rustic_core_amd.compress import compress_blobs, frame_layout, make_refs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--gib", type=float, default=8)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--kinds", default="random,zeros,mixed,text,csv,code")
ap.add_argument("--levels", default="0", help="comma-separated zstd levels")
ap.add_argument("--check", action="store_true", help="also decode every frame on the device "
                "(rcdc_zstd_check) and time it")
args = ap.parse_args()
dev = torch.device("cuda:0")
n = int(args.gib * (1 << 30))
rng = np.random.default_rng(1)
lens = []
while sum(lens) < n:
    lens.append(int(rng.integers(512 << 10, 8 << 20)))
lens[-1] -= sum(lens) - n
offs = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.uint64)
arena = torch.empty(n + 64, dtype=torch.uint8, device=dev)
f_offs, ftot = frame_layout(lens)
frames = torch.empty(ftot + 64, dtype=torch.uint8, device=dev)
ctx = Context.get(0x3DA3358B4DC173, 1 << 19, 1 << 20, 1 << 23, device=0)
refs = make_refs(offs, lens, f_offs)

words = [bytes(rng.integers(97, 123, size=int(rng.integers(2, 9))).astype(np.uint8)) for _ in range(400)]
text = np.frombuffer(b" ".join(words[int(i)] for i in rng.integers(0, 400, 16 << 20 >> 2)), np.uint8)
text = torch.from_numpy(text[:16 << 20].copy()).to(dev)
csv_rows = b"".join(b"%08d,%s,%d,%s\n" % (i, words[i % 400], (i * 7919) % 100000, words[(i * 31) % 400])
                    for i in range(600000))
csv_rows = torch.from_numpy(np.frombuffer(csv_rows, np.uint8)[:16 << 20].copy()).to(dev)
code_lines = b"".join(b"    x_%d = foo(%s, %d) + bar[%d];\n" % (i % 97, words[i % 50], i, (i * 13) % 1000)
                      for i in range(600000))
code_lines = torch.from_numpy(np.frombuffer(code_lines, np.uint8)[:16 << 20].copy()).to(dev)


def fill(kind):
    if kind == "random":
        arena.random_(0, 256)
    elif kind == "zeros":
        arena.zero_()
    elif kind in ("text", "csv", "code"):
        src = {"text": text, "csv": csv_rows, "code": code_lines}[kind]
        t = src.numel()
        for o in range(0, n, t):
            arena[o:o + min(t, n - o)] = src[:min(t, n - o)]
    elif kind == "mixed":  # C3: random runs 64 KiB-16 MiB, zero runs 4 KiB-16 MiB
        arena.random_(0, 256)
        o = 0
        while o < n:
            r = int(rng.integers(64 << 10, 16 << 20))
            z = int(rng.integers(4 << 10, 16 << 20))
            o += r
            arena[o:o + z] = 0
            o += z


for kind in args.kinds.split(","):
  fill(kind)
  for level in [int(x) for x in args.levels.split(",")]:
    torch.cuda.synchronize()
    st = torch.cuda.current_stream().cuda_stream
    for _ in range(3):  # warm-up (the first kind otherwise runs at a lower clock)
        ln = compress_blobs(ctx, arena.data_ptr(), refs, frames.data_ptr(), level, st)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(args.reps):
        ln = compress_blobs(ctx, arena.data_ptr(), refs, frames.data_ptr(), level, st)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.reps
    wall = (time.perf_counter() - t0) * 1e3 / args.reps
    bad = 0
    for i in [0, 1, len(lens) // 2, len(lens) - 1]:
        d = arena[int(offs[i]):int(offs[i]) + lens[i]].cpu().numpy().tobytes()
        f = frames[int(f_offs[i]):int(f_offs[i]) + int(ln[i])].cpu().numpy().tobytes()
        bad += zr.decompress(f) != d
    chk = ""
    if args.check:
        from rustic_core_amd.compress import check_frames
        t1 = time.perf_counter()
        cs = check_frames(ctx, frames.data_ptr(), f_offs, ln, arena.data_ptr(), offs, lens, st)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t1
        chk = f", device check {n / dt / 2**30:.1f} GiB/s ({int((cs != 0).sum())} bad)"
    piece = arena[:16 << 20].cpu().numpy().tobytes()
    ref = sum(len(zr.compress(piece[o:o + (1 << 20)], 3)) for o in range(0, len(piece), 1 << 20))
    print(f"{kind:7s} level {level:3d} {len(lens)} blobs {n / 2**30:.1f} GiB: {ms:.2f} ms "
          f"(wall {wall:.2f}) = {n / (ms / 1e3) / 2**30:.1f} GiB/s, ratio {int(ln.sum()) / n:.4f}, "
          f"libzstd-3 ratio on 16 x 1 MiB {ref / len(piece):.4f}, decode mismatches {bad}{chk}",
          flush=True)
