#!/usr/bin/env python
"""bench.py -- CDC chunking GiB/s, device-resident (BASELINE.json metric).

Default workload (BASELINE.json configs[1], "C2"): per GPU, 1024 independent
1 MiB random buffers resident in HBM; one step = one full chunking pass (scan
kernel + resolve kernels) over all of them, producing the cut offsets in HBM.
Parameters are rustic's defaults: P = 0x003DA3358B4DC173, min 512 KiB,
avg 1 MiB, max 8 MiB (crates/core/src/repofile/configfile.rs:36-41).

Other SURVEY.md 8(d) configurations (--workload, not the driver's line):
  C3  64 streams x 1 GiB per GPU, mixed entropy (random runs 64 KiB-16 MiB,
      zero runs 4 KiB-16 MiB, 50/50 by bytes); --e2e adds the pinned-H2D
      rate with the copy of the next batch overlapped on a side stream.
  C4  8192 files, sizes log-uniform in [4, 256] MiB (seed 4000, ~485 GiB),
      LPT-sharded over the ranks (shard.assign_lpt); a step is one pass over
      the rank's share, in HBM-resident batches when it exceeds --c4-batch
      (each batch generated on device before its timed chunking).
  C5  one all-zero stream of 12.5 GiB per GPU (100 GiB at 8 GPUs) split
      across ranks (shard.slice_bounds, max + 64 B halos); a step includes
      the cross-rank stitch (shard.SlicedStream: one fixed-size all_gather of
      crossing windows).

Multi-GPU: one process per GPU (torchrun).  C2/C3: each rank chunks its own
streams (independent files shard per GPU, no collective on the data path:
"scaling": "weak"); the only collectives are the timing barrier / max.

Output: ONE JSON line on rank 0 (the driver's contract), including the
roofline of the dominant kernel (scan, HIP events on its launch stream over
the timed region) and the CPU baseline (the oracle in reference-equivalent
mode, timed on this host, rank 0 at N=1 only), and the parity check of the
measured run's cuts against the oracle.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "CDC chunking GiB/s device-resident, 1/2/4/8 MI355X; bit-exact cut points vs ref"
POLY = 0x003DA3358B4DC173
MIN, AVG, MAX = 512 * 1024, 1 << 20, 8 << 20
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
GiB = float(1 << 30)
MiB = 1 << 20


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", choices=["C1", "C2", "C3", "C4", "C5"], default="C3",
                    help="default C3 (64 x 1 GiB mixed per GPU, BASELINE.json configs[2]): the "
                         "largest single-GPU configuration")
    ap.add_argument("--c4-files", type=int, default=8192)
    ap.add_argument("--c4-batch", type=float, default=96.0, help="C4: GiB per resident batch")
    ap.add_argument("--streams", type=int, default=None, help="C2: 1024, C3: 64")
    ap.add_argument("--stream-bytes", type=int, default=None,
                    help="C2: 1 MiB, C3: 1 GiB, C5: 12.5 GiB per GPU")
    ap.add_argument("--parity-streams", type=int, default=None,
                    help="cap on the streams diffed against the oracle (default: all)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--prewarm", type=float, default=0.5,
                    help="untimed seconds of steps after the W warmup steps (clock ramp)")
    ap.add_argument("--time-every", type=int, default=4,
                    help="HIP-event timing of the kernels on every n-th timed step")
    ap.add_argument("--sha256", action="store_true",
                    help="also measure the fused blob ids (rcdc_plan_hash, SURVEY 8(f) row 1), "
                         "reported as a separate object; the headline value is unchanged")
    ap.add_argument("--sha-steps", type=int, default=5)
    ap.add_argument("--sha-depth", type=int, default=8,
                    help="batches whose blob ids are in flight at once (pipelined ingest)")
    ap.add_argument("--pipeline", action="store_true",
                    help="overlap run k's chain kernels with run k+1's hashing kernels "
                         "(rcdc_plan_set_pipeline); the default for walked plans (C3, C4)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="serial runs even for walked plans")
    ap.add_argument("--aead", action="store_true",
                    help="also seal + open the chunks as blobs on the device (rcdc_aead_*)")
    ap.add_argument("--aead-streams", type=int, default=16,
                    help="--aead: blobs = the chunks of the first N streams")
    ap.add_argument("--pack", action="store_true",
                    help="also build pack files of the chunks on the device (rcdc_pack_build)")
    ap.add_argument("--zstd", action="store_true",
                    help="also compress the chunks as blobs on the device (rcdc_zstd_compress)")
    ap.add_argument("--zstd-level", type=int, default=0)
    ap.add_argument("--ingest", action="store_true",
                    help="also run the Python/torch device-resident backup byte path "
                         "(rustic_core_amd.ingest.DeviceIngest, a test reference: chunk, blob "
                         "ids, dedup, zstd, seal, verify, packs) over --ingest-streams streams; "
                         "the default C3 line measures the native engine instead (h2h)")
    ap.add_argument("--no-ingest", action="store_true")
    ap.add_argument("--no-flush", action="store_true",
                    help="pipelined plans: the last timed run's chain stays narrow (A/B)")
    ap.add_argument("--no-h2h", action="store_true",
                    help="C3 at N=1: skip the host-to-host object (tools/ingest_e2e)")
    ap.add_argument("--h2h-files", type=int, default=64,
                    help="files of 1 GiB for the host-to-host object (fewer if the disk under "
                         "TMPDIR cannot hold them)")
    ap.add_argument("--ingest-streams", type=int, default=64)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--abi-e2e", action="store_true",
                    help="also measure the drop-in C ABI path (rcdc_stream_feed from pageable host "
                         "memory, --abi-threads workers) on the workload's first --abi-files streams")
    ap.add_argument("--abi-threads", type=int, default=16)
    ap.add_argument("--abi-files", type=int, default=16)
    ap.add_argument("--e2e", action="store_true",
                    help="also measure the PCIe-inclusive rate (pinned H2D + chunk + D2H cuts)")
    return ap.parse_args()


# ----------------------------------------------------------------- workloads
def make_mixed(torch, arena, off, length, rng, dev):
    """C3 stream: random runs 64 KiB-16 MiB and zero runs 4 KiB-16 MiB
    (log-uniform lengths), each kind with probability 1/2.  The run layout is
    drawn on the host; the bytes come from one randint and one masked fill
    (a handful of launches per stream, so profilers see few foreign kernels)."""
    g = torch.Generator(device=dev)
    g.manual_seed(int(rng.integers(1 << 62)))
    pos, zero, lens = 0, [], []
    while pos < length:
        if rng.random() < 0.5:
            L = min(int(np.exp(rng.uniform(np.log(64 << 10), np.log(16 << 20)))), length - pos)
            zero.append(False)
        else:
            L = min(int(np.exp(rng.uniform(np.log(4 << 10), np.log(16 << 20)))), length - pos)
            zero.append(True)
        lens.append(L)
        pos += L
    view = arena[off:off + length]
    torch.randint(0, 256, (length,), dtype=torch.uint8, device=dev, generator=g, out=view)
    mask = torch.repeat_interleave(torch.tensor(zero, device=dev),
                                   torch.tensor(lens, dtype=torch.int64, device=dev),
                                   output_size=length)
    view.masked_fill_(mask, 0)
    del mask


def build_workload(args, torch, dev, rank, world):
    """Returns (arena tensor, offs, lens, description dict)."""
    from rustic_core_amd.device import pack_offsets
    w = args.workload
    if w == "C2":
        n = args.streams or 1024
        sb = args.stream_bytes or MiB
        lens = np.full(n, sb, dtype=np.uint64)
        offs, arena_len = pack_offsets(lens)
        g = torch.Generator(device=dev)
        g.manual_seed(1000 + rank)
        arena = torch.randint(0, 256, (arena_len,), dtype=torch.uint8, device=dev, generator=g)
        desc = {"workload": f"C2: {n} independent {sb >> 10} KiB random buffers per GPU, "
                            "device-resident (BASELINE.json configs[1])",
                "streams_per_gpu": n, "stream_bytes": sb,
                "data": "synthetic: uniform random bytes (torch.randint on device, seed 1000+rank)"}
    elif w == "C3":
        n = args.streams or 64
        sb = args.stream_bytes or (1 << 30)
        lens = np.full(n, sb, dtype=np.uint64)
        offs, arena_len = pack_offsets(lens)
        arena = torch.empty(arena_len, dtype=torch.uint8, device=dev)
        for j in range(n):
            make_mixed(torch, arena, int(offs[j]), sb,
                       np.random.default_rng(3000 + rank * n + j), dev)
        desc = {"workload": f"C3: {n} streams x {sb / GiB:g} GiB per GPU, mixed entropy "
                            "(random runs 64 KiB-16 MiB + zero runs 4 KiB-16 MiB), "
                            "device-resident (BASELINE.json configs[2])",
                "streams_per_gpu": n, "stream_bytes": sb,
                "data": "synthetic: torch.randint runs + zero runs on device, seed 3000+stream"}
    else:  # C5
        from rustic_core_amd.shard import slice_bounds
        per = args.stream_bytes or int(12.5 * GiB)
        total = per * world
        a, b, e = slice_bounds(total, world, MIN, MAX)[rank]
        lens = np.array([e - a], dtype=np.uint64)
        offs = np.zeros(1, dtype=np.uint64)
        arena = torch.zeros(int(e - a) + 256, dtype=torch.uint8, device=dev)
        desc = {"workload": f"C5: one all-zero stream of {total / GiB:g} GiB split over {world} "
                            f"GPU(s) ({per / GiB:g} GiB + {MAX + 64} B halo each), "
                            "every chunk = min (BASELINE.json configs[4])",
                "stream_bytes_total": total, "slice": [a, b, e],
                "data": "synthetic: zeros on device"}
    return arena, offs, lens, desc


# ------------------------------------------------------------------ StdRng
def stdrng_numpy(seed: int, n: int) -> np.ndarray:
    """rand 0.10 StdRng::seed_from_u64(seed).fill_bytes(n) (SURVEY.md
    Appendix B: PCG32 seed expansion, ChaCha12 keystream), vectorised over
    64-byte blocks.  Input generator for C1 (the reference's own test data
    recipe, rabin.rs:343-347); tests/test_bench_host.py pins it to the oracle."""
    def rotl(x, k):
        return ((x << np.uint32(k)) | (x >> np.uint32(32 - k))).astype(np.uint32)
    MUL, INC = 6364136223846793005, 11634580027462260723
    state, key = seed & (2**64 - 1), []
    for _ in range(8):
        state = (state * MUL + INC) & (2**64 - 1)
        xs = ((((state >> 18) ^ state) >> 27) & 0xFFFFFFFF)
        rot = state >> 59
        key.append(((xs >> rot) | (xs << ((32 - rot) & 31))) & 0xFFFFFFFF)
    nb = (n + 63) // 64
    ctr = np.arange(nb, dtype=np.uint64)
    x0 = [np.full(nb, c, np.uint32) for c in (0x61707865, 0x3320646E, 0x79622D32, 0x6B206574)]
    x0 += [np.full(nb, k, np.uint32) for k in key]
    x0 += [(ctr & 0xFFFFFFFF).astype(np.uint32), (ctr >> np.uint64(32)).astype(np.uint32),
           np.zeros(nb, np.uint32), np.zeros(nb, np.uint32)]
    x = [v.copy() for v in x0]

    def qr(a, b, c, d):
        x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 16)
        x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 12)
        x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 8)
        x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 7)
    for _ in range(6):
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
    out = np.stack([x[i] + x0[i] for i in range(16)], axis=1).astype("<u4")
    return out.view(np.uint8).reshape(-1)[:n]


def pcie_rates(torch, dev, nbytes: int = 1 << 30) -> dict:
    """Host->device copy rates on this box: pinned and pageable sources."""
    d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    out = {}
    for kind in ("pinned", "pageable"):
        h = torch.empty(nbytes, dtype=torch.uint8, pin_memory=(kind == "pinned"))
        h.fill_(1)
        d.copy_(h, non_blocking=True)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(3):
            d.copy_(h, non_blocking=True)
        torch.cuda.synchronize(dev)
        out[f"h2d_{kind}_gibs"] = round(3 * nbytes / (time.perf_counter() - t0) / GiB, 2)
        del h
    return out


def abi_e2e(files, threads: int, read_bytes: int = 16 << 20) -> dict:
    """The drop-in path under the caller's load: `threads` workers, one file
    each at a time (archiver.rs:195), each fed to rcdc_stream_feed in
    `read_bytes` reads from pageable host memory (ChunkIter's plumbing,
    chunker.rs:22-47 over a Read).  Returns the aggregate GiB/s and the cut
    lists (for the parity check)."""
    import threading
    from rustic_core_amd.chunker import Context, _Stream
    ctx = Context.get(POLY, MIN, AVG, MAX)
    nxt = [0]
    lock = threading.Lock()
    cuts = [None] * len(files)

    def work():
        while True:
            with lock:
                i = nxt[0]
                nxt[0] += 1
            if i >= len(files):
                return
            f = files[i]
            st = _Stream(ctx)
            out = []
            for o in range(0, max(f.size, 1), read_bytes):
                piece = f[o:o + read_bytes]
                out.append(st.feed(piece, o + read_bytes >= f.size))
            st.close()
            cuts[i] = np.concatenate(out) if out else np.zeros(0, np.uint64)

    work_warm = _Stream(ctx)  # lanes and plans warm up outside the timed span
    work_warm.feed(files[0][:64 << 20], True)
    work_warm.close()
    t0 = time.perf_counter()
    th = [threading.Thread(target=work) for _ in range(threads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    el = time.perf_counter() - t0
    total = sum(int(f.size) for f in files)
    return {"value": round(total / el / GiB, 2), "unit": "GiB/s", "threads": threads,
            "files": len(files), "bytes": total, "read_bytes": read_bytes,
            "path": "rcdc_stream_feed (C ABI) from pageable host memory, one stream per file, "
                    "files on worker threads sharing one rcdc_ctx"}, cuts


# ------------------------------------------------------------- baselines etc.
def cpu_threads():
    """Host threads for the CPU baseline: the process's CPU affinity, capped by
    OMP_NUM_THREADS when set (the GPU box gives one GPU's job a 16-CPU share
    and sets OMP_NUM_THREADS=16; nproc shows the whole machine)."""
    try:
        ncpu = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        ncpu = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        return min(ncpu, int(omp)), f"min(affinity {ncpu}, OMP_NUM_THREADS {omp})"
    return ncpu, f"affinity {ncpu}"


def cpu_baseline(arena, offs, lens, seconds: float, max_bytes: int = 16 << 30) -> dict:
    """Oracle (cdc_ref, reference-equivalent work: owned chunk buffers fed by
    4 KiB reads, rabin.rs:110-191) over a bounded sample of the workload's
    streams (whole streams, at most max_bytes), per-file threads as in
    archiver.rs:195.  Repeats whole passes until `seconds` elapsed.  `arena`
    is the device tensor: only the sampled streams are copied to the host."""
    from oracle import oracle
    from rustic_core_amd.device import pack_offsets
    threads, why = cpu_threads()
    k = len(lens)
    while k > 1 and int(np.sum(lens[:k])) > max_bytes:
        k -= 1
    slens = np.asarray(lens[:k], dtype=np.uint64)
    soffs, alen = pack_offsets(slens)
    host = np.empty(alen, dtype=np.uint8)
    for i in range(k):
        o, n = int(offs[i]), int(lens[i])
        x = arena[o:o + n]
        host[int(soffs[i]):int(soffs[i]) + n] = x.cpu().numpy() if hasattr(x, "cpu") else x
    total = int(np.sum(slens))
    oracle.chunk_many_owned(host, soffs, slens, nthreads=threads)  # warm
    t0 = time.perf_counter()
    passes = 0
    while True:
        oracle.chunk_many_owned(host, soffs, slens, nthreads=threads)
        passes += 1
        el = time.perf_counter() - t0
        if el >= seconds or el >= 30.0:
            break
    # one thread: the first streams up to ~256 MiB
    k1 = 1
    while k1 < k and int(np.sum(slens[:k1 + 1])) <= (256 << 20):
        k1 += 1
    t1 = time.perf_counter()
    oracle.chunk_many_owned(host, soffs[:k1], slens[:k1], nthreads=1)
    el1 = time.perf_counter() - t1
    return {
        "value": passes * total / el / GiB,
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"{passes} full passes over the first {k} streams of the workload "
                   f"({passes * total / GiB:.1f} GiB, {el:.1f} s), cdc_ref reference-equivalent "
                   f"mode, {threads} threads (per-file parallel, archiver.rs:195)"),
        "cores_note": why,
        "single_thread_gibs": int(np.sum(slens[:k1])) / el1 / GiB,
        "cpu_model": _cpu_model(),
    }


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def pmc_traffic(workload: str, kernel: str):
    """Per-launch HBM bytes of the dominant kernel from the committed rocprofv3
    PMC summary of this workload (profiles/pmc_<workload>.json: FETCH_SIZE +
    WRITE_SIZE in separate passes, converted with the calibration measured for
    this access pattern, profiles/r01_pmc_hbm.txt); (None, None) if absent."""
    p = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    try:
        d = json.load(open(p))
    except (OSError, ValueError):
        return None, None
    if kernel not in d.get("kernel", ""):
        return None, None
    return d.get("hbm_bytes_per_launch"), d


def ref_slide_bytes(cuts_list, mn: int) -> int:
    """Bytes the reference slides over for these chunks (rabin.rs:127-188):
    a chunk of at least min bytes costs 63 prefill bytes (:149-151) plus one
    slide per byte after s + min; a final chunk shorter than min costs none
    (:141-147)."""
    tot = 0
    for c in cuts_list:
        c = np.asarray(c, dtype=np.int64)
        if c.size == 0:
            continue
        L = np.diff(np.concatenate([[0], c]))
        full = L >= mn
        tot += int(np.sum(L[full] - mn)) + 63 * int(np.count_nonzero(full))
    return tot


def c4_files(n: int):
    """sizes log-uniform in [4, 256] MiB, seed 4000."""
    rng = np.random.default_rng(4000)
    return [int(np.exp(rng.uniform(np.log(4 * MiB), np.log(256 * MiB)))) for _ in range(n)]


def c4_fill(torch, arena, offs, files, sizes, dev):
    """File f = uniform random bytes from a generator seeded 4000 + f."""
    g = torch.Generator(device=dev)
    for o, f in zip(offs, files):
        g.manual_seed(4000 + f)
        arena[int(o):int(o) + sizes[f]] = torch.randint(0, 256, (sizes[f],), dtype=torch.uint8,
                                                        device=dev, generator=g)


def run_c4(args, torch, dist, dev, rank, world, local):
    """C4: the rank's LPT share of 8192 files, chunked in resident batches."""
    from rustic_core_amd.chunker import Context
    from rustic_core_amd.device import DevicePlan, pack_offsets
    from rustic_core_amd.shard import assign_lpt
    sizes = c4_files(args.c4_files)
    mine = assign_lpt(sizes, world)[rank]
    cap = int(args.c4_batch * GiB)
    batches, cur, acc = [], [], 0
    for f in sorted(mine, key=lambda f: -sizes[f]):
        if cur and acc + sizes[f] > cap:
            batches.append(cur)
            cur, acc = [], 0
        cur.append(f)
        acc += sizes[f]
    if cur:
        batches.append(cur)
    ctx = Context.get(POLY, MIN, AVG, MAX, device=local)
    arena_len = max(pack_offsets([sizes[f] for f in b])[1] for b in batches) if batches else 256
    arena = torch.empty(arena_len, dtype=torch.uint8, device=dev)
    layouts = []
    for b in batches:
        offs, alen = pack_offsets([sizes[f] for f in b])
        layouts.append((b, offs, DevicePlan(ctx, offs, [sizes[f] for f in b], alen)))
    sptr = torch.cuda.current_stream(dev).cuda_stream
    scan_ms = resolve_ms = 0.0
    runs = 0
    # One resident batch per rank (the 8-GPU share, ~60 GiB, fits one): the K
    # passes run back to back like C3's steps, pipelined (rcdc_plan_set_pipeline:
    # pass k's chain kernels and the tail of its walk overlap pass k + 1's walk)
    # unless --no-pipeline.  Several batches: each is refilled (untimed) and
    # timed on its own.
    single = len(layouts) == 1
    pipelined = (single and not args.no_pipeline
                 and layouts[0][2].info().get("walk_pieces", 0) > 0)
    # warmup on the first batch
    if layouts:
        b, offs, plan = layouts[0]
        c4_fill(torch, arena, offs, b, sizes, dev)
        if pipelined:
            plan.set_pipeline(True)
        t_w = time.perf_counter()
        nw = 0
        while nw < args.warmup or (single and time.perf_counter() - t_w < args.prewarm):
            plan.run(arena.data_ptr(), sptr)
            nw += 1
            if nw % 8 == 0:
                torch.cuda.synchronize(dev)
    torch.cuda.synchronize(dev)
    el = 0.0
    sample_cuts = {}
    ref_hashed = lane_hashed = walked_batches = 0
    rng = np.random.default_rng(4001)
    sample = set(int(x) for x in rng.choice(args.c4_files, size=min(64, args.c4_files),
                                             replace=False))
    parity_acc = [0, 0, 0, 0.0]  # files diffed, mismatches, cuts diffed, seconds
    if single and layouts:
        b, offs, plan = layouts[0]
        plan.set_timing(True, every=args.time_every)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            plan.run(arena.data_ptr(), sptr)
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        if world > 1:
            dist.barrier()
        plan.set_timing(False)
        runs, scan_ms, resolve_ms = plan.kernel_times()
        got = plan.results()
        ref_hashed = ref_slide_bytes(got, MIN)
        inf = plan.info()
        if inf["walk_pieces"]:
            wst = plan.walk_stats()
            lane_hashed = wst["round_bytes"] + wst["zones"] * 4096
            walked_batches = 1
        else:
            lane_hashed = inf["scanned_bytes"] + 64 * inf["segments"]
        if not args.no_parity:  # every file of the share (untimed)
            t_p = time.perf_counter()
            bad_b, cuts_b = oracle_diff(arena, offs, [sizes[f] for f in b], got, cpu_threads()[0])
            parity_acc[0] += len(b)
            parity_acc[1] += bad_b
            parity_acc[2] += cuts_b
            parity_acc[3] += time.perf_counter() - t_p
        for i, f in enumerate(b):
            if f in sample and not args.no_cpu_baseline:
                o = int(offs[i])
                sample_cuts[f] = (got[i], arena[o:o + sizes[f]].cpu().numpy())
    for step in range(args.steps if not single else 0):
        for b, offs, plan in layouts:
            if len(layouts) > 1 or step == 0:
                c4_fill(torch, arena, offs, b, sizes, dev)  # outside the timed span
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize(dev)
            plan.set_timing(True)
            t0 = time.perf_counter()
            plan.run(arena.data_ptr(), sptr)
            torch.cuda.synchronize(dev)
            el += time.perf_counter() - t0
            plan.set_timing(False)
            r, sm, rm = plan.kernel_times()
            if os.environ.get("RCDC_C4_VERBOSE") and rank == 0:
                inf = plan.info()
                print(f"c4 batch files={len(b)} gib={sum(sizes[f] for f in b) / GiB:.1f} "
                      f"min_mib={min(sizes[f] for f in b) / 2**20:.1f} "
                      f"wall_ms={(time.perf_counter() - t0) * 1e3:.2f} scan_ms={sm:.2f} "
                      f"chain_ms={rm:.2f} walk_pieces={inf['walk_pieces']} "
                      f"seg={inf['segment_bytes']} scanned_gib={inf['scanned_bytes'] / GiB:.1f}",
                      file=sys.stderr, flush=True)
            runs += r
            scan_ms += sm
            resolve_ms += rm
            if step == 0:
                got = plan.results()
                ref_hashed += ref_slide_bytes(got, MIN)
                inf = plan.info()
                if inf["walk_pieces"]:
                    wst = plan.walk_stats()
                    lane_hashed += wst["round_bytes"] + wst["zones"] * 4096
                    walked_batches += 1
                else:
                    lane_hashed += inf["scanned_bytes"] + 64 * inf["segments"]
                if not args.no_parity:
                    t_p = time.perf_counter()
                    bad_b, cuts_b = oracle_diff(arena, offs, [sizes[f] for f in b], got,
                                                cpu_threads()[0])
                    parity_acc[0] += len(b)
                    parity_acc[1] += bad_b
                    parity_acc[2] += cuts_b
                    parity_acc[3] += time.perf_counter() - t_p
                for i, f in enumerate(b):
                    if f in sample and not args.no_cpu_baseline:
                        o = int(offs[i])
                        sample_cuts[f] = (got[i], arena[o:o + sizes[f]].cpu().numpy())
    t = torch.tensor([el], dtype=torch.float64, device=coll_device(dev))
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el_max = float(t.item())
    total = sum(sizes) * args.steps
    share = sum(sizes[f] for f in mine)
    passes = max(runs if single else args.steps, 1)  # timed passes behind scan_ms
    hash_s = max(scan_ms / 1e3 / passes, 1e-9)  # hashing kernels per pass
    checked = torch.tensor([parity_acc[0], parity_acc[1], parity_acc[2]], dtype=torch.int64,
                           device=coll_device(dev))
    if world > 1:
        dist.all_reduce(checked)
    c4_traffic, c4_sq, c4_read = None, {}, None
    if walked_batches == len(layouts) and args.c4_files == 1024 and world == 1:
        c4_traffic, pmc = pmc_traffic("C4", "rcdc_walk_kernel")
        c4_sq = (pmc or {}).get("sq") or {}
        c4_read = (pmc or {}).get("hbm_read_bytes_per_launch")
    # north_star's fraction: HBM bytes read (rocprof FETCH_SIZE, calibrated)
    # / kernel time; the lanes' bytes stand in without a PMC file
    c4_phys = c4_read if c4_read else lane_hashed
    if rank == 0:
        line = {
            "metric": METRIC, "value": round(total / el_max / GiB, 2), "unit": "GiB/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el_max / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic: uniform random bytes per file (torch.randint, seed 4000+file)",
            "config": {"workload": f"C4: {args.c4_files} files, log-uniform 4-256 MiB "
                                   f"({sum(sizes) / GiB:.1f} GiB), LPT-sharded over {world} GPU(s) "
                                   "(BASELINE.json configs[3])",
                       "batches_on_rank0": len(batches), "rank0_share_gib": round(share / GiB, 2),
                       "poly": hex(POLY), "min": MIN, "avg": AVG, "max": MAX,
                       "parallelism": f"per-file LPT sharding over {world} GPU(s), no collectives"},
            "roofline": {"bound": "hbm",
                         "kernel": ("rcdc_walk_kernel" if walked_batches == len(layouts) else
                                    f"rcdc_walk_kernel ({walked_batches} batches) + "
                                    f"rcdc_scan_kernel ({len(layouts) - walked_batches})"),
                         "achieved": round(c4_phys / hash_s / 1e9, 1) if runs else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(c4_phys / hash_s / 1e9 / HBM_PEAK_GBS, 4) if runs else None,
                         "basis": ("HBM bytes read per pass: rocprof FETCH_SIZE (calibrated, "
                                   "profiles/pmc_C4.json) / hashing-kernel time" if c4_read else
                                   "bytes the lanes read per pass (device work counters) / "
                                   "hashing-kernel time (no PMC file for this configuration)"),
                         "traffic": c4_traffic,
                         "frac_fetch": (round(c4_read / hash_s / 1e9 / HBM_PEAK_GBS, 4)
                                        if c4_read else None),
                         "achieved_input_basis_gbs": round(share / hash_s / 1e9, 1) if runs else None,
                         "frac_input_basis": (round(share / hash_s / 1e9 / HBM_PEAK_GBS, 4)
                                              if runs else None),
                         "ref_hashed_bytes_per_pass": ref_hashed,
                         "frac_ref_hashed": round(ref_hashed / hash_s / 1e9 / HBM_PEAK_GBS, 4),
                         "lane_hashed_bytes_per_pass": lane_hashed,
                         "frac_lane_hashed": round(lane_hashed / hash_s / 1e9 / HBM_PEAK_GBS, 4),
                         "hash_ms_per_pass": round(scan_ms / passes, 3),
                         "chain_ms_per_pass": round(resolve_ms / passes, 3),
                         "timed_passes": passes, "pipelined": pipelined,
                         "valu_busy": c4_sq.get("valu_busy"),
                         "valu_per_lane_byte": c4_sq.get("valu_per_lane_byte"),
                         "limiter": "VALU issue (~7 VALU + 2 LDS reads per hashed byte; "
                                    "DESIGN.md 3)"},
            "parity": {"files_checked": int(checked[0]), "files_total": len(sizes),
                       "mismatches": int(checked[1]), "cuts_diffed": int(checked[2]),
                       "seconds_rank0": round(parity_acc[3], 2),
                       "checker": "oracle/cdc_ref on every file of every rank's share "
                                  "(untimed, after the timed passes)"},
        }
        if world == 1 and not args.no_cpu_baseline and sample_cuts:
            from rustic_core_amd.device import pack_offsets
            hosts = [h for _, h in sample_cuts.values()]
            offs, alen = pack_offsets([len(h) for h in hosts])
            buf = np.zeros(alen, np.uint8)
            for o, h in zip(offs, hosts):
                buf[int(o):int(o) + len(h)] = h
            line["cpu_baseline"] = cpu_baseline(buf, offs, np.array([len(h) for h in hosts],
                                                                    np.uint64), args.cpu_seconds)
            line["cpu_baseline"]["sample"] += " (the 64-file parity sample of C4)"
        print(json.dumps(line), flush=True)
    for _, _, p in layouts:
        p.close()


def run_c1(args, torch, dev, rank, world):
    """C1 (BASELINE.json configs[0]): one 256 MiB file through the chunker,
    examples/backup/examples/backup.rs:14-36 plumbing restated: a file on
    disk, opened and read by ChunkIter.from_config (chunker.rs:22-47) as
    FileArchiver::backup_reader does (archiver/file_archiver.rs:144-160).
    The bytes are StdRng::seed_from_u64(0x256).
    value: the drop-in path (file reads + rcdc_stream_feed: H2D, device
    chunking, cuts D2H), GiB/s; beside it the device-resident rate of the
    same bytes and the reference-equivalent CPU chunker on 1 thread (the
    configuration's own measurement: one file is one iterator, one thread)."""
    import tempfile
    from rustic_core_amd import ChunkIter, ConfigFile
    from rustic_core_amd.chunker import Context
    from rustic_core_amd.device import DevicePlan, pack_offsets
    n = args.stream_bytes or (256 << 20)
    cfg = ConfigFile.new(2, POLY)

    def drop_in(data):
        """(GiB/s, cut offsets) of the drop-in path over `data` in a file."""
        fd, path = tempfile.mkstemp(prefix="rcdc_c1_", dir=os.environ.get("TMPDIR", "/tmp"))
        with os.fdopen(fd, "wb") as f:
            f.write(data.tobytes())
        try:
            def one_pass():
                out = []
                with open(path, "rb") as f:
                    for c in ChunkIter.from_config(cfg, f, n):
                        out.append(len(c))
                return out
            lens = one_pass()  # warm: context, lanes, plans, page cache
            for _ in range(max(args.warmup - 1, 0)):
                one_pass()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                lens = one_pass()
            el = time.perf_counter() - t0
        finally:
            os.unlink(path)
        return el, np.cumsum(np.array(lens, dtype=np.uint64))

    # BASELINE.json configs[0] names a /dev/urandom file: one is read here
    # beside the reproducible StdRng(0x256) stand-in
    with open("/dev/urandom", "rb") as f:
        udata = np.frombuffer(f.read(n), dtype=np.uint8)
    el_u, cuts_u = drop_in(udata)
    data = stdrng_numpy(0x256, n)
    el, cuts = drop_in(data)
    # the same bytes device-resident
    ctx = Context.get(POLY, MIN, AVG, MAX, device=dev.index)
    offs, alen = pack_offsets([n])
    arena = torch.zeros(alen, dtype=torch.uint8, device=dev)
    arena[:n] = torch.from_numpy(data).to(dev)
    plan = DevicePlan(ctx, offs, [n], alen)
    sptr = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(20):
        plan.run(arena.data_ptr(), sptr)
    torch.cuda.synchronize(dev)
    plan.set_timing(True, 1)
    t1 = time.perf_counter()
    for _ in range(50):
        plan.run(arena.data_ptr(), sptr)
    torch.cuda.synchronize(dev)
    el_dev = (time.perf_counter() - t1) / 50
    plan.set_timing(False)
    runs, scan_ms, res_ms = plan.kernel_times()
    dev_cuts = plan.results()[0]
    inf = plan.info()
    plan.close()
    from oracle import oracle  # checker + CPU baseline
    want = oracle.chunk_cuts(data)
    t2 = time.perf_counter()
    reps = 0
    while time.perf_counter() - t2 < args.cpu_seconds:
        oracle.chunk_many_owned(data, np.zeros(1, np.uint64), np.array([n], np.uint64),
                                nthreads=1)
        reps += 1
    el_cpu = (time.perf_counter() - t2) / reps
    want_u = oracle.chunk_cuts(udata)
    t3 = time.perf_counter()
    reps_u = 0
    while time.perf_counter() - t3 < min(args.cpu_seconds, 3.0):
        oracle.chunk_many_owned(udata, np.zeros(1, np.uint64), np.array([n], np.uint64),
                                nthreads=1)
        reps_u += 1
    el_cpu_u = (time.perf_counter() - t3) / reps_u
    scan_s = scan_ms / max(runs, 1) / 1e3
    line = {
        "metric": METRIC, "value": round(n * args.steps / el / GiB, 3), "unit": "GiB/s",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "StdRng::seed_from_u64(0x256) bytes (ChaCha12, SURVEY.md 8(d)) in a file",
        "config": {"workload": f"C1: one {n >> 20} MiB file through ChunkIter.from_config "
                               "(file reads + C ABI stream: H2D, device chunking, cuts D2H; "
                               "BASELINE.json configs[0])",
                   "poly": hex(POLY), "min": MIN, "avg": AVG, "max": MAX,
                   "parallelism": "one file = one iterator (the reference runs it on one thread)"},
        "device_resident": {"gibs": round(n / el_dev / GiB, 1), "kernel_us": round(scan_s * 1e6, 1),
                            "chain_or_resolve_us": round(res_ms / max(runs, 1) * 1e3, 1),
                            "walk_pieces": inf["walk_pieces"]},
        "roofline": {"bound": "hbm", "kernel": "rcdc_scan_kernel" if not inf["walk_pieces"]
                     else "rcdc_walk_kernel", "achieved": round(n / scan_s / 1e9, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(n / scan_s / 1e9 / HBM_PEAK_GBS, 4), "traffic": None,
                     "basis": "input bytes / hashing-kernel time (one 256 MiB stream: "
                              "latency-bound, far too small to fill the chip)"},
        "parity": {"chunks": int(len(cuts)),
                   "mismatches": int(not np.array_equal(cuts, want)) +
                   int(not np.array_equal(dev_cuts, want)),
                   "checker": "oracle/cdc_ref on the same bytes (drop-in path and device plan)"},
        "cpu_baseline": {"value": round(n / el_cpu / GiB, 3), "unit": "GiB/s", "cores": 1,
                         "kind": "port", "sample": f"the whole {n >> 20} MiB file, {reps} passes, "
                         "cdc_ref reference-equivalent mode (owned chunks, 4 KiB reads)",
                         "cpu_model": _cpu_model()},
        "urandom_file": {"gibs": round(n * args.steps / el_u / GiB, 3),
                         "ms_per_pass": round(el_u / args.steps * 1e3, 3),
                         "chunks": int(len(cuts_u)),
                         "mismatches": int(not np.array_equal(cuts_u, want_u)),
                         "cpu_gibs_1_thread": round(n / el_cpu_u / GiB, 3),
                         "note": f"{n >> 20} MiB read from /dev/urandom into a file, then the same "
                                 "drop-in path and checker (BASELINE.json configs[0] as stated)"},
    }
    print(json.dumps(line), flush=True)


def coll_device(dev):
    """Device of the timing collectives' tensors: the GPU under RCCL, the host
    under the gloo rehearsal backend."""
    return "cpu" if os.environ.get("RCDC_BENCH_BACKEND") == "gloo" else dev


def spawn_ranks(args) -> None:
    """`bench.py --gpus N` without a launcher: start N ranks with torchrun as a
    child process (before anything touches the GPU) and exit with its code.
    Under a launcher, WORLD_SIZE must equal --gpus."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws}", file=sys.stderr)
            sys.exit(2)
        return
    if args.gpus <= 1:
        return
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    sys.exit(subprocess.run(cmd, env=env).returncode)


def main():
    args = parse()
    spawn_ranks(args)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # RCDC_BENCH_BACKEND=gloo: rehearse N ranks on fewer GPUs (ranks share
    # devices round-robin; timing collectives over gloo).  Default: RCCL,
    # one GPU per rank.
    backend = os.environ.get("RCDC_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(torch.cuda.device_count(), 1)
    if world > 1:
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from rustic_core_amd.chunker import Context
    from rustic_core_amd.device import DevicePlan

    if args.workload == "C1":
        run_c1(args, torch, dev, rank, world)
        return
    if args.workload == "C4":
        run_c4(args, torch, dist, dev, rank, world, local)
        if world > 1:
            dist.destroy_process_group()
        return

    arena, offs, lens, desc = build_workload(args, torch, dev, rank, world)
    ctx = Context.get(POLY, MIN, AVG, MAX, device=local)
    plan = DevicePlan(ctx, offs, lens, int(arena.numel()))
    info = plan.info()
    pipelined = False
    if not args.no_pipeline and (args.pipeline or info.get("walk_pieces", 0) > 0):
        # rcdc_plan_set_pipeline: run k's chain kernels (check / fixup /
        # assemble, resolve) overlap run k + 1's hashing kernels
        plan.set_pipeline(True)
        pipelined = True
    # Unpipelined plans (C2) run on a stream of the job's own: given the
    # legacy default stream (handle 0) every rcdc call is ordered with it
    # through two events (rcdc.h), ~20 us of cross-queue latency per C2 step.
    # A pipelined plan already spreads a run over its own streams; a fifth
    # stream would share one of HIP's 4 hardware queues with them and
    # serialise run k's chain with run k + 1's walk (C3: 9.6 -> 14 ms).
    stream = torch.cuda.current_stream(dev) if pipelined else torch.cuda.Stream(dev)
    sptr = stream.cuda_stream
    ptr = arena.data_ptr()
    torch.cuda.synchronize(dev)  # the workload was built on the default stream

    step = lambda: plan.run(ptr, sptr)  # noqa: E731
    sliced = None
    if args.workload == "C5":
        # one stream over the ranks: every step runs the slice's plan, then
        # the stitch -- the crossing window of the device cut list
        # (rcdc_plan_window), one fixed-size all_gather of the windows, the
        # host walk over them; the cut lists stay on their ranks (at N = 1
        # the chain from 0 is the truth and there is nothing to stitch)
        from rustic_core_amd.shard import SlicedStream
        sliced = SlicedStream(ctx, arena, plan, desc["stream_bytes_total"], rank, world, MIN, MAX,
                              stream=sptr)
        step = sliced.step  # noqa: F811

    # W warmup steps, then more untimed steps until the card has run the
    # workload for --prewarm seconds: the first ~20 ms of back-to-back C2
    # steps run ~12 % slower (clock ramp), and K = 100 C2 steps are ~18 ms
    t_w = time.perf_counter()
    nw = 0
    while nw < args.warmup or time.perf_counter() - t_w < args.prewarm:
        step()
        nw += 1
        if nw % 32 == 0:
            torch.cuda.synchronize(dev)
    torch.cuda.synchronize(dev)

    # ---- timed region: K steps, barrier + sync on both sides, HIP events
    # around the scan kernel of every --time-every-th step
    # (rcdc_plan_set_timing: sampling keeps most steps free of event gaps)
    plan.set_timing(True, every=args.time_every)
    stitch_warm = sliced.stitch_s if sliced is not None else 0.0  # (warmup steps' stitches)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    last = None
    for i in range(args.steps):
        if pipelined and i == args.steps - 1 and not args.no_flush:
            plan.flush_next()  # the last run's chain is not beside a next walk: whole chip
        last = step()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    plan.set_timing(False)
    runs, scan_ms, resolve_ms = plan.kernel_times()
    t = torch.tensor([el], dtype=torch.float64, device=coll_device(dev))
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el_max = float(t.item())

    stitch = None
    if sliced is not None and world > 1:
        # per step, the plan's end to the stitch result (SlicedStream.step):
        # the crossing window, one all_gather, its .cpu(), the host walk;
        # timed steps only (the counters restart here), max over ranks
        n_st = max(args.steps, 1)
        st_t = torch.tensor([(sliced.stitch_s - stitch_warm) / n_st * 1e3], dtype=torch.float64,
                            device=coll_device(dev))
        dist.all_reduce(st_t, op=dist.ReduceOp.MAX)
        stitch = {"ms_per_step_max_rank": round(float(st_t.item()), 4), "steps": n_st,
                  "backend": dist.get_backend(),
                  "how": "host clock from the plan's end (device synchronised) to the stitch "
                         "result: rcdc_plan_window, one all_gather_into_tensor of 3 + k words "
                         "per rank, its .cpu(), the host walk over the windows"}
    if args.workload == "C5":
        total_bytes = desc["stream_bytes_total"] * args.steps
    else:
        total_bytes = int(lens.sum()) * args.steps * world
    value = total_bytes / el_max / GiB

    # dominant kernel, HIP events on its launch stream over the timed region
    # (rcdc_plan_set_timing: the first event pair brackets the hashing
    # kernels -- rcdc_scan_kernel for short streams, rcdc_walk_kernel for
    # long ones -- and the second the resolve / chain kernels).
    # Algorithmic bytes per launch: 1 byte read per INPUT
    # byte -> achieved = input bytes / hashing-kernel time.  Beside it:
    #   ref_hashed: the bytes the reference itself slides over (rabin.rs:127-188:
    #     per chunk 63 prefill bytes + (cut - (s + min)); from the cut lists);
    #   lane_hashed: the bytes our lanes hashed (device work counters: walk
    #     round bytes (64 x (S + 64) per round, shorter last rounds where the
    #     search end is known) + zones x 64 x 64; the scan: every position
    #     after the first min of a stream plus 64 B of warm-up per segment).
    walked = info.get("walk_pieces", 0) > 0
    in_bytes = int(lens.sum())
    scan_s = scan_ms / max(runs, 1) / 1e3
    achieved = in_bytes / scan_s / 1e9
    got_cuts = plan.results() if args.workload != "C5" else [np.asarray(plan.results()[0])]
    ref_hashed = ref_slide_bytes(got_cuts, MIN)
    if walked:
        st = plan.walk_stats()
        seg = info["walk_seg_bytes"]
        lane_hashed = st["round_bytes"] + st["zones"] * 64 * 64
        kernel = "rcdc_walk_kernel"
    else:
        st = None
        lane_hashed = info["scanned_bytes"] + 64 * info["segments"]
        kernel = "rcdc_scan_kernel"
    traffic, pmc = pmc_traffic(args.workload, kernel)
    # The headline fraction is north_star's: HBM bytes READ per launch (rocprof
    # FETCH_SIZE, calibrated for gfx950, profiles/pmc_<workload>.json) / kernel
    # time / 8 TB/s -- a real bandwidth fraction, never above 1.  Without a PMC
    # file for the workload, the bytes the lanes read stand in (they are within
    # ~1 % of FETCH on C3/C4).  The input-basis rate (input bytes / time:
    # the kernel skips the min prefixes the reference skips) is beside it.
    read_bytes = (pmc or {}).get("hbm_read_bytes_per_launch") if traffic else None
    phys = read_bytes if read_bytes else lane_hashed
    roofline = {
        "bound": "hbm",
        "kernel": kernel,
        "achieved": round(phys / scan_s / 1e9, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(phys / scan_s / 1e9 / HBM_PEAK_GBS, 4),
        "basis": ("HBM bytes read per launch: rocprof FETCH_SIZE (calibrated) of this kernel "
                  "on this workload (traffic_source) / HIP-event kernel time"
                  if read_bytes else
                  "bytes the lanes read per launch (device work counters) / HIP-event kernel "
                  "time (no PMC file for this workload)"),
        "traffic": traffic,
        "frac_fetch": round(read_bytes / scan_s / 1e9 / HBM_PEAK_GBS, 4) if read_bytes else None,
        "algorithmic_bytes_per_launch": in_bytes,
        "achieved_input_basis_gbs": round(achieved, 1),
        "frac_input_basis": round(achieved / HBM_PEAK_GBS, 4),
        "input_basis_note": "input bytes per launch (SURVEY.md 8(d)) / kernel time: the kernel "
                            "skips the min prefixes the reference skips, so this exceeds the "
                            "bytes read",
        "kernel_us_per_launch": round(scan_s * 1e6, 2),
        "timed_launches": runs,
        ("chain_us_per_launch" if walked else "resolve_us_per_launch"):
            round(resolve_ms / max(runs, 1) * 1e3, 2),
        "ref_hashed_bytes_per_launch": ref_hashed,
        "achieved_ref_hashed_gbs": round(ref_hashed / scan_s / 1e9, 1),
        "frac_ref_hashed": round(ref_hashed / scan_s / 1e9 / HBM_PEAK_GBS, 4),
        "lane_hashed_bytes_per_launch": lane_hashed,
        "achieved_lane_hashed_gbs": round(lane_hashed / scan_s / 1e9, 1),
        "frac_lane_hashed": round(lane_hashed / scan_s / 1e9 / HBM_PEAK_GBS, 4),
        "segment_bytes": info["walk_seg_bytes"] if walked
        else info["segment_bytes"],
        "limiter": "VALU issue (~7 VALU + 2 LDS reads per hashed byte; DESIGN.md 3)",
        "pipelined": pipelined,
    }
    if st is not None:
        roofline["walk_work"] = st
    if pmc:
        roofline["traffic_source"] = pmc.get("source")
        sq = pmc.get("sq")
        if sq:  # the kernel's real limiter, from its SQ counters (tools/pmc_sq_json.py)
            roofline["valu_busy"] = sq.get("valu_busy")
            roofline["valu_per_lane_byte"] = sq.get("valu_per_lane_byte")
            roofline["sq_source"] = sq.get("source")
    if args.workload == "C5":
        # zeros: every chunk is decided by its all-zero prefill window; the
        # kernel reads ~64 B per chunk, so an input-basis "fraction of HBM"
        # is meaningless (it exceeds 1): report the bytes actually read
        read = lane_hashed + 64 * int(sum(len(c) for c in got_cuts))
        roofline.update({
            "achieved": round(read / scan_s / 1e9, 1),
            "frac": round(read / scan_s / 1e9 / HBM_PEAK_GBS, 6),
            "algorithmic_bytes_per_launch": read,
            "basis": "bytes the walk reads (zone windows + 64-B zero-run prefill windows); "
                     "input-basis rate beside it",
            "limiter": "latency of the zero-run hops (64 chunks per wave step), not bandwidth",
        })

    out_extra = {}
    if rank == 0 and not args.no_parity:
        out_extra["parity"] = parity_check(args, arena, offs, lens, plan,
                                           sliced.cuts(last) if sliced else last, desc)
    if rank == 0 and not args.no_cpu_baseline and world == 1:
        out_extra["cpu_baseline"] = cpu_baseline(arena, offs, lens, args.cpu_seconds)
    if args.sha256:
        out_extra["sha256"] = sha_measure(torch, plan, ptr, sptr, dev, args, arena, offs, lens,
                                          rank == 0 and world == 1 and not args.no_cpu_baseline)
    if args.aead and rank == 0:
        out_extra["aead"] = aead_measure(torch, plan, arena, offs, lens, dev, args,
                                         world == 1 and not args.no_cpu_baseline)
    if args.pack and rank == 0:
        out_extra["pack"] = pack_measure(torch, plan, arena, offs, lens, dev, args)
    # the backup data path is measured through the native engine (the C ABI's
    # rcdc_ingest_*, the `h2h` object); --ingest adds the Python/torch
    # device-resident variant (rustic_core_amd.ingest, a test reference)
    if rank == 0 and args.ingest and not args.no_ingest:
        out_extra["ingest"] = ingest_measure(torch, arena, offs, lens, dev, args)
    if rank == 0 and world == 1 and args.workload == "C3" and not args.no_h2h:
        out_extra["h2h"] = h2h_measure(args)
    if args.zstd and rank == 0:
        out_extra["zstd"] = zstd_measure(torch, plan, arena, offs, lens, dev, args,
                                         world == 1 and not args.no_cpu_baseline)
    if args.e2e and rank == 0:
        out_extra["e2e"] = e2e_rate(torch, arena, offs, lens, plan, args.workload)
    if args.abi_e2e and rank == 0 and os.path.exists(os.path.join(ROOT, "tools", "abi_e2e")):
        # the native driver of the C ABI (tools/abi_e2e.cpp): 16 threads,
        # 64 files x 256 MiB in pageable host memory, 16 MiB reads through
        # rcdc_stream_feed, and rcdc_chunk_batch over the same files; the
        # box's H2D copy rates beside them (the bound of this path)
        import subprocess
        r = subprocess.run([os.path.join(ROOT, "tools", "abi_e2e"), "--threads",
                            str(args.abi_threads), "--files", "64", "--file-mib", "256",
                            "--batch"] + (["--mixed"] if args.workload == "C3" else []),
                           capture_output=True, text=True, timeout=300)
        if r.returncode == 0:
            out_extra["abi_e2e_native"] = json.loads(r.stdout.strip().splitlines()[-1])
    if args.abi_e2e and rank == 0 and args.workload in ("C2", "C3"):
        k = min(len(lens), args.abi_files)
        files = [arena[int(offs[i]):int(offs[i]) + int(lens[i])].cpu().numpy() for i in range(k)]
        res, cuts = abi_e2e(files, args.abi_threads)
        from oracle import oracle
        res["mismatches"] = int(sum(not np.array_equal(c, oracle.chunk_cuts(f))
                                    for c, f in zip(cuts[:4], files[:4])))
        res["parity_files"] = min(4, k)
        res.update(pcie_rates(torch, dev))
        out_extra["abi_e2e"] = res

    if rank == 0:
        parallel = (f"per-stream sharding over {world} GPU(s), no collectives"
                    if args.workload != "C5" else
                    f"one stream sliced over {world} GPU(s); one fixed-size all_gather of "
                    "crossing windows per step for the cross-slice stitch (N > 1)")
        data = desc.pop("data")
        desc.pop("slice", None)
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": data,
            "config": dict(desc, poly=hex(POLY), min=MIN, avg=AVG, max=MAX,
                           parallelism=parallel),
            "roofline": roofline,
            "untimed_steps_run": nw,
        }
        if stitch is not None:
            line["stitch"] = stitch
        line.update(out_extra)
        print(json.dumps(line), flush=True)
    plan.close()
    if world > 1:
        dist.destroy_process_group()


def h2h_measure(args) -> dict:
    """The host-to-host backup data path through the C ABI (rcdc_ingest_*,
    the native engine), from files on disk: tools/ingest_e2e writes
    --h2h-files files of 1 GiB (mixed: about half zero runs), reads them once
    (page cache), then times reader threads pread-ing each file into the
    engine's page-locked slots -> chunk, ids, dedup, zstd, seal, verify,
    packs on the GPU -> pack files and pack ids in host memory; beside it the
    concurrent PCIe bound of the same bytes (file_archiver.rs:144-160,
    packer.rs:826-836).  A child process (its own HIP context)."""
    import shutil
    import subprocess
    import tempfile
    tool = os.path.join(ROOT, "tools", "ingest_e2e")
    if not os.path.exists(tool):
        return {"skipped": "tools/ingest_e2e not built"}
    tmp = os.environ.get("TMPDIR", "/tmp")
    # the files must fit the disk under TMPDIR (4 GiB to spare)
    files = args.h2h_files
    fit = int((shutil.disk_usage(tmp).free - (4 << 30)) // (1 << 30))
    if fit < files:
        files = max(min(fit, files), 4)
    with tempfile.TemporaryDirectory(prefix="rcdc_h2h_", dir=tmp) as d:
        out = os.path.join(d, "h2h.json")
        cuts_out = os.path.join(d, "cuts.bin")
        fdir = os.path.join(d, "files")
        r = subprocess.run([tool, "--dir", fdir, "--files", str(files), "--file-mib", "1024",
                            "--json", out, "--keep", "--cuts-out", cuts_out],
                           capture_output=True, text=True, timeout=600)
        if r.returncode not in (0, 3) or not os.path.exists(out):
            return {"error": f"ingest_e2e rc {r.returncode}: {r.stderr[-500:]}"}
        res = json.loads(open(out).read())
        if not args.no_parity and os.path.exists(cuts_out):
            res["checks"]["oracle"] = h2h_oracle_diff(fdir, cuts_out, files)
    if files != args.h2h_files:
        res["files_reduced_for_disk"] = {"asked": args.h2h_files, "ran": files}
    res["log"] = r.stderr.strip().splitlines()[-4:]
    return res


def h2h_oracle_diff(fdir: str, cuts_path: str, nfiles: int) -> dict:
    """The h2h run's cut lists (tools/ingest_e2e --cuts-out, the checked
    run) against the oracle, every file re-read from disk: untimed."""
    from oracle import oracle
    t0 = time.perf_counter()
    raw = np.fromfile(cuts_path, dtype=np.uint64)
    got, i = {}, 0
    while i < raw.size:
        f, n = int(raw[i]), int(raw[i + 1])
        got[f] = raw[i + 2:i + 2 + n]
        i += 2 + n
    threads = cpu_threads()[0]
    bad = diffed = 0
    group = 16  # files of 1 GiB per host batch
    for a in range(0, nfiles, group):
        fs = list(range(a, min(a + group, nfiles)))
        data = [np.fromfile(os.path.join(fdir, f"f{f}"), dtype=np.uint8) for f in fs]
        hoffs, pos = [], 0
        for x in data:
            hoffs.append(pos)
            pos += (x.size + 255) // 256 * 256
        host = np.empty(max(pos, 1), np.uint8)
        for o, x in zip(hoffs, data):
            host[o:o + x.size] = x
        want = oracle.chunk_many_cuts(host, hoffs, [x.size for x in data], POLY, MIN, AVG, MAX,
                                      nthreads=threads)
        for f, w in zip(fs, want):
            bad += f not in got or not np.array_equal(got[f], w)
            diffed += len(w)
        del host, data
    return {"files_checked": nfiles, "mismatches": bad, "cuts_diffed": diffed,
            "seconds": round(time.perf_counter() - t0, 2),
            "checker": f"oracle/cdc_ref on {threads} host threads, every file re-read from disk"}


def sha_measure(torch, plan, ptr, sptr, dev, args, arena, offs, lens, cpu: bool) -> dict:
    from rustic_core_amd.device import DevicePlan

    """Blob ids (SHA-256 per chunk, crypto/hasher.rs:17-19) on the device:
    hash-only kernel time over the plan's cut list (HIP events on the launch
    stream), the fused chunk + hash step rate, a hashlib spot check and a
    hashlib CPU rate.  The kernel is VALU-bound (~21 VALU ops per byte,
    DESIGN.md 3c), so its roofline is the measured VALU issue rate, not HBM."""
    import hashlib

    # a stream of our own: torch's current stream may be the null stream
    # (cuda_stream == 0), which the C ABI maps to the context's stream, and
    # the events must be on the stream the kernel is launched on
    side = torch.cuda.Stream(dev)
    sptr = side.cuda_stream
    plan.run(ptr, sptr)
    plan.hash(ptr, sptr)
    torch.cuda.synchronize(dev)
    cuts = plan.results()
    nchunks = int(sum(len(c) for c in cuts))
    in_bytes = int(lens.sum())
    k = max(args.sha_steps, 1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(side)
    for _ in range(k):
        plan.hash(ptr, sptr)
    e1.record(side)
    torch.cuda.synchronize(dev)
    hash_ms = e0.elapsed_time(e1) / k
    t0 = time.perf_counter()
    for _ in range(k):
        plan.run(ptr, sptr)
        plan.hash(ptr, sptr)
    torch.cuda.synchronize(dev)
    fused_s = (time.perf_counter() - t0) / k
    # spot check: the first chunks of up to 4 streams against hashlib
    digs = plan.digests()
    checked = mism = 0
    for i in range(min(4, len(lens))):
        o = int(offs[i])
        prev = 0
        for j, c in enumerate(cuts[i][:8]):
            b = arena[o + prev:o + int(c)].cpu().numpy().tobytes()
            mism += hashlib.sha256(b).digest() != bytes(digs[i][j])
            checked += 1
            prev = int(c)
    out = {
        "kernel": "rcdc_sha256_plan_split_kernel (+ count/order length buckets)",
        "chunks_per_launch": nchunks,
        "hash_ms_per_launch": round(hash_ms, 3),
        "hash_gibs": round(in_bytes / (hash_ms / 1e3) / GiB, 2),
        "fused_chunk_and_hash_gibs": round(in_bytes / fused_s / GiB, 2),
        "bound": "per-chunk chain latency (SHA-256 is sequential within a chunk; one lane "
                 "pair per chunk: schedule wave + rounds wave)",
        "spot_check": {"chunks": checked, "mismatches": mism, "checker": "hashlib"},
    }
    # ingest pipeline: 2 groups of D plans over the same (read-only) arena.
    # A group's D batches are chunked on the main stream and their blob ids
    # hashed in ONE launch (rcdc_plan_hash_many) on a side stream, while the
    # other group's batches are chunked: D batches share the longest-chunk
    # latency floor
    from rustic_core_amd.device import hash_many
    depth = min(max(args.sha_depth, 1), 8)
    plans = [plan] + [DevicePlan(plan.ctx, offs, lens, int(arena.numel()))
                      for _ in range(2 * depth - 1)]
    groups = [plans[:depth], plans[depth:]]
    sides = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    chunk_stream = torch.cuda.Stream(dev)
    done = [None, None]
    ngroups = max(2, -(-2 * k // depth))

    def ingest_group(j):
        grp, sd = groups[j % 2], sides[j % 2]
        if done[j % 2] is not None:
            chunk_stream.wait_event(done[j % 2])  # this group's last hash has finished
        for pl in grp:
            pl.run(ptr, chunk_stream.cuda_stream)
        ev_run = torch.cuda.Event()
        ev_run.record(chunk_stream)
        sd.wait_event(ev_run)
        hash_many(grp, [ptr] * len(grp), sd.cuda_stream)
        ev = torch.cuda.Event()
        ev.record(sd)
        done[j % 2] = ev

    for j in range(2):
        ingest_group(j)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for j in range(ngroups):
        ingest_group(j)
    torch.cuda.synchronize(dev)
    nb = ngroups * depth
    out["pipelined_ingest_gibs"] = round(in_bytes * nb / (time.perf_counter() - t0) / GiB, 2)
    out["pipelined_ingest_note"] = (f"groups of {depth} batches: chunked on one stream, blob ids "
                                    f"in one rcdc_plan_hash_many launch overlapping the next "
                                    f"group ({nb} batches timed)")
    last = groups[(ngroups - 1) % 2][-1]
    out["pipelined_ingest_consistent"] = bool(
        all(np.array_equal(a, b) for a, b in zip(last.results(), cuts))
        and all(np.array_equal(a, b) for a, b in zip(last.digests(), digs)))
    for pl in plans[1:]:
        pl.close()
    if cpu:
        sample = arena[int(offs[0]):int(offs[0]) + min(int(lens[0]), 256 << 20)].cpu().numpy()
        sample = sample.tobytes()
        t0, n = time.perf_counter(), 0
        while time.perf_counter() - t0 < 2.0:
            hashlib.sha256(sample).digest()
            n += len(sample)
        out["cpu_hashlib_gibs_1thread"] = round(n / (time.perf_counter() - t0) / GiB, 3)
    return out


def aead_measure(torch, plan, arena, offs, lens, dev, args, cpu: bool) -> dict:
    """Blob encryption of the chunks just cut: every
    chunk of the first --aead-streams streams becomes one blob, sealed
    (crypto/aespoly1305.rs:119-135, per blob as blob/packer.rs:268-270 does)
    into a packed output arena and opened back (:88-108).  Kernel time by
    HIP events on the launch stream; spot checks against the oracle; the
    oracle's 1-thread C AES-CTR + Poly1305 as the CPU rate."""
    from rustic_core_amd.crypto import Key, make_refs, sealed_layout
    ns = min(len(lens), max(args.aead_streams, 1))
    cuts = plan.results()[:ns]
    in_offs, blens = [], []
    for i in range(ns):
        prev = 0
        for c in cuts[i]:
            in_offs.append(int(offs[i]) + prev)
            blens.append(int(c) - prev)
            prev = int(c)
    nb = len(blens)
    tot = int(sum(blens))
    rng = np.random.default_rng(0x5EA1)
    key = Key(rng.integers(0, 256, 64, dtype=np.uint8).tobytes())
    nonces = rng.integers(0, 256, (nb, 16), dtype=np.uint8)
    oo, olen = sealed_layout(blens)
    seal_refs = make_refs(in_offs, blens, oo, nonces)
    sealed = torch.empty(olen + 64, dtype=torch.uint8, device=dev)
    po, p = [], 0
    for n in blens:
        po.append(p)
        p = (p + n + 15) // 16 * 16
    open_refs = make_refs(oo, [n + 32 for n in blens], po)
    plain = torch.empty(p + 64, dtype=torch.uint8, device=dev)
    side = torch.cuda.Stream(dev)
    sp = side.cuda_stream
    a, s_ptr, pl = arena.data_ptr(), sealed.data_ptr(), plain.data_ptr()
    key.seal_blobs(a, seal_refs, s_ptr, sp)
    st = key.open_blobs(s_ptr, open_refs, pl, sp)
    torch.cuda.synchronize(dev)
    k = 5
    e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    e[0].record(side)
    for _ in range(k):
        key.seal_blobs(a, seal_refs, s_ptr, sp)
    e[1].record(side)
    torch.cuda.synchronize(dev)
    seal_ms = e[0].elapsed_time(e[1]) / k
    # open is synchronous (status to the host): time the launches the same way
    e[2].record(side)
    for _ in range(k):
        st = key.open_blobs(s_ptr, open_refs, pl, sp)
    e[3].record(side)
    torch.cuda.synchronize(dev)
    open_ms = e[2].elapsed_time(e[3]) / k
    from oracle import oracle
    checked = mism = 0
    idx = sorted(set([0, 1, nb - 1] + [int(x) for x in rng.integers(0, nb, 5)]))
    for i in idx:
        d = arena[in_offs[i]:in_offs[i] + blens[i]].cpu().numpy().tobytes()
        want = oracle.seal(key._key, nonces[i].tobytes(), d)
        got = sealed[int(oo[i]):int(oo[i]) + blens[i] + 32].cpu().numpy().tobytes()
        back = plain[po[i]:po[i] + blens[i]].cpu().numpy().tobytes()
        mism += (got != want) + (back != d)
        checked += 1
    out = {
        "kernel": "rcdc_aead_unit_kernel (+ rcdc_aead_finish_kernel)",
        "blobs": nb,
        "bytes": tot,
        "seal_ms_per_launch": round(seal_ms, 3),
        "seal_gibs": round(tot / (seal_ms / 1e3) / GiB, 2),
        "open_ms_per_launch": round(open_ms, 3),
        "open_gibs": round(tot / (open_ms / 1e3) / GiB, 2),
        "hbm_frac_seal": round(2 * tot / (seal_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
        "bound": "VALU/LDS issue: AES-256 = 14 rounds x 16 T-table LDS lookups + ~40 VALU per "
                 "16-byte block, Poly1305 ~30 VALU per block (DESIGN.md 3d)",
        "mac_failures": int(np.count_nonzero(st)),
        "spot_check": {"blobs": checked, "mismatches": int(mism),
                       "checker": "oracle/crypto_ref (seal) + round trip (open)"},
    }
    if cpu:
        sample = arena[in_offs[0]:in_offs[0] + min(tot, 64 << 20)].cpu().numpy().tobytes()
        t0, n = time.perf_counter(), 0
        while time.perf_counter() - t0 < 3.0:
            oracle.seal(key._key, nonces[0].tobytes(), sample)
            n += len(sample)
        out["cpu_baseline"] = {"value": round(n / (time.perf_counter() - t0) / GiB, 3),
                               "unit": "GiB/s", "cores": 1, "kind": "port",
                               "sample": f"oracle seal of {len(sample) >> 20} MiB, repeated 3 s"}
    del sealed, plain
    torch.cuda.empty_cache()
    return out


def ingest_measure(torch, arena, offs, lens, dev, args) -> dict:
    """The backup data path of a version-2 repository on the device, end to
    end over the first --ingest-streams streams, through the product API
    (rustic_core_amd/ingest.py DeviceIngest: SURVEY.md 8(a) + 8(f)): chunk,
    blob ids (short and long chunks on two streams), dedup against the
    packer's and the index's ids (packer.rs:304-315), zstd of the new blobs
    (the long chunks speculatively under their ids), seal, extra_verify
    (open + decode + compare every sealed blob on the device, decrypt.rs:
    508-529, the reference's default), and the pack files (add_raw + sealed
    headers, packer.rs:615-735).  Wall time of the whole call (host steps
    included) after one untimed call, each with an empty index; one pack
    checked by the oracle: header, every blob opened, decoded by libzstd and
    hashed back to its id."""
    import hashlib
    from oracle import oracle, zstd_ref as zr
    from rustic_core_amd.chunker import ConfigFile
    from rustic_core_amd.crypto import Key
    from rustic_core_amd.ingest import DeviceIngest
    ns = min(len(lens), max(args.ingest_streams, 1))
    rng = np.random.default_rng(0x1A6E)
    key = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
    cfg = ConfigFile.new(2, POLY)
    cfg.compression = args.zstd_level if args.zstd_level != 0 else None
    ing = DeviceIngest(cfg, Key(key), device=dev.index or 0)
    o, n = [int(x) for x in offs[:ns]], [int(x) for x in lens[:ns]]
    times, res = [], None
    from rustic_core_amd.pack import PackSizer
    for r in range(4):
        ing.indexed = set()  # each call: a fresh repository (empty index and sizer)
        ing.sizer = PackSizer.from_config(cfg, 0, 0)
        del res
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        res = ing.ingest(arena, o, n, finalize=True)
        torch.cuda.synchronize(dev)
        if r:
            times.append((time.perf_counter() - t0, res.ms))
    best_t, best_ms = min(times, key=lambda x: x[0])
    inb = int(sum(n))
    # one pack, checked by the oracle
    j = len(res.pack_table) // 2
    f = res.pack_file(j)
    parsed = oracle.parse_pack(key, f)
    b0 = int(res.pack_table[j]["blob0"])
    nidx = np.nonzero(res.new)[0]
    ok = len(parsed) == int(res.pack_table[j]["nblobs"])
    for k, (tpe, off, ln, ulen, bid) in enumerate(parsed):
        plain = zr.decompress(oracle.open_(key, f[off:off + ln]))
        c = nidx[b0 + k]
        a0, n0 = int(res.chunk_offs[c]), int(res.chunk_lens[c])
        src = arena[a0:a0 + n0].cpu().numpy().tobytes()
        ok &= plain == src and hashlib.sha256(plain).digest() == bytes(bid) and ulen == len(src)
    uniq = len(np.unique(np.ascontiguousarray(res.ids).view(np.dtype((np.void, 32)))))
    out = {
        "path": "rustic_core_amd.ingest.DeviceIngest: chunk -> blob ids (short || long chunks) "
                "-> dedup -> zstd (new blobs; long chunks speculatively under their ids) -> seal "
                "-> extra_verify (open + decode + compare, on the device) -> packs (add_raw + "
                "sealed headers); all bytes stay in HBM",
        "streams": ns, "input_bytes": inb, "chunks": len(res.ids), "unique_blobs": uniq,
        "new_blobs": int(res.new.sum()), "unique_bytes": int(res.chunk_lens[res.new].sum()),
        "pack_bytes": res.pack_bytes, "packs": len(res.pack_table),
        "extra_verify": ing.extra_verify, "zstd_level": ing.level,
        "ms": {k: round(v, 2) for k, v in best_ms.items()},
        "gibs_input": round(inb / best_t / GiB, 2),
        "check": {"pack": j, "ok": bool(ok) and uniq == int(res.new.sum()),
                  "checker": "oracle.parse_pack + oracle.open_ + libzstd decode + sha256 == id "
                             "for every blob of one pack; new blobs == distinct ids"},
        "floor": "the longest chunk's SHA-256 chain (one lane, ~2 us per 64-B block: ~0.27 s "
                 "for an 8 MiB chunk) bounds one call (DESIGN.md 3c)",
        "note": "pack ids (SHA-256 of each pack file, packer.rs:833) are left to the writer",
    }
    ing.close()
    del res
    torch.cuda.empty_cache()
    return out


def zstd_measure(torch, plan, arena, offs, lens, dev, args, cpu: bool) -> dict:
    """Blob compression of the chunks just cut (the
    zstd half): every chunk of the first --aead-streams streams becomes one
    zstd frame (backend/decrypt.rs:489-503 encode_all, per blob as
    blob/packer.rs:268-270), one rcdc_zstd_compress call.  Time by HIP events
    on the launch stream; a sample of frames decoded with libzstd (the
    checker); libzstd level 3 on the host's threads as the CPU rate."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import zstd_ref as zr
    from rustic_core_amd.compress import compress_blobs, frame_layout, make_refs
    ns = min(len(lens), max(args.aead_streams, 1))
    cuts = plan.results()[:ns]
    in_offs, blens = [], []
    for i in range(ns):
        prev = 0
        for c in cuts[i]:
            in_offs.append(int(offs[i]) + prev)
            blens.append(int(c) - prev)
            prev = int(c)
    nb, tot = len(blens), int(sum(blens))
    f_offs, ftot = frame_layout(blens)
    frames = torch.empty(ftot + 64, dtype=torch.uint8, device=dev)
    refs = make_refs(in_offs, blens, f_offs)
    side = torch.cuda.Stream(dev)
    sp = side.cuda_stream
    ctx = plan.ctx
    a, f = arena.data_ptr(), frames.data_ptr()
    out_lens = compress_blobs(ctx, a, refs, f, args.zstd_level, sp)
    torch.cuda.synchronize(dev)
    k = 5
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    t0 = time.perf_counter()
    e[0].record(side)
    for _ in range(k):
        out_lens = compress_blobs(ctx, a, refs, f, args.zstd_level, sp)
    e[1].record(side)
    torch.cuda.synchronize(dev)
    wall_ms = (time.perf_counter() - t0) * 1e3 / k
    ms = e[0].elapsed_time(e[1]) / k
    flen = int(np.sum(out_lens))
    rng = np.random.default_rng(0x2575)
    idx = sorted(set([0, nb - 1] + [int(x) for x in rng.integers(0, nb, 10)]))
    mism = 0
    for i in idx:
        d = arena[in_offs[i]:in_offs[i] + blens[i]].cpu().numpy().tobytes()
        fr = frames[int(f_offs[i]):int(f_offs[i]) + int(out_lens[i])].cpu().numpy().tobytes()
        mism += zr.decompress(fr) != d
    out = {
        "kernels": "rcdc_zstd_block_kernel + rcdc_zstd_frame_kernel + rcdc_zstd_copy_kernel",
        "level": args.zstd_level, "blobs": nb, "bytes": tot, "frame_bytes": flen,
        "ratio": round(flen / max(tot, 1), 4),
        "ms_per_call": round(ms, 3), "wall_ms_per_call": round(wall_ms, 3),
        "gibs": round(tot / (ms / 1e3) / GiB, 2),
        "hbm_frac": round((tot + flen) / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
        "check": {"blobs": len(idx), "mismatches": int(mism),
                  "checker": f"libzstd {zr.version()} ZSTD_decompress (oracle/zstd_ref.py)"},
    }
    if cpu:
        # libzstd level 3 (the library rustic links, another version) on the
        # same chunks, one chunk per task on the process's threads, ~5 s
        thr = cpu_threads()[0]
        host = {}
        sample, sb = [], 0
        for i in range(nb):
            if sb >= (2 << 30):
                break
            sample.append(i)
            sb += blens[i]
        for i in sample:
            host[i] = arena[in_offs[i]:in_offs[i] + blens[i]].cpu().numpy()
        bufs = {i: np.empty(zr.lib().ZSTD_compressBound(blens[i]), np.uint8) for i in sample}

        def one(i):
            h, b = host[i], bufs[i]
            return zr.compress_into(b.ctypes.data, len(b), h.ctypes.data, len(h), 3)

        done, clen, t0 = 0, 0, time.perf_counter()
        with ThreadPoolExecutor(thr) as ex:
            while time.perf_counter() - t0 < 5.0:
                clen = sum(ex.map(one, sample))
                done += sb
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {
            "value": round(done / dt / GiB, 3), "unit": "GiB/s", "cores": thr,
            "kind": "reference",
            "sample": f"libzstd {zr.version()} ZSTD_compress level 3 over the first {len(sample)} "
                      f"chunks ({sb / GiB:.2f} GiB), repeated ~5 s, one chunk per task",
            "ratio_level3": round(clen / max(sb, 1), 4),
            "device_ratio_same_chunks": round(int(np.sum(out_lens[:len(sample)])) / max(sb, 1), 4),
        }
    del frames
    torch.cuda.empty_cache()
    return out


def pack_measure(torch, plan, arena, offs, lens, dev, args) -> dict:
    """The packer's byte work on the chunks just cut:
    blob ids on the device (rcdc_plan_hash), dedup by id (the indexer's
    has(), packer.rs:304-315), grouping by PackSizer (32 MiB data packs,
    packer.rs:65-200), then ONE rcdc_pack_build over all packs: every unique
    chunk sealed into its pack, headers sealed and appended.  Kernel time by
    HIP events on the launch stream; one pack checked with the oracle."""
    from rustic_core_amd.chunker import ConfigFile
    from rustic_core_amd.pack import PackSizer, build_packs, group_blobs, make_blobs, pack_layout
    ns = min(len(lens), max(args.aead_streams, 1))
    side = torch.cuda.Stream(dev)
    sp = side.cuda_stream
    ptr = arena.data_ptr()
    plan.run(ptr, sp)
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record(side)
    plan.hash(ptr, sp)
    e[1].record(side)
    torch.cuda.synchronize(dev)
    hash_ms = e[0].elapsed_time(e[1])
    cuts, digs = plan.results()[:ns], plan.digests()[:ns]
    seen, in_offs, blens, ids = set(), [], [], []
    nchunks = 0
    for i in range(ns):
        prev = 0
        for c, d in zip(cuts[i], digs[i]):
            nchunks += 1
            k = d.tobytes()
            if k not in seen:
                seen.add(k)
                in_offs.append(int(offs[i]) + prev)
                blens.append(int(c) - prev)
                ids.append(d)
            prev = int(c)
    rng = np.random.default_rng(0x9AC)
    nb = len(blens)
    blobs = make_blobs(in_offs, blens, ids, rng.integers(0, 256, (nb, 16), dtype=np.uint8))
    groups = group_blobs(blens, PackSizer.from_config(ConfigFile.new(2, POLY), 0, 0))
    packs, total = pack_layout(blobs, groups,
                               rng.integers(0, 256, (len(groups), 16), dtype=np.uint8))
    out = torch.empty(total + 64, dtype=torch.uint8, device=dev)
    key = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
    ctx = plan.ctx
    build_packs(ctx, key, ptr, blobs, packs, out.data_ptr(), total, sp)
    torch.cuda.synchronize(dev)
    k = 5
    e[0].record(side)
    for _ in range(k):
        offsets = build_packs(ctx, key, ptr, blobs, packs, out.data_ptr(), total, sp)
    e[1].record(side)
    torch.cuda.synchronize(dev)
    pack_ms = e[0].elapsed_time(e[1]) / k
    uniq = int(sum(blens))
    from oracle import oracle
    j = len(groups) // 2
    p = packs[j]
    f = out[int(p["out_off"]):int(p["out_off"]) + int(p["size"])].cpu().numpy().tobytes()
    parsed = oracle.parse_pack(key, f)
    b0 = int(p["blob0"])
    ok = [bytes(bid) for _, _, _, _, bid in parsed] == \
        [blobs[i]["id"].tobytes() for i in range(b0, b0 + int(p["nblobs"]))]
    o0, l0 = parsed[0][1], parsed[0][2]
    ok &= oracle.open_(key, f[o0:o0 + l0]) == \
        arena[in_offs[b0]:in_offs[b0] + blens[b0]].cpu().numpy().tobytes()
    ok &= [int(x) for x in offsets[b0:b0 + int(p["nblobs"])]] == [o for _, o, _, _, _ in parsed]
    del out
    torch.cuda.empty_cache()
    return {
        "kernels": "rcdc_sha256 plan kernels (ids) + rcdc_aead_unit/finish_kernel (blobs, headers)",
        "chunks": nchunks, "unique_blobs": nb, "packs": len(groups),
        "input_bytes": int(sum(int(x) for x in lens[:ns])), "unique_bytes": uniq,
        "pack_bytes": int(total),
        "hash_ms": round(hash_ms, 3), "pack_build_ms": round(pack_ms, 3),
        "pack_build_gibs_unique": round(uniq / (pack_ms / 1e3) / GiB, 2),
        "hash_plus_pack_gibs_input": round(int(sum(int(x) for x in lens[:ns])) /
                                           ((hash_ms + pack_ms) / 1e3) / GiB, 2),
        "check": {"pack": j, "ok": bool(ok),
                  "checker": "oracle.parse_pack (header ids, offsets) + oracle.open_ of its "
                             "first blob vs the source chunk"},
        "note": "pack ids (SHA-256 of each pack file, packer.rs:833) are left to the writer",
    }


def parity_check(args, arena, offs, lens, plan, last, desc) -> dict:
    """Diff the measured run's cut lists against the oracle: every stream of
    C2 and C3 (--parity-streams caps it); C5: the whole slice against the
    closed form (zeros: every chunk is exactly min) and the first 256 MiB of
    the slice against the oracle."""
    from oracle import oracle
    got = plan.results()
    if args.workload == "C5":
        cuts = np.asarray(last, dtype=np.uint64)
        a, b, _ = desc["slice"]
        total = desc["stream_bytes_total"]
        want = np.arange((a // MIN + 1) * MIN, total + MIN, MIN, dtype=np.uint64)
        want = np.minimum(want, total)
        want = want[: int(np.searchsorted(want, b)) + 1] if b < total else want
        bad_closed = int(not np.array_equal(cuts, want))
        k = min(256 * MiB, int(lens[0]))
        o = oracle.chunk_cuts(arena[:k].cpu().numpy())
        g0 = got[0]
        bad_oracle = int(not np.array_equal(g0[g0 < k], o[o < k]))
        return {"cuts": int(len(cuts)), "mismatches": bad_closed + bad_oracle,
                "checker": "closed form (zeros) over the slice + oracle/cdc_ref on its first "
                           "256 MiB"}
    n = len(lens)
    if args.parity_streams:
        n = min(len(lens), args.parity_streams)
    threads = cpu_threads()[0]
    t0 = time.perf_counter()
    bad, diffed = oracle_diff(arena, offs[:n], lens[:n], got[:n], threads)
    return {"streams_checked": n, "streams_total": int(len(lens)), "mismatches": bad,
            "cuts_diffed": int(diffed), "cuts_total": int(sum(len(x) for x in got)),
            "seconds": round(time.perf_counter() - t0, 2),
            "checker": f"oracle/cdc_ref reference-equivalent mode on {threads} host threads, "
                       "every stream of the measured run"}


def oracle_diff(arena, offs, lens, got, threads: int):
    """Diff device cut lists got[k] of streams [offs[k], +lens[k]) of the
    device arena against the oracle: in host batches of <= 16 GiB (D2H
    copy, then the oracle on the host's threads, one stream per thread as
    archiver.rs:195).  Returns (streams that differ, cuts diffed)."""
    import torch
    from oracle import oracle
    n = len(lens)
    bad = diffed = 0
    i = 0
    while i < n:
        j, tot = i, 0
        while j < n and (j == i or tot + int(lens[j]) <= (16 << 30)):
            tot += int(lens[j])
            j += 1
        hoffs, pos = [], 0
        for k in range(i, j):
            hoffs.append(pos)
            pos += (int(lens[k]) + 255) // 256 * 256
        host = np.empty(max(pos, 1), dtype=np.uint8)
        ht = torch.from_numpy(host)
        for k, ho in zip(range(i, j), hoffs):
            o, m = int(offs[k]), int(lens[k])
            ht[ho:ho + m].copy_(arena[o:o + m])
        want = oracle.chunk_many_cuts(host, hoffs, [int(lens[k]) for k in range(i, j)],
                                      POLY, MIN, AVG, MAX, nthreads=threads)
        for k, w in zip(range(i, j), want):
            bad += not np.array_equal(got[k], w)
            diffed += len(w)
        del host, ht
        i = j
    return bad, diffed


def e2e_rate(torch, arena, offs, lens, plan, workload, reps: int = 5) -> dict:
    """PCIe-inclusive rate: pinned host bytes -> H2D -> chunk -> D2H of the
    cuts.  C2/C5: serialised.  C3: the next batch's H2D (8 streams) on a side
    stream overlaps the chunking of the current one (double buffer)."""
    if workload != "C3":
        host = torch.empty(arena.numel(), dtype=torch.uint8, pin_memory=True)
        host.copy_(arena.cpu())
        dst = torch.empty_like(arena)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            dst.copy_(host, non_blocking=True)
            plan.run(dst.data_ptr(), torch.cuda.current_stream().cuda_stream)
            plan.results()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        return {"value": int(np.sum(lens)) * reps / el / GiB, "unit": "GiB/s",
                "note": "pinned H2D + scan + resolve + D2H cut lists, serialized (no overlap)"}
    from rustic_core_amd.chunker import Context
    from rustic_core_amd.device import DevicePlan, pack_offsets
    per = 8
    blens = np.asarray(lens[:per], dtype=np.uint64)
    boffs, blen = pack_offsets(blens)
    host = torch.empty(blen, dtype=torch.uint8, pin_memory=True)
    for j in range(per):
        o = int(offs[j])
        host[int(boffs[j]):int(boffs[j]) + int(blens[j])].copy_(arena[o:o + int(blens[j])].cpu())
    bufs = [torch.empty(blen, dtype=torch.uint8, device=arena.device) for _ in range(2)]
    ctx = Context.get(POLY, MIN, AVG, MAX, device=arena.device.index)
    plans = [DevicePlan(ctx, boffs, blens, blen) for _ in range(2)]
    copy_s = torch.cuda.Stream()
    comp = torch.cuda.current_stream()
    ev = [torch.cuda.Event() for _ in range(2)]
    nb = max(len(lens) // per, 1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(copy_s):
        bufs[0].copy_(host, non_blocking=True)
        ev[0].record(copy_s)
    for k in range(nb):
        cur = k % 2
        comp.wait_event(ev[cur])
        if k + 1 < nb:
            nxt = (k + 1) % 2
            copy_s.wait_stream(comp)  # bufs[nxt] is no longer read by batch k-1
            with torch.cuda.stream(copy_s):
                bufs[nxt].copy_(host, non_blocking=True)
                ev[nxt].record(copy_s)
        plans[cur].run(bufs[cur].data_ptr(), comp.cuda_stream)
        plans[cur].results()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    for p in plans:
        p.close()
    return {"value": nb * int(np.sum(blens)) / el / GiB, "unit": "GiB/s",
            "note": (f"{nb} batches of {per} x {int(blens[0]) / GiB:g} GiB: pinned H2D of batch "
                     "k+1 on a side stream overlapped with scan + resolve + D2H cuts of batch k "
                     "(the same pinned bytes re-sent per batch)")}


if __name__ == "__main__":
    main()
