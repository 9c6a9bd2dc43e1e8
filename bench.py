#!/usr/bin/env python
"""bench.py -- CDC chunking GiB/s, device-resident (BASELINE.json metric).

Workload (BASELINE.json configs[1], "C2"): per GPU, 1024 independent 1 MiB
random buffers resident in HBM; one step = one full chunking pass (scan
kernel + resolve kernel) over all of them, producing the cut offsets in HBM.
Parameters are rustic's defaults: P = 0x003DA3358B4DC173, min 512 KiB,
avg 1 MiB, max 8 MiB (crates/core/src/repofile/configfile.rs:36-41).

Multi-GPU: one process per GPU (torchrun), each rank chunks its own 1024
buffers (independent files shard per GPU, no collective on the data path:
"scaling": "weak"); the only collective is the timing barrier / max.

Output: ONE JSON line on rank 0 (the driver's contract), including the
roofline of the dominant kernel (scan, HIP events on its launch stream over
the timed region) and the CPU baseline (the oracle in reference-equivalent
mode, timed on this host, rank 0 at N=1 only; also the cut-list parity check).
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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--streams", type=int, default=1024)
    ap.add_argument("--stream-bytes", type=int, default=1 << 20)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--e2e", action="store_true",
                    help="also measure the PCIe-inclusive rate (pinned H2D + chunk + D2H cuts)")
    return ap.parse_args()


def cpu_baseline(host: np.ndarray, offs, lens, seconds: float) -> dict:
    """Oracle (cdc_ref, reference-equivalent work: owned chunk buffers fed by
    4 KiB reads, rabin.rs:110-191) over the same buffers, per-file threads as
    in archiver.rs:195.  Repeats whole passes until `seconds` elapsed."""
    from oracle import oracle
    try:
        ncpu = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        ncpu = os.cpu_count() or 1
    threads = max(1, min(16, ncpu))
    total = int(np.sum(lens))
    oracle.chunk_many_owned(host, offs, lens, nthreads=threads)  # warm
    t0 = time.perf_counter()
    passes = 0
    while True:
        oracle.chunk_many_owned(host, offs, lens, nthreads=threads)
        passes += 1
        el = time.perf_counter() - t0
        if el >= seconds or el >= 30.0:
            break
    # single-thread rate on a bounded sample (first 64 buffers)
    k = min(64, len(lens))
    t1 = time.perf_counter()
    oracle.chunk_many_owned(host, offs[:k], lens[:k], nthreads=1)
    el1 = time.perf_counter() - t1
    return {
        "value": passes * total / el / GiB,
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"{passes} full passes over the same {len(lens)} x "
                   f"{int(lens[0]) >> 10} KiB buffers ({passes * total / GiB:.1f} GiB, "
                   f"{el:.1f} s), cdc_ref reference-equivalent mode, {threads} threads "
                   f"(per-file parallel, archiver.rs:195)"),
        "single_thread_gibs": int(np.sum(lens[:k])) / el1 / GiB,
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


def pmc_traffic():
    """Per-launch HBM bytes of the scan kernel from the committed rocprofv3
    PMC summary (profiles/pmc_scan.json: FETCH_SIZE + WRITE_SIZE converted
    with the calibration for this access pattern, profiles/r01_pmc_hbm.txt);
    (None, None) if absent."""
    p = os.path.join(ROOT, "profiles", "pmc_scan.json")
    try:
        d = json.load(open(p))
        return d.get("hbm_bytes_per_launch"), d
    except (OSError, ValueError):
        return None, None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from rustic_core_amd.chunker import Context
    from rustic_core_amd.device import DevicePlan, pack_offsets

    n, sb = args.streams, args.stream_bytes
    lens = np.full(n, sb, dtype=np.uint64)
    offs, arena_len = pack_offsets(lens)
    g = torch.Generator(device=dev)
    g.manual_seed(1000 + rank)
    arena = torch.randint(0, 256, (arena_len,), dtype=torch.uint8, device=dev, generator=g)
    ctx = Context.get(POLY, MIN, AVG, MAX, device=local)
    plan = DevicePlan(ctx, offs, lens, arena_len)
    info = plan.info()
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    ptr = arena.data_ptr()

    for _ in range(args.warmup):
        plan.run(ptr, sptr)
    torch.cuda.synchronize(dev)

    # ---- timed region: K steps, barrier + sync on both sides, HIP events
    # around the scan kernel of every step (rcdc_plan_set_timing)
    plan.set_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        plan.run(ptr, sptr)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    plan.set_timing(False)
    runs, scan_ms, resolve_ms = plan.kernel_times()
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el_max = float(t.item())

    step_bytes = int(lens.sum())
    total_bytes = step_bytes * args.steps * world
    value = total_bytes / el_max / GiB

    # dominant kernel (scan), HIP events on its launch stream over the timed
    # region.  Algorithmic bytes per launch:
    # 1 byte read per INPUT byte -> achieved = input bytes / scan time.  The
    # kernel physically reads only the bytes it must hash, sum(N - min) (the
    # reference never hashes a chunk's first min bytes), plus 64 B of warm-up
    # per segment: that rate and the PMC-measured HBM traffic are reported
    # beside it.
    hashed = int(sum(max(int(x) - MIN, 0) for x in lens))
    scan_s = scan_ms / max(runs, 1) / 1e3
    achieved = step_bytes / scan_s / 1e9
    traffic, pmc = pmc_traffic()
    roofline = {
        "bound": "hbm",
        "kernel": "rcdc_scan_kernel",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": traffic,
        "algorithmic_bytes_per_launch": step_bytes,
        "scan_us_per_launch": round(scan_s * 1e6, 2),
        "resolve_us_per_launch": round(resolve_ms / max(runs, 1) * 1e3, 2),
        "hashed_bytes_per_launch": hashed,
        "achieved_hashed_gbs": round(hashed / scan_s / 1e9, 1),
        "frac_hashed": round(hashed / scan_s / 1e9 / HBM_PEAK_GBS, 4),
        "segment_bytes": info["segment_bytes"],
        "bytes_read_by_lanes": info["scanned_bytes"] + 64 * info["segments"],
        "limiter": "VALU issue (DESIGN.md 3: ~95% of the measured compute ceiling)",
    }
    if pmc:
        roofline["traffic_source"] = pmc.get("source")

    out_extra = {}
    if rank == 0 and not args.no_parity:
        from oracle import oracle
        host = arena.cpu().numpy()
        got = plan.results()
        bad = 0
        for i in range(n):
            o = int(offs[i])
            exp = oracle.chunk_cuts(host[o:o + int(lens[i])], POLY, MIN, AVG, MAX)
            bad += not np.array_equal(got[i], exp)
        out_extra["parity"] = {"streams_checked": n, "mismatches": bad,
                               "cuts": int(sum(len(x) for x in got)),
                               "checker": "oracle/cdc_ref (CPU restatement)"}
        if not args.no_cpu_baseline and world == 1:
            out_extra["cpu_baseline"] = cpu_baseline(host, offs, lens, args.cpu_seconds)
    if args.e2e and rank == 0:
        out_extra["e2e"] = e2e_rate(ctx, arena, offs, lens, plan)

    if rank == 0:
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
            "data": "synthetic: uniform random bytes (torch.randint on device, seed 1000+rank)",
            "config": {
                "workload": f"C2: {n} independent {sb >> 10} KiB random buffers per GPU, "
                            "device-resident (BASELINE.json configs[1])",
                "streams_per_gpu": n,
                "stream_bytes": sb,
                "poly": hex(POLY),
                "min": MIN, "avg": AVG, "max": MAX,
                "parallelism": f"per-stream sharding over {world} GPU(s), no collectives",
            },
            "roofline": roofline,
        }
        line.update(out_extra)
        print(json.dumps(line), flush=True)
    plan.close()
    if world > 1:
        dist.destroy_process_group()


def e2e_rate(ctx, arena, offs, lens, plan, reps: int = 5) -> dict:
    """PCIe-inclusive: pinned host bytes -> H2D -> chunk -> D2H of the cuts."""
    import torch
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


if __name__ == "__main__":
    main()
