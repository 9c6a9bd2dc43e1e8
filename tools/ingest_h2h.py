"""Host-to-host backup data path: files in host memory ->
pack files and pack ids in host memory, on one MI355X, through
rustic_core_amd.ingest.HostIngest, next to the concurrent PCIe bound of the
same bytes.

Files: --files streams of --file-gib GiB of C3-style mixed data (bench.py
make_mixed: random runs 64 KiB-16 MiB and zero runs 4 KiB-16 MiB, seed
3000 + j), built on the device and copied to pinned host memory before the
timed region (as a reader thread would read them into pinned buffers).

Timed: HostIngest.run (first H2D issued .. last pack id computed).
Bound: the same H2D copies (three device slots, one copy stream) with the run's
pack bytes copied D2H on a second stream at the same time, no compute --
what the PCIe link allows this job in both directions.
Checks (untimed): every pack id against hashlib over the host pack bytes,
every pack header opened and parsed by the oracle (blob count, ids, offsets,
sizes against the device's pack table), every chunk id against hashlib over
the source bytes, every cut list against the oracle, the dedup decisions
(new blobs == distinct ids), and every blob of --open-packs packs opened by
the oracle, decoded by libzstd and hashed back to its id.

  python tools/ingest_h2h.py [--files 96] [--file-gib 1] [--json out.json]
"""
import argparse
import hashlib
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

# more hardware queues than HIP's default 4 before anything initialises HIP:
# the pipeline's copy streams must not share a queue with its kernels
# (HostIngest docstring); --hw-queues=4 reproduces the shared-queue stall
_q = [a.split("=", 1)[1] for a in sys.argv if a.startswith("--hw-queues=")]
os.environ["GPU_MAX_HW_QUEUES"] = _q[0] if _q else "16"  # (the box exports 4)
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import POLY, make_mixed  # noqa: E402
from oracle import oracle, zstd_ref as zr  # noqa: E402
from rustic_core_amd.chunker import ConfigFile  # noqa: E402
from rustic_core_amd.crypto import Key  # noqa: E402
from rustic_core_amd.device import pack_offsets  # noqa: E402
from rustic_core_amd.ingest import HostIngest  # noqa: E402

GiB = 1 << 30


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_files(n, nbytes, dev):
    files = []
    tmp = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    for j in range(n):
        make_mixed(torch, tmp, 0, nbytes, np.random.default_rng(3000 + j), dev)
        h = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        h.copy_(tmp)
        files.append(h)
        if j % 16 == 15:
            log(f"files: {j + 1}/{n}")
    del tmp
    torch.cuda.synchronize(dev)
    return files


def pcie_bound(files, batches, d2h_bytes, dev, host_pack):
    """H2D of the run's batches into three slots (one stream) while d2h_bytes
    go device -> host on another stream: seconds."""
    sizes = [int(f.numel()) for f in files]
    lay = [pack_offsets([sizes[i] for i in b]) for b in batches]
    slot = max(a for _, a in lay)
    arenas = [torch.empty(slot, dtype=torch.uint8, device=dev) for _ in range(min(3, len(batches)))]
    src = torch.empty(min(d2h_bytes, 4 * GiB) + 1, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    with torch.cuda.stream(s2):
        o = 0
        while o < d2h_bytes:
            n = min(src.numel() - 1, d2h_bytes - o)
            host_pack[o:o + n].copy_(src[:n], non_blocking=True)
            o += n
    with torch.cuda.stream(s1):
        for k, b in enumerate(batches):
            a = arenas[k % len(arenas)]
            for i, off in zip(b, lay[k][0]):
                a[int(off):int(off) + sizes[i]].copy_(files[i], non_blocking=True)
    s1.synchronize()
    t_h2d = time.perf_counter() - t0
    s2.synchronize()
    t_both = time.perf_counter() - t0
    # each direction alone
    t0 = time.perf_counter()
    with torch.cuda.stream(s1):
        for k, b in enumerate(batches):
            a = arenas[k % len(arenas)]
            for i, off in zip(b, lay[k][0]):
                a[int(off):int(off) + sizes[i]].copy_(files[i], non_blocking=True)
    s1.synchronize()
    t_h2d_alone = time.perf_counter() - t0
    t0 = time.perf_counter()
    with torch.cuda.stream(s2):
        o = 0
        while o < d2h_bytes:
            n = min(src.numel() - 1, d2h_bytes - o)
            host_pack[o:o + n].copy_(src[:n], non_blocking=True)
            o += n
    s2.synchronize()
    t_d2h_alone = time.perf_counter() - t0
    del arenas, src
    torch.cuda.empty_cache()
    return {"seconds_both": t_both, "seconds_h2d_while_d2h": t_h2d,
            "h2d_alone_gibs": sum(sizes) / t_h2d_alone / GiB,
            "d2h_alone_gibs": d2h_bytes / t_d2h_alone / GiB}


def checks(res, files, key, open_packs, threads):
    out = {}
    pool = ThreadPoolExecutor(threads)
    # pack ids
    ids = list(pool.map(lambda k: hashlib.sha256(memoryview(
        res.packs_host[int(res.pack_offs[k]):int(res.pack_offs[k]) + int(res.pack_sizes[k])]
        .numpy())).digest(), range(len(res.pack_sizes))))
    out["pack_ids_ok"] = ids == res.pack_ids
    # pack headers by the oracle, against the device pack tables
    rows = []
    for r in res.batches:
        for p in r.pack_table:
            b0, nb = int(p["blob0"]), int(p["nblobs"])
            rows.append((int(p["size"]), r.blobs[b0:b0 + nb], r.blob_offsets[b0:b0 + nb]))
    hdr_ok = len(rows) == len(res.pack_sizes)
    for k, (size, blobs, boffs) in enumerate(rows):
        o = int(res.pack_offs[k])
        f = res.packs_host[o:o + size].numpy()
        hlen = int.from_bytes(f[-4:].tobytes(), "little")
        parsed = oracle.parse_pack(key, f[-4 - hlen:].tobytes())
        ok = size == int(res.pack_sizes[k]) and len(parsed) == len(blobs)
        end = 0
        for (tpe, off, ln, ulen, bid), b, bo in zip(parsed, blobs, boffs):
            ok &= (tpe == 0 and off == int(bo) and ln == int(b["len"]) and
                   bytes(bid) == bytes(b["id"]) and ulen == int(b["uncompressed_len"]))
            end = off + ln
        ok &= end + hlen + 4 == size
        hdr_ok &= bool(ok)
    out["pack_headers_ok"] = bool(hdr_ok)
    out["packs"] = len(rows)
    # chunk cuts against the oracle and chunk ids against hashlib, per batch
    cuts_ok = ids_ok = True
    nchunks = 0
    all_ids = []
    for r, b in zip(res.batches, res.batch_files):
        exp = list(pool.map(lambda i: oracle.chunk_cuts(files[i].numpy()), b))
        for got, e in zip(r.cuts, exp):
            cuts_ok &= np.array_equal(got, e)
        refs = []
        for i, c in zip(b, exp):
            prev = 0
            for x in c:
                refs.append((i, prev, int(x)))
                prev = int(x)
        hs = list(pool.map(lambda t: hashlib.sha256(memoryview(
            files[t[0]].numpy()[t[1]:t[2]])).digest(), refs))
        ids_ok &= hs == [bytes(x) for x in r.ids]
        nchunks += len(hs)
        all_ids += hs
    out["cuts_ok"] = bool(cuts_ok)
    out["chunk_ids_ok"] = bool(ids_ok)
    out["chunks"] = nchunks
    new = int(sum(int(r.new.sum()) for r in res.batches))
    packed = sum(len(b) for _, b, _ in rows)
    out["new_blobs"] = new
    out["dedup_ok"] = new == len(set(all_ids)) == packed
    # every blob of a few packs opened, decoded and hashed back to its id
    pick = sorted(set(np.linspace(0, len(rows) - 1, open_packs).astype(int).tolist())) if rows else []
    opened = 0
    ok = True
    for k in pick:
        size, blobs, boffs = rows[k]
        o = int(res.pack_offs[k])
        f = res.packs_host[o:o + size].numpy()
        for b, bo in zip(blobs, boffs):
            plain = oracle.open_(key, f[int(bo):int(bo) + int(b["len"])].tobytes())
            data = zr.decompress(plain)
            ok &= hashlib.sha256(data).digest() == bytes(b["id"]) and len(data) == int(
                b["uncompressed_len"])
            opened += 1
    out["blobs_opened"] = opened
    out["blobs_opened_ok"] = bool(ok)
    pool.shutdown()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=96)
    ap.add_argument("--file-gib", type=float, default=1.0)
    ap.add_argument("--first-gib", type=float, default=2)
    ap.add_argument("--batch-gib", type=float, default=8)
    ap.add_argument("--last-gib", type=float, default=1)
    ap.add_argument("--hash-threads", type=int, default=None)
    ap.add_argument("--open-packs", type=int, default=3)
    ap.add_argument("--repeat", type=int, default=1, help="timed runs (fresh repository each)")
    ap.add_argument("--no-checks", action="store_true")
    ap.add_argument("--no-multi-buffer", action="store_true",
                    help="pack ids with hashlib only (no rcdc_sha256_host)")
    ap.add_argument("--mb-half", type=int, default=None,
                    help="HostIngest.mb_half_batches (batches hashed 8 packs per call)")
    ap.add_argument("--hashlib-tail", type=int, default=None,
                    help="HostIngest.hashlib_tail (last batches hashed one pack per thread)")
    ap.add_argument("--json", default=None)
    ap.add_argument("--hw-queues", default="16", help="GPU_MAX_HW_QUEUES for this process "
                    "(set before HIP initialises; --hw-queues=N form)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    nbytes = int(a.file_gib * GiB)
    t = time.perf_counter()
    files = make_files(a.files, nbytes, dev)
    log(f"files ready ({time.perf_counter() - t:.1f} s)")
    key = np.random.default_rng(0x4A2).integers(0, 256, 64, dtype=np.uint8).tobytes()
    cfg = ConfigFile.new(2, POLY)
    kw = dict(first_batch=int(a.first_gib * GiB), batch=int(a.batch_gib * GiB),
              last_batch=int(a.last_gib * GiB), hash_threads=a.hash_threads)
    # warm-up: contexts, plans, kernels, pinned pools (a small run, its own repository)
    # (one batch as large as the run's largest, so the context's device
    # scratch -- zstd, AEAD, frame check -- is sized before the timed run)
    w = HostIngest(cfg, Key(key), **kw)
    nw = min(len(files), int(a.batch_gib * GiB) // nbytes + 1)
    w.first_batch = w.batch = w.last_batch = nw * nbytes
    w.run(files[:nw])
    w.close()
    del w
    torch.cuda.synchronize(dev)
    log("warm-up done")
    hi = HostIngest(cfg, Key(key), **kw)
    if a.no_multi_buffer:
        hi.multi_buffer_ids = False
    if a.mb_half is not None:
        hi.mb_half_batches = a.mb_half
    if a.hashlib_tail is not None:
        hi.hashlib_tail = a.hashlib_tail
    res = hi.run(files)
    total = sum(int(f.numel()) for f in files)
    log(f"run: {res.seconds:.3f} s, {total / res.seconds / GiB:.1f} GiB/s, "
        f"{len(res.pack_ids)} packs, {res.d2h_bytes / 1e9:.1f} GB D2H")
    chk = None
    if not a.no_checks:  # (before the bound run, which overwrites the host pack buffer)
        t = time.perf_counter()
        chk = checks(res, files, key, a.open_packs, hi.hash_threads)
        chk["seconds"] = round(time.perf_counter() - t, 1)
        log(f"checks: {chk}")
    # the host's pack-id budget on these very bytes: every pack hashed again
    # with the run's thread count, nothing else running
    t = time.perf_counter()
    with ThreadPoolExecutor(hi.hash_threads) as pool:
        list(pool.map(lambda k: hashlib.sha256(memoryview(res.packs_host[
            int(res.pack_offs[k]):int(res.pack_offs[k]) + int(res.pack_sizes[k])].numpy())).digest(),
            range(len(res.pack_sizes))))
    rehash_s = time.perf_counter() - t
    bound = pcie_bound(files, res.batch_files, res.d2h_bytes, dev, res.packs_host)
    bound_s = bound["seconds_both"]
    line = {
        "metric": "host-to-host backup data path GiB/s (files in host memory -> pack files + "
                  "pack ids in host memory), 1 x MI355X",
        "value": round(total / res.seconds / GiB, 2), "unit": "GiB/s",
        "seconds": round(res.seconds, 4),
        "input_bytes": total, "h2d_bytes": res.h2d_bytes, "d2h_bytes": res.d2h_bytes,
        "pcie_bound": {"gibs_input": round(total / bound_s / GiB, 2),
                       "seconds": round(bound_s, 4),
                       "h2d_alone_gibs": round(bound["h2d_alone_gibs"], 2),
                       "d2h_alone_gibs": round(bound["d2h_alone_gibs"], 2),
                       "how": "the run's H2D copies (3 device slots, one stream) with its pack "
                              "bytes D2H on a second stream at the same time, no compute"},
        "frac_of_bound": round(bound_s / res.seconds, 3),
        "pack_id_hashing": {"host_gbs_alone": round(res.d2h_bytes / rehash_s / 1e9, 2),
                            "seconds_alone": round(rehash_s, 3),
                            "thread_seconds_in_run": res.ms.get("hash_thread_s"),
                            "note": "SHA-256 of every pack file (packer.rs:832-834) on the "
                                    "job's host threads; hashing all packs alone takes "
                                    "seconds_alone"},
        "batches": [len(b) for b in res.batch_files],
        "hash_threads": hi.hash_threads,
        "multi_buffer_ids": hi.multi_buffer_ids,
        "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
        "host_ms": {k: (round(v, 1) if isinstance(v, float) else v) for k, v in res.ms.items()},
        "packs": len(res.pack_ids),
        "data": f"{a.files} x {a.file_gib:g} GiB C3-style mixed streams (bench.py make_mixed, "
                "seed 3000 + j) in pinned host memory; repository version 2 (zstd level 3), "
                "extra_verify on",
        "path": "rustic_core_amd.ingest.HostIngest: H2D (copy stream) -> DeviceIngest.begin "
                "(chunk, ids, long chunks speculatively) / end (dedup, short chunks, packs; "
                "packer open across batches) -> D2H (second copy stream) -> pack ids on host "
                "threads (rcdc_sha256_host, 16 packs per call in AVX-512 lanes; hashlib for "
                "the last batches)",
    }
    if chk is not None:
        line["checks"] = chk
    print(json.dumps(line), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            f.write(json.dumps(line) + "\n")
    hi.close()


if __name__ == "__main__":
    main()
