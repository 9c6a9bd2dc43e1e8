"""Host SHA-256 throughput over pack-sized buffers with 1..N threads: hashlib
(OpenSSL, one buffer per call) and rcdc_sha256_host (16 buffers per call in
AVX-512 lanes).  The pack-id budget of the host-to-host path (HostIngest
hashes every pack file on host threads, packer.rs:832-834)."""
import hashlib
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rustic_core_amd.device import sha256_host, sha256_host_supported  # noqa: E402

n_buf, size = 64, 32 << 20
bufs = [np.random.default_rng(i).integers(0, 256, size, dtype=np.uint8) for i in range(n_buf)]
out = {"buffer_mib": size >> 20, "buffers": n_buf, "cpu_affinity": len(os.sched_getaffinity(0))}
for t in [int(x) for x in (sys.argv[1:] or ["1", "8", "14", "16"])]:
    with ThreadPoolExecutor(t) as pool:
        list(pool.map(lambda b: hashlib.sha256(memoryview(b)).digest(), bufs[:t]))
        t0 = time.perf_counter()
        list(pool.map(lambda b: hashlib.sha256(memoryview(b)).digest(), bufs))
        el = time.perf_counter() - t0
    out[f"gbs_{t}_threads"] = round(n_buf * size / el / 1e9, 2)
    if sha256_host_supported():  # 16 buffers per call, t calls at a time
        groups = [bufs[i:i + 16] for i in range(0, n_buf, 16)] * max(1, t // 4)

        def one(g):
            return sha256_host([b.ctypes.data for b in g], [b.size for b in g])
        with ThreadPoolExecutor(t) as pool:
            t0 = time.perf_counter()
            list(pool.map(one, groups))
            el = time.perf_counter() - t0
        out[f"multibuffer_gbs_{t}_threads"] = round(len(groups) * 16 * size / el / 1e9, 2)
    from rustic_core_amd.native_ingest import sha256_host_ni  # noqa: E402
    for ways in (1, 2, 3, 4):  # SHA extensions, `ways` buffers interleaved per call
        groups = [bufs[i:i + ways] for i in range(0, n_buf, ways)]
        groups = groups[:max(t, len(groups) * t // 16)] if t < 16 else groups

        def ni(g, ways=ways):
            return sha256_host_ni([memoryview(b) for b in g], ways)
        with ThreadPoolExecutor(t) as pool:
            t0 = time.perf_counter()
            list(pool.map(ni, groups))
            el = time.perf_counter() - t0
        out[f"shani_x{ways}_gbs_{t}_threads"] = round(sum(len(g) for g in groups) * size / el / 1e9, 2)
print(json.dumps(out))
