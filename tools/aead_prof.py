"""Device blob encryption alone, for rocprofv3 (--kernel-trace --stats, --pmc):
seals and opens N random chunk-sized blobs (C3-like lengths: 512 KiB - 8 MiB)
``--reps`` times.  usage: python tools/aead_prof.py [--gib 8] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from rustic_core_amd import _lib  # noqa: E402
from rustic_core_amd.crypto import Key, make_refs, sealed_layout  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=8.0)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--lib", default=None, help="an experimental build of librcdc.so")
    a = ap.parse_args()
    if a.lib:
        _lib.LIB_PATH = os.path.abspath(a.lib)
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(11)
    total = int(a.gib * (1 << 30))
    lens = []
    while sum(lens) < total:
        lens.append(int(rng.integers(512 << 10, 8 << 20)))
    n = len(lens)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    tot = int(sum(lens))
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    arena = torch.randint(0, 256, (tot + 64,), dtype=torch.uint8, device=dev, generator=g)
    key = Key(rng.integers(0, 256, 64, dtype=np.uint8).tobytes())
    oo, olen = sealed_layout(lens)
    seal_refs = make_refs(offs, lens, oo, rng.integers(0, 256, (n, 16), dtype=np.uint8))
    sealed = torch.empty(olen + 64, dtype=torch.uint8, device=dev)
    po, p = [], 0
    for x in lens:
        po.append(p)
        p = (p + x + 15) // 16 * 16
    open_refs = make_refs(oo, [x + 32 for x in lens], po)
    plain = torch.empty(p + 64, dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream(dev)
    key.seal_blobs(arena.data_ptr(), seal_refs, sealed.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        key.seal_blobs(arena.data_ptr(), seal_refs, sealed.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    ts = (time.perf_counter() - t0) / a.reps
    t0 = time.perf_counter()
    for _ in range(a.reps):
        st = key.open_blobs(sealed.data_ptr(), open_refs, plain.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    to = (time.perf_counter() - t0) / a.reps
    ok = bool(torch.equal(plain[:lens[0]], arena[:lens[0]])) and not st.any()
    # checksum of the sealed arena: equal across builds that agree byte for byte
    w = sealed[:olen // 8 * 8].view(torch.int64)
    csum = int((w * torch.arange(1, w.numel() + 1, device=dev, dtype=torch.int64)).sum())
    print(json.dumps({"lib": os.path.basename(_lib.LIB_PATH), "blobs": n, "bytes": tot, "seal_gibs": tot / ts / (1 << 30),
                      "open_gibs": tot / to / (1 << 30), "roundtrip_ok": ok,
                      "sealed_checksum": csum}), flush=True)


if __name__ == "__main__":
    main()
