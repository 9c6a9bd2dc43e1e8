"""SHA-256 blob ids on the device (rcdc_sha256.hip) -- §8(f) row 1.

Reference: ``hash(&chunk)`` = SHA-256 (crates/core/src/crypto/hasher.rs:17-19)
of every chunk FileArchiver::backup_reader yields
(archiver/file_archiver.rs:151).  Pinned by the reference's own chunker
snapshots, which hold (len, sha256) per chunk (rabin.rs:341-358 and
fixed_size.rs:82-102), and by FIPS 180-4 known answers.  hashlib is the
checker for the random cases.  Bit-exact digests are the bar.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "reference_snapshots.json")
MiB = 1 << 20

FIPS = [  # FIPS 180-4 / NIST CAVP short messages
    (b"", "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"),
    (b"abc", "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"),
    (b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq",
     "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"),
]


def _sha_dev(gpu_ctx, host: np.ndarray, refs):
    import torch
    from rustic_core_amd.device import sha256_device
    dev = torch.from_numpy(host).to("cuda:0")
    r = torch.tensor(np.asarray(refs, dtype=np.int64).reshape(-1, 2), device="cuda:0")
    out = sha256_device(gpu_ctx, dev, r)
    torch.cuda.synchronize()
    return [bytes(row).hex() for row in out.cpu().numpy()]


def test_fips_known_answers(gpu_ctx):
    arena = np.zeros(4096, dtype=np.uint8)
    refs = []
    o = 0
    for msg, _ in FIPS:
        o += 7  # unaligned starts
        arena[o:o + len(msg)] = np.frombuffer(msg, np.uint8) if msg else arena[o:o]
        refs.append((o, len(msg)))
        o += len(msg)
    got = _sha_dev(gpu_ctx, arena, refs)
    assert got == [h for _, h in FIPS]


def test_every_length_and_alignment(gpu_ctx):
    """Lengths 0..200 (all padding cases: r < 56, r >= 56, exact blocks) at
    every start alignment mod 4, plus lengths straddling an arena end."""
    rng = np.random.default_rng(7)
    arena = rng.integers(0, 256, 1 << 16, dtype=np.uint8)
    refs = [(1000 + 3 * ln + a, ln) for ln in range(0, 201) for a in range(4)]
    refs += [(len(arena) - ln, ln) for ln in (1, 3, 55, 56, 63, 64, 65, 127, 128, 4093)]
    got = _sha_dev(gpu_ctx, arena, refs)
    exp = [hashlib.sha256(arena[o:o + n].tobytes()).hexdigest() for o, n in refs]
    assert got == exp


def test_fixed_size_snapshots(gpu_ctx):
    """fixed_size.rs:82-102 snapshots: FixedSize cuts + device SHA-256."""
    from rustic_core_amd.chunker import fixed_cuts
    for g in json.load(open(GOLDEN))["fixed_chunk_random"]:
        data = oracle.stdrng_bytes(g["seed"], g["size"])
        cuts = fixed_cuts(len(data), g["chunk_size"])
        starts = np.concatenate([[0], cuts[:-1]]).astype(np.int64)
        refs = np.stack([starts, cuts.astype(np.int64) - starts], 1)
        got = _sha_dev(gpu_ctx, data, refs)
        assert [[int(n), h] for n, h in zip(refs[:, 1], got)] == g["chunks"]


def test_rabin_snapshot_fused(gpu_ctx):
    """rabin.rs:341-358 + chunk_random.snap: cuts and blob ids both from the
    device (rcdc_plan_run + rcdc_plan_hash), all 29 (len, sha256) exact."""
    import torch
    from rustic_core_amd.chunker import Context
    from rustic_core_amd.device import DevicePlan, pack_offsets
    g = json.load(open(GOLDEN))["rabin_chunk_random"]
    ctx = Context.get(int(g["poly"], 16), g["min"], g["avg"], g["max"], device=0)
    data = oracle.stdrng_bytes(g["seed"], g["size"])
    offs, arena_len = pack_offsets([len(data)])
    host = np.zeros(arena_len, dtype=np.uint8)
    host[:len(data)] = data
    dev = torch.from_numpy(host).to("cuda:0")
    plan = DevicePlan(ctx, offs, [len(data)], arena_len)
    plan.run(dev.data_ptr())
    plan.hash(dev.data_ptr())
    dig = plan.digests()[0]
    cuts = plan.results()[0]
    plan.close()
    lens = np.diff(np.concatenate([[0], cuts])).tolist()
    assert [[int(n), bytes(d).hex()] for n, d in zip(lens, dig)] == g["chunks"]


@pytest.mark.parametrize("kind", ["random", "mixed"])
def test_plan_hash_batch(gpu_ctx, kind):
    """A C2/C3-shaped batch (ragged streams, unaligned offsets, zero runs):
    fused digests == hashlib over the oracle's chunks."""
    import torch
    from rustic_core_amd.device import DevicePlan
    rng = np.random.default_rng(11)
    lens = [int(x) for x in rng.integers(0, 3 * MiB, 48)] + [0, 1, 524288, 524289]
    offs, o = [], 0
    for n in lens:
        o += int(rng.integers(0, 64))
        offs.append(o)
        o += n
    arena = np.zeros(o + 512, dtype=np.uint8)
    for i, (s, n) in enumerate(zip(offs, lens)):
        b = oracle.stdrng_bytes(500 + i, n)
        if kind == "mixed" and n > 4096:
            b = b.copy()
            z0 = int(rng.integers(0, n // 2))
            b[z0:z0 + n // 3] = 0
        arena[s:s + n] = b
    dev = torch.from_numpy(arena).to("cuda:0")
    plan = DevicePlan(gpu_ctx, np.array(offs, np.uint64), lens, len(arena))
    plan.run(dev.data_ptr())
    plan.hash(dev.data_ptr())
    digs = plan.digests()
    cuts = plan.results()
    plan.close()
    for i, (s, n) in enumerate(zip(offs, lens)):
        exp_cuts = oracle.chunk_cuts(arena[s:s + n])
        assert np.array_equal(cuts[i], exp_cuts), i
        starts = np.concatenate([[0], exp_cuts[:-1]]) if len(exp_cuts) else []
        exp = [hashlib.sha256(arena[s + int(a):s + int(b)].tobytes()).digest()
               for a, b in zip(starts, exp_cuts)]
        assert [bytes(d) for d in digs[i]] == exp, i


@pytest.mark.parametrize("kind", ["random", "mixed"])
def test_plan_hash_walk_path(gpu_ctx, kind, monkeypatch):
    """Long streams take the walk path: the fused digests of
    every chunk of 4 x 40 MiB streams (plus short ones on the scan path in
    the same plan) == hashlib over the oracle's chunks; the plan is walked."""
    import torch
    from rustic_core_amd.device import DevicePlan, pack_offsets
    monkeypatch.setenv("RCDC_WALK_MIN_PIECES", "4")  # small batch: walk anyway
    lens = [40 * MiB + 13 * i for i in range(4)] + [MiB, 700000]
    rng = np.random.default_rng(5)
    bufs = []
    for i, n in enumerate(lens):
        b = oracle.stdrng_bytes(900 + i, n)
        if kind == "mixed":
            b = b.copy()
            for _ in range(8):
                z0 = int(rng.integers(0, n))
                b[z0:z0 + int(rng.integers(4096, 3 * MiB))] = 0
        bufs.append(b)
    offs, arena_len = pack_offsets(lens)
    arena = np.zeros(arena_len, dtype=np.uint8)
    for o, b in zip(offs, bufs):
        arena[int(o):int(o) + len(b)] = b
    dev = torch.from_numpy(arena).to("cuda:0")
    plan = DevicePlan(gpu_ctx, offs, lens, arena_len)
    assert plan.info()["walk_pieces"] > 0
    plan.run(dev.data_ptr())
    plan.hash(dev.data_ptr())
    digs = plan.digests()
    cuts = plan.results()
    plan.close()
    for i, b in enumerate(bufs):
        exp_cuts = oracle.chunk_cuts(b)
        assert np.array_equal(cuts[i], exp_cuts), i
        starts = np.concatenate([[0], exp_cuts[:-1]])
        exp = [hashlib.sha256(b[int(a):int(e)].tobytes()).digest()
               for a, e in zip(starts, exp_cuts)]
        assert [bytes(d) for d in digs[i]] == exp, i


def test_plan_hash_many(gpu_ctx):
    """rcdc_plan_hash_many: 3 plans (different layouts and arenas) hashed in
    one launch == each plan hashed alone == hashlib on a sample."""
    import torch
    from rustic_core_amd.device import DevicePlan, hash_many, pack_offsets
    plans, devs, hosts, layouts = [], [], [], []
    for a, lens in enumerate([[MiB] * 40, [3 * MiB + 5, 700001, 0, 2 * MiB], [524289] * 7]):
        offs, alen = pack_offsets(lens)
        h = np.zeros(alen, dtype=np.uint8)
        for i, (o, n) in enumerate(zip(offs, lens)):
            h[int(o):int(o) + n] = oracle.stdrng_bytes(3000 + 100 * a + i, n)
        d = torch.from_numpy(h).to("cuda:0")
        p = DevicePlan(gpu_ctx, offs, lens, alen)
        p.run(d.data_ptr())
        plans.append(p)
        devs.append(d)
        hosts.append(h)
        layouts.append((offs, lens))
    hash_many(plans, [d.data_ptr() for d in devs])
    many = [p.digests() for p in plans]
    for p, d in zip(plans, devs):
        p.hash(d.data_ptr())
    for p, m, h, (offs, lens) in zip(plans, many, hosts, layouts):
        single = p.digests()
        assert all(np.array_equal(x, y) for x, y in zip(m, single))
        cuts = p.results()
        for i in range(len(lens)):
            o, prev = int(offs[i]), 0
            for j, c in enumerate(cuts[i]):
                assert bytes(m[i][j]) == hashlib.sha256(h[o + prev:o + int(c)].tobytes()).digest()
                prev = int(c)
        p.close()
