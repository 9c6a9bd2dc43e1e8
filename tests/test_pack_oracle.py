"""CPU: the pack-file checker (oracle.pack_file / parse_pack: packer.rs
add_raw + save, packfile.rs HeaderEntry) and the host-side pack sizing of
rustic_core_amd.pack (PackSizer, packer.rs:65-200), before the device pack
builder is compared with them.

Pin: the reference's own pack file (repo-mixed fixture,
tests/golden/crypto_fixtures.json) is rebuilt byte for byte from its blobs'
plaintexts, nonces, ids and the header's nonce.
"""
import base64
import hashlib
import json
import os

import pytest

from tests.test_crypto_oracle import GOLD, _kdf, _master


def reference_pack(oracle_mod):
    """(master key, pack bytes, [(type, plain, id, nonce, raw_len)], header nonce)."""
    files = {k: base64.b64decode(v) for k, v in GOLD["repo_mixed"].items()}
    kname = [k for k in files if k.startswith("repo/keys/")][0]
    kf = json.loads(files[kname])
    mk = json.loads(oracle_mod.open_(_kdf(kf, GOLD["repo_mixed_password"]),
                                     base64.b64decode(kf["data"])))
    key = _master(mk)
    pack = [v for k, v in files.items() if k.startswith("repo/data/")][0]
    entries = oracle_mod.parse_pack(key, pack)
    blobs = []
    for tpe, off, length, ulen, bid in entries:
        sealed = pack[off:off + length]
        blobs.append((tpe, oracle_mod.open_(key, sealed), bid, sealed[:16], ulen))
    hlen = int.from_bytes(pack[-4:], "little")
    return key, pack, blobs, pack[-4 - hlen:-4 - hlen + 16]


def test_oracle_rebuilds_reference_pack(oracle_mod):
    key, pack, blobs, hnonce = reference_pack(oracle_mod)
    assert len(blobs) >= 2
    rebuilt, index = oracle_mod.pack_file(key, blobs, hnonce)
    assert rebuilt == pack
    # the pack id is the SHA-256 of the file (packer.rs:833): the fixture's name
    name = [k for k in GOLD["repo_mixed"] if k.startswith("repo/data/")][0]
    assert hashlib.sha256(rebuilt).hexdigest() == os.path.basename(name)
    # PackHeaderRef::pack_size (packfile.rs:364-369)
    assert len(pack) == 36 + sum(ln + (41 if b[4] else 37) for (_, ln), b in zip(index, blobs))


def test_pack_sizer():
    from rustic_core_amd.chunker import ConfigFile
    from rustic_core_amd.pack import MAX_SIZE, PackSizer
    cfg = ConfigFile.new(2, 0x3DA3358B4DC173)
    s = PackSizer.from_config(cfg, 0, 0)
    assert s.pack_size() == 32 << 20                       # DEFAULT_DATA_SIZE
    s.add_size(1 << 40)                                      # 1 TiB: + 32 * 2^20
    assert s.pack_size() == 64 << 20
    assert PackSizer.from_config(cfg, 1, 0).pack_size() == 4 << 20   # trees
    r = (126 << 20) + (1 << 19)                              # isqrt -> 32 r + 32 MiB = 4080 MiB
    big = PackSizer.from_config(cfg, 0, r * r)
    assert big.pack_size() == MAX_SIZE                       # clamped (packer.rs:145)
    # past 2^32 the u32 product wraps as the release build does
    # (`isqrt as u32 * grow_factor + default_size`, packer.rs:141)
    assert PackSizer.from_config(cfg, 0, 1 << 62).pack_size() == 32 << 20
    f = PackSizer.fixed(1000)
    assert f.pack_size() == 1000 and f.size_ok(1000) and f.is_too_small(999)
    assert f.is_too_large(1001)
    assert not s.is_too_large(10 ** 12)                      # max percent unset = u32::MAX
    assert s.is_too_small(int(0.29 * s.pack_size())) and not s.is_too_small(int(0.31 * s.pack_size()))


def test_group_blobs():
    from rustic_core_amd.pack import MAX_COUNT, PackSizer, group_blobs
    # size rule: a pack closes once its sealed bytes reach pack_size
    g = group_blobs([100] * 10, PackSizer.fixed(400))        # 132 B sealed each
    assert g == [(0, 4), (4, 4), (8, 2)]
    # count rule
    g = group_blobs([1] * (MAX_COUNT + 5), PackSizer.fixed(1 << 30))
    assert g == [(0, MAX_COUNT), (MAX_COUNT, 5)]
    # the sizer grows with what was written (take_data -> add_size)
    # (after the first 1000-byte pack, pack_size = isqrt(1073) + 1000 = 1032)
    s = PackSizer(1000, 1, 1 << 30, 0, 30, 0xFFFFFFFF)
    g = group_blobs([968] * 3, s)
    assert g == [(0, 1), (1, 2)]
    assert s.current_size == (1000 + 37 + 36) + (2000 + 2 * 37 + 36)


def test_group_blobs_open_matches_one_packer():
    """A packer that stays open between calls (packer.rs:659-671, 749-750)
    closes the same packs as one pass over all blobs: feed the blob lengths
    in several calls, carrying the open pack's blobs into the next call, and
    finalize at the end (one undersized pack per call before)."""
    import numpy as np
    from rustic_core_amd.pack import MAX_COUNT, PackSizer, group_blobs, group_blobs_open
    rng = np.random.default_rng(7)
    lens = [int(x) for x in rng.integers(1, 9000, 3000)]
    ulen = [int(x) if rng.random() < 0.5 else 0 for x in rng.integers(1, 20000, 3000)]
    one = group_blobs(lens, PackSizer(50_000, 8, 400_000, 0, 30, 200), ulen)
    sizer = PackSizer(50_000, 8, 400_000, 0, 30, 200)
    got, carry = [], []  # carry: indices of the open pack's blobs
    cuts = [0, 1, 17, 400, 401, 1500, 2999, 3000]
    for a, b in zip(cuts[:-1], cuts[1:]):
        idx = carry + list(range(a, b))
        last = b == cuts[-1]
        closed, open_from = group_blobs_open([lens[i] for i in idx], sizer,
                                             [ulen[i] for i in idx], finalize=last)
        got += [(idx[b0], n) for b0, n in closed]
        carry = idx[open_from:]
    assert not carry
    assert got == one
    assert sizer.current_size == PackSizer(50_000, 8, 400_000, 0, 30, 200).current_size + sum(
        sum(lens[b0:b0 + n]) + 32 * n + sum(41 if ulen[i] else 37 for i in range(b0, b0 + n))
        + 36 for b0, n in one)
    # the count rule closes a pack without finalize
    closed, open_from = group_blobs_open([1] * (MAX_COUNT + 5), PackSizer.fixed(1 << 30))
    assert closed == [(0, MAX_COUNT)] and open_from == MAX_COUNT
