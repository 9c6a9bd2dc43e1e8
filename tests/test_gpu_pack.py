"""Pack files built on the device (rcdc_pack_build) -- SURVEY.md 8(f) row 4.

Reference: ``BasicPacker::add_raw`` / ``save`` / ``write_header``
(blob/packer.rs:615-655, :505-510, :693-735) and ``HeaderEntry``
(repofile/packfile.rs:88-124): a pack is its blobs sealed back to back, the
sealed header (one entry per blob) and the header length as u32 LE.

Checker: oracle.pack_file / parse_pack, pinned in test_pack_oracle.py by
rebuilding the reference's own pack file byte for byte.  Here the device
rebuilds that same fixture pack byte for byte, and random batches of packs
(data/tree, compressed entries, unaligned inputs and outputs) match the
oracle exactly.  Sealed outputs at any alignment are also checked through
rcdc_aead_seal.
"""
import numpy as np
import pytest

from oracle import oracle
from tests.test_pack_oracle import reference_pack

pytestmark = pytest.mark.gpu


def _dev(host: np.ndarray):
    import torch
    return torch.from_numpy(np.ascontiguousarray(host)).to("cuda:0")


def _build(key, datas, specs, groups, hnonces, in_pads=None, align=1, fill=0xA5):
    """Device packs of `datas` (specs: (type, id, nonce, raw_len) per blob)."""
    import torch
    from rustic_core_amd.chunker import Context
    from rustic_core_amd.pack import build_packs, make_blobs, pack_layout
    offs, o = [], 0
    for i, d in enumerate(datas):
        o += in_pads[i] if in_pads else 0
        offs.append(o)
        o += len(d)
    arena = np.zeros(o + 64, np.uint8)
    for off, d in zip(offs, datas):
        arena[off:off + len(d)] = np.frombuffer(d, np.uint8)
    blobs = make_blobs(offs, [len(d) for d in datas], [s[1] for s in specs],
                       [np.frombuffer(s[2], np.uint8) for s in specs],
                       types=[s[0] for s in specs], uncompressed=[s[3] for s in specs])
    packs, total = pack_layout(blobs, groups, [np.frombuffer(h, np.uint8) for h in hnonces],
                               align=align)
    d_in = _dev(arena)
    d_out = torch.full((total + 64,), fill, dtype=torch.uint8, device="cuda:0")
    ctx = Context.get(oracle.DEFAULT_POLY, oracle.DEFAULT_MIN, oracle.DEFAULT_AVG,
                      oracle.DEFAULT_MAX, device=0)
    offsets = build_packs(ctx, key, d_in.data_ptr(), blobs, packs, d_out.data_ptr(), total)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    files = [out[int(p["out_off"]):int(p["out_off"]) + int(p["size"])].tobytes() for p in packs]
    return files, packs, offsets, out, total


def test_device_rebuilds_reference_pack(gpu_ctx):
    """The repo-mixed fixture's pack file, byte for byte, from its blobs
    (compressed and uncompressed entries), nonces, ids and header nonce."""
    key, pack, blobs, hnonce = reference_pack(oracle)
    datas = [b[1] for b in blobs]
    specs = [(b[0], np.frombuffer(b[2], np.uint8), b[3], b[4]) for b in blobs]
    files, packs, offsets, _, _ = _build(key, datas, specs, [(0, len(blobs))], [hnonce])
    assert files[0] == pack
    assert int(packs[0]["size"]) == len(pack)
    want = [(off, ln) for _, off, ln, _, _ in oracle.parse_pack(key, pack)]
    assert [(int(o), len(d) + 32) for o, d in zip(offsets, datas)] == want


def test_random_packs_match_oracle(gpu_ctx):
    """Three packs of ragged data/tree blobs, some with compressed entries,
    at unaligned input offsets and unaligned pack starts; nothing written
    outside the packs."""
    rng = np.random.default_rng(0xBAC)
    key = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
    lens = [0, 1, 15, 16, 17, 33, 1000, 4095, 65537, 70000, 3, 200000, 5, 64, 31]
    datas = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in lens]
    specs = []
    for i, d in enumerate(datas):
        tpe = int(rng.integers(0, 2))
        ulen = int(rng.integers(1, 1 << 20)) if i % 4 == 3 else 0
        specs.append((tpe, rng.integers(0, 256, 32, dtype=np.uint8),
                      rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), ulen))
    groups = [(0, 5), (5, 7), (12, 3)]
    hn = [rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in groups]
    pads = [int(x) for x in rng.integers(0, 16, len(lens))]
    files, packs, offsets, out, total = _build(key, datas, specs, groups, hn, pads, align=1)
    mask = np.ones(total + 64, bool)
    for (b0, n), f, p, h in zip(groups, files, packs, hn):
        blobs = [(specs[i][0], datas[i], specs[i][1].tobytes(), specs[i][2], specs[i][3])
                 for i in range(b0, b0 + n)]
        want, index = oracle.pack_file(key, blobs, h)
        assert f == want
        assert [int(offsets[i]) for i in range(b0, b0 + n)] == [o for o, _ in index]
        assert int(p["header_len"]) == int.from_bytes(want[-4:], "little")
        mask[int(p["out_off"]):int(p["out_off"]) + int(p["size"])] = False
        parsed = oracle.parse_pack(key, f)
        assert [(t, u, bytes(i)) for t, _, _, u, i in parsed] == \
            [(b[0], b[4], b[2]) for b in blobs]
    assert int(packs[0]["out_off"]) == 0 and int(packs[1]["out_off"]) % 16 != 0
    assert np.all(out[mask] == 0xA5)


def test_pack_build_rejects_bad_layouts(gpu_ctx):
    import torch
    from rustic_core_amd.errors import ErrorKind, RusticError
    from rustic_core_amd.pack import build_packs, make_blobs, pack_layout
    blobs = make_blobs([0], [10], [np.zeros(32, np.uint8)], [np.zeros(16, np.uint8)])
    d = torch.zeros(4096, dtype=torch.uint8, device="cuda:0")
    packs, total = pack_layout(blobs, [(0, 1)], [np.zeros(16, np.uint8)])
    with pytest.raises(RusticError) as e:  # output too small
        build_packs(gpu_ctx, bytes(64), d.data_ptr(), blobs, packs, d.data_ptr(), total - 1)
    assert e.value.kind == ErrorKind.InvalidInput
    packs["nblobs"] = 0
    with pytest.raises(RusticError):       # empty pack (the packer never saves one)
        build_packs(gpu_ctx, bytes(64), d.data_ptr(), blobs, packs, d.data_ptr(), 4096)
    packs["nblobs"] = 2
    with pytest.raises(RusticError):       # blob range past the array
        build_packs(gpu_ctx, bytes(64), d.data_ptr(), blobs, packs, d.data_ptr(), 4096)
    blobs["type"] = 2
    packs["nblobs"] = 1
    with pytest.raises(RusticError):       # BlobType is 0 or 1
        build_packs(gpu_ctx, bytes(64), d.data_ptr(), blobs, packs, d.data_ptr(), 4096)


def test_seal_open_unaligned_outputs(gpu_ctx):
    """rcdc_aead_seal / open with outputs at every alignment mod 16."""
    import torch
    from rustic_core_amd.crypto import Key, make_refs
    rng = np.random.default_rng(77)
    key = Key(rng.integers(0, 256, 64, dtype=np.uint8).tobytes())
    lens = [int(x) for x in rng.integers(0, 5000, 32)] + [65536 + 5, 16, 17]
    datas = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in lens]
    nonces = [rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in lens]
    ins, outs, o, p = [], [], 0, 0
    for i, d in enumerate(datas):
        ins.append(o)
        o += len(d) + (i % 7)
        p += i % 16 + 1
        outs.append(p)
        p += len(d) + 32
    arena = np.zeros(o + 64, np.uint8)
    for a, d in zip(ins, datas):
        arena[a:a + len(d)] = np.frombuffer(d, np.uint8)
    d_in = _dev(arena)
    d_out = torch.full((p + 64,), 0x5A, dtype=torch.uint8, device="cuda:0")
    key.seal_blobs(d_in.data_ptr(), make_refs(ins, lens, outs, b"".join(nonces)),
                   d_out.data_ptr())
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    mask = np.ones(p + 64, bool)
    for a, d, nc in zip(outs, datas, nonces):
        assert out[a:a + len(d) + 32].tobytes() == oracle.seal(key._key, nc, d)
        mask[a:a + len(d) + 32] = False
    assert np.all(out[mask] == 0x5A)
    # open them back to odd plaintext offsets
    back = torch.zeros(p + 64, dtype=torch.uint8, device="cuda:0")
    pos = [a + 3 for a in outs]
    st = key.open_blobs(d_out.data_ptr(), make_refs(outs, [n + 32 for n in lens], pos),
                        back.data_ptr())
    assert not st.any()
    b = back.cpu().numpy()
    for a, d in zip(pos, datas):
        assert b[a:a + len(d)].tobytes() == d
