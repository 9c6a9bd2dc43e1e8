"""The device ingest path (rustic_core_amd/ingest.py): chunk -> blob ids ->
dedup -> zstd -> seal -> verify -> packs, for streams in HBM.

Reference: archiver/file_archiver.rs:138-168 (chunk + id per chunk),
blob/packer.rs:304-315 (dedup by id against the index and the packer),
backend/decrypt.rs:566-572 + 508-529 (process_data + very_data),
blob/packer.rs:615-735 (add_raw, the sealed header), index/indexer.rs.

Checked against the oracle: every cut (oracle/cdc_ref), every id (hashlib
over the oracle's chunks), the dedup decision (first occurrence in chunk
order, minus what the index holds), and every pack file parsed and opened
by oracle.parse_pack / oracle.open_ with each blob decoded by libzstd back
to its chunk.
"""
import hashlib

import numpy as np
import pytest

from oracle import oracle, zstd_ref as zr

pytestmark = pytest.mark.gpu

MiB = 1 << 20


def _streams(seed=1, n=8):
    """Mixed streams (random runs, zero runs, text runs); stream 5 repeats
    stream 1 and stream 7 starts with stream 2's first 6 MiB, so whole
    chunks repeat across streams."""
    rng = np.random.default_rng(seed)
    words = [bytes(rng.integers(97, 123, int(rng.integers(2, 9))).astype(np.uint8))
             for _ in range(300)]
    text = b" ".join(words[int(j)] for j in rng.integers(0, 300, (8 * MiB) // 5))
    datas = []
    for i in range(n):
        size = int(rng.integers(6 * MiB, 40 * MiB))
        out = bytearray()
        while len(out) < size:
            k = int(rng.integers(64 << 10, 6 * MiB))
            c = int(rng.integers(0, 3))
            if c == 0:
                out += rng.integers(0, 256, k, dtype=np.uint8).tobytes()
            elif c == 1:
                out += bytes(k)
            else:
                a = int(rng.integers(0, len(text) - k))
                out += text[a:a + k]
        datas.append(bytes(out[:size]))
    datas[5] = datas[1]
    datas[7] = datas[2][:6 * MiB] + datas[7][6 * MiB:]
    return datas


def _arena(datas):
    import torch
    from rustic_core_amd.device import pack_offsets
    lens = [len(d) for d in datas]
    offs, total = pack_offsets(lens)
    host = np.zeros(total, np.uint8)
    for o, d in zip(offs, datas):
        host[int(o):int(o) + len(d)] = np.frombuffer(d, np.uint8)
    return host, torch.from_numpy(host).to("cuda:0"), offs, lens


def _ingest(version, indexed=None, extra_verify=None, key=bytes(range(64)), seed=1):
    from rustic_core_amd.chunker import ConfigFile
    from rustic_core_amd.crypto import Key
    from rustic_core_amd.ingest import DeviceIngest
    cfg = ConfigFile.new(version, oracle.DEFAULT_POLY)
    datas = _streams(seed)
    host, arena, offs, lens = _arena(datas)
    ing = DeviceIngest(cfg, Key(key), indexed=indexed, extra_verify=extra_verify)
    res = ing.ingest(arena, offs, lens, finalize=True)
    return ing, res, host, offs, lens, datas


def _check_result(res, host, offs, lens, key, compressed, known=frozenset()):
    from rustic_core_amd.chunker import ConfigFile
    from rustic_core_amd.pack import PackSizer, group_blobs
    # cuts and ids against the oracle
    chunks = []
    for i, (o, n) in enumerate(zip(offs, lens)):
        exp = oracle.chunk_cuts(host[int(o):int(o) + n])
        assert np.array_equal(res.cuts[i], exp), i
        prev = 0
        for c in exp:
            chunks.append(host[int(o) + prev:int(o) + int(c)].tobytes())
            prev = int(c)
    assert len(chunks) == len(res.ids)
    ids = [hashlib.sha256(c).digest() for c in chunks]
    assert [bytes(x) for x in res.ids] == ids
    # dedup: first occurrence in chunk order, not in the index
    seen, exp_new = set(known), []
    for bid in ids:
        exp_new.append(bid not in seen)
        seen.add(bid)
    assert res.new.tolist() == exp_new
    new_chunks = [c for c, f in zip(chunks, exp_new) if f]
    # pack grouping as the packer's PackSizer would
    ulens = [len(c) for c in new_chunks] if compressed else [0] * len(new_chunks)
    grp = group_blobs([int(x) - 32 for x in res.blobs["len"]],
                      PackSizer.from_config(ConfigFile.new(2, oracle.DEFAULT_POLY), 0, 0), ulens)
    assert [(int(p["blob0"]), int(p["nblobs"])) for p in res.pack_table] == grp
    # every pack parsed, every blob opened and decoded back to its chunk
    k = 0
    for j in range(len(res.pack_table)):
        f = res.pack_file(j)
        assert len(f) == int(res.pack_table[j]["size"])
        parsed = oracle.parse_pack(key, f)
        assert len(parsed) == int(res.pack_table[j]["nblobs"])
        for tpe, off, ln, ulen, bid in parsed:
            assert tpe == 0 and off == int(res.blob_offsets[k])
            plain = oracle.open_(key, f[off:off + ln])
            data = zr.decompress(plain) if compressed else plain
            assert data == new_chunks[k], k
            assert bytes(bid) == hashlib.sha256(data).digest()
            assert ulen == (len(data) if compressed else 0)
            k += 1
    assert k == len(new_chunks)
    return chunks, ids, new_chunks


def test_ingest_v2_matches_oracle():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    key = bytes(range(64))
    ing, res, host, offs, lens, _ = _ingest(2, key=key)
    chunks, ids, new_chunks = _check_result(res, host, offs, lens, key, compressed=True)
    assert len(new_chunks) < len(chunks)  # the repeated streams dedup
    assert (np.asarray(res.chunk_lens) > ing.long_chunk).any()  # both id launches ran
    # index packs (Indexer::add input) carry the blobs' locations
    ips = res.index_packs()
    assert sum(len(p.blobs) for p in ips) == len(new_chunks)
    for p, row in zip(ips, res.pack_table):
        assert p.pack_size() == int(row["size"])
    # a second backup of the same bytes: everything is in the index
    _, res2, _, _, _, _ = _ingest(2, indexed=set(ids), key=key)
    assert not res2.new.any() and len(res2.pack_table) == 0
    ing.close()


def test_ingest_partly_indexed_and_v1():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    key = bytes(range(1, 65))
    # ids of a different seed's first stream are "in the index" too: none match;
    # half of this batch's own ids are known
    _, res, host, offs, lens, _ = _ingest(2, key=key, seed=3)
    ids = [bytes(x) for x in res.ids]
    known = set(ids[::2])
    _, res2, host2, offs2, lens2, _ = _ingest(2, indexed=set(known), key=key, seed=3)
    _check_result(res2, host2, offs2, lens2, key, compressed=True, known=known)
    # version 1: stored blobs, verified as stored bytes; verify off too
    for ev in (None, False):
        _, res3, host3, offs3, lens3, _ = _ingest(1, extra_verify=ev, key=key, seed=4)
        _check_result(res3, host3, offs3, lens3, key, compressed=False)


def test_pack_build_raw_matches_sealed_build(gpu_ctx):
    """rcdc_pack_build_raw (add_raw: blobs sealed elsewhere) gives the same
    pack bytes as rcdc_pack_build sealing them in place."""
    import torch
    from rustic_core_amd.crypto import Key, make_refs, sealed_layout
    from rustic_core_amd.pack import build_packs, make_blobs, pack_layout
    rng = np.random.default_rng(21)
    key = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
    lens = [0, 1, 15, 17, 1000, 65537, 3, 1 << 20, 2 * MiB + 5, 31]
    datas = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in lens]
    offs, o = [], 0
    for d in datas:
        o += int(rng.integers(0, 16))
        offs.append(o)
        o += len(d)
    host = np.zeros(o + 64, np.uint8)
    for a, d in zip(offs, datas):
        host[a:a + len(d)] = np.frombuffer(d, np.uint8)
    d_in = torch.from_numpy(host).to("cuda:0")
    nonces = rng.integers(0, 256, (len(lens), 16), dtype=np.uint8)
    ids = rng.integers(0, 256, (len(lens), 32), dtype=np.uint8)
    ulen = [n + 7 if i % 3 == 0 else 0 for i, n in enumerate(lens)]
    groups, hn = [(0, 4), (4, 5), (9, 1)], rng.integers(0, 256, (3, 16), dtype=np.uint8)
    # in place
    blobs = make_blobs(offs, lens, ids, nonces, uncompressed=ulen)
    packs, total = pack_layout(blobs, groups, hn, align=3)
    out1 = torch.zeros(total + 64, dtype=torch.uint8, device="cuda:0")
    off1 = build_packs(gpu_ctx, key, d_in.data_ptr(), blobs, packs, out1.data_ptr(), total)
    # sealed first (at odd staging offsets), then add_raw
    s_offs, s_tot = sealed_layout(lens)
    s_offs = s_offs + np.arange(len(lens), dtype=np.uint64) * 3
    staging = torch.zeros(s_tot + 64 + 3 * len(lens), dtype=torch.uint8, device="cuda:0")
    Key(key).seal_blobs(d_in.data_ptr(), make_refs(offs, lens, s_offs, nonces),
                        staging.data_ptr(), None, gpu_ctx)
    rblobs = make_blobs(s_offs, [n + 32 for n in lens], ids, np.zeros_like(nonces),
                        uncompressed=ulen)
    rpacks, rtotal = pack_layout(rblobs, groups, hn, align=3, raw=True)
    assert rtotal == total
    out2 = torch.full((total + 64,), 7, dtype=torch.uint8, device="cuda:0")
    off2 = build_packs(gpu_ctx, key, staging.data_ptr(), rblobs, rpacks, out2.data_ptr(), total,
                       raw=True)
    torch.cuda.synchronize()
    assert np.array_equal(off1, off2)
    assert np.array_equal(packs["size"], rpacks["size"])
    a, b = out1.cpu().numpy(), out2.cpu().numpy()
    for p in packs:
        s, n = int(p["out_off"]), int(p["size"])
        assert np.array_equal(a[s:s + n], b[s:s + n])


def _packs_blobs(res, key, compressed):
    """(header entries, decoded blob bytes) of every pack of `res`, parsed and
    opened by the oracle."""
    out = []
    k = 0
    for j in range(len(res.pack_table)):
        f = res.pack_file(j)
        assert len(f) == int(res.pack_table[j]["size"])
        for tpe, off, ln, ulen, bid in oracle.parse_pack(key, f):
            assert tpe == 0 and off == int(res.blob_offsets[k])
            plain = oracle.open_(key, f[off:off + ln])
            out.append((bytes(bid), zr.decompress(plain) if compressed else plain))
            k += 1
    return out


def test_ingest_calls_keep_the_pack_open():
    """One packer across calls (packer.rs:659-671, 749-750): three
    ingest calls and finalize() close exactly the packs one pass over all new
    blobs closes -- no undersized pack per call -- with the open pack's sealed
    blobs carried on the device between calls (rcdc_copy_ranges) and built
    from several buffers (rcdc_pack_build_raw_multi).  Chunks repeated across
    calls are packed once."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rustic_core_amd.chunker import ConfigFile
    from rustic_core_amd.crypto import Key
    from rustic_core_amd.ingest import DeviceIngest
    from rustic_core_amd.pack import PackSizer, group_blobs
    key = bytes(range(3, 67))
    cfg = ConfigFile.new(2, oracle.DEFAULT_POLY)
    datas = _streams(seed=9, n=8)
    ing = DeviceIngest(cfg, Key(key))
    ing.sizer = PackSizer.fixed(24 * MiB)  # several packs per call, one left open
    results, all_chunks = [], []
    for part in (datas[0:3], datas[3:6], datas[6:8]):
        host, arena, offs, lens = _arena(part)
        res = ing.ingest(arena, offs, lens)
        results.append(res)
        for i, (o, n) in enumerate(zip(offs, lens)):
            exp = oracle.chunk_cuts(host[int(o):int(o) + n])
            assert np.array_equal(res.cuts[i], exp)
            prev = 0
            for c in exp:
                all_chunks.append(host[int(o) + prev:int(o) + int(c)].tobytes())
                prev = int(c)
        assert ing.open_blobs > 0
    results.append(ing.finalize())
    assert ing.open_blobs == 0
    seen, new_chunks = set(), []
    for c in all_chunks:
        h = hashlib.sha256(c).digest()
        if h not in seen:
            seen.add(h)
            new_chunks.append(c)
    got = []
    sizes = []
    for r in results:
        got += _packs_blobs(r, key, compressed=True)
        sizes += [int(p["nblobs"]) for p in r.pack_table]
    assert [d for _, d in got] == new_chunks
    assert [b for b, _ in got] == [hashlib.sha256(c).digest() for c in new_chunks]
    # the same grouping as one packer over every new blob (sealed sizes from
    # the packs themselves)
    sealed = np.concatenate([r.blobs["len"].astype(np.int64) for r in results])
    ulens = np.concatenate([r.blobs["uncompressed_len"].astype(np.int64) for r in results])
    one = group_blobs([int(x) - 32 for x in sealed], PackSizer.fixed(24 * MiB),
                      [int(x) for x in ulens])
    assert sizes == [n for _, n in one]
    assert sum(len(r.pack_table) for r in results[:-1]) >= 1  # closed inside a call


def test_ingest_rejects_a_corrupted_blob(monkeypatch):
    """extra_verify in the ingest path: a byte flipped in a sealed
    blob between seal and verify -- in the long and in the short staging --
    raises ErrorKind.Verification (backend/decrypt.rs:508-529, C003)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rustic_core_amd.chunker import ConfigFile
    from rustic_core_amd.crypto import Key
    from rustic_core_amd.errors import ErrorKind, RusticError
    from rustic_core_amd.ingest import DeviceIngest
    datas = _streams(seed=11, n=8)
    host, arena, offs, lens = _arena(datas)
    for which in (0, 1):  # 0: the first _process call (long chunks), 1: the second (short)
        ing = DeviceIngest(ConfigFile.new(2, oracle.DEFAULT_POLY), Key(bytes(range(64))))
        orig = ing._process
        calls = [0]

        def bad(torch_, arena_ptr, sel, c_offs, c_lens, frames, staging, s_off0, stream,
                _orig=orig, _calls=calls, _which=which):
            r = _orig(torch_, arena_ptr, sel, c_offs, c_lens, frames, staging, s_off0, stream)
            if _calls[0] == _which:
                so = int(r[0][len(r[0]) // 2])
                with torch.cuda.stream(torch.cuda.ExternalStream(stream)):
                    staging[so + 40] ^= 0x5A  # inside the ciphertext
            _calls[0] += 1
            return r
        monkeypatch.setattr(ing, "_process", bad)
        with pytest.raises(RusticError) as ei:
            ing.ingest(arena, offs, lens, finalize=True)
        assert ei.value.kind == ErrorKind.Verification
        assert calls[0] > which


def test_pack_build_raw_multi_matches_single_source(gpu_ctx):
    """rcdc_pack_build_raw_multi over blobs split across two buffers (odd
    offsets) gives the bytes rcdc_pack_build_raw gives from one buffer."""
    import torch
    from rustic_core_amd.pack import (build_packs, build_packs_multi, copy_ranges, make_blobs,
                                      pack_layout)
    rng = np.random.default_rng(5)
    key = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
    lens = [int(x) for x in rng.integers(32, 300_000, 12)] + [32, 33, (1 << 20) + 77]
    n = len(lens)
    offs = np.cumsum([0] + [x + 5 for x in lens[:-1]]).astype(np.uint64)
    total_in = int(offs[-1]) + lens[-1] + 64
    one = torch.from_numpy(rng.integers(0, 256, total_in, dtype=np.uint8)).to("cuda:0")
    # the same bytes spread over two buffers: odd blobs in the second, shifted by 3
    two = torch.zeros(total_in + 64, dtype=torch.uint8, device="cuda:0")
    src = np.arange(n) % 2
    offs2 = np.where(src == 1, offs + 3, offs).astype(np.uint64)
    copy_ranges(gpu_ctx, [one.data_ptr()], np.zeros(int((src == 1).sum()), np.uint32), offs[src == 1],
                np.asarray(lens, np.uint64)[src == 1], offs2[src == 1], two.data_ptr())
    ids = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    ulen = [x * 2 if i % 4 == 0 else 0 for i, x in enumerate(lens)]
    groups, hn = [(0, 5), (5, 9), (14, 1)], rng.integers(0, 256, (3, 16), dtype=np.uint8)
    b1 = make_blobs(offs, lens, ids, np.zeros((n, 16), np.uint8), uncompressed=ulen)
    p1, total = pack_layout(b1, groups, hn, align=7, raw=True)
    out1 = torch.zeros(total + 64, dtype=torch.uint8, device="cuda:0")
    o1 = build_packs(gpu_ctx, key, one.data_ptr(), b1, p1, out1.data_ptr(), total, raw=True)
    b2 = make_blobs(offs2, lens, ids, np.zeros((n, 16), np.uint8), uncompressed=ulen)
    b2["pad"] = src
    p2, _ = pack_layout(b2, groups, hn, align=7, raw=True)
    out2 = torch.full((total + 64,), 9, dtype=torch.uint8, device="cuda:0")
    o2 = build_packs_multi(gpu_ctx, key, [one.data_ptr(), two.data_ptr()], b2, p2,
                           out2.data_ptr(), total)
    torch.cuda.synchronize()
    assert np.array_equal(o1, o2) and np.array_equal(p1["size"], p2["size"])
    a, b = out1.cpu().numpy(), out2.cpu().numpy()
    for p in p1:
        s, m = int(p["out_off"]), int(p["size"])
        assert np.array_equal(a[s:s + m], b[s:s + m])
    b2["pad"][3] = 2  # no third buffer
    from rustic_core_amd.errors import RusticError
    with pytest.raises(RusticError):
        build_packs_multi(gpu_ctx, key, [one.data_ptr(), two.data_ptr()], b2, p2,
                          out2.data_ptr(), total)


def test_host_ingest_files_to_packs_and_pack_ids():
    """HostIngest: files in host memory -> pack files and
    pack ids in host memory, in several pipelined batches (begin(k + 1)
    before end(k), three arena slots, D2H + host hashing).  Every cut against
    the oracle, every pack id against hashlib, every pack parsed and every
    blob opened by the oracle and decoded by libzstd back to the new chunks
    in order, and the pack grouping of one packer over all batches."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rustic_core_amd.chunker import ConfigFile
    from rustic_core_amd.crypto import Key
    from rustic_core_amd.ingest import HostIngest
    from rustic_core_amd.pack import PackSizer, group_blobs
    key = bytes(range(5, 69))
    datas = _streams(seed=13, n=8)
    files = [torch.from_numpy(np.frombuffer(d, np.uint8).copy()).pin_memory() for d in datas]
    hi = HostIngest(ConfigFile.new(2, oracle.DEFAULT_POLY), Key(key), hash_threads=4,
                    first_batch=40 * MiB, batch=70 * MiB, last_batch=30 * MiB)
    hi.ingest.sizer = PackSizer.fixed(16 * MiB)
    res = hi.run(files)
    assert len(res.batch_files) >= 3
    assert res.h2d_bytes == sum(len(d) for d in datas)
    chunks = []
    for r, b in zip(res.batches, res.batch_files):
        for i, got in zip(b, r.cuts):
            exp = oracle.chunk_cuts(np.frombuffer(datas[i], np.uint8))
            assert np.array_equal(got, exp)
            prev = 0
            for c in exp:
                chunks.append(datas[i][prev:int(c)])
                prev = int(c)
    seen, new_chunks = set(), []
    for c in chunks:
        h = hashlib.sha256(c).digest()
        if h not in seen:
            seen.add(h)
            new_chunks.append(c)
    got, sealed, ulens = [], [], []
    for k in range(len(res.pack_ids)):
        f = res.pack_file(k)
        assert hashlib.sha256(f).digest() == res.pack_ids[k]
        for tpe, off, ln, ulen, bid in oracle.parse_pack(key, f):
            data = zr.decompress(oracle.open_(key, f[off:off + ln]))
            assert hashlib.sha256(data).digest() == bytes(bid) and ulen == len(data)
            got.append(data)
            sealed.append(ln)
            ulens.append(ulen)
    assert got == new_chunks
    assert res.d2h_bytes == int(sum(res.pack_sizes))
    one = group_blobs([x - 32 for x in sealed], PackSizer.fixed(16 * MiB), ulens)
    sizes = [int(p["nblobs"]) for r in res.batches for p in r.pack_table]
    assert sizes == [n for _, n in one]
    hi.close()
