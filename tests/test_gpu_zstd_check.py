"""Frames read back on the device (rcdc_zstd_check, rcdc_zstd_dec.hip): the
extra_verify check of the packer (crates/core/src/backend/decrypt.rs:508-529
``very_data``; on by default, configfile.rs:198).

Parity bar: the device verdict equals the standard decoder's.  A frame the
device accepts (status 0) must decode with libzstd (oracle/zstd_ref.py) to
exactly the blob; a frame libzstd decodes to the blob must be accepted.  The
frames come from this library's encoder and from libzstd itself at several
levels (treeless literals, repeat-mode tables, matches into earlier blocks,
FSE tables up to accuracy 9), plus corrupted copies of both.
"""
import numpy as np
import pytest

from oracle import zstd_ref as zr

pytestmark = pytest.mark.gpu

MiB = 1 << 20


def _words(rng, n):
    vocab = [bytes(rng.integers(97, 123, size=int(rng.integers(2, 9))).astype(np.uint8))
             for _ in range(400)]
    out = b" ".join(vocab[int(i)] for i in rng.integers(0, 400, size=n // 4 + 8))
    return out[:n]


def _data(rng, n, kind):
    if kind == "random":
        return rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    if kind == "zeros":
        return bytes(n)
    if kind == "text":
        return _words(rng, n)
    if kind == "csv":
        vocab = _words(rng, 4000).split(b" ")
        k = n // 24 + 2
        a, b = rng.integers(0, len(vocab), k), rng.integers(0, len(vocab), k)
        v = rng.integers(0, 10 ** 6, k)
        rows = b"".join(b"%08d,%s,%d,%s\n" % (i, vocab[a[i]], v[i], vocab[b[i]])
                        for i in range(k))
        return rows[:n]
    if kind == "binary":
        p = np.random.default_rng(98).dirichlet(np.ones(256) * 0.2)
        return bytes(rng.choice(256, n, p=p).astype(np.uint8))
    if kind == "periodic":
        pat = rng.integers(0, 256, int(rng.integers(1, 300)), dtype=np.uint8).tobytes()
        return (pat * (n // len(pat) + 1))[:n]
    if kind == "mixed":
        out = bytearray()
        while len(out) < n:
            k = int(rng.integers(1, 40000))
            c = int(rng.integers(0, 3))
            out += (rng.integers(0, 256, k, dtype=np.uint8).tobytes() if c == 0
                    else bytes(k) if c == 1 else _words(rng, k))
        return bytes(out[:n])
    raise ValueError(kind)


KINDS = ["random", "zeros", "text", "csv", "binary", "periodic", "mixed"]
LENS = [0, 1, 17, 255, 4096, 131071, 131072, 131073, 300001, MiB + 3]


def _layout(bufs, pad_seed=0):
    """bufs packed into one host array at ragged offsets."""
    rng = np.random.default_rng(pad_seed)
    offs, o = [], 0
    for b in bufs:
        o += int(rng.integers(0, 16))
        offs.append(o)
        o += len(b)
    arr = np.zeros(o + 64, np.uint8)
    for a, b in zip(offs, bufs):
        arr[a:a + len(b)] = np.frombuffer(b, np.uint8)
    return arr, offs


def _check(gpu_ctx, frames, datas, stored=False):
    import torch
    from rustic_core_amd.compress import check_frames
    farr, foffs = _layout(frames, 1)
    darr, doffs = _layout(datas, 2)
    d_f = torch.from_numpy(farr).to("cuda:0")
    d_d = torch.from_numpy(darr).to("cuda:0")
    st = check_frames(gpu_ctx, d_f.data_ptr(), foffs, [len(f) for f in frames], d_d.data_ptr(),
                      doffs, [len(d) for d in datas], stored=stored)
    torch.cuda.synchronize()
    return st


def _device_frames(gpu_ctx, datas, level=0):
    import torch
    from rustic_core_amd.compress import compress_blobs, frame_layout, make_refs
    arr, offs = _layout(datas, 3)
    f_offs, tot = frame_layout([len(d) for d in datas])
    d_in = torch.from_numpy(arr).to("cuda:0")
    d_out = torch.zeros(tot + 64, dtype=torch.uint8, device="cuda:0")
    ln = compress_blobs(gpu_ctx, d_in.data_ptr(), make_refs(offs, [len(d) for d in datas], f_offs),
                        d_out.data_ptr(), level)
    out = d_out.cpu().numpy()
    return [out[int(a):int(a) + int(n)].tobytes() for a, n in zip(f_offs, ln)]


def _libzstd_ok(frame, data):
    try:
        return zr.decompress(frame, len(data) + 64) == data and zr.frame_size(frame) == len(frame)
    except zr.ZstdError:
        return False


@pytest.mark.parametrize("kind", KINDS)
def test_device_frames_accepted(gpu_ctx, kind):
    rng = np.random.default_rng(sum(kind.encode()))
    datas = [_data(rng, n, kind) for n in LENS]
    frames = _device_frames(gpu_ctx, datas)
    st = _check(gpu_ctx, frames, datas)
    assert st.tolist() == [0] * len(datas)


@pytest.mark.parametrize("level", [-5, 1, 3, 9, 19])
def test_libzstd_frames_accepted(gpu_ctx, level):
    """Frames of the library rustic links (another version): every feature a
    standard encoder uses at these levels decodes and compares equal."""
    rng = np.random.default_rng(1000 + level)
    datas = [_data(rng, n, k) for k in KINDS for n in (1, 5000, 200001, 700000)]
    frames = [zr.compress(d, level) for d in datas]
    st = _check(gpu_ctx, frames, datas)
    assert st.tolist() == [0] * len(datas)


def test_mismatch_detected(gpu_ctx):
    rng = np.random.default_rng(7)
    datas = [_data(rng, n, k) for k, n in [("text", 300001), ("mixed", MiB), ("random", 70000),
                                          ("zeros", 200000), ("csv", 50000)]]
    frames = _device_frames(gpu_ctx, datas)
    changed = [bytearray(d) for d in datas]
    for d in changed:  # one byte each, somewhere in the middle
        d[len(d) // 2 + 1] ^= 0x40
    st = _check(gpu_ctx, frames, [bytes(d) for d in changed])
    assert st.tolist() == [1] * len(datas)
    # length off by one either way
    st = _check(gpu_ctx, frames + frames, [d[:-1] for d in datas] + [d + b"x" for d in datas])
    assert (st != 0).all()
    assert _check(gpu_ctx, frames, datas).tolist() == [0] * len(datas)


@pytest.mark.parametrize("source", ["device", "libzstd"])
def test_corrupted_frames_agree_with_libzstd(gpu_ctx, source):
    """Random single-byte corruptions: the device accepts exactly the frames
    libzstd decodes back to the blob."""
    rng = np.random.default_rng(11 if source == "device" else 12)
    base = [_data(rng, n, k) for k, n in [("text", 200000), ("csv", 150000), ("binary", 140000),
                                         ("mixed", 400000), ("periodic", 90000)]]
    good = _device_frames(gpu_ctx, base) if source == "device" else \
        [zr.compress(d, 3) for d in base]
    frames, datas = [], []
    for f, d in zip(good, base):
        for _ in range(40):
            g = bytearray(f)
            i = int(rng.integers(5, len(g)))
            g[i] ^= 1 << int(rng.integers(0, 8))
            frames.append(bytes(g))
            datas.append(d)
        frames.append(f[:len(f) - int(rng.integers(1, 8))])  # truncated
        datas.append(d)
    st = _check(gpu_ctx, frames, datas)
    exp = [_libzstd_ok(f, d) for f, d in zip(frames, datas)]
    assert [s == 0 for s in st.tolist()] == exp
    assert sum(exp) < len(exp) // 2  # the corruptions mostly break the frames


def test_odd_block_sizes(gpu_ctx):
    """Frames whose blocks are not 128 KiB (legal, no encoder here writes
    them): the block-parallel pass cannot place them and hands them to the
    in-order pass, which accepts the good ones and rejects the bad."""
    import sys
    sys.path.insert(0, __file__.rsplit("/", 1)[0])
    from zstd_model import frame
    rng = np.random.default_rng(31)
    d = rng.integers(0, 256, 1000 + 131072 + 500, dtype=np.uint8).tobytes()
    f1 = frame([(0, d[:1000], 1000), (0, d[1000:132072], 131072), (0, d[132072:], 500)], len(d))
    z = bytes(70000) + d[:5]
    f2 = frame([(1, bytes([0]), 70000), (0, d[:5], 5)], len(z))
    assert zr.decompress(f1) == d and zr.decompress(f2) == z
    bad = bytearray(d)
    bad[131500] ^= 1
    st = _check(gpu_ctx, [f1, f2, f1, f2], [d, z, bytes(bad), z[:-1] + b"?"])
    assert st.tolist() == [0, 0, 1, 1]


def test_stored_mode(gpu_ctx):
    rng = np.random.default_rng(5)
    datas = [_data(rng, n, "random") for n in (0, 3, 4096, 100003)]
    assert _check(gpu_ctx, datas, datas, stored=True).tolist() == [0, 0, 0, 0]
    other = [d[:-1] + bytes([d[-1] ^ 1]) if d else b"" for d in datas]
    assert _check(gpu_ctx, datas, other, stored=True).tolist()[1:] == [1, 1, 1]


def test_process_blobs_extra_verify(gpu_ctx):
    """process_data with extra_verify: compress + seal + open + decode +
    compare, as decrypt.rs:566-572 / 508-529; a corrupted sealed blob is a
    Verification error."""
    import torch
    from rustic_core_amd.compress import process_blobs, verify_sealed
    from rustic_core_amd.crypto import Key
    from rustic_core_amd.errors import ErrorKind, RusticError
    rng = np.random.default_rng(9)
    datas = [_data(rng, n, k) for k, n in [("text", 300000), ("random", 5000), ("zeros", 1 << 19),
                                          ("mixed", MiB)]]
    arr, offs = _layout(datas, 4)
    d_in = torch.from_numpy(arr).to("cuda:0")
    key = Key(bytes(range(64)))
    lens = [len(d) for d in datas]
    for level in (0, None):
        out, s_offs, s_lens, dlen, ulen = process_blobs(key, d_in.data_ptr(), offs, lens, level,
                                                        extra_verify=True)
        torch.cuda.synchronize()
        for i, d in enumerate(datas):
            sealed = out[int(s_offs[i]):int(s_offs[i]) + int(s_lens[i])].cpu().numpy().tobytes()
            plain = key.decrypt_data(sealed)
            assert (zr.decompress(plain) if level is not None else plain) == d
        bad = out.clone()
        bad[int(s_offs[3]) + 100] ^= 1  # inside blob 3's ciphertext
        with pytest.raises(RusticError) as e:
            verify_sealed(gpu_ctx, key, bad.data_ptr(), s_offs, s_lens, d_in.data_ptr(), offs, lens,
                          level is not None)
        assert e.value.kind == ErrorKind.Verification


def test_huffman_tree_without_full_length_codes_rejected(gpu_ctx):
    """tools/soak_zstd_check.py seed 5627: a libzstd level-2 frame whose
    FSE-coded Huffman weights had one bit changed (byte 16, 0x10 -> 0x12; the
    files are that case's frame, the untouched frame and the blob,
    tests/golden/zck_s5627.*).  The weights still decode to a table that
    decodes the blob, but it has no weight-1 symbol, and libzstd's
    HUF_readStats calls such a table corrupt (at least two weight-1
    symbols, an even number).  The device agrees: status 2; the untouched
    frame passes."""
    import os
    g = os.path.join(os.path.dirname(__file__), "golden", "zck_s5627.")
    bad, good, data = (open(g + x, "rb").read() for x in ("frame", "good", "data"))
    assert bad[16] == 0x12 and good[16] == 0x10 and bad[:16] == good[:16]
    for fr, ok in ((bad, False), (good, True)):
        try:
            dec = zr.decompress_stream(fr) == data
        except zr.ZstdError:
            dec = False
        assert dec == ok
    assert _check(gpu_ctx, [bad, good], [data, data]).tolist() == [2, 0]


def test_empty_compressed_block_as_decode_all(gpu_ctx):
    """tools/soak_zstd_check.py seeds 8485 and 8527: empty compressed blocks.
    decode_all's streaming decoder skips them, unless the frame declares a
    content size that fits its first 8 KiB output buffer: then it decodes in
    one pass, which calls them corrupt.  The device takes the same path."""
    import sys
    sys.path.insert(0, __file__.rsplit("/", 1)[0])
    from zstd_model import frame
    fr = bytes.fromhex("28b52ffd0002050000")
    assert zr.decompress_stream(fr) == b""
    d = bytes(range(256)) * 100
    f2 = frame([(2, b"", 0), (0, d, len(d))], len(d))  # an empty compressed block, then raw
    assert zr.decompress_stream(f2) == d
    bad = frame([(2, b"", 0), (0, d, len(d))], len(d) + 1)  # content size off by one
    assert _check(gpu_ctx, [fr, f2, bad], [b"", d, d + b"x"]).tolist() == [0, 0, 1]
    # seed 8527: the same block in a frame declaring content size 0 takes
    # decode_all's one-pass path (its first 8 KiB output buffer holds the
    # content), which calls the block corrupt
    one = bytes.fromhex("28b52ffd2000050000")
    with pytest.raises(zr.ZstdError):
        zr.decompress_stream(one)
    small = frame([(2, b"", 0), (0, d[:5000], 5000)], 5000)
    with pytest.raises(zr.ZstdError):
        zr.decompress_stream(small)
    assert _check(gpu_ctx, [one, small], [b"", d[:5000]]).tolist() == [2, 2]
