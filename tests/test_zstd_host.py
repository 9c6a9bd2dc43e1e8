"""CPU: the zstd checker and the device encoder's coding tables -- SURVEY.md
8(f) row 3 (blob compression, backend/decrypt.rs:478-506).

- The checker (oracle/zstd_ref.py: the system libzstd through ctypes, and
  pyarrow's bundled zstd) round-trips libzstd's own frames and agrees with
  itself across both builds.
- tests/zstd_model.py codes sequences with the library's FSE tables
  (rcdc_zstd_tables) exactly as the kernel's lane 0 does; both decoders must
  read every block back: every literal-length, match-length and offset code,
  the 1/2/3-byte section headers (including >= 0x7F00 sequences) and the
  frame-header size classes.  Compressed bytes themselves are parity-unpinned
  (library-version specific); decoding is the contract.
"""
import numpy as np
import pytest

from oracle import zstd_ref as zr
from tests import zstd_model as zm


@pytest.fixture(scope="module")
def T(rcdc_lib):
    return zm.tables()


def _synth(seqs, tail, rng):
    """Bytes whose parse is exactly ``seqs`` (+ ``tail`` literals)."""
    out = bytearray()
    for ll, ml, off in seqs:
        out += rng.integers(0, 256, ll, dtype=np.uint8).tobytes()
        assert off <= len(out)
        for _ in range(ml):  # overlapping copy, as the decoder does
            out.append(out[-off])
    out += rng.integers(0, 256, tail, dtype=np.uint8).tobytes()
    return bytes(out)


def _roundtrip(T, data, seqs):
    blk = zm.compressed_block(T, data, seqs)
    fr = zm.frame([(2, blk, len(data))], len(data))
    assert zr.decompress(fr) == data
    if len(blk) <= len(data):
        # zstd >= 1.5 rejects a compressed block larger than the frame's
        # window (its content size); the device never writes one
        assert zr.decompress_pyarrow(fr, len(data)) == data
    assert zr.content_size(fr) == len(data)
    assert zr.blocks(fr) == [(2, len(blk), True)]
    return fr


def test_checker_roundtrip():
    rng = np.random.default_rng(7)
    for n in (0, 1, 100, 70000, 300000):
        d = rng.integers(0, 4, n, dtype=np.uint8).tobytes()
        fr = zr.compress(d, 3)
        assert zr.decompress(fr) == d
        assert zr.decompress_pyarrow(fr, n) == d
        assert zr.frame_size(fr) == len(fr)
    assert zr.version().startswith("1.")


def test_tables_shape(T):
    # state tables are permutations of [size, 2 size)
    assert sorted(T["llst"]) == list(range(64, 128))
    assert sorted(T["mlst"]) == list(range(64, 128))
    assert sorted(T["ofst"][:32]) == list(range(32, 64))
    assert T["llcode"][15] == 15 and T["llcode"][16] == 16 and T["llcode"][63] == 24
    assert T["mlcode"][31] == 31 and T["mlcode"][32] == 32 and T["mlcode"][127] == 42


@pytest.mark.parametrize("seed", range(4))
def test_model_every_code(T, seed):
    rng = np.random.default_rng(seed)
    # literal lengths over every LL code, match lengths over every ML code,
    # offsets over every OF code a 128 KiB block can reach
    lls = [0, 1, 15, 16, 17, 63, 64, 65, 127, 128, 255, 256, 1000, 5000]
    mls = [3, 4, 34, 35, 36, 130, 131, 258, 259, 1000, 4098, 4099, 9000]
    seqs, size = [], 0
    for i in range(40):
        ll = int(rng.choice(lls))
        ml = int(rng.choice(mls))
        cap = size + ll
        if cap < 1:
            ll, cap = 1, size + 1
        off = int(min(cap, rng.choice([1, 2, 3, 4, 7, 100, 1 << 10, 1 << 14, 1 << 16, cap])))
        seqs.append((ll, ml, off))
        size += ll + ml
        if size > 100000:
            break
    data = _synth(seqs, int(rng.integers(0, 40)), rng)
    _roundtrip(T, data, seqs)


def test_model_long_lengths(T):
    rng = np.random.default_rng(11)
    # LL code 35 (>= 65536 literals), ML code 52 (>= 65539), the max offset
    seqs = [(70000, 3, 70000), (5, 60000, 1)]
    _roundtrip(T, _synth(seqs, 3, rng), seqs)
    seqs = [(4, 3, 4), (1, 65539 + 1000, 1)]
    _roundtrip(T, _synth(seqs, 0, rng), seqs)


@pytest.mark.parametrize("nseq", [1, 127, 128, 0x7EFF, 0x7F00, 0x7F00 + 300])
def test_model_sequence_counts(T, nseq):
    rng = np.random.default_rng(nseq)
    seqs = [(0 if i else 4, 3, 4 if i == 0 else int(rng.integers(1, 4 + 3 * i)))
            for i in range(nseq)]
    seqs = [(ll, ml, min(off, 4 + 3 * i)) for i, (ll, ml, off) in enumerate(seqs)]
    data = _synth(seqs, 5, rng)
    assert len(data) <= 131072
    _roundtrip(T, data, seqs)


def test_model_literal_header_classes(T):
    rng = np.random.default_rng(3)
    for lits in (5, 31, 32, 4095, 4096, 70000):
        seqs = [(lits, 40, min(lits, 8))]
        _roundtrip(T, _synth(seqs, 0, rng), seqs)


def test_frame_header_classes():
    # single-segment content-size classes: 1 byte < 256, 2 bytes (size - 256)
    # < 65792, 4 bytes otherwise (the device frame kernel's choice)
    for n in (0, 1, 255, 256, 257, 65791, 65792, 200000):
        data = bytes(range(256)) * (n // 256 + 1)
        data = data[:n]
        blocks_, pos = [], 0
        while True:
            k = min(131072, n - pos)
            blocks_.append((0, data[pos:pos + k], k))
            pos += k
            if pos >= n:
                break
        fr = zm.frame(blocks_, n)
        assert zr.content_size(fr) == n
        assert zr.decompress(fr) == data


def test_greedy_model_text(T):
    rng = np.random.default_rng(5)
    words = [bytes(rng.integers(97, 123, size=int(rng.integers(2, 9))).astype(np.uint8))
             for _ in range(300)]
    data = b" ".join(words[int(i)] for i in rng.integers(0, 300, size=20000))[:100000]
    seqs = zm.greedy_sequences(data)
    fr = _roundtrip(T, data, seqs)
    assert len(fr) < len(data) // 2


def test_abi_rejects(rcdc_lib):
    # NULL context / arguments: InvalidInput (2) before any HIP call
    assert rcdc_lib.rcdc_zstd_compress(None, 0, None, None, 0, None, None, None) == 2
    assert rcdc_lib.rcdc_zstd_bound(0) == 12
    assert rcdc_lib.rcdc_zstd_bound(131072) == 131072 + 3 + 9
    assert rcdc_lib.rcdc_zstd_bound(131073) == 131073 + 6 + 9


@pytest.mark.parametrize("kind", ["two", "ascii-text", "skewed", "flat-129", "clamped"])
def test_model_huffman_literals(T, kind):
    """Compressed_Literals_Block (4 streams, direct weights) as the device
    builds it (tests/zstd_model.py restates rcdc_zstd.hip encode_literals):
    every decoder reads it back, and the code is complete (Kraft sum 1)."""
    rng = np.random.default_rng(len(kind))
    if kind == "two":
        lits = bytes(rng.choice([97, 98], 5000, p=[0.9, 0.1]).astype(np.uint8))
    elif kind == "ascii-text":
        words = [bytes(rng.integers(97, 123, int(rng.integers(2, 9))).astype(np.uint8))
                 for _ in range(3000)]
        lits = b" ".join(words)[:100000]
    elif kind == "skewed":
        lits = bytes(rng.choice(129, 60000, p=rng.dirichlet(np.ones(129) * 0.05)).astype(np.uint8))
    elif kind == "flat-129":
        lits = bytes(rng.integers(0, 129, 70000).astype(np.uint8))
    else:  # many symbols rarer than 2^-11: the Kraft repair path
        p = np.r_[[0.9], np.full(128, 0.1 / 128)]
        lits = bytes(rng.choice(129, 131000, p=p).astype(np.uint8))
    counts = np.bincount(np.frombuffer(lits, np.uint8), minlength=256)
    L = zm.huf_lengths(counts)
    assert L is not None and max(L) <= 11
    assert sum(2.0 ** -l for l in L if l) == 1.0
    sec = zm.huf_literals_section(lits)
    assert sec is not None and len(sec) < len(lits)
    blk = sec + b"\x00"  # no sequences
    fr = zm.frame([(2, blk, len(lits))], len(lits))
    assert zr.decompress(fr) == lits
    assert zr.decompress_pyarrow(fr, len(lits)) == lits
    if kind in ("skewed", "two"):  # Huffman at least as small as libzstd here
        assert len(fr) <= 1.05 * len(zr.compress(lits, 3)) + 64


@pytest.mark.parametrize("case", ["text", "one-ml-code", "short-block", "long-offsets"])
def test_model_adaptive_sequences(T, case):
    """Sequences section with adaptive log-6 FSE tables where they beat the
    predefined ones (FSE_Compressed mode: FSE_writeNCount descriptions),
    as rcdc_zstd.hip codes it: both decoders read it back."""
    rng = np.random.default_rng(len(case))
    if case == "text":
        words = [bytes(rng.integers(97, 123, int(rng.integers(2, 9))).astype(np.uint8))
                 for _ in range(300)]
        data = b" ".join(words[int(i)] for i in rng.integers(0, 300, 30000))[:131072]
        seqs = zm.greedy_sequences(data)
    else:
        if case == "one-ml-code":
            seqs = [(int(rng.integers(0, 20)), 4, int(rng.integers(1, 200))) for _ in range(3000)]
        elif case == "short-block":
            seqs = [(3, 5, 2), (0, 6, 7), (1, 4, 3)]
        else:
            seqs = [(int(rng.integers(0, 40)), int(rng.integers(3, 300)), 0) for _ in range(300)]
        fixed, size = [], 0
        for ll, ml, off in seqs:
            size += ll
            off = off or int(rng.integers(1, max(2, size)))
            off = max(1, min(off, size))
            fixed.append((max(ll, 1) if size == ll else ll, ml, off))
            size += ml
        seqs = fixed
        if seqs[0][0] == 0:
            seqs[0] = (1,) + seqs[0][1:]
        data = _synth(seqs, 5, rng)
    blk = zm.compressed_block_adaptive(T, data, seqs)
    fr = zm.frame([(2, blk, len(data))], len(data))
    assert zr.decompress(fr) == data
    if len(blk) <= len(data):
        assert zr.decompress_pyarrow(fr, len(data)) == data
    if case == "text":
        assert len(fr) < 1.15 * len(zr.compress(data, 3))


@pytest.mark.parametrize("nsym,n,alpha", [(200, 5000, 0.05), (256, 50000, 0.3), (140, 131000, 1.0),
                                          (255, 777, 3.0), (256, 3333, 0.05)])
def test_model_huffman_fse_weights(T, nsym, n, alpha):
    """Literal bytes above 128: the Huffman weights go FSE-compressed (log 6,
    two interleaved states, FSE_compress_usingCTable order), as the device
    writes them (rcdc_zstd.hip fse_weights); both decoders read them."""
    rng = np.random.default_rng(nsym + n)
    lits = bytes(rng.choice(nsym, n, p=rng.dirichlet(np.ones(nsym) * alpha)).astype(np.uint8))
    sec = zm.huf_literals_section(lits)
    if sec is None:  # weights >= 128 bytes or no gain: raw literals
        return
    assert sec[{True: 3, False: 4}[n < 1024] if n < 16384 else 5] < 128  # FSE weights header byte
    fr = zm.frame([(2, sec + b"\x00", n)], n)
    assert zr.decompress(fr) == lits
    if len(sec) + 1 <= n:
        assert zr.decompress_pyarrow(fr, n) == lits


def test_model_repeat_offsets(T):
    """Repeat offset codes with a block-local history (RFC 8878 3.1.2.5:
    offset values 1-3, the LL = 0 shift, history updates): both decoders
    read them back.  (The device codes offsets literally; this pins the
    rules for a repeat-aware parse.)"""
    rng = np.random.default_rng(12)
    words = [bytes(rng.integers(97, 123, int(rng.integers(2, 9))).astype(np.uint8))
             for _ in range(400)]
    rows = b"".join(b"%08d,%s,%d,%s\n" % (i, words[i % 400], (i * 7919) % 100000,
                                          words[(i * 31) % 400]) for i in range(6000))[:131072]
    seqs = zm.greedy_sequences_rep(rows)
    vals = zm.offsets_to_values(seqs)
    assert any(v <= 3 for _, _, v in vals)
    # the LL = 0 rules too: force back-to-back matches at repeat offsets
    seqs2 = [(5, 4, 3), (0, 4, 3 + 0), (2, 5, 7), (0, 6, 3), (0, 4, 6), (1, 4, 3)]
    fixed = []
    size = 0
    for ll, ml, off in seqs2:
        size += ll
        fixed.append((ll, ml, min(off, size)))
        size += ml
    for d, s in [(rows, seqs), (_synth(fixed, 3, rng), fixed)]:
        blk = zm.compressed_block_adaptive(T, d, s, reps=True)
        fr = zm.frame([(2, blk, len(d))], len(d))
        assert zr.decompress(fr) == d
        if len(blk) <= len(d):
            assert zr.decompress_pyarrow(fr, len(d)) == d


def test_window_limit_of_decode_all():
    """rustic's decode_all (the zstd crate's streaming decoder) refuses
    frames asking for a window above 2^27 + 1 bytes; single-segment frames ask
    for their content size, so blobs above 128 MiB get a window descriptor
    (rcdc_zstd_frame_kernel) and one more header byte in the bound."""
    import sys
    sys.path.insert(0, __file__.rsplit("/", 1)[0])
    from zstd_model import frame
    B = 128 << 10
    for mib, ok in ((128, True), (129, False)):
        n = mib << 20
        fr = frame([(1, b"\x00", B)] * (n // B), n)
        assert len(zr.decompress(fr)) == n  # the one-shot decoder has no limit
        if ok:
            assert zr.decompress_stream(fr) == bytes(n)
        else:
            with pytest.raises(zr.ZstdError):
                zr.decompress_stream(fr)
    # the same 129 MiB with a 1 MiB window descriptor: accepted
    n = 129 << 20
    fr = frame([(1, b"\x00", B)] * (n // B), n)
    fr = fr[:4] + bytes([0x80, (20 - 10) << 3]) + n.to_bytes(4, "little") + fr[9:]
    assert zr.decompress_stream(fr) == bytes(n)


def test_bound_large_blobs(rcdc_lib):
    from rustic_core_amd.compress import zstd_bounds
    for n in (0, 1, 1 << 27, (1 << 27) + 1, (1 << 32) - 1):
        nb = max((n + (128 << 10) - 1) // (128 << 10), 1)
        want = n + 3 * nb + (10 if n > (1 << 27) else 9)
        assert rcdc_lib.rcdc_zstd_bound(n) == want
        assert int(zstd_bounds([n])[0]) == want


def test_checker_soak_verdict_helpers():
    """tools/soak_zstd_check.py's host side: block_spots walks libzstd frames
    (single-segment or with a window descriptor), reserved_modes_bits flags
    the seed-604 frame (RFC 8878 3.1.1.3.2.1) and not its source, and the
    verdict follows decode_all's streaming decoder."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "tools"))
    import soak_zstd_check as S
    bad = bytes.fromhex("28b52ffd60f61945000008000101f24aef84")
    good = bytes.fromhex("28b52ffd60f61945000008000100f24aef84")
    assert S.reserved_modes_bits(bad) and not S.reserved_modes_bits(good)
    d = zr.decompress(good)
    assert zr.decompress(bad) == d  # libzstd 1.4.8 decodes it; 1.5 and the device do not
    assert S.libzstd_ok(good, d) and not S.libzstd_ok(bad, d)
    rng = np.random.default_rng(3)
    for n, level in ((100, 3), (300000, 1), (700000, 19)):
        data = rng.integers(0, 8, n, dtype=np.uint8).tobytes()
        fr = zr.compress(data, level)
        heads, bodies = S.block_spots(fr)
        assert heads and heads[-1] + 3 <= len(fr)
        assert S.libzstd_ok(fr, data) and not S.libzstd_ok(fr, data + b"x")
        for _ in range(20):
            S.corrupt(rng, fr, fr)  # any corruption is a byte string
