"""CPU: pin the oracle (oracle/cdc_ref.c, oracle/pyref.py) to the reference's
own golden vectors before anything is compared against it.

Fixtures (tests/golden/reference_snapshots.json, made by make_golden.py from
the reference's insta snapshots):
  crates/core/src/chunker/rabin.rs:341-358      chunk_random (29 x (len, sha256))
  crates/core/src/chunker/rabin.rs:360-385      chunk_empty / _wrong_hint / chunk_zeros
  crates/core/src/chunker/fixed_size.rs:82-102  chunk-size1048576 / chunk-size1045504
The random input is rand 0.10 StdRng::seed_from_u64(23) (ChaCha12), restated
in cdc_ref_stdrng_fill; the FixedSize snapshots pin that stream on their own.
"""
import hashlib
import json
import os

import numpy as np
import pytest

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_snapshots.json")))


def _lens_hashes(data: np.ndarray, cuts) -> list:
    out, s = [], 0
    for c in cuts:
        c = int(c)
        out.append([c - s, hashlib.sha256(data[s:c].tobytes()).hexdigest()])
        s = c
    return out


@pytest.fixture(scope="module")
def random32(oracle_mod):
    g = GOLD["rabin_chunk_random"]
    return oracle_mod.stdrng_bytes(g["seed"], g["size"])


def test_rabin_chunk_random_snapshot(oracle_mod, random32):
    g = GOLD["rabin_chunk_random"]
    cuts = oracle_mod.chunk_cuts(random32, int(g["poly"], 16), g["min"], g["avg"], g["max"])
    assert _lens_hashes(random32, cuts) == g["chunks"]


def test_rabin_chunk_random_owned_mode(oracle_mod, random32):
    """Reference-equivalent mode (owned chunks, 4 KiB reads) = same cuts."""
    g = GOLD["rabin_chunk_random"]
    a = oracle_mod.chunk_cuts(random32, int(g["poly"], 16), g["min"], g["avg"], g["max"])
    b = oracle_mod.chunk_cuts_owned(random32, int(g["poly"], 16), g["min"], g["avg"], g["max"])
    assert np.array_equal(a, b)


@pytest.mark.parametrize("entry", GOLD["fixed_chunk_random"], ids=lambda e: str(e["chunk_size"]))
def test_fixed_size_snapshots(oracle_mod, random32, entry):
    assert entry["seed"] == GOLD["rabin_chunk_random"]["seed"]
    cuts = oracle_mod.fixed_cuts(entry["size"], entry["chunk_size"])
    assert _lens_hashes(random32[: entry["size"]], cuts) == entry["chunks"]


def test_known_answers(oracle_mod):
    ka = GOLD["known_answers"]
    assert len(oracle_mod.chunk_cuts(np.zeros(0, np.uint8))) == ka["chunk_empty"]["chunks"] == 0
    zeros = np.zeros(4 << 20, np.uint8)
    cuts = oracle_mod.chunk_cuts(zeros)
    assert int(cuts[0]) == ka["chunk_zeros"]["first_chunk_len"]
    # every zero chunk is exactly min long (fp(0...0) = 0 hits at s + min)
    assert np.all(np.diff(np.concatenate([[0], cuts])) == 512 * 1024)


def test_stdrng_skip_consistent(oracle_mod):
    full = oracle_mod.stdrng_bytes(7, 1 << 16)
    for skip in (0, 64, 128, 4096, 4096 + 64 * 7):
        part = oracle_mod.stdrng_bytes(7, 1000, skip=skip)
        assert np.array_equal(part, full[skip:skip + 1000])


@pytest.mark.parametrize("params", [(4096, 4096, 8192), (8192, 4096, 6000),
                                    (4096, 4096, 4096)])
def test_c_oracle_matches_pure_python(oracle_mod, params):
    """Two independent restatements of rabin.rs:107-191 agree: the C oracle
    (literal ring-window Rabin64) and pyref (closed-form fp per window).
    Small masks (avg 4096/8192) so that hits, max cuts and zone cuts occur
    within a few chunks; min >= 4096, the domain librcdc accepts."""
    from oracle import pyref
    avg, mn, mx = params
    rng = np.random.default_rng(avg + mx)
    parts = [rng.integers(0, 256, 14000, dtype=np.uint8), np.zeros(9000, np.uint8),
             rng.integers(0, 4, 9000, dtype=np.uint8)]
    data = np.concatenate(parts)
    c = oracle_mod.chunk_cuts(data, oracle_mod.DEFAULT_POLY, mn, avg, mx)
    p = pyref.chunk_cuts(data.tobytes(), oracle_mod.DEFAULT_POLY, mn, avg, mx)
    assert list(map(int, c)) == list(p)


def test_candidates_match_window_fp(oracle_mod):
    """cand(p) = fp(b[p-64, p)) & mask == 0 per position."""
    from oracle import pyref
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, 3000, dtype=np.uint8)
    mask = 15  # dense candidates
    flags = oracle_mod.candidates(data, 64, 2900, oracle_mod.DEFAULT_POLY, mask)
    want = [(pyref.fp(data[p - 64:p].tobytes(), oracle_mod.DEFAULT_POLY) & mask) == 0
            for p in range(64, 2964)]
    assert list(map(bool, flags)) == want


@pytest.mark.parametrize("avg,mn,mx,ok", [
    (1 << 20, 1 << 19, 1 << 23, True),
    (1 << 20, 1 << 20, 1 << 20, True),
    ((1 << 20) + 1, 1 << 19, 1 << 23, False),   # not a power of 2 (rabin.rs:22)
    (1 << 20, (1 << 20) + 1, 1 << 23, False),   # min > avg (rabin.rs:29)
    (1 << 20, 1 << 19, (1 << 20) - 1, False),   # max < avg (rabin.rs:35)
])
def test_check_params(oracle_mod, avg, mn, mx, ok):
    assert oracle_mod.check_params(avg, mn, mx) == ok


# ----------------------------------------------------------------------------
# The reference-equivalent mode (owned Vec per chunk fed from the 4 KiB read
# buffer, rabin.rs:110-191) equals the ideal cut function on every parameter
# set librcdc accepts, whatever the reader's read sizes.  Below min = 4096
# rabin.rs:124 underflows -- the reason librcdc rejects those parameters.
ACCEPTED = [(4096, 4096, 4096), (4096, 4096, 1 << 16), (4096, 8192, 16384),
            (5000, 8192, 12000), (4096, 1 << 16, 1 << 20), (65536, 1 << 16, 1 << 16),
            (1 << 19, 1 << 20, 1 << 23)]


def _kinds(n, seed):
    rng = np.random.default_rng(seed)
    mixed = np.zeros(n, np.uint8)
    p = 0
    while p < n:
        r = int(rng.integers(1, 20000))
        mixed[p:p + r] = rng.integers(0, 256, len(mixed[p:p + r]), dtype=np.uint8)
        p += r + int(rng.integers(1, 30000))
    return {"random": rng.integers(0, 256, n, dtype=np.uint8), "zeros": np.zeros(n, np.uint8),
            "mixed": mixed, "lowent": rng.integers(0, 2, n, dtype=np.uint8)}


@pytest.mark.parametrize("params", ACCEPTED, ids=lambda p: "-".join(map(str, p)))
def test_owned_mode_equals_ideal_on_accepted_params(oracle_mod, rcdc_lib, params):
    mn, avg, mx = params
    assert rcdc_lib.rcdc_check_params(avg, mn, mx) == 0
    n = 3 * (1 << 20) + 4321 if mn >= (1 << 19) else 600_000 + 777
    for kind, data in _kinds(n, mn + avg).items():
        ideal = oracle_mod.chunk_cuts(data, oracle_mod.DEFAULT_POLY, mn, avg, mx)
        for read_seed in (0, 12345):
            owned = oracle_mod.chunk_cuts_owned(data, oracle_mod.DEFAULT_POLY, mn, avg, mx,
                                                read_seed=read_seed)
            assert np.array_equal(ideal, owned), (kind, read_seed)


@pytest.mark.parametrize("mn", [64, 1024, 4000])
def test_reference_underflows_below_4096(oracle_mod, rcdc_lib, mn):
    """rabin.rs:124 on random bytes at min < 4096: a chunk ends mid-buffer
    with more read-ahead bytes than min -> the reference's subtraction
    underflows (the oracle reports it instead of wrapping), and librcdc
    rejects the parameters as Unsupported."""
    from oracle.oracle import ReferenceUnderflow
    data = np.random.default_rng(mn).integers(0, 256, 400_000, dtype=np.uint8)
    with pytest.raises(ReferenceUnderflow):
        oracle_mod.chunk_cuts_owned(data, oracle_mod.DEFAULT_POLY, mn, 4096, 16384)
    assert rcdc_lib.rcdc_check_params(4096, mn, 16384) == 1


def test_chunk_many_cuts_equals_per_file(oracle_mod):
    """The threaded batch checker (bench.py's parity leg over whole batches)
    returns each file's cut list exactly as the single-file oracle does,
    including empty, sub-min, unaligned and exactly-min files."""
    kinds = _kinds(5 * (1 << 20) + 333, 77)
    lens = [0, 100, 1 << 19, (1 << 19) + 1, 3 * (1 << 20) + 7, 5 * (1 << 20) + 333]
    files = [kinds["random"][:lens[0]], kinds["zeros"][:lens[1]], kinds["mixed"][:lens[2]],
             kinds["random"][:lens[3]], kinds["lowent"][:lens[4]], kinds["mixed"][:lens[5]]]
    offs, pos = [], 3
    arena = np.zeros(sum(lens) + 64 * len(lens), np.uint8)
    for f in files:
        offs.append(pos)
        arena[pos:pos + f.size] = f
        pos += f.size + 17
    got = oracle_mod.chunk_many_cuts(arena, offs, lens, nthreads=4)
    for g, f in zip(got, files):
        assert np.array_equal(g, oracle_mod.chunk_cuts(f))
