"""Host logic of the device ingest path (rustic_core_amd/ingest.py) that runs
without a GPU: the dedup rule (blob/packer.rs:304-315: first occurrence in
chunk order, skipped when the index has the id) and the configuration it
derives (configfile.rs:182-199: zstd level, extra_verify)."""
import numpy as np
import pytest

from rustic_core_amd.chunker import ConfigFile
from rustic_core_amd.errors import RusticError
from rustic_core_amd.ingest import first_occurrences


def _ids(seq):
    return np.array([[v] * 32 for v in seq], np.uint8)


def test_first_occurrence_in_chunk_order():
    ids = _ids([5, 3, 5, 7, 3, 3, 9])
    got = first_occurrences(ids, np.arange(7), set())
    assert got.tolist() == [True, True, False, True, False, False, True]


def test_subset_and_known_ids():
    ids = _ids([5, 3, 5, 7, 3, 3, 9])
    # only the chunks listed (any order) are considered
    got = first_occurrences(ids, np.array([6, 2, 4, 0]), set())
    assert got.tolist() == [True, False, False, False, True, False, True]
    known = {bytes([3] * 32), bytes([9] * 32)}
    got = first_occurrences(ids, np.arange(7), known)
    assert got.tolist() == [True, False, False, True, False, False, False]
    assert not first_occurrences(ids[:0], np.zeros(0, np.int64), known).any()


def test_matches_a_sequential_packer():
    rng = np.random.default_rng(1)
    vals = rng.integers(0, 40, 500)
    ids = _ids(vals)
    known = {bytes([v] * 32) for v in range(0, 40, 7)}
    seen, exp = set(known), []
    for v in vals:
        b = bytes([v] * 32)
        exp.append(b not in seen)
        seen.add(b)
    assert first_occurrences(ids, np.arange(len(vals)), known).tolist() == exp


def test_config_zstd_and_verify():
    c = ConfigFile.new(2, 0x3DA3358B4DC173)
    assert c.zstd() == 0 and c.extra_verify_()          # version 2 default: level 0, verify
    c.compression = 0
    assert c.zstd() is None                              # (2, Some(0)): no compression
    c.compression = 19
    assert c.zstd() == 19
    c.extra_verify = False
    assert not c.extra_verify_()
    assert ConfigFile.new(1, 0x3DA3358B4DC173).zstd() is None
    with pytest.raises(RusticError):
        ConfigFile.new(3, 0x3DA3358B4DC173).zstd()


def test_plan_batches():
    """HostIngest batches: whole files in order; a small first and last batch
    around middle ones of about `middle` bytes."""
    from rustic_core_amd.ingest import plan_batches
    G = 1 << 30
    b = plan_batches([G] * 96, 4 * G, 16 * G, 4 * G)
    assert [len(x) for x in b][0] == 4 and [len(x) for x in b][-1] == 4
    assert sum(b, []) == list(range(96))
    assert all(len(x) <= 16 for x in b)
    assert plan_batches([G] * 3, 4 * G, 16 * G, 4 * G) == [[0, 1, 2]]
    b = plan_batches([5 << 20] * 7 + [300 << 20], 10 << 20, 20 << 20, 10 << 20)
    assert sum(b, []) == list(range(8)) and b[-1] == [7]
