"""CPU: index files (rustic_core_amd/index.py) -- indexfile.rs:24-143 and
indexer.rs:16-191 -- pinned to the reference's own index file (repo-mixed
fixture, tests/golden/crypto_fixtures.json, decrypted with the oracle).

The device builds the packs (test_gpu_ingest.py, test_gpu_pack.py); here the host logic: JSON
shape and field order (serde_json::to_vec of the structs), parse of the
fixture, the IndexPack of the fixture pack from its pack-file index, the
Indexer's save rule and dedup lookups."""
import base64
import json

import pytest

from tests.test_crypto_oracle import GOLD
from tests.test_pack_oracle import reference_pack


def fixture_index(oracle_mod):
    """(key, pack id, decrypted fixture index JSON bytes)."""
    key, pack, blobs, hnonce = reference_pack(oracle_mod)
    files = {k: base64.b64decode(v) for k, v in GOLD["repo_mixed"].items()}
    name = [k for k in files if k.startswith("repo/index/")][0]
    pid = [k for k in files if k.startswith("repo/data/")][0].rsplit("/", 1)[1]
    return key, bytes.fromhex(pid), oracle_mod.open_(key, files[name])


def norm(obj):
    """Parsed index, uncompressed_length absent == null (Option::None)."""
    out = []
    for p in obj["packs"]:
        out.append((p["id"], [(b["id"], b["type"], b["offset"], b["length"],
                               b.get("uncompressed_length")) for b in p["blobs"]]))
    return out


def test_parse_fixture_index(oracle_mod):
    from rustic_core_amd.index import IndexFile
    _, pid, raw = fixture_index(oracle_mod)
    f = IndexFile.from_json(raw)
    assert len(f.packs) == 1 and f.packs[0].id == pid
    assert [b.type for b in f.packs[0].blobs] == [0, 1, 1, 1, 1]
    # serialised back: the same index (serde field order, compact)
    again = f.to_json()
    assert norm(json.loads(again)) == norm(json.loads(raw))
    assert again.startswith(b'{"packs":[{"id":"' + pid.hex().encode() + b'","blobs":[{"id":')
    assert b'"uncompressed_length":null' in again and b" " not in again


def test_index_pack_of_fixture_pack(oracle_mod):
    """The fixture's pack rebuilt by the oracle (pack_file: the checker of the
    device builder) -> IndexPack from the builder's outputs == the
    reference's index entries for that pack."""
    import numpy as np
    from rustic_core_amd.index import IndexFile, index_packs_from_build
    from rustic_core_amd.pack import make_blobs, pack_layout
    key, pack, blobs, hnonce = reference_pack(oracle_mod)
    _, pid, raw = fixture_index(oracle_mod)
    rebuilt, index = oracle_mod.pack_file(key, blobs, hnonce)
    assert rebuilt == pack
    mb = make_blobs([0] * len(blobs), [len(b[1]) for b in blobs],
                    [np.frombuffer(b[2], np.uint8) for b in blobs],
                    [np.frombuffer(b[3], np.uint8) for b in blobs],
                    types=[b[0] for b in blobs], uncompressed=[b[4] for b in blobs])
    packs, _ = pack_layout(mb, [(0, len(blobs))], [np.frombuffer(hnonce, np.uint8)])
    offsets = np.array([o for o, _ in index], np.uint32)
    ips = index_packs_from_build(mb, packs, offsets, [pid], time="2024-01-01T00:00:00+00:00")
    f = IndexFile(ips)
    assert norm(json.loads(f.to_json())) == norm(json.loads(raw))
    assert json.loads(f.to_json())["packs"][0]["time"] == "2024-01-01T00:00:00+00:00"
    assert ips[0].pack_size() == len(pack)  # PackHeaderRef::pack_size


def test_indexer_save_rule_and_has():
    from rustic_core_amd.index import MAX_COUNT, IndexPack, Indexer
    saved = []
    ix = Indexer(lambda f: saved.append(f) or bytes([len(saved)]) * 32, indexed=set())
    p = IndexPack(b"\x01" * 32)
    for i in range(MAX_COUNT - 1):
        p.add(i.to_bytes(32, "little"), 0, 37 * i, 37)
    ix.add(p)
    assert not saved and ix.has((5).to_bytes(32, "little")) and not ix.has(b"\xff" * 32)
    q = IndexPack(b"\x02" * 32)
    q.add(b"\xee" * 32, 1, 0, 100, 400)
    ix.add(q)  # reaches MAX_COUNT: saved and reset
    assert len(saved) == 1 and len(saved[0].packs) == 2 and ix.count == 0
    ix.finalize()  # nothing left
    assert len(saved) == 1
    ix.add(IndexPack(b"\x03" * 32), delete=True)
    ix.finalize()
    assert len(saved) == 2 and saved[1].packs == [] and len(saved[1].packs_to_delete) == 1
    assert b'"packs_to_delete"' in saved[1].to_json()
    assert ix.saved == [b"\x01" * 32, b"\x02" * 32]


def test_rustic_time_format():
    import datetime
    from rustic_core_amd.index import rustic_time
    t = datetime.datetime(2024, 5, 1, 12, 34, 56, 120000, tzinfo=datetime.timezone.utc)
    s = rustic_time(t)
    assert s[10] == "T" and s[19:22] == ".12" and s[-6] in "+-" and s[-3] == ":"
    local = t.astimezone()
    assert local.strftime("%Y-%m-%dT%H:%M:%S") == s[:19]
