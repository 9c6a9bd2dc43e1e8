"""Regenerate tests/golden/reference_snapshots.json from the reference's own
insta snapshots (run in the build container, where /root/reference exists).

The JSON holds DATA only: the inputs that the reference tests use (seed, size,
chunker parameters, rabin.rs:329-347 / fixed_size.rs:82-95) and the expected
(len, sha256) lists copied from
  crates/core/src/chunker/snapshots/rustic_core__chunker__rabin__tests__chunk_random.snap
  crates/core/src/chunker/snapshots/rustic_core__chunker__fixed_size__tests__chunk-size1048576.snap
  crates/core/src/chunker/snapshots/rustic_core__chunker__fixed_size__tests__chunk-size1045504.snap
plus the known answers of rabin.rs:360-385 (chunk_empty, chunk_empty_wrong_hint,
chunk_zeros).
"""
import json
import os
import re

REF = "/root/reference/crates/core/src/chunker/snapshots"
HERE = os.path.dirname(os.path.abspath(__file__))


def parse(name):
    text = open(os.path.join(REF, name)).read()
    return [[int(n), h] for n, h in re.findall(r'\((\d+), Id\("([0-9a-f]{64})"\)\)', text)]


def main():
    out = {
        "source": "rustic_core 0.12.0 crates/core/src/chunker (insta RON snapshots)",
        "rabin_chunk_random": {
            "ref": "crates/core/src/chunker/rabin.rs:341-358",
            "rng": "StdRng::seed_from_u64", "seed": 23, "size": 32 * 1024 * 1024,
            "poly": "0x003DA3358B4DC173", "avg": 1 << 20, "min": 512 * 1024,
            "max": 8 * 1024 * 1024,
            "chunks": parse("rustic_core__chunker__rabin__tests__chunk_random.snap"),
        },
        "fixed_chunk_random": [
            {"ref": "crates/core/src/chunker/fixed_size.rs:82-102", "seed": 23,
             "size": 32 * 1024 * 1024, "chunk_size": cs,
             "chunks": parse(f"rustic_core__chunker__fixed_size__tests__chunk-size{cs}.snap")}
            for cs in (1048576, 1045504)
        ],
        "known_answers": {
            "chunk_empty": {"ref": "rabin.rs:360-367", "n": 0, "chunks": 0},
            "chunk_empty_wrong_hint": {"ref": "rabin.rs:369-376", "n": 0, "size_hint": 100,
                                       "chunks": 0},
            "chunk_zeros": {"ref": "rabin.rs:378-385", "first_chunk_len": 512 * 1024},
        },
    }
    with open(os.path.join(HERE, "reference_snapshots.json"), "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
