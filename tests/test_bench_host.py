"""CPU: bench.py's host-side pieces -- the C1 input generator (rand 0.10
StdRng, pinned to the oracle's restatement, itself pinned to the reference
snapshots) and the --gpus / WORLD_SIZE contract."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_stdrng_numpy_matches_oracle(oracle_mod):
    sys.path.insert(0, ROOT)
    from bench import stdrng_numpy
    for seed, n in [(23, 4096 + 13), (0x256, 1 << 16), (1000, 777)]:
        assert np.array_equal(stdrng_numpy(seed, n), oracle_mod.stdrng_bytes(seed, n)), seed


def test_ref_slide_bytes():
    sys.path.insert(0, ROOT)
    from bench import ref_slide_bytes
    mn = 512 << 10
    # chunks: min exactly (63 prefill bytes, 0 slides), min + 100, and a short tail
    cuts = [np.array([mn, 2 * mn + 100, 2 * mn + 150], np.uint64)]
    assert ref_slide_bytes(cuts, mn) == 63 + (63 + 100)


def test_gpus_must_match_world_size():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr
