"""rcdc_sha256_host (include/rcdc.h): SHA-256 of many host buffers, 16 side
by side in AVX-512 lanes -- HostIngest's pack ids (blob/packer.rs:832-834
`hash_reader`).  Checked against hashlib on every padding case (lengths
around the 55/56/64-byte block edges), empty messages, and more messages
than lanes of unequal lengths (a lane takes the next message when its own
ends).  CPU only."""
import hashlib

import numpy as np
import pytest

from rustic_core_amd.device import sha256_host, sha256_host_supported

pytestmark = pytest.mark.skipif(not sha256_host_supported(), reason="CPU without AVX-512F/BW")


def _check(lens, seed=0):
    rng = np.random.default_rng(seed)
    bufs = [rng.integers(0, 256, n, dtype=np.uint8) for n in lens]
    got = sha256_host([b.ctypes.data for b in bufs], [b.size for b in bufs])
    assert got == [hashlib.sha256(b.tobytes()).digest() for b in bufs]


def test_block_edges():
    _check(list(range(0, 200)))


def test_more_messages_than_lanes():
    rng = np.random.default_rng(7)
    _check([int(x) for x in rng.integers(0, 70000, 53)] + [1 << 20, 3, 0, 64 * 1000 + 55], seed=1)


def test_none():
    assert sha256_host([], []) == []


def test_bad_input():
    from rustic_core_amd.errors import RusticError
    with pytest.raises(RusticError):
        sha256_host([0], [5])  # a null buffer with bytes


# ---- rcdc_sha256_host_one: one message on the SHA extensions (the pack ids
# whose latency matters), and its portable scalar rounds
_ONE_LENS = [0, 1, 55, 56, 63, 64, 65, 119, 120, 128, 1000, 12345, (1 << 20) + 7]


def test_sha256_host_one_matches_hashlib():
    from rustic_core_amd.native_ingest import sha256_host_one
    rng = np.random.default_rng(5)
    for n in _ONE_LENS:
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert sha256_host_one(b) == hashlib.sha256(b).digest(), n


def test_sha256_host_one_scalar_rounds():
    """RCDC_NO_SHANI=1: the fallback for CPUs without the SHA extensions."""
    import os
    import subprocess
    import sys
    code = ("import hashlib, numpy as np\n"
            "from rustic_core_amd.native_ingest import sha256_host_one\n"
            "rng = np.random.default_rng(6)\n"
            f"for n in {_ONE_LENS!r}:\n"
            "    b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()\n"
            "    assert sha256_host_one(b) == hashlib.sha256(b).digest(), n\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True,
                       env=dict(os.environ, RCDC_NO_SHANI="1"), timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]


@pytest.mark.parametrize("ways", [1, 2, 3, 4])
def test_sha256_host_ni_interleaved(ways):
    """rcdc_sha256_host_ni: `ways` messages interleaved on the SHA extensions
    (the ingest's last pack ids).  Unequal lengths in a group (the shared
    blocks run interleaved, the rest alone), every padding edge, and counts
    that do not fill the last group."""
    from rustic_core_amd.native_ingest import sha256_host_ni
    rng = np.random.default_rng(11 + ways)
    lens = _ONE_LENS + [int(x) for x in rng.integers(0, 300000, 9)]
    bufs = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in lens]
    assert sha256_host_ni(bufs, ways) == [hashlib.sha256(b).digest() for b in bufs]
    assert sha256_host_ni(bufs[:ways + 1], ways) == [hashlib.sha256(b).digest()
                                                     for b in bufs[:ways + 1]]


def test_sha256_host_ni_rejects():
    from rustic_core_amd.errors import RusticError
    from rustic_core_amd.native_ingest import sha256_host_ni
    assert sha256_host_ni([], 2) == []
    for ways in (0, 5):
        with pytest.raises(RusticError):
            sha256_host_ni([b"abc"], ways)
