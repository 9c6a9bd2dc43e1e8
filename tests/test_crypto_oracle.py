"""CPU: pin the blob-encryption oracle (oracle/crypto_ref.c: rustic's
Key::encrypt_data / decrypt_data, crates/core/src/crypto/aespoly1305.rs:88-135,
over aes256ctr_poly1305aes 0.2.1) before the device AEAD is compared with it.

Pins: FIPS-197 Appendix C (AES-128, AES-256), RFC 8439 2.5.2 (Poly1305), and
the reference's own encrypted fixtures (tests/golden/crypto_fixtures.json,
made by make_crypto_golden.py): key files opened with their passwords
(scrypt, hashlib), the config decrypted with the master key, and every blob
of the repo-mixed fixture's pack file decrypted with a valid MAC (uncompressed
blobs: sha256(plaintext) == the id in the pack header).
"""
import base64
import hashlib
import json
import os
import struct

import pytest

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "crypto_fixtures.json")))


def _kdf(keyfile: dict, password: str) -> bytes:
    return hashlib.scrypt(password.encode(), salt=base64.b64decode(keyfile["salt"]),
                          n=keyfile["N"], r=keyfile["r"], p=keyfile["p"], maxmem=1 << 30,
                          dklen=64)


def _master(mk: dict) -> bytes:
    """MasterKey JSON (repofile/keyfile.rs:308-335) -> the 64-byte key:
    encrypt || mac.k || mac.r (aespoly1305.rs Key::from_keys)."""
    return (base64.b64decode(mk["encrypt"]) + base64.b64decode(mk["mac"]["k"]) +
            base64.b64decode(mk["mac"]["r"]))


def test_aes_fips197(oracle_mod):
    pt = bytes.fromhex("00112233445566778899aabbccddeeff")
    assert oracle_mod.aes_encrypt_block(bytes(range(16)), pt).hex() == \
        "69c4e0d86a7b0430d8cdb78070b4c55a"
    assert oracle_mod.aes_encrypt_block(bytes(range(32)), pt).hex() == \
        "8ea2b7ca516745bfeafc49904b496089"


def test_poly1305_rfc8439(oracle_mod):
    r = bytes.fromhex("85d6be7857556d337f4452fe42d506a8")
    s = bytes.fromhex("0103808afb0db2fd4abff6af4149f51b")
    assert oracle_mod.poly1305(r, s, b"Cryptographic Forum Research Group").hex() == \
        "a8061dc1305136c6c22b8baf0c0127a9"


@pytest.mark.parametrize("name", ["key1", "key2"])
def test_reference_key_files_and_config(oracle_mod, name):
    """keys.rs:12-35: key1/key2 open with "test"/"test2", a wrong password
    fails the MAC; the config decrypts to the repository's JSON."""
    g = GOLD["keys_test"]
    kf = json.loads(base64.b64decode(g[name]))
    data = base64.b64decode(kf["data"])
    mk = json.loads(oracle_mod.open_(_kdf(kf, g["passwords"][name]), data))
    with pytest.raises(oracle_mod.MacMismatch):
        oracle_mod.open_(_kdf(kf, "wrong"), data)
    cfg = json.loads(oracle_mod.open_(_master(mk), base64.b64decode(g["config"])))
    assert cfg["version"] == 2 and cfg["chunker_polynomial"] == "379e1f8576e839"


def _repo_master(oracle_mod):
    files = {k: base64.b64decode(v) for k, v in GOLD["repo_mixed"].items()}
    kname = [k for k in files if k.startswith("repo/keys/")][0]
    kf = json.loads(files[kname])
    mk = json.loads(oracle_mod.open_(_kdf(kf, GOLD["repo_mixed_password"]),
                                     base64.b64decode(kf["data"])))
    return _master(mk), files


def pack_blobs(oracle_mod, key: bytes, pack: bytes):
    """restic pack: blobs, then the encrypted header, then its length (u32 LE).
    Header entries: type (0 data, 1 tree: + u32 length + 32-byte id; 2, 3:
    compressed, + u32 length + u32 uncompressed length + id)."""
    hlen = struct.unpack("<I", pack[-4:])[0]
    header = oracle_mod.open_(key, pack[-4 - hlen:-4])
    out, pos, off = [], 0, 0
    while pos < len(header):
        t = header[pos]
        length = struct.unpack("<I", header[pos + 1:pos + 5])[0]
        if t in (0, 1):
            bid, pos = header[pos + 5:pos + 37], pos + 37
        else:
            bid, pos = header[pos + 9:pos + 41], pos + 41
        out.append((t, off, length, bid))
        off += length
    return out


def test_reference_repo_pack_blobs(oracle_mod):
    key, files = _repo_master(oracle_mod)
    cfg = json.loads(oracle_mod.open_(key, files["repo/config"]))
    assert cfg["version"] in (1, 2)
    packs = [v for k, v in files.items() if k.startswith("repo/data/")]
    assert packs
    n = 0
    for pack in packs:
        for t, off, length, bid in pack_blobs(oracle_mod, key, pack):
            plain = oracle_mod.open_(key, pack[off:off + length])
            if t in (0, 1):
                assert hashlib.sha256(plain).digest() == bid
            else:
                assert plain[:4] == b"\x28\xb5\x2f\xfd"  # a zstd frame (not decompressed here)
            n += 1
    assert n >= 2
    # index and snapshot files: encrypted too (uncompressed JSON or a zstd frame)
    for k in files:
        if k.startswith(("repo/index/", "repo/snapshots/")):
            p = oracle_mod.open_(key, files[k])
            assert p[:1] in (b"{", b"[") or p[:1] == b"\x02"


def test_seal_open_roundtrip(oracle_mod):
    import numpy as np
    rng = np.random.default_rng(5)
    key = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
    for n in (0, 1, 15, 16, 17, 31, 32, 33, 1000, 65537):
        nonce = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        enc = oracle_mod.seal(key, nonce, data)
        assert len(enc) == n + 32 and enc[:16] == nonce
        assert oracle_mod.open_(key, enc) == data
        bad = bytearray(enc)
        bad[16 + n // 2 if n else 16] ^= 1
        with pytest.raises(oracle_mod.MacMismatch):
            oracle_mod.open_(key, bytes(bad))
