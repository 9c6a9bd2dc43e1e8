"""Blob encryption on the device (rcdc_aead.hip) -- SURVEY.md 8(f) row 3.

Reference: ``Key::encrypt_data`` / ``decrypt_data`` (crates/core/src/crypto/
aespoly1305.rs:88-135, aes256ctr_poly1305aes 0.2.1 -- the restic format
nonce || AES-256-CTR || Poly1305-AES tag), applied per blob by the packer
(blob/packer.rs:268-270) and the restore path (backend/decrypt.rs:566-572).

Checker: oracle/crypto_ref.c (pinned in test_crypto_oracle.py to FIPS-197,
RFC 8439 and the reference's encrypted fixtures).  Decryption is pinned
directly on the reference's own encrypted repository files
(tests/golden/crypto_fixtures.json): config, index, snapshot and every blob
of the pack file open with a valid MAC on the device and give the bytes the
pack header's SHA-256 ids name.  Bit-exact output is the bar.
"""
import base64
import hashlib
import json
import os
import struct

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "crypto_fixtures.json")))
MiB = 1 << 20


def _dev(host: np.ndarray):
    import torch
    return torch.from_numpy(np.ascontiguousarray(host)).to("cuda:0")


def _seal_dev(key, datas, nonces, in_pad=(), stream=None):
    """Seal ``datas`` in one batch; in_offs carry the given extra misalignment."""
    import torch
    from rustic_core_amd.crypto import make_refs, sealed_layout
    offs, o = [], 0
    for i, d in enumerate(datas):
        o += in_pad[i] if i < len(in_pad) else 0
        offs.append(o)
        o += len(d)
    arena = np.zeros(o + 64, np.uint8)
    for off, d in zip(offs, datas):
        arena[off:off + len(d)] = np.frombuffer(d, np.uint8)
    lens = [len(d) for d in datas]
    oo, olen = sealed_layout(lens)
    refs = make_refs(offs, lens, oo, b"".join(nonces))
    d_in = _dev(arena)
    d_out = torch.full((olen + 64,), 0xA5, dtype=torch.uint8, device="cuda:0")
    key.seal_blobs(d_in.data_ptr(), refs, d_out.data_ptr(), stream)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    return [out[int(a):int(a) + n + 32].tobytes() for a, n in zip(oo, lens)], out, oo, olen


def _open_dev(key, blobs, pads=()):
    import torch
    from rustic_core_amd.crypto import make_refs
    offs, o = [], 0
    for i, b in enumerate(blobs):
        o += pads[i] if i < len(pads) else 0
        offs.append(o)
        o += len(b)
    arena = np.zeros(o + 64, np.uint8)
    for off, b in zip(offs, blobs):
        arena[off:off + len(b)] = np.frombuffer(b, np.uint8)
    outs, p = [], 0
    for b in blobs:
        outs.append(p)
        p = (p + max(len(b) - 32, 0) + 15) // 16 * 16
    refs = make_refs(offs, [len(b) for b in blobs], outs)
    d_in = _dev(arena)
    d_out = torch.zeros(p + 64, dtype=torch.uint8, device="cuda:0")
    st = key.open_blobs(d_in.data_ptr(), refs, d_out.data_ptr())
    out = d_out.cpu().numpy()
    return st, [out[a:a + max(len(b) - 32, 0)].tobytes() for a, b in zip(outs, blobs)]


@pytest.fixture(scope="module")
def rng():
    return np.random.default_rng(0xAEAD)


def _rand(rng, n):
    return rng.integers(0, 256, n, dtype=np.uint8).tobytes()


LENS = [0, 1, 15, 16, 17, 31, 32, 33, 63, 64, 65, 1000, 1024, 4095, 65535, 65536, 65537,
        4096 * 16 - 1, 4096 * 16, 4096 * 16 + 1, 3 * 65536 + 7, MiB + 3]


def test_seal_matches_oracle_batch(gpu_ctx, oracle_mod, rng):
    """One batch of ragged blobs at every alignment; the unit size (4096
    blocks) and the partial final block straddled."""
    from rustic_core_amd.crypto import Key
    key = Key(_rand(rng, 64))
    datas = [_rand(rng, n) for n in LENS]
    nonces = [_rand(rng, 16) for _ in LENS]
    pads = [int(x) for x in rng.integers(0, 16, len(LENS))]
    got, out, oo, olen = _seal_dev(key, datas, nonces, pads)
    for n, d, nc, g in zip(LENS, datas, nonces, got):
        assert g == oracle_mod.seal(key._key, nc, d), f"len {n}"
    # nothing outside the sealed blobs was written (the gaps keep 0xA5)
    mask = np.ones(olen + 64, bool)
    for a, n in zip(oo, LENS):
        mask[int(a):int(a) + n + 32] = False
    assert np.all(out[mask] == 0xA5)


def test_seal_counter_carry(gpu_ctx, oracle_mod, rng):
    """The 128-bit big-endian counter carries across its 64-bit halves and
    wraps at 2^128 (nonces ending in ff..ff)."""
    from rustic_core_amd.crypto import Key
    key = Key(_rand(rng, 64))
    nonces = [b"\x00" * 8 + b"\xff" * 8, b"\xff" * 16, b"\x12" * 8 + b"\xff" * 7 + b"\xf0"]
    datas = [_rand(rng, 5000 * 16 + 9) for _ in nonces]
    got, *_ = _seal_dev(key, datas, nonces)
    for d, nc, g in zip(datas, nonces, got):
        assert g == oracle_mod.seal(key._key, nc, d)


def test_seal_max_chunk_and_many(gpu_ctx, oracle_mod, rng):
    """A max-size chunk (8 MiB, rabin.rs:12) and 200 chunk-like blobs."""
    from rustic_core_amd.crypto import Key
    key = Key(_rand(rng, 64))
    lens = [8 * MiB] + [int(x) for x in rng.integers(1, 200_000, 200)]
    datas = [_rand(rng, n) for n in lens]
    nonces = [_rand(rng, 16) for _ in lens]
    got, *_ = _seal_dev(key, datas, nonces)
    for i in [0, 1, 2, 50, 199, 200]:
        assert got[i] == oracle_mod.seal(key._key, nonces[i], datas[i]), i
    st, plain = _open_dev(key, got)
    assert not st.any()
    assert plain == datas


def _kdf(keyfile, password):
    return hashlib.scrypt(password.encode(), salt=base64.b64decode(keyfile["salt"]),
                          n=keyfile["N"], r=keyfile["r"], p=keyfile["p"], maxmem=1 << 30,
                          dklen=64)


def _master(mk):
    return (base64.b64decode(mk["encrypt"]) + base64.b64decode(mk["mac"]["k"]) +
            base64.b64decode(mk["mac"]["r"]))


def test_open_reference_key_files(gpu_ctx):
    """keys.rs:12-35 fixtures: the key files' data opens on the device with
    the scrypt key of the right password and fails with a wrong one; the
    config decrypts with the master key (aespoly1305.rs:88-108)."""
    from rustic_core_amd.crypto import Key
    from rustic_core_amd.errors import ErrorKind, RusticError
    g = GOLD["keys_test"]
    for name in ("key1", "key2"):
        kf = json.loads(base64.b64decode(g[name]))
        data = base64.b64decode(kf["data"])
        mk = json.loads(Key(_kdf(kf, g["passwords"][name])).decrypt_data(data))
        with pytest.raises(RusticError) as ei:
            Key(_kdf(kf, "wrong")).decrypt_data(data)
        assert ei.value.kind == ErrorKind.Cryptography
        cfg = json.loads(Key(_master(mk)).decrypt_data(base64.b64decode(g["config"])))
        assert cfg["chunker_polynomial"] == "379e1f8576e839"


def test_open_reference_repo_files(gpu_ctx, oracle_mod):
    """repo-mixed fixture: config, index, snapshot and every pack blob open in
    ONE device batch (unaligned offsets inside the pack) with valid MACs;
    uncompressed blobs hash to their pack-header ids."""
    from rustic_core_amd.crypto import Key, make_refs
    import torch
    files = {k: base64.b64decode(v) for k, v in GOLD["repo_mixed"].items()}
    kname = [k for k in files if k.startswith("repo/keys/")][0]
    kf = json.loads(files[kname])
    mk = json.loads(Key(_kdf(kf, GOLD["repo_mixed_password"])).decrypt_data(
        base64.b64decode(kf["data"])))
    key = Key(_master(mk))
    pack_name = [k for k in files if k.startswith("repo/data/")][0]
    pack = files[pack_name]
    hlen = struct.unpack("<I", pack[-4:])[0]
    header = key.decrypt_data(pack[-4 - hlen:-4])
    assert header == oracle_mod.open_(key._key, pack[-4 - hlen:-4])
    entries, pos, off = [], 0, 0
    while pos < len(header):
        t = header[pos]
        length = struct.unpack("<I", header[pos + 1:pos + 5])[0]
        bid = header[pos + 5:pos + 37] if t in (0, 1) else header[pos + 9:pos + 41]
        pos += 37 if t in (0, 1) else 41
        entries.append((t, off, length, bid))
        off += length
    assert len(entries) >= 2
    # the pack itself in HBM, blobs opened where they lie
    arena = np.zeros(len(pack) + 64, np.uint8)
    arena[:len(pack)] = np.frombuffer(pack, np.uint8)
    outs, p = [], 0
    for _, o, length, _ in entries:
        outs.append(p)
        p = (p + length - 32 + 15) // 16 * 16
    refs = make_refs([e[1] for e in entries], [e[2] for e in entries], outs)
    d_in = _dev(arena)
    d_out = torch.zeros(p + 64, dtype=torch.uint8, device="cuda:0")
    st = key.open_blobs(d_in.data_ptr(), refs, d_out.data_ptr())
    assert not st.any()
    out = d_out.cpu().numpy()
    for (t, o, length, bid), a in zip(entries, outs):
        plain = out[a:a + length - 32].tobytes()
        assert plain == oracle_mod.open_(key._key, pack[o:o + length])
        if t in (0, 1):
            assert hashlib.sha256(plain).digest() == bid
        else:
            assert plain[:4] == b"\x28\xb5\x2f\xfd"  # zstd frame (decompression: out of scope)
    for k in files:
        if k.startswith(("repo/index/", "repo/snapshots/", "repo/config")):
            assert key.decrypt_data(files[k]) == oracle_mod.open_(key._key, files[k])


def test_open_mac_failures_and_short_blobs(gpu_ctx, oracle_mod, rng):
    """A flipped bit anywhere (nonce, ciphertext, tag) fails only its own
    blob's MAC; < 16 bytes is status 2 (aespoly1305.rs:89-94), 16..31 fails
    the MAC check (status 1)."""
    from rustic_core_amd.crypto import Key
    key = Key(_rand(rng, 64))
    lens = [0, 1, 100, 70000]
    datas = [_rand(rng, n) for n in lens]
    sealed = [oracle_mod.seal(key._key, _rand(rng, 16), d) for d in datas]
    blobs, expect = [], []
    for s in sealed:
        blobs.append(s)
        expect.append(0)
        for pos in (0, 16, len(s) - 1, len(s) // 2):
            b = bytearray(s)
            b[pos] ^= 0x40
            blobs.append(bytes(b))
            expect.append(1)
    blobs += [b"", b"\x01" * 15, b"\x02" * 16, b"\x03" * 31]
    expect += [2, 2, 1, 1]
    pads = [int(x) for x in rng.integers(0, 16, len(blobs))]
    st, plain = _open_dev(key, blobs, pads)
    assert st.tolist() == expect
    k = 0
    for s, d in zip(sealed, datas):
        assert plain[k] == d
        k += 5


def test_encrypt_decrypt_data_roundtrip(gpu_ctx, oracle_mod, rng):
    """CryptoKey surface (aespoly1305.rs:78-135) with the device underneath:
    random nonce per call, decrypt(encrypt(x)) == x, matches the oracle."""
    from rustic_core_amd.crypto import Key
    from rustic_core_amd.errors import RusticError
    key = Key.new()
    for n in (0, 5, 16, 12345):
        d = _rand(rng, n)
        e = key.encrypt_data(d)
        assert len(e) == n + 32
        assert oracle_mod.open_(key._key, e) == d
        assert key.decrypt_data(e) == d
    with pytest.raises(RusticError):
        key.decrypt_data(b"short")
    enc, k, r = key.to_keys()
    assert Key.from_keys(enc, k, r)._key == key._key


def test_null_stream_orders_with_default_stream(gpu_ctx, oracle_mod, rng):
    """hip_stream = 0 (torch's default stream) with no explicit synchronize:
    the input is produced by a chain of async kernels on the default stream
    right before the seal / zstd / chunk calls, and their outputs are read
    back by default-stream copies right after (rcdc_runtime.cpp null_enter /
    null_leave order the context's own stream with the default stream)."""
    import torch
    from rustic_core_amd.compress import compress_blobs, frame_layout, make_refs as zrefs
    from rustic_core_amd.crypto import Key, make_refs, sealed_layout
    from oracle import zstd_ref
    n = 64 * MiB
    base = np.arange(n, dtype=np.uint64).astype(np.uint8) * np.uint8(7)
    want = base.copy()
    for _ in range(48):
        want = (want * np.uint8(3) + np.uint8(1)).astype(np.uint8)
    assert torch.cuda.current_stream().cuda_stream == 0
    key = Key(_rand(rng, 64))
    nonce = _rand(rng, 16)
    lens = [n - 69, 4]  # inputs end 64 bytes before the tensor (the kernel reads ahead)
    offs = [0, n - 69]
    oo, olen = sealed_layout(lens)
    for trial in range(2):
        x = torch.from_numpy(base).to("cuda:0")
        for _ in range(48):
            x.mul_(3).add_(1)
        out = torch.empty(olen + 64, dtype=torch.uint8, device="cuda:0")
        key.seal_blobs(x.data_ptr(), make_refs(offs, lens, oo, nonce * 2), out.data_ptr(), 0)
        got = out[:int(oo[0]) + lens[0] + 32].cpu().numpy().tobytes()
        assert got == oracle_mod.seal(key._key, nonce, want[:lens[0]].tobytes()), trial
        # zstd frames of the same bytes, again straight after the producer
        x2 = torch.from_numpy(base).to("cuda:0")
        for _ in range(48):
            x2.mul_(3).add_(1)
        f_offs, ftot = frame_layout([4 * MiB])
        fr = torch.empty(ftot + 16, dtype=torch.uint8, device="cuda:0")
        fl = compress_blobs(gpu_ctx, x2.data_ptr(), zrefs([8 * MiB], [4 * MiB], f_offs),
                            fr.data_ptr(), 0, 0)
        frame = fr[:int(fl[0])].cpu().numpy().tobytes()
        assert zstd_ref.decompress(frame) == want[8 * MiB:12 * MiB].tobytes()
