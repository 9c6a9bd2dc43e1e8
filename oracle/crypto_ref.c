/*
 * crypto_ref.c -- CPU ORACLE for the blob encryption stage (test
 * infrastructure only, like cdc_ref.c; see cdc_ref.h's header).
 *
 * Restates rustic's `Key::encrypt_data` / `decrypt_data`
 * (crates/core/src/crypto/aespoly1305.rs:88-135), which call the crates.io
 * dependency aes256ctr_poly1305aes 0.2.1 (crates/core/Cargo.toml:58,
 * /root/reference/Cargo.lock:33-36; NOT vendored, restated from its
 * published algorithm, the restic repository format):
 *   key (64 B)  = AES-256 key (32) || Poly1305-AES k (16) || r (16)
 *   output      = nonce (16) || AES-256-CTR(key, IV = nonce)(data) || tag (16)
 *   CTR         = the nonce as one 128-bit big-endian counter, +1 per block
 *   tag         = Poly1305-AES_{k,r}(nonce, ciphertext) with empty AAD:
 *                 (poly1305_r(ciphertext) + AES-128_k(nonce)) mod 2^128,
 *                 r clamped as in Poly1305
 * Pinned by tests/test_crypto_oracle.py: FIPS-197 AES vectors, the RFC 8439
 * Poly1305 vector, and the reference's own encrypted fixtures (key files +
 * config under crates/core/tests/fixtures, pack blobs of its repo tarballs).
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>

/* ------------------------------------------------------------ AES (FIPS-197) */
static const uint8_t SBOX[256] = {
    0x63,0x7c,0x77,0x7b,0xf2,0x6b,0x6f,0xc5,0x30,0x01,0x67,0x2b,0xfe,0xd7,0xab,0x76,
    0xca,0x82,0xc9,0x7d,0xfa,0x59,0x47,0xf0,0xad,0xd4,0xa2,0xaf,0x9c,0xa4,0x72,0xc0,
    0xb7,0xfd,0x93,0x26,0x36,0x3f,0xf7,0xcc,0x34,0xa5,0xe5,0xf1,0x71,0xd8,0x31,0x15,
    0x04,0xc7,0x23,0xc3,0x18,0x96,0x05,0x9a,0x07,0x12,0x80,0xe2,0xeb,0x27,0xb2,0x75,
    0x09,0x83,0x2c,0x1a,0x1b,0x6e,0x5a,0xa0,0x52,0x3b,0xd6,0xb3,0x29,0xe3,0x2f,0x84,
    0x53,0xd1,0x00,0xed,0x20,0xfc,0xb1,0x5b,0x6a,0xcb,0xbe,0x39,0x4a,0x4c,0x58,0xcf,
    0xd0,0xef,0xaa,0xfb,0x43,0x4d,0x33,0x85,0x45,0xf9,0x02,0x7f,0x50,0x3c,0x9f,0xa8,
    0x51,0xa3,0x40,0x8f,0x92,0x9d,0x38,0xf5,0xbc,0xb6,0xda,0x21,0x10,0xff,0xf3,0xd2,
    0xcd,0x0c,0x13,0xec,0x5f,0x97,0x44,0x17,0xc4,0xa7,0x7e,0x3d,0x64,0x5d,0x19,0x73,
    0x60,0x81,0x4f,0xdc,0x22,0x2a,0x90,0x88,0x46,0xee,0xb8,0x14,0xde,0x5e,0x0b,0xdb,
    0xe0,0x32,0x3a,0x0a,0x49,0x06,0x24,0x5c,0xc2,0xd3,0xac,0x62,0x91,0x95,0xe4,0x79,
    0xe7,0xc8,0x37,0x6d,0x8d,0xd5,0x4e,0xa9,0x6c,0x56,0xf4,0xea,0x65,0x7a,0xae,0x08,
    0xba,0x78,0x25,0x2e,0x1c,0xa6,0xb4,0xc6,0xe8,0xdd,0x74,0x1f,0x4b,0xbd,0x8b,0x8a,
    0x70,0x3e,0xb5,0x66,0x48,0x03,0xf6,0x0e,0x61,0x35,0x57,0xb9,0x86,0xc1,0x1d,0x9e,
    0xe1,0xf8,0x98,0x11,0x69,0xd9,0x8e,0x94,0x9b,0x1e,0x87,0xe9,0xce,0x55,0x28,0xdf,
    0x8c,0xa1,0x89,0x0d,0xbf,0xe6,0x42,0x68,0x41,0x99,0x2d,0x0f,0xb0,0x54,0xbb,0x16};

static uint8_t xtime(uint8_t x) { return (uint8_t)((x << 1) ^ ((x >> 7) * 0x1b)); }

/* Key expansion: nk = 4 (AES-128) or 8 (AES-256); rk gets 4 * (nr + 1) words
 * (big-endian column words, FIPS-197 5.2). Returns the round count. */
int crypto_ref_aes_expand(const uint8_t *key, int nk, uint32_t *rk) {
    const int nr = nk + 6;
    uint8_t rcon = 1;
    for (int i = 0; i < nk; i++)
        rk[i] = (uint32_t)key[4 * i] << 24 | (uint32_t)key[4 * i + 1] << 16 |
                (uint32_t)key[4 * i + 2] << 8 | key[4 * i + 3];
    for (int i = nk; i < 4 * (nr + 1); i++) {
        uint32_t t = rk[i - 1];
        if (i % nk == 0) {
            t = (t << 8) | (t >> 24);
            t = (uint32_t)SBOX[t >> 24] << 24 | (uint32_t)SBOX[(t >> 16) & 255] << 16 |
                (uint32_t)SBOX[(t >> 8) & 255] << 8 | SBOX[t & 255];
            t ^= (uint32_t)rcon << 24;
            rcon = xtime(rcon);
        } else if (nk > 6 && i % nk == 4) {
            t = (uint32_t)SBOX[t >> 24] << 24 | (uint32_t)SBOX[(t >> 16) & 255] << 16 |
                (uint32_t)SBOX[(t >> 8) & 255] << 8 | SBOX[t & 255];
        }
        rk[i] = rk[i - nk] ^ t;
    }
    return nr;
}

/* One block, byte-oriented (FIPS-197 5.1: SubBytes, ShiftRows, MixColumns). */
void crypto_ref_aes_encrypt(const uint32_t *rk, int nr, const uint8_t in[16], uint8_t out[16]) {
    uint8_t s[16];
    for (int c = 0; c < 4; c++)
        for (int r = 0; r < 4; r++) s[4 * c + r] = in[4 * c + r] ^ (uint8_t)(rk[c] >> (24 - 8 * r));
    for (int round = 1; round <= nr; round++) {
        uint8_t t[16];
        for (int c = 0; c < 4; c++)
            for (int r = 0; r < 4; r++) t[4 * c + r] = SBOX[s[4 * ((c + r) % 4) + r]];
        if (round != nr) {
            for (int c = 0; c < 4; c++) {
                uint8_t *a = t + 4 * c, a0 = a[0], a1 = a[1], a2 = a[2], a3 = a[3];
                uint8_t x = a0 ^ a1 ^ a2 ^ a3;
                a[0] ^= x ^ xtime(a0 ^ a1);
                a[1] ^= x ^ xtime(a1 ^ a2);
                a[2] ^= x ^ xtime(a2 ^ a3);
                a[3] ^= x ^ xtime(a3 ^ a0);
            }
        }
        for (int c = 0; c < 4; c++)
            for (int r = 0; r < 4; r++)
                s[4 * c + r] = t[4 * c + r] ^ (uint8_t)(rk[4 * round + c] >> (24 - 8 * r));
    }
    memcpy(out, s, 16);
}

/* AES-256-CTR, the 16-byte IV a big-endian 128-bit counter. */
void crypto_ref_aes256_ctr(const uint8_t key[32], const uint8_t iv[16], const uint8_t *in,
                           uint8_t *out, size_t n) {
    uint32_t rk[60];
    const int nr = crypto_ref_aes_expand(key, 8, rk);
    uint8_t ctr[16], ks[16];
    memcpy(ctr, iv, 16);
    for (size_t o = 0; o < n; o += 16) {
        crypto_ref_aes_encrypt(rk, nr, ctr, ks);
        const size_t k = n - o < 16 ? n - o : 16;
        for (size_t i = 0; i < k; i++) out[o + i] = in[o + i] ^ ks[i];
        for (int i = 15; i >= 0; i--)
            if (++ctr[i]) break;
    }
}

/* ------------------------------------------------ Poly1305 (RFC 8439 2.5) */
typedef unsigned __int128 u128;

/* poly1305 with r (clamped here) and s, over msg: tag = (poly + s) mod 2^128 */
void crypto_ref_poly1305(const uint8_t r_in[16], const uint8_t s_in[16], const uint8_t *msg,
                         size_t n, uint8_t tag[16]) {
    uint8_t rb[16];
    memcpy(rb, r_in, 16);
    rb[3] &= 15; rb[7] &= 15; rb[11] &= 15; rb[15] &= 15;
    rb[4] &= 252; rb[8] &= 252; rb[12] &= 252;
    /* 26-bit limbs */
    uint64_t r0, r1, r2, r3, r4;
    uint64_t t0 = 0, t1 = 0;
    for (int i = 7; i >= 0; i--) { t0 = t0 << 8 | rb[i]; t1 = t1 << 8 | rb[8 + i]; }
    r0 = t0 & 0x3ffffff;
    r1 = (t0 >> 26) & 0x3ffffff;
    r2 = ((t0 >> 52) | (t1 << 12)) & 0x3ffffff;
    r3 = (t1 >> 14) & 0x3ffffff;
    r4 = (t1 >> 40) & 0x3ffffff;
    uint64_t h0 = 0, h1 = 0, h2 = 0, h3 = 0, h4 = 0;
    for (size_t o = 0; o < n; o += 16) {
        uint8_t blk[17] = {0};
        const size_t k = n - o < 16 ? n - o : 16;
        memcpy(blk, msg + o, k);
        blk[k] = 1; /* the 2^(8k) bit */
        uint64_t m0 = 0, m1 = 0;
        for (int i = 7; i >= 0; i--) { m0 = m0 << 8 | blk[i]; m1 = m1 << 8 | blk[8 + i]; }
        const uint64_t hi = blk[16];
        h0 += m0 & 0x3ffffff;
        h1 += (m0 >> 26) & 0x3ffffff;
        h2 += ((m0 >> 52) | (m1 << 12)) & 0x3ffffff;
        h3 += (m1 >> 14) & 0x3ffffff;
        h4 += (m1 >> 40) | (hi << 24);
        const uint64_t s1 = r1 * 5, s2 = r2 * 5, s3 = r3 * 5, s4 = r4 * 5;
        u128 d0 = (u128)h0 * r0 + (u128)h1 * s4 + (u128)h2 * s3 + (u128)h3 * s2 + (u128)h4 * s1;
        u128 d1 = (u128)h0 * r1 + (u128)h1 * r0 + (u128)h2 * s4 + (u128)h3 * s3 + (u128)h4 * s2;
        u128 d2 = (u128)h0 * r2 + (u128)h1 * r1 + (u128)h2 * r0 + (u128)h3 * s4 + (u128)h4 * s3;
        u128 d3 = (u128)h0 * r3 + (u128)h1 * r2 + (u128)h2 * r1 + (u128)h3 * r0 + (u128)h4 * s4;
        u128 d4 = (u128)h0 * r4 + (u128)h1 * r3 + (u128)h2 * r2 + (u128)h3 * r1 + (u128)h4 * r0;
        uint64_t c;
        c = (uint64_t)(d0 >> 26); h0 = (uint64_t)d0 & 0x3ffffff; d1 += c;
        c = (uint64_t)(d1 >> 26); h1 = (uint64_t)d1 & 0x3ffffff; d2 += c;
        c = (uint64_t)(d2 >> 26); h2 = (uint64_t)d2 & 0x3ffffff; d3 += c;
        c = (uint64_t)(d3 >> 26); h3 = (uint64_t)d3 & 0x3ffffff; d4 += c;
        c = (uint64_t)(d4 >> 26); h4 = (uint64_t)d4 & 0x3ffffff; h0 += c * 5;
        c = h0 >> 26; h0 &= 0x3ffffff; h1 += c;
    }
    /* full carry, then h mod p, then + s */
    uint64_t c;
    c = h1 >> 26; h1 &= 0x3ffffff; h2 += c;
    c = h2 >> 26; h2 &= 0x3ffffff; h3 += c;
    c = h3 >> 26; h3 &= 0x3ffffff; h4 += c;
    c = h4 >> 26; h4 &= 0x3ffffff; h0 += c * 5;
    c = h0 >> 26; h0 &= 0x3ffffff; h1 += c;
    uint64_t g0 = h0 + 5; c = g0 >> 26; g0 &= 0x3ffffff;
    uint64_t g1 = h1 + c; c = g1 >> 26; g1 &= 0x3ffffff;
    uint64_t g2 = h2 + c; c = g2 >> 26; g2 &= 0x3ffffff;
    uint64_t g3 = h3 + c; c = g3 >> 26; g3 &= 0x3ffffff;
    uint64_t g4 = h4 + c - (1ull << 26);
    if (!(g4 >> 63)) { h0 = g0; h1 = g1; h2 = g2; h3 = g3; h4 = g4; }
    const uint64_t lo = h0 | h1 << 26 | h2 << 52, hi = (h2 >> 12) | h3 << 14 | h4 << 40;
    uint64_t s0 = 0, s1 = 0;
    for (int i = 7; i >= 0; i--) { s0 = s0 << 8 | s_in[i]; s1 = s1 << 8 | s_in[8 + i]; }
    const u128 t = ((u128)hi << 64 | lo) + ((u128)s1 << 64 | s0);
    for (int i = 0; i < 16; i++) tag[i] = (uint8_t)(t >> (8 * i));
}

/* Poly1305-AES_{k,r}(nonce, msg): s = AES-128_k(nonce). */
void crypto_ref_poly1305_aes(const uint8_t k[16], const uint8_t r[16], const uint8_t nonce[16],
                             const uint8_t *msg, size_t n, uint8_t tag[16]) {
    uint32_t rk[44];
    const int nr = crypto_ref_aes_expand(k, 4, rk);
    uint8_t s[16];
    crypto_ref_aes_encrypt(rk, nr, nonce, s);
    crypto_ref_poly1305(r, s, msg, n, tag);
}

/* rustic Key::encrypt_data with a given nonce (aespoly1305.rs:119-135):
 * out (n + 32 bytes) = nonce || ciphertext || tag. */
void crypto_ref_seal(const uint8_t key[64], const uint8_t nonce[16], const uint8_t *data,
                     size_t n, uint8_t *out) {
    memcpy(out, nonce, 16);
    crypto_ref_aes256_ctr(key, nonce, data, out + 16, n);
    crypto_ref_poly1305_aes(key + 32, key + 48, nonce, out + 16, n, out + 16 + n);
}

/* rustic Key::decrypt_data (aespoly1305.rs:88-110): in = nonce || ct || tag
 * (n >= 32 bytes); plaintext (n - 32 bytes) to out.  0 ok, 1 MAC mismatch,
 * 2 too short. */
int crypto_ref_open(const uint8_t key[64], const uint8_t *in, size_t n, uint8_t *out) {
    if (n < 32) return 2;
    uint8_t tag[16];
    crypto_ref_poly1305_aes(key + 32, key + 48, in, in + 16, n - 32, tag);
    uint8_t d = 0;
    for (int i = 0; i < 16; i++) d |= tag[i] ^ in[n - 16 + i];
    if (d) return 1;
    crypto_ref_aes256_ctr(key, in, in + 16, out, n - 32);
    return 0;
}
