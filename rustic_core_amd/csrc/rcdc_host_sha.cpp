// rcdc_host_sha.cpp -- SHA-256 of many host buffers at once (pack ids).
//
// The packer names each finished pack file by the SHA-256 of its bytes
// (crates/core/src/blob/packer.rs:832-834, `hash_reader`).  A pack is one
// Merkle-Damgard chain of ~40 MB, too long for a device lane (~2 us per
// 64-byte block), so HostIngest hashes the packs on host threads as they come
// back over PCIe.  One core with the SHA extensions (OpenSSL) does ~2.4 GB/s;
// this file hashes 16 packs side by side in the 16 32-bit lanes of AVX-512
// registers (multi-buffer SHA-256, FIPS 180-4 section 6.2): 16 chains per
// instruction stream, each block's rounds on ternary-logic Ch / Maj / xor3
// and native 32-bit rotates.  A lane that finishes its message takes the next
// one, so n messages of unequal lengths keep the lanes busy.  CPUs without
// AVX-512F/BW get RCDC_ERR_UNSUPPORTED (callers then use hashlib).  Host
// code only: built with the host compiler (Makefile), no device pass.
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include <immintrin.h>

namespace {

alignas(64) const uint32_t kK256[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u,
    0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu,
    0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu,
    0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, 0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u,
    0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu,
    0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu,
    0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u, 0x19a4c116u,
    0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u,
    0xc67178f2u};
const uint32_t kH0[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                         0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

#define RCDC_AVX512 __attribute__((target("avx512f,avx512bw")))

// ternary-logic truth tables over (A, B, C)
constexpr int kXor3 = 0x96, kCh = 0xCA, kMaj = 0xE8;

RCDC_AVX512 inline __m512i xor3(__m512i a, __m512i b, __m512i c) {
    return _mm512_ternarylogic_epi32(a, b, c, kXor3);
}
RCDC_AVX512 inline __m512i bsig0(__m512i x) {
    return xor3(_mm512_ror_epi32(x, 2), _mm512_ror_epi32(x, 13), _mm512_ror_epi32(x, 22));
}
RCDC_AVX512 inline __m512i bsig1(__m512i x) {
    return xor3(_mm512_ror_epi32(x, 6), _mm512_ror_epi32(x, 11), _mm512_ror_epi32(x, 25));
}
RCDC_AVX512 inline __m512i ssig0(__m512i x) {
    return xor3(_mm512_ror_epi32(x, 7), _mm512_ror_epi32(x, 18), _mm512_srli_epi32(x, 3));
}
RCDC_AVX512 inline __m512i ssig1(__m512i x) {
    return xor3(_mm512_ror_epi32(x, 17), _mm512_ror_epi32(x, 19), _mm512_srli_epi32(x, 10));
}

// 16 x 16 transpose of 32-bit words in registers: r[i] = row i -> r[c] =
// column c.  Unpacks of 32 then 64 bits give, in each 128-bit lane k of
// u[4g + j], column 4k + j of rows 4g .. 4g + 3; two 128-bit shuffles then
// gather the four row groups of a column.
RCDC_AVX512 inline void transpose16(__m512i r[16]) {
    __m512i t[16], u[16];
    for (int i = 0; i < 8; i++) {
        t[2 * i] = _mm512_unpacklo_epi32(r[2 * i], r[2 * i + 1]);
        t[2 * i + 1] = _mm512_unpackhi_epi32(r[2 * i], r[2 * i + 1]);
    }
    for (int g = 0; g < 4; g++) {
        u[4 * g] = _mm512_unpacklo_epi64(t[4 * g], t[4 * g + 2]);
        u[4 * g + 1] = _mm512_unpackhi_epi64(t[4 * g], t[4 * g + 2]);
        u[4 * g + 2] = _mm512_unpacklo_epi64(t[4 * g + 1], t[4 * g + 3]);
        u[4 * g + 3] = _mm512_unpackhi_epi64(t[4 * g + 1], t[4 * g + 3]);
    }
    for (int j = 0; j < 4; j++) {
        const __m512i x0 = _mm512_shuffle_i32x4(u[j], u[4 + j], 0x44);
        const __m512i x1 = _mm512_shuffle_i32x4(u[j], u[4 + j], 0xEE);
        const __m512i y0 = _mm512_shuffle_i32x4(u[8 + j], u[12 + j], 0x44);
        const __m512i y1 = _mm512_shuffle_i32x4(u[8 + j], u[12 + j], 0xEE);
        r[j] = _mm512_shuffle_i32x4(x0, y0, 0x88);
        r[4 + j] = _mm512_shuffle_i32x4(x0, y0, 0xDD);
        r[8 + j] = _mm512_shuffle_i32x4(x1, y1, 0x88);
        r[12 + j] = _mm512_shuffle_i32x4(x1, y1, 0xDD);
    }
}

struct Lane {
    const uint8_t *data;  // the message
    uint64_t nfull;       // its full 64-byte blocks
    uint64_t blk;         // next block
    uint64_t nblk;        // all blocks, padding included
    uint8_t tail[128];    // the padded last one or two blocks
    int32_t msg;          // message index, -1: idle
};

}  // namespace

namespace rcdc {

// Multi-buffer core: n messages, digests 32 bytes each.
RCDC_AVX512 static void sha256_many_avx512(const uint8_t *const *ptrs, const uint64_t *lens,
                                           uint32_t n, uint8_t *digests) {
    Lane L[16];
    uint32_t next = 0;
    auto start = [&](Lane &l) {
        if (next >= n) {
            l.msg = -1;
            return;
        }
        const uint32_t m = next++;
        const uint64_t len = lens[m];
        l.msg = (int32_t)m;
        l.data = ptrs[m];
        l.nfull = len / 64;
        l.blk = 0;
        const uint32_t rem = (uint32_t)(len % 64);
        std::memset(l.tail, 0, sizeof(l.tail));
        if (rem) std::memcpy(l.tail, ptrs[m] + l.nfull * 64, rem);
        l.tail[rem] = 0x80;
        const uint32_t tb = rem + 9 > 64 ? 2 : 1;
        const uint64_t bits = len * 8;
        for (int k = 0; k < 8; k++) l.tail[tb * 64 - 1 - k] = (uint8_t)(bits >> (8 * k));
        l.nblk = l.nfull + tb;
    };
    alignas(64) uint32_t st[8][16];
    for (int i = 0; i < 16; i++) {
        start(L[i]);
        for (int w = 0; w < 8; w++) st[w][i] = kH0[w];
    }
    const __m512i bswap = _mm512_set4_epi32(0x0c0d0e0f, 0x08090a0b, 0x04050607, 0x00010203);
    alignas(64) static const uint8_t zero_block[64] = {0};
    for (;;) {
        uint32_t active = 0;
        for (int i = 0; i < 16; i++)
            if (L[i].msg >= 0) active |= 1u << i;
        if (!active) break;
        // this round's block of every lane, words transposed into W[0..15]
        __m512i W[16];
        for (int i = 0; i < 16; i++) {
            const Lane &l = L[i];
            const uint8_t *p = l.msg < 0 ? zero_block
                               : l.blk < l.nfull ? l.data + l.blk * 64
                                                 : l.tail + (l.blk - l.nfull) * 64;
            W[i] = _mm512_loadu_si512((const void *)p);
        }
        transpose16(W);  // W[i] = block of lane i -> W[w] = word w of every lane
        for (int w = 0; w < 16; w++) W[w] = _mm512_shuffle_epi8(W[w], bswap);
        __m512i a = _mm512_load_si512(st[0]), b = _mm512_load_si512(st[1]);
        __m512i c = _mm512_load_si512(st[2]), d = _mm512_load_si512(st[3]);
        __m512i e = _mm512_load_si512(st[4]), f = _mm512_load_si512(st[5]);
        __m512i g = _mm512_load_si512(st[6]), h = _mm512_load_si512(st[7]);
        const __m512i a0 = a, b0 = b, c0 = c, d0 = d, e0 = e, f0 = f, g0 = g, h0 = h;
#pragma GCC unroll 64
        for (int t = 0; t < 64; t++) {
            if (t >= 16)
                W[t & 15] = _mm512_add_epi32(
                    _mm512_add_epi32(ssig1(W[(t - 2) & 15]), W[(t - 7) & 15]),
                    _mm512_add_epi32(ssig0(W[(t - 15) & 15]), W[t & 15]));
            const __m512i t1 = _mm512_add_epi32(
                _mm512_add_epi32(h, bsig1(e)),
                _mm512_add_epi32(_mm512_ternarylogic_epi32(e, f, g, kCh),
                                 _mm512_add_epi32(_mm512_set1_epi32((int)kK256[t]), W[t & 15])));
            const __m512i t2 = _mm512_add_epi32(bsig0(a), _mm512_ternarylogic_epi32(a, b, c, kMaj));
            h = g;
            g = f;
            f = e;
            e = _mm512_add_epi32(d, t1);
            d = c;
            c = b;
            b = a;
            a = _mm512_add_epi32(t1, t2);
        }
        const __mmask16 m = (__mmask16)active;
        _mm512_store_si512(st[0], _mm512_mask_add_epi32(a0, m, a0, a));
        _mm512_store_si512(st[1], _mm512_mask_add_epi32(b0, m, b0, b));
        _mm512_store_si512(st[2], _mm512_mask_add_epi32(c0, m, c0, c));
        _mm512_store_si512(st[3], _mm512_mask_add_epi32(d0, m, d0, d));
        _mm512_store_si512(st[4], _mm512_mask_add_epi32(e0, m, e0, e));
        _mm512_store_si512(st[5], _mm512_mask_add_epi32(f0, m, f0, f));
        _mm512_store_si512(st[6], _mm512_mask_add_epi32(g0, m, g0, g));
        _mm512_store_si512(st[7], _mm512_mask_add_epi32(h0, m, h0, h));
        for (int i = 0; i < 16; i++) {
            Lane &l = L[i];
            if (l.msg < 0) continue;
            if (++l.blk < l.nblk) continue;
            uint8_t *out = digests + (uint64_t)l.msg * 32;
            for (int w = 0; w < 8; w++) {
                const uint32_t v = st[w][i];
                out[4 * w] = (uint8_t)(v >> 24);
                out[4 * w + 1] = (uint8_t)(v >> 16);
                out[4 * w + 2] = (uint8_t)(v >> 8);
                out[4 * w + 3] = (uint8_t)v;
                st[w][i] = kH0[w];
            }
            start(l);
        }
    }
}

// ---- one message on the SHA extensions (SHA-NI): the pack ids whose
// latency matters (the last packs of a backup), ~2 GB/s on one core.  The
// state lives as ABEF / CDGH pairs (sha256rnds2's operand order); each
// 4-round group adds 4 round constants to 4 schedule words (msg1 / msg2 build
// W[t] for t >= 16 from the previous four groups, FIPS 180-4 6.2.2 step 1).
#define RCDC_SHANI __attribute__((target("sha,sse4.1,ssse3")))

// K messages interleaved on one core: sha256rnds2 is a long-latency
// instruction and one message's rounds form a single dependency chain, so
// one stream of them leaves the unit idle most cycles.  K independent chains
// fill those cycles: more bytes per second per core at the same latency per
// message (the tail of a backup, where the last packs' ids are on the
// critical path and every thread is busy).
template <int K>
RCDC_SHANI void sha256_ni_blocks_k(uint32_t *const *st, const uint8_t *const *pp, uint64_t nblk) {
    const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
    __m128i s0[K], s1[K];
    const uint8_t *p[K];
#pragma GCC unroll 4
    for (int k = 0; k < K; k++) {
        const __m128i t = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i *)&st[k][0]), 0xB1);  // CDAB
        const __m128i u = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i *)&st[k][4]), 0x1B);  // EFGH
        s0[k] = _mm_alignr_epi8(t, u, 8);      // ABEF
        s1[k] = _mm_blend_epi16(u, t, 0xF0);   // CDGH
        p[k] = pp[k];
    }
    for (; nblk; nblk--) {
        __m128i a0[K], c0[K], w[K][4];
#pragma GCC unroll 4
        for (int k = 0; k < K; k++) {
            a0[k] = s0[k];
            c0[k] = s1[k];
        }
#pragma GCC unroll 16
        for (int j = 0; j < 16; j++) {
            const __m128i kk = _mm_load_si128((const __m128i *)&kK256[4 * j]);
#pragma GCC unroll 4
            for (int k = 0; k < K; k++) {
                if (j < 4)
                    w[k][j] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i *)(p[k] + 16 * j)), bswap);
                else
                    w[k][j & 3] = _mm_sha256msg2_epu32(
                        _mm_add_epi32(_mm_sha256msg1_epu32(w[k][j & 3], w[k][(j - 3) & 3]),
                                      _mm_alignr_epi8(w[k][(j - 1) & 3], w[k][(j - 2) & 3], 4)),
                        w[k][(j - 1) & 3]);
                __m128i m = _mm_add_epi32(w[k][j & 3], kk);
                s1[k] = _mm_sha256rnds2_epu32(s1[k], s0[k], m);
                m = _mm_shuffle_epi32(m, 0x0E);
                s0[k] = _mm_sha256rnds2_epu32(s0[k], s1[k], m);
            }
        }
#pragma GCC unroll 4
        for (int k = 0; k < K; k++) {
            s0[k] = _mm_add_epi32(s0[k], a0[k]);
            s1[k] = _mm_add_epi32(s1[k], c0[k]);
            p[k] += 64;
        }
    }
#pragma GCC unroll 4
    for (int k = 0; k < K; k++) {
        const __m128i t = _mm_shuffle_epi32(s0[k], 0x1B);  // FEBA
        const __m128i u = _mm_shuffle_epi32(s1[k], 0xB1);  // DCHG
        _mm_storeu_si128((__m128i *)&st[k][0], _mm_blend_epi16(t, u, 0xF0));  // DCBA
        _mm_storeu_si128((__m128i *)&st[k][4], _mm_alignr_epi8(u, t, 8));     // HGFE
    }
}

RCDC_SHANI void sha256_ni_blocks(uint32_t st[8], const uint8_t *p, uint64_t nblk) {
    uint32_t *s[1] = {st};
    const uint8_t *q[1] = {p};
    sha256_ni_blocks_k<1>(s, q, nblk);
}

// Portable fallback (no SHA extensions): FIPS 180-4 rounds, one block.
void sha256_scalar_blocks(uint32_t st[8], const uint8_t *p, uint64_t nblk) {
    auto rotr = [](uint32_t x, int n) { return (x >> n) | (x << (32 - n)); };
    for (; nblk; nblk--, p += 64) {
        uint32_t w[64];
        for (int t = 0; t < 16; t++)
            w[t] = (uint32_t)p[4 * t] << 24 | (uint32_t)p[4 * t + 1] << 16 |
                   (uint32_t)p[4 * t + 2] << 8 | p[4 * t + 3];
        for (int t = 16; t < 64; t++) {
            const uint32_t s0 = rotr(w[t - 15], 7) ^ rotr(w[t - 15], 18) ^ (w[t - 15] >> 3);
            const uint32_t s1 = rotr(w[t - 2], 17) ^ rotr(w[t - 2], 19) ^ (w[t - 2] >> 10);
            w[t] = w[t - 16] + s0 + w[t - 7] + s1;
        }
        uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6],
                 h = st[7];
        for (int t = 0; t < 64; t++) {
            const uint32_t t1 = h + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) +
                                ((e & f) ^ (~e & g)) + kK256[t] + w[t];
            const uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
            h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
        }
        st[0] += a; st[1] += b; st[2] += c; st[3] += d;
        st[4] += e; st[5] += f; st[6] += g; st[7] += h;
    }
}

bool host_sha_ni() {
    static const bool ok = [] {
        if (getenv("RCDC_NO_SHANI")) return false;  // tests: the scalar rounds
        __builtin_cpu_init();
        unsigned a, b, c, d;
        // CPUID leaf 7: EBX bit 29 = SHA
        __asm__ volatile("cpuid" : "=a"(a), "=b"(b), "=c"(c), "=d"(d) : "a"(7), "c"(0));
        return ((b >> 29) & 1u) && __builtin_cpu_supports("sse4.1");
    }();
    return ok;
}

bool host_sha_supported() {
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw");
}

void host_sha256_many(const uint8_t *const *ptrs, const uint64_t *lens, uint32_t n,
                      uint8_t *digests) {
    sha256_many_avx512(ptrs, lens, n, digests);
}

// SHA-256 of one host message (SHA-NI when present, else the scalar rounds).
void host_sha256_one(const uint8_t *p, uint64_t len, uint8_t out[32]) {
    uint32_t st[8];
    memcpy(st, kH0, sizeof st);
    void (*blocks)(uint32_t *, const uint8_t *, uint64_t) =
        host_sha_ni() ? sha256_ni_blocks : sha256_scalar_blocks;
    const uint64_t full = len / 64;
    blocks(st, p, full);
    uint8_t tail[128] = {0};
    const uint64_t r = len - full * 64;
    memcpy(tail, p + full * 64, r);
    tail[r] = 0x80;
    const uint64_t nt = r + 9 <= 64 ? 1 : 2;
    const uint64_t bits = len * 8;
    for (int i = 0; i < 8; i++) tail[nt * 64 - 1 - i] = (uint8_t)(bits >> (8 * i));
    blocks(st, tail, nt);
    for (int w = 0; w < 8; w++) {
        out[4 * w] = (uint8_t)(st[w] >> 24);
        out[4 * w + 1] = (uint8_t)(st[w] >> 16);
        out[4 * w + 2] = (uint8_t)(st[w] >> 8);
        out[4 * w + 3] = (uint8_t)st[w];
    }
}


// The SHA-256 of n host messages on the SHA extensions, up to `ways` (1-4)
// interleaved on this thread: the blocks all messages of a group share run
// together, then each message's remaining blocks and padding alone.  Without
// SHA-NI: one message at a time.
void host_sha256_ni_many(const uint8_t *const *ptrs, const uint64_t *lens, uint32_t n,
                         uint8_t *digests, int ways) {
    ways = ways < 1 ? 1 : ways > 4 ? 4 : ways;
    if (!host_sha_ni()) ways = 1;
    for (uint32_t a = 0; a < n; a += (uint32_t)ways) {
        const int k = (int)(n - a < (uint32_t)ways ? n - a : (uint32_t)ways);
        if (k == 1) {
            host_sha256_one(ptrs[a], lens[a], digests + 32ull * a);
            continue;
        }
        uint32_t st[4][8];
        uint32_t *sp[4];
        const uint8_t *pp[4];
        uint64_t common = ~0ull;
        for (int i = 0; i < k; i++) {
            memcpy(st[i], kH0, sizeof st[i]);
            sp[i] = st[i];
            pp[i] = ptrs[a + i];
            common = lens[a + i] / 64 < common ? lens[a + i] / 64 : common;
        }
        if (k == 2) sha256_ni_blocks_k<2>(sp, pp, common);
        else if (k == 3) sha256_ni_blocks_k<3>(sp, pp, common);
        else sha256_ni_blocks_k<4>(sp, pp, common);
        for (int i = 0; i < k; i++) {
            const uint8_t *p = ptrs[a + i];
            const uint64_t len = lens[a + i], full = len / 64;
            sha256_ni_blocks(st[i], p + common * 64, full - common);
            uint8_t tail[128] = {0};
            const uint64_t r = len - full * 64;
            memcpy(tail, p + full * 64, r);
            tail[r] = 0x80;
            const uint64_t nt = r + 9 <= 64 ? 1 : 2;
            const uint64_t bits = len * 8;
            for (int b = 0; b < 8; b++) tail[nt * 64 - 1 - b] = (uint8_t)(bits >> (8 * b));
            sha256_ni_blocks(st[i], tail, nt);
            uint8_t *out = digests + 32ull * (a + i);
            for (int w = 0; w < 8; w++) {
                out[4 * w] = (uint8_t)(st[i][w] >> 24);
                out[4 * w + 1] = (uint8_t)(st[i][w] >> 16);
                out[4 * w + 2] = (uint8_t)(st[i][w] >> 8);
                out[4 * w + 3] = (uint8_t)st[i][w];
            }
        }
    }
}

}  // namespace rcdc
