// rcdc_aead.hip -- blob encryption on the device:
// rustic's Key::encrypt_data / decrypt_data (crates/core/src/crypto/
// aespoly1305.rs:88-135, aes256ctr_poly1305aes 0.2.1: the restic format),
// applied to chunks already in HBM (the packer's process_data,
// blob/packer.rs:268-270, decrypt.rs:566-572).
//
//   sealed blob = nonce (16) || AES-256-CTR_{K_enc, IV = nonce}(data) || tag (16)
//   tag         = (poly1305_r(ciphertext) + AES-128_{K_k}(nonce)) mod 2^128
//
// Work: a blob is cut into units of kAeadUnitBlocks 16-byte blocks; one wave
// per unit.  Lane l takes blocks l, l + 64, ... of the unit, two per step (two
// independent AES chains; the next step's data already loading): counter
// block = nonce + block index (128-bit big-endian), AES-256 by T-tables in
// LDS, keystream XOR data, and the ciphertext block goes into the lane's
// Poly1305 accumulator by Horner with R = r^64 (26-bit limbs).  The lanes
// combine with r^(unit end - lane's last block) and a wave reduction; the
// unit's partial is positioned with r^(blocks after the unit) (binary powers
// of r).  rcdc_aead_finish_kernel sums a blob's partials mod 2^130 - 5, adds
// AES-128_k(nonce) and writes (seal) or checks (open) the tag.  Poly1305 is
// linear in the message blocks, so this split is exact.
//
// Tables: T and its 3 byte rotations (no v_alignbit per lookup), 32 copies
// each (copy = lane & 31: ds_read_b32 banks are (a/4) mod 32 per 32-lane
// half, so every lookup is conflict-free), 128 KiB: one 1024-thread
// workgroup per CU.  A lookup address is ONE v_perm_b32 (tlu); a round is
// 16 v_perm + 16 ds_read_b32 + 8 v_bitop3 (3-input XOR, round key from an
// SGPR).  Measured (tools/aead_prof.py): ~725 GiB/s seal on
// 8 GiB of 0.5-8 MiB blobs; VALU and LDS each ~2/3 busy.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "rcdc_internal.h"

using namespace rcdc;

namespace rcdc {
// 16 waves, one workgroup per CU (the 128 KiB of tables): 4 waves per SIMD,
// up to 128 VGPRs
constexpr int kAeadThreads = 1024;
constexpr int kAeadBlocksPerCU = 1;
constexpr uint32_t kAeadTableWords = 2u * 256u * 64u;
}  // namespace rcdc

namespace {

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_amdgcn_perm(x, x, 0x00010203u); }
__device__ __forceinline__ uint32_t ror32(uint32_t x, int k) { return __builtin_amdgcn_alignbit(x, x, k); }

struct P26 {
    uint32_t h[5];
};

// a * b mod 2^130 - 5 (limbs of a below ~2^27, of b below 2^26; result limbs
// below 2^26 + a few).
__device__ __forceinline__ P26 pmul(const P26 &a, const uint32_t *b) {
    const uint64_t b0 = b[0], b1 = b[1], b2 = b[2], b3 = b[3], b4 = b[4];
    const uint64_t s1 = b1 * 5, s2 = b2 * 5, s3 = b3 * 5, s4 = b4 * 5;
    const uint64_t a0 = a.h[0], a1 = a.h[1], a2 = a.h[2], a3 = a.h[3], a4 = a.h[4];
    uint64_t d0 = a0 * b0 + a1 * s4 + a2 * s3 + a3 * s2 + a4 * s1;
    uint64_t d1 = a0 * b1 + a1 * b0 + a2 * s4 + a3 * s3 + a4 * s2;
    uint64_t d2 = a0 * b2 + a1 * b1 + a2 * b0 + a3 * s4 + a4 * s3;
    uint64_t d3 = a0 * b3 + a1 * b2 + a2 * b1 + a3 * b0 + a4 * s4;
    uint64_t d4 = a0 * b4 + a1 * b3 + a2 * b2 + a3 * b1 + a4 * b0;
    P26 r;
    d1 += d0 >> 26;
    r.h[0] = (uint32_t)d0 & 0x3ffffff;
    d2 += d1 >> 26;
    r.h[1] = (uint32_t)d1 & 0x3ffffff;
    d3 += d2 >> 26;
    r.h[2] = (uint32_t)d2 & 0x3ffffff;
    d4 += d3 >> 26;
    r.h[3] = (uint32_t)d3 & 0x3ffffff;
    const uint64_t c = d4 >> 26;
    r.h[4] = (uint32_t)d4 & 0x3ffffff;
    const uint64_t t0 = (uint64_t)r.h[0] + c * 5;
    r.h[0] = (uint32_t)t0 & 0x3ffffff;
    r.h[1] += (uint32_t)(t0 >> 26);
    return r;
}

__device__ __forceinline__ void pnorm(P26 &a) {
    uint32_t c;
    c = a.h[0] >> 26; a.h[0] &= 0x3ffffff; a.h[1] += c;
    c = a.h[1] >> 26; a.h[1] &= 0x3ffffff; a.h[2] += c;
    c = a.h[2] >> 26; a.h[2] &= 0x3ffffff; a.h[3] += c;
    c = a.h[3] >> 26; a.h[3] &= 0x3ffffff; a.h[4] += c;
    c = a.h[4] >> 26; a.h[4] &= 0x3ffffff; a.h[0] += c * 5;
    c = a.h[0] >> 26; a.h[0] &= 0x3ffffff; a.h[1] += c;
}

// The 16-byte message block w (4 little-endian words) plus 2^(8 k), k the
// block's byte count (16: the 2^128 bit).
__device__ __forceinline__ P26 pblock(const uint32_t w[4], uint32_t k) {
    uint32_t x[4] = {w[0], w[1], w[2], w[3]};
    uint32_t hib = 0;
    if (k < 16) {  // partial final block: bytes >= k are zero, then the 1 byte
        for (int i = 0; i < 4; i++) {
            const int lo = 4 * i;
            if ((int)k <= lo) x[i] = 0;
            else if ((int)k < lo + 4) x[i] &= (1u << (8 * (k - lo))) - 1u;
        }
        x[k >> 2] |= 1u << (8 * (k & 3));
    } else {
        hib = 1;
    }
    P26 m;
    m.h[0] = x[0] & 0x3ffffff;
    m.h[1] = ((x[0] >> 26) | (x[1] << 6)) & 0x3ffffff;
    m.h[2] = ((x[1] >> 20) | (x[2] << 12)) & 0x3ffffff;
    m.h[3] = ((x[2] >> 14) | (x[3] << 18)) & 0x3ffffff;
    m.h[4] = (x[3] >> 8) | (hib << 24);
    return m;
}

// a ^ b ^ c in one VALU op (gfx950 v_bitop3_b32, truth table 0x96)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// a ^ b ^ k, k a wave-uniform value held in an SGPR (the round key)
__device__ __forceinline__ uint32_t xor3k(uint32_t a, uint32_t b, uint32_t k) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(k));
    return r;
}

// Lookup of byte K of s in table j: LDS byte address
//   (j >> 1) << 16 | e << 8 | (j & 1) << 7 | c * 4      (e = the byte, c = lane & 31)
// i.e. byte 1 of the address is e and bytes 0, 2 come from the lane's
// constant Lj = the rest: ONE v_perm_b32 builds it.
template <int K>
__device__ __forceinline__ uint32_t tlu(const uint8_t *__restrict__ tt, uint32_t s, uint32_t Lj) {
    constexpr uint32_t sel = 0x0c020000u | ((4u + K) << 8);
    const uint32_t a = __builtin_amdgcn_perm(s, Lj, sel);
    return *reinterpret_cast<const uint32_t *>(tt + a);
}

// AES encryption of one block held as 4 big-endian column words; round keys
// uniform (rk: global, scalar loads), tables in LDS (see tlu; lane4 = L0).
template <int NR>
__device__ __forceinline__ void aes_block(uint32_t &s0, uint32_t &s1, uint32_t &s2, uint32_t &s3,
                                          const uint8_t *__restrict__ tt, uint32_t lane4,
                                          const uint32_t *__restrict__ rk) {
    s0 ^= rk[0]; s1 ^= rk[1]; s2 ^= rk[2]; s3 ^= rk[3];
    // table j = T rotated right by 8 j (no v_alignbit per lookup)
    const uint32_t L1 = lane4 + 128u, L2 = lane4 | 0x10000u, L3 = (lane4 + 128u) | 0x10000u;
#pragma unroll
    for (int r = 1; r < NR; r++) {
        const uint32_t t0 = xor3k(xor3(tlu<3>(tt, s0, lane4), tlu<2>(tt, s1, L1), tlu<1>(tt, s2, L2)),
                                  tlu<0>(tt, s3, L3), rk[4 * r]);
        const uint32_t t1 = xor3k(xor3(tlu<3>(tt, s1, lane4), tlu<2>(tt, s2, L1), tlu<1>(tt, s3, L2)),
                                  tlu<0>(tt, s0, L3), rk[4 * r + 1]);
        const uint32_t t2 = xor3k(xor3(tlu<3>(tt, s2, lane4), tlu<2>(tt, s3, L1), tlu<1>(tt, s0, L2)),
                                  tlu<0>(tt, s1, L3), rk[4 * r + 2]);
        const uint32_t t3 = xor3k(xor3(tlu<3>(tt, s3, lane4), tlu<2>(tt, s0, L1), tlu<1>(tt, s1, L2)),
                                  tlu<0>(tt, s2, L3), rk[4 * r + 3]);
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    // final round: SubBytes (S[x] = byte 2 of T[x]) + ShiftRows + AddRoundKey;
    // v_perm gathers byte 2 of four lookups into one word
    const uint32_t *k = rk + 4 * NR;
#define SBW(a, b, c, d)                                                                    \
    __builtin_amdgcn_perm(__builtin_amdgcn_perm(tlu<3>(tt, a, lane4), tlu<2>(tt, b, lane4), \
                                                0x0c0c0602u),                              \
                          __builtin_amdgcn_perm(tlu<1>(tt, c, lane4), tlu<0>(tt, d, lane4), \
                                                0x0c0c0602u),                              \
                          0x05040100u)
    const uint32_t t0 = SBW(s0, s1, s2, s3);
    const uint32_t t1 = SBW(s1, s2, s3, s0);
    const uint32_t t2 = SBW(s2, s3, s0, s1);
    const uint32_t t3 = SBW(s3, s0, s1, s2);
#undef SBW
    s0 = t0 ^ k[0]; s1 = t1 ^ k[1]; s2 = t2 ^ k[2]; s3 = t3 ^ k[3];
}

// Unaligned 16-byte load at byte address p (4 dwords + 1 from the 4-aligned
// base, funnel-shifted; reads at most 3 bytes past p + 16 inside the arena).
__device__ __forceinline__ void load16(const uint8_t *p, uint32_t w[4]) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint32_t *q = reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3) * 8;
    const uint32_t x0 = q[0], x1 = q[1], x2 = q[2], x3 = q[3];
    if (sh == 0) {
        w[0] = x0; w[1] = x1; w[2] = x2; w[3] = x3;
    } else {
        const uint32_t x4 = q[4];
        w[0] = __builtin_amdgcn_alignbit(x1, x0, sh);
        w[1] = __builtin_amdgcn_alignbit(x2, x1, sh);
        w[2] = __builtin_amdgcn_alignbit(x3, x2, sh);
        w[3] = __builtin_amdgcn_alignbit(x4, x3, sh);
    }
}

// 16 bytes (4 little-endian words) to any address: one dwordx4 when 16-B
// aligned, else the 3 whole dwords the block covers plus byte stores for the
// two partial ones (pack layouts put blobs at any offset).
__device__ __forceinline__ void store16(uint8_t *p, const uint32_t c[4]) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    if ((a & 15u) == 0) {
        *reinterpret_cast<uint4 *>(p) = make_uint4(c[0], c[1], c[2], c[3]);
        return;
    }
    const uint32_t m = (uint32_t)(a & 3u);
    if (m == 0) {
        uint32_t *q = reinterpret_cast<uint32_t *>(p);
        q[0] = c[0]; q[1] = c[1]; q[2] = c[2]; q[3] = c[3];
        return;
    }
    // bytes [m, m + 16) of the 5 dwords from the aligned base: dwords 1..3
    // whole (d_i = c[i-1] >> 8(4-m) | c[i] << 8m), dword 0 bytes m..3 and
    // dword 4 bytes 0..m-1 partial
    uint32_t *q = reinterpret_cast<uint32_t *>(p - m);
    const uint32_t sh = 8u * (4u - m);
    q[1] = __builtin_amdgcn_alignbit(c[1], c[0], sh);
    q[2] = __builtin_amdgcn_alignbit(c[2], c[1], sh);
    q[3] = __builtin_amdgcn_alignbit(c[3], c[2], sh);
    for (uint32_t i = 0; i < 4u - m; i++) p[i] = (uint8_t)(c[0] >> (8 * i));
    for (uint32_t i = 0; i < m; i++) p[12 + (4 - m) + i] = (uint8_t)(c[3] >> (8 * (4 - m + i)));
}

// Bytes [0, k) of a block of k < 16 bytes (no read past the data's end).
__device__ __forceinline__ void load_partial(const uint8_t *p, uint32_t k, uint32_t w[4]) {
    w[0] = w[1] = w[2] = w[3] = 0;
    for (uint32_t i = 0; i < k; i++) w[i >> 2] |= (uint32_t)p[i] << (8 * (i & 3));
}

// counter block nonce + b (128-bit big-endian) as big-endian column words
__device__ __forceinline__ void ctr_block(const uint32_t nle[4], uint64_t b, uint32_t &s0,
                                          uint32_t &s1, uint32_t &s2, uint32_t &s3) {
    const uint64_t hi = (uint64_t)bswap32(nle[0]) << 32 | bswap32(nle[1]);
    const uint64_t lo = (uint64_t)bswap32(nle[2]) << 32 | bswap32(nle[3]);
    const uint64_t l2 = lo + b;
    const uint64_t h2 = hi + (l2 < lo ? 1 : 0);
    s0 = (uint32_t)(h2 >> 32); s1 = (uint32_t)h2;
    s2 = (uint32_t)(l2 >> 32); s3 = (uint32_t)l2;
}

// The blob's nonce as 4 little-endian words: the caller's (seal) or the
// sealed blob's first 16 bytes (open, aespoly1305.rs:98-100).
template <bool OPEN>
__device__ __forceinline__ void blob_nonce(const uint8_t *in, const AeadBlob &B, uint32_t n[4]) {
    if (OPEN) {
        load16(in + B.in_off, n);
    } else {
        n[0] = B.nonce[0]; n[1] = B.nonce[1]; n[2] = B.nonce[2]; n[3] = B.nonce[3];
    }
}

// Carry-propagate and wrap until every limb is below 2^26 and the value is
// below 2^130 (limbs on entry below 2^31).
__device__ __forceinline__ void pfull(P26 &a) {
    for (int rep = 0; rep < 2; rep++) {
        for (int j = 0; j < 4; j++) {
            a.h[j + 1] += a.h[j] >> 26;
            a.h[j] &= 0x3ffffff;
        }
        const uint32_t c = a.h[4] >> 26;
        a.h[4] &= 0x3ffffff;
        a.h[0] += c * 5;
    }
    for (int j = 0; j < 4; j++) {
        a.h[j + 1] += a.h[j] >> 26;
        a.h[j] &= 0x3ffffff;
    }
}

__device__ __forceinline__ void fill_aead_lds(uint32_t *s_tt, uint32_t *s_rp,
                                              const AeadKeyDev *__restrict__ K) {
    // [pair p: 64 KiB][entry e: 256 B][half h: 128 B][copy c = lane & 31];
    // table 2p + h = T rotated right by 8 (2p + h)
    for (uint32_t i = threadIdx.x; i < kAeadTableWords; i += blockDim.x) {
        const uint32_t j = 2u * (i >> 14) + ((i >> 5) & 1u);
        const uint32_t t = K->te[(i >> 6) & 255u];
        s_tt[i] = j ? ror32(t, 8 * j) : t;
    }
    for (uint32_t i = threadIdx.x; i < 65u * 5u; i += blockDim.x) s_rp[i] = (&K->rpow[0][0])[i];
    __syncthreads();
}

}  // namespace

// One wave per unit: CTR en/decryption of the unit's blocks + the unit's
// Poly1305 partial (positioned in the whole ciphertext).  OPEN: input is
// nonce || ct || tag, the MAC runs over the input ciphertext; SEAL: the MAC
// runs over the ciphertext this lane produced.
template <bool OPEN>
__global__ __launch_bounds__(kAeadThreads, kAeadBlocksPerCU) void rcdc_aead_unit_kernel(
    const uint8_t *__restrict__ in, uint8_t *__restrict__ out, const AeadBlob *__restrict__ blobs,
    const AeadUnit *__restrict__ units, uint32_t nunits, const AeadKeyDev *__restrict__ K,
    uint32_t *__restrict__ partials) {
    __shared__ uint32_t s_tt[kAeadTableWords];
    __shared__ uint32_t s_rp[65 * 5];
    fill_aead_lds(s_tt, s_rp, K);
    const uint8_t *tt = reinterpret_cast<const uint8_t *>(s_tt);
    const uint32_t lane = threadIdx.x & 63u, lane4 = (lane & 31u) * 4u;
    const uint32_t wpb = blockDim.x / 64u;
    for (uint32_t u = blockIdx.x * wpb + (threadIdx.x >> 6); u < nunits; u += gridDim.x * wpb) {
        const AeadUnit U = units[u];
        const AeadBlob B = blobs[U.blob];
        const uint64_t len = B.len;
        const uint64_t nblocks = (len + 15) / 16;
        uint32_t nonce[4];
        blob_nonce<OPEN>(in, B, nonce);
        const uint8_t *src = in + B.in_off + (OPEN ? 16 : 0);
        uint8_t *dst = out + B.out_off + (OPEN ? 0 : 16);
        // full blocks: 4 dwords (+ 1 when src is not 4-aligned; the shift is
        // wave-uniform) from the 4-aligned base, loaded one step ahead
        const uintptr_t sa = reinterpret_cast<uintptr_t>(src);
        const uint32_t sh = (uint32_t)(sa & 3u) * 8u;
        const uint32_t *q0 = reinterpret_cast<const uint32_t *>(src - (sa & 3u));
        const uint64_t nfull = len / 16;
        const uint64_t b1 = U.b1;
        auto fetch = [&](uint64_t bb, uint32_t x[5]) {
            if (bb < b1 && bb < nfull) {
                const uint32_t *q = q0 + bb * 4;
                x[0] = q[0]; x[1] = q[1]; x[2] = q[2]; x[3] = q[3];
                if (sh) x[4] = q[4];
            }
        };
        P26 acc = {{0, 0, 0, 0, 0}};
        uint64_t last = ~0ull;
        // one block: keystream (s0..s3, big-endian words) XOR data, store,
        // Horner step acc = acc * r^64 + m (the MAC runs over the ciphertext)
        auto finish_block = [&](uint64_t bb, const uint32_t x[5], uint32_t s0, uint32_t s1,
                                uint32_t s2, uint32_t s3) {
            const uint64_t o = bb * 16;
            const uint32_t k = bb < nfull ? 16u : (uint32_t)(len - o);
            uint32_t w[4];
            if (k == 16) {
                w[0] = __builtin_amdgcn_alignbit(x[1], x[0], sh);
                w[1] = __builtin_amdgcn_alignbit(x[2], x[1], sh);
                w[2] = __builtin_amdgcn_alignbit(x[3], x[2], sh);
                w[3] = __builtin_amdgcn_alignbit(x[4], x[3], sh);
            } else {
                load_partial(src + o, k, w);
            }
            uint32_t c[4] = {w[0] ^ bswap32(s0), w[1] ^ bswap32(s1), w[2] ^ bswap32(s2),
                             w[3] ^ bswap32(s3)};
            if (k == 16) {
                store16(dst + o, c);
            } else {
                for (uint32_t i = 0; i < k; i++) dst[o + i] = (uint8_t)(c[i >> 2] >> (8 * (i & 3)));
            }
            const P26 m = pblock(OPEN ? w : c, k);
            acc = pmul(acc, K->rpow[64]);  // acc = 0 before the first block
            for (int i = 0; i < 5; i++) acc.h[i] += m.h[i];
            last = bb;
        };
        // two blocks per step (b, b + 64): two independent AES chains
        uint32_t xa[5] = {0, 0, 0, 0, 0}, xb[5] = {0, 0, 0, 0, 0};
        uint64_t b = (uint64_t)U.b0 + lane;
        fetch(b, xa);
        fetch(b + 64, xb);
        for (; b < b1; b += 128) {
            const uint32_t ca[5] = {xa[0], xa[1], xa[2], xa[3], xa[4]};
            const uint32_t cb[5] = {xb[0], xb[1], xb[2], xb[3], xb[4]};
            fetch(b + 128, xa);
            fetch(b + 192, xb);
            uint32_t a0, a1, a2, a3, e0, e1, e2, e3;
            ctr_block(nonce, b, a0, a1, a2, a3);
            ctr_block(nonce, b + 64, e0, e1, e2, e3);
            aes_block<14>(a0, a1, a2, a3, tt, lane4, K->rk256);
            aes_block<14>(e0, e1, e2, e3, tt, lane4, K->rk256);
            finish_block(b, ca, a0, a1, a2, a3);
            if (b + 64 < b1) finish_block(b + 64, cb, e0, e1, e2, e3);
        }
        // lane -> unit partial: acc * r^(b1 - last), then the wave's sum
        if (last != ~0ull) {
            acc = pmul(acc, s_rp + (U.b1 - last) * 5);
        }
        for (int off = 32; off > 0; off >>= 1) {
            P26 o;
            for (int i = 0; i < 5; i++) o.h[i] = __shfl_down(acc.h[i], off, 64);
            for (int i = 0; i < 5; i++) acc.h[i] += o.h[i];
            pnorm(acc);
        }
        if (lane == 0) {
            // position: * r^(nblocks - b1), by binary powers
            uint64_t e = nblocks - U.b1;
            for (int j = 0; e; j++, e >>= 1)
                if (e & 1) acc = pmul(acc, K->r2j[j]);
            pnorm(acc);
            for (int i = 0; i < 5; i++) partials[(uint64_t)u * 5 + i] = acc.h[i];
        }
    }
}

// One thread per blob: sum the units' partials, reduce mod 2^130 - 5, add
// AES-128_k(nonce), write the nonce and tag (seal) or check the tag (open).
template <bool OPEN>
__global__ __launch_bounds__(256) void rcdc_aead_finish_kernel(
    const uint8_t *__restrict__ in, uint8_t *__restrict__ out, const AeadBlob *__restrict__ blobs,
    const uint32_t *__restrict__ unit0, uint32_t nblobs, const AeadKeyDev *__restrict__ K,
    const uint32_t *__restrict__ partials, uint32_t *__restrict__ status) {
    __shared__ uint32_t s_te[256];
    for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) s_te[i] = K->te[i];
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nblobs) return;
    const AeadBlob B = blobs[i];
    P26 h = {{0, 0, 0, 0, 0}};
    for (uint32_t u = unit0[i]; u < unit0[i + 1]; u++) {
        for (int j = 0; j < 5; j++) h.h[j] += partials[(uint64_t)u * 5 + j];
        pnorm(h);
    }
    pfull(h);
    // h mod p: h - p if h >= p
    uint32_t g[5];
    uint32_t c = 5;
    for (int j = 0; j < 5; j++) {
        const uint32_t t = h.h[j] + c;
        g[j] = t & 0x3ffffff;
        c = t >> 26;
    }
    if (c) {  // h + 5 >= 2^130
        for (int j = 0; j < 5; j++) h.h[j] = g[j];
    }
    const uint64_t lo = (uint64_t)h.h[0] | (uint64_t)h.h[1] << 26 | (uint64_t)h.h[2] << 52;
    const uint64_t hi = (uint64_t)(h.h[2] >> 12) | (uint64_t)h.h[3] << 14 | (uint64_t)h.h[4] << 40;
    // s = AES-128_k(nonce): byte-oriented T-table lookups (one block per blob)
    uint32_t nonce[4];
    blob_nonce<OPEN>(in, B, nonce);
    uint32_t s0 = bswap32(nonce[0]), s1 = bswap32(nonce[1]), s2 = bswap32(nonce[2]),
             s3 = bswap32(nonce[3]);
    const uint32_t *rk = K->rk128;
    s0 ^= rk[0]; s1 ^= rk[1]; s2 ^= rk[2]; s3 ^= rk[3];
    for (int r = 1; r < 10; r++) {
        const uint32_t t0 = s_te[s0 >> 24] ^ ror32(s_te[(s1 >> 16) & 255], 8) ^
                            ror32(s_te[(s2 >> 8) & 255], 16) ^ ror32(s_te[s3 & 255], 24) ^ rk[4 * r];
        const uint32_t t1 = s_te[s1 >> 24] ^ ror32(s_te[(s2 >> 16) & 255], 8) ^
                            ror32(s_te[(s3 >> 8) & 255], 16) ^ ror32(s_te[s0 & 255], 24) ^ rk[4 * r + 1];
        const uint32_t t2 = s_te[s2 >> 24] ^ ror32(s_te[(s3 >> 16) & 255], 8) ^
                            ror32(s_te[(s0 >> 8) & 255], 16) ^ ror32(s_te[s1 & 255], 24) ^ rk[4 * r + 2];
        const uint32_t t3 = s_te[s3 >> 24] ^ ror32(s_te[(s0 >> 16) & 255], 8) ^
                            ror32(s_te[(s1 >> 8) & 255], 16) ^ ror32(s_te[s2 & 255], 24) ^ rk[4 * r + 3];
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
#define SB3(x) ((s_te[x] << 8) & 0xff000000u)
#define SB2(x) (s_te[x] & 0x00ff0000u)
#define SB1(x) ((s_te[x] >> 8) & 0x0000ff00u)
#define SB0(x) ((s_te[x] >> 16) & 0x000000ffu)
    const uint32_t f0 = (SB3(s0 >> 24) | SB2((s1 >> 16) & 255) | SB1((s2 >> 8) & 255) | SB0(s3 & 255)) ^ rk[40];
    const uint32_t f1 = (SB3(s1 >> 24) | SB2((s2 >> 16) & 255) | SB1((s3 >> 8) & 255) | SB0(s0 & 255)) ^ rk[41];
    const uint32_t f2 = (SB3(s2 >> 24) | SB2((s3 >> 16) & 255) | SB1((s0 >> 8) & 255) | SB0(s1 & 255)) ^ rk[42];
    const uint32_t f3 = (SB3(s3 >> 24) | SB2((s0 >> 16) & 255) | SB1((s1 >> 8) & 255) | SB0(s2 & 255)) ^ rk[43];
#undef SB0
#undef SB1
#undef SB2
#undef SB3
    // s as a little-endian 128-bit number (its bytes in order)
    const uint64_t slo = (uint64_t)bswap32(f1) << 32 | bswap32(f0);
    const uint64_t shi = (uint64_t)bswap32(f3) << 32 | bswap32(f2);
    const uint64_t tlo = lo + slo;
    const uint64_t thi = hi + shi + (tlo < lo ? 1 : 0);
    uint8_t tag[16];
    for (int j = 0; j < 8; j++) {
        tag[j] = (uint8_t)(tlo >> (8 * j));
        tag[8 + j] = (uint8_t)(thi >> (8 * j));
    }
    if (OPEN) {
        const uint8_t *t = in + B.in_off + 16 + B.len;
        uint32_t d = 0;
        for (int j = 0; j < 16; j++) d |= tag[j] ^ t[j];
        status[i] = d ? 1u : 0u;
    } else {
        uint8_t *o = out + B.out_off;
        store16(o, B.nonce);
        for (int j = 0; j < 16; j++) o[16 + B.len + j] = tag[j];
        if (B.flags & kAeadAppendLen) {  // packer.rs:713-725: the header length, unencrypted
            const uint32_t hl = (uint32_t)B.len + 32u;
            for (int j = 0; j < 4; j++) o[32 + B.len + j] = (uint8_t)(hl >> (8 * j));
        }
    }
}

namespace rcdc {

hipError_t launch_aead(bool open, const uint8_t *in, uint8_t *out, const AeadBlob *blobs,
                       uint32_t nblobs, const AeadUnit *units, uint32_t nunits,
                       const uint32_t *unit0, const AeadKeyDev *key, uint32_t *partials,
                       uint32_t *status, uint32_t cus, hipStream_t stream) {
    if (nblobs == 0) return hipSuccess;
    const uint32_t wpb = kAeadThreads / 64;
    const uint64_t want = (nunits + wpb - 1) / wpb, cap = (uint64_t)kAeadBlocksPerCU * cus;
    const uint32_t blocks = (uint32_t)(want < cap ? want : cap);
    if (nunits) {
        if (open)
            hipLaunchKernelGGL((rcdc_aead_unit_kernel<true>), dim3(blocks), dim3(kAeadThreads), 0,
                               stream, in, out, blobs, units, nunits, key, partials);
        else
            hipLaunchKernelGGL((rcdc_aead_unit_kernel<false>), dim3(blocks), dim3(kAeadThreads), 0,
                               stream, in, out, blobs, units, nunits, key, partials);
    }
    const uint32_t fb = (nblobs + 255) / 256;
    if (open)
        hipLaunchKernelGGL((rcdc_aead_finish_kernel<true>), dim3(fb), dim3(256), 0, stream, in, out,
                           blobs, unit0, nblobs, key, partials, status);
    else
        hipLaunchKernelGGL((rcdc_aead_finish_kernel<false>), dim3(fb), dim3(256), 0, stream, in,
                           out, blobs, unit0, nblobs, key, partials, status);
    return hipGetLastError();
}

}  // namespace rcdc
