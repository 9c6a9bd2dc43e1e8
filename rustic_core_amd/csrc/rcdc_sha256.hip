// rcdc_sha256.hip -- SHA-256 of every chunk, on the bytes already in HBM.
//
// Reference: the blob id of a chunk is `hash(&chunk)` = SHA-256
// (crates/core/src/crypto/hasher.rs:17-19), computed by
// FileArchiver::backup_reader right after the chunker yields the chunk
// (crates/core/src/archiver/file_archiver.rs:151).  The chunker test
// snapshot (src/chunker/snapshots/*chunk_random.snap) pins (len, sha256)
// pairs, so the digests are checked against it directly.
//
// SHA-256 (FIPS 180-4) is a strict Merkle-Damgard chain: a chunk's 64-byte
// blocks must be compressed in order, so the only parallelism is across
// chunks.  One lane owns one chunk.  Per 64-byte block the lane issues 16
// dword loads at its (4-aligned-down) address, realigns them with
// v_alignbyte and byte-swaps with v_perm, expands the message schedule in a
// 16-word register ring and runs the 64 rounds: ~1.4k VALU ops per block,
// ~21 per byte, so the kernel is VALU-bound (not HBM-bound) and reaches its
// throughput only with >= ~4 waves per SIMD of chunks in flight (C3/C4
// scale), not on 1409 chunks (C2).
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "rcdc_internal.h"

namespace rcdc {

namespace {

__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t n) {
    return __builtin_amdgcn_alignbit(x, x, n);
}

// Maj(x, y, z) in one v_bitop3_b32 (0xF0&0xCC | 0xF0&0xAA | 0xCC&0xAA);
// the compiler's own lowering is v_xor + v_bfi
__device__ __forceinline__ uint32_t maj3(uint32_t x, uint32_t y, uint32_t z) {
    return __builtin_amdgcn_bitop3_b32(x, y, z, 0xE8);
}

// x ^ y ^ z in one v_bitop3_b32 (truth table 0xF0 ^ 0xCC ^ 0xAA)
__device__ __forceinline__ uint32_t xor3(uint32_t x, uint32_t y, uint32_t z) {
    return __builtin_amdgcn_bitop3_b32(x, y, z, 0x96);
}

// Prefetch of the next block: 4 x global_load_dwordx4 (4-byte aligned
// addresses are accepted) + 1 dword, issued as inline asm.  Plain loads of
// read-only bytes get rematerialised next to their use by the compiler,
// which re-exposes the full HBM latency every block; volatile loads become
// uncached (sc0 sc1) with a wait after each.  The compiler does not track
// these loads, so wait_loads() must run before any use of their results;
// its "+v" operands order every use (and copy) after the wait.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
struct Blk {
    u32x4 v0, v1, v2, v3;
    uint32_t x16;
};
__device__ __forceinline__ void issue_loads(const uint32_t *p, uint32_t o16, Blk &b) {
    const uint32_t *p16 = p + o16;
    asm volatile(
        "global_load_dwordx4 %0, %5, off\n\t"
        "global_load_dwordx4 %1, %5, off offset:16\n\t"
        "global_load_dwordx4 %2, %5, off offset:32\n\t"
        "global_load_dwordx4 %3, %5, off offset:48\n\t"
        "global_load_dword %4, %6, off"
        : "=&v"(b.v0), "=&v"(b.v1), "=&v"(b.v2), "=&v"(b.v3), "=&v"(b.x16)
        : "v"(p), "v"(p16)
        : "memory");
}
__device__ __forceinline__ void wait_loads(Blk &b) {
    asm volatile("s_waitcnt vmcnt(0)"
                 : "+v"(b.v0), "+v"(b.v1), "+v"(b.v2), "+v"(b.v3), "+v"(b.x16)
                 :
                 : "memory");
}
__device__ __forceinline__ void unpack(const Blk &b, uint32_t (&x)[17]) {
    x[0] = b.v0.x; x[1] = b.v0.y; x[2] = b.v0.z; x[3] = b.v0.w;
    x[4] = b.v1.x; x[5] = b.v1.y; x[6] = b.v1.z; x[7] = b.v1.w;
    x[8] = b.v2.x; x[9] = b.v2.y; x[10] = b.v2.z; x[11] = b.v2.w;
    x[12] = b.v3.x; x[13] = b.v3.y; x[14] = b.v3.z; x[15] = b.v3.w;
    x[16] = b.x16;
}

__device__ __forceinline__ uint32_t bswap(uint32_t x) {
    return __builtin_bswap32(x);  // one v_perm_b32
}

constexpr uint32_t kK[64] = {
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

struct Sha {
    uint32_t s[8];
    __device__ __forceinline__ void init() {
        s[0] = 0x6a09e667u; s[1] = 0xbb67ae85u; s[2] = 0x3c6ef372u; s[3] = 0xa54ff53au;
        s[4] = 0x510e527fu; s[5] = 0x9b05688cu; s[6] = 0x1f83d9abu; s[7] = 0x5be0cd19u;
    }
    // w[]: the block as 16 big-endian words (consumed: becomes the schedule)
    __device__ __forceinline__ void compress(uint32_t w[16]) {
        uint32_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
#pragma unroll
        for (int t = 0; t < 64; t++) {
            uint32_t wt;
            if (t < 16) {
                wt = w[t];
            } else {
                const uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
                const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
                const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
                wt = w[t & 15] = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
            }
            const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
            const uint32_t ch = (e & f) ^ (~e & g);
            const uint32_t t1 = h + S1 + ch + kK[t] + wt;
            const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
            const uint32_t maj = maj3(a, b, c);
            const uint32_t t2 = S0 + maj;
            h = g; g = f; f = e; e = d + t1;
            d = c; c = b; b = a; a = t1 + t2;
        }
        s[0] += a; s[1] += b; s[2] += c; s[3] += d;
        s[4] += e; s[5] += f; s[6] += g; s[7] += h;
    }
    // rounds only: kw[t / 4][lane] holds K[t] + W[t] (schedule done elsewhere)
    __device__ __forceinline__ void compress_kw(const uint4 (*kw)[64], uint32_t lane) {
        uint32_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
#pragma unroll
        for (int t4 = 0; t4 < 16; t4++) {
            const uint4 v = kw[t4][lane];
            const uint32_t kwv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
                const uint32_t ch = (e & f) ^ (~e & g);
                const uint32_t t1 = h + S1 + ch + kwv[u];
                const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
                const uint32_t maj = maj3(a, b, c);
                const uint32_t t2 = S0 + maj;
                h = g; g = f; f = e; e = d + t1;
                d = c; c = b; b = a; a = t1 + t2;
            }
        }
        s[0] += a; s[1] += b; s[2] += c; s[3] += d;
        s[4] += e; s[5] += f; s[6] += g; s[7] += h;
    }
};

// K[t] + W[t] for t = 0..63 of one block (w: the 16 big-endian words),
// written to kw[t / 4][lane].
__device__ __forceinline__ void schedule_kw(uint32_t w[16], uint4 (*kw)[64], uint32_t lane) {
    uint32_t o[4];
#pragma unroll
    for (int t = 0; t < 64; t++) {
        uint32_t wt;
        if (t < 16) {
            wt = w[t];
        } else {
            const uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
            const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
            const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
            wt = w[t & 15] = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
        }
        o[t & 3] = wt + kK[t];
        if ((t & 3) == 3) kw[t >> 2][lane] = make_uint4(o[0], o[1], o[2], o[3]);
    }
}

__device__ __forceinline__ void sha256_tail(Sha &sh, const uint32_t *q, uint32_t k, uint64_t len,
                                            uint32_t *__restrict__ out);

// SHA-256 of arena[p, p + len) into out[0..8) (digest words, big-endian
// byte order when stored as bytes: out bytes = digest bytes).
__device__ __forceinline__ void sha256_range(const uint8_t *__restrict__ arena, uint64_t p,
                                             uint64_t len, uint32_t *__restrict__ out) {
    Sha sh;
    sh.init();
    const uint32_t k = (uint32_t)(p & 3);  // byte misalignment
    const uint32_t *q = (const uint32_t *)(arena + (p - k));
    const uint64_t nfull = len >> 6;
    // Block i is dwords q[16i .. 16i + 16] (17: the misaligned last word).
    // The next block's dwords are loaded before this block is compressed,
    // so HBM latency hides behind ~1.4k VALU ops of the current block.
    // q[16] is read from q[15] when k == 0 (unused then, and q[16] may lie
    // past the chunk's last dword); past the last full block the prefetch
    // re-reads the current block.
    const uint32_t o16 = k ? 16u : 15u;
    Blk cur, nxt;
    if (nfull) {
        issue_loads(q, o16, cur);
        wait_loads(cur);
    }
    for (uint64_t blk = 0; blk < nfull; blk++) {
        const uint32_t *qn = (blk + 1 < nfull) ? q + 16 : q;
        issue_loads(qn, o16, nxt);
        __builtin_amdgcn_sched_barrier(0);  // keep the prefetch at the top
        uint32_t d[17];
        unpack(cur, d);
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 16; i++) w[i] = bswap(__builtin_amdgcn_alignbyte(d[i + 1], d[i], k));
        sh.compress(w);
        wait_loads(nxt);
        cur = nxt;
        q += 16;
    }
    sha256_tail(sh, q, k, len, out);
}

// The last (len % 64) bytes at q (4-aligned-down, misalignment k) plus the
// padding: 0x80, zeros, 64-bit big-endian bit length; then the digest.
__device__ __forceinline__ void sha256_tail(Sha &sh, const uint32_t *q, uint32_t k, uint64_t len,
                                            uint32_t *__restrict__ out) {
    const uint32_t r = (uint32_t)(len & 63);
    // last valid byte relative to q (aligned base): k + r - 1; dword j holds
    // a valid byte iff 4j <= k + r - 1
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; i++) {
        const uint32_t j0 = (uint32_t)i, j1 = (uint32_t)i + 1;
        const uint32_t lo = (4 * j0 < k + r) ? q[j0] : 0;
        const uint32_t hi = (4 * j1 < k + r) ? q[j1] : 0;
        uint32_t v = __builtin_amdgcn_alignbyte(hi, lo, k);  // little-endian bytes 4i..4i+3
        const int nv = (int)r - 4 * i;                         // valid bytes in this word
        if (nv <= 0) v = 0;
        else if (nv < 4) v &= (1u << (8 * nv)) - 1u;
        if (nv >= 0 && nv < 4) v |= 0x80u << (8 * nv);
        w[i] = bswap(v);
    }
    const uint64_t bits = len << 3;
    if (r < 56) {
        w[14] = (uint32_t)(bits >> 32);
        w[15] = (uint32_t)bits;
        sh.compress(w);
    } else {
        sh.compress(w);
#pragma unroll
        for (int i = 0; i < 14; i++) w[i] = 0;
        w[14] = (uint32_t)(bits >> 32);
        w[15] = (uint32_t)bits;
        sh.compress(w);
    }
#pragma unroll
    for (int i = 0; i < 8; i++) out[i] = bswap(sh.s[i]);
}

// Chunk list: chunk c = arena[refs[c].x, refs[c].x + refs[c].y).
__global__ __launch_bounds__(64) void rcdc_sha256_list_kernel(const uint8_t *__restrict__ arena,
                                                              const ulonglong2 *__restrict__ refs,
                                                              uint32_t n,
                                                              uint32_t *__restrict__ digests) {
    const uint32_t c = blockIdx.x * 64 + threadIdx.x;
    if (c >= n) return;
    const ulonglong2 ref = refs[c];
    sha256_range(arena, ref.x, ref.y, digests + 8ull * c);
}

// A plan's results: slot g in [0, nslots) belongs to the stream i with
// cut_base <= g < cut_base + cut_cap; it is chunk j = g - cut_base of that
// stream when j < counts[i] (a count of ~0 marks a stream the host redoes).
__global__ __launch_bounds__(64) void rcdc_sha256_plan_kernel(
    const uint8_t *__restrict__ arena, const StreamDesc *__restrict__ sds, uint32_t nstreams,
    const uint64_t *__restrict__ cuts, const uint64_t *__restrict__ counts, uint64_t nslots,
    uint32_t *__restrict__ digests) {
    const uint64_t g = (uint64_t)blockIdx.x * 64 + threadIdx.x;
    if (g >= nslots) return;
    uint32_t lo = 0, hi = nstreams;  // last stream with cut_base <= g
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (sds[mid].cut_base <= g) lo = mid;
        else hi = mid;
    }
    const StreamDesc sd = sds[lo];
    const uint64_t j = g - sd.cut_base;
    const uint64_t cnt = counts[lo];
    if (cnt == ~0ull || j >= cnt) return;
    const uint64_t start = j ? cuts[g - 1] : 0;
    const uint64_t end = cuts[g];
    sha256_range(arena, sd.off + start, end - start, digests + 8ull * g);
}

// Two waves per 64 chunks.  Lane l of both waves owns the
// same chunk.  Wave 0 loads block i + 1 (prefetched one ahead), realigns it
// and expands the message schedule into LDS as K + W; wave 1 runs the 64
// rounds of block i from LDS.  This takes the schedule (~1/3 of the VALU
// ops) off the chain that bounds a chunk's latency.  The slots ping-pong
// with one barrier per block; both waves loop to the wave-wide maximum block
// count, so the barrier count is uniform.
struct ChunkLoc {
    uint64_t p, len;
    bool valid;
};

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t x) {
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {
        const uint64_t y = __shfl_xor(x, m, 64);
        x = y > x ? y : x;
    }
    return x;
}

__device__ __forceinline__ void sha256_split(const uint8_t *__restrict__ arena, ChunkLoc c,
                                             uint32_t *__restrict__ out) {
    __shared__ uint4 kw[2][16][64];  // [slot][t / 4][lane]: 32 KiB
    // issue priority over other kernels' waves on the same SIMD: a chunk's
    // chain is latency-bound, and next to compress / seal kernels (the
    // device ingest runs them under the ids) it otherwise gets a share of
    // the SIMD's issue slots (waves of this kernel stay equal among
    // themselves)
    __builtin_amdgcn_s_setprio(2);
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t k = (uint32_t)(c.p & 3);
    const uint32_t *q0 = (const uint32_t *)(arena + (c.p - k));
    const uint64_t nfull = c.valid ? c.len >> 6 : 0;
    const uint64_t nmax = wave_max_u64(nfull);
    if (nmax == 0 && !c.valid) return;  // whole wave idle (both waves agree)
    const uint32_t o16 = k ? 16u : 15u;
    Sha sh;
    sh.init();
    Blk cur, nxt;
    if (wv == 0 && nfull) {
        issue_loads(q0, o16, cur);
        wait_loads(cur);
    }
    for (uint64_t it = 0; it <= nmax; it++) {
        if (wv == 0) {
            if (it < nfull) {
                const uint32_t *q = q0 + 16 * it;
                const uint32_t *qn = (it + 1 < nfull) ? q + 16 : q;
                issue_loads(qn, o16, nxt);
                __builtin_amdgcn_sched_barrier(0);
                uint32_t d[17];
                unpack(cur, d);
                uint32_t w[16];
#pragma unroll
                for (int i = 0; i < 16; i++)
                    w[i] = bswap(__builtin_amdgcn_alignbyte(d[i + 1], d[i], k));
                schedule_kw(w, kw[it & 1], lane);
                wait_loads(nxt);
                cur = nxt;
            }
        } else if (it >= 1 && it - 1 < nfull) {
            sh.compress_kw(kw[(it - 1) & 1], lane);
        }
        __syncthreads();
    }
    if (wv == 1 && c.valid) sha256_tail(sh, q0 + 16 * nfull, k, c.len, out);
}

__global__ __launch_bounds__(128) void rcdc_sha256_list_split_kernel(
    const uint8_t *__restrict__ arena, const ulonglong2 *__restrict__ refs, uint32_t n,
    uint32_t *__restrict__ digests) {
    const uint32_t ci = blockIdx.x * 64 + (threadIdx.x & 63);
    ChunkLoc c{0, 0, false};
    if (ci < n) {
        const ulonglong2 ref = refs[ci];
        c = {ref.x, ref.y, true};
    }
    sha256_split(arena, c, digests + 8ull * ci);
}

// Locate cut slot g of a plan: chunk [cuts[g-1], cuts[g]) of the stream
// whose slot range holds g (binary search over cut_base).
__device__ __forceinline__ ChunkLoc plan_chunk(const StreamDesc *__restrict__ sds,
                                               uint32_t nstreams, const uint64_t *__restrict__ cuts,
                                               const uint64_t *__restrict__ counts, uint64_t g) {
    uint32_t lo = 0, hi = nstreams;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (sds[mid].cut_base <= g) lo = mid;
        else hi = mid;
    }
    const uint64_t j = g - sds[lo].cut_base;
    const uint64_t cnt = counts[lo];
    if (cnt == ~0ull || j >= cnt) return {0, 0, false};
    const uint64_t start = j ? cuts[g - 1] : 0;
    return {sds[lo].off + start, cuts[g] - start, true};
}

// Length buckets, longest first: a wave's time is its longest chunk, so
// chunks of similar length share a wave and the longest start first.
constexpr uint32_t kShaBuckets = 64;
__device__ __forceinline__ uint32_t len_bucket(uint64_t len, uint64_t max_len) {
    const uint64_t l = len < max_len ? len : max_len;
    const uint64_t b = (max_len - l) * kShaBuckets / (max_len + 1);
    return (uint32_t)b;
}

// Per-block LDS histograms: one global atomic per bucket per block (80 k
// global atomics on 64 counters serialised at L2 for ~0.6 ms per kernel).
__global__ __launch_bounds__(256) void rcdc_sha256_count_kernel(
    const StreamDesc *__restrict__ sds, uint32_t nstreams, const uint64_t *__restrict__ cuts,
    const uint64_t *__restrict__ counts, uint64_t nslots, uint64_t max_len,
    uint32_t *__restrict__ bcount) {
    __shared__ uint32_t hist[kShaBuckets];
    if (threadIdx.x < kShaBuckets) hist[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (g < nslots) {
        const ChunkLoc c = plan_chunk(sds, nstreams, cuts, counts, g);
        if (c.valid) atomicAdd(&hist[len_bucket(c.len, max_len)], 1u);
    }
    __syncthreads();
    if (threadIdx.x < kShaBuckets && hist[threadIdx.x])
        atomicAdd(&bcount[threadIdx.x], hist[threadIdx.x]);
}

// bcount[0..64) counts, bcount[64..128) cursors (zeroed), bcount[128] total
__global__ __launch_bounds__(256) void rcdc_sha256_order_kernel(
    const StreamDesc *__restrict__ sds, uint32_t nstreams, const uint64_t *__restrict__ cuts,
    const uint64_t *__restrict__ counts, uint64_t nslots, uint64_t max_len,
    uint32_t *__restrict__ bcount, uint32_t *__restrict__ order) {
    __shared__ uint32_t boff[kShaBuckets], hist[kShaBuckets], base[kShaBuckets];
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (uint32_t b = 0; b < kShaBuckets; b++) {
            boff[b] = acc;
            acc += bcount[b];
        }
        if (blockIdx.x == 0) bcount[2 * kShaBuckets] = acc;
    }
    if (threadIdx.x < kShaBuckets) hist[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    ChunkLoc c{0, 0, false};
    if (g < nslots) c = plan_chunk(sds, nstreams, cuts, counts, g);
    const uint32_t b = c.valid ? len_bucket(c.len, max_len) : 0;
    const uint32_t local = c.valid ? atomicAdd(&hist[b], 1u) : 0;
    __syncthreads();
    if (threadIdx.x < kShaBuckets)
        base[threadIdx.x] =
            hist[threadIdx.x] ? atomicAdd(&bcount[kShaBuckets + threadIdx.x], hist[threadIdx.x]) : 0;
    __syncthreads();
    if (c.valid) order[boff[b] + base[b] + local] = (uint32_t)g;
}

__global__ __launch_bounds__(128) void rcdc_sha256_plan_split_kernel(
    const uint8_t *__restrict__ arena, const StreamDesc *__restrict__ sds, uint32_t nstreams,
    const uint64_t *__restrict__ cuts, const uint64_t *__restrict__ counts, uint64_t nslots,
    const uint32_t *__restrict__ order, const uint32_t *__restrict__ total,
    uint32_t *__restrict__ digests) {
    const uint64_t i = (uint64_t)blockIdx.x * 64 + (threadIdx.x & 63);
    ChunkLoc c{0, 0, false};
    uint64_t g = i;
    if (order) {
        if (i < *total) {
            g = order[i];
            c = plan_chunk(sds, nstreams, cuts, counts, g);
        }
    } else if (i < nslots) {
        c = plan_chunk(sds, nstreams, cuts, counts, g);
    }
    sha256_split(arena, c, digests + 8ull * g);
}

// Several plans in one launch (rcdc_plan_hash_many): blockIdx.x % n picks
// the plan, so D batches share the longest-chunk floor without depending on
// how many hardware queues the streams map to.
constexpr uint32_t kShaMaxPlans = 8;
struct ShaPlanDesc {
    const uint8_t *arena;
    const StreamDesc *sds;
    const uint64_t *cuts;
    const uint64_t *counts;
    const uint32_t *order;
    const uint32_t *total;
    uint32_t *digests;
    uint32_t nstreams;
    uint32_t pad;
};
struct ShaMulti {
    ShaPlanDesc p[kShaMaxPlans];
};

__global__ __launch_bounds__(128) void rcdc_sha256_multi_split_kernel(ShaMulti m, uint32_t n) {
    // plan-minor block order: every plan's longest chunks dispatch first
    const uint32_t pj = blockIdx.x % n, xb = blockIdx.x / n;
    const ShaPlanDesc &d = m.p[pj];
    const uint64_t i = (uint64_t)xb * 64 + (threadIdx.x & 63);
    ChunkLoc c{0, 0, false};
    uint64_t g = i;
    if (i < *d.total) {
        g = d.order[i];
        c = plan_chunk(d.sds, d.nstreams, d.cuts, d.counts, g);
    }
    sha256_split(d.arena, c, d.digests + 8ull * g);
}

}  // namespace

// RCDC_SHA_LANE=1 selects the one-wave kernels (one lane does schedule and
// rounds) for A/B measurements.
static bool lane_variant() {
    static const bool v = getenv("RCDC_SHA_LANE") != nullptr;
    return v;
}

hipError_t launch_sha256_list(const uint8_t *arena, const ulonglong2 *refs, uint32_t n,
                              uint32_t *digests, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    if (lane_variant())
        hipLaunchKernelGGL(rcdc_sha256_list_kernel, dim3((n + 63) / 64), dim3(64), 0, stream,
                           arena, refs, n, digests);
    else
        hipLaunchKernelGGL(rcdc_sha256_list_split_kernel, dim3((n + 63) / 64), dim3(128), 0,
                           stream, arena, refs, n, digests);
    return hipGetLastError();
}

hipError_t launch_sha256_plan(const uint8_t *arena, const StreamDesc *sds, uint32_t nstreams,
                              const uint64_t *cuts, const uint64_t *counts, uint64_t nslots,
                              uint64_t max_len, uint32_t *bwork, uint32_t *order,
                              uint32_t *digests, hipStream_t stream) {
    if (nslots == 0 || nstreams == 0) return hipSuccess;
    const dim3 grid((uint32_t)((nslots + 63) / 64));
    if (lane_variant()) {
        hipLaunchKernelGGL(rcdc_sha256_plan_kernel, grid, dim3(64), 0, stream, arena, sds,
                           nstreams, cuts, counts, nslots, digests);
        return hipGetLastError();
    }
    const bool sorted = order && bwork && nslots < (1ull << 32);
    if (sorted) {
        const dim3 g256((uint32_t)((nslots + 255) / 256));
        hipError_t e = hipMemsetAsync(bwork, 0, (2 * kShaBuckets + 1) * sizeof(uint32_t), stream);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(rcdc_sha256_count_kernel, g256, dim3(256), 0, stream, sds, nstreams,
                           cuts, counts, nslots, max_len, bwork);
        hipLaunchKernelGGL(rcdc_sha256_order_kernel, g256, dim3(256), 0, stream, sds, nstreams,
                           cuts, counts, nslots, max_len, bwork, order);
    }
    hipLaunchKernelGGL(rcdc_sha256_plan_split_kernel, grid, dim3(128), 0, stream, arena, sds,
                       nstreams, cuts, counts, nslots, sorted ? order : nullptr,
                       sorted ? bwork + 2 * kShaBuckets : nullptr, digests);
    return hipGetLastError();
}

hipError_t launch_sha256_multi(uint32_t n, const uint8_t *const *arenas,
                               const StreamDesc *const *sds, const uint32_t *nstreams,
                               const uint64_t *const *cuts, const uint64_t *const *counts,
                               const uint64_t *nslots, uint64_t max_len, uint32_t *const *bwork,
                               uint32_t *const *order, uint32_t *const *digests,
                               hipStream_t stream) {
    if (n == 0) return hipSuccess;
    if (n > kShaMaxPlans) return hipErrorInvalidValue;
    ShaMulti m{};
    uint64_t maxslots = 0;
    for (uint32_t j = 0; j < n; j++) {
        if (nslots[j] >= (1ull << 32)) return hipErrorInvalidValue;
        const dim3 g256((uint32_t)((nslots[j] + 255) / 256));
        hipError_t e = hipMemsetAsync(bwork[j], 0, (2 * kShaBuckets + 1) * sizeof(uint32_t), stream);
        if (e != hipSuccess) return e;
        if (nslots[j] && nstreams[j]) {
            hipLaunchKernelGGL(rcdc_sha256_count_kernel, g256, dim3(256), 0, stream, sds[j],
                               nstreams[j], cuts[j], counts[j], nslots[j], max_len, bwork[j]);
            hipLaunchKernelGGL(rcdc_sha256_order_kernel, g256, dim3(256), 0, stream, sds[j],
                               nstreams[j], cuts[j], counts[j], nslots[j], max_len, bwork[j],
                               order[j]);
        }
        m.p[j] = {arenas[j], sds[j], cuts[j], counts[j], order[j], bwork[j] + 2 * kShaBuckets,
                  digests[j], nstreams[j], 0};
        maxslots = nslots[j] > maxslots ? nslots[j] : maxslots;
    }
    if (maxslots == 0) return hipGetLastError();
    const uint64_t blocks = (maxslots + 63) / 64 * n;
    if (blocks >= (1ull << 31)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(rcdc_sha256_multi_split_kernel, dim3((uint32_t)blocks), dim3(128), 0,
                       stream, m, n);
    return hipGetLastError();
}

}  // namespace rcdc
