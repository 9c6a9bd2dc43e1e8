// rcdc_slide.h -- device building blocks shared by the scan and walk kernels
// (gfx950): the Rabin64 slide on LDS tables, 64-byte register units, the
// per-lane segment scan and the LDS table prologue.  See rcdc_scan.hip for
// the cost model these follow.
#pragma once
#include <hip/hip_runtime.h>

#include "rcdc_internal.h"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

namespace {

using namespace rcdc;

constexpr uint32_t kOpA = 0xF0, kOpB = 0xCC, kOpC = 0xAA;  // v_bitop3 operand truth tables
constexpr uint32_t kXor3 = kOpA ^ kOpB ^ kOpC;
constexpr uint32_t kAndOr = (kOpA & kOpB) | kOpC;

// Materialise a wave-uniform value in a VGPR once (keeps the compiler from
// folding it back into an SGPR operand of every use).
__device__ __forceinline__ uint32_t in_vgpr(uint32_t x) {
    uint32_t r;
    asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "s"(x));
    return r;
}

// The tables always live in LDS: address them there even where the pointer
// reaches the code as a generic one (a non-inlined round, rcdc_walk.hip), so
// the lookups are ds_read_b64 and not flat loads.
typedef const __attribute__((address_space(3))) uint8_t lds_u8;
typedef const __attribute__((address_space(3))) unsigned long long lds_u64;

__device__ __forceinline__ uint2 lds_u2(const uint8_t *tab, uint32_t byte_addr) {
#if defined(__HIP_DEVICE_COMPILE__)
    const unsigned long long v = *reinterpret_cast<lds_u64 *>((lds_u8 *)tab + byte_addr);
    return make_uint2((uint32_t)v, (uint32_t)(v >> 32));
#else  // (host pass: never called)
    return *reinterpret_cast<const uint2 *>(tab + byte_addr);
#endif
}

struct Unit {
    u32x4 v[4];
};
#define UDW(u, d) ((u).v[(d) >> 2][(d) & 3])

struct Consts {
    uint32_t lwo, lwm;  // lane's table-copy offset in OUT / MOD
    uint32_t kff00;     // 0xFF00 in a VGPR
    uint32_t mask;      // avg - 1 in a VGPR
    uint32_t tsh;       // deg - 8 (generic-degree path only)
};

// MOD table address of the top byte of h (h1 = hi32(h), a1 = hi32(h << 8)).
// TSH >= 100: compile-time shift TSH - 100 = deg - 48 straight from h1, so the
//   address does not wait for the v_alignbit (critical path per byte:
//   v_lshrrev, v_bitop3, ds_read_b64, v_bitop3);
// 0 <= TSH < 100: compile-time deg - 40 from a1 (v_lshrrev by an inline
//   constant + one v_bitop3 (x & 0xFF00) | lwm);
// TSH < 0: any degree 9..56, runtime 64-bit shift of h by deg - 8 (the
//   top byte straddles h1:h0 for deg < 40; half-rate shift, off the deg-53
//   fast path).
template <int TSH>
__device__ __forceinline__ uint32_t mod_addr(uint32_t h0, uint32_t h1, uint32_t a1,
                                             const Consts &k) {
    if constexpr (TSH >= 100)
        return __builtin_amdgcn_bitop3_b32(h1 >> (TSH - 100), k.kff00, k.lwm, kAndOr);
    else if constexpr (TSH >= 0)
        return __builtin_amdgcn_bitop3_b32(a1 >> TSH, k.kff00, k.lwm, kAndOr);
    else
        return (((uint32_t)(((uint64_t)h1 << 32 | h0) >> k.tsh) & 255u) << 8) | k.lwm;
}

// One slide: h ^= out[o]; i = top byte; h = ((h<<8)|n) ^ mod[i]
// with h = h1:h0 (53 bits for deg 53).
//
// The LDS "OUT" table holds OM[b] = b * x^512 mod P = (out[b] << 8) reduced
// (built in the kernel prologue).  MOD is linear in its index, so
//   mod[top(h ^ out[o])] = mod[top(h)] ^ mod[top(out[o])]
// and the slide becomes h' = ((h << 8) | n) ^ mod[top(h)] ^ OM[o]: the MOD
// index no longer waits for the OUT lookup, and h1 takes one v_bitop3
// (xor3) instead of two XORs -- 7 VALU + 2 ds_read_b64 per byte.
template <int K, int TSH>
__device__ __forceinline__ void slide(uint32_t &h0, uint32_t &h1, uint32_t dnew, uint32_t dold,
                                      const uint8_t *tab, const Consts &k) {
    const uint2 o = lds_u2(tab, __builtin_amdgcn_perm(dold, k.lwo, 0x0C0C0000u | ((4u + K) << 8)));
    const uint32_t a1 = __builtin_amdgcn_alignbit(h1, h0, 24);
    const uint2 m = lds_u2(tab, mod_addr<TSH>(h0, h1, a1, k));
    h0 = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_perm(h0, dnew, 0x06050400u | K), o.x, m.x, kXor3);
    h1 = __builtin_amdgcn_bitop3_b32(a1, o.y, m.y, kXor3);
}

// Warm-up slide (the window is still filling: nothing leaves it).
template <int K, int TSH>
__device__ __forceinline__ void slide_in(uint32_t &h0, uint32_t &h1, uint32_t dnew,
                                         const uint8_t *tab, const Consts &k) {
    const uint32_t a1 = __builtin_amdgcn_alignbit(h1, h0, 24);
    const uint2 m = lds_u2(tab, mod_addr<TSH>(h0, h1, a1, k));
    h0 = __builtin_amdgcn_perm(h0, dnew, 0x06050400u | K) ^ m.x;
    h1 = a1 ^ m.y;
}

template <int TSH>
__device__ __forceinline__ void slide_b(int b, uint32_t &h0, uint32_t &h1, uint32_t dn,
                                        uint32_t d_o, const uint8_t *tab, const Consts &k) {
    switch (b & 3) {
        case 0: slide<0, TSH>(h0, h1, dn, d_o, tab, k); break;
        case 1: slide<1, TSH>(h0, h1, dn, d_o, tab, k); break;
        case 2: slide<2, TSH>(h0, h1, dn, d_o, tab, k); break;
        default: slide<3, TSH>(h0, h1, dn, d_o, tab, k); break;
    }
}

struct Chain {
    uint32_t h0, h1;
    uint32_t first, last, count;  // candidate summary (segment-relative)
    uint32_t rlo, rhi;            // relative positions that count: [rlo, rhi)
};

// Rare path: exact test of the G fingerprints of group rb .. rb + G - 1.
template <int G>
__device__ __forceinline__ void record_group(Chain &c, const uint32_t (&hk)[G], uint32_t mask,
                                             uint32_t rb) {
    // every position of the group a candidate (zero runs, dense data):
    // one OR-reduction (v_bitop3 3-input OR) instead of G compares
    static_assert(G % 2 == 0, "group of an even size");
    uint32_t any = 0;
#pragma unroll
    for (int j = 0; j < G; j += 2)
        any = __builtin_amdgcn_bitop3_b32(any, hk[j], hk[j + 1], kOpA | kOpB | kOpC);
    uint32_t hb;
    if ((any & mask) == 0u) {
        hb = (1u << G) - 1u;
    } else {
        hb = 0;
#pragma unroll
        for (int j = 0; j < G; j++) hb |= (uint32_t)((hk[j] & mask) == 0u) << j;
    }
    const int lo = min(max((int)c.rlo - (int)rb, 0), G);
    const int hi = min(max((int)c.rhi - (int)rb, 0), G);
    hb &= ((1u << hi) - 1u) & ~((1u << lo) - 1u);
    if (hb) {
        c.count += __builtin_popcount(hb);
        c.last = rb + 31u - __builtin_clz(hb);
        if (c.first == kNone) c.first = rb + __builtin_ctz(hb);
    }
}

// 64 slides over unit `un` (bytes 64 back in `uo`), 64 / G groups of G.
// SMALL: mask < 0xFFFF, the prefilter then runs on h & mask (exact).
// G >= 100: groups of G - 100 that keep no fingerprints: a flagged lane
// re-rolls its group from the saved state (P ~ 2^-12 per lane-group).
template <int TSH, int G>
__device__ __forceinline__ void rescan_group(Chain &c, uint32_t h0, uint32_t h1, const Unit &un,
                                             const Unit &uo, const uint8_t *tab, const Consts &k,
                                             uint32_t rb, int g) {
#pragma unroll
    for (int j = 0; j < G; j++) {
        const int b = g * G + j;
        slide_b<TSH>(b, h0, h1, UDW(un, b >> 2), UDW(uo, b >> 2), tab, k);
        const uint32_t rel = rb + (uint32_t)j;
        if ((h0 & k.mask) == 0u && rel >= c.rlo && rel < c.rhi) {
            c.count++;
            c.last = rel;
            if (c.first == kNone) c.first = rel;
        }
    }
}

template <int TSH, bool SMALL, int G>
__device__ __forceinline__ void scan_unit(Chain &c, const Unit &un, const Unit &uo,
                                          const uint8_t *tab, const Consts &k, bool lv,
                                          uint32_t rb) {
    if constexpr (G >= 100) {
        constexpr int GG = G - 100;
#pragma unroll
        for (int g = 0; g < 64 / GG; g++) {
            const uint32_t h0s = c.h0, h1s = c.h1;
            uint16_t acc = 0xFFFFu;
#pragma unroll
            for (int j = 0; j < GG; j++) {
                const int b = g * GG + j;
                slide_b<TSH>(b, c.h0, c.h1, UDW(un, b >> 2), UDW(uo, b >> 2), tab, k);
                const uint16_t t = SMALL ? (uint16_t)(c.h0 & k.mask) : (uint16_t)c.h0;
                acc = __builtin_elementwise_min(acc, t);
            }
            // a divergent branch on the lane mask (exec-skip when no lane is
            // flagged): the compare is the only VALU of the test
            if (acc == 0 && lv) rescan_group<TSH, GG>(c, h0s, h1s, un, uo, tab, k, rb + g * GG, g);
        }
    } else {
#pragma unroll
    for (int g = 0; g < 64 / G; g++) {
        uint32_t hk[G];
        uint16_t acc = 0xFFFFu;
#pragma unroll
        for (int j = 0; j < G; j++) {
            const int b = g * G + j;
            slide_b<TSH>(b, c.h0, c.h1, UDW(un, b >> 2), UDW(uo, b >> 2), tab, k);
            hk[j] = c.h0;
            const uint16_t t = SMALL ? (uint16_t)(c.h0 & k.mask) : (uint16_t)c.h0;
            acc = __builtin_elementwise_min(acc, t);
        }
        // one ballot per group; the prefilter is necessary, not sufficient:
        // flagged lanes run the exact test
        if (acc == 0 && lv) record_group<G>(c, hk, k.mask, rb + g * G);
    }
    }
}

template <int TSH>
__device__ __forceinline__ void warm_unit(Chain &c, const Unit &u, const uint8_t *tab,
                                          const Consts &k) {
#pragma unroll
    for (int b = 0; b < 64; b++) {
        const uint32_t dn = UDW(u, b >> 2);
        switch (b & 3) {
            case 0: slide_in<0, TSH>(c.h0, c.h1, dn, tab, k); break;
            case 1: slide_in<1, TSH>(c.h0, c.h1, dn, tab, k); break;
            case 2: slide_in<2, TSH>(c.h0, c.h1, dn, tab, k); break;
            default: slide_in<3, TSH>(c.h0, c.h1, dn, tab, k); break;
        }
    }
}

__device__ __forceinline__ void load_unit(Unit &u, __amdgpu_buffer_rsrc_t rsrc, uint32_t voff) {
#pragma unroll
    for (int i = 0; i < 4; i++)
        u.v[i] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)(voff + 16u * i), 0, 0);
}

// Ring step: process unit i (buffer B = i % R, old = (i-1) % R), then refill
// the freed buffer(s) with unit i - 1 + R (PAIR: units i-2+R, i-1+R after
// even i, one 128-B line per lane).  Returns false after the last unit.
template <int R, bool PAIR, int TSH, bool SMALL, int G, int B>
__device__ __forceinline__ bool ring_step(Chain &c, Unit (&u)[R], uint32_t &i, uint32_t nunits,
                                          __amdgpu_buffer_rsrc_t rsrc, uint32_t voff,
                                          const uint8_t *tab, const Consts &k, bool lv) {
    scan_unit<TSH, SMALL, G>(c, u[B], u[(B + R - 1) % R], tab, k, lv, (i - 1) * 64u);
    if constexpr (PAIR) {
        if ((B & 1) == 0) {  // i even (R even, so B = i % R has i's parity)
            const uint32_t nxt = i - 2 + R;  // units nxt, nxt + 1 -> buffers B-2, B-1
            if (nxt <= nunits) {
                load_unit(u[(B + R - 2) % R], rsrc, voff + nxt * 64u);
                load_unit(u[(B + R - 1) % R], rsrc, voff + (nxt + 1) * 64u);
            }
        }
    } else {
        const uint32_t nxt = i - 1 + R;
        if (nxt <= nunits) load_unit(u[(B + R - 1) % R], rsrc, voff + nxt * 64u);
    }
    return ++i <= nunits;
}

template <int R, bool PAIR, int TSH, bool SMALL, int G, int B = 1>
__device__ __forceinline__ bool ring_pass(Chain &c, Unit (&u)[R], uint32_t &i, uint32_t nunits,
                                          __amdgpu_buffer_rsrc_t rsrc, uint32_t voff,
                                          const uint8_t *tab, const Consts &k, bool lv) {
    if (!ring_step<R, PAIR, TSH, SMALL, G, B % R>(c, u, i, nunits, rsrc, voff, tab, k, lv))
        return false;
    if constexpr (B < R) return ring_pass<R, PAIR, TSH, SMALL, G, B + 1>(c, u, i, nunits, rsrc,
                                                                        voff, tab, k, lv);
    else return true;
}

// One lane's segment: bytes [voff, voff + 64 + S) of `rsrc` (64 warm-up
// bytes, then S = 64 * nunits tested positions); positions rlo .. rhi - 1
// (segment-relative) count.  `valid`: lanes of the wave with a segment.
template <int R, bool PAIR, int TSH, bool SMALL, int G>
__device__ __forceinline__ Chain scan_segment(__amdgpu_buffer_rsrc_t rsrc, uint32_t voff,
                                              uint32_t nunits, uint32_t rlo, uint32_t rhi,
                                              const uint8_t *tab, const Consts &k, uint64_t valid,
                                              uint32_t lane) {
    Chain c;
    c.h0 = c.h1 = 0;
    c.first = c.last = kNone;
    c.count = 0;
    c.rlo = rlo;
    c.rhi = rhi;
    Unit u[R];
#pragma unroll
    for (int j = 0; j < R; j++)
        if ((uint32_t)j <= nunits) load_unit(u[j], rsrc, voff + j * 64u);
    warm_unit<TSH>(c, u[0], tab, k);
    const bool lv = (valid >> lane) & 1u;
    uint32_t i = 1;
    while (ring_pass<R, PAIR, TSH, SMALL, G>(c, u, i, nunits, rsrc, voff, tab, k, lv)) {
    }
    return c;
}

// scan_segment that stops early (the walk's hit rounds): after each ring pass,
// when a lane below 32 has a hit and at least 4 units per lane are left, it
// returns with *done = the units every lane tested (else nunits).  The lanes
// before the first hit lane then owe the rest of their segments, which the
// caller spreads over all 64 lanes (walk round_first).
template <int R, bool PAIR, int TSH, bool SMALL, int G>
__device__ __forceinline__ Chain scan_segment_early(__amdgpu_buffer_rsrc_t rsrc, uint32_t voff,
                                                    uint32_t nunits, uint32_t rlo, uint32_t rhi,
                                                    const uint8_t *tab, const Consts &k,
                                                    uint64_t valid, uint32_t lane, uint32_t &done,
                                                    bool may_stop) {
    Chain c;
    c.h0 = c.h1 = 0;
    c.first = c.last = kNone;
    c.count = 0;
    c.rlo = rlo;
    c.rhi = rhi;
    Unit u[R];
#pragma unroll
    for (int j = 0; j < R; j++)
        if ((uint32_t)j <= nunits) load_unit(u[j], rsrc, voff + j * 64u);
    warm_unit<TSH>(c, u[0], tab, k);
    const bool lv = (valid >> lane) & 1u;
    uint32_t i = 1;
    done = nunits;
    while (ring_pass<R, PAIR, TSH, SMALL, G>(c, u, i, nunits, rsrc, voff, tab, k, lv)) {
        const uint64_t hb = __builtin_amdgcn_ballot_w64(c.first != kNone) & valid;
        if (may_stop && hb && __builtin_ctzll(hb) < 32 && nunits - (i - 1) >= 4) {
            done = i - 1;
            break;
        }
    }
    return c;
}

// Kernel prologue: 32 lane-private copies of OM and MOD into LDS (entry e of
// copy c at e * 256 + c * 8; MOD kTableBytes further).  OM[e] = OUT'[e]
// reduced: the top byte of out << 8 sits at bits deg .. deg + 7 and MOD's
// (i << deg) term cancels it.  idx_shift = deg - 32 mod 2^32 (wraps for
// deg < 32; idx_shift + 32 = deg either way).  Ends with a workgroup barrier.
//
// In three LDS steps: the 512 global words are read once (one load per
// thread, not a dependent pair per copy: the prologue is on the critical
// path of short launches -- C5's walk and check, C2's scan), OM is formed in
// copy 0, and copy 0 is replicated.
#ifdef RCDC_AB_FILL_DIRECT  // A/B only (tools/ab_lib.sh): round 5's direct fill
__device__ __forceinline__ void fill_tables(uint8_t *s_tab, const uint64_t *__restrict__ gtab,
                                            uint32_t idx_shift, uint32_t tid, uint32_t nthreads) {
    for (uint32_t i = tid; i < 256u * kTableRepl; i += nthreads) {
        const uint32_t e = i / kTableRepl, c = i % kTableRepl;
        const uint64_t ot = gtab[e], m = gtab[256 + e];
        const uint64_t o = ot ^ gtab[256 + ((ot >> (idx_shift + 32u)) & 255u)];
        *reinterpret_cast<uint2 *>(s_tab + e * 256u + c * 8u) =
            make_uint2((uint32_t)o, (uint32_t)(o >> 32));
        *reinterpret_cast<uint2 *>(s_tab + kTableBytes + e * 256u + c * 8u) =
            make_uint2((uint32_t)m, (uint32_t)(m >> 32));
    }
    __syncthreads();
}
#else
__device__ __forceinline__ void fill_tables(uint8_t *s_tab, const uint64_t *__restrict__ gtab,
                                            uint32_t idx_shift, uint32_t tid, uint32_t nthreads) {
    static_assert(kTableRepl == 32, "copy layout: entry e, copy c at e * 256 + c * 8");
    uint2 *om = reinterpret_cast<uint2 *>(s_tab);
    uint2 *md = reinterpret_cast<uint2 *>(s_tab + kTableBytes);
    // 1. raw OUT[e] into OM copy 1 (overwritten in step 3), MOD[e] into MOD copy 0
    for (uint32_t i = tid; i < 512u; i += nthreads) {
        const uint64_t v = gtab[i];
        const uint2 w = make_uint2((uint32_t)v, (uint32_t)(v >> 32));
        if (i < 256u) om[i * 32u + 1u] = w;
        else md[(i - 256u) * 32u] = w;
    }
    __syncthreads();
    // 2. OM[e] = OUT[e] ^ MOD[top(OUT[e])] (idx_shift + 32 = deg) into copy 0
    for (uint32_t e = tid; e < 256u; e += nthreads) {
        const uint2 ot = om[e * 32u + 1u];
        const uint32_t idx = (uint32_t)(((((uint64_t)ot.y << 32) | ot.x) >> (idx_shift + 32u)) & 255u);
        const uint2 mt = md[idx * 32u];
        om[e * 32u] = make_uint2(ot.x ^ mt.x, ot.y ^ mt.y);
    }
    __syncthreads();
    // 3. copies 1 .. 31 of both tables from copy 0
    for (uint32_t i = tid; i < 256u * 32u; i += nthreads) {
        const uint32_t e = i >> 5, c = i & 31u;
        if (c) {
            om[i] = om[e * 32u];
            md[i] = md[e * 32u];
        }
    }
    __syncthreads();
}
#endif

__device__ __forceinline__ Consts make_consts(uint32_t lane, uint32_t mask, uint32_t idx_shift) {
    Consts k;
    k.lwo = (lane & 31u) * 8u;
    k.lwm = k.lwo | kTableBytes;
    k.kff00 = in_vgpr(0xFF00u);
    k.mask = in_vgpr(mask);
    k.tsh = idx_shift + 24u;  // deg - 8
    return k;
}

}  // namespace
