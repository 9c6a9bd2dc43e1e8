// rcdc_scan.hip -- scan kernel of the rcdc chunker (gfx950).
//
// Replaces the per-byte hot loop of crates/core/src/chunker/rabin.rs:153-188
// (rustic_cdc Rabin64::slide + `hash & split_mask == 0`): every lane owns one
// S-byte segment of one stream, rolls the 64-byte-window Rabin64 fingerprint
// over it and records the first / last / number of candidate positions
// (fp(b[p-64, p)) & mask == 0).  Output format as rcdc_internal.h.
//
// Cost model (profiles/r01_slide_bench*.txt): the loop is VALU-issue bound at
// ~8 VALU + 2 ds_read_b64 per byte; the LDS array is at ~40 % and HBM at
// ~45 % of their peaks.  Choices that follow from it:
//   * candidate test: a v_min3_u16 over the low halves of 16 consecutive
//     fingerprints (0.5 VALU/byte) and ONE wave ballot per 16 bytes; the
//     exact test (h & mask) == 0 runs only on the rare groups whose minimum
//     is 0 (P ~ 2^-12 per lane-group for mask >= 0xFFFF).  The per-byte
//     and + v_cmp + s_or form it replaces cost 2-3x as much.
//   * every operand of the hot loop is a VGPR or an inline constant (SGPR
//     operands and 64-bit shifts issue at half rate on gfx950).
//   * loads: each lane streams its own segment in 64-B units (4 x
//     buffer_load_dwordx4 into one cache-line half: the runtime aligns lane
//     starts to 64 B), a ring of R units so loads run R-2 units ahead; no
//     load beyond the segment.  PAIR issues two units (one 128-B line) at
//     once; it only paid off while lane starts were unaligned.
#include <hip/hip_runtime.h>

#include "rcdc_internal.h"

using namespace rcdc;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

namespace {

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

__device__ __forceinline__ uint2 lds_u2(const uint8_t *tab, uint32_t byte_addr) {
    return *reinterpret_cast<const uint2 *>(tab + byte_addr);
}

struct Unit {
    u32x4 v[4];
};
#define UDW(u, d) ((u).v[(d) >> 2][(d) & 3])

struct Consts {
    uint32_t lwo, lwm;  // lane's table-copy offset in OUT / MOD
    uint32_t kff00;     // 0xFF00 in a VGPR
    uint32_t mask;      // avg - 1 in a VGPR
    uint32_t tsh;       // deg - 32 (generic-degree path only)
};

// MOD table address of the top byte of h (h1 = hi32(h), a1 = hi32(h << 8)).
// TSH >= 100: compile-time shift TSH - 100 = deg - 48 straight from h1, so the
//   address does not wait for the v_alignbit (critical path per byte:
//   v_lshrrev, v_bitop3, ds_read_b64, v_bitop3);
// 0 <= TSH < 100: compile-time deg - 40 from a1 (v_lshrrev by an inline
//   constant + one v_bitop3 (x & 0xFF00) | lwm);
// TSH < 0: any degree, runtime shift of a1.
template <int TSH>
__device__ __forceinline__ uint32_t mod_addr(uint32_t h1, uint32_t a1, const Consts &k) {
    if constexpr (TSH >= 100)
        return __builtin_amdgcn_bitop3_b32(h1 >> (TSH - 100), k.kff00, k.lwm, kAndOr);
    else if constexpr (TSH >= 0)
        return __builtin_amdgcn_bitop3_b32(a1 >> TSH, k.kff00, k.lwm, kAndOr);
    else
        return ((a1 >> k.tsh) << 8) | k.lwm;
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
    const uint2 m = lds_u2(tab, mod_addr<TSH>(h1, a1, k));
    h0 = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_perm(h0, dnew, 0x06050400u | K), o.x, m.x, kXor3);
    h1 = __builtin_amdgcn_bitop3_b32(a1, o.y, m.y, kXor3);
}

// Warm-up slide (the window is still filling: nothing leaves it).
template <int K, int TSH>
__device__ __forceinline__ void slide_in(uint32_t &h0, uint32_t &h1, uint32_t dnew,
                                         const uint8_t *tab, const Consts &k) {
    const uint32_t a1 = __builtin_amdgcn_alignbit(h1, h0, 24);
    const uint2 m = lds_u2(tab, mod_addr<TSH>(h1, a1, k));
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
                                          const uint8_t *tab, const Consts &k, uint64_t valid,
                                          uint32_t lane, uint32_t rb) {
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
            const uint64_t flagged = __builtin_amdgcn_ballot_w64(acc == 0) & valid;
            if (flagged) {
                if ((flagged >> lane) & 1u)
                    rescan_group<TSH, GG>(c, h0s, h1s, un, uo, tab, k, rb + g * GG, g);
            }
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
        const uint64_t flagged = __builtin_amdgcn_ballot_w64(acc == 0) & valid;
        if (flagged) {
            if ((flagged >> lane) & 1u) record_group<G>(c, hk, k.mask, rb + g * G);
        }
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
                                          const uint8_t *tab, const Consts &k, uint64_t valid,
                                          uint32_t lane) {
    scan_unit<TSH, SMALL, G>(c, u[B], u[(B + R - 1) % R], tab, k, valid, lane, (i - 1) * 64u);
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
                                          const uint8_t *tab, const Consts &k, uint64_t valid,
                                          uint32_t lane) {
    if (!ring_step<R, PAIR, TSH, SMALL, G, B % R>(c, u, i, nunits, rsrc, voff, tab, k, valid, lane))
        return false;
    if constexpr (B < R) return ring_pass<R, PAIR, TSH, SMALL, G, B + 1>(c, u, i, nunits, rsrc,
                                                                        voff, tab, k, valid, lane);
    else return true;
}

// One wave scans one item (64 segments): lane l owns segment l.
template <int R, bool PAIR, int TSH, bool SMALL, int G>
__device__ __forceinline__ void scan_item(const uint8_t *__restrict__ arena, const ScanItem &item,
                                          uint32_t lane, const uint8_t *tab, const Consts &k,
                                          uint32_t S, uint4 *__restrict__ sums,
                                          uint64_t *__restrict__ item_mask) {
    const uint32_t nunits = S / kUnit;  // plus unit 0 = the 64-byte warm-up window
    const uint64_t segpos = item.pos0 + (uint64_t)lane * S;
    const bool lv = lane < item.nvalid;
    const uint64_t valid = __builtin_amdgcn_ballot_w64(lv);
    Chain c;
    c.h0 = c.h1 = 0;
    c.first = c.last = kNone;
    c.count = 0;
    c.rlo = (lv && item.lo > segpos) ? (uint32_t)min(item.lo - segpos, (uint64_t)S) : 0u;
    c.rhi = (lv && item.hi > segpos) ? (uint32_t)min(item.hi - segpos, (uint64_t)S) : 0u;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(arena + item.q0), (short)0, (int)(uint32_t)item.rec_bytes, 0x00020000);
    const uint32_t voff = lane * S;

    Unit u[R];
#pragma unroll
    for (int j = 0; j < R; j++)
        if ((uint32_t)j <= nunits) load_unit(u[j], rsrc, voff + j * 64u);
    warm_unit<TSH>(c, u[0], tab, k);
    uint32_t i = 1;
    while (ring_pass<R, PAIR, TSH, SMALL, G>(c, u, i, nunits, rsrc, voff, tab, k, valid, lane)) {
    }
    if (lv) sums[item.sum_idx + lane] = make_uint4(c.first, c.last, c.count, 0u);
    const uint64_t hits = __builtin_amdgcn_ballot_w64(c.count != 0u) & valid;
    if (lane == 0) *item_mask = hits;
}

}  // namespace

// One workgroup of THREADS lanes per CU; 128 KiB of LDS tables (32
// lane-private copies of OUT' and MOD: ds_read_b64 never bank-conflicts).
template <int R, bool PAIR, int THREADS, int TSH, bool SMALL, int G>
__global__ __launch_bounds__(THREADS, 1) void rcdc_scan_kernel(
    const uint8_t *__restrict__ arena, const ScanItem *__restrict__ items, uint32_t nitems,
    const uint64_t *__restrict__ gtab, ScanParams prm, uint4 *__restrict__ sums,
    uint64_t *__restrict__ item_masks) {
    __shared__ __attribute__((aligned(16))) uint8_t s_tab[kLdsBytes];
    for (uint32_t i = threadIdx.x; i < 256u * kTableRepl; i += THREADS) {
        const uint32_t e = i / kTableRepl, c = i % kTableRepl;
        // OM[e] = OUT'[e] reduced: the top byte of out << 8 sits at bits
        // deg .. deg + 7 and MOD's (i << deg) term cancels it
        const uint64_t ot = gtab[e], m = gtab[256 + e];
        const uint64_t o = ot ^ gtab[256 + ((ot >> (prm.idx_shift + 32u)) & 255u)];
        *reinterpret_cast<uint2 *>(s_tab + e * 256u + c * 8u) =
            make_uint2((uint32_t)o, (uint32_t)(o >> 32));
        *reinterpret_cast<uint2 *>(s_tab + kTableBytes + e * 256u + c * 8u) =
            make_uint2((uint32_t)m, (uint32_t)(m >> 32));
    }
    __syncthreads();

    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = threadIdx.x >> 6;
    constexpr uint32_t kWaves = THREADS / 64;
    Consts k;
    k.lwo = (lane & 31u) * 8u;
    k.lwm = k.lwo | kTableBytes;
    k.kff00 = in_vgpr(0xFF00u);
    k.mask = in_vgpr(prm.mask);
    k.tsh = prm.idx_shift;
    for (uint32_t it = blockIdx.x * kWaves + wave; it < nitems; it += gridDim.x * kWaves) {
        const uint32_t iu = __builtin_amdgcn_readfirstlane(it);
        scan_item<R, PAIR, TSH, SMALL, G>(arena, items[iu], lane, s_tab, k, prm.seg_bytes, sums,
                                       item_masks + iu);
    }
}

namespace rcdc {

// Kernel configuration `code` (RCDC_SCAN_VARIANT, default kDefaultScanCode):
// 100 * (group == 8) + 10 * ring + pair; + 1000: 768 threads; 3116: groups of
// 16 re-rolled on a flag instead of kept; 930: MOD index from hi32(h << 8)
// (the pre-OM form's index).  Measured on the C2 workload with 64-B aligned
// lane starts, HIP-event medians in one process (tools/variants.py,
// profiles/r01_scan_variants.txt):
//   before the OM table: 30 174 us, 130 the same, 41 193 us, 50 204 us;
//   OM table, MOD index from hi32(h << 8) (930): 164 us;
//   OM table, MOD index from h1 (30, default): 161-165 us; 130 170 us;
//   3116 168 us; no candidate test at all (cost floor, wrong output) 157 us.
// deg 53 uses the compile-time index shift, other degrees the generic path;
// avg < 2^16 the masked prefilter.
template <int R, bool PAIR, int THREADS, int G, bool HIDX = true>
static hipError_t launch4(const uint8_t *arena, const ScanItem *items, uint32_t nitems,
                          const uint64_t *gtab, const ScanParams &prm, uint4 *sums,
                          uint64_t *item_masks, uint32_t blocks, hipStream_t stream) {
    const bool small = prm.mask < 0xFFFFu;
    if (prm.idx_shift == 21 && !small)
        hipLaunchKernelGGL((rcdc_scan_kernel<R, PAIR, THREADS, HIDX ? 105 : 13, false, G>), dim3(blocks),
                           dim3(THREADS), 0, stream, arena, items, nitems, gtab, prm, sums,
                           item_masks);
    else if (small)
        hipLaunchKernelGGL((rcdc_scan_kernel<R, PAIR, THREADS, -1, true, G>), dim3(blocks),
                           dim3(THREADS), 0, stream, arena, items, nitems, gtab, prm, sums,
                           item_masks);
    else
        hipLaunchKernelGGL((rcdc_scan_kernel<R, PAIR, THREADS, -1, false, G>), dim3(blocks),
                           dim3(THREADS), 0, stream, arena, items, nitems, gtab, prm, sums,
                           item_masks);
    return hipGetLastError();
}

int scan_threads(int code) { return (code >= 1000 && code < 2000) ? 768 : 1024; }

hipError_t launch_scan(int code, const uint8_t *arena, const ScanItem *items, uint32_t nitems,
                        const uint64_t *gtab, const ScanParams &prm, uint4 *sums,
                        uint64_t *item_masks, uint32_t blocks, hipStream_t stream) {
    if (nitems == 0) return hipSuccess;
    switch (code) {
        case 30: return launch4<3, false, 1024, 16>(arena, items, nitems, gtab, prm, sums, item_masks, blocks, stream);
        case 3116: return launch4<3, false, 1024, 116>(arena, items, nitems, gtab, prm, sums, item_masks, blocks, stream);
        case 930: return launch4<3, false, 1024, 16, false>(arena, items, nitems, gtab, prm, sums, item_masks, blocks, stream);
        case 50: return launch4<5, false, 1024, 16>(arena, items, nitems, gtab, prm, sums, item_masks, blocks, stream);
        case 150: return launch4<5, false, 1024, 8>(arena, items, nitems, gtab, prm, sums, item_masks, blocks, stream);
        case 130: return launch4<3, false, 1024, 8>(arena, items, nitems, gtab, prm, sums, item_masks, blocks, stream);
        case 41: return launch4<4, true, 1024, 16>(arena, items, nitems, gtab, prm, sums, item_masks, blocks, stream);
        case 141: return launch4<4, true, 1024, 8>(arena, items, nitems, gtab, prm, sums, item_masks, blocks, stream);
        case 1161: return launch4<6, true, 768, 8>(arena, items, nitems, gtab, prm, sums, item_masks, blocks, stream);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace rcdc
