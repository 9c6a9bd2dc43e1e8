// rcdc_scan.hip -- the candidate-scan kernel (gfx950), v3.
//
// Replaces the per-byte loop of crates/core/src/chunker/rabin.rs:153-188
// (rustic_cdc Rabin64::slide + `hash & split_mask == 0`): every lane owns one
// S-byte segment of one stream, rolls the 64-byte-window Rabin64 fingerprint
// over it and records first / last / number of candidate positions.
//
// Design points (measured on MI355X, see DESIGN.md "Scan kernel"):
//  * VALU-issue bound: wave64 v_xor/v_and/v_or/shift-by-constant and
//    v_bitop3 (VGPR operands) issue at ~2 cycles per SIMD, v_perm /
//    v_alignbit / v_cmp / any SGPR-operand op at ~4.  The byte step uses
//    2 v_perm + 1 v_alignbit + 1 v_cmp + 6 fast ops; constants live in VGPRs.
//  * Loads: lanes l and l+32 read the two 16-byte halves of one 32-byte piece
//    of segment (l mod 32) -- one instruction covers 32 x 32 contiguous bytes
//    instead of 64 scattered lines -- and one v_permlane32_swap per dword
//    gives every lane its own segment's bytes back.
//  * NC independent segments ("chains") per lane interleave their dependency
//    chains (LDS lookup -> 4 VALU -> LDS lookup) for latency hiding.
//  * Tables: 32 lane-private copies of OUT' (out[b] << 8) and MOD in LDS
//    (128 KiB), entry e of copy c at e*256 + c*8: ds_read_b64 is conflict-free
//    whatever the data.
#include <hip/hip_runtime.h>

#include "rcdc_internal.h"

using namespace rcdc;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

namespace {

constexpr uint32_t kLutA = 0xF0, kLutB = 0xCC, kLutC = 0xAA;  // v_bitop3 operand LUTs

// Materialise a value in a VGPR the compiler cannot turn back into an SGPR
// or an inline constant (SGPR operands halve the VALU issue rate).
__device__ __forceinline__ uint32_t in_vgpr(uint32_t x) {
    uint32_t r;
    asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "s"(x));
    return r;
}

__device__ __forceinline__ uint2 lds_u2(const uint8_t *tab, uint32_t byte_addr) {
    return *reinterpret_cast<const uint2 *>(tab + byte_addr);
}

// 32 bytes of one lane's segment: dwords 0..3 then 4..7.
struct Unit32 {
    u32x4 a, b;
};
template <int D>
__device__ __forceinline__ uint32_t dw(const Unit32 &u) {
    if constexpr (D < 4) return u.a[D];
    else return u.b[D - 4];
}

// Issue the two paired loads of a 32-byte unit (see header).
__device__ __forceinline__ void load_unit(Unit32 &u, __amdgpu_buffer_rsrc_t rsrc, uint32_t voffa,
                                          uint32_t pair_stride, uint32_t off) {
    u.a = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)(voffa + off), 0, 0);
    u.b = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)(voffa + pair_stride + off), 0, 0);
}

// After the loads land: lane l < 32 holds (seg l: bytes 0-15, seg l+32: 0-15),
// lane l+32 holds (seg l: 16-31, seg l+32: 16-31); swap the cross halves.
__device__ __forceinline__ void fix_unit(Unit32 &u) {
#pragma unroll
    for (int i = 0; i < 4; i++) {
        auto r = __builtin_amdgcn_permlane32_swap(u.a[i], u.b[i], false, false);
        u.a[i] = r[0];
        u.b[i] = r[1];
    }
}

// Adjacent-lane pairing: lanes 2p and 2p+1 read the two 16-byte halves of a
// 32-byte piece of segment 2p (first load) and of segment 2p+1 (second load);
// the 2x2 exchange is one DPP (quad_perm swap) v_cndmask per dword.
__device__ __forceinline__ void fix_unit_adjacent(Unit32 &u, uint64_t even, uint64_t odd) {
    uint32_t c0, c1, c2, c3, d0, d1, d2, d3;
    asm volatile(
        "s_mov_b64 vcc, %16\n\t"
        "s_nop 1\n\t"
        "v_cndmask_b32_dpp %0, %12, %8, vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_cndmask_b32_dpp %1, %13, %9, vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_cndmask_b32_dpp %2, %14, %10, vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_cndmask_b32_dpp %3, %15, %11, vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "s_mov_b64 vcc, %17\n\t"
        "s_nop 1\n\t"
        "v_cndmask_b32_dpp %4, %8, %12, vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_cndmask_b32_dpp %5, %9, %13, vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_cndmask_b32_dpp %6, %10, %14, vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_cndmask_b32_dpp %7, %11, %15, vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
        : "=&v"(c0), "=&v"(c1), "=&v"(c2), "=&v"(c3), "=&v"(d0), "=&v"(d1), "=&v"(d2), "=&v"(d3)
        : "v"(u.a[0]), "v"(u.a[1]), "v"(u.a[2]), "v"(u.a[3]), "v"(u.b[0]), "v"(u.b[1]),
          "v"(u.b[2]), "v"(u.b[3]), "s"(even), "s"(odd)
        : "vcc");
    u.a[0] = c0; u.a[1] = c1; u.a[2] = c2; u.a[3] = c3;
    u.b[0] = d0; u.b[1] = d1; u.b[2] = d2; u.b[3] = d3;
}

struct Consts {
    uint32_t lwo, lwm;  // lane part of the OUT / MOD table addresses
    uint32_t kff00;     // 0xFF00 in a VGPR
    uint32_t mask;      // split mask (avg - 1) in a VGPR
    uint32_t tsh;       // deg - 40: top byte of h from hi32(h << 8) >> tsh
    uint64_t even, odd; // lane masks for the adjacent-pair exchange
};

// Warm-up slide (window still filling: nothing leaves).
template <int K>
__device__ __forceinline__ void slide_warm(uint32_t &h0, uint32_t &h1, uint32_t dnew,
                                           const uint8_t *tab, const Consts &k) {
    const uint32_t a1 = __builtin_amdgcn_alignbit(h1, h0, 24);
    const uint32_t am = __builtin_amdgcn_bitop3_b32(a1 >> k.tsh, k.kff00, k.lwm,
                                                    (kLutA & kLutB) | kLutC);
    const uint2 m = lds_u2(tab, am);
    h0 = __builtin_amdgcn_perm(h0, dnew, 0x06050400u | K) ^ m.x;
    h1 = a1 ^ m.y;
}

// One Rabin64 slide: h ^= out[o]; i = top byte; h = ((h<<8)|n) ^ mod[i].
//   a1x = hi32(h << 8) ^ hi32(out[o] << 8)        v_alignbit, v_xor
//   am  = ((a1x >> (deg-40)) & 0xFF00) | lwm       v_lshrrev, v_bitop3   (MOD address)
//   h1  = a1x ^ hi32(mod[i])                       v_xor   (mod[i] carries i << deg)
//   h0  = ((h0 << 8) | n) ^ lo32(out<<8) ^ lo32(mod[i])   v_perm, v_bitop3
// ABL (timing-only ablations, wrong results): bit 1 = no LDS lookups.
template <int ABL>
__device__ __forceinline__ uint2 lookup(const uint8_t *tab, uint32_t a) {
    if constexpr (ABL & 2) {
        return make_uint2(a * 0x9E3779B1u, a ^ 0x7F4A7C15u);
    } else {
        return lds_u2(tab, a);
    }
}

template <int K, int ABL = 0>
__device__ __forceinline__ void slide(uint32_t &h0, uint32_t &h1, uint32_t dnew, uint32_t dold,
                                      const uint8_t *tab, const Consts &k) {
    const uint2 o = lookup<ABL>(tab, __builtin_amdgcn_perm(dold, k.lwo, 0x0C0C0000u | ((4u + K) << 8)));
    const uint32_t a1x = __builtin_amdgcn_alignbit(h1, h0, 24) ^ o.y;
    const uint32_t am = __builtin_amdgcn_bitop3_b32(a1x >> k.tsh, k.kff00, k.lwm,
                                                    (kLutA & kLutB) | kLutC);
    const uint2 m = lookup<ABL>(tab, am);
    h0 = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_perm(h0, dnew, 0x06050400u | K), o.x, m.x,
                                     kLutA ^ kLutB ^ kLutC);
    h1 = a1x ^ m.y;
}

struct Chain {
    uint32_t h0, h1;
    uint32_t first, last, count;  // candidates, relative positions
    uint32_t rlo, rhi;            // relative positions that count
    Unit32 u[4];                  // rotating 32-byte units
};

// hb = 2*hb + (this lane's bit of m)
__device__ __forceinline__ uint32_t shift_in(uint32_t hb, uint64_t m) {
    uint32_t r;
    asm("v_addc_co_u32 %0, vcc, %1, %1, %2" : "=v"(r) : "v"(hb), "s"(m) : "vcc");
    return r;
}

// Rare path: lanes of this chain saw candidates at rb + j, j < 8 (m[j]).
__device__ __forceinline__ void record_hits(Chain &c, const uint64_t (&m)[8], uint32_t rb) {
    uint32_t hb = 0;
#pragma unroll
    for (int j = 7; j >= 0; j--) hb = shift_in(hb, m[j]);  // bit j <-> position rb + j
    const int lo = min(max((int)c.rlo - (int)rb, 0), 8);
    const int hi = min(max((int)c.rhi - (int)rb, 0), 8);
    hb &= ((1u << hi) - 1u) & ~((1u << lo) - 1u);
    if (hb) {
        c.count += __builtin_popcount(hb);
        c.last = rb + 31u - __builtin_clz(hb);
        if (c.first == kNone) c.first = rb + __builtin_ctz(hb);
    }
}

template <int NC, int B, int IN, int IO, int ABL>
__device__ __forceinline__ void step_all(Chain (&ch)[NC], const uint8_t *tab, const Consts &k,
                                         uint64_t (&m)[NC][8], int j) {
#pragma unroll
    for (int c = 0; c < NC; c++) {
        const uint32_t dn = dw<(B >> 2)>(ch[c].u[IN]);
        const uint32_t d_o = dw<(B >> 2)>(ch[c].u[IO]);
        slide<(B & 3), ABL>(ch[c].h0, ch[c].h1, dn, d_o, tab, k);
        if constexpr (ABL & 4) m[c][j] = 0;  // ablation: no test
        else m[c][j] = __builtin_amdgcn_ballot_w64((ch[c].h0 & k.mask) == 0u);
    }
}

// Bytes [B, E) of the current unit for every chain (compile-time unrolled).
template <int NC, int B, int E, int IN, int IO, int ABL>
__device__ __forceinline__ void steps(Chain (&ch)[NC], const uint8_t *tab, const Consts &k,
                                      uint64_t (&m)[NC][8]) {
    if constexpr (B < E) {
        step_all<NC, B, IN, IO, ABL>(ch, tab, k, m, B & 7);
        steps<NC, B + 1, E, IN, IO, ABL>(ch, tab, k, m);
    }
}

template <int NC, int G, int IN, int IO, int ABL>
__device__ __forceinline__ void scan_group(Chain (&ch)[NC], const uint8_t *tab, const Consts &k,
                                           const uint64_t (&valid)[NC], uint32_t rb) {
    uint64_t m[NC][8];
    steps<NC, G * 8, G * 8 + 8, IN, IO, ABL>(ch, tab, k, m);
#pragma unroll
    for (int c = 0; c < NC; c++) {
        uint64_t any = m[c][0];
#pragma unroll
        for (int j = 1; j < 8; j++) any |= m[c][j];
        if (any & valid[c]) record_hits(ch[c], m[c], rb + G * 8);
    }
}

// 32 slides per chain: new bytes in unit IN, bytes 64 earlier in unit IO.
template <int NC, int IN, int IO, int ABL>
__device__ __forceinline__ void scan_unit(Chain (&ch)[NC], const uint8_t *tab, const Consts &k,
                                          const uint64_t (&valid)[NC], uint32_t rb) {
    if constexpr (!(ABL & 8)) {
#pragma unroll
        for (int c = 0; c < NC; c++) {
            if constexpr (ABL & 16) fix_unit(ch[c].u[IN]);
            else fix_unit_adjacent(ch[c].u[IN], k.even, k.odd);
        }
    }
    scan_group<NC, 0, IN, IO, ABL>(ch, tab, k, valid, rb);
    scan_group<NC, 1, IN, IO, ABL>(ch, tab, k, valid, rb);
    scan_group<NC, 2, IN, IO, ABL>(ch, tab, k, valid, rb);
    scan_group<NC, 3, IN, IO, ABL>(ch, tab, k, valid, rb);
}

template <int NC, int IN, int ABL>
__device__ __forceinline__ void warm_unit(Chain (&ch)[NC], const uint8_t *tab, const Consts &k) {
#pragma unroll
    for (int c = 0; c < NC; c++) {
        if constexpr (ABL & 16) fix_unit(ch[c].u[IN]);
        else fix_unit_adjacent(ch[c].u[IN], k.even, k.odd);
    }
#pragma unroll
    for (int b = 0; b < 32; b++) {
#pragma unroll
        for (int c = 0; c < NC; c++) {
            const Unit32 &u = ch[c].u[IN];
            const uint32_t dn = (b >> 2) < 4 ? u.a[(b >> 2) & 3] : u.b[(b >> 2) & 3];
            switch (b & 3) {
                case 0: slide_warm<0>(ch[c].h0, ch[c].h1, dn, tab, k); break;
                case 1: slide_warm<1>(ch[c].h0, ch[c].h1, dn, tab, k); break;
                case 2: slide_warm<2>(ch[c].h0, ch[c].h1, dn, tab, k); break;
                default: slide_warm<3>(ch[c].h0, ch[c].h1, dn, tab, k); break;
            }
        }
    }
}

// Scan NC items (64 segments each) with one wave; lane l owns segment l.
template <int NC, int ABL = 0>
__device__ __forceinline__ void scan_items(const uint8_t *__restrict__ arena,
                                           const ScanItem *__restrict__ items, uint32_t it0,
                                           uint32_t lane, const uint8_t *tab, const Consts &k,
                                           uint32_t S, uint4 *__restrict__ sums,
                                           uint64_t *__restrict__ item_masks) {
    Chain ch[NC];
    __amdgpu_buffer_rsrc_t rsrc[NC];
    uint64_t valid[NC];
    uint64_t sum_idx[NC];
    // ABL & 16 (old scheme): lane l reads half (l >> 5) of segment (l & 31)
    // and of segment (l & 31) + 32.  Default: lanes 2p, 2p+1 read the halves
    // of segment 2p, then of segment 2p+1.
    const uint32_t voffa = (ABL & 16) ? (lane & 31u) * S + (lane >> 5) * 16u
                                      : (lane & ~1u) * S + (lane & 1u) * 16u;
    const uint32_t pstride = (ABL & 16) ? 32u * S : S;
    const uint32_t nunits = S / 32u;
#pragma unroll
    for (int c = 0; c < NC; c++) {
        const ScanItem item = items[it0 + c];
        const uint64_t segpos = item.pos0 + (uint64_t)lane * S;
        const bool lv = lane < item.nvalid;
        valid[c] = __builtin_amdgcn_ballot_w64(lv);
        ch[c].h0 = ch[c].h1 = 0;
        ch[c].first = ch[c].last = kNone;
        ch[c].count = 0;
        ch[c].rlo = (lv && item.lo > segpos) ? (uint32_t)min(item.lo - segpos, (uint64_t)S) : 0u;
        ch[c].rhi = (lv && item.hi > segpos) ? (uint32_t)min(item.hi - segpos, (uint64_t)S) : 0u;
        sum_idx[c] = item.sum_idx;
        rsrc[c] = __builtin_amdgcn_make_buffer_rsrc((void *)(arena + item.q0), (short)0,
                                                    (int)(uint32_t)item.rec_bytes, 0x00020000);
        load_unit(ch[c].u[0], rsrc[c], voffa, pstride, 0u);    // warm-up bytes 0-31
        load_unit(ch[c].u[1], rsrc[c], voffa, pstride, 32u);   // warm-up bytes 32-63
        load_unit(ch[c].u[2], rsrc[c], voffa, pstride, 64u);   // first tested unit
        load_unit(ch[c].u[3], rsrc[c], voffa, pstride, 96u);
    }
    warm_unit<NC, 0, ABL>(ch, tab, k);
    warm_unit<NC, 1, ABL>(ch, tab, k);

    // unit u (u >= 2) uses new = u[u%4], old = u[(u-2)%4]; afterwards the old
    // buffer takes unit u+2.
    uint32_t u = 2, rb = 0;
    for (;;) {
        scan_unit<NC, 2, 0, ABL>(ch, tab, k, valid, rb);
#pragma unroll
        for (int c = 0; c < NC; c++)
            if constexpr (!(ABL & 1)) load_unit(ch[c].u[0], rsrc[c], voffa, pstride, (u + 2) * 32u);
        rb += 32;
        if (++u >= nunits + 2) break;
        scan_unit<NC, 3, 1, ABL>(ch, tab, k, valid, rb);
#pragma unroll
        for (int c = 0; c < NC; c++)
            if constexpr (!(ABL & 1)) load_unit(ch[c].u[1], rsrc[c], voffa, pstride, (u + 2) * 32u);
        rb += 32;
        if (++u >= nunits + 2) break;
        scan_unit<NC, 0, 2, ABL>(ch, tab, k, valid, rb);
#pragma unroll
        for (int c = 0; c < NC; c++)
            if constexpr (!(ABL & 1)) load_unit(ch[c].u[2], rsrc[c], voffa, pstride, (u + 2) * 32u);
        rb += 32;
        if (++u >= nunits + 2) break;
        scan_unit<NC, 1, 3, ABL>(ch, tab, k, valid, rb);
#pragma unroll
        for (int c = 0; c < NC; c++)
            if constexpr (!(ABL & 1)) load_unit(ch[c].u[3], rsrc[c], voffa, pstride, (u + 2) * 32u);
        rb += 32;
        if (++u >= nunits + 2) break;
    }
#pragma unroll
    for (int c = 0; c < NC; c++) {
        if ((valid[c] >> lane) & 1)
            sums[sum_idx[c] + lane] = make_uint4(ch[c].first, ch[c].last, ch[c].count, 0u);
        const uint64_t hits = __builtin_amdgcn_ballot_w64(ch[c].count != 0u) & valid[c];
        if (lane == 0) item_masks[it0 + c] = hits;
    }
}

}  // namespace

template <int NC, int THREADS, int ABL = 0>
__global__ __launch_bounds__(THREADS, 1) void rcdc_scan3_kernel(
    const uint8_t *__restrict__ arena, const ScanItem *__restrict__ items, uint32_t nitems,
    const uint64_t *__restrict__ gtab, ScanParams prm, uint4 *__restrict__ sums,
    uint64_t *__restrict__ item_masks) {
    __shared__ __attribute__((aligned(16))) uint8_t s_tab[kLdsBytes];
    for (uint32_t i = threadIdx.x; i < 256u * kTableRepl; i += THREADS) {
        const uint32_t e = i / kTableRepl, c = i % kTableRepl;
        const uint64_t o = gtab[e], m = gtab[256 + e];
        *reinterpret_cast<uint2 *>(s_tab + e * 256u + c * 8u) =
            make_uint2((uint32_t)o, (uint32_t)(o >> 32));
        *reinterpret_cast<uint2 *>(s_tab + kTableBytes + e * 256u + c * 8u) =
            make_uint2((uint32_t)m, (uint32_t)(m >> 32));
    }
    __syncthreads();

    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = threadIdx.x >> 6;
    constexpr uint32_t waves = THREADS / 64;
    Consts k;
    k.lwo = (lane & 31u) * 8u;
    k.lwm = k.lwo | kTableBytes;
    k.kff00 = in_vgpr(0xFF00u);
    k.mask = in_vgpr(prm.mask);
    k.tsh = prm.idx_shift - 8u;  // (deg - 32) - 8: idx lands in bits 8..15
    k.even = 0x5555555555555555ull;
    k.odd = 0xAAAAAAAAAAAAAAAAull;
    const uint32_t nsuper = (nitems + NC - 1) / NC;
    for (uint32_t sp = blockIdx.x * waves + wave; sp < nsuper; sp += gridDim.x * waves) {
        const uint32_t it0 = __builtin_amdgcn_readfirstlane(sp * NC);
        if (it0 + NC <= nitems) {
            scan_items<NC, ABL>(arena, items, it0, lane, s_tab, k, prm.seg_bytes, sums, item_masks);
        } else {
            for (uint32_t it = it0; it < nitems; it++)
                scan_items<1>(arena, items, it, lane, s_tab, k, prm.seg_bytes, sums, item_masks);
        }
    }
}

namespace rcdc {

// variant 12 + (NC - 1): v3 kernels
hipError_t launch_scan3(int nc, const uint8_t *arena, const ScanItem *items, uint32_t nitems,
                        const uint64_t *gtab, const ScanParams &prm, uint4 *sums,
                        uint64_t *item_masks, uint32_t blocks, hipStream_t stream) {
    if (nitems == 0) return hipSuccess;
#define RCDC_ABL(NC_, T_, A_)                                                                  \
    case (NC_) + 10 * (A_):                                                                  \
        hipLaunchKernelGGL((rcdc_scan3_kernel<NC_, T_, A_>), dim3(blocks), dim3(T_), 0, stream, \
                           arena, items, nitems, gtab, prm, sums, item_masks);                \
        return hipGetLastError();
    switch (nc) {
        RCDC_ABL(1, 1024, 1) RCDC_ABL(1, 1024, 3) RCDC_ABL(1, 1024, 7) RCDC_ABL(1, 1024, 15)
        RCDC_ABL(1, 1024, 4) RCDC_ABL(1, 1024, 9)
        RCDC_ABL(2, 1024, 1) RCDC_ABL(2, 1024, 3) RCDC_ABL(2, 1024, 7) RCDC_ABL(2, 1024, 15)
        RCDC_ABL(1, 1024, 16) RCDC_ABL(2, 1024, 16)
        default: break;
    }
#undef RCDC_ABL
    switch (nc) {
        case 1:
            hipLaunchKernelGGL((rcdc_scan3_kernel<1, 1024>), dim3(blocks), dim3(1024), 0, stream,
                               arena, items, nitems, gtab, prm, sums, item_masks);
            break;
        case 2:
            hipLaunchKernelGGL((rcdc_scan3_kernel<2, 1024>), dim3(blocks), dim3(1024), 0, stream,
                               arena, items, nitems, gtab, prm, sums, item_masks);
            break;
        default:
            hipLaunchKernelGGL((rcdc_scan3_kernel<3, 768>), dim3(blocks), dim3(768), 0, stream,
                               arena, items, nitems, gtab, prm, sums, item_masks);
            break;
    }
    return hipGetLastError();
}

}  // namespace rcdc
