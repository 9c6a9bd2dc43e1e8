// rcdc_kernels.hip -- CDNA4 (gfx950) kernels of the rcdc chunker.
//
// Replaces the per-byte hot loop of crates/core/src/chunker/rabin.rs:153-188
// (rustic_cdc Rabin64::slide + the `hash & split_mask == 0` test) and the
// chunk-to-chunk iteration of ChunkIter::next (rabin.rs:107-191).
//
//   rcdc_scan_kernel    every lane owns one S-byte segment of one stream and
//                       rolls the 64-byte-window Rabin64 fingerprint over it,
//                       recording the first / last / number of positions p
//                       with fp(b[p-64, p)) & mask == 0 ("candidates").
//                       HBM-bound integer byte hashing; no MFMA.
//   rcdc_resolve_kernel one wave per stream hops chunk to chunk with the
//                       reference's min / max / min-zone rules, reading the
//                       segment summaries (rare in-segment rescans on device).
#include <hip/hip_runtime.h>

#include "rcdc_internal.h"

using namespace rcdc;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

namespace {

// ---------------------------------------------------------------------------
// scan kernel building blocks
// ---------------------------------------------------------------------------

// three-input XOR as one gfx950 v_bitop3_b32 (truth table 0x96 = a^b^c);
// the builtin keeps the compiler from splitting it into two v_xor_b32
// around a fused mask test.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// hb = 2*hb + (this lane's bit of m): builds per-lane hit bits from wave
// ballots kept in SGPRs (v_addc_co_u32 with an SGPR-pair carry-in).
__device__ __forceinline__ uint32_t shift_in(uint32_t hb, uint64_t m) {
    uint32_t r;
    asm("v_addc_co_u32 %0, vcc, %1, %1, %2" : "=v"(r) : "v"(hb), "s"(m) : "vcc");
    return r;
}

__device__ __forceinline__ uint2 lds_u2(const uint8_t *tab, uint32_t byte_addr) {
    return *reinterpret_cast<const uint2 *>(tab + byte_addr);
}

// 64 bytes of one lane's segment in 16 VGPRs.
struct Unit {
    u32x4 v[4];
};
#define UDW(u, d) ((u).v[(d) >> 2][(d) & 3])

// Rabin64 state h (< 2^deg, deg in [33,56]) lives in two dwords, h1:h0.
// One slide of byte n with old byte o:
//     h ^= out[o];  i = h >> (deg-8);  h = ((h << 8) | n) ^ mod[i]
// is evaluated as
//     a1x = hi32(h << 8) ^ hi32(out[o] << 8)     v_alignbit, v_xor  (OUT table pre-shifted)
//     i   = a1x >> (deg - 32)                    top byte, from the high word
//     h1  = a1x ^ hi32(mod[i])                   mod[i] carries i << deg
//     h0  = ((h0 << 8) | n) ^ lo32(out[o] << 8) ^ lo32(mod[i])   v_perm + v_xor3
// The table entry of byte e for lane-copy c sits at LDS byte e*256 + c*8, so
// a half-wave's 32 lanes hit 32 distinct bank pairs: ds_read_b64 never
// conflicts whatever the data.  Addresses are one v_perm (OUT, old byte
// placed in bits 8..15) or v_lshrrev + v_lshl_or (MOD).
template <int K>
__device__ __forceinline__ void slide_warm(uint32_t &h0, uint32_t &h1, uint32_t dnew,
                                           const uint8_t *tab, uint32_t lwm, uint32_t tsh) {
    const uint32_t a1 = __builtin_amdgcn_alignbit(h1, h0, 24);
    const uint2 m = lds_u2(tab, ((a1 >> tsh) << 8) | lwm);
    h0 = __builtin_amdgcn_perm(h0, dnew, 0x06050400u | K) ^ m.x;
    h1 = a1 ^ m.y;
}

template <int K>
__device__ __forceinline__ void slide(uint32_t &h0, uint32_t &h1, uint32_t dnew, uint32_t dold,
                                      const uint8_t *tab, uint32_t lwo, uint32_t lwm,
                                      uint32_t tsh) {
    const uint2 o = lds_u2(tab, __builtin_amdgcn_perm(dold, lwo, 0x0C0C0000u | ((4u + K) << 8)));
    const uint32_t a1x = __builtin_amdgcn_alignbit(h1, h0, 24) ^ o.y;
    const uint2 m = lds_u2(tab, ((a1x >> tsh) << 8) | lwm);
    h0 = xor3(__builtin_amdgcn_perm(h0, dnew, 0x06050400u | K), o.x, m.x);
    h1 = a1x ^ m.y;
}

template <int K>
__device__ __forceinline__ void slide_k(uint32_t &h0, uint32_t &h1, uint32_t dnew, uint32_t dold,
                                        const uint8_t *tab, uint32_t lwo, uint32_t lwm,
                                        uint32_t tsh) {
    slide<K>(h0, h1, dnew, dold, tab, lwo, lwm, tsh);
}

__device__ __forceinline__ void load_unit(Unit &u, __amdgpu_buffer_rsrc_t rsrc, uint32_t voff) {
#pragma unroll
    for (int i = 0; i < 4; i++) {
        u.v[i] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)(voff + 16u * i), 0, 0);
    }
}

// One lane's scan of one segment ("chain").  NC chains per lane run
// interleaved so that a wave always has independent dependency chains.
struct Chain {
    uint32_t h0, h1;
    uint32_t first, last, count;  // candidate summary (relative positions)
    uint32_t rlo, rhi;            // relative positions that count
    Unit u[3];                    // rotating: new / old (64 bytes back) / in flight
};

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

// 64 slides per chain (new bytes in unit IN, bytes 64 earlier in unit IO),
// testing the position after every slide; groups of 8 positions share one
// uniform branch into the rare path.
template <int NC, int IN, int IO>
__device__ __forceinline__ void scan_units(Chain (&ch)[NC], const uint8_t *tab, uint32_t lwo,
                                           uint32_t lwm, uint32_t tsh, uint32_t mask,
                                           const uint64_t (&valid)[NC], uint32_t rb) {
#pragma unroll
    for (int g = 0; g < 8; g++) {
        uint64_t m[NC][8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int b = g * 8 + j;
#pragma unroll
            for (int c = 0; c < NC; c++) {
                const uint32_t dn = UDW(ch[c].u[IN], b >> 2), d_o = UDW(ch[c].u[IO], b >> 2);
                switch (b & 3) {
                    case 0: slide_k<0>(ch[c].h0, ch[c].h1, dn, d_o, tab, lwo, lwm, tsh); break;
                    case 1: slide_k<1>(ch[c].h0, ch[c].h1, dn, d_o, tab, lwo, lwm, tsh); break;
                    case 2: slide_k<2>(ch[c].h0, ch[c].h1, dn, d_o, tab, lwo, lwm, tsh); break;
                    default: slide_k<3>(ch[c].h0, ch[c].h1, dn, d_o, tab, lwo, lwm, tsh); break;
                }
                m[c][j] = __builtin_amdgcn_ballot_w64((ch[c].h0 & mask) == 0u);
            }
        }
#pragma unroll
        for (int c = 0; c < NC; c++) {
            uint64_t any = m[c][0];
#pragma unroll
            for (int j = 1; j < 8; j++) any |= m[c][j];
            if (any & valid[c]) record_hits(ch[c], m[c], rb + g * 8);
        }
    }
}

template <int NC>
__device__ __forceinline__ void warm_units(Chain (&ch)[NC], const uint8_t *tab, uint32_t lwm,
                                           uint32_t tsh) {
#pragma unroll
    for (int b = 0; b < 64; b++) {
#pragma unroll
        for (int c = 0; c < NC; c++) {
            const uint32_t dn = UDW(ch[c].u[1], b >> 2);
            switch (b & 3) {
                case 0: slide_warm<0>(ch[c].h0, ch[c].h1, dn, tab, lwm, tsh); break;
                case 1: slide_warm<1>(ch[c].h0, ch[c].h1, dn, tab, lwm, tsh); break;
                case 2: slide_warm<2>(ch[c].h0, ch[c].h1, dn, tab, lwm, tsh); break;
                default: slide_warm<3>(ch[c].h0, ch[c].h1, dn, tab, lwm, tsh); break;
            }
        }
    }
}

// Scan NC items (64 segments each) with one wave: lane l owns segment l of
// every item.
template <int NC, bool ROT3, int LOADPAT = 0>
__device__ __forceinline__ void scan_items(const uint8_t *__restrict__ arena,
                                           const ScanItem *__restrict__ items, uint32_t it0,
                                           uint32_t lane, const uint8_t *tab, uint32_t lwo,
                                           uint32_t lwm, const ScanParams &prm,
                                           uint4 *__restrict__ sums,
                                           uint64_t *__restrict__ item_masks) {
    const uint32_t S = prm.seg_bytes, nunits = S / kUnit;
    Chain ch[NC];
    __amdgpu_buffer_rsrc_t rsrc[NC];
    uint64_t valid[NC];
    uint64_t sum_idx[NC];
    // LOADPAT != 0: timing-only experiments (wrong results): 1 = groups of 4
    // lanes read 64 contiguous bytes, 2 = fully coalesced 1 KiB per load.
    const uint32_t voff = LOADPAT == 0 ? lane * S
                        : LOADPAT == 1 ? (lane & ~3u) * S + (lane & 3u) * 16u
                        : LOADPAT == 2 ? lane * 16u
                        : LOADPAT == 3 ? lane * 256u
                        : LOADPAT == 4 ? lane * 4096u
                        : LOADPAT == 5 ? (lane & ~1u) * S + (lane & 1u) * 16u
                                       : lane * 128u;
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
        load_unit(ch[c].u[1], rsrc[c], voff);        // unit 0: the 64-byte warm-up window
        load_unit(ch[c].u[0], rsrc[c], voff + 64u);  // unit 1
    }
    warm_units<NC>(ch, tab, lwm, prm.idx_shift);

    uint32_t i = 1, rb = 0;
    const uint32_t tsh = prm.idx_shift, mask = prm.mask;
    if constexpr (ROT3) {
        // three register units rotate (new, old, in flight): no moves, 3x code
        for (;;) {
#pragma unroll
            for (int c = 0; c < NC; c++) load_unit(ch[c].u[2], rsrc[c], voff + (i + 1) * 64u);
            scan_units<NC, 0, 1>(ch, tab, lwo, lwm, tsh, mask, valid, rb);
            rb += 64;
            if (++i > nunits) break;
#pragma unroll
            for (int c = 0; c < NC; c++) load_unit(ch[c].u[1], rsrc[c], voff + (i + 1) * 64u);
            scan_units<NC, 2, 0>(ch, tab, lwo, lwm, tsh, mask, valid, rb);
            rb += 64;
            if (++i > nunits) break;
#pragma unroll
            for (int c = 0; c < NC; c++) load_unit(ch[c].u[0], rsrc[c], voff + (i + 1) * 64u);
            scan_units<NC, 1, 2>(ch, tab, lwo, lwm, tsh, mask, valid, rb);
            rb += 64;
            if (++i > nunits) break;
        }
    } else {
        // one unit per iteration, registers shifted with v_mov (compact loop)
        for (;;) {
#pragma unroll
            for (int c = 0; c < NC; c++) load_unit(ch[c].u[2], rsrc[c], voff + (i + 1) * 64u);
            scan_units<NC, 0, 1>(ch, tab, lwo, lwm, tsh, mask, valid, rb);
            rb += 64;
            if (++i > nunits) break;
#pragma unroll
            for (int c = 0; c < NC; c++) {
                ch[c].u[1] = ch[c].u[0];
                ch[c].u[0] = ch[c].u[2];
            }
        }
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

// ---------------------------------------------------------------------------
// scan kernel: one workgroup (16 waves) per CU, 128 KiB of LDS tables.
// A wave takes NC items (64 segments each) at a time.
// ---------------------------------------------------------------------------
template <int NC, bool ROT3, int LOADPAT = 0>
__global__ __launch_bounds__(kScanThreads, 1) void rcdc_scan_kernel(
    const uint8_t *__restrict__ arena, const ScanItem *__restrict__ items, uint32_t nitems,
    const uint64_t *__restrict__ gtab, ScanParams prm, uint4 *__restrict__ sums,
    uint64_t *__restrict__ item_masks) {
    __shared__ __attribute__((aligned(16))) uint8_t s_tab[kLdsBytes];

    // 32 lane-private copies of OUT' (out[b] << 8) and MOD.
    for (uint32_t i = threadIdx.x; i < 256u * kTableRepl; i += kScanThreads) {
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
    const uint32_t lwo = (lane & 31u) * 8u;
    const uint32_t lwm = lwo | kTableBytes;
    const uint32_t nsuper = (nitems + NC - 1) / NC;

    for (uint32_t sp = blockIdx.x * kScanWaves + wave; sp < nsuper;
         sp += gridDim.x * kScanWaves) {
        const uint32_t it0 = __builtin_amdgcn_readfirstlane(sp * NC);
        if (it0 + NC <= nitems) {
            scan_items<NC, ROT3, LOADPAT>(arena, items, it0, lane, s_tab, lwo, lwm, prm, sums,
                                          item_masks);
        } else {
            for (uint32_t it = it0; it < nitems; it++)
                scan_items<1, ROT3>(arena, items, it, lane, s_tab, lwo, lwm, prm, sums, item_masks);
        }
    }
}

// ---------------------------------------------------------------------------
// resolver: one wave per stream
// ---------------------------------------------------------------------------
namespace {

struct RTables {
    uint64_t out[256];  // out_table[b] (unshifted)
    uint64_t mod[256];
};

__device__ __forceinline__ uint64_t rabin_in(const RTables &t, uint64_t h, uint32_t b,
                                             uint32_t shift) {
    return ((h << 8) | b) ^ t.mod[(h >> shift) & 255u];
}

__device__ __forceinline__ uint64_t wave_ffs(uint64_t m) { return (uint64_t)__builtin_ctzll(m); }

// first candidate in [q, e) (e - q <= S): a from-scratch wave-parallel rescan
__device__ uint64_t rescan(const uint8_t *s, const RTables &t, uint64_t q, uint64_t e,
                           uint32_t shift, uint32_t mask, uint32_t lane) {
    const uint64_t len = e - q;
    const uint64_t per = (len + 63) / 64;
    const uint64_t a = q + per * lane;
    const uint64_t b = min(a + per, e);
    uint64_t res = ~0ull;
    if (a < b) {
        uint64_t h = 0;
        for (uint64_t p = a - 64; p < a; p++) h = rabin_in(t, h, s[p], shift);
        for (uint64_t p = a;; p++) {
            if ((h & mask) == 0) { res = p; break; }
            if (p + 1 >= b) break;
            h ^= t.out[s[p - 64]];
            h = rabin_in(t, h, s[p], shift);
        }
    }
    const uint64_t found = __builtin_amdgcn_ballot_w64(res != ~0ull);
    if (!found) return ~0ull;
    return __shfl(res, (int)wave_ffs(found));
}

}  // namespace

__global__ __launch_bounds__(64) void rcdc_resolve_kernel(
    const uint8_t *__restrict__ arena, const StreamDesc *__restrict__ sds, uint32_t nstreams,
    const uint64_t *__restrict__ gtab, ResolveParams prm, const uint4 *__restrict__ sums,
    const uint64_t *__restrict__ item_masks, uint64_t *__restrict__ cuts,
    uint64_t *__restrict__ counts) {
    __shared__ RTables t;
    __shared__ uint8_t win[128];
    const uint32_t lane = threadIdx.x;
    for (uint32_t i = lane; i < 256; i += 64) {
        t.out[i] = gtab[i] >> 8;
        t.mod[i] = gtab[256 + i];
    }
    __syncthreads();

    const uint32_t sid = blockIdx.x;
    if (sid >= nstreams) return;
    const StreamDesc d = sds[sid];
    const uint8_t *s = arena + d.off;
    const uint64_t N = d.n, mn = prm.min_size, mx = prm.max_size, S = prm.seg_bytes;
    const uint32_t mask = prm.mask, shift = prm.shift;
    const uint64_t nitems = (d.nseg + 63) / 64;

    uint64_t pos = 0, nc = 0;
    while (pos < N) {
        if (N - pos < mn) {  // rabin.rs:141-147
            if (lane == 0 && nc < d.cut_cap) cuts[d.cut_base + nc] = N;
            nc++;
            break;
        }
        const uint64_t z = pos + mn;                  // first test position
        const uint64_t limit = min(pos + mx, N);      // rabin.rs:154 / EOF
        uint64_t cut = limit;

        // min-zone (V1): positions z + k, k < 64, hash of the last 64 bytes
        // of b[z-64, z-1) ++ b[z, z+k)   (rustic_cdc prefills 63 bytes)
        if (z < limit) {
            __syncthreads();
            for (uint32_t i = lane; i < 128; i += 64) {
                const uint64_t p = z - 64 + i;
                win[i] = p < N ? s[p] : 0;
            }
            __syncthreads();
            const uint32_t k = lane;
            uint64_t h = 0;
            for (uint32_t i = 0; i < 64; i++) {
                const int src = (i < 64 - k) ? (int)(k + i) - 1 : (int)(i + k);
                const uint32_t byte = src >= 0 ? win[src] : 0u;
                h = rabin_in(t, h, byte, shift);
            }
            const uint64_t hit = __builtin_amdgcn_ballot_w64(z + k < limit && (h & mask) == 0);
            if (hit) cut = z + wave_ffs(hit);
        }

        // first candidate p >= z + 64 (pure 64-byte windows) below `cut`
        const uint64_t q = z + 64;
        if (q < cut && d.nseg) {
            uint64_t found = ~0ull;
            uint64_t j = (q - d.pos0) / S;
            if (j < d.nseg) {
                const uint64_t segstart = d.pos0 + j * S;
                const uint4 sm = sums[d.sum_base + j];
                if (sm.x != kNone) {
                    const uint64_t f = segstart + sm.x, l = segstart + sm.y;
                    if (f >= q) {
                        found = f;
                    } else if (l >= q) {
                        if (sm.z == sm.y - sm.x + 1u) {
                            found = q;  // every position of [first, last] qualifies
                        } else {
                            found = rescan(s, t, q, min(segstart + S, min(cut, N)), shift,
                                           mask, lane);
                        }
                    }
                }
                // following segments: item masks, 64 items (4096 segments) per pass
                uint64_t jj = j + 1;
                while (found == ~0ull && jj < d.nseg && d.pos0 + jj * S < cut) {
                    const uint64_t it0 = jj / 64;
                    uint64_t mk = 0;
                    if (it0 + lane < nitems) mk = item_masks[d.item_base + it0 + lane];
                    if (lane == 0) mk &= ~0ull << (jj % 64);
                    const uint64_t b = __builtin_amdgcn_ballot_w64(mk != 0);
                    if (!b) {
                        jj = (it0 + 64) * 64;
                        continue;
                    }
                    const uint32_t L = (uint32_t)wave_ffs(b);
                    const uint64_t mkL = __shfl(mk, (int)L);
                    const uint64_t seg = (it0 + L) * 64 + wave_ffs(mkL);
                    if (seg < d.nseg) found = d.pos0 + seg * S + sums[d.sum_base + seg].x;
                    break;
                }
            }
            if (found < cut) cut = found;
        }
        if (lane == 0 && nc < d.cut_cap) cuts[d.cut_base + nc] = cut;
        nc++;
        pos = cut;
    }
    if (lane == 0) counts[sid] = nc;
}

// ---------------------------------------------------------------------------
// host-side launchers (called from rcdc_runtime.cpp)
// ---------------------------------------------------------------------------
namespace rcdc {

hipError_t launch_scan3(int nc, const uint8_t *arena, const ScanItem *items, uint32_t nitems,
                        const uint64_t *gtab, const ScanParams &prm, uint4 *sums,
                        uint64_t *item_masks, uint32_t blocks, hipStream_t stream);

int scan_variant_chains(int variant) {
    if (variant >= 100) return variant % 10;  // ablations: 100 + 10*abl + nc
    if (variant >= 12) return variant - 11;
    return (variant == 1 || variant == 3 || variant == 6 || variant == 7) ? 2 : 1;
}
int scan_variant_threads(int variant) { return variant == 14 ? 768 : 1024; }

hipError_t launch_scan(int variant, const uint8_t *arena, const ScanItem *items, uint32_t nitems,
                       const uint64_t *gtab, const ScanParams &prm, uint4 *sums,
                       uint64_t *item_masks, uint32_t blocks, hipStream_t stream) {
    if (nitems == 0) return hipSuccess;
    if (variant >= 100)
        return launch_scan3(variant - 100, arena, items, nitems, gtab, prm, sums, item_masks,
                            blocks, stream);
    if (variant >= 12)
        return launch_scan3(variant - 11, arena, items, nitems, gtab, prm, sums, item_masks, blocks,
                            stream);
    switch (variant) {
        case 0:
            hipLaunchKernelGGL((rcdc_scan_kernel<1, true>), dim3(blocks), dim3(kScanThreads), 0,
                               stream, arena, items, nitems, gtab, prm, sums, item_masks);
            break;
        case 1:
            hipLaunchKernelGGL((rcdc_scan_kernel<2, true>), dim3(blocks), dim3(kScanThreads), 0,
                               stream, arena, items, nitems, gtab, prm, sums, item_masks);
            break;
        case 2:
            hipLaunchKernelGGL((rcdc_scan_kernel<1, false>), dim3(blocks), dim3(kScanThreads), 0,
                               stream, arena, items, nitems, gtab, prm, sums, item_masks);
            break;
        case 3:
            hipLaunchKernelGGL((rcdc_scan_kernel<2, false>), dim3(blocks), dim3(kScanThreads), 0,
                               stream, arena, items, nitems, gtab, prm, sums, item_masks);
            break;
        case 4:  // timing-only experiment (wrong results)
            hipLaunchKernelGGL((rcdc_scan_kernel<1, true, 1>), dim3(blocks), dim3(kScanThreads), 0,
                               stream, arena, items, nitems, gtab, prm, sums, item_masks);
            break;
        case 5:  // timing-only experiment (wrong results)
            hipLaunchKernelGGL((rcdc_scan_kernel<1, true, 2>), dim3(blocks), dim3(kScanThreads), 0,
                               stream, arena, items, nitems, gtab, prm, sums, item_masks);
            break;
        case 6:  // timing-only experiment (wrong results)
            hipLaunchKernelGGL((rcdc_scan_kernel<2, true, 2>), dim3(blocks), dim3(kScanThreads), 0,
                               stream, arena, items, nitems, gtab, prm, sums, item_masks);
            break;
        case 7:  // timing-only experiment (wrong results)
            hipLaunchKernelGGL((rcdc_scan_kernel<2, false, 2>), dim3(blocks), dim3(kScanThreads), 0,
                               stream, arena, items, nitems, gtab, prm, sums, item_masks);
            break;
        case 8:
            hipLaunchKernelGGL((rcdc_scan_kernel<1, true, 3>), dim3(blocks), dim3(kScanThreads), 0,
                               stream, arena, items, nitems, gtab, prm, sums, item_masks);
            break;
        case 9:
            hipLaunchKernelGGL((rcdc_scan_kernel<1, true, 4>), dim3(blocks), dim3(kScanThreads), 0,
                               stream, arena, items, nitems, gtab, prm, sums, item_masks);
            break;
        case 10:
            hipLaunchKernelGGL((rcdc_scan_kernel<1, true, 5>), dim3(blocks), dim3(kScanThreads), 0,
                               stream, arena, items, nitems, gtab, prm, sums, item_masks);
            break;
        default:
            hipLaunchKernelGGL((rcdc_scan_kernel<1, true, 6>), dim3(blocks), dim3(kScanThreads), 0,
                               stream, arena, items, nitems, gtab, prm, sums, item_masks);
            break;
    }
    return hipGetLastError();
}

hipError_t launch_resolve(const uint8_t *arena, const StreamDesc *sds, uint32_t nstreams,
                          const uint64_t *gtab, const ResolveParams &prm, const uint4 *sums,
                          const uint64_t *item_masks, uint64_t *cuts, uint64_t *counts,
                          hipStream_t stream) {
    if (nstreams == 0) return hipSuccess;
    hipLaunchKernelGGL(rcdc_resolve_kernel, dim3(nstreams), dim3(64), 0, stream, arena, sds,
                       nstreams, gtab, prm, sums, item_masks, cuts, counts);
    return hipGetLastError();
}

}  // namespace rcdc
