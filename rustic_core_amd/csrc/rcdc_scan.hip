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

#include "rcdc_slide.h"

namespace {

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
    const uint32_t rlo = (lv && item.lo > segpos) ? (uint32_t)min(item.lo - segpos, (uint64_t)S) : 0u;
    const uint32_t rhi = (lv && item.hi > segpos) ? (uint32_t)min(item.hi - segpos, (uint64_t)S) : 0u;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(arena + item.q0), (short)0, (int)(uint32_t)item.rec_bytes, 0x00020000);
    const Chain c = scan_segment<R, PAIR, TSH, SMALL, G>(rsrc, lane * S, nunits, rlo, rhi, tab, k,
                                                         valid, lane);
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
    fill_tables(s_tab, gtab, prm.idx_shift, threadIdx.x, THREADS);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = threadIdx.x >> 6;
    constexpr uint32_t kWaves = THREADS / 64;
    const Consts k = make_consts(lane, prm.mask, prm.idx_shift);
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
        case 4116: return launch4<4, true, 1024, 116>(arena, items, nitems, gtab, prm, sums, item_masks, blocks, stream);
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

// A capacity plan's stream set to length n (rcdc_runtime.cpp plan_set_len):
// the descriptor's length and segment count, and the end position of the
// items the scan runs.
__global__ void rcdc_plan_set_len_kernel(StreamDesc *sds, ScanItem *items, uint32_t nitems,
                                         uint64_t n, uint64_t nseg) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) {
        sds[0].n = n;
        sds[0].nseg = nseg;
    }
    if (i < nitems) items[i].hi = n;
}

namespace rcdc {

hipError_t launch_plan_set_len(StreamDesc *sds, ScanItem *items, uint32_t nitems, uint64_t n,
                               uint64_t nseg, hipStream_t stream) {
    hipLaunchKernelGGL(rcdc_plan_set_len_kernel, dim3((nitems + 255) / 256 + 1), dim3(256), 0,
                       stream, sds, items, nitems, n, nseg);
    return hipGetLastError();
}

}  // namespace rcdc
