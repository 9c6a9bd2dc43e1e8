// rcdc_resolve.hip -- resolver kernel of the rcdc chunker (gfx950).
//
// Replaces the chunk-to-chunk iteration of ChunkIter::next
// (crates/core/src/chunker/rabin.rs:107-191): one wave per stream hops from
// cut to cut with the reference's min / max / min-zone rules, reading the
// per-segment candidate summaries written by rcdc_scan_kernel (rare
// in-segment rescans on device).
#include <hip/hip_runtime.h>

#include "rcdc_internal.h"

using namespace rcdc;

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
