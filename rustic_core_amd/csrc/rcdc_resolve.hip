// rcdc_resolve.hip -- resolver kernels of the rcdc chunker (gfx950).
//
// Replace the chunk-to-chunk iteration of ChunkIter::next
// (crates/core/src/chunker/rabin.rs:107-191).  One wave hops from cut to cut
// with the reference's min / max / min-zone rules (next_cut), reading the
// per-segment candidate summaries written by rcdc_scan_kernel.
//
//   rcdc_resolve_kernel  one wave per ResolveUnit: a whole stream, or one
//                        piece of a long stream resolved speculatively from
//                        the piece start (a chunk boundary is assumed there);
//                        stops after its first cut at or past the piece end.
//   rcdc_stitch_kernel   one wave per long stream: walks the pieces in order
//                        and keeps a piece's speculative cuts from the first
//                        one the true chain also reaches (from there on the
//                        two chains are the same function of the same start).
//                        Where they have not merged it hops on itself, so the
//                        result is exact for every input; CDC chains
//                        resynchronise within a chunk or two on real data, and
//                        piece starts are multiples of min, which keeps long
//                        zero runs (all chunks == min) in phase.
#include <hip/hip_runtime.h>

#include "rcdc_internal.h"

using namespace rcdc;

namespace {

struct RTables {
    uint64_t out[256];  // out_table[b] (unshifted)
    uint64_t mod[256];
};

struct Shared {
    RTables t;
    uint8_t win[128];
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

struct Hop {
    const StreamDesc &d;
    const uint8_t *s;  // stream byte 0
    const ResolveParams &prm;
    const uint4 *sums;
    const uint64_t *item_masks;
    Shared &sh;
    uint32_t lane;
};

// The end of the chunk that starts at `pos` (< N): rabin.rs:110-191.
// Wave-cooperative; every lane returns the same value.  *zero is set when
// the cut came from the all-zero prefill rule (see below).
__device__ uint64_t next_cut(const Hop &H, uint64_t pos, bool *zero) {
    *zero = false;
    const StreamDesc &d = H.d;
    const uint64_t N = d.n, mn = H.prm.min_size, mx = H.prm.max_size, S = H.prm.seg_bytes;
    const uint32_t mask = H.prm.mask, shift = H.prm.shift, lane = H.lane;
    if (N - pos < mn) return N;  // rabin.rs:141-147: the rest is the last chunk
    const uint64_t z = pos + mn;              // first test position
    const uint64_t limit = min(pos + mx, N);  // rabin.rs:154 / EOF
    const uint64_t q = z + 64;                // first pure 64-byte window

    // Round 1 of loads, all independent: the 128 bytes around z (min-zone),
    // the summary of q's segment, the item masks of the 64 items from there.
    const bool zone = z < limit;
    uint8_t w0 = 0, w1 = 0;
    if (zone) {
        const uint64_t p0 = z - 64 + lane, p1 = z + lane;
        w0 = H.s[p0];
        w1 = p1 < N ? H.s[p1] : 0;
    }
    const bool query = q < limit && d.nseg;
    uint64_t j = ~0ull;
    uint4 sm = make_uint4(kNone, kNone, 0, 0);
    uint64_t mk = 0;
    const uint64_t nitems = (d.nseg + 63) / 64;
    if (query) {
        j = (q - d.pos0) / S;
        if (j < d.nseg) {
            sm = H.sums[d.sum_base + j];
            const uint64_t it = j / 64 + lane;
            if (it < nitems) mk = H.item_masks[d.item_base + it];
        }
    }

    uint64_t cut = limit;
    // All-zero prefill: the k = 0 zone window is the 63 bytes b[z-64, z-1);
    // if they are all zero its hash is 0, which passes any mask, so the cut
    // is z = pos + min (rabin.rs:149-158).  Free: w0 holds those bytes.
    if (zone && __builtin_amdgcn_ballot_w64(lane < 63 && w0 != 0) == 0) {
        *zero = true;
        return z;
    }
    // min-zone (V1): positions z + k, k < 64, hash of the last 64 bytes of
    // b[z-64, z-1) ++ b[z, z+k)   (rustic_cdc prefills 63 bytes)
    if (zone) {
        __syncthreads();
        H.sh.win[lane] = w0;
        H.sh.win[64 + lane] = w1;
        __syncthreads();
        const uint32_t k = lane;
        uint64_t h = 0;
        for (uint32_t i = 0; i < 64; i++) {
            const int src = (i < 64 - k) ? (int)(k + i) - 1 : (int)(i + k);
            const uint32_t byte = src >= 0 ? H.sh.win[src] : 0u;
            h = rabin_in(H.sh.t, h, byte, shift);
        }
        const uint64_t hit = __builtin_amdgcn_ballot_w64(z + k < limit && (h & mask) == 0);
        if (hit) cut = z + wave_ffs(hit);
    }

    // first candidate p >= q (pure windows) below `cut`
    if (query && q < cut && j < d.nseg) {
        uint64_t found = ~0ull;
        const uint64_t segstart = d.pos0 + j * S;
        if (sm.x != kNone) {
            const uint64_t f = segstart + sm.x, l = segstart + sm.y;
            if (f >= q) {
                found = f;
            } else if (l >= q) {
                if (sm.z == sm.y - sm.x + 1u) {
                    found = q;  // every position of [first, last] qualifies
                } else {
                    found = rescan(H.s, H.sh.t, q, min(segstart + S, min(cut, N)), shift, mask,
                                   lane);
                }
            }
        }
        // following segments from the item masks already loaded (64 items =
        // 4096 segments); further passes only for small S
        uint64_t jj = j + 1, it0 = j / 64;
        bool first_pass = true;
        while (found == ~0ull && jj < d.nseg && d.pos0 + jj * S < cut) {
            if (!first_pass) {
                it0 = jj / 64;
                mk = (it0 + lane < nitems) ? H.item_masks[d.item_base + it0 + lane] : 0;
            }
            first_pass = false;
            // drop segments below jj (lane L holds item it0 + L)
            const uint64_t base = (it0 + lane) * 64;
            if (base + 64 <= jj) mk = 0;
            else if (base < jj) mk &= ~0ull << (jj - base);
            const uint64_t b = __builtin_amdgcn_ballot_w64(mk != 0);
            if (!b) {
                jj = (it0 + 64) * 64;
                continue;
            }
            const uint32_t L = (uint32_t)wave_ffs(b);
            const uint64_t mkL = __shfl(mk, (int)L);
            const uint64_t seg = (it0 + L) * 64 + wave_ffs(mkL);
            if (seg < d.nseg) found = d.pos0 + seg * S + H.sums[d.sum_base + seg].x;
            break;
        }
        if (found < cut) cut = found;
    }
    return cut;
}

// Consecutive chunks of exactly min bytes from `pos` by the all-zero prefill
// rule: lane i checks the chunk starting at pos + i*min (it must have at
// least min bytes left, and its 63 prefill bytes must be zero; min < max).
// Returns how many leading lanes qualify (0..64).
__device__ uint32_t zero_hops(const Hop &H, uint64_t pos) {
    const uint64_t N = H.d.n, mn = H.prm.min_size;
    if (mn >= H.prm.max_size) return 0;
    const uint64_t si = pos + (uint64_t)H.lane * mn;
    bool ok = si + mn <= N;
    if (ok) {
        // stream bytes [w, e), e = w + 63: whole aligned 8-byte words inside,
        // single bytes at the two ends (never reads outside the window)
        const uint64_t w = si + mn - 64, e = w + 63;
        const uint64_t abs_w = H.d.off + w;
        const uint64_t wa = (abs_w + 7) & ~7ull;           // first whole word
        const uint64_t we = (H.d.off + e) & ~7ull;         // end of whole words
        const uint8_t *arena = H.s - H.d.off;
        uint64_t acc = 0;
        for (uint64_t a = abs_w; a < min(wa, H.d.off + e); a++) acc |= arena[a];
        for (uint64_t a = wa; a + 8 <= we; a += 8) acc |= *reinterpret_cast<const uint64_t *>(arena + a);
        for (uint64_t a = max(we, wa); a < H.d.off + e; a++) acc |= arena[a];
        ok = acc == 0;
    }
    const uint64_t bad = __builtin_amdgcn_ballot_w64(!ok);
    return bad ? (uint32_t)wave_ffs(bad) : 64u;
}

__device__ __forceinline__ void load_tables(Shared &sh, const uint64_t *gtab, uint32_t lane) {
    for (uint32_t i = lane; i < 256; i += 64) {
        sh.t.out[i] = gtab[i] >> 8;
        sh.t.mod[i] = gtab[256 + i];
    }
    __syncthreads();
}

}  // namespace

// One wave per unit: hop from unit.start until the first cut >= unit.stop
// (or N), writing cuts to out[unit.out_base ..].
__global__ __launch_bounds__(64) void rcdc_resolve_kernel(
    const uint8_t *__restrict__ arena, const StreamDesc *__restrict__ sds,
    const ResolveUnit *__restrict__ units, uint32_t nunits, const uint64_t *__restrict__ gtab,
    ResolveParams prm, const uint4 *__restrict__ sums, const uint64_t *__restrict__ item_masks,
    uint64_t *__restrict__ cuts, uint64_t *__restrict__ counts, uint64_t *__restrict__ piece_cuts,
    uint64_t *__restrict__ piece_counts) {
    __shared__ Shared sh;
    const uint32_t lane = threadIdx.x;
    load_tables(sh, gtab, lane);
    const uint32_t u = blockIdx.x;
    if (u >= nunits) return;
    const ResolveUnit U = units[u];
    const StreamDesc d = sds[U.stream];
    const Hop H{d, arena + d.off, prm, sums, item_masks, sh, lane};
    uint64_t *out = U.direct ? cuts : piece_cuts;
    const uint64_t mn = prm.min_size;
    uint64_t pos = U.start, nc = 0;
    while (pos < d.n) {
        bool zero;
        const uint64_t cut = next_cut(H, pos, &zero);
        if (lane == 0 && nc < U.out_cap) out[U.out_base + nc] = cut;
        nc++;
        pos = cut;
        if (pos >= U.stop) break;
        // inside a zero run: up to 64 further min-sized chunks per round
        while (zero && pos < d.n) {
            uint32_t m = zero_hops(H, pos);
            if (m == 0) break;
            // stop after the first cut >= stop
            if (pos + (uint64_t)m * mn >= U.stop) m = (uint32_t)((U.stop - pos + mn - 1) / mn);
            if (lane < m && nc + lane < U.out_cap) out[U.out_base + nc + lane] = pos + (lane + 1) * mn;
            nc += m;
            pos += (uint64_t)m * mn;
            if (pos >= U.stop || m < 64) break;
        }
        if (pos >= U.stop) break;
    }
    if (lane == 0) {
        if (U.direct) counts[U.stream] = nc;
        else piece_counts[u] = nc;
    }
}

// One wave per long stream: stitch its pieces (units[unit0 .. unit0 + np)).
__global__ __launch_bounds__(64) void rcdc_stitch_kernel(
    const uint8_t *__restrict__ arena, const StreamDesc *__restrict__ sds,
    const ResolveUnit *__restrict__ units, const StitchDesc *__restrict__ stitches,
    uint32_t nstitch, const uint64_t *__restrict__ gtab, ResolveParams prm,
    const uint4 *__restrict__ sums, const uint64_t *__restrict__ item_masks,
    uint64_t *__restrict__ cuts, uint64_t *__restrict__ counts,
    const uint64_t *__restrict__ piece_cuts, const uint64_t *__restrict__ piece_counts,
    uint64_t *__restrict__ stats) {
    __shared__ Shared sh;
    const uint32_t lane = threadIdx.x;
    load_tables(sh, gtab, lane);
    if (blockIdx.x >= nstitch) return;
    const StitchDesc SD = stitches[blockIdx.x];
    const StreamDesc d = sds[SD.stream];
    const Hop H{d, arena + d.off, prm, sums, item_masks, sh, lane};
    const uint64_t N = d.n, cap = d.cut_cap, mn = prm.min_size;
    uint64_t *out = cuts + d.cut_base;
    uint64_t nc = 0, extra_hops = 0;

    // append src[a, b) to out (wave-wide copy)
    auto append = [&](const uint64_t *src, uint64_t a, uint64_t b) {
        for (uint64_t i = a + lane; i < b; i += 64)
            if (nc + (i - a) < cap) out[nc + (i - a)] = src[i];
        nc += b - a;
    };

    // piece 0 is the true chain from byte 0
    const ResolveUnit U0 = units[SD.unit0];
    const uint64_t n0 = min(piece_counts[SD.unit0], (uint64_t)U0.out_cap);
    append(piece_cuts, U0.out_base, U0.out_base + n0);
    uint64_t c = n0 ? piece_cuts[U0.out_base + n0 - 1] : N;

    for (uint32_t p = 1; p < SD.npieces && c < N; p++) {
        const uint32_t u = SD.unit0 + p;
        const ResolveUnit U = units[u];
        if (c >= U.stop) continue;  // the true chain jumped over this piece
        const uint64_t base = U.out_base, n = min(piece_counts[u], (uint64_t)U.out_cap);
        const uint64_t *L = piece_cuts + base;
        // c lies in [U.start, U.stop).  Merge point: c == start, or c in L.
        int64_t at = -1;  // index in L of the first cut to keep
        for (;;) {
            if (c == U.start) {
                at = 0;
                break;
            }
            // wave search of c in the sorted list (nearly always in the first 64)
            for (uint64_t i0 = 0; i0 < n; i0 += 64) {
                const uint64_t i = i0 + lane;
                const uint64_t v = i < n ? L[i] : ~0ull;
                const uint64_t eq = __builtin_amdgcn_ballot_w64(v == c);
                if (eq) {
                    at = (int64_t)(i0 + wave_ffs(eq)) + 1;
                    break;
                }
                const uint64_t gt = __builtin_amdgcn_ballot_w64(v > c);
                if (gt) break;  // sorted: c is not in L
            }
            if (at >= 0) break;
            // not merged: one exact hop of the true chain (zero runs: up to
            // 64 min-sized chunks per round)
            bool zero;
            c = next_cut(H, c, &zero);
            extra_hops++;
            if (lane == 0 && nc < cap) out[nc] = c;
            nc++;
            while (zero && c < U.stop && c < N) {
                uint32_t m = zero_hops(H, c);
                if (m == 0) break;
                if (c + (uint64_t)m * mn >= U.stop) m = (uint32_t)((U.stop - c + mn - 1) / mn);
                if (lane < m && nc + lane < cap) out[nc + lane] = c + (lane + 1) * mn;
                nc += m;
                c += (uint64_t)m * mn;
                extra_hops += m;
                if (m < 64) break;
            }
            if (c >= U.stop || c >= N) break;
        }
        if (at >= 0) {
            append(piece_cuts, base + (uint64_t)at, base + n);
            if (n > (uint64_t)at) c = L[n - 1];
        }
    }
    if (lane == 0) {
        counts[SD.stream] = nc;
        if (stats) atomicAdd((unsigned long long *)stats, (unsigned long long)extra_hops);
    }
}

// Crossing window of one stream's device cut list (rcdc_plan_window), for the
// cross-rank stitch of one stream sliced over GPUs: out[0] = the
// count n, out[1] = j, the index of the first cut >= bound (n if none),
// out[2] = that cut (~0 if none), out[3 + t] = cut t for t < k (~0 past n).
// The list is sorted, so exactly one index satisfies c[j] >= bound >
// c[j - 1]; every thread tests a strided share and only that one writes.
// n == ~0 (a walked stream that needs host completion) is passed through.
__global__ __launch_bounds__(256) void rcdc_window_kernel(const uint64_t *__restrict__ cuts,
                                                          const uint64_t *__restrict__ counts,
                                                          uint32_t stream, uint64_t base,
                                                          uint64_t bound, uint32_t k,
                                                          uint64_t *__restrict__ out) {
    const uint64_t n = counts[stream];
    const uint64_t *c = cuts + base;
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t nthr = gridDim.x * blockDim.x;
    if (n == ~0ull) {
        if (tid == 0) out[0] = n;
        return;
    }
    if (tid == 0) {
        out[0] = n;
        if (n == 0 || c[n - 1] < bound) {  // no cut >= bound
            out[1] = n;
            out[2] = ~0ull;
        }
    }
    for (uint32_t t = tid; t < k; t += nthr) out[3 + t] = t < n ? c[t] : ~0ull;
    for (uint64_t i = tid; i < n; i += nthr) {
        if (c[i] >= bound && (i == 0 || c[i - 1] < bound)) {
            out[1] = i;
            out[2] = c[i];
        }
    }
}

// ---------------------------------------------------------------------------
// host-side launchers (called from rcdc_runtime.cpp)
// ---------------------------------------------------------------------------
namespace rcdc {

hipError_t launch_window(const uint64_t *cuts, const uint64_t *counts, uint32_t stream,
                         uint64_t base, uint64_t bound, uint32_t k, uint64_t *out,
                         hipStream_t hs) {
    hipLaunchKernelGGL(rcdc_window_kernel, dim3(32), dim3(256), 0, hs, cuts, counts, stream, base,
                       bound, k, out);
    return hipGetLastError();
}

hipError_t launch_resolve(const uint8_t *arena, const StreamDesc *sds, const ResolveUnit *units,
                          uint32_t nunits, const StitchDesc *stitches, uint32_t nstitch,
                          const uint64_t *gtab, const ResolveParams &prm, const uint4 *sums,
                          const uint64_t *item_masks, uint64_t *cuts, uint64_t *counts,
                          uint64_t *piece_cuts, uint64_t *piece_counts, uint64_t *stats,
                          hipStream_t stream) {
    if (nunits == 0) return hipSuccess;
    hipLaunchKernelGGL(rcdc_resolve_kernel, dim3(nunits), dim3(64), 0, stream, arena, sds, units,
                       nunits, gtab, prm, sums, item_masks, cuts, counts, piece_cuts,
                       piece_counts);
    if (nstitch)
        hipLaunchKernelGGL(rcdc_stitch_kernel, dim3(nstitch), dim3(64), 0, stream, arena, sds,
                           units, stitches, nstitch, gtab, prm, sums, item_masks, cuts, counts,
                           piece_cuts, piece_counts, stats);
    return hipGetLastError();
}

}  // namespace rcdc
