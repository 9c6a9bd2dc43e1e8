// rcdc_walk.hip -- walk path of the rcdc chunker for long streams (gfx950).
//
// The scan path (rcdc_scan.hip) hashes every byte after a stream's first
// min bytes.  The reference hashes less: ChunkIter::next
// (crates/core/src/chunker/rabin.rs:110-191) copies each chunk's first min
// bytes unhashed (:127-139), prefills the window with the 64 bytes before
// s + min (:149-151) and slides only from there to the cut (:153-188).  On
// random data that skips a third of the bytes; in zero runs (every chunk
// exactly min, decided by the all-zero prefill) it skips almost all of them.
// The walk path does the same on the device:
//
//   rcdc_walk_kernel         one wave per piece [start, stop) of a long
//                            stream (dynamic queue): hops chunk to chunk from
//                            `start` like the reference loop; the pure-window
//                            search of a chunk runs in rounds of 64 lanes x S
//                            bytes (the scan kernel's per-lane segment code),
//                            the 64 min-zone hashes lane-parallel, zero runs
//                            64 chunks per step.  A piece other than the
//                            first assumes a chunk starts at `start`; it
//                            stops at its first cut >= stop, or "open" once
//                            its search passes stop + min + 64, so adjacent
//                            pieces never hash the same bytes.
//   rcdc_walk_check_kernel   one wave per piece boundary: from the previous
//                            piece's end state, finds where the true chain
//                            meets this piece's chain, using what the walker
//                            verified (each cut's kind: the window it searched
//                            was hit-free); rarely it needs bytes nobody
//                            hashed and hands the boundary to
//   rcdc_walk_fixup_kernel   one workgroup per such boundary (rounds of 1024
//                            lanes): walks the exact chain until it meets a
//                            piece's chain;
//   rcdc_walk_assemble_kernel one wave per stream: concatenates.
//
// The result is exact for any input and any piece size; the piece size only
// moves work between the walk and the (rare) fixups.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "rcdc_internal.h"

using namespace rcdc;

#include "rcdc_slide.h"

namespace {

// Round loop shape: a ring of 4 register units refilled a 128-byte line (two
// units) per lane at a time, and groups of 16 positions that keep no
// fingerprints (a flagged lane re-rolls its group, P ~ 2^-12): refilled one
// 64-byte unit at a time the line's second half was often evicted from L2
// before its load (PMC: 1.37 x the lane bytes fetched, now 1.02 x; walk
// 9.83 -> 9.55 ms on C3).  Keeping the 16 fingerprints would not fit the
// 4-unit ring in 128 VGPRs.
constexpr int kWR = 4, kWG = 116;
constexpr bool kWPair = true;
constexpr uint64_t kNoCut = ~0ull;
constexpr uint64_t kOpen = ~0ull - 1;
constexpr uint32_t kNoUnit = 0xFFFFFFFFu;

__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t l) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

// A value every lane holds, made provably wave-uniform (an SGPR): branches on
// it are scalar and barriers around them stay matched across waves
// (cdna_hip_programming.md Guideline 5).
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// MOD-table access in the two LDS layouts: the scan layout (32 lane copies,
// entry e at kTableBytes + e * 256 + copy * 8) and a plain 256-entry table.
struct ModRepl {
    const uint8_t *tab;
    uint32_t lwm;
    __device__ uint64_t operator()(uint32_t e) const {
        const uint2 v = *reinterpret_cast<const uint2 *>(tab + lwm + e * 256u);
        return ((uint64_t)v.y << 32) | v.x;
    }
};
struct ModPlain {
    const uint64_t *mod;
    __device__ uint64_t operator()(uint32_t e) const { return mod[e]; }
};

// The min-zone of the chunk starting at pos (z = pos + min), one wave:
// position z + k (k < 64) hashes the last 64 bytes of
// b[z-64, z-1) ++ b[z, z+k) (rustic_cdc prefills 63 bytes).
// Returns the first zone cut below `limit`, or kNoCut; *zero: the cut came
// from the all-zero prefill (its hash is 0, which passes any mask).
template <typename Mod>
__device__ uint64_t zone_wave(const uint8_t *s, uint64_t N, uint64_t z, uint64_t limit,
                              uint32_t mask, uint32_t shift, const Mod &mod, uint8_t *win,
                              uint32_t lane, bool *zero) {
    const uint32_t w0 = s[z - 64 + lane];
    const uint32_t w1 = (z + lane < N) ? s[z + lane] : 0u;
    *zero = false;
    if (__builtin_amdgcn_ballot_w64(lane < 63 && w0 != 0) == 0) {
        *zero = true;
        return z;
    }
    // X = 0 ++ b[z-64, z-1) ++ b[z, z+64): lane k hashes X[k, k+64)
    wave_sync();
    if (lane < 63) win[lane + 1] = (uint8_t)w0;
    else win[0] = 0;
    win[64 + lane] = (uint8_t)w1;
    wave_sync();
    uint64_t h = 0;
    for (uint32_t i = 0; i < 64; i++) {
        const uint32_t b = win[lane + i];
        h = ((h << 8) | b) ^ mod((uint32_t)(h >> shift) & 255u);
    }
    wave_sync();
    const uint64_t hit = __builtin_amdgcn_ballot_w64(z + lane < limit && (h & mask) == 0);
    return hit ? z + (uint64_t)__builtin_ctzll(hit) : kNoCut;
}

// zone_wave on the scan's LDS tables and slide (rcdc_slide.h): lane k builds
// its 64 bytes X[k, k+64) from the 128-byte LDS window with 17 dword reads and
// 16 v_alignbit, then warms its state over them with the scan's slide_in
// (6 VALU + 1 ds_read_b64 per byte) instead of the generic 64-bit loop
// (~12 VALU + 2 LDS reads per byte).  Same positions, same first cut.
template <int TSH>
__device__ uint64_t zone_wave_fast(const uint8_t *s, uint64_t N, uint64_t z, uint64_t limit,
                                   uint32_t mask, const uint8_t *tab, const Consts &kc,
                                   uint8_t *win, uint32_t lane, bool *zero) {
    const uint32_t w0 = s[z - 64 + lane];
    const uint32_t w1 = (z + lane < N) ? s[z + lane] : 0u;
    *zero = false;
    if (__builtin_amdgcn_ballot_w64(lane < 63 && w0 != 0) == 0) {
        *zero = true;
        return z;
    }
    wave_sync();
    if (lane < 63) win[lane + 1] = (uint8_t)w0;
    else win[0] = 0;
    win[64 + lane] = (uint8_t)w1;
    wave_sync();
    const uint32_t *wd = reinterpret_cast<const uint32_t *>(win);
    const uint32_t d = lane >> 2, sh = (lane & 3u) * 8u;
    Unit u;
    uint32_t lo = wd[d];
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const uint32_t hi = wd[d + j + 1];
        UDW(u, j) = __builtin_amdgcn_alignbit(hi, lo, sh);
        lo = hi;
    }
    wave_sync();
    Chain c;
    c.h0 = c.h1 = 0;
    warm_unit<TSH>(c, u, tab, kc);
    const uint64_t hit = __builtin_amdgcn_ballot_w64(z + lane < limit && (c.h0 & mask) == 0);
    return hit ? z + (uint64_t)__builtin_ctzll(hit) : kNoCut;
}

// Consecutive chunks of exactly min bytes from `pos` by the all-zero prefill
// rule: lane i checks the chunk starting at pos + i*min.  Returns how many
// leading lanes qualify (0..64).  (As rcdc_resolve.hip zero_hops.)
__device__ uint32_t zero_run(const uint8_t *s, uint64_t N, uint64_t mn, uint64_t mx, uint64_t pos,
                             uint32_t lane) {
    if (mn >= mx) return 0;
    const uint64_t si = pos + (uint64_t)lane * mn;
    bool ok = si + mn <= N;
    if (ok) {
        const uint64_t w = si + mn - 64, e = w + 63;
        uint32_t acc = 0;
        const uintptr_t aw = (reinterpret_cast<uintptr_t>(s + w) + 3) & ~(uintptr_t)3;
        const uintptr_t ae = reinterpret_cast<uintptr_t>(s + e) & ~(uintptr_t)3;
        const uint8_t *p = s + w;
        for (; reinterpret_cast<uintptr_t>(p) < aw && p < s + e; p++) acc |= *p;
        for (; reinterpret_cast<uintptr_t>(p) + 4 <= ae; p += 4) acc |= *reinterpret_cast<const uint32_t *>(p);
        for (; p < s + e; p++) acc |= *p;
        ok = acc == 0;
    }
    const uint64_t bad = __builtin_amdgcn_ballot_w64(!ok);
    return bad ? (uint32_t)__builtin_ctzll(bad) : 64u;
}

// Work counters (WalkParams.stats): per-workgroup sums in LDS and one global
// atomic per counter and workgroup at the end -- the same few global
// addresses hit once per piece serialise at the L2 (C5: 5120 pieces, 15 k
// atomics on one line cost more than the walk itself).
struct BlockStats {
    unsigned long long v[kWalkStats];
};

__device__ __forceinline__ void stats_init(BlockStats &S) {
    if (threadIdx.x < kWalkStats) S.v[threadIdx.x] = 0;  // (a barrier follows)
}

__device__ __forceinline__ void stats_add(BlockStats &S, int i, uint64_t x) {
    if (x) atomicAdd(&S.v[i], (unsigned long long)x);
}

__device__ __forceinline__ void stats_flush(BlockStats &S, unsigned long long *g) {
    __syncthreads();
    if (threadIdx.x < kWalkStats && S.v[threadIdx.x]) atomicAdd(&g[threadIdx.x], S.v[threadIdx.x]);
}

struct GapQueue;

// A walker over one stream: one wave (LANES = 64) or one workgroup of 1024.
struct Walk {
    const uint8_t *arena;
    uint64_t arena_len;
    uint64_t off, N, mn, mx;
    uint32_t S, mask, shift;
    const uint8_t *tab;
    Consts k;
    uint8_t *win;      // 128 B of LDS (the zone window)
    uint64_t *red;     // LDS: 16 reduction slots (workgroup walker)
    uint32_t lane, wave, tid;
    // work counters of this walker (wave-uniform): hashing rounds, zones,
    // and the bytes its rounds hashed (LANES x (S + 64) per round)
    uint32_t rounds, zones;
    uint64_t lbytes;
    // walk kernel: the workgroup's round ring (nullptr elsewhere); a walker
    // posts rounds ahead of its search there while waves of its workgroup
    // are idle (the walk's tail), at most help_max per round of its own
    GapQueue *Q;
    uint32_t help_max;
    uint32_t early;  // walk rounds: WalkParams.early (0 elsewhere)
    uint32_t zonefast;  // WalkParams.flags & kWalkZoneFast
};

// Segment of a round that starts at A and only needs positions below end:
// the walker's S, or -- for the last round of a known end (a piece that
// stops "open", a chunk's max, EOF, a gap of the check) -- the fewest
// 64-byte units per lane that still cover [A + 1, end).  The round after a
// shrunk one never runs (A + LANES x S >= end).
template <int LANES>
__device__ __forceinline__ uint32_t round_seg(uint32_t S, uint64_t A, uint64_t end) {
    const uint64_t span = end > A ? end - A : 0;
    if (span >= (uint64_t)LANES * S) return S;
    const uint64_t per = (span + LANES - 1) / LANES;
    return (uint32_t)max((per + 63) / 64 * 64, (uint64_t)64);
}

// Start A of the first round that tests position q (A + 1 <= q, A >= q -
// 128), placed so that the lanes' reads (from off + A - 64 + t * S, S a
// multiple of 128) start on 128-byte lines: with 64-byte-aligned starts
// every lane's first line is fetched for half its bytes (PMC: the scan
// kernel read 1.16 x its bytes that way, 1.03 x from 128-byte lines).
__device__ __forceinline__ uint64_t round_base(uint64_t off, uint64_t q) {
    return (((off + q - 1 - 64) & ~127ull) + 64) - off;
}

// First pure-window candidate p in [q, end) among the positions of one round
// (A: stream position with off + A 64-byte aligned); kNoCut if none.  Lane t
// hashes bytes [A - 64 + t*S, A + (t+1)*S): after the 64-byte warm-up the
// first slide gives the window of position A + t*S + 1, so lane t tests
// [A + 1 + t*S, A + 1 + (t+1)*S) (the scan kernel's r = 0 <-> lane start + 65).
//
// EARLY (the walker's own rounds, W.early): a hit round stops once a lane L
// below 32 has a hit (scan_segment_early); lanes 0 .. L-1 owe the rest of
// their segments, [done, S) each, which all 64 lanes then hash in one shorter
// round (64 / L lanes per owed tail).  The first hit there, else lane L's, is
// the round's.  *lb: the bytes the lanes hashed.
template <int LANES, int TSH, bool SMALL, bool EARLY = false>
__device__ uint64_t round_first(const Walk &W, uint64_t A, uint64_t q, uint64_t end, uint32_t S,
                               uint64_t *lb = nullptr) {
    const uint64_t P0 = A + 1 + (uint64_t)W.tid * S;
    // signed clamps: hipcc (ROCm 7.2) dropped the `end > P0 ?` guard of the
    // unsigned form in the workgroup instantiation (lanes past `end` then
    // counted a full segment; seen in the .s and on the device)
    const int64_t dlo = (int64_t)q - (int64_t)P0, dhi = (int64_t)end - (int64_t)P0;
    const uint32_t rlo = (uint32_t)min(max(dlo, (int64_t)0), (int64_t)S);
    const uint32_t rhi = (uint32_t)min(max(dhi, (int64_t)0), (int64_t)S);
    const uint64_t valid = __builtin_amdgcn_ballot_w64(rlo < rhi);
    uint64_t best = kNoCut;
    if (valid) {
        const uint64_t base = W.off + A - 64;  // >= off: A >= q - 64 >= pos + min
        const uint64_t wbase = base + (uint64_t)W.wave * 64u * S;
        const uint64_t rest = W.arena_len > wbase ? W.arena_len - wbase : 0;
        // integer clamp, made provably uniform: a descriptor hipcc cannot
        // prove uniform costs a waterfall loop per buffer load
        // (cdna_hip_programming.md T20); min(uint64_t, unsigned long long)
        // had resolved to the double overload
        const uint32_t rec = __builtin_amdgcn_readfirstlane(
            (uint32_t)(rest < 0xFFFFFFFFull ? rest : 0xFFFFFFFFull));
        const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(W.arena + wbase), (short)0, (int)rec, 0x00020000);
        if constexpr (EARLY && LANES == 64) {
            // one scan_segment site, run twice at most: the round (stopping
            // early only while W.early), then the owed tails
            uint32_t voff = W.lane * S, nun = S / kUnit, lo = rlo, hi = rhi, done;
            uint64_t vm = valid, pbase = P0;
            bool again = W.early != 0;
            for (;;) {
                const Chain c = scan_segment_early<kWR, kWPair, TSH, SMALL, kWG>(
                    rsrc, voff, nun, lo, hi, W.tab, W.k, vm, W.lane, done, again);
                const uint64_t hits = __builtin_amdgcn_ballot_w64(c.first != kNone) & vm;
                if (hits) best = readlane64(pbase + c.first, (uint32_t)__builtin_ctzll(hits));
                if (!again || done == nun) break;  // the tails' round, or a full round
                // stopped early (a lane L < 32 has a hit): lanes 0 .. L-1 owe
                // [done units, S) of their segments
                again = false;
                const uint32_t L = (uint32_t)__builtin_ctzll(hits);
                if (lb) *lb = 64ull * (done * 64u + 64u);
                if (L == 0) break;
                const uint32_t kk = 64u / L;  // >= 2 lanes per owed tail
                const uint32_t t0 = done * 64u, rem = S - t0;
                const uint32_t part = ((rem + kk - 1) / kk + 63u) / 64u * 64u;
                const uint32_t i = W.lane / kk, j = W.lane % kk;
                const uint32_t st = t0 + j * part;
                const bool on = i < L && st < S;
                const uint32_t len = on ? min(part, S - st) : 0u;
                // the owed lane's range of counted positions, shifted to this part
                const int32_t ilo = __shfl((int32_t)rlo, (int)min(i, 63u));
                const int32_t ihi = __shfl((int32_t)rhi, (int)min(i, 63u));
                lo = (uint32_t)min(max(ilo - (int32_t)st, 0), (int32_t)len);
                hi = (uint32_t)min(max(ihi - (int32_t)st, 0), (int32_t)len);
                vm = __builtin_amdgcn_ballot_w64(on && lo < hi);
                if (!vm) break;
                voff = i * S + st;
                nun = part / kUnit;
                pbase = A + 1 + (uint64_t)i * S + st;
                if (lb) *lb += 64ull * (part + 64u);
            }
            return best;
        }
        const Chain c = scan_segment<kWR, kWPair, TSH, SMALL, kWG>(rsrc, W.lane * S, S / kUnit,
                                                                   rlo, rhi, W.tab, W.k, valid,
                                                                   W.lane);
        const uint64_t hits = __builtin_amdgcn_ballot_w64(c.first != kNone) & valid;
        if (hits) {
            const uint32_t L = (uint32_t)__builtin_ctzll(hits);
            best = readlane64(P0 + c.first, L);
#ifdef RCDC_WALK_PRINTF
            if (LANES > 64 && W.lane == L)
                printf("round wave %u lane %u A %llu q %llu end %llu P0 %llu first %u rlo %u rhi %u -> %llu\n",
                       W.wave, L, (unsigned long long)A, (unsigned long long)q,
                       (unsigned long long)end, (unsigned long long)P0, c.first, rlo, rhi,
                       (unsigned long long)(P0 + c.first));
#endif
        }
    }
    if constexpr (LANES > 64) {
        if (W.lane == 0) W.red[W.wave] = best;
        __syncthreads();
        best = kNoCut;
        for (int w = 0; w < LANES / 64; w++) best = min(best, W.red[w]);
        best = uni64(best);
        __syncthreads();
    }
    return best;
}

// ---- gap rounds shared inside a check workgroup ----------------------------
// The chain phase lasts as long as its slowest boundary, and the slow ones
// hash unsearched gaps (up to min + 64 bytes: 8 sequential 64-lane rounds).
// A wave with a gap of >= 2 rounds posts them as jobs in an LDS ring; every
// wave of the workgroup that waits -- for its own jobs, or because no
// boundaries are left -- pops and runs jobs, so in the tail up to 16 waves
// hash one gap.  No barriers: LDS atomics, per-slot ready flags, s_sleep.
// Termination: a waiting wave runs jobs itself (its own included), so every
// posted job is run; idle waves leave when no wave is active and the ring is
// empty.  The walk kernel reuses the ring for its tail (walk_post below).
constexpr uint32_t kGapSlots = 256;  // >= 16 check waves x 16 rounds (walk: 16 x kHelpMax)
constexpr uint32_t kGapReq = 16;     // requesting waves (a workgroup of 1024)
struct GapQueue {
    uint32_t head, tail, active, idle;  // idle: walk waves that found no piece left
    uint32_t ready[kGapSlots];
    uint32_t req[kGapSlots];
    uint64_t A[kGapSlots], lo[kGapSlots], hi[kGapSlots], off[kGapSlots];
    unsigned long long hit[kGapReq];  // per requesting wave: min over its rounds
    uint32_t left[kGapReq];           // its rounds not yet run
};

__device__ __forceinline__ uint32_t lds_load(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ void lds_store(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Pop one job (wave-uniform): its ring slot, or kGapSlots if the ring is empty.
__device__ uint32_t gap_pop(GapQueue &Q, uint32_t lane) {
    uint32_t got = 0xFFFFFFFFu;
    if (lane == 0) {
        uint32_t h = lds_load(&Q.head);
        while (h < lds_load(&Q.tail)) {
            const uint32_t prev = atomicCAS(&Q.head, h, h + 1);
            if (prev == h) {
                got = h;
                break;
            }
            h = prev;
        }
    }
    got = __builtin_amdgcn_readfirstlane(got);
    if (got == 0xFFFFFFFFu) return kGapSlots;
    const uint32_t sl = got % kGapSlots, lap = got / kGapSlots + 1;
    // ready[sl] holds the lap of the job it carries (0: empty), so a job of
    // an earlier lap not yet copied out is never taken for this one
    while (__builtin_amdgcn_readfirstlane(lds_load(&Q.ready[sl])) != lap) __builtin_amdgcn_s_sleep(1);
    return sl;
}

// Run the job in slot sl: one 64-lane round, its first hit into hit[req].
template <int TSH, bool SMALL>
__device__ void gap_run(GapQueue &Q, Walk &W, uint32_t sl, uint64_t &rounds, uint64_t &lbytes) {
    const uint64_t A = Q.A[sl], lo = Q.lo[sl], hi = Q.hi[sl];
    const uint64_t off = Q.off[sl], own_off = W.off;
    const uint32_t r = Q.req[sl];
    wave_sync();
    if (W.lane == 0) lds_store(&Q.ready[sl], 0);  // fields copied: the slot is free
    // a hit the requester already has before this round makes it moot
    if (readlane64(__hip_atomic_load(&Q.hit[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP), 0) <= A) {
        if (W.lane == 0) atomicSub(&Q.left[r], 1u);
        return;
    }
    const uint32_t S = round_seg<64>(W.S, A, hi);
    W.off = off;  // (the requester's stream)
    const uint64_t h = round_first<64, TSH, SMALL>(W, A, lo, hi, S);
    W.off = own_off;
    rounds++;
    lbytes += 64ull * (S + 64);
    if (W.lane == 0) {
        if (h != kNoCut) atomicMin(&Q.hit[r], (unsigned long long)h);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        atomicSub(&Q.left[r], 1u);
    }
}

// The walk's tail: while waves of the workgroup have no piece left, a
// walker posts up to kHelpMax rounds after its round A to the ring, hashes
// A itself and then waits for the idle waves to run the posted ones (it runs
// none itself: one copy of the round loop per wave role keeps the walk
// kernel spill-free).  Rounds past a hit are wasted, but only on waves that
// would idle.
constexpr uint32_t kHelpMax = 15;  // WalkParams.helpers <= kHelpMax; x 16 walkers <= kGapSlots

__device__ void walk_post(Walk &W, uint64_t A, uint64_t q, uint64_t end, uint32_t K) {
    GapQueue &Q = *W.Q;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t step = 64ull * W.S;
    uint32_t t = 0;
    if (W.lane == 0) {
        Q.hit[wv] = kNoCut;
        lds_store(&Q.left[wv], K);
        t = atomicAdd(&Q.tail, K);
        for (uint32_t r = 0; r < K; r++) {
            const uint32_t sl = (t + r) % kGapSlots, lap = (t + r) / kGapSlots + 1;
            while (lds_load(&Q.ready[sl]) != 0) __builtin_amdgcn_s_sleep(1);
            Q.A[sl] = A + (r + 1) * step;
            Q.lo[sl] = q;
            Q.hi[sl] = end;
            Q.off[sl] = W.off;
            Q.req[sl] = wv;
            lds_store(&Q.ready[sl], lap);
        }
    }
    wave_sync();
}

// The first hit over the walker's own round (own) and its posted ones.
__device__ uint64_t walk_wait(Walk &W, uint64_t own) {
    GapQueue &Q = *W.Q;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (W.lane == 0 && own != kNoCut) atomicMin(&Q.hit[wv], (unsigned long long)own);
    while (__builtin_amdgcn_readfirstlane(lds_load(&Q.left[wv])) != 0) __builtin_amdgcn_s_sleep(2);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    uint64_t h = 0;
    if (W.lane == 0) h = Q.hit[wv];
    return readlane64(h, 0);
}

template <int LANES, int TSH, bool SMALL>
__device__ uint64_t walk_search(Walk &W, uint64_t q, uint64_t limit, uint64_t stop_scan,
                                uint64_t *kind);

// The end of the chunk starting at pos (rabin.rs:110-191), or kOpen if no
// cut was found below stop_scan (the search stopped there).  *kind: what the
// walker verified (rcdc_internal.h kKind*); *zero: all-zero prefill cut.
// cont_q != 0: the chunk from pos was searched hit-free up to cont_q by
// someone else (a seeded start continuing the previous piece's open chunk):
// no zone, the search resumes at cont_q.  (One call site of walk_search per
// kernel: a second inlined copy of the round loop spilled.)
template <int LANES, int TSH, bool SMALL>
__device__ uint64_t walk_next(Walk &W, uint64_t pos, uint64_t stop_scan, uint64_t *kind,
                              bool *zero, uint64_t cont_q = 0) {
    *zero = false;
    const uint64_t limit = min(pos + W.mx, W.N);  // rabin.rs:154 / EOF
    if (!cont_q && W.N - pos <= W.mn) {  // rabin.rs:141-147: the rest is the last chunk
        *kind = kKindEof;
        return W.N;
    }
    const uint64_t z = pos + W.mn;
    uint64_t zc = kNoCut;
    bool zz = false;
    if (cont_q) {
        // (the search below resumes at cont_q)
    } else if constexpr (LANES == 64) {
        W.zones++;
        if (W.zonefast)
            zc = zone_wave_fast<TSH>(W.arena + W.off, W.N, z, limit, W.mask, W.tab, W.k, W.win,
                                     W.lane, &zz);
        else
            zc = zone_wave(W.arena + W.off, W.N, z, limit, W.mask, W.shift, ModRepl{W.tab, W.k.lwm},
                           W.win, W.lane, &zz);
    } else {
        W.zones++;
        if (W.wave == 0) {
            zc = zone_wave_fast<TSH>(W.arena + W.off, W.N, z, limit, W.mask, W.tab, W.k, W.win,
                                     W.lane, &zz);
            if (W.lane == 0) {
                W.red[0] = zc;
                W.red[1] = zz;
            }
        }
        __syncthreads();
        zc = uni64(W.red[0]);
        zz = uni64(W.red[1]) != 0;
        __syncthreads();
    }
    if (zc != kNoCut) {
        *kind = kKindZone;
        *zero = zz;
        return zc;
    }
    if (!cont_q && limit <= z + 64) {
        *kind = limit == W.N ? kKindEof : kKindMax;
        return limit;
    }
    return walk_search<LANES, TSH, SMALL>(W, cont_q ? cont_q : z + 64, limit, stop_scan, kind);
}

// The pure-window search of a chunk (rabin.rs:153-188) from position q: its
// first hit below min(limit, stop_scan), else limit (kind Max / Eof) if the
// search reached it, else kOpen.  In rounds of LANES x S bytes; in the walk
// kernel's tail, idle waves of the workgroup hash rounds ahead (walk_post).
template <int LANES, int TSH, bool SMALL>
__device__ uint64_t walk_search(Walk &W, uint64_t q, uint64_t limit, uint64_t stop_scan,
                                uint64_t *kind) {
    const uint64_t end = min(limit, stop_scan);
    uint64_t A = round_base(W.off, q);
    while (A < end) {
        uint32_t K = 0;  // rounds posted for idle waves (the walk kernel's tail)
        if constexpr (LANES == 64) {
            if (W.Q) {
                const uint32_t idle = __builtin_amdgcn_readfirstlane(lds_load(&W.Q->idle));
                if (idle) {
                    const uint64_t step = 64ull * W.S, R = (end - A + step - 1) / step;
                    K = (uint32_t)min((uint64_t)min(idle, W.help_max), R - 1);
                    if (K) walk_post(W, A, q, end, K);
                }
            }
        }
        const uint32_t S = round_seg<LANES>(W.S, A, end);
        W.rounds++;
        uint64_t lb = (uint64_t)LANES * (S + 64);
        uint64_t p = round_first<LANES, TSH, SMALL, true>(W, A, q, end, S, &lb);
        W.lbytes += lb;
        if constexpr (LANES == 64) {
            if (K) p = walk_wait(W, p);
        }
        if (p != kNoCut) {
            *kind = kKindHit;
            return p;
        }
        A += (uint64_t)LANES * W.S * (K + 1);
    }
    if (end == limit) {
        *kind = limit == W.N ? kKindEof : kKindMax;
        return limit;
    }
    return kOpen;
}

// Index of cut value c in the sorted piece list L[0, n) (kind bits masked),
// or -2; one wave.
__device__ int64_t find_cut(const uint64_t *L, uint64_t n, uint64_t c, uint32_t lane) {
    for (uint64_t i0 = 0; i0 < n; i0 += 64) {
        const uint64_t i = i0 + lane;
        const uint64_t v = i < n ? (L[i] & kCutVal) : ~0ull;
        const uint64_t eq = __builtin_amdgcn_ballot_w64(v == c);
        if (eq) return (int64_t)(i0 + __builtin_ctzll(eq));
        if (__builtin_amdgcn_ballot_w64(v > c)) break;
    }
    return -2;
}

// Per-lane form of find_cut: binary search in the sorted list.
__device__ int64_t find_cut_lane(const uint64_t *L, uint64_t n, uint64_t c) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if ((L[mid] & kCutVal) < c) lo = mid + 1;
        else hi = mid;
    }
    return (lo < n && (L[lo] & kCutVal) == c) ? (int64_t)lo : -2;
}

}  // namespace

// ---------------------------------------------------------------------------
// Walk: one wave per unit, units pulled from ctr[0].
template <int TSH, bool SMALL>
__global__ __launch_bounds__(1024, 1) void rcdc_walk_kernel(
    const uint8_t *__restrict__ arena, const StreamDesc *__restrict__ sds,
    const WalkUnit *__restrict__ units, WalkParams prm, const uint64_t *__restrict__ gtab,
    uint64_t *__restrict__ piece_cuts, uint64_t *__restrict__ pstatus, uint32_t *ctr) {
    __shared__ __attribute__((aligned(16))) uint8_t s_tab[kLdsBytes];
    __shared__ __attribute__((aligned(16))) uint8_t s_win[16][128];
    __shared__ BlockStats s_st;
    __shared__ GapQueue s_q;
    // this run's counters (WalkParams.qbase): the chain counters of the set
    // start at 0 (the chain of the set's previous run has finished -- the run
    // waits for it -- and this run's chain starts after this kernel), and the
    // work counters of run r + 2 (WalkParams.stats_next)
    // (device-scope atomics, like the adds: a plain store could sit in this
    // XCD's L2 and be written back over the other XCDs' atomic adds)
    if (blockIdx.x == 0 && (prm.flags & kWalkKReset)) {
        if (threadIdx.x >= 1 && threadIdx.x < 4) atomicExch(&ctr[threadIdx.x], 0u);
        if (threadIdx.x < kWalkStats && prm.stats_next) atomicExch(&prm.stats_next[threadIdx.x], 0ull);
    }
    stats_init(s_st);
    if (threadIdx.x == 0) {
        s_q.head = s_q.tail = 0;
        s_q.active = 16;
        s_q.idle = 0;
    }
    for (uint32_t i = threadIdx.x; i < kGapSlots; i += blockDim.x) s_q.ready[i] = 0;
    fill_tables(s_tab, gtab, prm.idx_shift, threadIdx.x, 1024);  // (ends with a barrier)
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    Walk W;
    W.arena = arena;
    W.arena_len = prm.arena_len;
    W.mn = prm.min_size;
    W.mx = prm.max_size;
    W.S = prm.seg_bytes;
    W.mask = prm.mask;
    W.shift = prm.shift;
    W.tab = s_tab;
    W.k = make_consts(lane, prm.mask, prm.idx_shift);
    W.win = s_win[wave];
    W.red = nullptr;
    W.lane = lane;
    W.wave = 0;  // a wave walker: lane t of the round is t
    W.tid = lane;
    W.Q = prm.helpers ? &s_q : nullptr;
    W.help_max = __builtin_amdgcn_readfirstlane(min(prm.helpers, kHelpMax));
    W.early = prm.early;
    W.zonefast = __builtin_amdgcn_readfirstlane(prm.flags & kWalkZoneFast);
    uint64_t help_rounds = 0, help_bytes = 0;  // rounds this wave ran for others
    // kWalkStatic: the first piece is the wave's global index, later ones
    // come from the counter, offset by the launch's waves (all scalars: no
    // state live across the walk)
    auto take = [&]() -> uint32_t {
        uint32_t t = 0;
        if (lane == 0)
            t = atomicAdd(&ctr[0], 1u) - prm.qbase + ((prm.flags & kWalkStatic) ? gridDim.x * 16u : 0u);
        return __builtin_amdgcn_readfirstlane(t);
    };
    uint32_t q = (prm.flags & kWalkStatic) ? __builtin_amdgcn_readfirstlane(blockIdx.x * 16u + wave)
                                           : take();
    for (;; q = take()) {
        if (q >= prm.nunits) break;
        const uint32_t u = __builtin_amdgcn_readfirstlane(prm.order[q]);
        const uint64_t t0 = prm.trace ? (uint64_t)wall_clock64() : 0;
        W.rounds = W.zones = 0;
        W.lbytes = 0;
        const WalkUnit U = units[u];
        const StreamDesc d = sds[U.stream];
        W.off = d.off;
        W.N = d.n;
        const uint8_t *s = arena + d.off;
        uint64_t *out = piece_cuts + U.out_base;
        const uint64_t stop_scan = U.stop < d.n ? U.stop + W.mn + 64 : ~0ull;
        uint64_t pos = U.start, n = 0;
        bool open = false;
        // Seeded start: if the previous piece of the stream has finished in
        // this run, continue its chain (closed at its last cut, or inside its
        // open chunk) instead of assuming a cut at U.start -- the chains then
        // agree from here on and this piece hashes nothing the true chain
        // skips (rcdc_internal.h WalkParams.wstate).
        uint64_t seedw = kSeedNone << 62;  // (stored now: nothing live across the walk)
        bool cont = false;
        if (prm.seed && U.piece > 0) {
            uint64_t pe = 0;
            if (lane == 0)
                pe = __hip_atomic_load(prm.wstate + (u - 1), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            pe = readlane64(pe, 0);
            if (end_epoch(pe) == prm.epoch && (pe & kEndPos) != kEndNone) {
                const uint64_t pp = pe & kEndPos;
                if ((pe & kEndOpen) && pp < U.start) {
                    cont = true;  // chunk [pp, ...) searched hit-free up to U.start + min + 64
                    pos = pp;
                    seedw = (kSeedOpen << 62) | pp;
                } else if (!(pe & kEndOpen) && pp >= U.start && pp < U.stop) {
                    pos = pp;
                    seedw = (kSeedClosed << 62) | pp;
                }
            }
        }
        if (prm.wstate && lane == 0) prm.wstate[prm.nunits + u] = seedw;
        while (pos < d.n && (n == 0 || pos < U.stop)) {
            uint64_t kind;
            bool zero;
            const uint64_t c = walk_next<64, TSH, SMALL>(W, pos, stop_scan, &kind, &zero,
                                                         cont ? U.start + W.mn + 64 : 0);
            cont = false;
            if (c == kOpen) {
                open = true;
                break;
            }
            if (lane == 0 && n < U.out_cap) out[n] = c | (kind << 62);
            n++;
            pos = c;
            if (pos >= U.stop) break;
            // inside a zero run: up to 64 further min-sized chunks per step
            while (zero && pos < d.n) {
                uint32_t m = zero_run(s, d.n, W.mn, W.mx, pos, lane);
                if (m == 0) break;
                if (pos + (uint64_t)m * W.mn >= U.stop)
                    m = (uint32_t)((U.stop - pos + W.mn - 1) / W.mn);
                if (lane < m && n + lane < U.out_cap)
                    out[n + lane] = (pos + (lane + 1) * W.mn) | (kKindZone << 62);
                n += m;
                pos += (uint64_t)m * W.mn;
                if (pos >= U.stop || m < 64) break;
            }
            if (pos >= U.stop) break;
        }
        if (lane == 0) {
            pstatus[u] = min(n, (uint64_t)U.out_cap) | (open ? kOpenFlag : 0ull) |
                         (n > U.out_cap ? (kOpenFlag << 1) : 0ull);
            if (prm.wstate)
                __hip_atomic_store(prm.wstate + u,
                                   end_word(open, prm.epoch, n > U.out_cap ? kEndNone : pos),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            stats_add(s_st, kWalkStatRounds, W.rounds);
            stats_add(s_st, kWalkStatZones, W.zones);
            stats_add(s_st, kWalkStatBytes, W.lbytes);
            stats_add(s_st, kWalkStatChunks, n);
            if (prm.trace) {
                unsigned long long *tr = prm.trace + (uint64_t)u * kTraceWords;
                tr[0] = t0;
                tr[1] = (uint64_t)wall_clock64();
                tr[2] = W.rounds;
                tr[3] = n;
            }
        }
    }
    // no piece left: hash other walkers' rounds until every walker of the
    // workgroup is done and the ring is empty
    if (lane == 0) {
        atomicAdd(&s_q.idle, 1u);
        atomicSub(&s_q.active, 1u);
    }
    for (;;) {
        const uint32_t sl = gap_pop(s_q, lane);
        if (sl < kGapSlots) {
            gap_run<TSH, SMALL>(s_q, W, sl, help_rounds, help_bytes);
            continue;
        }
        const uint32_t act = __builtin_amdgcn_readfirstlane(lds_load(&s_q.active));
        const uint32_t hd = __builtin_amdgcn_readfirstlane(lds_load(&s_q.head));
        const uint32_t tl = __builtin_amdgcn_readfirstlane(lds_load(&s_q.tail));
        if (act == 0 && hd == tl) break;
        __builtin_amdgcn_s_sleep(2);
    }
    if (lane == 0) {
        stats_add(s_st, kWalkStatRounds, help_rounds);
        stats_add(s_st, kWalkStatBytes, help_bytes);
    }
    stats_flush(s_st, prm.stats);
}

// ---------------------------------------------------------------------------
// Check: one wave per boundary (piece j >= 1 starts at a_j), boundaries pulled
// from ctr[2]; 16 waves per workgroup share the LDS tables.
//
// From the exact chain state at the end of piece j - 1 the wave steps the
// true chain (rabin.rs:110-191) until one of its cuts lies on a later
// piece's chain (a piece start or a cut of its list: from there both chains
// are the same function of the position).  A step needs, for the chunk from
// c, its zone (zone_wave) and the first pure-window hit >= c + min + 64.
// What the walkers verified answers most of that: every walked chunk t of
// any piece searched [prev_t + min + 64, cut_t) hit-free, ending at a hit
// (kind Hit), at prev_t + max (Max) or at N (Eof), and an open piece
// searched [c_last + min + 64, stop + min + 64).  These are facts about
// positions, whichever chain produced them.  Positions nobody hashed (the
// skipped min-prefix of a piece's own chunks: the true chain is out of phase
// there) are hashed here, at most min + 64 bytes per gap, with the walk's
// 64-lane rounds.  Inside a zero run (all-zero prefill: every chunk exactly
// min) the chain advances 64 chunks per step and records them as one run.
// A boundary that needs more than kMaxHops entries or kCheckBudget hashed
// bytes goes on the fixup list.
constexpr uint64_t kHopRun = 1;  // hop entry kind: cuts prev + min, prev + 2 min, ..., value

struct PieceView {
    const uint64_t *L;
    uint64_t n, start, stop;
    uint64_t cstart;  // the chain's first point (a cut; kNoCut: it continues an
                      // open chunk of the previous piece, kSeedOpen)
    uint64_t prev0;   // chunk 0 searched [prev0 + min + 64, L[0])
    bool open, full;  // full: the list holds every cut the walker found
};

// pseed: WalkParams.wstate + nunits (nullptr: no seeding, every chain starts
// with a cut at its piece start).
__device__ __forceinline__ PieceView piece_view(const WalkUnit *units, const uint64_t *pstatus,
                                                const uint64_t *piece_cuts, uint32_t uk,
                                                const uint64_t *pseed) {
    const WalkUnit Uk = units[uk];
    const uint64_t st = pstatus[uk];
    PieceView V;
    V.L = piece_cuts + Uk.out_base;
    V.n = st & 0xFFFFFFFFu;
    V.start = Uk.start;
    V.stop = Uk.stop;
    V.open = (st & kOpenFlag) != 0;
    V.full = (st & (kOpenFlag << 1)) == 0;
    V.cstart = Uk.start;
    V.prev0 = Uk.start;
    if (pseed) {
        const uint64_t sd = pseed[uk], kind = sd >> 62, pos = sd & kCutVal;
        if (kind == kSeedClosed) V.cstart = V.prev0 = pos;
        else if (kind == kSeedOpen) V.cstart = kNoCut;  // (prev0 = start: its first
                                                        // search began at start + min + 64)
    }
    return V;
}

// First index t with cut value >= p (n if none); uniform binary search.
__device__ __forceinline__ uint64_t lower_cut(const uint64_t *L, uint64_t n, uint64_t p) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if ((L[mid] & kCutVal) < p) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// lower_cut for a wave-uniform query: piece lists are short (<= Lp / min +
// max / min + 4 entries), so a wave reads 64 of them per round trip instead
// of a chain of dependent loads.
__device__ __forceinline__ uint64_t lower_cut_wave(const uint64_t *L, uint64_t n, uint64_t p) {
    const uint32_t lane = __lane_id();
    for (uint64_t i0 = 0; i0 < n; i0 += 64) {
        const uint64_t i = i0 + lane;
        const uint64_t v = i < n ? (L[i] & kCutVal) : ~0ull;
        const uint64_t ge = __builtin_amdgcn_ballot_w64(v >= p);
        if (ge) return i0 + (uint64_t)__builtin_ctzll(ge);
    }
    return n;
}

// What piece V knows about position p: returns true if a searched interval
// holds p -- [p, *vend) is hit-free, and *vkind says what *vend is (kKindHit:
// a hit; kKindMax / kOpen: nothing known at *vend; kKindEof: p .. N hit-free);
// otherwise *next = the start of V's next searched interval after p (~0 if
// none known).
__device__ bool cover(const PieceView &V, uint64_t p, uint64_t mn, uint64_t *vend, uint64_t *vkind,
                      uint64_t *next) {
    *next = ~0ull;
    if (!V.full) return false;
    const uint64_t t = lower_cut_wave(V.L, V.n, p);
    if (t < V.n) {
        const uint64_t prev = t ? (V.L[t - 1] & kCutVal) : V.prev0;
        const uint64_t base = prev + mn + 64;
        const uint64_t kd = V.L[t] >> 62, v = V.L[t] & kCutVal;
        // chunk t searched [base, v) hit-free; v is a hit (Hit), untested
        // (Max: the reference stops before testing prev + max) or N (Eof)
        if (kd != kKindZone && base <= p && (p < v || kd == kKindHit)) {
            *vend = v;
            *vkind = kd;
            return true;
        }
        // otherwise the next searched interval: chunk t's own (p before it),
        // or chunk t + 1's, which starts at v (Zone cuts search nothing;
        // p == v: the untested end of a Max chunk)
        *next = (kd != kKindZone && p < base) ? base : v + mn + 64;
        return false;
    }
    if (V.open) {
        const uint64_t base = (V.n ? (V.L[V.n - 1] & kCutVal) : V.prev0) + mn + 64;
        const uint64_t oend = V.stop + mn + 64;
        if (base <= p && p < oend) {
            *vend = oend;
            *vkind = kOpen;
            return true;
        }
        if (p < base) *next = base;
    }
    return false;
}

struct CheckCtx {
    const WalkUnit *units;
    const uint64_t *pstatus, *piece_cuts;
    const uint64_t *pseed;  // nullptr: no seeded starts
    WalkUnit U;   // the boundary's unit (piece j)
    uint32_t u;   // its index
    uint64_t N, mn, mx;
    uint64_t Lp, Ls;  // piece sizes (piece_at)
    uint64_t budget;  // bytes this boundary may still hash
};


// Piece index k (within the stream of unit0, npieces pieces) holding
// position p: the last piece with start <= p (pieces differ in size).
__device__ __forceinline__ uint32_t piece_at(const WalkUnit *units, uint32_t unit0,
                                             uint32_t npieces, uint64_t p) {
    uint32_t lo = 0, hi = npieces - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (units[unit0 + mid].start <= p) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// The same in closed form: nbig pieces of Lp, then pieces of Ls, the last
// one running to N.
__device__ __forceinline__ uint32_t piece_at(const WalkUnit &U, uint64_t Lp, uint64_t Ls,
                                             uint64_t p) {
    const uint64_t B = (uint64_t)U.nbig * Lp;
    const uint64_t k = p < B ? p / Lp : (uint64_t)U.nbig + (p - B) / Ls;
    return (uint32_t)min(k, (uint64_t)U.npieces - 1);
}

__device__ __forceinline__ uint32_t piece_of(const CheckCtx &C, uint64_t p) {
    return piece_at(C.U, C.Lp, C.Ls, p);
}

// First pure-window hit in [lo, lim) of the stream, or lim if none;
// kNoCut if the hashing budget ran out.
template <int TSH, bool SMALL>
__device__ uint64_t check_first_hit(Walk &W, CheckCtx &C, uint64_t lo, uint64_t lim,
                                    GapQueue *Q, uint32_t wave, uint64_t *shared_rounds,
                                    uint64_t *shared_lbytes) {
    uint64_t p = lo;
    // every iteration passes one searched interval or one gap: at most ~2 per
    // min bytes of [lo, lim); the cap only guarantees termination
    const uint64_t max_iter = 2 * ((lim - lo) / C.mn) + 16;
    for (uint64_t it = 0; p < lim; it++) {
        if (it > max_iter) return kNoCut;  // (never) -> fixup list
        const uint32_t k = piece_of(C, p);
        bool known = false;
        uint64_t gap_end = lim;
        for (int back = 0; back < 2 && !known; back++) {
            if (back == 1 && k == 0) break;
            const PieceView V = piece_view(C.units, C.pstatus, C.piece_cuts, C.U.unit0 + k - back,
                                           C.pseed);
            uint64_t vend, vkind, nxt;
            if (cover(V, p, C.mn, &vend, &vkind, &nxt)) {
                if (vkind == kKindHit) return min(vend, lim);
                if (vkind == kKindEof || lim <= vend) return lim;
                p = vend;  // Max / open: hit-free below vend, vend itself unknown
                known = true;
            } else {
                gap_end = min(gap_end, nxt);
            }
        }
        if (known) continue;
        gap_end = max(gap_end, p + 1);
        // hash [p, gap_end): nobody searched it
        if (gap_end - p > C.budget) return kNoCut;
        C.budget -= gap_end - p;
        uint64_t A = round_base(W.off, p);
        const uint64_t step = 64ull * W.S;
        const uint64_t R = (gap_end - A + step - 1) / step;
        if (Q && R >= 2 && R <= 16) {  // (ring capacity: 16 waves x 16)
            // post the R rounds, then run jobs until ours are done
            uint32_t t = 0;
            if (W.lane == 0) {
                Q->hit[wave] = kNoCut;
                lds_store(&Q->left[wave], (uint32_t)R);
                t = atomicAdd(&Q->tail, (uint32_t)R);
            }
            t = __builtin_amdgcn_readfirstlane(t);
            if (W.lane == 0) {
                for (uint32_t r = 0; r < (uint32_t)R; r++) {
                    const uint32_t sl = (t + r) % kGapSlots, lap = (t + r) / kGapSlots + 1;
                    while (lds_load(&Q->ready[sl]) != 0) __builtin_amdgcn_s_sleep(1);
                    Q->A[sl] = A + r * step;
                    Q->lo[sl] = p;
                    Q->hi[sl] = gap_end;
                    Q->off[sl] = W.off;
                    Q->req[sl] = wave;
                    lds_store(&Q->ready[sl], lap);
                }
            }
            wave_sync();
            while (__builtin_amdgcn_readfirstlane(lds_load(&Q->left[wave])) != 0) {
                const uint32_t sl = gap_pop(*Q, W.lane);
                if (sl < kGapSlots) gap_run<TSH, SMALL>(*Q, W, sl, *shared_rounds, *shared_lbytes);
                else __builtin_amdgcn_s_sleep(2);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            uint64_t h = 0;
            if (W.lane == 0) h = Q->hit[wave];
            h = readlane64(h, 0);
            if (h != kNoCut) return h;
        } else {
            while (A < gap_end) {
                const uint32_t S = round_seg<64>(W.S, A, gap_end);
                W.rounds++;
                W.lbytes += 64ull * (S + 64);
                const uint64_t h = round_first<64, TSH, SMALL>(W, A, p, gap_end, S);
                if (h != kNoCut) return h;
                A += step;
            }
        }
        p = gap_end;
    }
    return lim;
}

// The true chain has a cut at c: does a later piece's chain (unit >= C.u)
// have one there too?  *mu / *idx: the unit and list index (-1 = its start).
__device__ __forceinline__ bool merged_at(const CheckCtx &C, uint64_t c, uint32_t *mu, int32_t *idx) {
    const uint32_t k = piece_of(C, c);
    for (int back = 0; back < 2; back++) {
        if (back == 1 && k == 0) break;
        const uint32_t uk = C.U.unit0 + k - back;
        if (uk < C.u) break;
        const PieceView V = piece_view(C.units, C.pstatus, C.piece_cuts, uk, C.pseed);
        if (back == 0 && c == V.cstart) {
            *mu = uk;
            *idx = -1;
            return true;
        }
        if (!V.full) continue;
        const uint64_t t = lower_cut(V.L, V.n, c);
        if (t < V.n && (V.L[t] & kCutVal) == c) {
            *mu = uk;
            *idx = (int32_t)t;
            return true;
        }
    }
    return false;
}

// Workgroup size CT: 512 threads (8 waves, 256 VGPRs, spill-free) for
// serial runs; 1024 (16 waves) beside the next walk of a pipelined plan:
// the check is latency bound and there each workgroup holds a CU the walk
// waits for, so more boundaries in flight per CU free it sooner (C3 step
// 9.33 -> 9.26 ms in an interleaved A/B) although at 128 VGPRs the gap
// search spills (~280 B per lane).  Serial C5 was slower with 1024
// (chain 126 -> 154 us).

template <int TSH, bool SMALL, int CT>
__global__ __launch_bounds__(CT, 1) void rcdc_walk_check_kernel(
    const uint8_t *__restrict__ arena, const StreamDesc *__restrict__ sds,
    const WalkUnit *__restrict__ units, WalkParams prm, const uint64_t *__restrict__ gtab,
    const uint64_t *__restrict__ piece_cuts, const uint64_t *__restrict__ pstatus,
    BoundRes *__restrict__ bres, uint32_t *ctr, uint32_t *__restrict__ fixlist) {
    __shared__ __attribute__((aligned(16))) uint8_t s_tab[kLdsBytes];
    __shared__ __attribute__((aligned(16))) uint8_t s_win[CT / 64][128];
    __shared__ uint64_t s_hops[CT / 64][kMaxHops];  // the wave's hop entries
    __shared__ BlockStats s_st;
    __shared__ GapQueue s_q;
    // this run's counters (WalkParams.qbase): the chain counters of the set
    // start at 0 (the chain of the set's previous run has finished -- the run
    // waits for it -- and this run's chain starts after this kernel), and the
    // work counters of run r + 2 (WalkParams.stats_next)
    // (device-scope atomics, like the adds: a plain store could sit in this
    // XCD's L2 and be written back over the other XCDs' atomic adds)
    if (blockIdx.x == 0 && (prm.flags & kWalkKReset)) {
        if (threadIdx.x >= 1 && threadIdx.x < 4) atomicExch(&ctr[threadIdx.x], 0u);
        if (threadIdx.x < kWalkStats && prm.stats_next) atomicExch(&prm.stats_next[threadIdx.x], 0ull);
    }
    stats_init(s_st);
    if (threadIdx.x == 0) {
        s_q.head = s_q.tail = 0;
        s_q.active = CT / 64;
    }
    for (uint32_t i = threadIdx.x; i < kGapSlots; i += blockDim.x) s_q.ready[i] = 0;
    fill_tables(s_tab, gtab, prm.idx_shift, threadIdx.x, CT);  // (ends with a barrier)
    uint64_t shared_rounds = 0, shared_lbytes = 0;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    Walk W;
    W.arena = arena;
    W.arena_len = prm.arena_len;
    W.mn = prm.min_size;
    W.mx = prm.max_size;
    W.S = prm.seg_bytes;
    W.mask = prm.mask;
    W.shift = prm.shift;
    W.tab = s_tab;
    W.k = make_consts(lane, prm.mask, prm.idx_shift);
    W.win = s_win[wave];
    W.red = nullptr;
    W.lane = lane;
    W.wave = 0;
    W.tid = lane;
    W.Q = nullptr;
    W.help_max = 0;
    W.early = 0;
    W.zonefast = __builtin_amdgcn_readfirstlane(prm.flags & kWalkZoneFast);
    const uint64_t mn = prm.min_size, mx = prm.max_size;
    auto take = [&]() -> uint32_t {  // (kWalkStatic as the walk kernel)
        uint32_t t = 0;
        if (lane == 0)
            t = atomicAdd(&ctr[2], 1u) + ((prm.flags & kWalkStatic) ? gridDim.x * (CT / 64u) : 0u);
        return __builtin_amdgcn_readfirstlane(t);
    };
    uint32_t u = (prm.flags & kWalkStatic)
                     ? __builtin_amdgcn_readfirstlane(blockIdx.x * (CT / 64u) + wave)
                     : take();
    for (;; u = take()) {
        if (u >= prm.nunits) break;
        const WalkUnit U = units[u];
        if (U.piece == 0) continue;
        const uint64_t t0 = prm.trace ? (uint64_t)wall_clock64() : 0;
        W.rounds = W.zones = 0;
        W.lbytes = 0;
        const StreamDesc d = sds[U.stream];
        W.off = d.off;
        W.N = d.n;
        const uint8_t *s = arena + d.off;
        const uint64_t N = d.n;
        CheckCtx C;
        C.units = units;
        C.pstatus = pstatus;
        C.piece_cuts = piece_cuts;
        C.pseed = prm.wstate ? prm.wstate + prm.nunits : nullptr;
        C.U = U;
        C.u = u;
        C.N = N;
        C.mn = mn;
        C.mx = mx;
        C.Lp = prm.piece_bytes;
        C.Ls = prm.small_bytes;
        C.budget = prm.chk_budget;
        // result (wave-uniform scalars; the hop entries in LDS, not in a
        // dynamically indexed register array, which would go to scratch)
        struct {
            uint32_t kind, nhops, merge_unit;
            int32_t merge_idx;
            uint64_t fix_from;
        } R = {kBoundNone, 0, u, -1, 0};
        uint64_t *hops = s_hops[wave];
        // exact state at the previous piece's end: closed at c, or open from c
        // ([c+min+64, a_j+min+64) hit-free, no zone cut in c's zone)
        const PieceView Vp = piece_view(units, pstatus, piece_cuts, u - 1, C.pseed);
        uint64_t c;
        bool pending = false;
        if (prm.wstate) {  // the end state the previous walker published
            const uint64_t pe = prm.wstate[u - 1];
            c = pe & kEndPos;
            pending = (pe & kEndOpen) != 0;
            if (c == kEndNone) c = Vp.n ? (Vp.L[Vp.n - 1] & kCutVal) : Vp.start;  // (!full below)
        } else if (Vp.open) {
            c = Vp.n ? (Vp.L[Vp.n - 1] & kCutVal) : Vp.start;
            pending = true;
        } else {
            c = Vp.n ? (Vp.L[Vp.n - 1] & kCutVal) : N;
        }
        if (!Vp.full) {
            R.kind = kBoundFixup;  // (never: lists are sized for every cut)
            R.fix_from = c;
        } else if (!pending && c >= N) {
            // the stream ended before this piece: kBoundNone
        } else {
            for (;;) {
                if (!pending) {
                    uint32_t mu;
                    int32_t mi;
                    if (merged_at(C, c, &mu, &mi)) {
                        R.kind = kBoundMerged;
                        R.merge_unit = mu;
                        R.merge_idx = mi;
                        break;
                    }
                    if (R.nhops >= (uint32_t)kMaxHops) {
                        R.kind = kBoundFixup;
                        R.fix_from = c;
                        break;
                    }
                }
                uint64_t nxt = kNoCut, lo = 0;
                const uint64_t lim = min(c + mx, N);
                bool zz = false;
                if (pending) {
                    pending = false;
                    lo = U.start + mn + 64;
                } else if (N - c <= mn) {
                    nxt = N;
                } else {
                    const uint64_t z = c + mn;
                    W.zones++;
                    const uint64_t zc =
                        W.zonefast ? zone_wave_fast<TSH>(s, N, z, lim, prm.mask, s_tab, W.k, W.win,
                                                         lane, &zz)
                                   : zone_wave(s, N, z, lim, prm.mask, prm.shift,
                                               ModRepl{s_tab, W.k.lwm}, W.win, lane, &zz);
                    if (zc != kNoCut) nxt = zc;
                    else if (lim <= z + 64) nxt = lim;
                    else lo = z + 64;
                }
                if (lo) nxt = check_first_hit<TSH, SMALL>(W, C, lo, lim, &s_q, wave, &shared_rounds,
                                                                &shared_lbytes);
                if (nxt == kNoCut) {
                    R.kind = kBoundFixup;
                    R.fix_from = c;
                    break;
                }
                hops[R.nhops++] = nxt;
                c = nxt;
                if (c >= N) {
                    R.kind = kBoundEnd;
                    break;
                }
                // inside a zero run: 64 min-sized chunks per step, the first
                // one on a later piece's chain ends the boundary
                bool done = false;
                while (zz && c < N) {
                    uint32_t mu0;
                    int32_t mi0;
                    if (merged_at(C, c, &mu0, &mi0)) break;  // the loop top merges
                    const uint32_t m = zero_run(s, N, mn, mx, c, lane);
                    if (m == 0) break;
                    const uint64_t cut = c + (uint64_t)(lane + 1) * mn;
                    uint32_t mu = kNoUnit;
                    int32_t mi = -1;
                    const bool on = lane < m && merged_at(C, cut, &mu, &mi);
                    const uint64_t hit = __builtin_amdgcn_ballot_w64(on);
                    const uint32_t f = hit ? (uint32_t)__builtin_ctzll(hit) : m - 1;
                    const uint64_t end = c + (uint64_t)(f + 1) * mn;
                    // record c+min .. end as one run entry (extending a run
                    // just before it)
                    if (R.nhops > 0 && (hops[R.nhops - 1] >> 62) == kHopRun) {
                        hops[R.nhops - 1] = end | (kHopRun << 62);
                    } else if (R.nhops < (uint32_t)kMaxHops) {
                        hops[R.nhops++] = end | (kHopRun << 62);
                    } else {
                        R.kind = kBoundFixup;
                        R.fix_from = c;
                        done = true;
                        break;
                    }
                    c = end;
                    if (hit) {
                        R.kind = kBoundMerged;
                        R.merge_unit = (uint32_t)__builtin_amdgcn_readlane(mu, f);
                        R.merge_idx = (int32_t)__builtin_amdgcn_readlane((uint32_t)mi, f);
                        done = true;
                        break;
                    }
                    if (c >= N) {
                        R.kind = kBoundEnd;
                        done = true;
                        break;
                    }
                    if (m < 64) break;
                }
                if (done) break;
            }
        }
        wave_sync();
        BoundRes *B = bres + u;
        if (lane < R.nhops) B->hops[lane] = hops[lane];
        if (lane == 0) {
            B->kind = R.kind;
            B->nhops = R.nhops;
            B->merge_unit = R.merge_unit;
            B->merge_idx = R.merge_idx;
            B->fix_from = R.fix_from;
            if (R.kind == kBoundFixup) fixlist[atomicAdd(&ctr[1], 1u)] = u;
            stats_add(s_st, kWalkStatChkRounds, W.rounds);
            stats_add(s_st, kWalkStatChkZones, W.zones);
            stats_add(s_st, kWalkStatChkBytes, W.lbytes);
            if (prm.trace) {
                unsigned long long *tr = prm.trace + ((uint64_t)prm.nunits + u) * kTraceWords;
                tr[0] = t0;
                tr[1] = (uint64_t)wall_clock64();
                tr[2] = W.rounds;
                tr[3] = R.nhops;
            }
        }
    }
    // no boundaries left: run the other waves' gap rounds until none can come
    if (lane == 0) atomicSub(&s_q.active, 1u);
    for (;;) {
        const uint32_t sl = gap_pop(s_q, lane);
        if (sl < kGapSlots) {
            gap_run<TSH, SMALL>(s_q, W, sl, shared_rounds, shared_lbytes);
            continue;
        }
        const uint32_t act = __builtin_amdgcn_readfirstlane(lds_load(&s_q.active));
        const uint32_t hd = __builtin_amdgcn_readfirstlane(lds_load(&s_q.head));
        const uint32_t tl = __builtin_amdgcn_readfirstlane(lds_load(&s_q.tail));
        if (act == 0 && hd == tl) break;
        __builtin_amdgcn_s_sleep(2);
    }
    if (lane == 0) {
        stats_add(s_st, kWalkStatChkRounds, shared_rounds);
        stats_add(s_st, kWalkStatChkBytes, shared_lbytes);
    }
    stats_flush(s_st, prm.stats);
}

// ---------------------------------------------------------------------------
// Fixup: persistent workgroups over the boundaries the check could not
// resolve; each walks the exact chain with 1024-lane rounds until a cut lies
// on a piece's chain (that piece's list, or the previous one's crossing cut).
template <int TSH, bool SMALL>
__global__ __launch_bounds__(1024, 1) void rcdc_walk_fixup_kernel(
    const uint8_t *__restrict__ arena, const StreamDesc *__restrict__ sds,
    const WalkUnit *__restrict__ units, WalkParams prm, const uint64_t *__restrict__ gtab,
    const uint64_t *__restrict__ piece_cuts, const uint64_t *__restrict__ pstatus,
    const BoundRes *__restrict__ bres, uint32_t *ctr, const uint32_t *__restrict__ fixlist,
    uint64_t *__restrict__ fix_cuts, FixRes *__restrict__ fixres) {
    const uint32_t nfix = __atomic_load_n(&ctr[1], __ATOMIC_RELAXED);
    if (blockIdx.x >= nfix) return;
    __shared__ __attribute__((aligned(16))) uint8_t s_tab[kLdsBytes];
    __shared__ __attribute__((aligned(16))) uint8_t s_win[128];
    __shared__ uint64_t s_red[16];
    __shared__ uint64_t s_bc[4];
    fill_tables(s_tab, gtab, prm.idx_shift, threadIdx.x, 1024);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    Walk W;
    W.arena = arena;
    W.arena_len = prm.arena_len;
    W.mn = prm.min_size;
    W.mx = prm.max_size;
    W.S = prm.fix_seg;
    W.mask = prm.mask;
    W.shift = prm.shift;
    W.tab = s_tab;
    W.k = make_consts(lane, prm.mask, prm.idx_shift);
    W.win = s_win;
    W.red = s_red;
    W.lane = lane;
    W.wave = wave;
    W.tid = threadIdx.x;
    W.Q = nullptr;
    W.help_max = 0;
    W.early = 0;
    W.zonefast = __builtin_amdgcn_readfirstlane(prm.flags & kWalkZoneFast);
    for (uint32_t idx = blockIdx.x; idx < nfix; idx += gridDim.x) {
        const uint32_t u = fixlist[idx];
        const WalkUnit U = units[u];
        const StreamDesc d = sds[U.stream];
        W.off = d.off;
        W.N = d.n;
        const uint8_t *s = arena + d.off;
        uint64_t *out = fix_cuts + (uint64_t)u * prm.fix_cap;
        uint64_t c = bres[u].fix_from, n = 0;
        W.rounds = W.zones = 0;
        W.lbytes = 0;
        uint32_t munit = kNoUnit;
        int32_t midx = -1;
        while (c < d.n && n <= prm.fix_cap) {
            uint64_t kind;
            bool zero;
            uint64_t nxt = walk_next<1024, TSH, SMALL>(W, c, ~0ull, &kind, &zero);
            // The cuts nxt, nxt + min, ... (m > 1 inside a zero run); wave 0
            // checks them lane-parallel and the first one on a piece chain (or
            // at N) ends the run of cuts.
            if (wave == 0) {
                uint32_t m = 1;
                if (zero && nxt < d.n)
                    m = 1 + min(zero_run(s, d.n, W.mn, W.mx, nxt, lane), 63u);
                const uint64_t cut = nxt + (uint64_t)lane * W.mn;
                uint32_t mu = kNoUnit;
                int64_t at = -2;
                bool stop = false;
                if (lane < m) {
                    if (cut >= d.n) {
                        stop = true;
                    } else {
                        const uint64_t k = piece_at(U, prm.piece_bytes, prm.small_bytes, cut);
                        for (int back = 0; back < 2 && mu == kNoUnit; back++) {
                            if (back == 1 && k == 0) break;
                            const uint32_t uk = U.unit0 + (uint32_t)(k - back);
                            if (uk < u) break;  // never before the boundary's own piece
                            const WalkUnit Uk = units[uk];
                            uint64_t cst = Uk.start;  // the chain's first point (PieceView.cstart)
                            if (prm.wstate) {
                                const uint64_t sd = prm.wstate[prm.nunits + uk];
                                if ((sd >> 62) == kSeedClosed) cst = sd & kCutVal;
                                else if ((sd >> 62) == kSeedOpen) cst = kNoCut;
                            }
                            if (back == 0 && cut == cst) {
                                mu = uk;
                                at = -1;
                            } else {
                                at = find_cut_lane(piece_cuts + Uk.out_base,
                                                   pstatus[uk] & 0xFFFFFFFFu, cut);
                                if (at >= 0) mu = uk;
                            }
                        }
                        stop = mu != kNoUnit;
                    }
                }
                const uint64_t hit = __builtin_amdgcn_ballot_w64(stop);
                const uint32_t first = hit ? (uint32_t)__builtin_ctzll(hit) : m - 1;
                if (lane <= first && n + lane < prm.fix_cap) out[n + lane] = cut;
                if (lane == first) {
                    s_bc[0] = cut;
                    s_bc[1] = first + 1;
                    s_bc[2] = mu;
                    s_bc[3] = (uint64_t)at;
                }
            }
            __syncthreads();
            c = uni64(s_bc[0]);
            n += uni64(s_bc[1]);
            const uint32_t mu_all = (uint32_t)uni64(s_bc[2]);
            const bool merged = mu_all != kNoUnit && c < d.n;
            if (merged) {
                munit = mu_all;
                midx = (int32_t)(int64_t)uni64(s_bc[3]);
            }
            __syncthreads();
            if (merged) break;
        }
        if (threadIdx.x == 0) {
            atomicAdd(&prm.stats[kWalkStatFixRounds], (unsigned long long)W.rounds);
            atomicAdd(&prm.stats[kWalkStatFixZones], (unsigned long long)W.zones);
            atomicAdd(&prm.stats[kWalkStatFixCuts], (unsigned long long)n);
            FixRes F;
            F.count = (uint32_t)min(n, (uint64_t)prm.fix_cap + 1);
            F.merge_unit = munit;
            F.merge_idx = midx;
            F.pad = 0;
            fixres[u] = F;
        }
    }
}

// ---------------------------------------------------------------------------
// Assemble: one workgroup per walked stream (units[unit0 .. unit0 + npieces)).
// Node j >= 1 is the boundary at piece j's start; on the exact chain it adds
// its hops, its fixup cuts and the tail of the list it merged into, then the
// chain goes on at node next(j) = piece(merge unit) + 1 > j.  Nodes are taken
// kAsmB at a time: every thread prepares one node, thread 0 follows the chain
// through the block by runs of "simple" nodes (next = j + 1, the common case),
// and a block prefix sum places each on-chain node's segment.
// counts[stream] = ~0 flags a stream whose fixup overflowed (the host redoes
// it on the scan path).
// Round 5: the workgroup places the segments and leaves each on-chain node's
// output offset in its BoundRes (fix_from, dead after the fixups; kOffNone
// off the chain); rcdc_walk_scatter_kernel then writes every node's
// segment, a thread per node over the whole grid.  A long stream has
// thousands of nodes (C5: 3 200), and copying them one workgroup per stream
// made the chain outlast the walk beside it (assemble 74.5 us, r5c5prof).
constexpr int kAsmB = 1024;
constexpr uint64_t kOffNone = ~0ull;

__global__ __launch_bounds__(kAsmB) void rcdc_walk_assemble_kernel(
    const StreamDesc *__restrict__ sds, const WalkUnit *__restrict__ units,
    const uint32_t *__restrict__ stream_unit0, uint32_t nstreams, WalkParams prm,
    const uint64_t *__restrict__ piece_cuts, const uint64_t *__restrict__ pstatus,
    BoundRes *__restrict__ bres, uint64_t *__restrict__ cuts, uint64_t *__restrict__ counts,
    const FixRes *__restrict__ fixres) {
    constexpr int NW = kAsmB / 64;
    __shared__ uint64_t s_ns[NW];          // bitmap: node is not simple
    __shared__ uint32_t s_next[kAsmB];     // next node (stream piece index)
    __shared__ uint8_t s_term[kAsmB];      // node ends the chain
    __shared__ uint32_t s_rng[2 * kAsmB];  // on-chain ranges [lo, hi) of this block
    __shared__ uint64_t s_wsum[NW];
    __shared__ uint32_t s_st[4];           // cur, done, nranges
    if (blockIdx.x >= nstreams) return;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t u0 = stream_unit0[blockIdx.x];
    const WalkUnit U0 = units[u0];
    const StreamDesc d = sds[U0.stream];
    uint64_t *out = cuts + d.cut_base;
    const uint64_t cap = d.cut_cap;
    const uint32_t P = U0.npieces;
    auto list_n = [&](uint32_t uu) { return pstatus[uu] & 0xFFFFFFFFu; };

    const uint64_t n0 = list_n(u0);
    for (uint64_t i = tid; i < n0 && i < cap; i += kAsmB)
        out[i] = piece_cuts[U0.out_base + i] & kCutVal;
    // every node off the chain until placed (the thread that places node j
    // below, j = b + tid, is the one that clears it here)
    for (uint32_t j = 1 + tid; j < P; j += kAsmB) bres[u0 + j].fix_from = kOffNone;
    uint64_t nc = n0;
    bool bad = false;
    uint32_t cur = 1, done = P <= 1;
    for (uint32_t b = 1; !done && b < P; b += kAsmB) {
        if (cur >= b + kAsmB) continue;
        // ---- this thread's node
        const uint32_t j = b + tid;
        const bool valid = j < P;
        bool term = true, nbad = false;
        uint32_t nh = 0, fc = 0, mu = kNoUnit, nxt = P;
        uint64_t tail_lo = 0, tail_hi = 0;
        const uint32_t u = u0 + j;
        if (valid) {
            const uint32_t kind = bres[u].kind;
            if (kind != kBoundNone) {
                nh = min(bres[u].nhops, (uint32_t)kMaxHops);
                if (kind == kBoundMerged || kind == kBoundFixup) {
                    int32_t mi = bres[u].merge_idx;
                    mu = bres[u].merge_unit;
                    if (kind == kBoundFixup) {
                        const FixRes F = fixres[u];
                        mu = F.merge_unit;
                        mi = F.merge_idx;
                        if (F.count > prm.fix_cap) {
                            nbad = true;
                            mu = kNoUnit;
                        } else {
                            fc = F.count;
                        }
                    }
                    if (mu != kNoUnit) {
                        term = false;
                        tail_lo = (uint64_t)(mi + 1);
                        tail_hi = list_n(mu);
                        nxt = units[mu].piece + 1;
                    }
                }
            }
        }
        // hop entries: single cuts, or runs of min-sized chunks (kHopRun)
        uint64_t nhc = 0;
        if (valid) {
            uint64_t pv = 0;
            for (uint32_t i = 0; i < nh; i++) {
                const uint64_t e = bres[u].hops[i], v = e & kCutVal;
                nhc += (e >> 62) == kHopRun ? (v - pv) / prm.min_size : 1;
                pv = v;
            }
        }
        const uint64_t len = nbad ? 0 : nhc + fc + (tail_hi - tail_lo);
        s_next[tid] = nxt;
        s_term[tid] = term;
        const uint64_t ns = __builtin_amdgcn_ballot_w64(!(valid && !term && nxt == j + 1));
        if (lane == 0) s_ns[wave] = ns;
        __syncthreads();
        // ---- the chain through this block (thread 0)
        if (tid == 0) {
            uint32_t c = cur - b, nr = 0, dn = 0, cu = cur;
            while (true) {
                // first non-simple node f >= c
                uint32_t f = kAsmB;
                for (uint32_t w = c >> 6; w < (uint32_t)NW; w++) {
                    uint64_t m = s_ns[w];
                    if (w == (c >> 6)) m &= ~0ull << (c & 63u);
                    if (m) {
                        f = w * 64u + (uint32_t)__builtin_ctzll(m);
                        break;
                    }
                }
                if (f == (uint32_t)kAsmB) {  // runs through the block
                    s_rng[2 * nr] = c;
                    s_rng[2 * nr + 1] = kAsmB;
                    nr++;
                    cu = b + kAsmB;
                    break;
                }
                if (b + f >= P) {  // past the last piece
                    s_rng[2 * nr] = c;
                    s_rng[2 * nr + 1] = f;
                    nr++;
                    dn = 1;
                    break;
                }
                s_rng[2 * nr] = c;
                s_rng[2 * nr + 1] = f + 1;
                nr++;
                if (s_term[f] || s_next[f] >= P) {
                    dn = 1;
                    break;
                }
                cu = s_next[f];
                if (cu >= b + kAsmB) break;
                c = cu - b;
            }
            s_st[0] = cu;
            s_st[1] = dn;
            s_st[2] = nr;
        }
        __syncthreads();
        const uint32_t nr = __builtin_amdgcn_readfirstlane(s_st[2]);
        bool on = false;
        for (uint32_t r = 0; r < nr; r++)
            on |= tid >= s_rng[2 * r] && tid < s_rng[2 * r + 1];
        on = on && valid;
        bad |= on && nbad;
        // ---- block exclusive prefix sum of the on-chain segment lengths
        uint64_t v = on ? len : 0;
        for (uint32_t o = 1; o < 64; o <<= 1) {
            const uint64_t t = __shfl_up(v, o, 64);
            if (lane >= o) v += t;
        }
        if (lane == 63) s_wsum[wave] = v;
        __syncthreads();
        uint64_t base = 0, total = 0;
        for (uint32_t w = 0; w < (uint32_t)NW; w++) {
            const uint64_t t = s_wsum[w];
            if (w < wave) base += t;
            total += t;
        }
        if (on && !nbad) bres[u].fix_from = nc + base + v - len;  // (the scatter writes it)
        nc += total;
        cur = __builtin_amdgcn_readfirstlane(s_st[0]);
        done = __builtin_amdgcn_readfirstlane(s_st[1]);
        __syncthreads();
    }
    const bool any_bad = __syncthreads_or(bad);
    if (tid == 0) counts[U0.stream] = (any_bad || nc > cap) ? ~0ull : nc;
}

// A thread per node of every walked stream: an on-chain node's segment --
// its hops (single cuts, or runs of min-sized chunks), its fixup cuts and the
// tail of the list it merged into -- at the offset the assembly left in its
// BoundRes.
__global__ __launch_bounds__(256) void rcdc_walk_scatter_kernel(
    const StreamDesc *__restrict__ sds, const WalkUnit *__restrict__ units, WalkParams prm,
    const uint64_t *__restrict__ piece_cuts, const uint64_t *__restrict__ pstatus,
    const BoundRes *__restrict__ bres, const uint64_t *__restrict__ fix_cuts,
    const FixRes *__restrict__ fixres, uint64_t *__restrict__ cuts) {
    const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= prm.nunits) return;
    const WalkUnit U = units[u];
    if (U.piece == 0) return;
    const BoundRes &R = bres[u];
    uint64_t o = R.fix_from;
    if (o == kOffNone) return;
    const StreamDesc d = sds[U.stream];
    uint64_t *out = cuts + d.cut_base;
    const uint64_t cap = d.cut_cap;
    const uint32_t kind = R.kind;
    const uint32_t nh = kind != kBoundNone ? min(R.nhops, (uint32_t)kMaxHops) : 0u;
    uint32_t fc = 0, mu = kNoUnit;
    int32_t mi = 0;
    if (kind == kBoundMerged) {
        mu = R.merge_unit;
        mi = R.merge_idx;
    } else if (kind == kBoundFixup) {
        const FixRes F = fixres[u];
        if (F.count > prm.fix_cap) return;  // (flagged by the assembly)
        fc = F.count;
        mu = F.merge_unit;
        mi = F.merge_idx;
    }
    uint64_t pv = 0;
    for (uint32_t i = 0; i < nh; i++) {
        const uint64_t e = R.hops[i], v = e & kCutVal;
        if ((e >> 62) == kHopRun) {
            for (uint64_t x = pv + prm.min_size; x <= v && o < cap; x += prm.min_size, o++)
                out[o] = x;
        } else {
            if (o < cap) out[o] = v;
            o++;
        }
        pv = v;
    }
    const uint64_t *fsrc = fix_cuts + (uint64_t)u * prm.fix_cap;
    for (uint32_t i = 0; i < fc; i++, o++)
        if (o < cap) out[o] = fsrc[i];
    if ((kind == kBoundMerged || kind == kBoundFixup) && mu != kNoUnit) {
        const uint64_t *L = piece_cuts + units[mu].out_base;
        const uint64_t hi = pstatus[mu] & 0xFFFFFFFFu;
        for (uint64_t i = (uint64_t)(mi + 1); i < hi; i++, o++)
            if (o < cap) out[o] = L[i] & kCutVal;
    }
}

// ---------------------------------------------------------------------------
// Cost-ordered queue.  A piece's walk time is its hashed bytes: its length
// times the share of it that is not zero runs (those cost 64 B per chunk).
// One wave per piece samples 64 aligned 8-byte words spread over the piece
// and counts the non-zero ones (0..64); the key is length x that share in
// units of Lp / 48 (a full random piece of Lp: 48), and one workgroup
// counting-sorts the queue by it, descending (longest-processing-time first:
// the last pieces the waves take are the cheap ones; a stream's last piece,
// up to 1.5 Lp, goes early).  Only the schedule changes, never the cuts.
// With seeded starts (WalkParams.seed) the key's low bit puts a stream's
// even pieces before its odd ones of the same cost: an odd piece then mostly
// starts after its predecessor has finished and continues its chain.
constexpr int kCostKeys = 256;

__global__ __launch_bounds__(1024) void rcdc_walk_cost_kernel(
    const uint8_t *__restrict__ arena, const StreamDesc *__restrict__ sds,
    const WalkUnit *__restrict__ units, WalkParams prm, uint8_t *__restrict__ key) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wpb = blockDim.x / 64u;
    for (uint32_t q = blockIdx.x * wpb + (threadIdx.x >> 6); q < prm.nunits; q += gridDim.x * wpb) {
        const uint32_t u = prm.order_in[q];
        const WalkUnit U = units[u];
        const StreamDesc d = sds[U.stream];
        const uint64_t len = U.stop - U.start;
        const uint32_t ns = prm.cost_samples ? prm.cost_samples : 64u;
        const uint64_t a = (d.off + U.start + (len * lane) / ns) & ~7ull;
        const uint64_t w = lane < ns && a + 8 <= d.off + d.n
                               ? *reinterpret_cast<const uint64_t *>(arena + a) : 0;
        const uint32_t cls = (uint32_t)__builtin_popcountll(__ballot(w != 0)) * (64u / ns);
        const uint64_t quantum = max(prm.piece_bytes / 48, (uint64_t)1);
        // K classes by piece index: at equal cost, a stream's pieces 0, K,
        // 2K, ... go first, then 1, K + 1, ... (each then mostly starts
        // after its predecessor has finished and continues its chain)
        const uint32_t K = prm.seed ? max(prm.seed_classes, 1u) : 1u;
        const uint64_t cost = min(len * cls / 64 / quantum, (uint64_t)(kCostKeys / K - 1));
        const uint64_t cl = K - 1u - U.piece % K;
        if (lane == 0) key[q] = (uint8_t)(cost * K + cl);
    }
}

// One workgroup: counting sort of the queue by key, descending (LDS atomics
// per lane: 23 us for C3's 26 k pieces; a wave-aggregated form, one atomic
// per key and wave, was 10x slower -- the keys of a wave are mostly distinct).
__global__ __launch_bounds__(1024) void rcdc_walk_sort_kernel(WalkParams prm,
                                                              const uint8_t *__restrict__ key) {
    __shared__ uint32_t s_cnt[kCostKeys];
    for (uint32_t i = threadIdx.x; i < (uint32_t)kCostKeys; i += blockDim.x) s_cnt[i] = 0;
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < prm.nunits; q += blockDim.x) atomicAdd(&s_cnt[key[q]], 1u);
    __syncthreads();
    if (threadIdx.x == 0) {  // exclusive prefix, highest key first
        uint32_t acc = 0;
        for (int k = kCostKeys - 1; k >= 0; k--) {
            const uint32_t c = s_cnt[k];
            s_cnt[k] = acc;
            acc += c;
        }
    }
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < prm.nunits; q += blockDim.x)
        prm.order_out[atomicAdd(&s_cnt[key[q]], 1u)] = prm.order_in[q];
}

namespace rcdc {

// The queue's cost order of a run (reads only the arena and the units;
// writes order_out, which no chain kernel reads): a pipelined run enqueues it
// before waiting for the chain that last used its buffer set.
hipError_t launch_walk_order(const uint8_t *arena, const StreamDesc *sds, const WalkUnit *units,
                             const WalkParams &prm, hipStream_t stream) {
    if (prm.nunits == 0 || !prm.order_in || !prm.order_out) return hipSuccess;
    // the key bytes follow order_out in the same buffer (plan_build)
    uint8_t *key = reinterpret_cast<uint8_t *>(prm.order_out + prm.nunits);
    // A run's order is computed right after the walk before the last on its
    // hashing stream ends: with thousands of workgroups the cost kernel took
    // every CU that walk freed and the next walk (other stream, ready) waited
    // ~100 us for it (profiles/r05/gaps_*.txt).  A few fat workgroups leave
    // the CUs to that walk and finish long before this run's walk is due.
    const bool fat = prm.cost_blocks <= 256;  // (> 256: round 4's grid, a wave per piece)
    const uint32_t per = fat ? 16u : 4u;        // waves per workgroup
    const uint32_t cb = std::max<uint32_t>(
        std::min<uint32_t>((prm.nunits + per - 1) / per, prm.cost_blocks), 1);
    hipLaunchKernelGGL(rcdc_walk_cost_kernel, dim3(cb), dim3(64 * per), 0, stream, arena, sds,
                       units, prm, key);
    hipLaunchKernelGGL(rcdc_walk_sort_kernel, dim3(1), dim3(1024), 0, stream, prm,
                       (const uint8_t *)key);
    return hipGetLastError();
}

// The hashing part: counters reset, the queue's cost order (unless already
// enqueued: `ordered`), the walk kernel.
hipError_t launch_walk(const uint8_t *arena, const StreamDesc *sds, const WalkUnit *units,
                       const WalkParams &prm, const uint64_t *gtab, uint64_t *piece_cuts,
                       uint64_t *pstatus, uint32_t *ctr, uint32_t blocks, hipStream_t stream,
                       bool ordered) {
    if (prm.nunits == 0) return hipSuccess;
    hipError_t e = hipSuccess;
    if (!(prm.flags & kWalkKReset)) {  // (A/B: resets on the walk's queue, queue from 0)
        e = hipMemsetAsync(ctr, 0, 4 * sizeof(uint32_t), stream);
        if (e == hipSuccess)
            e = hipMemsetAsync(prm.stats, 0, kWalkStats * sizeof(unsigned long long), stream);
        if (e != hipSuccess) return e;
    }
    if (!ordered) {
        e = launch_walk_order(arena, sds, units, prm, stream);
        if (e != hipSuccess) return e;
    }
    const bool small = prm.mask < 0xFFFFu;
#define RCDC_WALK_LAUNCH(TSH, SM)                                                                  \
    hipLaunchKernelGGL((rcdc_walk_kernel<TSH, SM>), dim3(blocks), dim3(1024), 0, stream, arena,   \
                       sds, units, prm, gtab, piece_cuts, pstatus, ctr)
    if (prm.idx_shift == 21 && !small) RCDC_WALK_LAUNCH(105, false);
    else if (small) RCDC_WALK_LAUNCH(-1, true);
    else RCDC_WALK_LAUNCH(-1, false);
#undef RCDC_WALK_LAUNCH
    return hipGetLastError();
}

// The chain part: boundary checks, fixups, assembly into cuts / counts.
hipError_t launch_walk_chain(const uint8_t *arena, const StreamDesc *sds, const WalkUnit *units,
                             const uint32_t *stream_unit0, uint32_t nstreams,
                             const WalkParams &prm, const uint64_t *gtab,
                             const uint64_t *piece_cuts, const uint64_t *pstatus, BoundRes *bres,
                             uint32_t *ctr, uint32_t *fixlist, uint64_t *fix_cuts,
                             FixRes *fixres, uint64_t *cuts, uint64_t *counts,
                             uint32_t fix_blocks, uint32_t chk_cap, hipStream_t stream,
                             bool wide) {
    if (prm.nunits == 0) return hipSuccess;
    static const bool dbg = getenv("RCDC_DEBUG_SYNC") != nullptr;
    const bool small = prm.mask < 0xFFFFu;
    const uint32_t chk_blocks =
        std::max<uint32_t>(std::min<uint32_t>(std::min(fix_blocks, chk_cap), (prm.nunits + 7) / 8), 1);
#define RCDC_CHK_LAUNCH(TSH, SM, CT)                                                               \
    hipLaunchKernelGGL((rcdc_walk_check_kernel<TSH, SM, CT>), dim3(chk_blocks), dim3(CT), 0,      \
                       stream,                                                                     \
                       arena, sds, units, prm, gtab, piece_cuts, pstatus, bres, ctr, fixlist)
    // (the wide form only for the default degree: pipelined C3 / C4 plans)
    if (prm.idx_shift == 21 && !small && wide) RCDC_CHK_LAUNCH(105, false, 1024);
    else if (prm.idx_shift == 21 && !small) RCDC_CHK_LAUNCH(105, false, 512);
    else if (small) RCDC_CHK_LAUNCH(-1, true, 512);
    else RCDC_CHK_LAUNCH(-1, false, 512);
#undef RCDC_CHK_LAUNCH
    if (dbg) {
        (void)hipStreamSynchronize(stream);
        uint32_t h[4];
        (void)hipMemcpy(h, ctr, 16, hipMemcpyDeviceToHost);
        fprintf(stderr, "rcdc: check done, %u fixups\n", h[1]);
    }
#define RCDC_FIX_LAUNCH(TSH, SM)                                                                   \
    hipLaunchKernelGGL((rcdc_walk_fixup_kernel<TSH, SM>), dim3(fix_blocks), dim3(1024), 0, stream, \
                       arena, sds, units, prm, gtab, piece_cuts, pstatus, bres, ctr, fixlist,      \
                       fix_cuts, fixres)
    if (prm.idx_shift == 21 && !small) RCDC_FIX_LAUNCH(105, false);
    else if (small) RCDC_FIX_LAUNCH(-1, true);
    else RCDC_FIX_LAUNCH(-1, false);
#undef RCDC_FIX_LAUNCH
    if (dbg) {
        (void)hipStreamSynchronize(stream);
        fprintf(stderr, "rcdc: fixup done\n");
    }
    hipLaunchKernelGGL(rcdc_walk_assemble_kernel, dim3(nstreams), dim3(kAsmB), 0, stream, sds, units,
                       stream_unit0, nstreams, prm, piece_cuts, pstatus, bres, cuts, counts,
                       fixres);
    hipLaunchKernelGGL(rcdc_walk_scatter_kernel, dim3((prm.nunits + 255) / 256), dim3(256), 0, stream,
                       sds, units, prm, piece_cuts, pstatus, bres, fix_cuts, fixres, cuts);
    return hipGetLastError();
}

}  // namespace rcdc
