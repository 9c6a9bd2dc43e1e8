// rcdc_runtime.cpp -- host runtime behind include/rcdc.h.
//
// Owns the device (tables, work lists, summaries, cut lists, pinned staging)
// and maps the reference's chunker surface onto the two kernels:
//   rcdc_check_params  <- crates/core/src/chunker/rabin.rs:17-42
//   rcdc_parse_poly    <- crates/core/src/repofile/configfile.rs:165-175
//   rcdc_ctx_create    <- crates/core/src/chunker.rs:29-38 (Rabin64 tables once)
//   rcdc_chunk_batch   <- per-file parallel ChunkIter (archiver.rs:195)
//   rcdc_stream_*      <- one ChunkIter over a Read (rabin.rs:110-191)
//   rcdc_plan_*        <- device-resident batches (the measured path)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cerrno>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "../../include/rcdc.h"
#include "rcdc_internal.h"

namespace rcdc {
int scan_threads(int code);
hipError_t launch_scan(int code, const uint8_t *arena, const ScanItem *items, uint32_t nitems,
                       const uint64_t *gtab, const ScanParams &prm, uint4 *sums,
                       uint64_t *item_masks, uint32_t blocks, hipStream_t stream);
hipError_t launch_resolve(const uint8_t *arena, const StreamDesc *sds, const ResolveUnit *units,
                          uint32_t nunits, const StitchDesc *stitches, uint32_t nstitch,
                          const uint64_t *gtab, const ResolveParams &prm, const uint4 *sums,
                          const uint64_t *item_masks, uint64_t *cuts, uint64_t *counts,
                          uint64_t *piece_cuts, uint64_t *piece_counts, uint64_t *stats,
                          hipStream_t stream);
hipError_t launch_window(const uint64_t *cuts, const uint64_t *counts, uint32_t stream,
                         uint64_t base, uint64_t bound, uint32_t k, uint64_t *out,
                         hipStream_t hs);
bool host_sha_supported();
void host_sha256_many(const uint8_t *const *ptrs, const uint64_t *lens, uint32_t n,
                      uint8_t *digests);
hipError_t launch_walk(const uint8_t *arena, const StreamDesc *sds, const WalkUnit *units,
                       const WalkParams &prm, const uint64_t *gtab, uint64_t *piece_cuts,
                       uint64_t *pstatus, uint32_t *ctr, uint32_t blocks, hipStream_t stream,
                       bool ordered);
hipError_t launch_walk_order(const uint8_t *arena, const StreamDesc *sds, const WalkUnit *units,
                             const WalkParams &prm, hipStream_t stream);
hipError_t launch_walk_chain(const uint8_t *arena, const StreamDesc *sds, const WalkUnit *units,
                             const uint32_t *stream_unit0, uint32_t nstreams,
                             const WalkParams &prm, const uint64_t *gtab,
                             const uint64_t *piece_cuts, const uint64_t *pstatus, BoundRes *bres,
                             uint32_t *ctr, uint32_t *fixlist, uint64_t *fix_cuts,
                             FixRes *fixres, uint64_t *cuts, uint64_t *counts,
                             uint32_t fix_blocks, uint32_t chk_cap, hipStream_t stream,
                             bool wide);
hipError_t launch_sha256_list(const uint8_t *arena, const ulonglong2 *refs, uint32_t n,
                              uint32_t *digests, hipStream_t stream);
hipError_t launch_sha256_plan(const uint8_t *arena, const StreamDesc *sds, uint32_t nstreams,
                              const uint64_t *cuts, const uint64_t *counts, uint64_t nslots,
                              uint64_t max_len, uint32_t *bwork, uint32_t *order,
                              uint32_t *digests, hipStream_t stream);
hipError_t launch_sha256_multi(uint32_t n, const uint8_t *const *arenas,
                               const StreamDesc *const *sds, const uint32_t *nstreams,
                               const uint64_t *const *cuts, const uint64_t *const *counts,
                               const uint64_t *nslots, uint64_t max_len, uint32_t *const *bwork,
                               uint32_t *const *order, uint32_t *const *digests,
                               hipStream_t stream);
hipError_t launch_aead(bool open, const uint8_t *in, uint8_t *out, const AeadBlob *blobs,
                       uint32_t nblobs, const AeadUnit *units, uint32_t nunits,
                       const uint32_t *unit0, const AeadKeyDev *key, uint32_t *partials,
                       uint32_t *status, uint32_t cus, hipStream_t stream);
uint32_t zstd_block_grid(uint32_t cus, int level);
uint64_t zstd_far_words(int level, uint64_t nblk);
void zstd_prof_dump();
void zstd_check_prof_dump();
hipError_t launch_zstd(const uint8_t *in, uint8_t *out, const ZstdBlob *blobs, uint32_t nblobs,
                       const ZstdBlk *blks, uint32_t nblk, const ZstdTables *tabs, uint8_t *slots,
                       uint64_t *seqbuf, uint32_t grid, uint2 *res, uint64_t *bpos,
                       uint64_t *out_lens, uint32_t *queue, uint32_t *far, int level,
                       hipStream_t stream);
uint64_t zstd_check_scratch_bytes(uint32_t grid);
uint64_t zstd_blkdesc_bytes();
uint32_t zstd_check_waves_per_cu();
hipError_t launch_zstd_check_blocks(const uint8_t *frames, const uint8_t *data, const void *refs,
                                    const uint64_t *blk0, uint32_t n, void *blks, uint64_t nblk,
                                    uint8_t *scratch, uint32_t grid, uint32_t *status,
                                    uint32_t *ctr, hipStream_t stream);
hipError_t launch_plan_set_len(StreamDesc *sds, ScanItem *items, uint32_t nitems, uint64_t n,
                               uint64_t nseg, hipStream_t stream);
hipError_t launch_copy_ranges(uint8_t *out, const void *units, uint32_t n, uint32_t cus,
                              hipStream_t stream);
hipError_t launch_zstd_check(const uint8_t *frames, const uint8_t *data, const void *refs,
                             const uint32_t *order, uint32_t n, bool stored, uint8_t *scratch,
                             uint32_t grid,
                             uint32_t *status, uint32_t *ctr, hipStream_t stream);
}  // namespace rcdc

using namespace rcdc;

// ---------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------
namespace {
thread_local std::string g_err;

rcdc_status fail(rcdc_status st, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return st;
}

#define HIP_TRY(expr)                                                                   \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess)                                                           \
            return fail(RCDC_ERR_INTERNAL, "%s failed: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

// ---------------------------------------------------------------------------
// GF(2) polynomial arithmetic for the Rabin64 tables (rustic_cdc Polynom64)
// ---------------------------------------------------------------------------
int poly_degree(uint64_t p) { return p ? 63 - __builtin_clzll(p) : -1; }

uint64_t poly_mod(uint64_t p, uint64_t m) {
    const int dm = poly_degree(m);
    while (p) {
        const int dp = poly_degree(p);
        if (dp < dm) break;
        p ^= m << (dp - dm);
    }
    return p;
}

// Device table image: [0,256) out[b] << 8, [256,512) mod[i]
// out[b] = b * x^(8*63) mod P;  mod[i] = ((i << deg) mod P) | (i << deg).
void build_tables(uint64_t poly, uint64_t *img) {
    const int deg = poly_degree(poly);
    for (uint64_t b = 0; b < 256; b++) {
        uint64_t h = poly_mod(b, poly);
        for (int i = 0; i < kWindow - 1; i++) h = poly_mod(h << 8, poly);
        img[b] = h << 8;
        const uint64_t p = b << deg;
        img[256 + b] = poly_mod(p, poly) | p;
    }
}

uint64_t round_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }
}  // namespace

// ---------------------------------------------------------------------------
// context / plan objects
// ---------------------------------------------------------------------------
struct rcdc_plan {
    rcdc_ctx *ctx = nullptr;
    uint32_t n = 0;
    uint64_t arena_len = 0;
    uint32_t seg_bytes = 0;
    uint32_t blocks = 0;
    uint64_t nseg = 0, ncuts = 0, scanned = 0;
    // capacity plans (single-stream host passes): the scan runs the first
    // run_items items (0: all) on run_blocks workgroups; set by plan_set_len
    uint32_t run_items = 0, run_blocks = 0;
    std::vector<ScanItem> items;
    std::vector<StreamDesc> sds;
    std::vector<uint64_t> cut_base;
    std::vector<ResolveUnit> units;
    std::vector<StitchDesc> stitches;
    uint64_t npiece_cuts = 0;
    // device
    ScanItem *d_items = nullptr;
    StreamDesc *d_sds = nullptr;
    ResolveUnit *d_units = nullptr;
    StitchDesc *d_stitches = nullptr;
    uint64_t *d_piece_cuts = nullptr;
    uint64_t *d_piece_counts = nullptr;
    uint64_t cap_units = 0, cap_stitches = 0, cap_piece_cuts = 0, cap_piece_counts = 0;
    uint4 *d_sums = nullptr;
    uint64_t *d_masks = nullptr;
    uint64_t *d_cuts = nullptr;
    uint64_t *d_counts = nullptr;
    uint64_t cap_items = 0, cap_sds = 0, cap_sums = 0, cap_cuts = 0, cap_masks = 0,
             cap_counts = 0;
    // walk path (long streams, rcdc_walk.hip)
    bool no_walk = false;             // force the scan path (fallback re-runs)
    bool no_pieces = false;           // one resolve unit per stream (capacity plans)
    std::vector<WalkUnit> wunits;
    std::vector<uint32_t> wstream_u0;  // unit0 of every walked stream
    std::vector<uint32_t> worder;      // walk queue order (big pieces first)
    uint32_t nsmall_units = 0;         // the split pieces at worder's end
    bool walk_many = false;            // pieces outnumber 2x the wave slots
    uint64_t walk_small = 0;           // Ls of the split pieces
    std::vector<uint8_t> walked;       // per stream: on the walk path
    uint64_t nwpiece_cuts = 0;
    WalkParams wprm{};
    WalkUnit *d_wunits = nullptr;
    uint32_t *d_wsu0 = nullptr;
    uint32_t *d_worder = nullptr;
    uint64_t *d_wpiece = nullptr;
    uint64_t *d_pstatus = nullptr;
    uint64_t *d_wstate = nullptr, *d_wstate2 = nullptr;  // WalkParams.wstate of set 0 / 1
    uint64_t cap_wstate = 0, cap_wstate2 = 0;
    uint64_t walk_epoch = 0;  // runs of the walk kernel (WalkParams.epoch)
    uint32_t wqbase[2] = {0, 0};  // walk queue counter at the next run of set 0 / 1 (WalkParams.qbase)
    BoundRes *d_bres = nullptr;
    uint32_t *d_ctr = nullptr;
    uint32_t *d_fixlist = nullptr;
    uint64_t *d_fixcuts = nullptr;
    FixRes *d_fixres = nullptr;
    unsigned long long *d_wstats = nullptr;  // kWalkStats work counters of the last run
    unsigned long long *d_wtrace = nullptr;  // per-unit trace (RCDC_WALK_TRACE=1)
    uint64_t cap_wstats = 0, cap_wtrace = 0;
    uint64_t cap_worder = 0;
    uint64_t cap_wunits = 0, cap_wsu0 = 0, cap_wpiece = 0, cap_pstatus = 0, cap_bres = 0,
             cap_ctr = 0, cap_fixlist = 0, cap_fixcuts = 0, cap_fixres = 0;
    const void *last_arena = nullptr;  // of the last run (fallback re-runs)
    hipStream_t last_stream = nullptr;
    hipEvent_t done = nullptr;
    bool ran = false;
    // pipelined runs (rcdc_plan_set_pipeline): run k's hashing kernels (scan,
    // walk) go to hashing stream k % 2, its chain kernels (resolve, check,
    // fixup, assemble) to the chain stream.  Hashing k + 1 thus overlaps
    // chain k, and the next walk fills the tail of the previous one.  Every
    // per-run buffer the chain reads ping-pongs between two sets.
    bool pipelined = false;
    // boundary-check workgroups of a pipelined run: the check is latency
    // bound and each workgroup holds a whole CU (128 KiB of LDS tables), so
    // overlapped with the next walk it runs on few CUs (RCDC_CHK_BLOCKS)
    uint32_t chk_blocks_pipe = 64;
    uint32_t fix_blocks_pipe = 64;  // chain workgroups beside the next walk (RCDC_CHAIN_BLOCKS;
                                    // 64 vs 32: C3 -0.7 %, C4 +1.5 %, profiles/r04/chain_blocks.txt)
    bool flush_next = false;          // the next pipelined run is the last: its chain runs on
                                      // every CU (rcdc_plan_set_pipeline(plan, 2))
    uint32_t pp = 0;                  // buffer set of the next run
    uint32_t last_set = 0;            // buffer set of the last run
    uint64_t wruns = 0;               // walk runs (the work-counter slot: wruns % 4)
    uint32_t last_wslot = 0;          // the last run's work-counter slot
    uint4 *d_sums2 = nullptr;
    uint64_t *d_masks2 = nullptr;
    uint64_t cap_sums2 = 0, cap_masks2 = 0;
    hipStream_t rstream = nullptr;
    hipStream_t hstream[2] = {nullptr, nullptr};
    hipEvent_t ev_in[2] = {nullptr, nullptr};
    hipEvent_t ev_scan[2] = {nullptr, nullptr};
    hipEvent_t ev_res[2] = {nullptr, nullptr};
    bool res_pending[2] = {false, false};
    // walk buffer set 1 (set 0 is the d_w* fields above)
    uint64_t *d_wpiece2 = nullptr, *d_pstatus2 = nullptr, *d_fixcuts2 = nullptr;
    BoundRes *d_bres2 = nullptr;
    uint32_t *d_ctr2 = nullptr, *d_fixlist2 = nullptr, *d_worder2 = nullptr;
    FixRes *d_fixres2 = nullptr;
    unsigned long long *d_wstats2 = nullptr;
    uint64_t cap_wpiece2 = 0, cap_pstatus2 = 0, cap_fixcuts2 = 0, cap_bres2 = 0, cap_ctr2 = 0,
             cap_fixlist2 = 0, cap_worder2 = 0, cap_fixres2 = 0, cap_wstats2 = 0;
    // SHA-256 of every chunk (rcdc_plan_hash), slot-indexed like d_cuts
    uint32_t *d_dig = nullptr;
    uint64_t cap_dig = 0;
    uint32_t *d_shaw = nullptr;   // length-bucket counters + total
    uint32_t *d_order = nullptr;  // slots sorted by chunk length, longest first
    uint64_t cap_shaw = 0, cap_order = 0;
    bool hashed = false;
    bool finished = false;           // rcdc_plan_finish done for the last run
    std::vector<uint64_t> fin_counts;  // per-stream counts after the finish
    // optional per-run kernel timing
    bool timing = false;
    uint32_t tperiod = 1;         // record every tperiod-th run (rcdc_plan_set_timing)
    uint64_t tcalls = 0;          // runs since timing was enabled
    std::vector<hipEvent_t> tev;  // 3 per timed run: before scan, after scan, after resolve
    uint64_t truns = 0;
};

// One host-buffer worker of a context ("lane"): a HIP stream of its own, two
// pinned staging slots (the caller's pageable bytes are copied into one while
// the other's DMA runs), a device arena and a cached plan.  Calling threads
// take a free lane for the duration of a call, so concurrent files
// (archiver.rs:195) run on separate streams without a context-wide lock.
struct Lane {
    hipStream_t stream = nullptr;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    uint8_t *pinned[4] = {nullptr, nullptr, nullptr, nullptr};
    uint32_t nslots = 2;
    uint64_t stage = 0;  // bytes per staging slot
    uint8_t *d_arena = nullptr;
    uint64_t arena_cap = 0;
    rcdc_plan *plan = nullptr;
    std::vector<uint64_t> lay_offs, lay_lens;  // layout of the cached plan
    uint64_t lay_arena = 0;
    bool lay_cap = false;  // a capacity plan (one stream, length set per pass)
};

struct rcdc_ctx {
    int device = 0;
    uint64_t poly = 0, min = 0, avg = 0, max = 0;
    int deg = 0;
    int num_cus = 0;
    int variant = kDefaultScanCode;  // scan-kernel configuration (RCDC_SCAN_VARIANT)
    hipStream_t stream = nullptr;
    uint64_t *d_tables = nullptr;
    // host-buffer path: a pool of lanes (RCDC_LANES, default 16)
    std::mutex pool_mu;
    std::condition_variable pool_cv;
    std::vector<Lane *> lanes, free_lanes;
    uint32_t max_lanes = 16;
    // blob encryption (rcdc_aead_*): calls on one context take turns
    std::mutex aead_mu;
    uint8_t aead_key[64] = {0};
    bool aead_key_set = false;
    AeadKeyDev *d_aead_key = nullptr;
    AeadBlob *d_aead_blobs = nullptr;
    AeadUnit *d_aead_units = nullptr;
    uint32_t *d_aead_unit0 = nullptr, *d_aead_partials = nullptr, *d_aead_status = nullptr;
    uint8_t *d_aead_stage = nullptr;  // pack headers
    uint8_t *h_aead_up = nullptr;     // page-locked source of a call's uploads
    uint64_t cap_aead_up = 0;
    uint64_t cap_aead_key = 0, cap_aead_blobs = 0, cap_aead_units = 0, cap_aead_unit0 = 0,
             cap_aead_partials = 0, cap_aead_status = 0, cap_aead_stage = 0;
    hipEvent_t aead_done = nullptr;
    // ordering of calls on the context's stream (hip_stream == 0) with the
    // legacy default stream (null_enter / null_leave)
    hipEvent_t ev_null_in = nullptr, ev_null_out = nullptr;
    // device tails of open streams (max + 256 bytes each): a pool, so opening
    // and closing streams never calls hipMalloc / hipFree (which synchronise
    // the device) once warm
    std::mutex tail_mu;
    std::vector<uint8_t *> tail_pool, tail_all;
    // blob compression (rcdc_zstd_compress): calls on one context take turns
    std::mutex zstd_mu;
    ZstdTables *d_zstd_tabs = nullptr;
    ZstdBlob *d_zstd_blobs = nullptr;
    ZstdBlk *d_zstd_blks = nullptr;
    uint2 *d_zstd_res = nullptr;
    uint64_t *d_zstd_bpos = nullptr, *d_zstd_lens = nullptr, *d_zstd_seq = nullptr;
    uint32_t *d_zstd_queue = nullptr;  // per window: blocks taken past the first grid
    uint64_t cap_zstd_queue = 0;
    uint8_t *d_zstd_slots = nullptr;
    uint32_t *d_zstd_far = nullptr;  // far candidates: tables + maps per block (levels >= 3)
    uint64_t cap_zstd_far = 0;
    uint64_t cap_zstd_tabs = 0, cap_zstd_blobs = 0, cap_zstd_blks = 0, cap_zstd_res = 0,
             cap_zstd_bpos = 0, cap_zstd_lens = 0, cap_zstd_seq = 0, cap_zstd_slots = 0;
    // frame checks (rcdc_zstd_check): calls on one context take turns
    std::mutex zck_mu;
    uint64_t *d_zck_refs = nullptr;
    uint32_t *d_zck_order = nullptr, *d_zck_status = nullptr;
    uint8_t *d_zck_scratch = nullptr;
    uint64_t cap_zck_refs = 0, cap_zck_order = 0, cap_zck_status = 0, cap_zck_scratch = 0;
    uint64_t *d_zck_blk0 = nullptr;  // block-parallel pass: per-frame block slots
    uint8_t *d_zck_blks = nullptr;
    uint64_t cap_zck_blk0 = 0, cap_zck_blks = 0;
    // pack files from sealed blobs (rcdc_pack_build_raw): copy units
    uint64_t *d_copy_units = nullptr;
    uint64_t cap_copy_units = 0;
};

struct rcdc_stream {
    rcdc_ctx *ctx = nullptr;
    std::vector<uint8_t> pending;  // bytes from the current chunk start
    uint64_t base = 0;             // absolute offset of pending[0]
    uint64_t batch = 0;            // bytes buffered before a device pass
    bool done = false;
    std::deque<uint64_t> out;      // final cuts not yet handed to the caller
    // the same pending bytes, kept on the device after a pass, so the next
    // pass sends only the new bytes over PCIe (tail_len == pending.size()
    // when valid, 0 otherwise)
    uint8_t *d_tail = nullptr;  // from the context's pool, ctx->max + 256 bytes
    uint64_t tail_len = 0;
    hipEvent_t tail_ev = nullptr;  // the copy into d_tail (on the last pass's lane stream)
};

namespace {

struct DeviceGuard {
    int prev = 0;
    explicit DeviceGuard(int dev) {
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(dev);
    }
    ~DeviceGuard() { (void)hipSetDevice(prev); }
};

// hip_stream == 0 selects the context's own stream.  That stream is created
// non-blocking, so on its own it is not ordered with the legacy default
// stream (torch's default stream is that stream).  A call given 0 is ordered
// as if it ran there: after the work queued on the default stream before
// the call (null_enter) and before the work queued there after it
// (null_leave).
rcdc_status null_enter(rcdc_ctx *ctx, const void *hip_stream, hipStream_t *st) {
    if (hip_stream) {
        *st = (hipStream_t)hip_stream;
        return RCDC_OK;
    }
    *st = ctx->stream;
    HIP_TRY(hipEventRecord(ctx->ev_null_in, nullptr));
    HIP_TRY(hipStreamWaitEvent(ctx->stream, ctx->ev_null_in, 0));
    return RCDC_OK;
}

rcdc_status null_leave(rcdc_ctx *ctx, const void *hip_stream, hipStream_t st) {
    if (hip_stream) return RCDC_OK;
    HIP_TRY(hipEventRecord(ctx->ev_null_out, st));
    HIP_TRY(hipStreamWaitEvent(nullptr, ctx->ev_null_out, 0));
    return RCDC_OK;
}

// Waits of the library's own calls poll (hipEventQuery + a 50 us sleep)
// instead of blocking in HIP: a thread blocked in hipStreamSynchronize /
// hipEventSynchronize held up other threads' launches and copies (the
// ingest engine's threads, r5r).  RCDC_POLL=0: blocking calls.
static bool poll_mode() {
    static const bool p = !(getenv("RCDC_POLL") && atoi(getenv("RCDC_POLL")) == 0);
    return p;
}

hipError_t poll_event(hipEvent_t ev) {
    if (!poll_mode()) return hipEventSynchronize(ev);
    for (;;) {
        const hipError_t e = hipEventQuery(ev);
        if (e != hipErrorNotReady) return e;
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

// One polling event per device and thread: an event can only be recorded on
// a stream of the device it was created on, and a thread may serve contexts
// on several GPUs.  The events are destroyed when the thread exits.
struct PollEvents {
    static constexpr int kMaxDev = 64;
    hipEvent_t ev[kMaxDev] = {};
    ~PollEvents() {
        for (int d = 0; d < kMaxDev; d++)
            if (ev[d] && hipSetDevice(d) == hipSuccess) (void)hipEventDestroy(ev[d]);
    }
};

hipError_t poll_stream(hipStream_t st) {
    if (!poll_mode()) return hipStreamSynchronize(st);
    thread_local PollEvents pe;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);  // the caller's DeviceGuard: the stream's device
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= PollEvents::kMaxDev) return hipStreamSynchronize(st);
    hipEvent_t &ev = pe.ev[dev];
    if (!ev && (e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) {
        ev = nullptr;
        return e;
    }
    if ((e = hipEventRecord(ev, st)) != hipSuccess) return e;
    return poll_event(ev);
}

// Device buffer of at least `need` elements.  Grows with 25 % headroom: a
// reallocation's hipFree synchronises the whole device (every lane of every
// thread), so slowly varying sizes (stream passes of batch + tail bytes)
// must not reallocate each time.
template <typename T>
rcdc_status ensure_dev(T **p, uint64_t *cap, uint64_t need) {
    if (need <= *cap && *p) return RCDC_OK;
    static const bool log = getenv("RCDC_ALLOC_LOG") != nullptr;
    if (log && *p)
        fprintf(stderr, "rcdc: regrow %llu -> %llu x %zu B (hipFree: device sync)\n",
                (unsigned long long)*cap, (unsigned long long)need, sizeof(T));
    if (*p) HIP_TRY(hipFree(*p));
    *p = nullptr;
    *cap = 0;
    // at least 64 KiB: small per-stream arrays (walk streams, piece cuts)
    // otherwise regrew from 1-2 elements when a layout first had more of
    // them, each regrow a device-wide sync inside a pipeline (r5u)
    const uint64_t n = std::max<uint64_t>(need + need / 4, std::max<uint64_t>(65536 / sizeof(T), 1));
    HIP_TRY(hipMalloc((void **)p, n * sizeof(T)));
    *cap = n;
    return RCDC_OK;
}

// Choose the per-lane segment S (multiple of 128 in [512, 4096]): the scan
// runs ceil(items / wave_slots) rounds of S + 64 slides per lane (64 = the
// warm-up window), items = sum over streams of ceil(ceil(span / S) / 64).
// Minimise rounds * (S + 64); ties go to the smaller S (finer summaries).
uint32_t choose_segment(const std::vector<uint64_t> &spans, int cus, int chains, int threads) {
    const uint64_t slots = (uint64_t)std::max(cus, 1) * (threads / 64) * chains;
    uint64_t best_cost = ~0ull;
    uint32_t best = 2048;
    for (uint32_t S = 512; S <= 4096; S += 128) {
        uint64_t items = 0;
        for (uint64_t sp : spans) items += ((sp + S - 1) / S + 63) / 64;
        const uint64_t rounds = std::max<uint64_t>((items + slots - 1) / slots, 1);
        const uint64_t cost = rounds * (S + kWindow);
        if (cost < best_cost) {
            best_cost = cost;
            best = S;
        }
    }
    return best;
}

// Arena offset of lane 0's first byte for a stream at `off`: aligned to
// `align` (a power of two, 16..128) unless that would start before the
// stream's first byte - 64, then 16-aligned.  64 (default) puts every 64-B
// register unit of every lane in one cache-line half: the unaligned layout
// fetched each line twice (profiles/r01_pmc_hbm.txt).  128 adds up to 63
// bytes per stream, which on 1 MiB streams costs an extra segment.
static inline uint64_t stream_q0(uint64_t off, uint64_t pos_lo, uint64_t align) {
    const uint64_t x = off + pos_lo - 65;
    const uint64_t q = x & ~(align - 1);
    return q + 64 >= off ? q : (x & ~(uint64_t)15);
}

static uint64_t q0_align() {
    const char *e = getenv("RCDC_Q0_ALIGN");  // experiments: 16, 32, 64, 128
    const uint64_t v = e ? (uint64_t)atoll(e) : 64;
    return (v == 128 || v == 64 || v == 32 || v == 16) ? v : (uint64_t)64;
}

// Resolver work list.  A stream of N >= kPieceStreams * min bytes is cut into
// pieces of Lp bytes (a multiple of min, >= 16 min), resolved speculatively in
// parallel and stitched (rcdc_resolve.hip).  Lp ~ sqrt(N * min / 2) balances
// the hops of one piece (Lp / chunk) against the stitch's per-piece step.
constexpr uint64_t kPieceStreams = 64;  // in units of min

static uint64_t piece_bytes(uint64_t N, uint64_t mn) {
    if (const char *e = getenv("RCDC_PIECE_BYTES")) {  // experiments; 0 disables
        const uint64_t v = (uint64_t)atoll(e);
        return v ? std::max<uint64_t>(v / mn, 1) * mn : 0;
    }
    if (N < kPieceStreams * mn) return 0;
    const double lp = std::sqrt((double)N * (double)mn / 2.0);
    return std::max<uint64_t>((uint64_t)(lp / (double)mn), 16) * mn;
}

void build_resolve_units(rcdc_plan *pl, uint64_t mn) {
    pl->units.clear();
    pl->stitches.clear();
    pl->npiece_cuts = 0;
    for (uint32_t i = 0; i < pl->n; i++) {
        if (pl->walked[i]) continue;
        const StreamDesc &d = pl->sds[i];
        const uint64_t N = d.n;
        const uint64_t Lp = pl->no_pieces ? 0 : piece_bytes(N, mn);
        if (Lp == 0 || N <= 2 * Lp) {
            ResolveUnit u{};
            u.start = 0;
            u.stop = N;
            u.out_base = d.cut_base;
            u.out_cap = (uint32_t)std::min<uint64_t>(d.cut_cap, 0xFFFFFFFFu);
            u.stream = i;
            u.direct = 1;
            pl->units.push_back(u);
            continue;
        }
        StitchDesc sd{};
        sd.stream = i;
        sd.unit0 = (uint32_t)pl->units.size();
        for (uint64_t a = 0; a < N; a += Lp) {
            ResolveUnit u{};
            u.start = a;
            u.stop = std::min(a + Lp, N);
            u.out_base = pl->npiece_cuts;
            // chunks >= min except the last: (stop - start) / min + the crossing cut
            u.out_cap = (uint32_t)((u.stop - u.start) / mn + 3);
            u.stream = i;
            u.direct = 0;
            pl->npiece_cuts += u.out_cap;
            pl->units.push_back(u);
        }
        sd.npieces = (uint32_t)pl->units.size() - sd.unit0;
        pl->stitches.push_back(sd);
    }
}

// Walk-path selection (rcdc_walk.hip).  The walk hashes what the reference
// hashes (~2/3 of random bytes, ~nothing of zero runs) but parallelises only
// over pieces of Lp bytes, so it needs many of them to fill the chip: a
// stream of N >= 2 Lp is walked when the plan's walkable bytes give at least
// kWalkMinPieces pieces.  Lp ~ walkable / (4 x 4096 wave slots), so the
// dynamic queue balances cheap (zero) and expensive (random) pieces, clamped
// to [4 MiB, 32 MiB] and a multiple of min.  RCDC_WALK_PIECE (bytes; 0 = scan
// path only) and RCDC_WALK_MIN_PIECES override.
constexpr uint64_t kWalkMinPieces = 1024;

static uint64_t walk_piece_bytes(const uint64_t *lens, uint32_t n, uint64_t mn, uint64_t mx) {
    uint64_t lp_env = ~0ull, min_pieces = kWalkMinPieces;
    if (const char *e = getenv("RCDC_WALK_PIECE")) lp_env = (uint64_t)atoll(e);
    if (const char *e = getenv("RCDC_WALK_MIN_PIECES")) min_pieces = (uint64_t)atoll(e);
    if (lp_env == 0) return 0;
    // Floor 4 MiB for files averaging >= 256 MiB, 3 MiB below (round-4 sweep
    // with seeded starts, profiles/r04/piece_sweep.txt: C4's 4-256 MiB files
    // +1.8 % at 3 MiB, C3's 1 GiB files -1.5 %).
    const uint64_t hi = 32ull << 20;
    uint64_t total = 0, nbig = 0;
    for (uint32_t i = 0; i < n; i++)
        if (lens[i] >= 6ull << 20) total += lens[i], nbig++;
    const uint64_t lo = nbig && total / nbig >= 256ull << 20 ? 4ull << 20 : 3ull << 20;
    uint64_t lp = lp_env != ~0ull ? lp_env : std::min(std::max(total / 32768, lo), hi);
    lp = std::max<uint64_t>(lp / mn, 1) * mn;
    (void)mx;
    uint64_t walkable = 0;
    for (uint32_t i = 0; i < n; i++)
        if (lens[i] >= 2 * lp) walkable += lens[i];
    if (walkable / lp < min_pieces) return 0;
    return lp;
}

// up: the stream the work lists are uploaded on (nullptr: synchronous copies).
// Uploads from the plan's own host vectors, which stay unchanged until the
// next build of this plan (after its previous run has been waited for).
rcdc_status plan_build(rcdc_ctx *ctx, rcdc_plan *pl, const uint64_t *offs, const uint64_t *lens,
                       uint32_t n, uint64_t arena_len, hipStream_t up = nullptr) {
    const uint64_t pos_lo = ctx->min + kWindow;  // first pure-window test position
    pl->ctx = ctx;
    pl->n = n;
    pl->arena_len = arena_len;
    for (uint32_t i = 0; i < n; i++)
        if (offs[i] > arena_len || lens[i] > arena_len - offs[i])
            return fail(RCDC_ERR_INVALID_INPUT, "stream %u [%llu,+%llu) outside arena of %llu B", i,
                        (unsigned long long)offs[i], (unsigned long long)lens[i],
                        (unsigned long long)arena_len);
    const uint64_t Lp = pl->no_walk ? 0 : walk_piece_bytes(lens, n, ctx->min, ctx->max);
    pl->walked.assign(n, 0);
    for (uint32_t i = 0; i < n; i++) pl->walked[i] = Lp && lens[i] >= 2 * Lp;
    std::vector<uint64_t> spans;
    spans.reserve(n);
    for (uint32_t i = 0; i < n; i++)
        if (!pl->walked[i] && lens[i] > pos_lo)
            spans.push_back(lens[i] - (stream_q0(offs[i], pos_lo, q0_align()) - offs[i] + 65));
    const int nc = 1;
    const int nthreads = scan_threads(ctx->variant);
    uint32_t S = choose_segment(spans, ctx->num_cus, nc, nthreads);
    if (const char *e = getenv("RCDC_SEG_BYTES")) S = (uint32_t)(atoi(e) / 128 * 128);  // experiments
    pl->seg_bytes = S;
    pl->items.clear();
    pl->sds.assign(n, StreamDesc{});
    pl->cut_base.assign(n, 0);
    uint64_t nseg = 0, ncut = 0;
    pl->scanned = 0;
    for (uint32_t i = 0; i < n; i++) {
        StreamDesc &d = pl->sds[i];
        const uint64_t N = lens[i], off = offs[i];
        d.off = off;
        d.n = N;
        d.cut_base = ncut;
        d.cut_cap = N / ctx->min + 1;
        pl->cut_base[i] = ncut;
        ncut += d.cut_cap;
        d.sum_base = nseg;
        d.item_base = pl->items.size();
        if (N <= pos_lo || pl->walked[i]) continue;
        // lane start q (arena offset) 16-aligned; tests positions q+65 ..
        const uint64_t q0 = stream_q0(off, pos_lo, q0_align());
        const uint64_t p0 = q0 - off + 65;
        const uint64_t segs = (N - p0 + S - 1) / S;
        d.pos0 = p0;
        d.nseg = segs;
        pl->scanned += segs * (uint64_t)S;
        for (uint64_t j = 0; j < segs; j += 64) {
            ScanItem it{};
            it.q0 = q0 + j * S;
            it.pos0 = p0 + j * S;
            it.lo = pos_lo;
            it.hi = N;
            it.sum_idx = nseg + j;
            const uint64_t rest = arena_len > it.q0 ? arena_len - it.q0 : 0;
            it.rec_bytes = std::min<uint64_t>(rest, 0xFFFFFFFFull);
            it.nvalid = (uint32_t)std::min<uint64_t>(64, segs - j);
            it.stream = i;
            pl->items.push_back(it);
        }
        nseg += segs;
    }
    pl->nseg = nseg;
    pl->ncuts = ncut;
    build_resolve_units(pl, ctx->min);
    // walk units: pieces of Lp bytes of every walked stream (the last one to
    // N), except that the last RCDC_WALK_SPLIT % (default 20) of a stream's
    // pieces are cut into pieces of Ls = Lp / 4 (a multiple of min).  Units
    // stay in stream order (the chain kernels need that); the walk kernel's
    // queue hands out all big pieces first and the small ones last, so the
    // last pieces the waves take are short and the grid drains evenly.
    pl->wunits.clear();
    pl->wstream_u0.clear();
    pl->worder.clear();
    pl->nwpiece_cuts = 0;
    {
        // splitting pays only when a wave takes several pieces (the tail is
        // then the last pieces' length); with about one piece per wave slot
        // (C5: 3200 pieces, 4096 slots) it only adds boundaries
        // a stream of N bytes has round(N / Lp) pieces of Lp, the last one
        // running to N (0.5 - 1.5 Lp): with floor(N / Lp) a stream just under
        // 3 Lp ended in a piece of ~2 Lp, the longest job of the queue (C4's
        // 8-12 MiB files: 8 MiB pieces started last and set the makespan)
        auto npieces = [Lp](uint64_t N) { return std::max<uint64_t>((N + Lp / 2) / Lp, 1); };
        uint64_t big_total = 0;
        for (uint32_t i = 0; i < n && Lp; i++)
            if (pl->walked[i]) big_total += npieces(lens[i]);
        const uint64_t slots = (uint64_t)std::max(ctx->num_cus, 1) * 16;
        pl->walk_many = big_total >= 2 * slots;
        uint64_t split_pct = pl->walk_many ? 20 : 0;
        if (const char *e = getenv("RCDC_WALK_SPLIT")) split_pct = std::min<uint64_t>(atoll(e), 100);
        const uint64_t Ls = Lp ? std::max<uint64_t>(Lp / 4 / ctx->min, 1) * ctx->min : 0;
        pl->walk_small = Ls;
        std::vector<uint32_t> small;
        for (uint32_t i = 0; i < n && Lp; i++) {
            if (!pl->walked[i]) continue;
            const uint64_t N = lens[i];
            const uint64_t P = npieces(N);
            const uint64_t nsplit = Ls < Lp ? (P * split_pct + 50) / 100 : 0;
            const uint32_t u0 = (uint32_t)pl->wunits.size();
            pl->wstream_u0.push_back(u0);
            uint32_t j = 0;
            auto add = [&](uint64_t a, uint64_t e, bool is_small) {
                WalkUnit u{};
                u.start = a;
                u.stop = e;
                u.out_base = pl->nwpiece_cuts;
                // cuts in [start, first cut >= stop]: >= min apart, plus the crossing and EOF cuts
                u.out_cap = (uint32_t)((e - a) / ctx->min + ctx->max / ctx->min + 4);
                u.stream = i;
                u.piece = j++;
                u.unit0 = u0;
                pl->nwpiece_cuts += u.out_cap;
                (is_small ? small : pl->worder).push_back((uint32_t)pl->wunits.size());
                pl->wunits.push_back(u);
            };
            for (uint64_t b = 0; b < P; b++) {
                const uint64_t a = b * Lp, e = b + 1 < P ? (b + 1) * Lp : N;
                if (b + nsplit < P) {
                    add(a, e, false);
                } else {
                    const uint64_t q = std::max<uint64_t>((e - a) / Ls, 1);
                    for (uint64_t k = 0; k < q; k++)
                        add(a + k * Ls, k + 1 < q ? a + (k + 1) * Ls : e, true);
                }
            }
            for (uint32_t k = u0; k < (uint32_t)pl->wunits.size(); k++) {
                pl->wunits[k].npieces = j;
                pl->wunits[k].nbig = (uint32_t)(P - nsplit);
            }
        }
        pl->worder.insert(pl->worder.end(), small.begin(), small.end());
        pl->nsmall_units = (uint32_t)small.size();
    }
    WalkParams &wp = pl->wprm;
    wp = WalkParams{};
    wp.min_size = ctx->min;
    wp.max_size = ctx->max;
    wp.arena_len = arena_len;
    wp.piece_bytes = Lp ? Lp : 1;
    wp.small_bytes = pl->walk_small ? pl->walk_small : wp.piece_bytes;
    // 64 lanes x 1.5 KiB per round: a chunk's search stops in its last
    // round (sized to the known search end), so shorter rounds hash less past
    // the cut and longer ones warm up less (64 B per segment); on C3 1536
    // beats 1024 by ~0.9 % and 768 / 2048 by 1-2 % (profiles/r03f)
    wp.seg_bytes = 1536;
    if (const char *e = getenv("RCDC_WALK_SEG")) wp.seg_bytes = (uint32_t)std::max(atoi(e) / 128 * 128, 128);
    wp.mask = (uint32_t)(ctx->avg - 1);
    wp.idx_shift = (uint32_t)(ctx->deg - 32);
    wp.shift = (uint32_t)(ctx->deg - 8);
    wp.nunits = (uint32_t)pl->wunits.size();
    // the walk's tail: waves without a piece hash rounds for the busy ones
    // (up to wp.helpers rounds posted per round of the walker's own, <= 15)
    wp.helpers = 7;
    if (const char *e = getenv("RCDC_WALK_HELPMAX")) wp.helpers = (uint32_t)std::min(std::max(atoi(e), 1), 15);
    if (const char *e = getenv("RCDC_WALK_HELP"); e && atoi(e) == 0) wp.helpers = 0;
    // a fixup walks until it meets a piece's chain: a few chunks, longer only
    // through phase-shifted zero runs (min-sized chunks); more -> host redo
    wp.fix_cap = (uint32_t)(4 * (Lp ? Lp : 1) / ctx->min + ctx->max / ctx->min + 64);
    wp.fix_seg = 512;
    wp.chk_budget = 4 * ctx->max;  // gap hashing in the check kernel (64 lanes) before the fixup (1024)
    // seeded piece starts (a walker continues its finished predecessor's chain)
    wp.seed = 1;
    if (const char *e = getenv("RCDC_WALK_SEED")) wp.seed = atoi(e) != 0;
    // queue classes by piece index mod K: even pieces before odd ones (K = 2)
    // for streams of many pieces; thirds (K = 3) when streams average under
    // 64 pieces (C4 share +1.2 %, lane/ref 1.110 -> 1.102; C3's 256-piece
    // streams lose 0.3 % at K = 3, profiles/r04/seed_classes.txt)
    const uint64_t nws = std::max<uint64_t>(pl->wstream_u0.size(), 1);
    wp.seed_classes = pl->wunits.size() / nws < 64 ? 3 : 2;
    // (RCDC_WALK_CLASSES: 1-8, experiments)
    if (const char *e = getenv("RCDC_WALK_CLASSES")) wp.seed_classes = (uint32_t)std::min(std::max(atoi(e), 1), 8);
    // a hit round stops early and spreads the lanes' owed tails (round_first)
    wp.early = 1;
    if (const char *e = getenv("RCDC_WALK_EARLY")) wp.early = atoi(e) != 0;
    // round 5: fast zones, in-kernel counter resets (RCDC_WALK_ZONEFAST /
    // RCDC_WALK_KRESET = 0 turn them off for A/B runs); the cost kernel on a
    // few fat workgroups with RCDC_COST_BLOCKS <= 256 (16: 312 us against 48 us
    // on the default grid, r5e)
    wp.flags = kWalkZoneFast | kWalkKReset;
    if (const char *e = getenv("RCDC_WALK_ZONEFAST"); e && atoi(e) == 0) wp.flags &= ~kWalkZoneFast;
    if (const char *e = getenv("RCDC_WALK_KRESET"); e && atoi(e) == 0) wp.flags &= ~kWalkKReset;
    wp.flags |= kWalkStatic;
    if (const char *e = getenv("RCDC_WALK_STATIC"); e && atoi(e) == 0) wp.flags &= ~kWalkStatic;
    wp.cost_blocks = 4096;
    wp.cost_samples = 64;
    if (const char *e = getenv("RCDC_COST_SAMPLES")) {
        const int v = atoi(e);
        wp.cost_samples = v >= 64 ? 64u : v >= 32 ? 32u : 16u;
    }
    if (const char *e = getenv("RCDC_COST_BLOCKS")) wp.cost_blocks = (uint32_t)std::max(atoi(e), 1);
    if (const char *e = getenv("RCDC_CHECK_BUDGET")) wp.chk_budget = strtoull(e, nullptr, 10);
    if (const char *e = getenv("RCDC_FIX_SEG")) wp.fix_seg = (uint32_t)std::max(atoi(e) / 128 * 128, 128);
    if (const char *e = getenv("RCDC_WALK_FIXCAP")) wp.fix_cap = (uint32_t)std::max(atoi(e), 1);  // tests
    const uint64_t supers = (pl->items.size() + nc - 1) / nc;
    const uint64_t waves_needed = (supers + nthreads / 64 - 1) / (nthreads / 64);
    pl->blocks = (uint32_t)std::min<uint64_t>(waves_needed, (uint64_t)std::max(ctx->num_cus, 1));

    DeviceGuard g(ctx->device);
    auto upload = [up](void *dst, const void *src, size_t bytes) {
        return up ? hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, up)
                  : hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice);
    };
    rcdc_status st;
    if ((st = ensure_dev(&pl->d_items, &pl->cap_items, pl->items.size()))) return st;
    if ((st = ensure_dev(&pl->d_sds, &pl->cap_sds, n))) return st;
    if ((st = ensure_dev(&pl->d_sums, &pl->cap_sums, nseg))) return st;
    if ((st = ensure_dev(&pl->d_masks, &pl->cap_masks, pl->items.size()))) return st;
    if ((st = ensure_dev(&pl->d_cuts, &pl->cap_cuts, ncut))) return st;
    if ((st = ensure_dev(&pl->d_counts, &pl->cap_counts, n))) return st;
    if ((st = ensure_dev(&pl->d_units, &pl->cap_units, pl->units.size()))) return st;
    if ((st = ensure_dev(&pl->d_stitches, &pl->cap_stitches, pl->stitches.size()))) return st;
    if ((st = ensure_dev(&pl->d_piece_cuts, &pl->cap_piece_cuts, pl->npiece_cuts))) return st;
    if ((st = ensure_dev(&pl->d_piece_counts, &pl->cap_piece_counts, pl->units.size()))) return st;
    const uint64_t nw = pl->wunits.size();
    if (nw) {
        if ((st = ensure_dev(&pl->d_wunits, &pl->cap_wunits, nw))) return st;
        if ((st = ensure_dev(&pl->d_wsu0, &pl->cap_wsu0, pl->wstream_u0.size()))) return st;
        // d_worder: the static order, then (cost ordering) the per-run
        // sorted order and one key byte per piece
        // (only when waves take several pieces each: with about one piece
        // per wave slot the order hardly matters and the two extra launches
        // are most of C5's latency-bound step)
        bool cost = pl->walk_many;
        if (const char *e = getenv("RCDC_WALK_COSTSORT")) cost = atoi(e) != 0;
        if ((st = ensure_dev(&pl->d_worder, &pl->cap_worder, cost ? 2 * nw + (nw + 3) / 4 : nw)))
            return st;
        pl->wprm.order = cost ? pl->d_worder + nw : pl->d_worder;
        pl->wprm.order_in = cost ? pl->d_worder : nullptr;
        pl->wprm.order_out = cost ? pl->d_worder + nw : nullptr;
        pl->wprm.nbig_units = (uint32_t)(nw - pl->nsmall_units);
        HIP_TRY(upload(pl->d_worder, pl->worder.data(), nw * sizeof(uint32_t)));
        if ((st = ensure_dev(&pl->d_wpiece, &pl->cap_wpiece, pl->nwpiece_cuts))) return st;
        if ((st = ensure_dev(&pl->d_pstatus, &pl->cap_pstatus, nw))) return st;
        if ((st = ensure_dev(&pl->d_wstate, &pl->cap_wstate, 2 * nw))) return st;
        // epoch 0 = no run (a rebuilt plan keeps counting its runs)
        HIP_TRY(up ? hipMemsetAsync(pl->d_wstate, 0, 2 * nw * 8, up)
                   : hipMemset(pl->d_wstate, 0, 2 * nw * 8));
        if (pl->d_wstate2) {
            if ((st = ensure_dev(&pl->d_wstate2, &pl->cap_wstate2, 2 * nw))) return st;
            HIP_TRY(up ? hipMemsetAsync(pl->d_wstate2, 0, 2 * nw * 8, up)
                       : hipMemset(pl->d_wstate2, 0, 2 * nw * 8));
        }
        if ((st = ensure_dev(&pl->d_bres, &pl->cap_bres, nw))) return st;
        if ((st = ensure_dev(&pl->d_ctr, &pl->cap_ctr, 4))) return st;
        HIP_TRY(up ? hipMemsetAsync(pl->d_ctr, 0, 16, up) : hipMemset(pl->d_ctr, 0, 16));
        if (pl->d_ctr2) HIP_TRY(up ? hipMemsetAsync(pl->d_ctr2, 0, 16, up) : hipMemset(pl->d_ctr2, 0, 16));
        pl->wqbase[0] = pl->wqbase[1] = 0;
        if ((st = ensure_dev(&pl->d_fixlist, &pl->cap_fixlist, nw))) return st;
        if ((st = ensure_dev(&pl->d_fixcuts, &pl->cap_fixcuts, nw * pl->wprm.fix_cap))) return st;
        if ((st = ensure_dev(&pl->d_fixres, &pl->cap_fixres, nw))) return st;
        // four slots of work counters (WalkParams.stats_next); slot 0 is also
        // the single buffer of set 0 when counters are reset by memsets
        if ((st = ensure_dev(&pl->d_wstats, &pl->cap_wstats, 4 * kWalkStats))) return st;
        HIP_TRY(up ? hipMemsetAsync(pl->d_wstats, 0, 4 * kWalkStats * 8, up)
                   : hipMemset(pl->d_wstats, 0, 4 * kWalkStats * 8));
        pl->wruns = 0;
        pl->wprm.stats = pl->d_wstats;
        pl->wprm.trace = nullptr;
        if (const char *e = getenv("RCDC_WALK_TRACE"); e && atoi(e) > 0) {
            if ((st = ensure_dev(&pl->d_wtrace, &pl->cap_wtrace, 2 * nw * kTraceWords))) return st;
            HIP_TRY(hipMemset(pl->d_wtrace, 0, 2 * nw * kTraceWords * 8));
            pl->wprm.trace = pl->d_wtrace;
        }
        HIP_TRY(upload(pl->d_wunits, pl->wunits.data(), nw * sizeof(WalkUnit)));

        HIP_TRY(upload(pl->d_wsu0, pl->wstream_u0.data(),
                          pl->wstream_u0.size() * sizeof(uint32_t)));
    }
    if (!pl->units.empty())
        HIP_TRY(upload(pl->d_units, pl->units.data(), pl->units.size() * sizeof(ResolveUnit)));
    if (!pl->stitches.empty())
        HIP_TRY(upload(pl->d_stitches, pl->stitches.data(),
                          pl->stitches.size() * sizeof(StitchDesc)));
    if (!pl->items.empty())
        HIP_TRY(upload(pl->d_items, pl->items.data(), pl->items.size() * sizeof(ScanItem)));
    if (n)
        HIP_TRY(upload(pl->d_sds, pl->sds.data(), n * sizeof(StreamDesc)));
    if (!pl->done) HIP_TRY(hipEventCreateWithFlags(&pl->done, hipEventDisableTiming));
    pl->ran = false;
    return RCDC_OK;
}

rcdc_status plan_run(rcdc_plan *pl, const void *d_arena, hipStream_t stream) {
    rcdc_ctx *ctx = pl->ctx;
    if (((uintptr_t)d_arena & 255u) != 0)
        return fail(RCDC_ERR_INVALID_INPUT, "device arena %p is not 256-byte aligned", d_arena);
    DeviceGuard g(ctx->device);
    const void *caller_stream = stream;
    if (rcdc_status ns = null_enter(ctx, caller_stream, &stream)) return ns;
    ScanParams sp{};
    sp.seg_bytes = pl->seg_bytes;
    sp.mask = (uint32_t)(ctx->avg - 1);
    sp.idx_shift = (uint32_t)(ctx->deg - 32);
    hipEvent_t *ev = nullptr;
    if (pl->timing && (pl->tcalls++ % pl->tperiod) == 0) {
        if (pl->tev.size() < 3 * (pl->truns + 1)) {
            for (int k = 0; k < 3; k++) {
                hipEvent_t e;
                HIP_TRY(hipEventCreate(&e));
                pl->tev.push_back(e);
            }
        }
        ev = &pl->tev[3 * pl->truns];
        pl->truns++;
    }
    const uint32_t set = pl->pipelined ? pl->pp : 0;
    uint4 *sums = set ? pl->d_sums2 : pl->d_sums;
    uint64_t *masks = set ? pl->d_masks2 : pl->d_masks;
    // this run's walk buffers and parameters
    WalkParams wprm = pl->wprm;
    uint64_t *wpiece = pl->d_wpiece, *pstatus = pl->d_pstatus, *fixcuts = pl->d_fixcuts;
    wprm.wstate = wprm.seed ? pl->d_wstate : nullptr;
    pl->walk_epoch = pl->walk_epoch % ((1ull << 21) - 1) + 1;  // 1 .. 2^21 - 1
    wprm.epoch = pl->walk_epoch;
    BoundRes *bres = pl->d_bres;
    uint32_t *ctr = pl->d_ctr, *fixlist = pl->d_fixlist;
    FixRes *fixres = pl->d_fixres;
    if (set && !pl->wunits.empty()) {
        const uint64_t nw = pl->wunits.size();
        wpiece = pl->d_wpiece2;
        pstatus = pl->d_pstatus2;
        if (wprm.seed) wprm.wstate = pl->d_wstate2;
        fixcuts = pl->d_fixcuts2;
        bres = pl->d_bres2;
        ctr = pl->d_ctr2;
        fixlist = pl->d_fixlist2;
        fixres = pl->d_fixres2;
        wprm.stats = pl->d_wstats2;
        if (wprm.order_out) {  // the cost-sorted queue (and its key bytes) of this run
            wprm.order_out = pl->d_worder2;
            wprm.order = pl->d_worder2;
        }
        (void)nw;
    }
    bool ordered = false;  // the walk queue's order already enqueued
    if (pl->pipelined) {
        // hashing on this set's stream, after the caller's earlier work and
        // after the chain that last read this set (run k - 2)
        HIP_TRY(hipEventRecord(pl->ev_in[set], stream));
        stream = pl->hstream[set];
        HIP_TRY(hipStreamWaitEvent(stream, pl->ev_in[set], 0));
        // the walk queue's cost order reads only the arena: it need not wait
        // for the chain of run k - 2, and fills CUs the last walk frees
        if (!pl->wunits.empty()) {
            HIP_TRY(launch_walk_order((const uint8_t *)d_arena, pl->d_sds, pl->d_wunits, wprm,
                                      stream));
            ordered = true;
        }
        if (pl->res_pending[set]) HIP_TRY(hipStreamWaitEvent(stream, pl->ev_res[set], 0));
    }
    if (ev) HIP_TRY(hipEventRecord(ev[0], stream));
    HIP_TRY(launch_scan(ctx->variant, (const uint8_t *)d_arena, pl->d_items,
                        pl->run_items ? pl->run_items : (uint32_t)pl->items.size(), ctx->d_tables,
                        sp, sums, masks, pl->run_items ? pl->run_blocks : pl->blocks, stream));
    const uint32_t cus = (uint32_t)std::max(ctx->num_cus, 1);
    static const bool dbg = getenv("RCDC_DEBUG_SYNC") != nullptr;  // stage-by-stage sync
    if (dbg) {
        HIP_TRY(hipStreamSynchronize(stream));
        fprintf(stderr, "rcdc: scan done\n");
    }
    // chain kernels beside the next walk run narrow; the last run of a
    // pipeline (flush) has no next walk and takes every CU
    const bool narrow = pl->pipelined && !pl->flush_next;
    pl->flush_next = false;
    const uint32_t wblocks = (uint32_t)std::min<uint64_t>(cus, (pl->wunits.size() + 15) / 16);
    wprm.qbase = pl->wqbase[set];
    wprm.stats_next = nullptr;
    if ((wprm.flags & kWalkKReset) && !pl->wunits.empty()) {
        const uint32_t slot = (uint32_t)(pl->wruns % 4);
        wprm.stats = pl->d_wstats + slot * kWalkStats;
        wprm.stats_next = pl->d_wstats + ((slot + 2) % 4) * kWalkStats;
        pl->last_wslot = slot;
        pl->wruns++;
    } else {
        pl->last_wslot = set ? 4 : 0;  // (4: d_wstats2)
    }
    HIP_TRY(launch_walk((const uint8_t *)d_arena, pl->d_sds, pl->d_wunits, wprm, ctx->d_tables,
                        wpiece, pstatus, ctr, wblocks, stream, ordered));
    if (!pl->wunits.empty() && (wprm.flags & kWalkKReset))  // takes of this run: one per
        pl->wqbase[set] += (uint32_t)pl->wunits.size() +     // piece, one failed per wave;
                           ((wprm.flags & kWalkStatic) ? 0u : wblocks * 16u);  // static: nunits
    if (dbg) {
        HIP_TRY(hipStreamSynchronize(stream));
        uint32_t h[4] = {0, 0, 0, 0};
        if (!pl->wunits.empty()) HIP_TRY(hipMemcpy(h, ctr, 16, hipMemcpyDeviceToHost));
        fprintf(stderr, "rcdc: walk done (%zu units; queue %u)\n", pl->wunits.size(), h[0]);
    }
    if (ev) HIP_TRY(hipEventRecord(ev[1], stream));
    const hipStream_t scan_stream = stream;
    if (pl->pipelined) {  // resolve on the plan's own stream, after this scan
        HIP_TRY(hipEventRecord(pl->ev_scan[set], stream));
        stream = pl->rstream;
        HIP_TRY(hipStreamWaitEvent(stream, pl->ev_scan[set], 0));
    }
    ResolveParams rp{};
    rp.min_size = ctx->min;
    rp.max_size = ctx->max;
    rp.seg_bytes = pl->seg_bytes;
    rp.mask = (uint32_t)(ctx->avg - 1);
    rp.shift = (uint32_t)(ctx->deg - 8);
    HIP_TRY(launch_resolve((const uint8_t *)d_arena, pl->d_sds, pl->d_units,
                           (uint32_t)pl->units.size(), pl->d_stitches,
                           (uint32_t)pl->stitches.size(), ctx->d_tables, rp, sums,
                           masks, pl->d_cuts, pl->d_counts, pl->d_piece_cuts,
                           pl->d_piece_counts, nullptr, stream));
    if (dbg) {
        HIP_TRY(hipStreamSynchronize(stream));
        fprintf(stderr, "rcdc: resolve done\n");
    }
    HIP_TRY(launch_walk_chain((const uint8_t *)d_arena, pl->d_sds, pl->d_wunits, pl->d_wsu0,
                              (uint32_t)pl->wstream_u0.size(), wprm, ctx->d_tables,
                              wpiece, pstatus, bres, ctr, fixlist,
                              fixcuts, fixres, pl->d_cuts, pl->d_counts,
                              narrow ? std::min<uint32_t>(cus, pl->fix_blocks_pipe) : cus,
                              narrow ? pl->chk_blocks_pipe : cus, stream,
                              pl->pipelined));
    if (ev) HIP_TRY(hipEventRecord(ev[2], stream));
    pl->last_set = set;
    if (pl->pipelined) {
        HIP_TRY(hipEventRecord(pl->ev_res[set], stream));
        pl->res_pending[set] = true;
        pl->pp ^= 1u;
    }
    (void)scan_stream;
    pl->last_arena = d_arena;
    pl->last_stream = stream;
    HIP_TRY(hipEventRecord(pl->done, stream));
    // (pipelined runs stay asynchronous beyond the caller's stream: their
    // completion is rcdc_plan_finish / the device synchronisation)
    if (!pl->pipelined)
        if (rcdc_status ns = null_leave(ctx, caller_stream, stream)) return ns;
    pl->ran = true;
    pl->hashed = false;
    pl->finished = false;
    return RCDC_OK;
}

void plan_release(rcdc_plan *pl);

// SHA-256 of (offset, length) refs of the plan's last arena into the plan's
// digest slots (a stream the walk path handed back to the scan path).
rcdc_status launch_list_hash(rcdc_plan *pl, const std::vector<ulonglong2> &refs,
                             const std::vector<uint64_t> &slots) {
    DeviceGuard g(pl->ctx->device);
    ulonglong2 *d_refs = nullptr;
    uint32_t *d_out = nullptr;
    std::vector<uint8_t> out(refs.size() * 32);
    hipStream_t st = pl->ctx->stream;
    hipError_t e = hipMalloc((void **)&d_refs, refs.size() * sizeof(ulonglong2));
    if (e == hipSuccess) e = hipMalloc((void **)&d_out, out.size());
    if (e == hipSuccess)
        e = hipMemcpy(d_refs, refs.data(), refs.size() * sizeof(ulonglong2), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipStreamWaitEvent(st, pl->done, 0);  // after the plan's hash
    if (e == hipSuccess)
        e = launch_sha256_list((const uint8_t *)pl->last_arena, d_refs, (uint32_t)refs.size(),
                               d_out, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e == hipSuccess) e = hipMemcpy(out.data(), d_out, out.size(), hipMemcpyDeviceToHost);
    for (size_t r = 0; r < refs.size() && e == hipSuccess; r++)
        e = hipMemcpy((uint8_t *)pl->d_dig + slots[r] * 32, out.data() + r * 32, 32,
                      hipMemcpyHostToDevice);
    (void)hipFree(d_refs);
    (void)hipFree(d_out);
    HIP_TRY(e);
    return RCDC_OK;
}


// Completes the last run: waits for it, redoes on the scan path any walked
// stream whose fixup overflowed (device count ~0; never seen outside forced
// tests) and writes those cuts -- and, if the run was hashed, their digests
// -- back into the device buffers, so the device views are complete.
rcdc_status plan_finish(rcdc_plan *pl) {
    if (!pl->ran) return fail(RCDC_ERR_INVALID_INPUT, "plan has not been run");
    if (pl->finished) return RCDC_OK;
    DeviceGuard g(pl->ctx->device);
    HIP_TRY(poll_event(pl->done));
    std::vector<uint64_t> &cnt = pl->fin_counts;
    cnt.assign(pl->n, 0);
    // read-backs on the run's own stream, not hipMemcpy: the legacy default
    // stream sits on one of HIP's hardware queues too, and a copy queued
    // there waits for whatever long kernel another stream put on that queue
    // (the ingest's 62 ms chunk-id kernels serialised its batches, r5l)
    if (pl->n) {
        HIP_TRY(hipMemcpyAsync(cnt.data(), pl->d_counts, pl->n * 8, hipMemcpyDeviceToHost,
                               pl->last_stream));
        HIP_TRY(poll_stream(pl->last_stream));
    }
    if (const char *e = getenv("RCDC_WALK_DUMP"); e && !pl->wunits.empty()) {  // debugging aid
        const uint32_t want = (uint32_t)atoi(e);
        const size_t nw = pl->wunits.size();
        std::vector<uint64_t> ps(nw), pc(pl->nwpiece_cuts);
        std::vector<BoundRes> br(nw);
        std::vector<FixRes> fr(nw);
        std::vector<uint64_t> fc(nw * pl->wprm.fix_cap);
        HIP_TRY(hipMemcpy(ps.data(), pl->d_pstatus, nw * 8, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(pc.data(), pl->d_wpiece, pc.size() * 8, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(br.data(), pl->d_bres, nw * sizeof(BoundRes), hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(fr.data(), pl->d_fixres, nw * sizeof(FixRes), hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(fc.data(), pl->d_fixcuts, fc.size() * 8, hipMemcpyDeviceToHost));
        for (size_t u = 0; u < nw; u++) {
            const WalkUnit &U = pl->wunits[u];
            if (U.stream != want) continue;
            fprintf(stderr, "unit %zu piece %u [%llu,%llu) n=%llu open=%d:", u, U.piece,
                    (unsigned long long)U.start, (unsigned long long)U.stop,
                    (unsigned long long)(ps[u] & 0xFFFFFFFFu), (int)((ps[u] >> 32) & 1));
            for (uint64_t i = 0; i < (ps[u] & 0xFFFFFFFFu); i++) {
                const uint64_t v = pc[U.out_base + i];
                fprintf(stderr, " %llu%c", (unsigned long long)(v & kCutVal), "hmez"[v >> 62]);
            }
            if (U.piece) {
                const BoundRes &B = br[u];
                fprintf(stderr, "\n   bound kind %u nhops %u merge %u/%d fix_from %llu hops:", B.kind,
                        B.nhops, B.merge_unit, B.merge_idx, (unsigned long long)B.fix_from);
                for (uint32_t i = 0; i < B.nhops && i < (uint32_t)kMaxHops; i++)
                    fprintf(stderr, " %llu%s", (unsigned long long)(B.hops[i] & kCutVal),
                            (B.hops[i] >> 62) ? "r" : "");
                if (B.kind == kBoundFixup) {
                    fprintf(stderr, "\n   fix count %u merge %u/%d:", fr[u].count, fr[u].merge_unit,
                            fr[u].merge_idx);
                    for (uint32_t i = 0; i < fr[u].count && i < pl->wprm.fix_cap; i++)
                        fprintf(stderr, " %llu", (unsigned long long)fc[u * pl->wprm.fix_cap + i]);
                }
            }
            fprintf(stderr, "\n");
        }
    }
    std::vector<ulonglong2> refs;
    std::vector<uint64_t> slots;
    for (uint32_t i = 0; i < pl->n; i++) {
        if (cnt[i] != ~0ull) continue;
        rcdc_plan tmp;
        tmp.no_walk = true;
        const uint64_t off = pl->sds[i].off, len = pl->sds[i].n;
        rcdc_status st = plan_build(pl->ctx, &tmp, &off, &len, 1, pl->arena_len);
        if (!st) st = plan_run(&tmp, pl->last_arena, pl->last_stream);
        if (!st) st = tmp.done ? (hipEventSynchronize(tmp.done) == hipSuccess ? RCDC_OK
                                  : fail(RCDC_ERR_INTERNAL, "redo sync")) : RCDC_OK;
        uint64_t c1 = 0;
        std::vector<uint64_t> redo;
        if (!st && hipMemcpy(&c1, tmp.d_counts, 8, hipMemcpyDeviceToHost) != hipSuccess)
            st = fail(RCDC_ERR_INTERNAL, "redo counts");
        if (!st && c1 > pl->sds[i].cut_cap)
            st = fail(RCDC_ERR_INTERNAL, "stream %u: %llu cuts > bound", i, (unsigned long long)c1);
        if (!st) {
            redo.resize(c1);
            if (c1 && hipMemcpy(redo.data(), tmp.d_cuts, c1 * 8, hipMemcpyDeviceToHost) != hipSuccess)
                st = fail(RCDC_ERR_INTERNAL, "redo cuts");
        }
        plan_release(&tmp);
        if (st) return st;
        if (c1) HIP_TRY(hipMemcpy(pl->d_cuts + pl->cut_base[i], redo.data(), c1 * 8,
                                  hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(pl->d_counts + i, &c1, 8, hipMemcpyHostToDevice));
        cnt[i] = c1;
        uint64_t prev = 0;
        for (uint64_t j = 0; j < c1; j++) {
            refs.push_back({pl->sds[i].off + prev, redo[j] - prev});
            slots.push_back(pl->cut_base[i] + j);
            prev = redo[j];
        }
    }
    if (pl->hashed && !refs.empty()) {
        rcdc_status st = launch_list_hash(pl, refs, slots);
        if (st) return st;
    }
    pl->finished = true;
    return RCDC_OK;
}

rcdc_status plan_results(rcdc_plan *pl, uint64_t *cuts, uint64_t cap, uint64_t *counts) {
    rcdc_status st = plan_finish(pl);
    if (st) return st;
    const std::vector<uint64_t> &cnt = pl->fin_counts;
    uint64_t total = 0;
    for (uint32_t i = 0; i < pl->n; i++) {
        if (cnt[i] > pl->sds[i].cut_cap)
            return fail(RCDC_ERR_INTERNAL, "stream %u produced %llu cuts > bound %llu", i,
                        (unsigned long long)cnt[i], (unsigned long long)pl->sds[i].cut_cap);
        counts[i] = cnt[i];
        total += cnt[i];
    }
    if (total > cap) return fail(RCDC_ERR_CAPACITY, "need %llu cut slots, have %llu",
                                 (unsigned long long)total, (unsigned long long)cap);
    DeviceGuard g(pl->ctx->device);
    std::vector<uint64_t> all(pl->ncuts);
    if (pl->ncuts) {
        HIP_TRY(hipMemcpyAsync(all.data(), pl->d_cuts, pl->ncuts * 8, hipMemcpyDeviceToHost,
                               pl->last_stream));
        HIP_TRY(poll_stream(pl->last_stream));
    }
    uint64_t o = 0;
    for (uint32_t i = 0; i < pl->n; i++) {
        memcpy(cuts + o, all.data() + pl->cut_base[i], cnt[i] * 8);
        o += cnt[i];
    }
    return RCDC_OK;
}

void plan_release(rcdc_plan *pl) {
    DeviceGuard g(pl->ctx ? pl->ctx->device : 0);
    (void)hipFree(pl->d_wunits);
    (void)hipFree(pl->d_wsu0);
    (void)hipFree(pl->d_worder);
    (void)hipFree(pl->d_wpiece);
    (void)hipFree(pl->d_pstatus);
    (void)hipFree(pl->d_bres);
    (void)hipFree(pl->d_ctr);
    (void)hipFree(pl->d_fixlist);
    (void)hipFree(pl->d_fixcuts);
    (void)hipFree(pl->d_fixres);
    (void)hipFree(pl->d_wstats);
    (void)hipFree(pl->d_wtrace);
    (void)hipFree(pl->d_items);
    (void)hipFree(pl->d_sds);
    (void)hipFree(pl->d_sums);
    (void)hipFree(pl->d_masks);
    (void)hipFree(pl->d_sums2);
    (void)hipFree(pl->d_masks2);
    (void)hipFree(pl->d_wpiece2);
    (void)hipFree(pl->d_pstatus2);
    (void)hipFree(pl->d_wstate);
    (void)hipFree(pl->d_wstate2);
    (void)hipFree(pl->d_fixcuts2);
    (void)hipFree(pl->d_bres2);
    (void)hipFree(pl->d_ctr2);
    (void)hipFree(pl->d_fixlist2);
    (void)hipFree(pl->d_worder2);
    (void)hipFree(pl->d_fixres2);
    (void)hipFree(pl->d_wstats2);
    for (int k = 0; k < 2; k++) {
        if (pl->ev_in[k]) (void)hipEventDestroy(pl->ev_in[k]);
        if (pl->ev_scan[k]) (void)hipEventDestroy(pl->ev_scan[k]);
        if (pl->ev_res[k]) (void)hipEventDestroy(pl->ev_res[k]);
        if (pl->hstream[k]) (void)hipStreamDestroy(pl->hstream[k]);
    }
    if (pl->rstream) (void)hipStreamDestroy(pl->rstream);
    (void)hipFree(pl->d_cuts);
    (void)hipFree(pl->d_counts);
    (void)hipFree(pl->d_dig);
    (void)hipFree(pl->d_shaw);
    (void)hipFree(pl->d_order);
    (void)hipFree(pl->d_units);
    (void)hipFree(pl->d_stitches);
    (void)hipFree(pl->d_piece_cuts);
    (void)hipFree(pl->d_piece_counts);
    if (pl->done) (void)hipEventDestroy(pl->done);
    for (hipEvent_t e : pl->tev) (void)hipEventDestroy(e);
}

void plan_free(rcdc_plan *pl) {
    if (!pl) return;
    plan_release(pl);
    delete pl;
}

void lane_free(rcdc_ctx *ctx, Lane *L) {
    if (!L) return;
    DeviceGuard g(ctx->device);
    if (L->stream) (void)hipStreamSynchronize(L->stream);
    plan_free(L->plan);
    for (int k = 0; k < 4; k++) {
        if (L->ev[k]) (void)hipEventDestroy(L->ev[k]);
        if (L->pinned[k]) (void)hipHostFree(L->pinned[k]);
    }
    (void)hipFree(L->d_arena);
    if (L->stream) (void)hipStreamDestroy(L->stream);
    delete L;
}

// Take a free lane (creating one while fewer than max_lanes exist, else
// waiting for one); give it back with lane_release.
rcdc_status lane_acquire(rcdc_ctx *ctx, Lane **out) {
    std::unique_lock<std::mutex> lk(ctx->pool_mu);
    while (ctx->free_lanes.empty() && ctx->lanes.size() >= ctx->max_lanes) ctx->pool_cv.wait(lk);
    if (!ctx->free_lanes.empty()) {
        *out = ctx->free_lanes.back();
        ctx->free_lanes.pop_back();
        return RCDC_OK;
    }
    Lane *L = new Lane();
    ctx->lanes.push_back(L);  // counted now; its HIP objects are made below
    lk.unlock();
    DeviceGuard g(ctx->device);
    hipError_t e = hipStreamCreateWithFlags(&L->stream, hipStreamNonBlocking);
    for (int k = 0; k < 4 && e == hipSuccess; k++)
        e = hipEventCreateWithFlags(&L->ev[k], hipEventDisableTiming);
    if (e != hipSuccess) {
        std::lock_guard<std::mutex> lk2(ctx->pool_mu);
        ctx->lanes.erase(std::find(ctx->lanes.begin(), ctx->lanes.end(), L));
        lane_free(ctx, L);
        ctx->pool_cv.notify_one();
        return fail(RCDC_ERR_INTERNAL, "lane setup: %s", hipGetErrorString(e));
    }
    *out = L;
    return RCDC_OK;
}

void lane_release(rcdc_ctx *ctx, Lane *L) {
    std::lock_guard<std::mutex> lk(ctx->pool_mu);
    ctx->free_lanes.push_back(L);
    ctx->pool_cv.notify_one();
}

// pinned staging per lane: 4 slots of 4 MiB (a 16-24 MiB stream pass's host
// copies run ahead of its own DMA; 2 x 16 MiB: 40-46 GiB/s, 4 x 4 MiB:
// 46.5-47.5 GiB/s through rcdc_stream_feed, tools/gpu_abi.sh)
constexpr uint64_t kStageBytes = 4ull << 20;

// RCDC_STAGE_MIB / RCDC_STAGE_SLOTS: staging slot size and count per lane
// (A/B runs; smaller slots overlap a pass's host copy with its own DMA, more
// slots let the copies run further ahead of the DMA)
static uint64_t stage_bytes() {
    static const uint64_t b = getenv("RCDC_STAGE_MIB")
                                  ? std::max<uint64_t>((uint64_t)atoll(getenv("RCDC_STAGE_MIB")), 1) << 20
                                  : kStageBytes;
    return b;
}

static uint32_t stage_slots() {
    static const uint32_t k = getenv("RCDC_STAGE_SLOTS")
                                  ? std::min<uint32_t>(std::max(atoi(getenv("RCDC_STAGE_SLOTS")), 2), 4)
                                  : 4u;
    return k;
}

// Capacity class of a single-stream host pass: a lane's plan is built for
// the class and reused for every length in it (the stream path's passes are
// 16 MiB plus a tail of up to max bytes: a plan per exact length rebuilt it
// on almost every pass).  Up to 64 MiB, built without walk pieces or
// resolver pieces (one resolve wave per pass: a few tens of hops).
static uint64_t cap_class(const rcdc_ctx *ctx, uint64_t n) {
    const uint64_t c = round_up(std::max<uint64_t>(n, 1), 8ull << 20);
    (void)ctx;
    return c <= (64ull << 20) ? c : 0;
}

// The plan (built for a capacity of one stream) set to length n: the
// stream's descriptor and the first items' end position on the device
// (values as kernel arguments: nothing to copy), and the items the scan runs.
static rcdc_status plan_set_len(rcdc_plan *pl, uint64_t n, hipStream_t st) {
    const StreamDesc &d = pl->sds[0];
    const uint64_t pos_lo = pl->ctx->min + kWindow;
    uint64_t nseg = 0;
    if (n > pos_lo && d.nseg) nseg = std::min<uint64_t>(d.nseg, (n - d.pos0 + pl->seg_bytes - 1) / pl->seg_bytes);
    const uint32_t nit = (uint32_t)((nseg + 63) / 64);
    pl->run_items = nit ? nit : 1;  // (an all-masked item when there is nothing to scan)
    const uint32_t waves = pl->run_items;
    pl->run_blocks = std::min<uint32_t>((waves + 15) / 16, (uint32_t)std::max(pl->ctx->num_cus, 1));
    HIP_TRY(launch_plan_set_len(pl->d_sds, pl->d_items, nit ? nit : (uint32_t)std::min<size_t>(1, pl->items.size()),
                                n, nseg, st));
    return RCDC_OK;
}

// Host-path phase timing (RCDC_HOST_PROFILE=1: summary on stderr when the
// context is destroyed): staging copies, waits for a staging slot, plan
// (re)builds, device run + result copy.
struct HostProfile {
    std::atomic<uint64_t> ns[4] = {{0}, {0}, {0}, {0}};
    std::atomic<uint64_t> passes{0}, bytes{0}, builds{0};
};
HostProfile g_hprof;
const bool g_hprof_on = getenv("RCDC_HOST_PROFILE") != nullptr;

inline uint64_t now_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Whether a host address lies in page-locked memory HIP knows of (pageable
// memory answers with an error or "unregistered"; the error is cleared so no
// later launch check sees it).
bool host_pinned(const void *p) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// One piece of host memory at an arena offset.
struct HostPiece {
    uint64_t off;
    const uint8_t *p;
    uint64_t n;
};

// Host bytes -> pinned staging (two slots, copy k + 1 overlapping the DMA of
// copy k) -> the lane's device arena -> plan -> cuts, all on the lane's
// stream.  Stream i of the batch is the concatenation of its pieces (a
// streaming caller's buffered tail and its new read need no intermediate
// copy).  The plan is rebuilt only when the batch layout changes.
// d_prefix (optional): the first prefix_len bytes of the arena come from
// device memory (a stream's tail kept from its previous pass), not the host.
rcdc_status run_host_pieces(rcdc_ctx *ctx, Lane *L, const std::vector<uint64_t> &lens,
                            const std::vector<HostPiece> &pieces, uint64_t *cuts, uint64_t cap,
                            uint64_t *counts, const uint8_t *d_prefix = nullptr,
                            uint64_t prefix_len = 0, hipEvent_t prefix_ready = nullptr) {
    const uint32_t n = (uint32_t)lens.size();
    std::vector<uint64_t> offs(n);
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; i++) {
        offs[i] = total;
        total = round_up(total + lens[i], 256);
    }
    const uint64_t arena_len = total + 256;
    // one stream short of pieces and walk: a plan per capacity class, set
    // to this pass's length on the device; otherwise a plan per exact layout
    static const bool capacity = !getenv("RCDC_EXACT_PLANS");
    const uint64_t cap1 = (capacity && n == 1) ? cap_class(ctx, lens[0]) : 0;
    std::vector<uint64_t> klens = cap1 ? std::vector<uint64_t>{cap1} : lens;
    const uint64_t karena = cap1 ? round_up(cap1, 256) + 256 : arena_len;
    DeviceGuard g(ctx->device);
    rcdc_status st;
    if ((st = ensure_dev(&L->d_arena, &L->arena_cap, std::max(arena_len, karena)))) return st;
    if (!L->pinned[0]) {
        L->stage = stage_bytes();
        L->nslots = stage_slots();
        for (uint32_t k = 0; k < L->nslots; k++)
            HIP_TRY(hipHostMalloc((void **)&L->pinned[k], L->stage, hipHostMallocDefault));
    }
    uint64_t t_copy = 0, t_wait = 0, t0 = g_hprof_on ? now_ns() : 0;
    // From the first copy on, an early error return must not leave a DMA
    // from the caller's buffer (direct) or the lane's slots (staged) in
    // flight: the header promises the buffer is free on return, and the lane
    // goes back to the pool.  Disarmed once plan_results has waited.
    struct DrainOnError {
        hipStream_t s;
        bool armed = true;
        ~DrainOnError() {
            if (armed) (void)hipStreamSynchronize(s);
        }
    } drain{L->stream};
    if (prefix_len) {
        if (prefix_ready) HIP_TRY(hipStreamWaitEvent(L->stream, prefix_ready, 0));
        HIP_TRY(hipMemcpyAsync(L->d_arena, d_prefix, prefix_len, hipMemcpyDeviceToDevice,
                               L->stream));
    }
    // every piece page-locked (rcdc_host_alloc): DMA straight from the
    // caller's buffer; plan_results below waits for the pass, so the buffer
    // is free again when this returns
    static const bool direct_ok = !getenv("RCDC_NO_DIRECT_DMA");
    bool direct = direct_ok && !pieces.empty();
    for (size_t j = 0; direct && j < pieces.size(); j++)
        direct = host_pinned(pieces[j].p) && host_pinned(pieces[j].p + pieces[j].n - 1);
    if (direct)
        for (const HostPiece &pc : pieces)
            HIP_TRY(hipMemcpyAsync(L->d_arena + pc.off, pc.p, pc.n, hipMemcpyHostToDevice,
                                   L->stream));
    // staged copies: block k of the arena goes through slot k & 1
    size_t pi = 0;  // first piece that may overlap the block
    uint64_t k = 0;
    for (uint64_t p = prefix_len; !direct && p < total; p += L->stage, k++) {
        const uint64_t e = std::min(p + L->stage, total);
        const int slot = (int)(k % L->nslots);
        if (k >= L->nslots) {
            const uint64_t w0 = g_hprof_on ? now_ns() : 0;
            HIP_TRY(hipEventSynchronize(L->ev[slot]));  // its previous DMA is done
            if (g_hprof_on) t_wait += now_ns() - w0;
        }
        const uint64_t c0 = g_hprof_on ? now_ns() : 0;
        uint8_t *dst = L->pinned[slot];
        while (pi < pieces.size() && pieces[pi].off + pieces[pi].n <= p) pi++;
        for (size_t j = pi; j < pieces.size() && pieces[j].off < e; j++) {
            const uint64_t a = std::max(pieces[j].off, p), b = std::min(pieces[j].off + pieces[j].n, e);
            if (a < b) memcpy(dst + (a - p), pieces[j].p + (a - pieces[j].off), b - a);
        }
        if (g_hprof_on) t_copy += now_ns() - c0;
        HIP_TRY(hipMemcpyAsync(L->d_arena + p, dst, e - p, hipMemcpyHostToDevice, L->stream));
        HIP_TRY(hipEventRecord(L->ev[slot], L->stream));
    }
    const uint64_t b0 = g_hprof_on ? now_ns() : 0;
    // a lane's capacity plan serves any single-stream pass it covers (the
    // scan runs only the items the pass needs)
    const bool covers = cap1 && L->plan && L->lay_cap && L->lay_offs == offs &&
                        L->lay_lens.size() == 1 && L->lay_lens[0] >= lens[0];
    if (covers) klens = L->lay_lens;
    if (!covers &&
        (!L->plan || L->lay_offs != offs || L->lay_lens != klens || L->lay_arena != karena)) {
        if (!L->plan) L->plan = new rcdc_plan();
        L->plan->no_walk = L->plan->no_pieces = cap1 != 0;
        if ((st = plan_build(ctx, L->plan, offs.data(), klens.data(), n, karena, L->stream))) {
            L->lay_offs.clear();
            return st;
        }
        L->plan->run_items = 0;
        if (cap1 && (!L->plan->wunits.empty() || !L->plan->stitches.empty())) {
            // not the shape a length can be set on: exact plans from here
            L->plan->no_walk = L->plan->no_pieces = false;
            if ((st = plan_build(ctx, L->plan, offs.data(), lens.data(), n, arena_len, L->stream))) {
                L->lay_offs.clear();
                return st;
            }
            klens = lens;
        }
        L->lay_offs = offs;
        L->lay_lens = klens;
        L->lay_cap = cap1 && klens[0] == cap1;
        L->lay_arena = L->lay_cap ? karena : arena_len;
        if (g_hprof_on) g_hprof.builds++;
    }
    if (cap1 && L->lay_cap && (st = plan_set_len(L->plan, lens[0], L->stream))) return st;
    const uint64_t r0 = g_hprof_on ? now_ns() : 0;
    if ((st = plan_run(L->plan, L->d_arena, L->stream))) return st;
    st = plan_results(L->plan, cuts, cap, counts);
    drain.armed = st != RCDC_OK && st != RCDC_ERR_CAPACITY;  // capacity: the pass completed
    if (g_hprof_on) {
        const uint64_t t1 = now_ns();
        g_hprof.ns[0] += t_copy;
        g_hprof.ns[1] += t_wait;
        g_hprof.ns[2] += r0 - b0;
        g_hprof.ns[3] += t1 - r0;
        g_hprof.passes++;
        g_hprof.bytes += total;
        (void)t0;
    }
    return st;
}

rcdc_status run_host_batch(rcdc_ctx *ctx, Lane *L, const rcdc_buf *bufs, uint32_t n,
                           uint64_t *cuts, uint64_t cap, uint64_t *counts) {
    std::vector<uint64_t> lens(n);
    std::vector<HostPiece> pieces;
    pieces.reserve(n);
    uint64_t off = 0;
    for (uint32_t i = 0; i < n; i++) {
        if (bufs[i].len && !bufs[i].data)
            return fail(RCDC_ERR_INVALID_INPUT, "buffer %u is NULL with length %llu", i,
                        (unsigned long long)bufs[i].len);
        lens[i] = bufs[i].len;
        if (bufs[i].len) pieces.push_back({off, bufs[i].data, bufs[i].len});
        off = round_up(off + bufs[i].len, 256);
    }
    return run_host_pieces(ctx, L, lens, pieces, cuts, cap, counts);
}

bool valid_ctx(const rcdc_ctx *c) { return c != nullptr; }

}  // namespace

// ---------------------------------------------------------------------------
// internal entry points for the ingest engine (rcdc_ingest.cpp), which is
// otherwise a client of the C ABI below
// ---------------------------------------------------------------------------
namespace rcdc {
// Rebuild `pl` (created by rcdc_plan_create, its last run waited for) for a
// new batch layout, reusing its device buffers; uploads on `up`.
rcdc_status plan_relayout(rcdc_plan *pl, const uint64_t *offs, const uint64_t *lens, uint32_t n,
                          uint64_t arena_len, hipStream_t up) {
    if (!pl || !pl->ctx) return fail(RCDC_ERR_INVALID_INPUT, "null plan");
    pl->ran = false;
    pl->finished = false;
    return plan_build(pl->ctx, pl, offs, lens, n, arena_len, up);
}
int ctx_device(const rcdc_ctx *ctx) { return ctx ? ctx->device : 0; }
uint64_t ctx_min_size(const rcdc_ctx *ctx) { return ctx ? ctx->min : 0; }
uint64_t ctx_max_size(const rcdc_ctx *ctx) { return ctx ? ctx->max : 0; }
rcdc_status set_error(rcdc_status st, const char *msg) { return fail(st, "%s", msg); }
}  // namespace rcdc

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

uint32_t rcdc_abi_version(void) { return RCDC_ABI_VERSION; }

const char *rcdc_last_error(void) { return g_err.c_str(); }

rcdc_status rcdc_check_params(uint64_t avg, uint64_t min, uint64_t max) {
    // rabin.rs:21-40, same order and same ErrorKind
    if (avg == 0 || (avg & (avg - 1)) != 0)
        return fail(RCDC_ERR_UNSUPPORTED,
                    "Chunk size must be a power of 2 for the rabin chunker. chunk size = %llu.",
                    (unsigned long long)avg);
    if (min > avg)
        return fail(RCDC_ERR_UNSUPPORTED,
                    "Chunk min size must be smaller or equal than the chunk size.");
    if (max < avg)
        return fail(RCDC_ERR_UNSUPPORTED,
                    "Chunk max size must be larger or equal than the chunk size.");
    // The reference accepts any min, but its iterator is only well defined
    // for min >= BUF_SIZE = 4096 (rabin.rs:12): a chunk that ends mid-buffer
    // leaves up to 4095 read-ahead bytes, and the next chunk does
    // `min_size -= open_buf_len` (rabin.rs:124).  Below 4096 that underflows:
    // a panic under debug assertions (the reference's test profile), and in
    // release a wrap that makes take(huge) return the whole remaining stream
    // as one chunk -- dependent on how the reader splits its reads, not a
    // function of the bytes.  No bit-exact cut list exists there, so such
    // parameters are Unsupported (the same ErrorKind as rabin.rs:22-40).
    if (min < (uint64_t)kRefBufSize)
        return fail(RCDC_ERR_UNSUPPORTED,
                    "Chunk min size must be at least 4096 bytes (the reference's read buffer, "
                    "rabin.rs:12,124). chunk min size = %llu.", (unsigned long long)min);
    if (avg > (1ull << 32) || max > (1ull << 40))
        return fail(RCDC_ERR_UNSUPPORTED, "chunk size > 4 GiB or max size > 1 TiB");
    return RCDC_OK;
}

rcdc_status rcdc_parse_poly(const char *hex, uint64_t *poly) {
    // u64::from_str_radix(s, 16): optional leading '+', hex digits only, no
    // prefix, no whitespace, non-empty, must fit in 64 bits.
    if (!hex || !poly) return fail(RCDC_ERR_INVALID_INPUT, "null argument");
    const char *p = hex;
    if (*p == '+') p++;
    if (!*p)
        return fail(RCDC_ERR_INVALID_INPUT,
                    "Parsing u64 from hex failed for polynomial `%s`, the value must be a valid "
                    "hexadecimal string.", hex);
    uint64_t v = 0;
    for (; *p; p++) {
        int d;
        if (*p >= '0' && *p <= '9') d = *p - '0';
        else if (*p >= 'a' && *p <= 'f') d = *p - 'a' + 10;
        else if (*p >= 'A' && *p <= 'F') d = *p - 'A' + 10;
        else
            return fail(RCDC_ERR_INVALID_INPUT,
                        "Parsing u64 from hex failed for polynomial `%s`, the value must be a "
                        "valid hexadecimal string.", hex);
        if (v >> 60)
            return fail(RCDC_ERR_INVALID_INPUT,
                        "Parsing u64 from hex failed for polynomial `%s`, the value must be a "
                        "valid hexadecimal string.", hex);
        v = (v << 4) | (uint64_t)d;
    }
    *poly = v;
    return RCDC_OK;
}

rcdc_status rcdc_ctx_create(uint64_t poly, uint64_t min, uint64_t avg_pow2, uint64_t max,
                            int device, rcdc_ctx **out) {
    if (!out) return fail(RCDC_ERR_INVALID_INPUT, "out is NULL");
    *out = nullptr;
    rcdc_status st = rcdc_check_params(avg_pow2, min, max);
    if (st) return st;
    const int deg = poly_degree(poly);
    // deg <= 56: `h << 8` of the reference's slide must not overflow u64;
    // deg >= 9: polynom_shift = deg - 8 must be positive
    if (deg < 9 || deg > 56)
        return fail(RCDC_ERR_UNSUPPORTED, "polynomial %#llx has degree %d; supported 9..56",
                    (unsigned long long)poly, deg);
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev)
        return fail(RCDC_ERR_INVALID_INPUT, "device %d not present (%d devices)", device, ndev);
    rcdc_ctx *c = new rcdc_ctx();
    c->device = device;
    c->poly = poly;
    c->min = min;
    c->avg = avg_pow2;
    c->max = max;
    c->deg = deg;
    DeviceGuard g(device);
    hipDeviceProp_t prop;
    hipError_t e = hipGetDeviceProperties(&prop, device);
    if (e != hipSuccess) {
        delete c;
        return fail(RCDC_ERR_INTERNAL, "hipGetDeviceProperties: %s", hipGetErrorString(e));
    }
    c->num_cus = prop.multiProcessorCount;
    if (const char *v = getenv("RCDC_SCAN_VARIANT")) c->variant = atoi(v);
    if (const char *v = getenv("RCDC_LANES")) c->max_lanes = (uint32_t)std::max(atoi(v), 1);
    uint64_t img[512];
    build_tables(poly, img);
    if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&c->ev_null_in, hipEventDisableTiming)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&c->ev_null_out, hipEventDisableTiming)) != hipSuccess ||
        (e = hipMalloc((void **)&c->d_tables, sizeof img)) != hipSuccess ||
        (e = hipMemcpy(c->d_tables, img, sizeof img, hipMemcpyHostToDevice)) != hipSuccess) {
        rcdc_ctx_destroy(c);
        return fail(RCDC_ERR_INTERNAL, "context setup: %s", hipGetErrorString(e));
    }
    *out = c;
    return RCDC_OK;
}

void rcdc_ctx_destroy(rcdc_ctx *c) {
    if (!c) return;
    if (g_hprof_on && g_hprof.passes)
        fprintf(stderr,
                "rcdc host path: %llu passes, %.1f MiB, %llu plan builds; thread-summed ms: "
                "staging copy %.1f, slot waits %.1f, plan build %.1f, run+results %.1f\n",
                (unsigned long long)g_hprof.passes.load(), g_hprof.bytes.load() / 1048576.0,
                (unsigned long long)g_hprof.builds.load(), g_hprof.ns[0] / 1e6,
                g_hprof.ns[1] / 1e6, g_hprof.ns[2] / 1e6, g_hprof.ns[3] / 1e6);
    {
        DeviceGuard g(c->device);
        if (c->stream) (void)hipStreamSynchronize(c->stream);
        for (Lane *L : c->lanes) lane_free(c, L);
        (void)hipFree(c->d_tables);
        (void)hipFree(c->d_aead_key);
        (void)hipFree(c->d_aead_blobs);
        (void)hipFree(c->d_aead_units);
        (void)hipFree(c->d_aead_unit0);
        (void)hipFree(c->d_aead_partials);
        (void)hipFree(c->d_aead_status);
        (void)hipFree(c->d_aead_stage);
        (void)hipHostFree(c->h_aead_up);
        if (c->aead_done) (void)hipEventDestroy(c->aead_done);
        if (c->ev_null_in) (void)hipEventDestroy(c->ev_null_in);
        if (c->ev_null_out) (void)hipEventDestroy(c->ev_null_out);
        for (uint8_t *t : c->tail_all) (void)hipFree(t);
        (void)hipFree(c->d_zstd_tabs);
        (void)hipFree(c->d_zstd_blobs);
        (void)hipFree(c->d_zstd_blks);
        (void)hipFree(c->d_zstd_res);
        (void)hipFree(c->d_zstd_bpos);
        (void)hipFree(c->d_zstd_lens);
        (void)hipFree(c->d_zstd_queue);
        (void)hipFree(c->d_zstd_seq);
        (void)hipFree(c->d_zstd_slots);
        (void)hipFree(c->d_zstd_far);
        (void)hipFree(c->d_zck_refs);
        (void)hipFree(c->d_zck_order);
        (void)hipFree(c->d_zck_status);
        (void)hipFree(c->d_zck_scratch);
        (void)hipFree(c->d_zck_blk0);
        (void)hipFree(c->d_zck_blks);
        (void)hipFree(c->d_copy_units);
        if (c->stream) (void)hipStreamDestroy(c->stream);
    }
    delete c;
}

uint64_t rcdc_max_cuts(const rcdc_ctx *c, uint64_t n) { return c ? n / c->min + 1 : 0; }

rcdc_status rcdc_chunk_batch(rcdc_ctx *ctx, const rcdc_buf *bufs, uint32_t n, uint64_t *cuts,
                             uint64_t cuts_cap, uint64_t *cut_counts) {
    if (!valid_ctx(ctx)) return fail(RCDC_ERR_INVALID_INPUT, "ctx is NULL");
    if (n && (!bufs || !cut_counts)) return fail(RCDC_ERR_INVALID_INPUT, "null argument");
    Lane *L = nullptr;
    rcdc_status st = lane_acquire(ctx, &L);
    if (st) return st;
    st = run_host_batch(ctx, L, bufs, n, cuts, cuts_cap, cut_counts);
    lane_release(ctx, L);
    return st;
}

rcdc_status rcdc_plan_create(rcdc_ctx *ctx, const uint64_t *offs, const uint64_t *lens,
                             uint32_t n, uint64_t arena_len, rcdc_plan **out) {
    if (!valid_ctx(ctx) || !out || (n && (!offs || !lens)))
        return fail(RCDC_ERR_INVALID_INPUT, "null argument");
    rcdc_plan *pl = new rcdc_plan();
    rcdc_status st = plan_build(ctx, pl, offs, lens, n, arena_len);
    if (st) {
        plan_free(pl);
        return st;
    }
    *out = pl;
    return RCDC_OK;
}

void rcdc_plan_destroy(rcdc_plan *plan) { plan_free(plan); }

rcdc_status rcdc_plan_run(rcdc_plan *plan, const void *d_arena, void *hip_stream) {
    if (!plan || (!d_arena && plan->arena_len))
        return fail(RCDC_ERR_INVALID_INPUT, "null argument");
    return plan_run(plan, d_arena, (hipStream_t)hip_stream);
}

rcdc_status rcdc_plan_results(rcdc_plan *plan, uint64_t *cuts, uint64_t cuts_cap,
                              uint64_t *cut_counts) {
    if (!plan || (plan->n && !cut_counts)) return fail(RCDC_ERR_INVALID_INPUT, "null argument");
    return plan_results(plan, cuts, cuts_cap, cut_counts);
}

rcdc_status rcdc_plan_device_results(rcdc_plan *plan, uint64_t *d_cuts, uint64_t *d_counts,
                                     const uint64_t **cut_base) {
    if (!plan || !d_cuts || !d_counts || !cut_base)
        return fail(RCDC_ERR_INVALID_INPUT, "null argument");
    *d_cuts = (uint64_t)(uintptr_t)plan->d_cuts;
    *d_counts = (uint64_t)(uintptr_t)plan->d_counts;
    *cut_base = plan->cut_base.data();
    return RCDC_OK;
}

rcdc_status rcdc_plan_window(rcdc_plan *plan, uint32_t stream, uint64_t bound, uint32_t k,
                             uint64_t *d_out, void *hip_stream) {
    if (!plan || !d_out) return fail(RCDC_ERR_INVALID_INPUT, "null argument");
    if (stream >= plan->n)
        return fail(RCDC_ERR_INVALID_INPUT, "stream %u of a %u-stream plan", stream, plan->n);
    if (!plan->ran) return fail(RCDC_ERR_INVALID_INPUT, "plan has not been run");
    if (((uintptr_t)d_out & 7u) != 0) return fail(RCDC_ERR_INVALID_INPUT, "d_out not 8-B aligned");
    rcdc_ctx *ctx = plan->ctx;
    DeviceGuard g(ctx->device);
    hipStream_t st;
    if (rcdc_status ns = null_enter(ctx, hip_stream, &st)) return ns;
    // a pipelined run ends on the plan's chain stream: order after it
    if (plan->pipelined) HIP_TRY(hipStreamWaitEvent(st, plan->done, 0));
    HIP_TRY(launch_window(plan->d_cuts, plan->d_counts, stream, plan->cut_base[stream], bound, k,
                          d_out, st));
    return null_leave(ctx, hip_stream, st);
}

rcdc_status rcdc_plan_set_pipeline(rcdc_plan *plan, int enable) {
    if (!plan) return fail(RCDC_ERR_INVALID_INPUT, "null argument");
    if (!enable) {
        if (plan->pipelined && plan->ran) {
            DeviceGuard g(plan->ctx->device);
            HIP_TRY(hipEventSynchronize(plan->done));
        }
        plan->pipelined = false;
        plan->pp = 0;
        return RCDC_OK;
    }
    if (enable == 2) plan->flush_next = true;  // (set up below on first use)
    if (plan->pipelined) return RCDC_OK;
    DeviceGuard g(plan->ctx->device);
    if (plan->ran) HIP_TRY(hipEventSynchronize(plan->done));  // set 0's buffers are free
    rcdc_status st;
    if ((st = ensure_dev(&plan->d_sums2, &plan->cap_sums2, std::max<uint64_t>(plan->cap_sums, 1))))
        return st;
    if ((st = ensure_dev(&plan->d_masks2, &plan->cap_masks2, std::max<uint64_t>(plan->cap_masks, 1))))
        return st;
    if (const uint64_t nw = plan->wunits.size()) {
        if ((st = ensure_dev(&plan->d_wpiece2, &plan->cap_wpiece2, plan->nwpiece_cuts))) return st;
        if ((st = ensure_dev(&plan->d_pstatus2, &plan->cap_pstatus2, nw))) return st;
        if ((st = ensure_dev(&plan->d_wstate2, &plan->cap_wstate2, 2 * nw))) return st;
        HIP_TRY(hipMemset(plan->d_wstate2, 0, 2 * nw * 8));
        if ((st = ensure_dev(&plan->d_bres2, &plan->cap_bres2, nw))) return st;
        if ((st = ensure_dev(&plan->d_ctr2, &plan->cap_ctr2, 4))) return st;
        HIP_TRY(hipMemset(plan->d_ctr2, 0, 16));
        plan->wqbase[1] = 0;
        if ((st = ensure_dev(&plan->d_fixlist2, &plan->cap_fixlist2, nw))) return st;
        if ((st = ensure_dev(&plan->d_fixcuts2, &plan->cap_fixcuts2, nw * plan->wprm.fix_cap)))
            return st;
        if ((st = ensure_dev(&plan->d_fixres2, &plan->cap_fixres2, nw))) return st;
        if ((st = ensure_dev(&plan->d_wstats2, &plan->cap_wstats2, kWalkStats))) return st;
        if (plan->wprm.order_out &&
            (st = ensure_dev(&plan->d_worder2, &plan->cap_worder2, nw + (nw + 3) / 4)))
            return st;
    }
    const int prio_mode = getenv("RCDC_PIPE_PRIO") ? atoi(getenv("RCDC_PIPE_PRIO")) : 0;
    int prio_lo = 0, prio_hi = 0;
    if (prio_mode) {
        HIP_TRY(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
        if (getenv("RCDC_PIPE_PRIO_PRINT"))
            fprintf(stderr, "rcdc: stream priorities %d..%d\n", prio_lo, prio_hi);
    }
    if (!plan->rstream) {
        if (prio_mode >= 3)  // the chain kernels first on freed CUs
            HIP_TRY(hipStreamCreateWithPriority(&plan->rstream, hipStreamNonBlocking, prio_hi));
        else
            HIP_TRY(hipStreamCreateWithFlags(&plan->rstream, hipStreamNonBlocking));
    }
    for (int k = 0; k < 2; k++) {
        if (!plan->hstream[k]) {
            // RCDC_PIPE_PRIO (experiments): the two hashing streams at different
            // priorities, so they sit on different hardware queues and run k + 1's
            // walk can start on the CUs run k's walk frees in its tail
            if (prio_mode == 1 || prio_mode == 2)
                HIP_TRY(hipStreamCreateWithPriority(&plan->hstream[k], hipStreamNonBlocking,
                                                    k ? (prio_mode == 2 ? prio_lo : prio_hi) : prio_lo));
            else if (prio_mode == 4)  // three levels: chain high, the hashing streams low / middle
                HIP_TRY(hipStreamCreateWithPriority(&plan->hstream[k], hipStreamNonBlocking,
                                                    k ? (prio_lo + prio_hi) / 2 : prio_lo));
            else
                HIP_TRY(hipStreamCreateWithFlags(&plan->hstream[k], hipStreamNonBlocking));
        }
        if (!plan->ev_in[k])
            HIP_TRY(hipEventCreateWithFlags(&plan->ev_in[k], hipEventDisableTiming));
        if (!plan->ev_scan[k])
            HIP_TRY(hipEventCreateWithFlags(&plan->ev_scan[k], hipEventDisableTiming));
        if (!plan->ev_res[k])
            HIP_TRY(hipEventCreateWithFlags(&plan->ev_res[k], hipEventDisableTiming));
        plan->res_pending[k] = false;
    }
    plan->pp = 0;
    if (const char *e = getenv("RCDC_CHK_BLOCKS")) plan->chk_blocks_pipe = (uint32_t)std::max(atoi(e), 1);
    if (const char *e = getenv("RCDC_CHAIN_BLOCKS")) plan->fix_blocks_pipe = (uint32_t)std::max(atoi(e), 1);
    plan->pipelined = true;
    return RCDC_OK;
}

rcdc_status rcdc_plan_get_info(const rcdc_plan *plan, rcdc_plan_info *info) {
    if (!plan || !info) return fail(RCDC_ERR_INVALID_INPUT, "null argument");
    info->scanned_bytes = plan->scanned;
    info->segments = plan->nseg;
    info->segment_bytes = plan->seg_bytes;
    info->work_items = (uint32_t)plan->items.size();
    info->scan_blocks = plan->blocks;
    info->walk_pieces = (uint32_t)plan->wunits.size();
    info->walk_seg_bytes = plan->wprm.seg_bytes;
    info->pad = 0;
    return RCDC_OK;
}

rcdc_status rcdc_plan_walk_stats(rcdc_plan *plan, uint64_t *stats, uint64_t *trace,
                                 uint64_t trace_cap) {
    if (!plan || !stats) return fail(RCDC_ERR_INVALID_INPUT, "null argument");
    memset(stats, 0, RCDC_WALK_STATS * sizeof(uint64_t));
    if (plan->wunits.empty()) return RCDC_OK;
    if (!plan->ran) return fail(RCDC_ERR_INVALID_INPUT, "plan has not been run");
    DeviceGuard g(plan->ctx->device);
    HIP_TRY(hipEventSynchronize(plan->done));
    static_assert(RCDC_WALK_STATS == kWalkStats, "stats slots");
    HIP_TRY(hipMemcpy(stats, plan->last_wslot == 4 ? plan->d_wstats2
                                                    : plan->d_wstats + plan->last_wslot * kWalkStats,
                      kWalkStats * 8,
                      hipMemcpyDeviceToHost));
    const uint64_t nw = 2 * plan->wunits.size() * kTraceWords;  // walk rows, then check rows
    if (trace && trace_cap && plan->wprm.trace)
        HIP_TRY(hipMemcpy(trace, plan->d_wtrace, std::min(trace_cap, nw) * 8,
                          hipMemcpyDeviceToHost));
    return RCDC_OK;
}

rcdc_status rcdc_plan_set_timing(rcdc_plan *plan, int enable) {
    if (!plan) return fail(RCDC_ERR_INVALID_INPUT, "null argument");
    plan->timing = enable > 0;
    if (enable > 0) {
        plan->truns = 0;
        plan->tcalls = 0;
        plan->tperiod = (uint32_t)enable;
    }
    return RCDC_OK;
}

rcdc_status rcdc_plan_kernel_times(rcdc_plan *plan, uint64_t *runs, double *scan_ms,
                                   double *resolve_ms) {
    if (!plan || !runs || !scan_ms || !resolve_ms)
        return fail(RCDC_ERR_INVALID_INPUT, "null argument");
    DeviceGuard g(plan->ctx->device);
    double s = 0, r = 0;
    for (uint64_t i = 0; i < plan->truns; i++) {
        hipEvent_t *ev = &plan->tev[3 * i];
        HIP_TRY(hipEventSynchronize(ev[2]));
        float a = 0, b = 0;
        HIP_TRY(hipEventElapsedTime(&a, ev[0], ev[1]));
        HIP_TRY(hipEventElapsedTime(&b, ev[1], ev[2]));
        s += a;
        r += b;
    }
    *runs = plan->truns;
    *scan_ms = s;
    *resolve_ms = r;
    return RCDC_OK;
}

uint64_t rcdc_fixed_cuts(uint64_t n, uint64_t size, uint64_t *cuts, uint64_t cap) {
    // fixed_size.rs:41-70: `take(size).read_to_end`, short final chunk, none if empty
    if (size == 0) return 0;
    uint64_t k = 0;
    for (uint64_t s = 0; s < n;) {
        const uint64_t e = (n - s < size) ? n : s + size;
        if (k < cap) cuts[k] = e;
        k++;
        s = e;
    }
    return k;
}

rcdc_status rcdc_host_alloc(uint64_t bytes, void **out) {
    if (!out) return fail(RCDC_ERR_INVALID_INPUT, "null argument");
    *out = nullptr;
    HIP_TRY(hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault));
    return RCDC_OK;
}

void rcdc_host_free(void *p) {
    if (p) (void)hipHostFree(p);
}

// ---- SHA-256 blob ids (crypto/hasher.rs:17-19, file_archiver.rs:151) -----

rcdc_status rcdc_sha256_host(const void *const *ptrs, const uint64_t *lens, uint32_t n,
                             uint8_t *digests) {
    if (n && (!ptrs || !lens || !digests)) return fail(RCDC_ERR_INVALID_INPUT, "null argument");
    for (uint32_t i = 0; i < n; i++)
        if (!ptrs[i] && lens[i]) return fail(RCDC_ERR_INVALID_INPUT, "null buffer");
    if (!host_sha_supported()) return fail(RCDC_ERR_UNSUPPORTED, "CPU without AVX-512F/BW");
    host_sha256_many(reinterpret_cast<const uint8_t *const *>(ptrs), lens, n, digests);
    return RCDC_OK;
}

rcdc_status rcdc_sha256_chunks(rcdc_ctx *ctx, const void *d_arena, const rcdc_chunk_ref *d_refs,
                               uint32_t n, uint8_t *d_digests, void *hip_stream) {
    if (!valid_ctx(ctx) || (n && (!d_arena || !d_refs || !d_digests)))
        return fail(RCDC_ERR_INVALID_INPUT, "null argument");
    if (((uintptr_t)d_digests & 3) || ((uintptr_t)d_refs & 15))
        return fail(RCDC_ERR_INVALID_INPUT, "digests must be 4-byte and refs 16-byte aligned");
    DeviceGuard g(ctx->device);
    hipStream_t st;
    if (rcdc_status ns = null_enter(ctx, hip_stream, &st)) return ns;
    HIP_TRY(launch_sha256_list((const uint8_t *)d_arena, (const ulonglong2 *)d_refs, n,
                               (uint32_t *)d_digests, st));
    return null_leave(ctx, hip_stream, st);
}

rcdc_status rcdc_plan_hash(rcdc_plan *plan, const void *d_arena, void *hip_stream) {
    if (!plan || (!d_arena && plan->arena_len)) return fail(RCDC_ERR_INVALID_INPUT, "null argument");
    if (!plan->ran) return fail(RCDC_ERR_INVALID_INPUT, "plan has not been run");
    if (d_arena != plan->last_arena)
        return fail(RCDC_ERR_INVALID_INPUT, "arena differs from the last rcdc_plan_run");
    DeviceGuard g(plan->ctx->device);
    hipStream_t st;
    rcdc_status rs;
    if ((rs = null_enter(plan->ctx, hip_stream, &st))) return rs;
    if ((rs = ensure_dev(&plan->d_dig, &plan->cap_dig, plan->ncuts * 8))) return rs;
    if ((rs = ensure_dev(&plan->d_shaw, &plan->cap_shaw, 256))) return rs;
    if ((rs = ensure_dev(&plan->d_order, &plan->cap_order, plan->ncuts))) return rs;
    if (st != plan->last_stream) HIP_TRY(hipStreamWaitEvent(st, plan->done, 0));
    HIP_TRY(launch_sha256_plan((const uint8_t *)d_arena, plan->d_sds, plan->n, plan->d_cuts,
                               plan->d_counts, plan->ncuts, plan->ctx->max, plan->d_shaw,
                               plan->d_order, plan->d_dig, st));
    HIP_TRY(hipEventRecord(plan->done, st));
    plan->hashed = true;
    return null_leave(plan->ctx, hip_stream, st);
}

rcdc_status rcdc_plan_hash_many(rcdc_plan *const *plans, uint32_t n,
                                const void *const *d_arenas, void *hip_stream) {
    if (n == 0) return RCDC_OK;
    if (!plans || !d_arenas) return fail(RCDC_ERR_INVALID_INPUT, "null argument");
    if (n > 8) return fail(RCDC_ERR_INVALID_INPUT, "at most 8 plans per call, got %u", n);
    rcdc_ctx *ctx = plans[0] ? plans[0]->ctx : nullptr;
    for (uint32_t j = 0; j < n; j++) {
        rcdc_plan *pl = plans[j];
        if (!pl || (!d_arenas[j] && pl->arena_len)) return fail(RCDC_ERR_INVALID_INPUT, "null argument");
        if (!pl->ran) return fail(RCDC_ERR_INVALID_INPUT, "plan %u has not been run", j);
        if (d_arenas[j] != pl->last_arena)
            return fail(RCDC_ERR_INVALID_INPUT, "arena %u differs from its last rcdc_plan_run", j);
        if (pl->ctx != ctx) return fail(RCDC_ERR_INVALID_INPUT, "plans of different contexts");
        for (uint32_t i = 0; i < j; i++)
            if (plans[i] == pl) return fail(RCDC_ERR_INVALID_INPUT, "plan %u repeated", j);
    }
    DeviceGuard g(ctx->device);
    hipStream_t st;
    if (rcdc_status ns = null_enter(ctx, hip_stream, &st)) return ns;
    const uint8_t *ar[8];
    const StreamDesc *sd[8];
    uint32_t ns[8];
    const uint64_t *cu[8], *co[8];
    uint64_t nsl[8];
    uint32_t *bw[8], *od[8], *dg[8];
    for (uint32_t j = 0; j < n; j++) {
        rcdc_plan *pl = plans[j];
        rcdc_status rs;
        if ((rs = ensure_dev(&pl->d_dig, &pl->cap_dig, pl->ncuts * 8))) return rs;
        if ((rs = ensure_dev(&pl->d_shaw, &pl->cap_shaw, 256))) return rs;
        if ((rs = ensure_dev(&pl->d_order, &pl->cap_order, pl->ncuts))) return rs;
        if (st != pl->last_stream) HIP_TRY(hipStreamWaitEvent(st, pl->done, 0));
        ar[j] = (const uint8_t *)d_arenas[j];
        sd[j] = pl->d_sds;
        ns[j] = pl->n;
        cu[j] = pl->d_cuts;
        co[j] = pl->d_counts;
        nsl[j] = pl->ncuts;
        bw[j] = pl->d_shaw;
        od[j] = pl->d_order;
        dg[j] = pl->d_dig;
    }
    HIP_TRY(launch_sha256_multi(n, ar, sd, ns, cu, co, nsl, ctx->max, bw, od, dg, st));
    for (uint32_t j = 0; j < n; j++) {
        HIP_TRY(hipEventRecord(plans[j]->done, st));
        plans[j]->hashed = true;
    }
    return null_leave(ctx, hip_stream, st);
}

rcdc_status rcdc_plan_finish(rcdc_plan *plan) {
    if (!plan) return fail(RCDC_ERR_INVALID_INPUT, "null argument");
    return plan_finish(plan);
}

rcdc_status rcdc_plan_digests(rcdc_plan *plan, uint8_t *digests, uint64_t cap_chunks,
                              uint64_t *cut_counts) {
    if (!plan || (plan->n && !cut_counts)) return fail(RCDC_ERR_INVALID_INPUT, "null argument");
    if (!plan->hashed) return fail(RCDC_ERR_INVALID_INPUT, "rcdc_plan_hash has not been run");
    rcdc_status rs = plan_finish(plan);
    if (rs) return rs;
    DeviceGuard g(plan->ctx->device);
    HIP_TRY(hipEventSynchronize(plan->done));  // the hash may follow the finish
    const std::vector<uint64_t> &cnt = plan->fin_counts;
    uint64_t total = 0;
    for (uint32_t i = 0; i < plan->n; i++) {
        cut_counts[i] = cnt[i];
        total += cnt[i];
    }
    if (total > cap_chunks)
        return fail(RCDC_ERR_CAPACITY, "need %llu digest slots, have %llu",
                    (unsigned long long)total, (unsigned long long)cap_chunks);
    std::vector<uint8_t> all(plan->ncuts * 32);
    if (plan->ncuts)
        HIP_TRY(hipMemcpy(all.data(), plan->d_dig, all.size(), hipMemcpyDeviceToHost));
    uint64_t o = 0;
    for (uint32_t i = 0; i < plan->n; i++) {
        memcpy(digests + o * 32, all.data() + plan->cut_base[i] * 32, cnt[i] * 32);
        o += cnt[i];
    }
    return RCDC_OK;
}

rcdc_status rcdc_plan_device_digests(rcdc_plan *plan, uint64_t *d_digests) {
    if (!plan || !d_digests) return fail(RCDC_ERR_INVALID_INPUT, "null argument");
    if (!plan->hashed) return fail(RCDC_ERR_INVALID_INPUT, "rcdc_plan_hash has not been run");
    *d_digests = (uint64_t)(uintptr_t)plan->d_dig;
    return RCDC_OK;
}

// ---- blob encryption (crypto/aespoly1305.rs:88-135 over HBM) ---------------

}  // extern "C"

namespace {

// AES S-box from its definition (multiplicative inverse in GF(2^8), then the
// affine map; FIPS-197 5.1.1), and the T-table / key schedules on the host.
void aes_sbox(uint8_t sb[256]) {
    uint8_t p = 1, q = 1;
    do {
        p = (uint8_t)(p ^ (p << 1) ^ ((p & 0x80) ? 0x1b : 0));  // p * 3
        q ^= (uint8_t)(q << 1);                                  // q / 3
        q ^= (uint8_t)(q << 2);
        q ^= (uint8_t)(q << 4);
        if (q & 0x80) q ^= 0x09;
        const uint8_t x = (uint8_t)(q ^ (uint8_t)((q << 1) | (q >> 7)) ^
                                    (uint8_t)((q << 2) | (q >> 6)) ^
                                    (uint8_t)((q << 3) | (q >> 5)) ^ (uint8_t)((q << 4) | (q >> 4)));
        sb[p] = x ^ 0x63;
    } while (p != 1);
    sb[0] = 0x63;
}

void aes_expand_host(const uint8_t *key, int nk, const uint8_t sb[256], uint32_t *rk) {
    const int nr = nk + 6;
    uint8_t rcon = 1;
    for (int i = 0; i < nk; i++)
        rk[i] = (uint32_t)key[4 * i] << 24 | (uint32_t)key[4 * i + 1] << 16 |
                (uint32_t)key[4 * i + 2] << 8 | key[4 * i + 3];
    auto sub = [&](uint32_t t) {
        return (uint32_t)sb[t >> 24] << 24 | (uint32_t)sb[(t >> 16) & 255] << 16 |
               (uint32_t)sb[(t >> 8) & 255] << 8 | sb[t & 255];
    };
    for (int i = nk; i < 4 * (nr + 1); i++) {
        uint32_t t = rk[i - 1];
        if (i % nk == 0) {
            t = sub((t << 8) | (t >> 24)) ^ (uint32_t)rcon << 24;
            rcon = (uint8_t)((rcon << 1) ^ ((rcon & 0x80) ? 0x1b : 0));
        } else if (nk > 6 && i % nk == 4) {
            t = sub(t);
        }
        rk[i] = rk[i - nk] ^ t;
    }
}

// 2^130 - 5 arithmetic in 26-bit limbs (the device pmul, on the host)
void p26_mul(const uint32_t a[5], const uint32_t b[5], uint32_t r[5]) {
    const uint64_t b0 = b[0], b1 = b[1], b2 = b[2], b3 = b[3], b4 = b[4];
    const uint64_t s1 = b1 * 5, s2 = b2 * 5, s3 = b3 * 5, s4 = b4 * 5;
    const uint64_t a0 = a[0], a1 = a[1], a2 = a[2], a3 = a[3], a4 = a[4];
    uint64_t d0 = a0 * b0 + a1 * s4 + a2 * s3 + a3 * s2 + a4 * s1;
    uint64_t d1 = a0 * b1 + a1 * b0 + a2 * s4 + a3 * s3 + a4 * s2;
    uint64_t d2 = a0 * b2 + a1 * b1 + a2 * b0 + a3 * s4 + a4 * s3;
    uint64_t d3 = a0 * b3 + a1 * b2 + a2 * b1 + a3 * b0 + a4 * s4;
    uint64_t d4 = a0 * b4 + a1 * b3 + a2 * b2 + a3 * b1 + a4 * b0;
    d1 += d0 >> 26; d2 += d1 >> 26; d3 += d2 >> 26; d4 += d3 >> 26;
    uint64_t h0 = (d0 & 0x3ffffff) + (d4 >> 26) * 5;
    r[1] = (uint32_t)((d1 & 0x3ffffff) + (h0 >> 26));
    r[0] = (uint32_t)(h0 & 0x3ffffff);
    r[2] = (uint32_t)(d2 & 0x3ffffff);
    r[3] = (uint32_t)(d3 & 0x3ffffff);
    r[4] = (uint32_t)(d4 & 0x3ffffff);
    // fully normalise (r[1] may carry)
    const uint32_t c = r[1] >> 26;
    r[1] &= 0x3ffffff;
    r[2] += c;
}

void aead_key_material(const uint8_t key[64], AeadKeyDev *K) {
    uint8_t sb[256];
    aes_sbox(sb);
    for (int x = 0; x < 256; x++) {
        const uint8_t s1 = sb[x], s2 = (uint8_t)((s1 << 1) ^ ((s1 & 0x80) ? 0x1b : 0));
        const uint8_t s3 = s2 ^ s1;
        K->te[x] = (uint32_t)s2 << 24 | (uint32_t)s1 << 16 | (uint32_t)s1 << 8 | s3;
    }
    aes_expand_host(key, 8, sb, K->rk256);
    aes_expand_host(key + 32, 4, sb, K->rk128);
    uint8_t rb[16];
    memcpy(rb, key + 48, 16);
    rb[3] &= 15; rb[7] &= 15; rb[11] &= 15; rb[15] &= 15;
    rb[4] &= 252; rb[8] &= 252; rb[12] &= 252;
    uint64_t t0 = 0, t1 = 0;
    for (int i = 7; i >= 0; i--) {
        t0 = t0 << 8 | rb[i];
        t1 = t1 << 8 | rb[8 + i];
    }
    const uint32_t r[5] = {(uint32_t)(t0 & 0x3ffffff), (uint32_t)((t0 >> 26) & 0x3ffffff),
                           (uint32_t)(((t0 >> 52) | (t1 << 12)) & 0x3ffffff),
                           (uint32_t)((t1 >> 14) & 0x3ffffff), (uint32_t)((t1 >> 40) & 0x3ffffff)};
    const uint32_t one[5] = {1, 0, 0, 0, 0};
    memcpy(K->rpow[0], one, sizeof one);
    for (int i = 1; i <= 64; i++) p26_mul(K->rpow[i - 1], r, K->rpow[i]);
    memcpy(K->r2j[0], r, sizeof r);
    for (int j = 1; j < 32; j++) p26_mul(K->r2j[j - 1], K->r2j[j - 1], K->r2j[j]);
}

// A list of blobs over one input base, cut into units of kAeadUnitBlocks.
struct AeadBatch {
    const uint8_t *in = nullptr;
    std::vector<AeadBlob> blobs;
    std::vector<AeadUnit> units;
    std::vector<uint32_t> unit0;  // per blob + 1 (closed by aead_launch)
};

rcdc_status aead_add(AeadBatch &B, const AeadBlob &b, uint32_t caller_index) {
    const uint64_t nb = (b.len + 15) / 16;
    if (nb >= (1ull << 32)) return fail(RCDC_ERR_UNSUPPORTED, "blob %u too large", caller_index);
    const uint32_t bi = (uint32_t)B.blobs.size();
    B.unit0.push_back((uint32_t)B.units.size());
    B.blobs.push_back(b);
    for (uint64_t b0 = 0; b0 < nb; b0 += kAeadUnitBlocks)
        B.units.push_back({bi, (uint32_t)b0, (uint32_t)std::min<uint64_t>(nb, b0 + kAeadUnitBlocks), 0});
    return RCDC_OK;
}

// Launch the batches (each its own input base) on one context scratch.
// `staging` (optional) is copied to the scratch input buffer first and a
// batch whose `in` is nullptr reads from it.  open: status per blob of the
// batches in order (synchronous).  Calls on one context take turns.
rcdc_status aead_launch(rcdc_ctx *ctx, bool open, const uint8_t key[64], std::vector<AeadBatch> &bt,
                        uint8_t *out, hipStream_t st, const std::vector<uint8_t> *staging,
                        std::vector<uint32_t> *status) {
    std::lock_guard<std::mutex> lk(ctx->aead_mu);
    DeviceGuard g(ctx->device);
    // (the last call's work is done: every call ends synchronised)
    if (!ctx->aead_done) HIP_TRY(hipEventCreateWithFlags(&ctx->aead_done, hipEventDisableTiming));
    rcdc_status rs;
    if ((rs = ensure_dev(&ctx->d_aead_key, &ctx->cap_aead_key, 1))) return rs;
    if (!ctx->aead_key_set || memcmp(ctx->aead_key, key, 64) != 0) {
        AeadKeyDev K;
        aead_key_material(key, &K);
        HIP_TRY(hipMemcpy(ctx->d_aead_key, &K, sizeof K, hipMemcpyHostToDevice));
        memcpy(ctx->aead_key, key, 64);
        ctx->aead_key_set = true;
    }
    uint64_t nb = 0, nu = 0;
    for (AeadBatch &B : bt) {
        B.unit0.push_back((uint32_t)B.units.size());
        nb += B.blobs.size();
        nu += B.units.size();
    }
    if ((rs = ensure_dev(&ctx->d_aead_blobs, &ctx->cap_aead_blobs, nb))) return rs;
    if ((rs = ensure_dev(&ctx->d_aead_units, &ctx->cap_aead_units, nu))) return rs;
    if ((rs = ensure_dev(&ctx->d_aead_unit0, &ctx->cap_aead_unit0, nb + bt.size()))) return rs;
    if ((rs = ensure_dev(&ctx->d_aead_partials, &ctx->cap_aead_partials, nu * 5))) return rs;
    if ((rs = ensure_dev(&ctx->d_aead_status, &ctx->cap_aead_status, nb))) return rs;
    // the call's uploads go async on st from one page-locked buffer (free
    // again: the last call's work is done, aead_done above).  Synchronous
    // copies from pageable memory queued behind other streams' multi-GiB
    // copies on the DMA engine (the ingest engine's batches) and stalled
    // the calling thread for up to a whole copy.
    auto r16 = [](uint64_t x) { return (x + 15) & ~15ull; };
    uint64_t up = staging ? r16(staging->size()) : 0;
    for (AeadBatch &B : bt)
        up += r16(B.blobs.size() * sizeof(AeadBlob)) + r16(B.unit0.size() * 4) +
              r16(B.units.size() * sizeof(AeadUnit));
    if (up > ctx->cap_aead_up) {
        if (ctx->h_aead_up) HIP_TRY(hipHostFree(ctx->h_aead_up));
        ctx->h_aead_up = nullptr;
        ctx->cap_aead_up = 0;
        const uint64_t c = up + up / 2 + 4096;
        HIP_TRY(hipHostMalloc((void **)&ctx->h_aead_up, c, hipHostMallocDefault));
        ctx->cap_aead_up = c;
    }
    uint64_t hp = 0;
    auto upload = [&](void *dst, const void *src, uint64_t n) -> hipError_t {
        if (!n) return hipSuccess;
        memcpy(ctx->h_aead_up + hp, src, n);
        const hipError_t e = hipMemcpyAsync(dst, ctx->h_aead_up + hp, n, hipMemcpyHostToDevice, st);
        hp += r16(n);
        return e;
    };
    if (staging && !staging->empty()) {
        if ((rs = ensure_dev(&ctx->d_aead_stage, &ctx->cap_aead_stage, staging->size() + 16)))
            return rs;
        HIP_TRY(upload(ctx->d_aead_stage, staging->data(), staging->size()));
    }
    uint64_t ob = 0, ou = 0, o0 = 0;
    for (AeadBatch &B : bt) {
        const uint32_t m = (uint32_t)B.blobs.size(), u = (uint32_t)B.units.size();
        if (m) {
            HIP_TRY(upload(ctx->d_aead_blobs + ob, B.blobs.data(), m * sizeof(AeadBlob)));
            HIP_TRY(upload(ctx->d_aead_unit0 + o0, B.unit0.data(), (m + 1) * 4));
        }
        if (u) HIP_TRY(upload(ctx->d_aead_units + ou, B.units.data(), u * sizeof(AeadUnit)));
        const uint8_t *in = B.in ? B.in : ctx->d_aead_stage;
        HIP_TRY(launch_aead(open, in, out, ctx->d_aead_blobs + ob, m, ctx->d_aead_units + ou, u,
                            ctx->d_aead_unit0 + o0, ctx->d_aead_key, ctx->d_aead_partials + ou * 5,
                            ctx->d_aead_status + ob, (uint32_t)std::max(ctx->num_cus, 1), st));
        ob += m;
        ou += u;
        o0 += m + 1;
    }
    // The call returns once its work is done: the context's scratch is then
    // free for the next call with no event kept across calls.  (An event
    // recorded on the caller's stream and synchronised in the next call
    // failed once that stream had been destroyed in between, r5g; one
    // recorded on the context's stream waited behind whatever long kernel
    // shared that stream's hardware queue, r5l.)
    HIP_TRY(hipEventRecord(ctx->aead_done, st));
    HIP_TRY(poll_event(ctx->aead_done));
    if (open && status) {
        HIP_TRY(poll_event(ctx->aead_done));
        status->assign(nb, 0);
        if (nb) {  // on st (see plan_finish: not the legacy default stream)
            HIP_TRY(hipMemcpyAsync(status->data(), ctx->d_aead_status, nb * 4, hipMemcpyDeviceToHost, st));
            HIP_TRY(poll_stream(st));
        }
    }
    return RCDC_OK;
}

rcdc_status aead_run(rcdc_ctx *ctx, bool open, const uint8_t key[64], const void *d_in,
                     const rcdc_aead_ref *refs, uint32_t n, void *d_out, uint32_t *status,
                     void *hip_stream) {
    if (!valid_ctx(ctx) || !key || (n && (!refs || !d_in || !d_out)) || (open && n && !status))
        return fail(RCDC_ERR_INVALID_INPUT, "null argument");
    std::vector<AeadBatch> bt(1);
    bt[0].in = (const uint8_t *)d_in;
    std::vector<uint32_t> which;  // device blob -> caller index
    rcdc_status rs;
    for (uint32_t i = 0; i < n; i++) {
        const rcdc_aead_ref &r = refs[i];
        if (open && r.len < 32) {
            // no room for nonce + tag: aespoly1305.rs:89-94 (< 16 bytes) and
            // the AEAD's own length check (16..31) both fail before any MAC
            status[i] = r.len < 16 ? 2u : 1u;
            continue;
        }
        AeadBlob b{};
        b.in_off = r.in_off;
        b.len = open ? r.len - 32 : r.len;
        b.out_off = r.out_off;
        memcpy(b.nonce, r.nonce, 16);  // little-endian words of the nonce bytes
        if ((rs = aead_add(bt[0], b, i))) return rs;
        which.push_back(i);
    }
    std::vector<uint32_t> ds;
    hipStream_t st;
    {
        DeviceGuard g(ctx->device);
        if ((rs = null_enter(ctx, hip_stream, &st))) return rs;
        if ((rs = aead_launch(ctx, open, key, bt, (uint8_t *)d_out, st, nullptr,
                              open ? &ds : nullptr)))
            return rs;
        if ((rs = null_leave(ctx, hip_stream, st))) return rs;
    }
    if (open)
        for (size_t j = 0; j < which.size(); j++) status[which[j]] = ds[j];
    return RCDC_OK;
}

static_assert(sizeof(rcdc_pack_blob) == 72, "rcdc_pack_blob is 72 B");
static_assert(sizeof(rcdc_pack) == 48, "rcdc_pack is 48 B");

// Pack files (blob/packer.rs:615-655, 693-735; repofile/packfile.rs): blobs
// sealed back to back, then the sealed header (one HeaderEntry per blob:
// type, u32 length, [u32 raw length], id) and its u32 length.
// raw (add_raw): the blobs at in_off are sealed already (len = sealed bytes,
// >= 32); they are copied into place and only the headers are sealed.
// Device range copies (units of {src, dst, len, source base address}, at
// most 1 MiB each) into d_out on st.  The unit list lives in the context
// until the copy has run: calls take turns under the AEAD lock.
rcdc_status copy_units_run(rcdc_ctx *ctx, const std::vector<uint64_t> &copies, void *d_out,
                           hipStream_t st) {
    if (copies.empty()) return RCDC_OK;
    std::lock_guard<std::mutex> lk(ctx->aead_mu);
    const uint64_t nu = copies.size() / 4;
    rcdc_status rs;
    if ((rs = ensure_dev(&ctx->d_copy_units, &ctx->cap_copy_units, copies.size()))) return rs;
    HIP_TRY(hipMemcpyAsync(ctx->d_copy_units, copies.data(), copies.size() * 8,
                           hipMemcpyHostToDevice, st));
    HIP_TRY(launch_copy_ranges((uint8_t *)d_out, ctx->d_copy_units, (uint32_t)nu,
                               (uint32_t)std::max(ctx->num_cus, 1), st));
    // the host vector dies with the caller's call
    HIP_TRY(poll_stream(st));
    return RCDC_OK;
}

void push_copy(std::vector<uint64_t> &copies, const void *src_base, uint64_t src, uint64_t dst,
               uint64_t len) {
    for (uint64_t c = 0; c < len; c += 1u << 20) {
        copies.push_back(src + c);
        copies.push_back(dst + c);
        copies.push_back(std::min<uint64_t>(1u << 20, len - c));
        copies.push_back((uint64_t)(uintptr_t)src_base);
    }
}

// srcs (raw only, n_src > 0): blob i's bytes are at srcs[blobs[i].pad] +
// in_off (rcdc_pack_build_raw_multi); otherwise at d_in + in_off.
rcdc_status pack_build(rcdc_ctx *ctx, const uint8_t key[64], const void *d_in,
                       const rcdc_pack_blob *blobs, uint32_t nblobs, rcdc_pack *packs,
                       uint32_t npacks, void *d_out, uint64_t out_len, uint32_t *blob_offsets,
                       void *hip_stream, bool raw = false, const void *const *srcs = nullptr,
                       uint32_t n_src = 0) {
    if (n_src) {
        if (!srcs) return fail(RCDC_ERR_INVALID_INPUT, "null argument");
        for (uint32_t j = 0; j < n_src; j++)
            if (!srcs[j]) return fail(RCDC_ERR_INVALID_INPUT, "source %u is null", j);
        d_in = srcs[0];
    }
    if (!valid_ctx(ctx) || !key || (npacks && (!packs || !d_out)) || (nblobs && (!blobs || !d_in)))
        return fail(RCDC_ERR_INVALID_INPUT, "null argument");
    std::vector<AeadBatch> bt(2);
    bt[0].in = (const uint8_t *)d_in;
    bt[1].in = nullptr;  // headers: from the staging buffer
    std::vector<uint8_t> hdr;
    std::vector<uint64_t> copies;  // raw: (src, dst, len, 0) per unit of <= 1 MiB
    rcdc_status rs;
    for (uint32_t p = 0; p < npacks; p++) {
        rcdc_pack &P = packs[p];
        if (P.nblobs == 0 || (uint64_t)P.blob0 + P.nblobs > nblobs)
            return fail(RCDC_ERR_INVALID_INPUT, "pack %u: blobs [%u, +%u) of %u", p, P.blob0,
                        P.nblobs, nblobs);
        uint64_t off = 0;
        const size_t h0 = hdr.size();
        for (uint32_t i = P.blob0; i < P.blob0 + P.nblobs; i++) {
            const rcdc_pack_blob &b = blobs[i];
            if (b.type > 1) return fail(RCDC_ERR_INVALID_INPUT, "blob %u: type %u", i, b.type);
            if (raw && b.len < 32)
                return fail(RCDC_ERR_INVALID_INPUT, "blob %u: %u sealed bytes (< 32)", i, b.len);
            if (!raw && b.len > 0xFFFFFFFFu - 32u)
                return fail(RCDC_ERR_UNSUPPORTED, "blob %u: %u bytes", i, b.len);
            const uint32_t sealed = raw ? b.len : b.len + 32u;
            if (blob_offsets) blob_offsets[i] = (uint32_t)off;
            if (raw) {
                if (n_src && b.pad >= n_src)
                    return fail(RCDC_ERR_INVALID_INPUT, "blob %u: source %u of %u", i, b.pad, n_src);
                push_copy(copies, n_src ? srcs[b.pad] : d_in, b.in_off, P.out_off + off, sealed);
            } else {
                AeadBlob a{};
                a.in_off = b.in_off;
                a.len = b.len;
                a.out_off = P.out_off + off;
                memcpy(a.nonce, b.nonce, 16);
                if ((rs = aead_add(bt[0], a, i))) return rs;
            }
            // HeaderEntry (packfile.rs:88-124, little-endian)
            hdr.push_back((uint8_t)(b.type + (b.uncompressed_len ? 2u : 0u)));
            for (int j = 0; j < 4; j++) hdr.push_back((uint8_t)(sealed >> (8 * j)));
            if (b.uncompressed_len)
                for (int j = 0; j < 4; j++) hdr.push_back((uint8_t)(b.uncompressed_len >> (8 * j)));
            hdr.insert(hdr.end(), b.id, b.id + 32);
            off += sealed;
        }
        const uint64_t hlen = hdr.size() - h0;
        P.header_len = (uint32_t)(hlen + 32);
        P.size = off + hlen + 32 + 4;
        if (P.size > 0xFFFFFFFFull)  // packer.rs:58 MAX_SIZE; offsets are u32
            return fail(RCDC_ERR_UNSUPPORTED, "pack %u: %llu bytes", p, (unsigned long long)P.size);
        if (P.out_off + P.size > out_len)
            return fail(RCDC_ERR_INVALID_INPUT, "pack %u does not fit the output (%llu + %llu > %llu)",
                        p, (unsigned long long)P.out_off, (unsigned long long)P.size,
                        (unsigned long long)out_len);
        AeadBlob h{};
        h.in_off = h0;
        h.len = hlen;
        h.out_off = P.out_off + off;
        memcpy(h.nonce, P.header_nonce, 16);
        h.flags = kAeadAppendLen;
        if ((rs = aead_add(bt[1], h, p))) return rs;
    }
    hdr.resize(hdr.size() + 4, 0);  // the kernel may read 3 bytes past a blob
    DeviceGuard g(ctx->device);
    hipStream_t st;
    if ((rs = null_enter(ctx, hip_stream, &st))) return rs;
    if ((rs = copy_units_run(ctx, copies, d_out, st))) return rs;
    if ((rs = aead_launch(ctx, false, key, bt, (uint8_t *)d_out, st, &hdr, nullptr))) return rs;
    return null_leave(ctx, hip_stream, st);
}

// ---- blob compression (zstd frames, RFC 8878) --------------------------------

// FSE_buildCTable of a normalized distribution (the format's symbol spread:
// RFC 8878 4.1.1; zstd lib/compress/fse_compress.c): state table sorted by
// symbol, and per symbol {deltaFindState, deltaNbBits}.
void fse_build_ctable(const int16_t *norm, int nsym, int tlog, ZstdFseSym *tt, uint16_t *st) {
    const int size = 1 << tlog, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
    std::vector<int> sym(size), cumul(nsym + 1);
    int high = size - 1;
    for (int u = 1; u <= nsym; u++) {
        if (norm[u - 1] == -1) {
            cumul[u] = cumul[u - 1] + 1;
            sym[high--] = u - 1;
        } else {
            cumul[u] = cumul[u - 1] + norm[u - 1];
        }
    }
    int pos = 0;
    for (int s = 0; s < nsym; s++)
        for (int k = 0; k < norm[s]; k++) {
            sym[pos] = s;
            pos = (pos + step) & mask;
            while (pos > high) pos = (pos + step) & mask;
        }
    for (int u = 0; u < size; u++) st[cumul[sym[u]]++] = (uint16_t)(size + u);
    int total = 0;
    for (int s = 0; s < nsym; s++) {
        const int c = norm[s];
        if (c == -1 || c == 1) {
            tt[s].nbits = ((uint32_t)tlog << 16) - (uint32_t)size;
            tt[s].find = total - 1;
            total++;
        } else if (c > 1) {
            const int mbo = tlog - (31 - __builtin_clz((uint32_t)(c - 1)));
            tt[s].nbits = ((uint32_t)mbo << 16) - ((uint32_t)c << mbo);
            tt[s].find = total - c;
            total += c;
        } else {
            tt[s].nbits = ((uint32_t)(tlog + 1) << 16) - (uint32_t)size;
            tt[s].find = 0;
        }
    }
}

// The predefined distributions and code tables (RFC 8878 3.1.1.3.2.1-2).
const ZstdTables &zstd_tables() {
    static ZstdTables T;
    static std::once_flag once;
    std::call_once(once, [] {
        static const int16_t ll_norm[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                            2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
        static const int16_t ml_norm[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                            1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                            1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
        static const int16_t of_norm[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                            1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
        static const uint32_t ll_base[36] = {0,  1,  2,   3,   4,   5,   6,    7,    8,    9,
                                             10, 11, 12,  13,  14,  15,  16,   18,   20,   22,
                                             24, 28, 32,  40,  48,  64,  128,  256,  512,  1024,
                                             2048, 4096, 8192, 16384, 32768, 65536};
        static const uint8_t ll_bits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1,
                                            1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
        static const uint32_t ml_base[53] = {
            3,  4,  5,  6,  7,  8,  9,  10, 11,  12,  13,  14,   15,   16,   17,   18,   19, 20,
            21, 22, 23, 24, 25, 26, 27, 28, 29,  30,  31,  32,   33,   34,   35,   37,   39, 41,
            43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
        static const uint8_t ml_bits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                            0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1,
                                            2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
        memset(&T, 0, sizeof T);
        fse_build_ctable(ll_norm, 36, 6, T.ll, T.llst);
        fse_build_ctable(ml_norm, 53, 6, T.ml, T.mlst);
        fse_build_ctable(of_norm, 29, 5, T.of, T.ofst);
        for (uint32_t v = 0; v < 64; v++) {
            int c = 0;
            while (c + 1 < 36 && ll_base[c + 1] <= v) c++;
            T.llcode[v] = (uint8_t)c;
        }
        for (uint32_t v = 0; v < 128; v++) {
            int c = 0;
            while (c + 1 < 53 && ml_base[c + 1] - 3 <= v) c++;
            T.mlcode[v] = (uint8_t)c;
        }
        memcpy(T.llbits, ll_bits, sizeof ll_bits);
        memcpy(T.mlbits, ml_bits, sizeof ml_bits);
    });
    return T;
}

uint64_t zstd_blocks(uint64_t len) { return len ? (len + kZstdBlock - 1) / kZstdBlock : 1; }

// Blocks per launch window: bounds the per-block scratch (32768 x 128 KiB);
// windows run back to back on the stream, reusing it.
constexpr uint64_t kZstdWindowBlocks = 32768;

// RCDC_ZSTD_WINDOW_BLOCKS (tests): a smaller window, so a modest batch runs
// the multi-window path (per-window queues, rebased indices, reused slots)
static uint64_t zstd_window_blocks() {
    if (const char *e = getenv("RCDC_ZSTD_WINDOW_BLOCKS")) {
        const long long v = atoll(e);
        if (v > 0) return std::min<uint64_t>((uint64_t)v, kZstdWindowBlocks);
    }
    return kZstdWindowBlocks;
}

rcdc_status zstd_compress(rcdc_ctx *ctx, int level, const void *d_in, const rcdc_zstd_ref *refs,
                          uint32_t n, void *d_out, uint64_t *out_lens, void *hip_stream) {
    if (!valid_ctx(ctx) || (n && (!refs || !d_in || !d_out || !out_lens)))
        return fail(RCDC_ERR_INVALID_INPUT, "null argument");
    // zstd's accepted levels (ZSTD_minCLevel() .. ZSTD_maxCLevel(); decrypt.rs:20-24)
    if (level < -(1 << 17) || level > 22)
        return fail(RCDC_ERR_INVALID_INPUT, "zstd level %d outside [-131072, 22]", level);
    for (uint32_t i = 0; i < n; i++)
        if (refs[i].len > 0xFFFFFFFFull)  // decrypt.rs:479-487: data length must fit u32
            return fail(RCDC_ERR_UNSUPPORTED, "blob %u: %llu bytes", i,
                        (unsigned long long)refs[i].len);
    if (!n) return RCDC_OK;
    // descriptors of every window (block indices relative to the window,
    // blob indices too), uploaded once
    struct Win {
        uint64_t blob0, nblob, blk0, nblk;
    };
    std::vector<ZstdBlob> blobs;
    std::vector<ZstdBlk> blks;
    std::vector<Win> wins;
    uint64_t maxw = 0;
    const uint64_t wblocks = zstd_window_blocks();
    for (uint32_t i = 0; i < n;) {
        Win w{blobs.size(), 0, blks.size(), 0};
        while (i < n) {
            const uint64_t nb = zstd_blocks(refs[i].len);
            if (w.nblk && w.nblk + nb > wblocks) break;
            ZstdBlob B{};
            B.in_off = refs[i].in_off;
            B.out_off = refs[i].out_off;
            B.len = (uint32_t)refs[i].len;
            B.blk0 = (uint32_t)w.nblk;
            B.nblk = (uint32_t)nb;
            for (uint64_t k = 0; k < nb; k++) {
                ZstdBlk b{};
                b.blob = (uint32_t)w.nblob;
                b.start = (uint32_t)(k * kZstdBlock);
                b.len = (uint32_t)std::min<uint64_t>(kZstdBlock, refs[i].len - k * kZstdBlock);
                b.flags = (k == 0 ? 1u : 0u) | (k + 1 == nb ? 2u : 0u);
                blks.push_back(b);
            }
            blobs.push_back(B);
            w.nblk += nb;
            w.nblob++;
            i++;
        }
        maxw = std::max(maxw, w.nblk);
        wins.push_back(w);
    }
    std::lock_guard<std::mutex> lk(ctx->zstd_mu);
    DeviceGuard g(ctx->device);
    hipStream_t st;
    rcdc_status rs;
    if ((rs = null_enter(ctx, hip_stream, &st))) return rs;
    if (!ctx->d_zstd_tabs) {
        if ((rs = ensure_dev(&ctx->d_zstd_tabs, &ctx->cap_zstd_tabs, 1))) return rs;
        HIP_TRY(hipMemcpy(ctx->d_zstd_tabs, &zstd_tables(), sizeof(ZstdTables),
                          hipMemcpyHostToDevice));
    }
    const uint32_t grid = zstd_block_grid((uint32_t)std::max(ctx->num_cus, 1), level);
    // (+ 8 words: the last wave's 16-byte literal loads may pass its region by 20 bytes)
    if ((rs = ensure_dev(&ctx->d_zstd_seq, &ctx->cap_zstd_seq, (uint64_t)grid * kZstdMaxSeq + 8)))
        return rs;
    const uint64_t nbl = blks.size(), nbo = blobs.size();
    if ((rs = ensure_dev(&ctx->d_zstd_blobs, &ctx->cap_zstd_blobs, nbo))) return rs;
    if ((rs = ensure_dev(&ctx->d_zstd_blks, &ctx->cap_zstd_blks, nbl))) return rs;
    if ((rs = ensure_dev(&ctx->d_zstd_res, &ctx->cap_zstd_res, nbl))) return rs;
    if ((rs = ensure_dev(&ctx->d_zstd_bpos, &ctx->cap_zstd_bpos, nbl))) return rs;
    if ((rs = ensure_dev(&ctx->d_zstd_lens, &ctx->cap_zstd_lens, nbo))) return rs;
    if ((rs = ensure_dev(&ctx->d_zstd_slots, &ctx->cap_zstd_slots, maxw * kZstdSlot))) return rs;
    const uint64_t farw = zstd_far_words(level, maxw);
    if (farw && (rs = ensure_dev(&ctx->d_zstd_far, &ctx->cap_zstd_far, farw))) return rs;
    // the block kernel's queue: 8 counters 64 B apart per window
    if ((rs = ensure_dev(&ctx->d_zstd_queue, &ctx->cap_zstd_queue, wins.size() * 128))) return rs;
    HIP_TRY(hipMemsetAsync(ctx->d_zstd_queue, 0, wins.size() * 128 * 4, st));
    HIP_TRY(hipMemcpyAsync(ctx->d_zstd_blobs, blobs.data(), nbo * sizeof(ZstdBlob),
                           hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ctx->d_zstd_blks, blks.data(), nbl * sizeof(ZstdBlk),
                           hipMemcpyHostToDevice, st));
    if (const char *e = getenv("RCDC_ZSTD_DBG"); e && (atoi(e) & 32)) {  // the buffers, to place a fault
        auto rng = [](const char *nm, const void *p, uint64_t bytes) {
            fprintf(stderr, "rcdc zstd buf %-6s [%p, %p) %llu B\n", nm, p, (const void *)((const char *)p + bytes),
                    (unsigned long long)bytes);
        };
        rng("seq", ctx->d_zstd_seq, ctx->cap_zstd_seq * 8);
        rng("slots", ctx->d_zstd_slots, ctx->cap_zstd_slots);
        rng("far", ctx->d_zstd_far, ctx->cap_zstd_far * 4);
        rng("res", ctx->d_zstd_res, ctx->cap_zstd_res * 8);
        rng("bpos", ctx->d_zstd_bpos, ctx->cap_zstd_bpos * 8);
        rng("blobs", ctx->d_zstd_blobs, ctx->cap_zstd_blobs * sizeof(ZstdBlob));
        rng("blks", ctx->d_zstd_blks, ctx->cap_zstd_blks * sizeof(ZstdBlk));
        rng("tabs", ctx->d_zstd_tabs, ctx->cap_zstd_tabs * sizeof(ZstdTables));
        rng("queue", ctx->d_zstd_queue, ctx->cap_zstd_queue * 4);
        rng("in", d_in, 0);
        rng("out", d_out, 0);
        fprintf(stderr, "rcdc zstd grid %u nblk %llu maxw %llu level %d\n", grid, (unsigned long long)nbl,
                (unsigned long long)maxw, level);
    }
    // RCDC_ZSTD_GUARD=1 (debugging): every scratch buffer of this call is a
    // fresh allocation with 16 MiB of 0xCD before and after it, checked after
    // the call; a kernel that strays past one is reported, not faulted
    struct GBuf {
        uint8_t *base = nullptr;
        uint64_t bytes = 0;
        const char *name = "";
    };
    std::vector<GBuf> gbufs;
    static const bool zguard = getenv("RCDC_ZSTD_GUARD") != nullptr;
    constexpr uint64_t kG = 16ull << 20;
    auto galloc = [&](const char *nm, uint64_t bytes) -> uint8_t * {
        GBuf b;
        b.name = nm;
        b.bytes = bytes;
        if (hipMalloc((void **)&b.base, bytes + 2 * kG) != hipSuccess) return nullptr;
        (void)hipMemset(b.base, 0xCD, bytes + 2 * kG);
        gbufs.push_back(b);
        return b.base + kG;
    };
    ZstdBlob *u_blobs = ctx->d_zstd_blobs;
    ZstdBlk *u_blks = ctx->d_zstd_blks;
    ZstdTables *u_tabs = ctx->d_zstd_tabs;
    uint8_t *u_slots = ctx->d_zstd_slots;
    uint64_t *u_seq = ctx->d_zstd_seq, *u_bpos = ctx->d_zstd_bpos, *u_lens = ctx->d_zstd_lens;
    uint2 *u_res = ctx->d_zstd_res;
    uint32_t *u_queue = ctx->d_zstd_queue, *u_far = farw ? ctx->d_zstd_far : nullptr;
    if (zguard) {
        HIP_TRY(hipStreamSynchronize(st));
        u_blobs = (ZstdBlob *)galloc("blobs", nbo * sizeof(ZstdBlob));
        u_blks = (ZstdBlk *)galloc("blks", nbl * sizeof(ZstdBlk));
        u_tabs = (ZstdTables *)galloc("tabs", sizeof(ZstdTables));
        u_slots = galloc("slots", maxw * kZstdSlot);
        u_seq = (uint64_t *)galloc("seq", ((uint64_t)grid * kZstdMaxSeq + 8) * 8);
        u_bpos = (uint64_t *)galloc("bpos", nbl * 8);
        u_lens = (uint64_t *)galloc("lens", nbo * 8);
        u_res = (uint2 *)galloc("res", nbl * 8);
        u_queue = (uint32_t *)galloc("queue", wins.size() * 128 * 4);
        if (farw) u_far = (uint32_t *)galloc("far", farw * 4);
        for (const GBuf &gb : gbufs)
            if (!gb.base) return fail(RCDC_ERR_INTERNAL, "zstd guard allocation");
        HIP_TRY(hipMemcpy(u_blobs, blobs.data(), nbo * sizeof(ZstdBlob), hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(u_blks, blks.data(), nbl * sizeof(ZstdBlk), hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(u_tabs, &zstd_tables(), sizeof(ZstdTables), hipMemcpyHostToDevice));
        HIP_TRY(hipMemset(u_queue, 0, wins.size() * 128 * 4));
        for (const GBuf &gb : gbufs)
            fprintf(stderr, "rcdc zstd guarded %-6s [%p, %p)\n", gb.name, (void *)(gb.base + kG),
                    (void *)(gb.base + kG + gb.bytes));
    }
    for (size_t k = 0; k < wins.size(); k++) {
        const Win &w = wins[k];
        HIP_TRY(launch_zstd((const uint8_t *)d_in, (uint8_t *)d_out, u_blobs + w.blob0,
                            (uint32_t)w.nblob, u_blks + w.blk0, (uint32_t)w.nblk,
                            u_tabs, u_slots, u_seq, grid, u_res + w.blk0, u_bpos + w.blk0,
                            u_lens + w.blob0, u_queue + 128 * k, u_far, level, st));
    }
    if (zguard) {
        HIP_TRY(hipStreamSynchronize(st));
        std::vector<uint8_t> gh(kG);
        for (const GBuf &gb : gbufs)
            for (int side = 0; side < 2; side++) {
                const uint8_t *gp = side ? gb.base + kG + gb.bytes : gb.base;
                HIP_TRY(hipMemcpy(gh.data(), gp, kG, hipMemcpyDeviceToHost));
                int64_t lo = -1, hi = -1;
                for (uint64_t i = 0; i < kG; i++)
                    if (gh[i] != 0xCD) {
                        if (lo < 0) lo = (int64_t)i;
                        hi = (int64_t)i;
                    }
                if (lo >= 0)
                    fprintf(stderr, "rcdc zstd GUARD HIT %s %s: guard bytes %lld..%lld written\n", gb.name,
                            side ? "after" : "before", (long long)lo, (long long)hi);
            }
        HIP_TRY(hipMemcpy(out_lens, u_lens, nbo * 8, hipMemcpyDeviceToHost));
        for (const GBuf &gb : gbufs) (void)hipFree(gb.base);
        return null_leave(ctx, hip_stream, st);
    }
    HIP_TRY(hipMemcpyAsync(out_lens, ctx->d_zstd_lens, nbo * 8, hipMemcpyDeviceToHost, st));
    // the host descriptors die with this call
    HIP_TRY(poll_stream(st));
    if (const char *e = getenv("RCDC_ZSTD_DBG"))
        if (atoi(e) & 4) zstd_prof_dump();
    return null_leave(ctx, hip_stream, st);
}

// Frame checks.  Compressed frames: the block-parallel pass (a wave per
// block at the position it has when the frame's blocks are 128 KiB), then
// the frames it could not settle checked in order, a wave per frame, longest
// first.  Stored bytes: a wave per blob.
rcdc_status zstd_check(rcdc_ctx *ctx, const void *d_frames, const void *d_data,
                       const rcdc_zstd_check_ref *refs, uint32_t n, uint32_t flags,
                       uint32_t *status, void *hip_stream) {
    if (!valid_ctx(ctx) || (n && (!refs || !d_frames || !d_data || !status)))
        return fail(RCDC_ERR_INVALID_INPUT, "null argument");
    if (!n) return RCDC_OK;
    const bool stored = (flags & RCDC_CHECK_STORED) != 0;
    static const bool blockpar = !(getenv("RCDC_CHECK_BLOCKS") && atoi(getenv("RCDC_CHECK_BLOCKS")) == 0);
    std::lock_guard<std::mutex> lk(ctx->zck_mu);
    DeviceGuard g(ctx->device);
    hipStream_t st;
    rcdc_status rs;
    if ((rs = null_enter(ctx, hip_stream, &st))) return rs;
    // resident waves per CU (12 or 16, by the registers' budget)
    const uint32_t grid = (uint32_t)std::max(ctx->num_cus, 1) * zstd_check_waves_per_cu();
    if ((rs = ensure_dev(&ctx->d_zck_refs, &ctx->cap_zck_refs, 4ull * n))) return rs;
    if ((rs = ensure_dev(&ctx->d_zck_order, &ctx->cap_zck_order, (uint64_t)n + 16))) return rs;
    if ((rs = ensure_dev(&ctx->d_zck_status, &ctx->cap_zck_status, n))) return rs;
    if ((rs = ensure_dev(&ctx->d_zck_scratch, &ctx->cap_zck_scratch, zstd_check_scratch_bytes(grid))))
        return rs;
    uint32_t *ctr = ctx->d_zck_order + n;  // the queue counter sits after the order array
    HIP_TRY(hipMemcpyAsync(ctx->d_zck_refs, refs, sizeof(rcdc_zstd_check_ref) * n,
                           hipMemcpyHostToDevice, st));
    std::vector<uint32_t> order;
    if (!stored && blockpar) {
        std::vector<uint64_t> blk0(n + 1, 0);
        for (uint32_t i = 0; i < n; i++)
            blk0[i + 1] = blk0[i] + std::max<uint64_t>((refs[i].data_len + kZstdBlock - 1) / kZstdBlock, 1);
        const uint64_t nblk = blk0[n];
        if ((rs = ensure_dev(&ctx->d_zck_blk0, &ctx->cap_zck_blk0, n + 1ull))) return rs;
        if ((rs = ensure_dev(&ctx->d_zck_blks, &ctx->cap_zck_blks, nblk * zstd_blkdesc_bytes())))
            return rs;
        HIP_TRY(hipMemcpyAsync(ctx->d_zck_blk0, blk0.data(), 8ull * (n + 1), hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemsetAsync(ctr, 0, 4, st));
        HIP_TRY(launch_zstd_check_blocks((const uint8_t *)d_frames, (const uint8_t *)d_data,
                                         ctx->d_zck_refs, ctx->d_zck_blk0, n, ctx->d_zck_blks, nblk,
                                         ctx->d_zck_scratch, grid, ctx->d_zck_status, ctr, st));
        HIP_TRY(hipMemcpyAsync(status, ctx->d_zck_status, 4ull * n, hipMemcpyDeviceToHost, st));
        HIP_TRY(poll_stream(st));
        for (uint32_t i = 0; i < n; i++)
            if (status[i] == 3u) order.push_back(i);
    } else {
        order.resize(n);
        for (uint32_t i = 0; i < n; i++) order[i] = i;
    }
    if (!order.empty()) {
        std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
            return refs[a].frame_len > refs[b].frame_len;
        });
        HIP_TRY(hipMemsetAsync(ctr, 0, 4, st));
        HIP_TRY(hipMemcpyAsync(ctx->d_zck_order, order.data(), 4ull * order.size(),
                               hipMemcpyHostToDevice, st));
        HIP_TRY(launch_zstd_check((const uint8_t *)d_frames, (const uint8_t *)d_data, ctx->d_zck_refs,
                                  ctx->d_zck_order, (uint32_t)order.size(), stored,
                                  ctx->d_zck_scratch, grid, ctx->d_zck_status, ctr, st));
        HIP_TRY(hipMemcpyAsync(status, ctx->d_zck_status, 4ull * n, hipMemcpyDeviceToHost, st));
        HIP_TRY(poll_stream(st));
    }
    if (const char *e = getenv("RCDC_ZSTD_DBG"))
        if (atoi(e) & 8) zstd_check_prof_dump();
    return null_leave(ctx, hip_stream, st);
}

}  // namespace

extern "C" {

rcdc_status rcdc_zstd_check(rcdc_ctx *ctx, const void *d_frames, const void *d_data,
                            const rcdc_zstd_check_ref *refs, uint32_t n, uint32_t flags,
                            uint32_t *status, void *hip_stream) {
    return zstd_check(ctx, d_frames, d_data, refs, n, flags, status, hip_stream);
}

rcdc_status rcdc_aead_seal(rcdc_ctx *ctx, const uint8_t *key, const void *d_in,
                           const rcdc_aead_ref *refs, uint32_t n, void *d_out, void *hip_stream) {
    return aead_run(ctx, false, key, d_in, refs, n, d_out, nullptr, hip_stream);
}

rcdc_status rcdc_aead_open(rcdc_ctx *ctx, const uint8_t *key, const void *d_in,
                           const rcdc_aead_ref *refs, uint32_t n, void *d_out, uint32_t *status,
                           void *hip_stream) {
    return aead_run(ctx, true, key, d_in, refs, n, d_out, status, hip_stream);
}

rcdc_status rcdc_pack_build(rcdc_ctx *ctx, const uint8_t *key, const void *d_in,
                            const rcdc_pack_blob *blobs, uint32_t nblobs, rcdc_pack *packs,
                            uint32_t npacks, void *d_out, uint64_t out_len,
                            uint32_t *blob_offsets, void *hip_stream) {
    return pack_build(ctx, key, d_in, blobs, nblobs, packs, npacks, d_out, out_len, blob_offsets,
                      hip_stream);
}

rcdc_status rcdc_pack_build_raw(rcdc_ctx *ctx, const uint8_t *key, const void *d_in,
                                const rcdc_pack_blob *blobs, uint32_t nblobs, rcdc_pack *packs,
                                uint32_t npacks, void *d_out, uint64_t out_len,
                                uint32_t *blob_offsets, void *hip_stream) {
    return pack_build(ctx, key, d_in, blobs, nblobs, packs, npacks, d_out, out_len, blob_offsets,
                      hip_stream, true);
}

rcdc_status rcdc_pack_build_raw_multi(rcdc_ctx *ctx, const uint8_t *key,
                                      const void *const *d_ins, uint32_t n_ins,
                                      const rcdc_pack_blob *blobs, uint32_t nblobs,
                                      rcdc_pack *packs, uint32_t npacks, void *d_out,
                                      uint64_t out_len, uint32_t *blob_offsets, void *hip_stream) {
    if (n_ins == 0) return fail(RCDC_ERR_INVALID_INPUT, "no input buffers");
    return pack_build(ctx, key, nullptr, blobs, nblobs, packs, npacks, d_out, out_len,
                      blob_offsets, hip_stream, true, d_ins, n_ins);
}

rcdc_status rcdc_copy_ranges(rcdc_ctx *ctx, const void *const *d_ins, uint32_t n_ins,
                             const rcdc_copy_ref *refs, uint32_t n, void *d_out,
                             void *hip_stream) {
    if (!valid_ctx(ctx) || (n && (!refs || !d_out || !d_ins || !n_ins)))
        return fail(RCDC_ERR_INVALID_INPUT, "null argument");
    std::vector<uint64_t> copies;
    copies.reserve(4 * (size_t)n);
    for (uint32_t i = 0; i < n; i++) {
        const rcdc_copy_ref &c = refs[i];
        if (c.src >= n_ins || !d_ins[c.src])
            return fail(RCDC_ERR_INVALID_INPUT, "copy %u: source %u of %u", i, c.src, n_ins);
        push_copy(copies, d_ins[c.src], c.in_off, c.out_off, c.len);
    }
    DeviceGuard g(ctx->device);
    hipStream_t st;
    rcdc_status rs;
    if ((rs = null_enter(ctx, hip_stream, &st))) return rs;
    if ((rs = copy_units_run(ctx, copies, d_out, st))) return rs;
    return null_leave(ctx, hip_stream, st);
}

uint64_t rcdc_zstd_bound(uint64_t len) {
    return len + 3 * zstd_blocks(len) + (len > kZstdSingleMax ? 10 : 9);  // + the window byte
}

rcdc_status rcdc_zstd_compress(rcdc_ctx *ctx, int level, const void *d_in,
                               const rcdc_zstd_ref *refs, uint32_t n, void *d_out,
                               uint64_t *out_lens, void *hip_stream) {
    return zstd_compress(ctx, level, d_in, refs, n, d_out, out_lens, hip_stream);
}

void rcdc_zstd_tables(void *out) { memcpy(out, &zstd_tables(), sizeof(ZstdTables)); }

uint64_t rcdc_zstd_tables_size(void) { return sizeof(ZstdTables); }

// ---- streaming: one file fed in pieces -------------------------------------

rcdc_status rcdc_stream_open(rcdc_ctx *ctx, rcdc_stream **out) {
    if (!valid_ctx(ctx) || !out) return fail(RCDC_ERR_INVALID_INPUT, "null argument");
    rcdc_stream *s = new rcdc_stream();
    s->ctx = ctx;
    s->batch = rcdc_stream_batch_bytes(ctx);
    s->pending.reserve(s->batch + ctx->max);
    *out = s;
    return RCDC_OK;
}

void rcdc_stream_close(rcdc_stream *st) {
    if (st && st->tail_ev) {  // the last tail copy is done before d_tail is reused
        (void)hipEventSynchronize(st->tail_ev);
        (void)hipEventDestroy(st->tail_ev);
    }
    if (st && st->d_tail) {  // back to the context's pool
        std::lock_guard<std::mutex> lk(st->ctx->tail_mu);
        st->ctx->tail_pool.push_back(st->d_tail);
    }
    delete st;
}

uint64_t rcdc_stream_batch_bytes(const rcdc_ctx *ctx) {
    if (!ctx) return 0;
    // a pass per 16 MiB: large enough that a pass's fixed cost (plan, launch,
    // result copy) is small, small enough that a typical read size triggers a
    // pass straight from the caller's buffer (no intermediate copy)
    uint64_t b = 16ull << 20;
    if (const char *e = getenv("RCDC_STREAM_BATCH")) b = (uint64_t)atoll(e);
    return std::max<uint64_t>(b, 2 * ctx->max + 256);
}

uint64_t rcdc_stream_queued(const rcdc_stream *st) { return st ? st->out.size() : 0; }

// One device pass over the buffered bytes: every cut except the one at the
// end of the buffer depends only on bytes before it, so it is final; the
// end-of-buffer cut is final only at EOF.  The unfinished tail (< max bytes
// from the last final cut) stays buffered and is re-chunked with more data.
static rcdc_status stream_pass(rcdc_stream *st, const uint8_t *data, uint64_t len,
                               bool is_final) {
    rcdc_ctx *ctx = st->ctx;
    const uint64_t P = st->pending.size(), N = P + len;
    if (!N) return RCDC_OK;
    std::vector<uint64_t> tmp(rcdc_max_cuts(ctx, N));
    std::vector<uint64_t> lens{N};
    std::vector<HostPiece> pieces;
    // the pending bytes come from the device copy of the last pass's tail
    // when there is one; otherwise from the host buffer
    const bool dev_tail = P && st->d_tail && st->tail_len == P;
    if (P && !dev_tail) pieces.push_back({0, st->pending.data(), P});
    if (len) pieces.push_back({P, data, len});
    uint64_t cnt = 0;
    Lane *L = nullptr;
    rcdc_status s2 = lane_acquire(ctx, &L);
    if (s2) return s2;
    st->tail_len = 0;
    s2 = run_host_pieces(ctx, L, lens, pieces, tmp.data(), tmp.size(), &cnt,
                         dev_tail ? st->d_tail : nullptr, dev_tail ? P : 0,
                         dev_tail ? st->tail_ev : nullptr);
    uint64_t keep = cnt;
    if (!s2 && !is_final && cnt && tmp[cnt - 1] == N) keep = cnt - 1;
    const uint64_t consumed = keep ? tmp[keep - 1] : 0;
    static const bool devtail = !getenv("RCDC_STREAM_HOSTTAIL");
    if (!s2 && !is_final && N > consumed && devtail) {
        // keep the unfinished tail on the device for the next pass (the lane's
        // arena is reused as soon as the lane is released)
        // (the tail is the last, unfinished chunk: at most max bytes)
        DeviceGuard g(ctx->device);
        if (!st->d_tail) {
            std::lock_guard<std::mutex> lk(ctx->tail_mu);
            if (!ctx->tail_pool.empty()) {
                st->d_tail = ctx->tail_pool.back();
                ctx->tail_pool.pop_back();
            } else if (hipMalloc((void **)&st->d_tail, ctx->max + 256) == hipSuccess) {
                ctx->tail_all.push_back(st->d_tail);
            } else {
                st->d_tail = nullptr;
            }
        }
        // asynchronous: the next pass (any lane) waits on tail_ev before
        // it reads d_tail; the lane's next user queues behind the copy on
        // the same stream before it overwrites the arena
        if (!st->tail_ev && hipEventCreateWithFlags(&st->tail_ev, hipEventDisableTiming) != hipSuccess)
            st->tail_ev = nullptr;
        if (st->d_tail && st->tail_ev && N - consumed <= ctx->max + 256 &&
            hipMemcpyAsync(st->d_tail, L->d_arena + consumed, N - consumed,
                           hipMemcpyDeviceToDevice, L->stream) == hipSuccess &&
            hipEventRecord(st->tail_ev, L->stream) == hipSuccess)
            st->tail_len = N - consumed;
        s2 = RCDC_OK;  // without a device tail the next pass sends the host copy
    }
    lane_release(ctx, L);
    if (s2) return s2;
    for (uint64_t i = 0; i < keep; i++) st->out.push_back(st->base + tmp[i]);
    // the unfinished tail [consumed, N) becomes the new pending bytes (in
    // place: the buffer keeps its capacity)
    if (consumed < P) {
        st->pending.erase(st->pending.begin(), st->pending.begin() + (long)consumed);
        st->pending.insert(st->pending.end(), data, data + len);
    } else {
        const uint64_t d0 = consumed - P;
        st->pending.assign(data + d0, data + len);
    }
    st->base += consumed;
    return RCDC_OK;
}

rcdc_status rcdc_stream_feed(rcdc_stream *st, const uint8_t *data, uint64_t len, int is_final,
                             uint64_t *cuts, uint64_t cap, uint64_t *n_cuts) {
    if (!st || !n_cuts || (len && !data) || (cap && !cuts))
        return fail(RCDC_ERR_INVALID_INPUT, "null argument");
    *n_cuts = 0;
    if (st->done && len) return fail(RCDC_ERR_INVALID_INPUT, "stream already finished");
    if (!st->done) {
        // a device pass once enough bytes are buffered that cuts are certain
        // (every chunk ends by chunk start + max), or at EOF; the new bytes
        // go straight from the caller's buffer to the staging slots
        if (is_final || st->pending.size() + len >= st->batch) {
            rcdc_status s2 = stream_pass(st, data, len, is_final != 0);
            if (s2) {
                // keep the bytes buffered: the caller may retry the feed with
                // len = 0, or close the stream
                st->pending.insert(st->pending.end(), data, data + len);
                return s2;
            }
            if (is_final) {
                st->pending.clear();
                st->done = true;
            }
        } else {
            st->pending.insert(st->pending.end(), data, data + len);
        }
    }
    // hand out what fits; the rest stays queued for the next call
    uint64_t k = 0;
    while (k < cap && !st->out.empty()) {
        cuts[k++] = st->out.front();
        st->out.pop_front();
    }
    *n_cuts = k;
    return RCDC_OK;
}

}  // extern "C"
