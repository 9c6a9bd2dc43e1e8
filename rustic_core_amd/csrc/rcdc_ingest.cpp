// rcdc_ingest.cpp -- the backup data path from files in host memory to pack
// files and pack ids in host memory, native (include/rcdc.h "ingest").
//
// Reference (rustic_core 0.12.0):
//   FileArchiver::backup_reader (archiver/file_archiver.rs:144-160): read a
//     file, ChunkIter, `hash(&chunk)`, `index.has_data`, `Packer::add`;
//   Packer (blob/packer.rs): process_data = zstd + Key::encrypt_data
//     (backend/decrypt.rs:478-506, 566-572) + extra_verify (:508-529),
//     add_raw (:615-655), should_save / PackSizer (:65-200, 659-671),
//     save + write_header (:693-735), finalize (:385-398);
//   the file writer's pack id: hash_reader of the pack file (:826-836).
//
// The engine is a client of the C ABI (rcdc_plan_*, rcdc_sha256_chunks,
// rcdc_zstd_compress, rcdc_aead_seal / _open, rcdc_zstd_check,
// rcdc_pack_build_raw_multi, rcdc_copy_ranges, the host SHA-256) -- the call
// sequence a Rust integration would run -- with its own threads:
//   callers      reserve space in a page-locked input slot, read a file into
//                it (the reference's Read), commit;
//   worker       per batch (one closed input slot): H2D, chunk, ids of the
//                short chunks on the device, zstd + seal + verify of every
//                chunk (stage A); once the batch's ids are in: dedup in chunk
//                order, per-file results, PackSizer grouping with the packer
//                open across batches, pack build, D2H (stage B);
//   pool         SHA-256 on the host: the long chunks' ids from the input
//                slot (a device lane needs ~0.27 s for an 8 MiB chain, a host
//                core ~4 ms) and the pack ids from the pinned pack buffer;
//   waiter       waits for each batch's pack D2H and hands the packs to the
//                pool, whose last job per pack calls the caller's callback.
// Stage A of batch b + 1 .. b + depth - 1 runs before stage B of batch b, so
// the short ids' device chains of several batches overlap.
//
// Streams (rcdc_ingest_stream_*): a file of any length arrives as pieces in
// several slots.  Each batch chunks a stream's bytes of that batch after
// its carry -- the open chunk of the previous batch, at most max bytes, kept
// in a device carry slot (and a host copy for host-hashed ids) -- as one
// plan stream; all but the last chunk are final (a cut at L depends only on
// the bytes before L and the chunk start, rabin.rs:153-188), the last one
// becomes the next carry.  Pieces that are not contiguous in the slot, or
// follow a carry, are gathered into the arena's assembly region first
// (one D2D copy at HBM rate, against the piece's PCIe copy).  Slots holding
// stream pieces enter the pipeline in the order they closed.
#include <hip/hip_runtime.h>

#include <sys/random.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/rcdc.h"

namespace rcdc {
rcdc_status plan_relayout(rcdc_plan *pl, const uint64_t *offs, const uint64_t *lens, uint32_t n,
                          uint64_t arena_len, hipStream_t up);
int ctx_device(const rcdc_ctx *ctx);
uint64_t ctx_min_size(const rcdc_ctx *ctx);
uint64_t ctx_max_size(const rcdc_ctx *ctx);
rcdc_status set_error(rcdc_status st, const char *msg);
void host_sha256_many(const uint8_t *const *ptrs, const uint64_t *lens, uint32_t n,
                      uint8_t *digests);
void host_sha256_one(const uint8_t *p, uint64_t len, uint8_t out[32]);
void host_sha256_ni_many(const uint8_t *const *ptrs, const uint64_t *lens, uint32_t n,
                         uint8_t *digests, int ways);
hipError_t launch_stream_copy(void *dst, const void *src, uint64_t len, uint32_t blocks,
                              hipStream_t stream);
bool host_sha_supported();
bool host_sha_ni();
}  // namespace rcdc

using namespace rcdc;

namespace {

constexpr uint64_t kMaxPackSize = 4076ull << 20;  // packer.rs:58
constexpr uint32_t kMaxPackCount = 10000;         // packer.rs:60
constexpr uint32_t kSrcStaging = 0, kSrcCarry = 1;

uint64_t round_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }
double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

void random_bytes(uint8_t *p, size_t n) {  // the nonces (aespoly1305.rs:120-121: OS RNG)
    while (n) {
        const ssize_t r = getrandom(p, n, 0);
        if (r <= 0) continue;
        p += r;
        n -= (size_t)r;
    }
}

struct Id32 {
    uint8_t b[32];
    bool operator==(const Id32 &o) const { return memcmp(b, o.b, 32) == 0; }
};
struct Id32Hash {
    size_t operator()(const Id32 &x) const {
        uint64_t v;
        memcpy(&v, x.b, 8);
        return (size_t)v;  // ids are SHA-256 digests: any 8 bytes are uniform
    }
};

// PackSizer (packer.rs:65-200): only pack_size() steers should_save.
struct PackSizer {
    uint64_t default_size, grow, limit, current;
    uint64_t pack_size() const {
        uint64_t size = default_size;
        if (grow) size = ((uint64_t)std::sqrt((double)current) * grow + default_size) & 0xFFFFFFFFull;
        return std::min(std::min(size, limit), kMaxPackSize);
    }
};

// One stream (rcdc_ingest_stream_open .. close): its carry between batches
// and its results so far.  Fields by owner: `fed`, `open_pieces`, `closed`
// under the engine's mutex (callers); `base`, `carry_len`, `hcarry`,
// `cslot` on the worker thread (stage A, in batch order); `cuts`, `ids`,
// `nnew` on the back thread (stage B, in batch order).
struct StreamSt {
    uint64_t handle = 0, tag = 0, hint = 0;
    uint64_t fed = 0;          // bytes committed
    uint32_t open_pieces = 0;  // reserved, not committed or cancelled
    bool closed = false, aborted = false;
    int cslot = -1;            // device carry slot
    uint64_t base = 0;         // stream offset of the carry's first byte (the last final cut)
    uint64_t carry_len = 0;
    std::vector<uint8_t> hcarry;
    std::vector<uint64_t> cuts;
    std::vector<uint8_t> ids;
    uint32_t nnew = 0;
};

struct FileEnt {
    uint64_t tag = 0;
    uint64_t off = 0;   // in the batch (whole files 256-aligned)
    uint64_t res = 0;   // bytes reserved
    uint64_t len = 0;   // bytes committed
    bool done = false;
    bool cancelled = false;
    bool final = false;  // a stream's end (close / abort): zero bytes
    std::shared_ptr<StreamSt> st;  // null: a whole file
};

// One plan stream of a batch: a whole file in place, or a stream's bytes of
// this batch (after its carry), in place or gathered in the assembly region.
struct Unit {
    uint64_t tag = 0;
    std::shared_ptr<StreamSt> st;
    bool final = true, aborted = false;
    uint64_t base = 0;       // stream offset of the unit's first byte
    uint64_t carry = 0;      // leading carry bytes
    uint64_t off = 0, len = 0;
    uint64_t fresh = 0;      // bytes new in this batch
    std::vector<std::pair<uint64_t, uint64_t>> segs;          // (slot offset, len)
    std::vector<std::pair<const uint8_t *, uint64_t>> host;   // the unit's bytes in host memory
};

enum SlotState { kFree = 0, kOpen, kClosed, kSubmitted };

struct InSlot {
    uint8_t *host = nullptr;
    uint64_t cap = 0, used = 0;
    uint32_t open_res = 0;
    SlotState state = kFree;
    std::vector<FileEnt> files;
    hipEvent_t h2d = nullptr;
    bool h2d_pending = false;
    std::atomic<int> host_jobs{0};  // long-id jobs still reading this slot
    std::atomic<bool> h2d_issued{false};  // its last H2D piece and h2d are enqueued
    uint64_t close_seq = 0;
    bool has_stream = false;        // holds stream pieces: enters the pipeline in close order
    double t_first = 0;             // its first reservation (slot_max_age_ms)
};

// A batch between stage A and stage B.
struct Batch {
    uint64_t index = 0;
    uint32_t pslot = 0;             // pipeline slot (device buffers, plan)
    InSlot *in = nullptr;
    std::vector<FileEnt> files;
    std::vector<Unit> units;
    std::vector<uint64_t> cuts;     // per unit, consecutive (relative to the unit)
    std::vector<uint32_t> ncuts;    // per unit: chunks final in this batch
    std::vector<uint64_t> c_off, c_len;  // per chunk: arena offset, length
    std::vector<const uint8_t *> c_host;  // long chunks: their bytes in host memory
    std::vector<std::vector<uint8_t>> gathers;  // long chunks split over host pieces; old carries
    std::vector<uint8_t> ids;            // 32 B per chunk
    std::vector<uint32_t> short_idx;     // chunks whose ids the device computes
    std::vector<uint64_t> seal_off, seal_len, ulen;
    hipEvent_t ids_ev = nullptr;
    std::atomic<int> long_jobs{0};
    bool finalize = false;
};

// Device buffers of one pipeline slot.
struct PSlot {
    rcdc_plan *plan = nullptr;
    uint8_t *arena = nullptr;
    uint64_t arena_cap = 0;
    uint8_t *staging = nullptr;  // sealed blobs
    uint64_t staging_cap = 0;
    uint64_t *d_refs = nullptr;  // (off, len) of the short chunks
    uint64_t refs_cap = 0;       // chunks
    uint64_t *h_refs = nullptr;  // page-locked upload source
    uint8_t *d_dig = nullptr;
    hipStream_t s_ids = nullptr;
    hipEvent_t ev_ids = nullptr;
    hipEvent_t ev_sealed = nullptr;   // stage A's device work done (s_comp)
    hipEvent_t ev_retired = nullptr;  // stage B done with the staging area (s_back)
    bool busy = false;                // a batch holds this slot (submit .. stage B)
};

struct OutSlot {
    uint8_t *host = nullptr;
    uint64_t cap = 0;
    std::atomic<int> packs_left{0};
    bool busy = false;
};

struct PackJob {
    OutSlot *out = nullptr;
    uint64_t off = 0, size = 0, seq = 0, batch = 0;
    uint32_t header_len = 0;
    std::vector<rcdc_ingest_blob> blobs;
    uint8_t id[32];
};

}  // namespace

// One dedup set (the packer's ids + the index's), shareable by the engines of
// several devices: 64 shards, one lock each.
struct rcdc_index {
    static constexpr int kShards = 64;
    struct Shard {
        std::mutex mu;
        std::unordered_set<Id32, Id32Hash> set;
    };
    Shard sh[kShards];
    // true: the id was not in the set (the caller packs it)
    bool insert(const Id32 &id) {
        Shard &s = sh[id.b[31] & (kShards - 1)];
        std::lock_guard<std::mutex> lk(s.mu);
        return s.set.insert(id).second;
    }
    uint64_t size() {
        uint64_t n = 0;
        for (auto &s : sh) {
            std::lock_guard<std::mutex> lk(s.mu);
            n += s.set.size();
        }
        return n;
    }
};

struct rcdc_ingest {
    rcdc_ctx *ctx = nullptr;
    rcdc_ingest_config cfg{};
    rcdc_ingest_pack_fn pack_cb = nullptr;
    rcdc_ingest_file_fn file_cb = nullptr;
    void *user = nullptr;
    int device = 0;
    int level = 0;
    bool compress = true, verify = true;
    uint64_t batch_cap = 0, long_chunk = 0;
    uint64_t copy_piece = 64ull << 20;  // bytes per H2D / D2H copy (RCDC_INGEST_COPY_PIECE)
    uint32_t kcopy = 0;  // RCDC_INGEST_KCOPY: batch copies by a shader kernel on this many workgroups
    uint32_t depth = 4, nin = 4, nout = 4, nthreads = 8;
    PackSizer sizer{};
    // input slots
    std::mutex mu;
    std::condition_variable cv_slot;    // a slot became free / a batch ready
    std::vector<std::unique_ptr<InSlot>> in;
    InSlot *open = nullptr;
    std::deque<InSlot *> ready;         // closed, all commits in: stage A order
    // device pipeline
    std::vector<PSlot> ps;
    uint8_t *frames = nullptr;  // zstd frames, then the verify's opened frames
    uint64_t frames_cap = 0;
    uint8_t *d_packs = nullptr;
    uint64_t d_packs_cap = 0;
    uint8_t *carry[2] = {nullptr, nullptr};
    uint64_t carry_cap[2] = {0, 0};
    int carry_cur = 0;
    std::vector<rcdc_pack_blob> carry_blobs;  // the open pack's blobs (src = kSrcCarry)
    hipStream_t s_in = nullptr, s_comp = nullptr, s_out = nullptr;
    hipEvent_t ev_comp = nullptr, ev_out = nullptr, ev_back = nullptr;  // (front / back / out)
    std::vector<std::unique_ptr<OutSlot>> outs;
    std::deque<std::unique_ptr<Batch>> submitted;  // H2D issued, stage A next (front thread)
    std::deque<std::unique_ptr<Batch>> inflight;   // stage A done, stage B next (back thread)
    bool front_done = false;                       // every batch has been through stage A
    uint64_t nclosed = 0;                          // input slots closed so far
    hipStream_t s_back = nullptr;                  // stage B's device work
    uint64_t nbatches = 0, next_seq = 0;
    rcdc_index *idx = nullptr;  // the index's ids + the packer's (own, or shared)
    bool own_idx = true;
    // streams
    uint64_t max_chunk = 0;          // ctx max: a carry's bound
    uint64_t asm_base = 0, asm_cap = 0;  // the arena's assembly region
    uint8_t *carry_pool = nullptr;   // max_streams device carry slots of max_chunk bytes
    std::vector<int> free_cslots;
    std::unordered_map<uint64_t, std::shared_ptr<StreamSt>> streams;  // open handles
    uint64_t next_stream = 1;
    uint32_t closing_streams = 0;    // closed, carry slot not yet released
    std::deque<InSlot *> closed_q;   // closed slots not yet ready, in close order
    double pack_t0 = 0;              // the open pack's first blob (MAX_AGE)
    double pack_max_age = 300, slot_max_age = 1;
    // allocations of this engine (rcdc_ingest_mem_live); RCDC_INGEST_FAIL_ALLOC
    // = k fails the k-th allocation of create (tests)
    uint32_t nalloc = 0, fail_alloc = 0;
    // threads
    std::thread worker, back, waiter, feeder;
    // the feeder's copy pump: batches waiting for their H2D pieces
    struct H2DJob {
        uint8_t *dst;
        const uint8_t *src;
        uint64_t len, done;
        InSlot *in;
    };
    std::deque<H2DJob> h2d_q;
    // ... and the pack bytes' D2H, queued by stage B (back thread)
    struct D2HJob {
        uint8_t *dst;
        const uint8_t *src;
        uint64_t len, done;
        hipEvent_t after;  // the pack build (s_back); the first piece waits on it
        hipEvent_t fin;    // recorded after the last piece (the waiter syncs on it)
        std::shared_ptr<std::atomic<bool>> issued;  // ev_out and fin are enqueued
        bool waited;
    };
    std::mutex d2h_mu;
    std::deque<D2HJob> d2h_q;
    std::shared_ptr<std::atomic<bool>> last_d2h;  // the last D2H job's `issued`
    int submitting = 0;  // slots taken from `ready` whose batch is not in `submitted` yet
    std::vector<std::thread> pool;
    std::mutex pool_mu;
    std::condition_variable pool_cv;
    std::deque<std::function<void()>> jobs;   // pack ids, in order
    std::deque<std::function<void()>> ujobs;  // long chunk ids (urgent), in order
    uint32_t running_packs = 0;               // pack-id jobs running
    std::mutex wait_mu;
    std::condition_variable wait_cv;
    struct WaitItem {
        hipEvent_t ev;
        std::shared_ptr<std::atomic<bool>> issued;
        uint64_t batch;
        std::vector<std::shared_ptr<PackJob>> jobs;
    };
    std::deque<WaitItem> wait_q;
    std::mutex cb_mu;  // callbacks run one at a time
    std::atomic<bool> stop{false};
    bool finishing = false, finished = false;
    std::atomic<int> packs_pending{0};
    std::condition_variable cv_done;
    rcdc_status err = RCDC_OK;
    std::string err_msg;
    rcdc_ingest_stats st{};
    double t_first = 0;
    // RCDC_INGEST_PROF=1: per batch (stage A start, sync points, end; stage B
    // start, ids wait end, end), printed by rcdc_ingest_finish
    int prof = 0;
    std::vector<std::vector<double>> tl;
    std::vector<double> tl_d2h, tl_ids;  // per batch: packs landed, last pack id
};

namespace {

using Ing = rcdc_ingest;

void set_err(Ing *g, rcdc_status s, const std::string &m) {
    std::lock_guard<std::mutex> lk(g->mu);
    if (!g->err) {
        g->err = s;
        g->err_msg = m;
    }
    g->cv_slot.notify_all();
    g->cv_done.notify_all();
}

#define ING_HIP(g, expr)                                                                  \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess) {                                                           \
            set_err(g, RCDC_ERR_INTERNAL, std::string(#expr " failed: ") + hipGetErrorString(e_)); \
            return false;                                                                 \
        }                                                                                 \
    } while (0)
#define ING_ST(g, expr, what)                                                             \
    do {                                                                                  \
        rcdc_status s_ = (expr);                                                          \
        if (s_ != RCDC_OK) {                                                              \
            set_err(g, s_, std::string(what ": ") + rcdc_last_error());                   \
            return false;                                                                 \
        }                                                                                 \
    } while (0)

// ---- the engine's allocations: counted (rcdc_ingest_mem_live), freed on
// every path (free_all), and failable on demand (RCDC_INGEST_FAIL_ALLOC)
std::mutex g_alloc_mu;
std::unordered_map<void *, std::pair<uint64_t, bool>> g_allocs;  // ptr -> (bytes, pinned)
uint64_t g_live_pinned = 0, g_live_dev = 0;

hipError_t ing_alloc(Ing *g, void **p, uint64_t n, bool pinned) {
    *p = nullptr;
    if (g && g->fail_alloc && ++g->nalloc == g->fail_alloc) return hipErrorOutOfMemory;
    const hipError_t e = pinned ? hipHostMalloc(p, n, hipHostMallocDefault) : hipMalloc(p, n);
    if (e != hipSuccess) {
        *p = nullptr;
        return e;
    }
    std::lock_guard<std::mutex> lk(g_alloc_mu);
    g_allocs[*p] = {n, pinned};
    (pinned ? g_live_pinned : g_live_dev) += n;
    return hipSuccess;
}

template <typename T>
hipError_t ing_alloc(Ing *g, T **p, uint64_t n, bool pinned) {
    return ing_alloc(g, (void **)p, n, pinned);
}

// Frees and nulls *p (no-op on null).
template <typename T>
hipError_t ing_free(T **p) {
    if (!*p) return hipSuccess;
    void *q = (void *)*p;
    *p = nullptr;
    bool pinned = false;
    {
        std::lock_guard<std::mutex> lk(g_alloc_mu);
        auto it = g_allocs.find(q);
        if (it != g_allocs.end()) {
            pinned = it->second.second;
            (pinned ? g_live_pinned : g_live_dev) -= it->second.first;
            g_allocs.erase(it);
        }
    }
    return pinned ? hipHostFree(q) : hipFree(q);
}

template <typename T>
bool ensure_dev(Ing *g, T **p, uint64_t *cap, uint64_t need) {
    if (*p && *cap >= need) return true;
    static const bool log = getenv("RCDC_ALLOC_LOG") != nullptr;
    if (log && *p)
        fprintf(stderr, "rcdc ingest: regrow %llu -> %llu x %zu B (hipFree: device sync)\n",
                (unsigned long long)*cap, (unsigned long long)need, sizeof(T));
    ING_HIP(g, ing_free(p));
    *cap = 0;
    const uint64_t n = need + need / 8 + 1;
    ING_HIP(g, ing_alloc(g, p, n * sizeof(T), false));
    *cap = n;
    return true;
}

// Host SHA-256 jobs; `urgent` ones (the long chunks' ids, which gate a
// batch's stage B) go before the pack ids, in the order posted (longest
// first).  Pack-id jobs hold a thread for tens of ms (4 packs of ~40 MB), so
// RCDC_INGEST_ID_THREADS (default 2) threads never take one: a long-id job
// then starts at once instead of after the running pack jobs (r5z2: the last
// batches' stage B waited ~14 ms for a free thread).
void post(Ing *g, std::function<void()> fn, bool urgent = false) {
    {
        std::lock_guard<std::mutex> lk(g->pool_mu);
        (urgent ? g->ujobs : g->jobs).push_back(std::move(fn));
    }
    if (urgent) g->pool_cv.notify_all();  // (a thread free for ids may be
    else g->pool_cv.notify_one();         //  among the waiters)
}

void pool_main(Ing *g) {
    static const uint32_t reserve =
        getenv("RCDC_INGEST_ID_THREADS") ? (uint32_t)atoi(getenv("RCDC_INGEST_ID_THREADS")) : 0u;
    const uint32_t pack_cap = g->nthreads > reserve ? g->nthreads - reserve : 1u;
    for (;;) {
        std::function<void()> fn;
        bool pack = false;
        {
            std::unique_lock<std::mutex> lk(g->pool_mu);
            g->pool_cv.wait(lk, [&] {
                return g->stop || !g->ujobs.empty() ||
                       (!g->jobs.empty() && g->running_packs < pack_cap);
            });
            if (!g->ujobs.empty()) {
                fn = std::move(g->ujobs.front());
                g->ujobs.pop_front();
            } else if (!g->jobs.empty() && g->running_packs < pack_cap) {
                fn = std::move(g->jobs.front());
                g->jobs.pop_front();
                pack = true;
                g->running_packs++;
            } else {
                return;  // stop, nothing left this thread may take
            }
        }
        fn();
        if (pack) {
            {
                std::lock_guard<std::mutex> lk(g->pool_mu);
                g->running_packs--;
            }
            g->pool_cv.notify_all();
        }
    }
}

// Wait for an event by polling (RCDC_INGEST_POLL, default on) instead of
// hipEventSynchronize: a thread blocked in a HIP synchronisation call for a
// 60-70 ms chunk-id kernel held up the other threads' launches (r5r: each
// batch's chunking started only after the previous batch's ids were done).
hipError_t wait_event(hipEvent_t ev) {
    static const bool poll = !(getenv("RCDC_INGEST_POLL") && atoi(getenv("RCDC_INGEST_POLL")) == 0);
    if (!poll) return hipEventSynchronize(ev);
    for (;;) {
        const hipError_t e = hipEventQuery(ev);
        if (e != hipErrorNotReady) return e;
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

// Hand one finished pack to the caller (pack ids are computed by then).
void deliver(Ing *g, const std::shared_ptr<PackJob> &pj) {
    rcdc_ingest_pack p{};
    p.data = pj->out->host + pj->off;
    p.size = pj->size;
    p.seq = pj->seq;
    memcpy(p.id, pj->id, 32);
    p.nblobs = (uint32_t)pj->blobs.size();
    p.header_len = pj->header_len;
    p.blobs = pj->blobs.data();
    {
        std::lock_guard<std::mutex> lk(g->cb_mu);
        if (g->pack_cb) g->pack_cb(g->user, &p);
        if (g->prof) {
            if (g->tl_ids.size() <= pj->batch) g->tl_ids.resize(pj->batch + 1, 0);
            g->tl_ids[pj->batch] = std::max(g->tl_ids[pj->batch], now_s() - g->t_first);
        }
    }
    if (--pj->out->packs_left == 0) {
        std::lock_guard<std::mutex> lk(g->mu);
        pj->out->busy = false;
        g->cv_slot.notify_all();
    }
    if (--g->packs_pending == 0) {
        std::lock_guard<std::mutex> lk(g->mu);
        g->cv_done.notify_all();
    }
}

// Host SHA-256 for pack ids and long chunk ids (RCDC_INGEST_SHA): "ni" (the
// default on CPUs with the SHA extensions) runs `ways` messages interleaved
// per call on one core; "mb" 16 per call in AVX-512 lanes.  On the box's
// cores (r5z, 32 MiB messages, profiles/r05/host_sha_rate.json) SHA-NI gives
// 2.44 / 3.51 / 3.88 / 4.30 GB/s per core at 1 / 2 / 3 / 4 ways and the
// multi-buffer form 4.73: 4 ways match the lanes' throughput at a quarter of
// their latency per message (a 40 MB pack: ~37 ms instead of ~130 ms), and
// the latency of the last batches' ids is the end of the run.
struct ShaPolicy {
    bool mb;
    int ways, ways_last;
};
const ShaPolicy &sha_policy() {
    static const ShaPolicy p = [] {
        ShaPolicy q{};
        const char *m = getenv("RCDC_INGEST_SHA");
        q.mb = host_sha_supported() && (!host_sha_ni() || (m && strcmp(m, "mb") == 0));
        const char *w = getenv("RCDC_SHANI_WAYS"), *wl = getenv("RCDC_SHANI_WAYS_LAST");
        q.ways = std::max(1, std::min(4, w ? atoi(w) : 4));
        q.ways_last = std::max(1, std::min(4, wl ? atoi(wl) : 2));
        return q;
    }();
    return p;
}

// SHA-256 of n host messages (one job's group).
void hash_group(const uint8_t *const *ptrs, const uint64_t *lens, uint32_t n, uint8_t *dig,
                bool mb) {
    if (mb)
        host_sha256_many(ptrs, lens, n, dig);
    else
        host_sha256_ni_many(ptrs, lens, n, dig, (int)n);
}

// After a batch's packs are in host memory: their ids, in groups of `ways`
// interleaved on the SHA extensions (fewer for the last batches, whose ids
// end the run), or 16 per call in AVX-512 lanes ("mb"; the last batches then
// on the SHA extensions).
void hash_packs(Ing *g, std::vector<std::shared_ptr<PackJob>> packs, bool last) {
    const ShaPolicy &pol = sha_policy();
    const bool mb = pol.mb && !last;
    const size_t per = mb ? 16 : (size_t)(last ? pol.ways_last : pol.ways);
    for (size_t a = 0; a < packs.size(); a += per) {
        std::vector<std::shared_ptr<PackJob>> grp(packs.begin() + a,
                                                  packs.begin() + std::min(a + per, packs.size()));
        post(g, [g, grp, mb] {
            std::vector<const uint8_t *> ptrs;
            std::vector<uint64_t> lens;
            std::vector<uint8_t> dig(32 * grp.size());
            for (auto &pj : grp) {
                ptrs.push_back(pj->out->host + pj->off);
                lens.push_back(pj->size);
            }
            hash_group(ptrs.data(), lens.data(), (uint32_t)grp.size(), dig.data(), mb);
            for (size_t i = 0; i < grp.size(); i++) {
                memcpy(grp[i]->id, dig.data() + 32 * i, 32);
                deliver(g, grp[i]);
            }
        });
    }
}

void waiter_main(Ing *g) {
    (void)hipSetDevice(g->device);
    for (;;) {
        Ing::WaitItem w;
        {
            std::unique_lock<std::mutex> lk(g->wait_mu);
            g->wait_cv.wait(lk, [&] { return g->stop || !g->wait_q.empty(); });
            if (g->wait_q.empty()) return;
            w = std::move(g->wait_q.front());
            g->wait_q.pop_front();
        }
        // the pump enqueues the copy's last piece and its event later
        while (!w.issued->load() && !g->err && !g->stop)
            std::this_thread::sleep_for(std::chrono::microseconds(50));
        if (!w.issued->load()) continue;
        if (wait_event(w.ev) != hipSuccess) {
            set_err(g, RCDC_ERR_INTERNAL, "pack copy-back failed");
            continue;
        }
        (void)hipEventDestroy(w.ev);
        if (g->prof) {
            std::lock_guard<std::mutex> lk(g->cb_mu);
            if (g->tl_d2h.size() <= w.batch) g->tl_d2h.resize(w.batch + 1, 0);
            g->tl_d2h[w.batch] = now_s() - g->t_first;
        }
        bool is_last;
        {
            std::lock_guard<std::mutex> lk(g->mu);
            // the last four batches (every batch after rcdc_ingest_finish
            // was too many: throughput, r5v2; the last one alone left ~100 ms
            // of multi-buffer jobs after the last copy, r5u3).  Once the
            // caller has called finish, the batch count is known: a 16-pack
            // call takes ~115 ms, so a batch landing before the last stage A
            // (front_done) still counts as one of the last.
            is_last = g->front_done && g->inflight.size() <= 2;
            if (!is_last && g->finishing && g->ready.size() + g->nbatches <= w.batch + 4)
                is_last = true;
        }
        hash_packs(g, std::move(w.jobs), is_last);
    }
}

// ---- stage A: one closed input slot becomes a batch in flight ------------
void mark(Ing *g, uint64_t b, double t) {
    if (!g->prof) return;
    std::lock_guard<std::mutex> lk(g->cb_mu);
    if (g->tl.size() <= b) g->tl.resize(b + 1);
    g->tl[b].push_back(t - g->t_first);
}

// A ready input slot becomes a batch: a free pipeline slot, and its H2D
// enqueued at once on the copy stream (it runs while earlier batches are in
// stage A), in slot order.
bool submit_ready(Ing *g) {
    for (;;) {
        InSlot *in = nullptr;
        uint32_t ps = 0;
        std::unique_ptr<Batch> B;
        {
            std::lock_guard<std::mutex> lk(g->mu);
            if (g->ready.empty()) return true;
            for (ps = 0; ps < g->depth && g->ps[ps].busy; ps++) {
            }
            if (ps == g->depth) return true;
            in = g->ready.front();
            g->ready.pop_front();
            g->submitting++;
            g->ps[ps].busy = true;
            B = std::make_unique<Batch>();
            B->index = g->nbatches++;
            if (g->t_first == 0) g->t_first = now_s();
        }
        B->pslot = ps;
        B->in = in;
        B->files = in->files;
        mark(g, B->index, now_s());
        PSlot &P = g->ps[ps];
        const uint64_t used = in->used;
        if (!ensure_dev(g, &P.arena, &P.arena_cap, round_up(used, 256) + 512)) return false;
        // the arena's previous batch is retired: its ids (the last reader)
        // are done.  The copy goes to the pump (feeder_main), piece by piece.
        in->h2d_issued = false;
        g->h2d_q.push_back({P.arena, in->host, used, 0, in});
        std::lock_guard<std::mutex> lk(g->mu);
        g->submitted.push_back(std::move(B));
        g->submitting--;
        g->cv_slot.notify_all();
    }
}

void reap_inputs(Ing *g);
void close_open_locked(Ing *g);

// Feeder thread: a ready input slot's H2D is enqueued as soon as a pipeline
// slot is free, whatever stage A is doing (the front thread used to enqueue
// it only between two stage A runs: each copy then started only after the
// previous batch's stage A, r5g timeline).
//
// It also pumps the H2D copies: at most two 64 MiB pieces are enqueued at a
// time.  HIP's copies go to DMA engine queues in order, and stage A's small
// uploads (plan tables, AEAD and zstd descriptors) landed behind every piece
// already queued: with a whole 2 GiB batch enqueued at once each upload
// waited ~40 ms (r5n: seal 40 ms after zstd; the next batch's stage A
// started only after the previous chunk ids).  With two pieces in flight an
// upload waits ~2.4 ms at most and the engine never idles.
bool pump_h2d(Ing *g, std::deque<hipEvent_t> &inflight, std::vector<hipEvent_t> &free_ev) {
    while (!inflight.empty() && hipEventQuery(inflight.front()) == hipSuccess) {
        free_ev.push_back(inflight.front());
        inflight.pop_front();
    }
    while (!g->h2d_q.empty() && inflight.size() < 2 && !free_ev.empty()) {
        Ing::H2DJob &J = g->h2d_q.front();
        const uint64_t n = std::min(g->copy_piece, J.len - J.done);
        if (n) {
            if (g->kcopy)
                ING_HIP(g, launch_stream_copy(J.dst + J.done, J.src + J.done, (n + 15) & ~15ull,
                                              g->kcopy, g->s_in));
            else
                ING_HIP(g, hipMemcpyAsync(J.dst + J.done, J.src + J.done, n, hipMemcpyHostToDevice,
                                          g->s_in));
            hipEvent_t ev = free_ev.back();
            free_ev.pop_back();
            ING_HIP(g, hipEventRecord(ev, g->s_in));
            inflight.push_back(ev);
            J.done += n;
        }
        if (J.done == J.len) {
            ING_HIP(g, hipEventRecord(J.in->h2d, g->s_in));
            J.in->h2d_issued = true;
            g->h2d_q.pop_front();
            std::lock_guard<std::mutex> lk(g->mu);
            g->cv_slot.notify_all();
        }
    }
    return true;
}

// The D2H of the pack bytes the same way (small read-backs of stage A wait
// behind a whole 1 GiB pack copy otherwise: r5p, the next batch's chunking
// started only when the previous batch's packs were in host memory).
bool pump_d2h(Ing *g, std::deque<hipEvent_t> &inflight, std::vector<hipEvent_t> &free_ev) {
    while (!inflight.empty() && hipEventQuery(inflight.front()) == hipSuccess) {
        free_ev.push_back(inflight.front());
        inflight.pop_front();
    }
    std::lock_guard<std::mutex> lq(g->d2h_mu);
    while (!g->d2h_q.empty() && inflight.size() < 2 && !free_ev.empty()) {
        Ing::D2HJob &J = g->d2h_q.front();
        if (!J.waited) {
            ING_HIP(g, hipStreamWaitEvent(g->s_out, J.after, 0));
            ING_HIP(g, hipEventDestroy(J.after));
            J.waited = true;
        }
        const uint64_t n = std::min(g->copy_piece, J.len - J.done);
        if (n) {
            if (g->kcopy)
                ING_HIP(g, launch_stream_copy(J.dst + J.done, J.src + J.done, (n + 15) & ~15ull,
                                              g->kcopy, g->s_out));
            else
                ING_HIP(g, hipMemcpyAsync(J.dst + J.done, J.src + J.done, n, hipMemcpyDeviceToHost,
                                          g->s_out));
            hipEvent_t ev = free_ev.back();
            free_ev.pop_back();
            ING_HIP(g, hipEventRecord(ev, g->s_out));
            inflight.push_back(ev);
            J.done += n;
        }
        if (J.done == J.len) {
            ING_HIP(g, hipEventRecord(g->ev_out, g->s_out));
            ING_HIP(g, hipEventRecord(J.fin, g->s_out));
            J.issued->store(true);
            g->d2h_q.pop_front();
        }
    }
    return true;
}

void feeder_main(Ing *g) {
    (void)hipSetDevice(g->device);
    std::deque<hipEvent_t> inflight, inflight_o;
    std::vector<hipEvent_t> free_ev(4, nullptr), free_o(4, nullptr);
    for (auto *v : {&free_ev, &free_o})
        for (auto &e : *v)
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
                set_err(g, RCDC_ERR_INTERNAL, "feeder events");
                return;
            }
    auto release = [&] {
        (void)hipStreamSynchronize(g->s_in);
        (void)hipStreamSynchronize(g->s_out);
        for (auto e : inflight) free_ev.push_back(e);
        for (auto e : inflight_o) free_o.push_back(e);
        for (auto e : free_ev) (void)hipEventDestroy(e);
        for (auto e : free_o) (void)hipEventDestroy(e);
    };
    for (;;) {
        reap_inputs(g);
        if (!submit_ready(g) || !pump_h2d(g, inflight, free_ev) || !pump_d2h(g, inflight_o, free_o)) {
            release();
            return;
        }
        bool d2h_idle;
        {
            std::lock_guard<std::mutex> lq(g->d2h_mu);
            d2h_idle = g->d2h_q.empty();
        }
        std::unique_lock<std::mutex> lk(g->mu);
        // an open slot with files that stopped filling goes to the device
        // (a trickle of small files is not held back until finish)
        if (g->open && !g->open->files.empty() && now_s() - g->open->t_first >= g->slot_max_age)
            close_open_locked(g);
        // the back thread queues D2H jobs until the very end (finalize)
        if (g->err || (g->finished && g->h2d_q.empty() && d2h_idle)) {
            lk.unlock();
            release();
            return;
        }
        // a piece is ~1.2 ms: poll often while copies are queued
        g->cv_slot.wait_for(lk, std::chrono::microseconds(g->h2d_q.empty() && d2h_idle ? 200 : 50));
    }
}

// The bytes [rel, rel + len) of a unit in host memory: a pointer into one of
// its host pieces, or null when they span pieces.
const uint8_t *unit_host(const Unit &u, uint64_t rel, uint64_t len) {
    uint64_t at = 0;
    for (const auto &h : u.host) {
        if (rel >= at && rel + len <= at + h.second) return h.first + (rel - at);
        at += h.second;
    }
    return nullptr;
}

void unit_gather(const Unit &u, uint64_t rel, uint64_t len, uint8_t *dst) {
    uint64_t at = 0;
    for (const auto &h : u.host) {
        const uint64_t a = std::max(rel, at), e = std::min(rel + len, at + h.second);
        if (a < e) memcpy(dst + (a - rel), h.first + (a - at), e - a);
        at += h.second;
    }
}

// The batch's plan streams: whole files in place; per stream, its carry and
// its pieces of this batch, in place when that is one contiguous piece and
// no carry, else gathered into the assembly region (copies appended to cr).
bool build_units(Ing *g, Batch *B, std::vector<rcdc_copy_ref> &cr, uint64_t *asm_used) {
    InSlot *in = B->in;
    std::unordered_map<StreamSt *, size_t> unit_of;
    for (const FileEnt &f : B->files) {
        if (f.cancelled) continue;
        if (!f.st) {
            Unit u;
            u.tag = f.tag;
            u.off = f.off;
            u.len = u.fresh = f.len;
            u.segs.push_back({f.off, f.len});
            B->units.push_back(std::move(u));
            continue;
        }
        auto it = unit_of.find(f.st.get());
        if (it == unit_of.end()) {
            Unit u;
            u.st = f.st;
            u.tag = f.st->tag;
            u.final = false;
            u.base = f.st->base;
            u.carry = f.st->carry_len;
            it = unit_of.emplace(f.st.get(), B->units.size()).first;
            B->units.push_back(std::move(u));
        }
        Unit &u = B->units[it->second];
        if (f.final) {
            u.final = true;
            u.aborted = f.st->aborted;
        }
        if (!f.len) continue;
        if (!u.segs.empty() && u.segs.back().first + u.segs.back().second == f.off)
            u.segs.back().second += f.len;  // laid out back to back (stream_reserve)
        else
            u.segs.push_back({f.off, f.len});
        u.fresh += f.len;
    }
    uint64_t ao = 0;
    for (Unit &u : B->units) {
        if (!u.st) {
            u.host.push_back({in->host + u.off, u.len});
            continue;
        }
        u.len = u.carry + u.fresh;
        if (!u.carry && u.segs.size() <= 1) {  // in place
            u.off = u.segs.empty() ? 0 : u.segs[0].first;
            if (u.fresh) u.host.push_back({in->host + u.off, u.fresh});
            continue;
        }
        u.off = g->asm_base + ao;
        uint64_t o = u.off;
        if (u.carry) {
            rcdc_copy_ref c{};
            c.in_off = (uint64_t)u.st->cslot * g->max_chunk;
            c.out_off = o;
            c.len = u.carry;
            c.src = 1;
            cr.push_back(c);
            u.host.push_back({u.st->hcarry.data(), u.carry});
            o += u.carry;
        }
        for (const auto &sg : u.segs) {
            rcdc_copy_ref c{};
            c.in_off = sg.first;
            c.out_off = o;
            c.len = sg.second;
            c.src = 0;
            cr.push_back(c);
            u.host.push_back({in->host + sg.first, sg.second});
            o += sg.second;
        }
        ao = round_up(ao + u.len, 256);
        if (ao > g->asm_cap) {
            set_err(g, RCDC_ERR_INTERNAL, "ingest: assembly region overflow");
            return false;
        }
    }
    *asm_used = ao;
    return true;
}

bool stage_a(Ing *g, Batch *B) {
    InSlot *in = B->in;
    PSlot &P = g->ps[B->pslot];
    const uint64_t used = in->used;
    // 1. the H2D (the feeder's pump) lands before the chunking: wait until
    // its event is enqueued, then order the compute stream after it
    {
        std::unique_lock<std::mutex> lk(g->mu);
        while (!in->h2d_issued && !g->err) g->cv_slot.wait_for(lk, std::chrono::microseconds(100));
        if (g->err) return false;
    }
    ING_HIP(g, hipStreamWaitEvent(g->s_comp, in->h2d, 0));
    if (g->prof > 1) mark(g, B->index, now_s());
    // 2. the plan streams; streams' carries and scattered pieces gathered
    std::vector<rcdc_copy_ref> gcr;
    uint64_t asm_used = 0;
    if (!build_units(g, B, gcr, &asm_used)) return false;
    if (!gcr.empty()) {
        const void *gsrc[2] = {P.arena, g->carry_pool};
        ING_ST(g, rcdc_copy_ranges(g->ctx, gsrc, 2, gcr.data(), (uint32_t)gcr.size(), P.arena,
                                   g->s_comp),
               "stream gather");
    }
    const uint32_t nf = (uint32_t)B->units.size();
    std::vector<uint64_t> offs(nf), lens(nf);
    uint64_t bytes = 0, ubytes = 0, nfiles = 0;
    for (uint32_t i = 0; i < nf; i++) {
        offs[i] = B->units[i].off;
        lens[i] = B->units[i].len;
        bytes += B->units[i].fresh;
        ubytes += lens[i];
        nfiles += !B->units[i].st || (B->units[i].final && !B->units[i].aborted);
    }
    const uint64_t arena_len =
        std::max(round_up(used, 256) + 256, asm_used ? g->asm_base + asm_used + 256 : 0);
    // 3. chunk
    if (!P.plan) {
        ING_ST(g, rcdc_plan_create(g->ctx, offs.data(), lens.data(), nf, arena_len, &P.plan),
               "plan");
    } else {
        ING_ST(g, plan_relayout(P.plan, offs.data(), lens.data(), nf, arena_len, g->s_comp),
               "plan");
    }
    if (g->prof > 1) mark(g, B->index, now_s());
    ING_ST(g, rcdc_plan_run(P.plan, P.arena, g->s_comp), "chunk");
    if (g->prof > 1) {  // (RCDC_INGEST_PROF=2: the H2D's and the chunking's own ends)
        (void)hipEventSynchronize(in->h2d);
        mark(g, B->index, now_s());
    }
    const uint64_t cap = (uint64_t)nf + ubytes / 4096 + 16;  // min >= 4096 (rcdc_check_params)
    std::vector<uint64_t> cuts(std::max<uint64_t>(cap, 1)), counts(std::max<uint32_t>(nf, 1));
    rcdc_status rs = rcdc_plan_results(P.plan, cuts.data(), cuts.size(), counts.data());
    if (rs == RCDC_ERR_CAPACITY) {
        uint64_t tot = 0;
        for (uint32_t i = 0; i < nf; i++) tot += counts[i];
        cuts.resize(tot);
        rs = rcdc_plan_results(P.plan, cuts.data(), cuts.size(), counts.data());
    }
    ING_ST(g, rs, "chunk results");
    mark(g, B->index, now_s());
    // chunk lists: a stream's last chunk of a batch (not its end) is its
    // carry, not a chunk yet -- every earlier cut is final
    B->ncuts.resize(nf);
    std::vector<rcdc_copy_ref> ccr;  // the new carries, device
    std::vector<std::pair<Unit *, uint64_t>> carries;  // (unit, carry start in the unit)
    {
        uint64_t k = 0;
        for (uint32_t i = 0; i < nf; i++) {
            Unit &u = B->units[i];
            const uint64_t n = counts[i];
            uint64_t keep = n;
            if (u.st && (!u.final || u.aborted)) {
                keep = n ? n - 1 : 0;
                const uint64_t from = keep ? cuts[k + keep - 1] : 0;
                if (!u.aborted) {
                    carries.push_back({&u, from});
                    if (u.len > from) {
                        rcdc_copy_ref c{};
                        c.in_off = u.off + from;
                        c.out_off = (uint64_t)u.st->cslot * g->max_chunk;
                        c.len = u.len - from;
                        c.src = 0;
                        ccr.push_back(c);
                    }
                }
            }
            B->ncuts[i] = (uint32_t)keep;
            uint64_t prev = 0;
            for (uint64_t j = 0; j < keep; j++) {
                B->cuts.push_back(cuts[k + j]);
                B->c_off.push_back(u.off + prev);
                B->c_len.push_back(cuts[k + j] - prev);
                prev = cuts[k + j];
            }
            k += n;
        }
    }
    const uint64_t nchunks = B->c_off.size();
    B->ids.assign(nchunks * 32, 0);
    // 3. ids: short chunks on the device (own stream per pipeline slot), long
    // ones on host threads from the input slot
    // The last batches' ids bound the run's end: a batch's longest device
    // chain (~34 MB/s per lane: 62 ms for a 2 MiB chunk) holds its stage B,
    // and stage B runs in batch order, so the host takes the chunks above
    // 1 MiB of the last RCDC_INGEST_TAIL_BATCHES (default 2) batches too and
    // both sides end together (~30 ms).  (The last batch alone: the one
    // before it still waited ~40 ms for its device ids, r5y.)
    static const size_t tail_batches =
        getenv("RCDC_INGEST_TAIL_BATCHES") ? (size_t)atoi(getenv("RCDC_INGEST_TAIL_BATCHES")) : 2;
    bool tail;
    {
        std::lock_guard<std::mutex> lk(g->mu);
        const size_t after = g->ready.size() + g->submitted.size() + (size_t)g->submitting +
                             (g->open != nullptr ? 1 : 0);
        tail = g->finishing && after < tail_batches;
    }
    const uint64_t long_thr = tail ? std::min<uint64_t>(g->long_chunk, 1ull << 20) : g->long_chunk;
    std::vector<uint32_t> long_idx;
    for (uint64_t k = 0; k < nchunks; k++)
        (B->c_len[k] > long_thr ? long_idx : B->short_idx).push_back((uint32_t)k);
    // the long chunks' host bytes: in place, or gathered from a stream's
    // host pieces (a chunk that starts in the carry) before the carries move
    B->c_host.assign(nchunks, nullptr);
    if (!long_idx.empty()) {
        std::vector<uint32_t> unit_of(nchunks);
        for (uint32_t i = 0, k = 0; i < nf; i++)
            for (uint32_t j = 0; j < B->ncuts[i]; j++) unit_of[k++] = i;
        for (uint32_t k : long_idx) {
            const Unit &u = B->units[unit_of[k]];
            const uint64_t rel = B->c_off[k] - u.off;
            B->c_host[k] = unit_host(u, rel, B->c_len[k]);
            if (!B->c_host[k]) {
                B->gathers.emplace_back(B->c_len[k]);
                unit_gather(u, rel, B->c_len[k], B->gathers.back().data());
                B->c_host[k] = B->gathers.back().data();
            }
        }
    }
    // the streams' new carries (device: one copy; host: their bytes), and
    // the carry slots of streams that ended
    if (!ccr.empty()) {
        const void *csrc[1] = {P.arena};
        ING_ST(g, rcdc_copy_ranges(g->ctx, csrc, 1, ccr.data(), (uint32_t)ccr.size(), g->carry_pool,
                                   g->s_comp),
               "stream carry");
    }
    // A long chunk's host bytes may lie inside the old carry (c_host points
    // into it: a chunk of exactly max bytes that ended a batch's unit is
    // the next batch's carry, whole): the old carries stay with the batch
    // until its host id jobs are done (stage B runs after them)
    for (auto &c : carries) {
        Unit &u = *c.first;
        StreamSt &st = *u.st;
        std::vector<uint8_t> h(u.len - c.second);
        if (!h.empty()) unit_gather(u, c.second, h.size(), h.data());
        B->gathers.push_back(std::move(st.hcarry));
        st.hcarry = std::move(h);
        st.base = u.base + c.second;
        st.carry_len = u.len - c.second;
    }
    {
        std::lock_guard<std::mutex> lk(g->mu);
        for (Unit &u : B->units)
            if (u.st && u.final && u.st->cslot >= 0) {
                g->free_cslots.push_back(u.st->cslot);
                u.st->cslot = -1;
                B->gathers.push_back(std::move(u.st->hcarry));
                u.st->hcarry = std::vector<uint8_t>();
                g->closing_streams--;
            }
        g->cv_slot.notify_all();
    }
    std::sort(B->short_idx.begin(), B->short_idx.end(),
              [&](uint32_t a, uint32_t b) { return B->c_len[a] > B->c_len[b]; });
    const uint64_t ns = B->short_idx.size();
    if (ns > P.refs_cap) {
        if (getenv("RCDC_ALLOC_LOG") && P.refs_cap)
            fprintf(stderr, "rcdc ingest: regrow refs %llu -> %llu\n", (unsigned long long)P.refs_cap,
                    (unsigned long long)ns);
        ING_HIP(g, ing_free(&P.h_refs));
        ING_HIP(g, ing_free(&P.d_refs));
        ING_HIP(g, ing_free(&P.d_dig));
        P.refs_cap = ns + ns / 4 + 64;
        ING_HIP(g, ing_alloc(g, &P.h_refs, P.refs_cap * 16, true));
        ING_HIP(g, ing_alloc(g, &P.d_refs, P.refs_cap * 16, false));
        ING_HIP(g, ing_alloc(g, &P.d_dig, P.refs_cap * 32, false));
    }
    for (uint64_t j = 0; j < ns; j++) {
        P.h_refs[2 * j] = B->c_off[B->short_idx[j]];
        P.h_refs[2 * j + 1] = B->c_len[B->short_idx[j]];
    }
    ING_HIP(g, hipEventRecord(g->ev_comp, g->s_comp));
    ING_HIP(g, hipStreamWaitEvent(P.s_ids, g->ev_comp, 0));
    if (ns) {
        ING_HIP(g, hipMemcpyAsync(P.d_refs, P.h_refs, ns * 16, hipMemcpyHostToDevice, P.s_ids));
        ING_ST(g, rcdc_sha256_chunks(g->ctx, P.arena, (const rcdc_chunk_ref *)P.d_refs,
                                     (uint32_t)ns, P.d_dig, P.s_ids),
               "chunk ids");
    }
    ING_HIP(g, hipEventRecord(P.ev_ids, P.s_ids));
    // long ids: groups of similar lengths (longest first), `ways` per call on
    // the SHA extensions or 16 per multi-buffer call (sha_policy)
    std::sort(long_idx.begin(), long_idx.end(),
              [&](uint32_t a, uint32_t b) { return B->c_len[a] > B->c_len[b]; });
    Batch *bp = B;
    const bool mb = sha_policy().mb;
    const size_t per = mb ? 16 : (size_t)sha_policy().ways;
    for (size_t a = 0; a < long_idx.size(); a += per) {
        std::vector<uint32_t> grp(long_idx.begin() + a,
                                  long_idx.begin() + std::min(a + per, long_idx.size()));
        bp->long_jobs++;
        in->host_jobs++;
        post(g, [g, bp, in, grp, mb] {
            std::vector<const uint8_t *> ptrs;
            std::vector<uint64_t> ls;
            std::vector<uint8_t> dig(32 * grp.size());
            for (uint32_t k : grp) {
                ptrs.push_back(bp->c_host[k]);
                ls.push_back(bp->c_len[k]);
            }
            hash_group(ptrs.data(), ls.data(), (uint32_t)grp.size(), dig.data(), mb);
            for (size_t i = 0; i < grp.size(); i++)
                memcpy(bp->ids.data() + 32ull * grp[i], dig.data() + 32 * i, 32);
            in->host_jobs--;
            bp->long_jobs--;
            std::lock_guard<std::mutex> lk(g->mu);
            g->cv_slot.notify_all();
        }, true);
    }
    {  // from here the slot is freed once its H2D and long-id jobs are done
        std::lock_guard<std::mutex> lk(g->mu);
        in->h2d_pending = true;
        in->state = kSubmitted;
    }
    // 4. every chunk: zstd (version 2), seal into the staging area, verify
    std::vector<uint64_t> src_off(nchunks), src_len(nchunks);
    const uint8_t *src = P.arena;
    B->ulen.assign(nchunks, 0);
    if (g->compress && nchunks) {
        uint64_t fo = 0;
        std::vector<rcdc_zstd_ref> zr(nchunks);
        for (uint64_t k = 0; k < nchunks; k++) {
            zr[k].in_off = B->c_off[k];
            zr[k].len = B->c_len[k];
            zr[k].out_off = fo;
            src_off[k] = fo;
            fo = round_up(fo + rcdc_zstd_bound(B->c_len[k]) + 48, 16);
        }
        if (!ensure_dev(g, &g->frames, &g->frames_cap, fo + 64)) return false;
        ING_ST(g, rcdc_zstd_compress(g->ctx, g->level, P.arena, zr.data(), (uint32_t)nchunks,
                                     g->frames, src_len.data(), g->s_comp),
               "zstd");
        src = g->frames;
        for (uint64_t k = 0; k < nchunks; k++) B->ulen[k] = B->c_len[k];
        mark(g, B->index, now_s());
    } else {
        for (uint64_t k = 0; k < nchunks; k++) {
            src_off[k] = B->c_off[k];
            src_len[k] = B->c_len[k];
        }
    }
    B->seal_off.resize(nchunks);
    B->seal_len.resize(nchunks);
    std::vector<rcdc_aead_ref> ar(nchunks);
    uint64_t so = 0;
    for (uint64_t k = 0; k < nchunks; k++) {
        ar[k].in_off = src_off[k];
        ar[k].len = src_len[k];
        ar[k].out_off = so;
        B->seal_off[k] = so;
        B->seal_len[k] = src_len[k] + 32;
        so = round_up(so + src_len[k] + 64, 16);
    }
    if (nchunks) {
        std::vector<uint8_t> nonces(16 * nchunks);
        random_bytes(nonces.data(), nonces.size());
        for (uint64_t k = 0; k < nchunks; k++) memcpy(ar[k].nonce, nonces.data() + 16 * k, 16);
    }
    if (!ensure_dev(g, &P.staging, &P.staging_cap, so + 64)) return false;
    // the staging area's previous batch has been packed (stage B, s_back)
    ING_HIP(g, hipStreamWaitEvent(g->s_comp, P.ev_retired, 0));
    if (nchunks)
        ING_ST(g, rcdc_aead_seal(g->ctx, g->cfg.key, src, ar.data(), (uint32_t)nchunks, P.staging,
                                 g->s_comp),
               "seal");
    if (g->verify && nchunks) {
        // very_data (decrypt.rs:508-529): open (MAC) into the frames buffer,
        // decode, compare with the chunk in place
        std::vector<rcdc_aead_ref> orf(nchunks);
        std::vector<rcdc_zstd_check_ref> cr(nchunks);
        uint64_t po = 0;
        for (uint64_t k = 0; k < nchunks; k++) {
            orf[k].in_off = B->seal_off[k];
            orf[k].len = B->seal_len[k];
            orf[k].out_off = po;
            cr[k].frame_off = po;
            cr[k].frame_len = src_len[k];
            cr[k].data_off = B->c_off[k];
            cr[k].data_len = B->c_len[k];
            po = round_up(po + src_len[k] + 16, 16);
        }
        if (!g->compress && !ensure_dev(g, &g->frames, &g->frames_cap, po + 64)) return false;
        std::vector<uint32_t> stat(nchunks, 0);
        ING_ST(g, rcdc_aead_open(g->ctx, g->cfg.key, P.staging, orf.data(), (uint32_t)nchunks,
                                 g->frames, stat.data(), g->s_comp),
               "verify open");
        for (uint64_t k = 0; k < nchunks; k++)
            if (stat[k]) {
                set_err(g, RCDC_ERR_VERIFICATION, "Verifying data failed (MAC)");
                return false;
            }
        ING_ST(g, rcdc_zstd_check(g->ctx, g->frames, P.arena, cr.data(), (uint32_t)nchunks,
                                  g->compress ? 0u : RCDC_CHECK_STORED, stat.data(), g->s_comp),
               "verify check");
        for (uint64_t k = 0; k < nchunks; k++)
            if (stat[k]) {
                set_err(g, RCDC_ERR_VERIFICATION,
                        "Verifying compressed data failed (extra_verify, decrypt.rs:516-526)");
                return false;
            }
    }
    ING_HIP(g, hipEventRecord(P.ev_sealed, g->s_comp));
    mark(g, B->index, now_s());
    {
        std::lock_guard<std::mutex> lk(g->mu);
        g->st.bytes_in += bytes;
        g->st.files += nfiles;
        g->st.chunks += nchunks;
        g->st.batches++;
    }
    return true;
}

// ---- stage B: dedup, per-file results, packs ------------------------------
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;  // stage B with no batch: close the open pack

bool stage_b(Ing *g, Batch *B, bool finalize) {
    const bool has_slot = B->pslot != kNoSlot;
    PSlot &P = g->ps[has_slot ? B->pslot : 0];
    const uint64_t n = B->c_len.size();
    mark(g, B->index, now_s());
    if (has_slot) {
        ING_HIP(g, wait_event(P.ev_ids));
        ING_HIP(g, hipStreamWaitEvent(g->s_back, P.ev_sealed, 0));
    }
    mark(g, B->index, now_s());
    const uint64_t ns = B->short_idx.size();
    if (ns) {
        std::vector<uint8_t> dig(ns * 32);
        // on the ids' own stream (not the legacy default stream's queue)
        ING_HIP(g, hipMemcpyAsync(dig.data(), P.d_dig, ns * 32, hipMemcpyDeviceToHost, P.s_ids));
        ING_HIP(g, hipEventRecord(P.ev_ids, P.s_ids));
        ING_HIP(g, wait_event(P.ev_ids));
        for (uint64_t j = 0; j < ns; j++)
            memcpy(B->ids.data() + 32ull * B->short_idx[j], dig.data() + 32 * j, 32);
    }
    // Packer::add (packer.rs:304-315): the first occurrence of an id the
    // index does not have is added, in chunk order
    std::vector<uint8_t> is_new(n, 0);
    std::vector<rcdc_pack_blob> nb;
    nb.reserve(n);
    for (uint64_t k = 0; k < n; k++) {
        Id32 id;
        memcpy(id.b, B->ids.data() + 32 * k, 32);
        if (!g->idx->insert(id)) continue;
        is_new[k] = 1;
        rcdc_pack_blob b{};
        b.in_off = B->seal_off[k];
        b.len = (uint32_t)B->seal_len[k];
        b.uncompressed_len = (uint32_t)B->ulen[k];
        b.type = 0;
        b.pad = kSrcStaging;
        memcpy(b.id, id.b, 32);
        nb.push_back(b);
    }
    // per-file results (the tree's content lists, file_archiver.rs:144-168):
    // a whole file at once; a stream's chunks accumulate until its end
    {
        uint64_t k = 0;
        for (size_t i = 0; i < B->units.size(); i++) {
            const Unit &u = B->units[i];
            const uint32_t ne = B->ncuts[i];
            uint32_t nnew = 0;
            for (uint32_t j = 0; j < ne; j++) nnew += is_new[k + j];
            rcdc_ingest_file_result fr{};
            bool deliver_file = false;
            if (!u.st) {
                fr.tag = u.tag;
                fr.len = u.len;
                fr.nchunks = ne;
                fr.nnew = nnew;
                fr.cuts = B->cuts.data() + k;
                fr.ids = B->ids.data() + 32 * k;
                deliver_file = true;
            } else {
                StreamSt &st = *u.st;
                for (uint32_t j = 0; j < ne; j++) st.cuts.push_back(u.base + B->cuts[k + j]);
                st.ids.insert(st.ids.end(), B->ids.begin() + 32 * k, B->ids.begin() + 32 * (k + ne));
                st.nnew += nnew;
                if (u.final && !u.aborted) {
                    fr.tag = st.tag;
                    fr.len = u.base + u.len;  // the stream's length (its last cut)
                    fr.nchunks = (uint32_t)st.cuts.size();
                    fr.nnew = st.nnew;
                    fr.cuts = st.cuts.data();
                    fr.ids = st.ids.data();
                    deliver_file = true;
                }
            }
            k += ne;
            if (deliver_file && g->file_cb) {
                std::lock_guard<std::mutex> lk(g->cb_mu);
                g->file_cb(g->user, &fr);
            }
            if (u.st && u.final) {
                std::vector<uint64_t>().swap(u.st->cuts);
                std::vector<uint8_t>().swap(u.st->ids);
            }
        }
    }
    // the open pack's blobs first, then this batch's new ones
    std::vector<rcdc_pack_blob> blobs = g->carry_blobs;
    blobs.insert(blobs.end(), nb.begin(), nb.end());
    // should_save (packer.rs:659-671) pack by pack; take_data adds each closed
    // pack's size to the sizer (:749-758)
    // ... and by age (MAX_AGE, packer.rs:63,668-670): the open pack carried in
    // from earlier batches is saved once its first blob is pack_max_age old
    const double tnow = now_s();
    const bool carried = !g->carry_blobs.empty();
    const bool aged = carried && tnow - g->pack_t0 >= g->pack_max_age;
    std::vector<std::pair<uint32_t, uint32_t>> grp;
    size_t b0 = 0;
    while (b0 < blobs.size()) {
        const uint64_t limit = g->sizer.pack_size();
        uint64_t sz = 0, hdr = 0;
        size_t e = b0;
        while (e < blobs.size() && sz < limit && e - b0 < kMaxPackCount) {
            sz += blobs[e].len;
            hdr += blobs[e].uncompressed_len ? 41 : 37;
            e++;
        }
        const bool closed = sz >= limit || e - b0 >= kMaxPackCount;
        if (!closed && !finalize && !(aged && b0 == 0)) break;
        grp.push_back({(uint32_t)b0, (uint32_t)(e - b0)});
        g->sizer.current += sz + hdr + 32 + 4;
        b0 = e;
    }
    const size_t open_from = b0;
    std::vector<rcdc_pack> packs(grp.size());
    uint64_t total = 0;
    {
        std::vector<uint8_t> hn(16 * grp.size());
        random_bytes(hn.data(), hn.size());
        for (size_t j = 0; j < grp.size(); j++) {
            uint64_t sz = 32 + 4;
            for (uint32_t i = grp[j].first; i < grp[j].first + grp[j].second; i++)
                sz += blobs[i].len + (blobs[i].uncompressed_len ? 41 : 37);
            packs[j].out_off = total;
            packs[j].blob0 = grp[j].first;
            packs[j].nblobs = grp[j].second;
            memcpy(packs[j].header_nonce, hn.data() + 16 * j, 16);
            total += sz;
        }
    }
    const void *cur_carry = g->carry[g->carry_cur];
    const void *srcs[2] = {has_slot ? (const void *)P.staging : cur_carry,
                           cur_carry ? cur_carry : (const void *)P.staging};
    std::vector<uint32_t> boffs(std::max<size_t>(open_from, 1));
    OutSlot *out = nullptr;
    // The packs go back in groups of whole packs of ~256 MiB, each with its
    // own end event: a group's pack ids start as soon as it has landed, not
    // after the batch's whole D2H (~20 ms for a 2 GiB batch's ~1 GB of packs;
    // the last batch's ids end the run).
    struct D2HGroup {
        size_t first, last;  // packs [first, last)
        hipEvent_t fin;
        std::shared_ptr<std::atomic<bool>> flag;
    };
    std::vector<D2HGroup> d2h_groups;
    if (!grp.empty()) {
        // the last pack build's D2H must be done with d_packs: once the pump
        // has enqueued its last piece, ev_out marks its end
        if (g->last_d2h)
            while (!g->last_d2h->load() && !g->err)
                std::this_thread::sleep_for(std::chrono::microseconds(50));
        if (g->err) return false;
        if (total + 64 > g->d_packs_cap) {
            // a regrow frees d_packs: every D2H piece reading it must have
            // run, not only been enqueued (hipFree waits for queued work, but
            // the pump enqueues pieces one by one)
            ING_HIP(g, wait_event(g->ev_out));
            if (!ensure_dev(g, &g->d_packs, &g->d_packs_cap, total + 64)) return false;
        }
        ING_HIP(g, hipStreamWaitEvent(g->s_back, g->ev_out, 0));
        ING_ST(g, rcdc_pack_build_raw_multi(g->ctx, g->cfg.key, srcs, 2, blobs.data(),
                                            (uint32_t)open_from, packs.data(),
                                            (uint32_t)packs.size(), g->d_packs, total,
                                            boffs.data(), g->s_back),
               "pack build");
        {  // a free page-locked output slot
            std::unique_lock<std::mutex> lk(g->mu);
            for (;;) {
                for (auto &o : g->outs)
                    if (!o->busy) {
                        out = o.get();
                        break;
                    }
                if (out || g->err) break;
                g->cv_slot.wait_for(lk, std::chrono::milliseconds(2));
            }
            if (!out) return false;
            out->busy = true;
        }
        if (out->cap < total) {
            if (getenv("RCDC_ALLOC_LOG") && out->cap)
                fprintf(stderr, "rcdc ingest: regrow out slot %llu -> %llu\n",
                        (unsigned long long)out->cap, (unsigned long long)total);
            ING_HIP(g, ing_free(&out->host));
            out->cap = total + total / 4;
            ING_HIP(g, ing_alloc(g, &out->host, out->cap, true));
        }
        // the D2H goes to the feeder's pump, piece by piece, after the build
        // (the first group's job orders the copy stream after it; the rest
        // follow on that stream)
        hipEvent_t after;
        ING_HIP(g, hipEventCreateWithFlags(&after, hipEventDisableTiming));
        ING_HIP(g, hipEventRecord(after, g->s_back));
        static const uint64_t group_bytes_env =
            getenv("RCDC_INGEST_D2H_GROUP") ? strtoull(getenv("RCDC_INGEST_D2H_GROUP"), nullptr, 10)
                                            : 256ull << 20;
        // The last two batches' packs go back one pack per group: each pack's
        // id starts as soon as that pack has landed.  Their ids are the end of
        // the run, and in groups of ~256 MiB the last group's packs were
        // still being hashed ~43 ms after the last copy (r6i timeline, 16
        // files: landed 385 ms, last id 429 ms).
        static const bool tail_single =
            !(getenv("RCDC_INGEST_TAIL_SINGLE") && atoi(getenv("RCDC_INGEST_TAIL_SINGLE")) == 0);
        bool tail_b;
        {
            std::lock_guard<std::mutex> lk(g->mu);
            tail_b = finalize || (g->finishing && g->front_done && g->inflight.size() <= 1);
        }
        const uint64_t group_bytes = tail_single && tail_b ? 1 : group_bytes_env;
        for (size_t a = 0; a < grp.size();) {
            size_t b = a + 1;
            while (b < grp.size() && packs[b].out_off - packs[a].out_off < group_bytes) b++;
            D2HGroup G{a, b, nullptr, std::make_shared<std::atomic<bool>>(false)};
            ING_HIP(g, hipEventCreateWithFlags(&G.fin, hipEventDisableTiming));
            const uint64_t lo = packs[a].out_off, hi = b < grp.size() ? packs[b].out_off : total;
            {
                std::lock_guard<std::mutex> lq(g->d2h_mu);
                g->d2h_q.push_back({out->host + lo, g->d_packs + lo, hi - lo, 0,
                                    a == 0 ? after : nullptr, G.fin, G.flag, a != 0});
            }
            g->last_d2h = G.flag;
            d2h_groups.push_back(G);
            a = b;
        }
        g->cv_slot.notify_all();
    }
    // the still open pack: its blobs into the other carry buffer
    std::vector<rcdc_pack_blob> rest(blobs.begin() + open_from, blobs.end());
    if (!rest.empty()) {
        const int nx = g->carry_cur ^ 1;
        std::vector<rcdc_copy_ref> cr(rest.size());
        uint64_t o = 0;
        for (size_t i = 0; i < rest.size(); i++) {
            cr[i].in_off = rest[i].in_off;
            cr[i].out_off = o;
            cr[i].len = rest[i].len;
            cr[i].src = rest[i].pad;
            rest[i].in_off = o;
            rest[i].pad = kSrcCarry;
            o = round_up(o + rest[i].len, 16);
        }
        if (!ensure_dev(g, &g->carry[nx], &g->carry_cap[nx], o + 64)) return false;
        ING_ST(g, rcdc_copy_ranges(g->ctx, srcs, 2, cr.data(), (uint32_t)cr.size(), g->carry[nx],
                                   g->s_back),
               "carry");
        g->carry_cur = nx;
    }
    // the open pack's age: from its first blob (a pack that starts in this
    // batch is new; one carried on keeps its time)
    if (!rest.empty() && (open_from > 0 || !carried)) g->pack_t0 = tnow;
    g->carry_blobs = std::move(rest);
    if (!grp.empty()) {
        std::vector<std::shared_ptr<PackJob>> jobs;
        for (size_t j = 0; j < grp.size(); j++) {
            auto pj = std::make_shared<PackJob>();
            pj->out = out;
            pj->off = packs[j].out_off;
            pj->size = packs[j].size;
            pj->header_len = packs[j].header_len;
            pj->seq = g->next_seq++;
            pj->batch = B->index;
            for (uint32_t i = grp[j].first; i < grp[j].first + grp[j].second; i++) {
                rcdc_ingest_blob e{};
                memcpy(e.id, blobs[i].id, 32);
                e.offset = boffs[i];
                e.length = blobs[i].len;
                e.uncompressed_length = blobs[i].uncompressed_len;
                e.type = blobs[i].type;
                pj->blobs.push_back(e);
            }
            jobs.push_back(pj);
        }
        out->packs_left += (int)jobs.size();
        g->packs_pending += (int)jobs.size();
        {
            std::lock_guard<std::mutex> lk(g->mu);
            g->st.packs += jobs.size();
            g->st.pack_bytes += total;
        }
        {
            std::lock_guard<std::mutex> lk(g->wait_mu);
            for (const D2HGroup &G : d2h_groups)
                g->wait_q.push_back({G.fin, G.flag, B->index,
                                     std::vector<std::shared_ptr<PackJob>>(
                                         jobs.begin() + G.first, jobs.begin() + G.last)});
        }
        g->wait_cv.notify_one();
    }
    if (has_slot) ING_HIP(g, hipEventRecord(P.ev_retired, g->s_back));
    {
        std::lock_guard<std::mutex> lk(g->mu);
        g->st.new_blobs += nb.size();
    }
    mark(g, B->index, now_s());
    return true;
}

// The input slot of a batch is free again once its H2D has landed and the
// host long-id jobs have read it.
void reap_inputs(Ing *g) {
    std::lock_guard<std::mutex> lk(g->mu);
    for (auto &s : g->in)
        if (s->state == kSubmitted && s->host_jobs == 0 &&
            (!s->h2d_pending || hipEventQuery(s->h2d) == hipSuccess)) {
            s->h2d_pending = false;
            s->state = kFree;
            s->used = 0;
            s->files.clear();
            s->has_stream = false;
            s->t_first = 0;
            g->cv_slot.notify_all();
        }
}

// Front thread: the copies in (submit_ready) and stage A, in batch order.
void worker_main(Ing *g) {
    (void)hipSetDevice(g->device);
    for (;;) {
        std::unique_ptr<Batch> B;
        bool done = false;
        {
            std::unique_lock<std::mutex> lk(g->mu);
            if (g->err) {
                g->cv_done.notify_all();
                return;
            }
            if (!g->submitted.empty()) {
                B = std::move(g->submitted.front());
                g->submitted.pop_front();
            } else {
                // closed slots whose files are not all in wait in closed_q
                done = g->finishing && g->ready.empty() && g->open == nullptr &&
                       g->closed_q.empty() && g->submitting == 0;
            }
        }
        if (B) {
            if (!stage_a(g, B.get())) return;
            std::lock_guard<std::mutex> lk(g->mu);
            g->inflight.push_back(std::move(B));
            g->cv_slot.notify_all();
            continue;
        }
        std::unique_lock<std::mutex> lk(g->mu);
        if (done) {
            g->front_done = true;
            g->cv_slot.notify_all();
            return;
        }
        g->cv_slot.wait_for(lk, std::chrono::microseconds(200));
    }
}

// Back thread: stage B in batch order once a batch's ids are in, then the
// pipeline slot is free for the next batch; at the end, Packer::finalize.
void back_main(Ing *g) {
    (void)hipSetDevice(g->device);
    for (;;) {
        std::unique_ptr<Batch> B;
        bool last = false, all_done = false, fin_carry = false, aged = false;
        {
            std::unique_lock<std::mutex> lk(g->mu);
            for (;;) {
                if (g->err) {
                    g->cv_done.notify_all();
                    return;
                }
                if (!g->inflight.empty() && g->inflight.front()->long_jobs == 0) break;
                if (g->inflight.empty() && g->front_done) break;
                // MAX_AGE with no batch coming: the open pack is saved on its
                // own (a trickle backup leaves recent packs behind)
                if (g->inflight.empty() && !g->carry_blobs.empty() &&
                    now_s() - g->pack_t0 >= g->pack_max_age) {
                    aged = true;
                    break;
                }
                g->cv_slot.wait_for(lk, std::chrono::microseconds(200));
            }
            if (aged) {
            } else if (!g->inflight.empty()) {
                B = std::move(g->inflight.front());
                g->inflight.pop_front();
                last = g->front_done && g->inflight.empty();
            } else {
                all_done = true;
                fin_carry = !g->carry_blobs.empty();
            }
        }
        if (aged) {
            Batch empty;
            empty.pslot = kNoSlot;
            empty.index = g->nbatches;
            if (!stage_b(g, &empty, true)) return;
            continue;
        }
        if (B) {
            if (!stage_b(g, B.get(), last)) return;
            std::lock_guard<std::mutex> lk(g->mu);
            g->ps[B->pslot].busy = false;
            g->cv_slot.notify_all();
            continue;
        }
        if (all_done) {
            if (fin_carry) {  // Packer::finalize with nothing else left
                Batch empty;
                empty.pslot = kNoSlot;
                empty.index = g->nbatches;
                if (!stage_b(g, &empty, true)) return;
            }
            std::unique_lock<std::mutex> lk(g->mu);
            g->finished = true;
            g->cv_done.notify_all();
            return;
        }
    }
}

// Closed slots whose reservations are all in enter the pipeline (`ready`).
// A slot holding stream pieces enters only at the head of the close order:
// a stream's pieces are chunked in the order they were reserved, and its
// carry passes from batch to batch.  Others may pass a slot still waiting
// for a commit.  A slot left with nothing (every file cancelled) is free.
void promote_locked(Ing *g) {
    bool head = true;
    for (auto it = g->closed_q.begin(); it != g->closed_q.end();) {
        InSlot *s = *it;
        if (s->open_res == 0 && (head || !s->has_stream)) {
            it = g->closed_q.erase(it);
            bool empty = true;
            for (const FileEnt &f : s->files) empty &= f.cancelled;
            if (empty) {
                s->state = kFree;
                s->used = 0;
                s->files.clear();
                s->has_stream = false;
                s->t_first = 0;
            } else {
                g->ready.push_back(s);
            }
            g->cv_slot.notify_all();
            continue;
        }
        head = false;
        ++it;
    }
}

void close_open_locked(Ing *g) {
    InSlot *s = g->open;
    if (!s) return;
    g->open = nullptr;
    s->close_seq = g->nclosed++;
    s->state = kClosed;
    g->closed_q.push_back(s);
    promote_locked(g);
    g->cv_slot.notify_all();
}

// Space for len bytes in the open slot (a new one when it does not fit).  A
// stream's piece goes right after the stream's previous piece when that is
// committed and the last thing in the slot (the two are then one range).
rcdc_status reserve_locked(Ing *g, std::unique_lock<std::mutex> &lk, uint64_t len,
                           const std::shared_ptr<StreamSt> &st, bool final, uint8_t **buf,
                           uint64_t *ticket) {
    for (;;) {
        if (g->err) return set_error(g->err, g->err_msg.c_str());
        if (g->finishing) return set_error(RCDC_ERR_INVALID_INPUT, "ingest already finishing");
        InSlot *s = g->open;
        // the first slot closes at a quarter: the device starts sooner
        const uint64_t cap_now = g->nclosed == 0 ? std::max(g->batch_cap / 4, len)
                                                 : (s ? s->cap : 0);
        uint64_t place = s ? s->used : 0;
        if (s && st && !s->files.empty()) {
            const FileEnt &b = s->files.back();
            if (b.st == st && b.done && !b.cancelled && s->used == round_up(b.off + b.res, 256))
                place = b.off + b.len;
        }
        if (s && place + len > cap_now) {
            close_open_locked(g);
            s = nullptr;
            place = 0;
        }
        if (!s) {
            for (auto &x : g->in)
                if (x->state == kFree) {
                    s = x.get();
                    break;
                }
            if (s) {
                s->state = kOpen;
                s->used = 0;
                s->files.clear();
                s->has_stream = false;
                s->t_first = 0;
                g->open = s;
            }
        }
        if (s) {
            FileEnt f;
            f.off = place;
            f.res = len;
            f.st = st;
            f.final = final;
            s->files.push_back(f);
            s->used = round_up(place + len, 256);
            s->open_res++;
            s->has_stream |= st != nullptr;
            if (s->files.size() == 1) s->t_first = now_s();
            size_t idx = 0;
            for (; idx < g->in.size(); idx++)
                if (g->in[idx].get() == s) break;
            *ticket = ((uint64_t)idx << 32) | (uint64_t)(s->files.size() - 1);
            *buf = s->host + place;
            return RCDC_OK;
        }
        g->cv_slot.wait_for(lk, std::chrono::milliseconds(1));
        lk.unlock();
        reap_inputs(g);
        lk.lock();
    }
}

// Commit (or cancel) a reservation.
rcdc_status commit_locked(Ing *g, uint64_t ticket, uint64_t tag, uint64_t len, bool cancel) {
    const uint64_t si = ticket >> 32, fi = ticket & 0xFFFFFFFFull;
    if (si >= g->in.size() || fi >= g->in[si]->files.size() || g->in[si]->files[fi].done ||
        (g->in[si]->state != kOpen && g->in[si]->state != kClosed))
        return set_error(RCDC_ERR_INVALID_INPUT, "bad ticket");
    InSlot *s = g->in[si].get();
    FileEnt &f = s->files[fi];
    if (len > f.res) return set_error(RCDC_ERR_INVALID_INPUT, "commit longer than the reservation");
    if (!f.st) f.tag = tag;
    f.len = cancel ? 0 : len;
    f.done = true;
    f.cancelled = cancel;
    if (f.st) {
        f.st->fed += f.len;
        f.st->open_pieces--;
    }
    s->open_res--;
    if (s->state == kClosed && s->open_res == 0) promote_locked(g);
    return RCDC_OK;
}

std::shared_ptr<StreamSt> find_stream(Ing *g, uint64_t h) {
    auto it = g->streams.find(h);
    return it == g->streams.end() ? nullptr : it->second;
}

rcdc_status stream_end(Ing *g, uint64_t handle, bool abort) {
    if (!g) return set_error(RCDC_ERR_INVALID_INPUT, "null argument");
    std::unique_lock<std::mutex> lk(g->mu);
    auto st = find_stream(g, handle);
    if (!st) return set_error(RCDC_ERR_INVALID_INPUT, "unknown stream");
    if (st->open_pieces)
        return set_error(RCDC_ERR_INVALID_INPUT, "stream has pieces not committed or cancelled");
    // a zero-byte final piece carries the end through the pipeline
    uint8_t *buf;
    uint64_t t;
    if (rcdc_status rs = reserve_locked(g, lk, 0, st, true, &buf, &t)) return rs;
    st->closed = true;
    st->aborted = abort;
    g->streams.erase(handle);
    g->closing_streams++;
    return commit_locked(g, t, 0, 0, false);
}

// Engine buffer sizes for a config (create and rcdc_ingest_footprint).
struct Sizes {
    uint64_t batch_cap, max_chunk, min_chunk;
    uint32_t depth, nin, nout, nthreads, max_streams;
    uint64_t out_slot, asm_base, asm_cap, arena, staging, refs_cap, frames, carry, carry_pool;
    uint64_t pinned() const { return nin * batch_cap + nout * out_slot + depth * refs_cap * 16; }
    uint64_t device() const {
        return depth * (arena + staging + refs_cap * 48) + 2 * frames + 2 * carry + carry_pool;
    }
};

Sizes engine_sizes(const rcdc_ctx *ctx, const rcdc_ingest_config *cfg, uint64_t pack_size) {
    Sizes z{};
    z.batch_cap = round_up(cfg->batch_bytes ? cfg->batch_bytes : (2ull << 30), 256);
    z.max_chunk = round_up(std::max<uint64_t>(ctx_max_size(ctx), 64), 256);
    z.min_chunk = std::max<uint64_t>(ctx_min_size(ctx), 4096);
    z.depth = cfg->depth ? cfg->depth : 4;
    z.nin = std::max(cfg->in_slots ? cfg->in_slots : 4u, 2u);
    z.nout = std::max(cfg->out_slots ? cfg->out_slots : 4u, 1u);
    z.nthreads = cfg->hash_threads ? cfg->hash_threads : 10;
    z.max_streams = cfg->max_streams ? cfg->max_streams : 16;
    z.out_slot = z.batch_cap + z.batch_cap / 16 + (64ull << 20);
    // a batch's stream units gathered: its pieces plus one carry per stream
    z.asm_base = round_up(z.batch_cap + 1024, 256);
    z.asm_cap = z.batch_cap + (uint64_t)z.max_streams * (z.max_chunk + 256) + 256;
    z.arena = z.asm_base + z.asm_cap + 1024;
    const uint64_t chunked = z.batch_cap + (uint64_t)z.max_streams * z.max_chunk;
    z.staging = chunked + chunked / 64 + (64ull << 20);
    z.frames = z.staging;
    z.refs_cap = chunked / z.min_chunk * 2 + 1024;
    z.carry = std::max<uint64_t>(pack_size * 2, 128ull << 20);
    z.carry_pool = (uint64_t)z.max_streams * z.max_chunk;
    return z;
}

// Every buffer, stream, event and plan of the engine (threads stopped or
// never started); safe on a partly built engine.
void free_all(Ing *g) {
    (void)hipSetDevice(g->device);
    for (auto &s : g->in) {
        (void)ing_free(&s->host);
        if (s->h2d) (void)hipEventDestroy(s->h2d);
        s->h2d = nullptr;
    }
    for (auto &o : g->outs) (void)ing_free(&o->host);
    for (auto &P : g->ps) {
        if (P.plan) rcdc_plan_destroy(P.plan);
        P.plan = nullptr;
        (void)ing_free(&P.arena);
        (void)ing_free(&P.staging);
        (void)ing_free(&P.d_refs);
        (void)ing_free(&P.d_dig);
        (void)ing_free(&P.h_refs);
        for (hipEvent_t *e : {&P.ev_ids, &P.ev_sealed, &P.ev_retired})
            if (*e) (void)hipEventDestroy(*e), *e = nullptr;
        if (P.s_ids) (void)hipStreamDestroy(P.s_ids);
        P.s_ids = nullptr;
    }
    (void)ing_free(&g->frames);
    (void)ing_free(&g->d_packs);
    (void)ing_free(&g->carry[0]);
    (void)ing_free(&g->carry[1]);
    (void)ing_free(&g->carry_pool);
    for (hipStream_t *q : {&g->s_in, &g->s_comp, &g->s_out, &g->s_back})
        if (*q) (void)hipStreamDestroy(*q), *q = nullptr;
    for (hipEvent_t *e : {&g->ev_comp, &g->ev_back, &g->ev_out})
        if (*e) (void)hipEventDestroy(*e), *e = nullptr;
    if (g->own_idx) delete g->idx;
    g->idx = nullptr;
}

}  // namespace

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

void rcdc_ingest_config_default(rcdc_ingest_config *c) {
    if (!c) return;
    memset(c, 0, sizeof *c);
    c->zstd_level = 0;
    c->compress = 1;
    c->extra_verify = 1;
    c->pack_size = 32ull << 20;  // configfile.rs:211-231 (data packs)
    c->pack_grow_factor = 32;
    c->pack_size_limit = 0xFFFFFFFFull;
    c->batch_bytes = 2ull << 30;
    c->depth = 4;
    c->in_slots = 4;
    c->out_slots = 4;
    c->hash_threads = 10;
    c->max_streams = 16;
    c->long_chunk = 2ull << 20;
    c->pack_max_age_ms = 300000;  // packer.rs:63 MAX_AGE = 5 min
    c->slot_max_age_ms = 1000;
}

rcdc_status rcdc_ingest_footprint(const rcdc_ctx *ctx, const rcdc_ingest_config *cfg,
                                  uint64_t *pinned, uint64_t *device) {
    if (!ctx || !cfg) return set_error(RCDC_ERR_INVALID_INPUT, "null argument");
    PackSizer ps{cfg->pack_size ? cfg->pack_size : (32ull << 20), cfg->pack_grow_factor,
                 cfg->pack_size_limit ? cfg->pack_size_limit : 0xFFFFFFFFull, cfg->pack_current_size};
    const Sizes z = engine_sizes(ctx, cfg, ps.pack_size());
    if (pinned) *pinned = z.pinned();
    if (device) *device = z.device();
    return RCDC_OK;
}

void rcdc_ingest_mem_live(uint64_t *pinned, uint64_t *device) {
    std::lock_guard<std::mutex> lk(g_alloc_mu);
    if (pinned) *pinned = g_live_pinned;
    if (device) *device = g_live_dev;
}

rcdc_status rcdc_ingest_create(rcdc_ctx *ctx, const rcdc_ingest_config *cfg,
                               rcdc_ingest_pack_fn pack_cb, rcdc_ingest_file_fn file_cb,
                               void *user, rcdc_ingest **out) {
    if (!ctx || !cfg || !out) return set_error(RCDC_ERR_INVALID_INPUT, "null argument");
    if (cfg->zstd_level < -131072 || cfg->zstd_level > 22)
        return set_error(RCDC_ERR_INVALID_INPUT, "zstd level out of range");
    auto g = std::make_unique<rcdc_ingest>();
    g->ctx = ctx;
    g->cfg = *cfg;
    g->pack_cb = pack_cb;
    g->file_cb = file_cb;
    g->user = user;
    g->device = ctx_device(ctx);
    g->prof = getenv("RCDC_INGEST_PROF") ? std::max(atoi(getenv("RCDC_INGEST_PROF")), 1) : 0;
    if (const char *e = getenv("RCDC_INGEST_FAIL_ALLOC")) g->fail_alloc = (uint32_t)std::max(atoi(e), 0);
    g->level = cfg->zstd_level;
    g->compress = cfg->compress != 0;
    g->verify = cfg->extra_verify != 0;
    g->sizer.default_size = cfg->pack_size ? cfg->pack_size : (32ull << 20);
    g->sizer.grow = cfg->pack_grow_factor;
    g->sizer.limit = cfg->pack_size_limit ? cfg->pack_size_limit : 0xFFFFFFFFull;
    g->sizer.current = cfg->pack_current_size;
    const Sizes z = engine_sizes(ctx, cfg, g->sizer.pack_size());
    g->batch_cap = z.batch_cap;
    g->long_chunk = cfg->long_chunk ? cfg->long_chunk : (2ull << 20);
    if (const char *e = getenv("RCDC_INGEST_KCOPY")) g->kcopy = (uint32_t)std::max(atoi(e), 0);
    if (const char *e = getenv("RCDC_INGEST_COPY_PIECE"))
        g->copy_piece = std::max<uint64_t>(strtoull(e, nullptr, 10), 1ull << 20);
    g->depth = z.depth;
    g->nin = z.nin;
    g->nout = z.nout;
    g->nthreads = z.nthreads;
    g->max_chunk = z.max_chunk;
    g->asm_base = z.asm_base;
    g->asm_cap = z.asm_cap;
    g->pack_max_age = (cfg->pack_max_age_ms ? cfg->pack_max_age_ms : 300000) / 1e3;
    g->slot_max_age = (cfg->slot_max_age_ms ? cfg->slot_max_age_ms : 1000) / 1e3;
    g->idx = new rcdc_index();
    g->own_idx = true;
    for (uint32_t i = 0; i < z.max_streams; i++) g->free_cslots.push_back((int)(z.max_streams - 1 - i));
    Ing *gp = g.get();
    (void)hipSetDevice(g->device);
    // any failure below: everything allocated so far is freed
    auto fail_hip = [&](hipError_t e, const char *what) {
        free_all(gp);
        return set_error(RCDC_ERR_INTERNAL,
                         (std::string(what) + ": " + hipGetErrorString(e)).c_str());
    };
    auto fail_st = [&](rcdc_status st) {
        const std::string m = rcdc_last_error();
        free_all(gp);
        return set_error(st, m.c_str());
    };
    hipError_t e;
    for (uint32_t i = 0; i < g->nin; i++) {
        auto s = std::make_unique<InSlot>();
        s->cap = g->batch_cap;
        InSlot *sp = s.get();
        g->in.push_back(std::move(s));
        if ((e = ing_alloc(gp, &sp->host, sp->cap, true)) != hipSuccess) return fail_hip(e, "input slot");
        if ((e = hipEventCreateWithFlags(&sp->h2d, hipEventDisableTiming)) != hipSuccess)
            return fail_hip(e, "event");
    }
    for (uint32_t i = 0; i < g->nout; i++) {
        auto o = std::make_unique<OutSlot>();
        o->cap = z.out_slot;
        OutSlot *op = o.get();
        g->outs.push_back(std::move(o));
        if ((e = ing_alloc(gp, &op->host, op->cap, true)) != hipSuccess) return fail_hip(e, "output slot");
    }
    // the open pack's carry buffers, sized for a default pack and its slack
    for (int c = 0; c < 2; c++) {
        if ((e = ing_alloc(gp, &g->carry[c], z.carry, false)) != hipSuccess) return fail_hip(e, "carry");
        g->carry_cap[c] = z.carry;
    }
    if ((e = ing_alloc(gp, &g->carry_pool, z.carry_pool, false)) != hipSuccess)
        return fail_hip(e, "stream carries");
    g->ps.resize(g->depth);
    for (auto &P : g->ps) {
        // the chunk-id kernel runs for up to ~60 ms (a 2 MiB chunk's
        // SHA-256 chain on one lane): its stream gets the lowest priority, so
        // HIP puts it on a hardware queue of its own class -- a stream that
        // shared its queue waited behind it in order (r5o: each batch's
        // chunking started only when the previous batch's ids were done)
        int prio_lo = 0, prio_hi = 0;
        (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
        if ((e = hipStreamCreateWithPriority(&P.s_ids, hipStreamNonBlocking, prio_lo)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&P.ev_ids, hipEventDisableTiming)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&P.ev_sealed, hipEventDisableTiming)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&P.ev_retired, hipEventDisableTiming)) != hipSuccess)
            return fail_hip(e, "stream");
        // device buffers sized for a full batch up front (a hipFree inside
        // the pipeline would synchronise the device): the slot's bytes, then
        // the assembly region for streams' gathered pieces and carries
        if ((e = ing_alloc(gp, &P.arena, z.arena, false)) != hipSuccess) return fail_hip(e, "arena");
        P.arena_cap = z.arena;
        if ((e = ing_alloc(gp, &P.staging, z.staging, false)) != hipSuccess)
            return fail_hip(e, "staging");
        P.staging_cap = z.staging;
        // the plan built once for a full-batch layout (allocations and
        // synchronous uploads here, not inside the pipeline); each batch then
        // re-lays it out on its compute stream, reusing the buffers
        // (256 streams: its per-stream arrays then hold any batch of up to
        // 256 files without a regrow; r5j logged five regrows per slot with
        // a one-stream layout, each a device-wide hipFree)
        constexpr uint32_t kPlanStreams = 256;
        std::vector<uint64_t> off0(kPlanStreams), len0(kPlanStreams);
        const uint64_t per = (g->batch_cap / kPlanStreams) & ~255ull;
        for (uint32_t i = 0; i < kPlanStreams; i++) {
            off0[i] = i * per;
            len0[i] = per;
        }
        if (rcdc_status ps = rcdc_plan_create(ctx, off0.data(), len0.data(), kPlanStreams,
                                              g->batch_cap + 256, &P.plan))
            return fail_st(ps);
        // ... and run once in that layout and in the one-stream layout (the
        // walk path's buffers at full size; the arena's bytes do not matter):
        // a plan's first run in a new layout allocated inside the pipeline,
        // and each allocation's hipFree waited for every queued copy and
        // kernel (r5u: 30-55 ms in each slot's first relayout)
        {
            std::vector<uint64_t> wc(g->batch_cap / 4096 + kPlanStreams + 16), wn(kPlanStreams);
            if (rcdc_status ps = rcdc_plan_run(P.plan, P.arena, nullptr)) return fail_st(ps);
            if (rcdc_status ps = rcdc_plan_results(P.plan, wc.data(), wc.size(), wn.data());
                ps && ps != RCDC_ERR_CAPACITY)
                return fail_st(ps);
            for (uint32_t ns : {1u, 2u, 4u, 16u}) {  // walked layouts of 1-16 streams
                std::vector<uint64_t> o(ns), l(ns);
                const uint64_t each = (g->batch_cap / ns) & ~255ull;
                for (uint32_t i = 0; i < ns; i++) {
                    o[i] = i * each;
                    l[i] = each;
                }
                if (rcdc_status ps = rcdc::plan_relayout(P.plan, o.data(), l.data(), ns,
                                                         g->batch_cap + 256, nullptr))
                    return fail_st(ps);
                if (rcdc_status ps = rcdc_plan_run(P.plan, P.arena, nullptr)) return fail_st(ps);
                if (rcdc_status ps = rcdc_plan_results(P.plan, wc.data(), wc.size(), wn.data());
                    ps && ps != RCDC_ERR_CAPACITY)
                    return fail_st(ps);
            }
        }
        // short-chunk refs for a batch of minimum-size chunks
        P.refs_cap = z.refs_cap;
        if ((e = ing_alloc(gp, &P.h_refs, P.refs_cap * 16, true)) != hipSuccess ||
            (e = ing_alloc(gp, &P.d_refs, P.refs_cap * 16, false)) != hipSuccess ||
            (e = ing_alloc(gp, &P.d_dig, P.refs_cap * 32, false)) != hipSuccess)
            return fail_hip(e, "refs");
    }
    if ((e = ing_alloc(gp, &g->frames, z.frames, false)) != hipSuccess) return fail_hip(e, "frames");
    g->frames_cap = z.frames;
    if ((e = ing_alloc(gp, &g->d_packs, z.frames, false)) != hipSuccess) return fail_hip(e, "packs");
    g->d_packs_cap = z.frames;
    if ((e = hipStreamCreateWithFlags(&g->s_in, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipStreamCreateWithFlags(&g->s_comp, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipStreamCreateWithFlags(&g->s_out, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipStreamCreateWithFlags(&g->s_back, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&g->ev_comp, hipEventDisableTiming)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&g->ev_back, hipEventDisableTiming)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&g->ev_out, hipEventDisableTiming)) != hipSuccess)
        return fail_hip(e, "streams");
    if ((e = hipEventRecord(g->ev_out, g->s_out)) != hipSuccess) return fail_hip(e, "event");
    for (uint32_t i = 0; i < g->nthreads; i++) g->pool.emplace_back(pool_main, gp);
    g->waiter = std::thread(waiter_main, gp);
    g->worker = std::thread(worker_main, gp);
    g->feeder = std::thread(feeder_main, gp);
    g->back = std::thread(back_main, gp);
    *out = g.release();
    return RCDC_OK;
}

rcdc_status rcdc_ingest_add_index(rcdc_ingest *g, const uint8_t *ids, uint64_t n) {
    if (!g || (n && !ids)) return set_error(RCDC_ERR_INVALID_INPUT, "null argument");
    std::lock_guard<std::mutex> lk(g->mu);
    if (g->nbatches) return set_error(RCDC_ERR_INVALID_INPUT, "index ids after the first batch");
    for (uint64_t i = 0; i < n; i++) {
        Id32 id;
        memcpy(id.b, ids + 32 * i, 32);
        g->idx->insert(id);
    }
    return RCDC_OK;
}

rcdc_status rcdc_ingest_reserve(rcdc_ingest *g, uint64_t len, uint8_t **buf, uint64_t *ticket) {
    if (!g || !buf || !ticket) return set_error(RCDC_ERR_INVALID_INPUT, "null argument");
    if (len > g->batch_cap)
        return set_error(RCDC_ERR_UNSUPPORTED,
                         "file larger than the ingest batch (batch_bytes): feed it as a stream "
                         "(rcdc_ingest_stream_open)");
    std::unique_lock<std::mutex> lk(g->mu);
    return reserve_locked(g, lk, len, nullptr, false, buf, ticket);
}

rcdc_status rcdc_ingest_commit(rcdc_ingest *g, uint64_t ticket, uint64_t tag, uint64_t len) {
    if (!g) return set_error(RCDC_ERR_INVALID_INPUT, "null argument");
    std::lock_guard<std::mutex> lk(g->mu);
    return commit_locked(g, ticket, tag, len, false);
}

rcdc_status rcdc_ingest_cancel(rcdc_ingest *g, uint64_t ticket) {
    if (!g) return set_error(RCDC_ERR_INVALID_INPUT, "null argument");
    std::lock_guard<std::mutex> lk(g->mu);
    return commit_locked(g, ticket, 0, 0, true);
}

rcdc_status rcdc_ingest_stream_open(rcdc_ingest *g, uint64_t tag, uint64_t size_hint,
                                    uint64_t *stream) {
    if (!g || !stream) return set_error(RCDC_ERR_INVALID_INPUT, "null argument");
    std::unique_lock<std::mutex> lk(g->mu);
    for (;;) {
        if (g->err) return set_error(g->err, g->err_msg.c_str());
        if (g->finishing) return set_error(RCDC_ERR_INVALID_INPUT, "ingest already finishing");
        if (!g->free_cslots.empty()) break;
        if (!g->closing_streams)
            return set_error(RCDC_ERR_UNSUPPORTED, "max_streams streams are open");
        // streams that ended free their carry slots once their last batch
        // has been chunked: send the open slot on its way
        close_open_locked(g);
        g->cv_slot.wait_for(lk, std::chrono::milliseconds(1));
    }
    auto st = std::make_shared<StreamSt>();
    st->handle = g->next_stream++;
    st->tag = tag;
    st->hint = size_hint;
    st->cslot = g->free_cslots.back();
    g->free_cslots.pop_back();
    g->streams[st->handle] = st;
    *stream = st->handle;
    return RCDC_OK;
}

rcdc_status rcdc_ingest_stream_reserve(rcdc_ingest *g, uint64_t stream, uint64_t len,
                                       uint8_t **buf, uint64_t *ticket) {
    if (!g || !buf || !ticket) return set_error(RCDC_ERR_INVALID_INPUT, "null argument");
    if (len > g->batch_cap)
        return set_error(RCDC_ERR_UNSUPPORTED, "piece larger than the ingest batch (batch_bytes)");
    std::unique_lock<std::mutex> lk(g->mu);
    auto st = find_stream(g, stream);
    if (!st) return set_error(RCDC_ERR_INVALID_INPUT, "unknown stream");
    st->open_pieces++;
    const rcdc_status rs = reserve_locked(g, lk, len, st, false, buf, ticket);
    if (rs) st->open_pieces--;
    return rs;
}

rcdc_status rcdc_ingest_stream_close(rcdc_ingest *g, uint64_t stream) {
    return stream_end(g, stream, false);
}

rcdc_status rcdc_ingest_stream_abort(rcdc_ingest *g, uint64_t stream) {
    return stream_end(g, stream, true);
}

rcdc_status rcdc_ingest_add(rcdc_ingest *g, uint64_t tag, const void *data, uint64_t len) {
    if (!g || (len && !data)) return set_error(RCDC_ERR_INVALID_INPUT, "null argument");
    uint8_t *buf;
    uint64_t t;
    if (len <= g->batch_cap) {
        rcdc_status s = rcdc_ingest_reserve(g, len, &buf, &t);
        if (s) return s;
        memcpy(buf, data, len);
        return rcdc_ingest_commit(g, t, tag, len);
    }
    // larger than a batch: a stream of quarter-batch pieces
    uint64_t h;
    if (rcdc_status s = rcdc_ingest_stream_open(g, tag, len, &h)) return s;
    const uint64_t piece = std::max<uint64_t>(g->batch_cap / 4 & ~255ull, 256);
    for (uint64_t o = 0; o < len; o += piece) {
        const uint64_t n = std::min(piece, len - o);
        rcdc_status s = rcdc_ingest_stream_reserve(g, h, n, &buf, &t);
        if (s) {
            (void)rcdc_ingest_stream_abort(g, h);
            return s;
        }
        memcpy(buf, (const uint8_t *)data + o, n);
        if ((s = rcdc_ingest_commit(g, t, 0, n))) {
            const std::string m = rcdc_last_error();
            (void)rcdc_ingest_cancel(g, t);  // (a failed commit leaves the piece open)
            (void)rcdc_ingest_stream_abort(g, h);
            return set_error(s, m.c_str());
        }
    }
    return rcdc_ingest_stream_close(g, h);
}

rcdc_status rcdc_ingest_flush(rcdc_ingest *g) {
    if (!g) return set_error(RCDC_ERR_INVALID_INPUT, "null argument");
    std::lock_guard<std::mutex> lk(g->mu);
    close_open_locked(g);
    return g->err ? set_error(g->err, g->err_msg.c_str()) : RCDC_OK;
}

rcdc_status rcdc_ingest_finish(rcdc_ingest *g, rcdc_ingest_stats *stats) {
    if (!g) return set_error(RCDC_ERR_INVALID_INPUT, "null argument");
    {
        std::unique_lock<std::mutex> lk(g->mu);
        if (!g->streams.empty())
            return set_error(RCDC_ERR_INVALID_INPUT, "streams still open (close or abort them first)");
        close_open_locked(g);
        g->finishing = true;
        g->cv_slot.notify_all();
        g->cv_done.wait(lk, [&] { return g->finished || g->err; });
        g->cv_done.wait(lk, [&] { return g->packs_pending == 0 || g->err; });
        g->st.seconds = g->t_first ? now_s() - g->t_first : 0;
        if (stats) *stats = g->st;
        if (g->prof) {
            std::lock_guard<std::mutex> lk2(g->cb_mu);
            for (size_t b = 0; b < g->tl.size(); b++) {
                fprintf(stderr, "ingest batch %zu:", b);
                for (double t : g->tl[b]) fprintf(stderr, " %.1f", t * 1e3);
                if (b < g->tl_d2h.size() && g->tl_d2h[b] > 0)
                    fprintf(stderr, " | landed %.1f", g->tl_d2h[b] * 1e3);
                if (b < g->tl_ids.size() && g->tl_ids[b] > 0)
                    fprintf(stderr, " ids %.1f", g->tl_ids[b] * 1e3);
                fprintf(stderr, " ms\n");
            }
            fprintf(stderr, "ingest end %.1f ms\n", g->st.seconds * 1e3);
        }
        if (g->err) return set_error(g->err, g->err_msg.c_str());
    }
    return RCDC_OK;
}

void rcdc_ingest_destroy(rcdc_ingest *g) {
    if (!g) return;
    {
        std::unique_lock<std::mutex> lk(g->mu);
        if (!g->finished && !g->err) {  // abandoned: stop after what is queued
            g->err = RCDC_ERR_INTERNAL;
            g->err_msg = "destroyed";
        }
        g->cv_slot.notify_all();
    }
    if (g->worker.joinable()) g->worker.join();
    if (g->feeder.joinable()) g->feeder.join();
    if (g->back.joinable()) g->back.join();
    {
        std::unique_lock<std::mutex> lk(g->mu);
        g->cv_done.wait_for(lk, std::chrono::seconds(30), [&] { return g->packs_pending == 0; });
    }
    g->stop = true;
    g->wait_cv.notify_all();
    g->pool_cv.notify_all();
    if (g->waiter.joinable()) g->waiter.join();
    for (auto &t : g->pool)
        if (t.joinable()) t.join();
    (void)hipSetDevice(g->device);
    (void)hipDeviceSynchronize();
    free_all(g);
    delete g;
}

rcdc_status rcdc_index_create(rcdc_index **out) {
    if (!out) return set_error(RCDC_ERR_INVALID_INPUT, "null argument");
    *out = new rcdc_index();
    return RCDC_OK;
}

void rcdc_index_destroy(rcdc_index *idx) { delete idx; }

rcdc_status rcdc_index_add(rcdc_index *idx, const uint8_t *ids, uint64_t n) {
    if (!idx || (n && !ids)) return set_error(RCDC_ERR_INVALID_INPUT, "null argument");
    for (uint64_t i = 0; i < n; i++) {
        Id32 id;
        memcpy(id.b, ids + 32 * i, 32);
        idx->insert(id);
    }
    return RCDC_OK;
}

uint64_t rcdc_index_size(const rcdc_index *idx) {
    return idx ? const_cast<rcdc_index *>(idx)->size() : 0;
}

rcdc_status rcdc_ingest_set_index(rcdc_ingest *g, rcdc_index *idx) {
    if (!g || !idx) return set_error(RCDC_ERR_INVALID_INPUT, "null argument");
    std::lock_guard<std::mutex> lk(g->mu);
    if (g->nbatches) return set_error(RCDC_ERR_INVALID_INPUT, "index set after the first batch");
    if (g->idx == idx) return RCDC_OK;
    for (auto &sh : g->idx->sh) {
        std::lock_guard<std::mutex> l2(sh.mu);
        for (const Id32 &id : sh.set) idx->insert(id);
    }
    if (g->own_idx) delete g->idx;
    g->idx = idx;
    g->own_idx = false;
    return RCDC_OK;
}

rcdc_status rcdc_sha256_host_one(const void *data, uint64_t len, uint8_t *digest) {
    if ((len && !data) || !digest) return set_error(RCDC_ERR_INVALID_INPUT, "null argument");
    host_sha256_one((const uint8_t *)data, len, digest);
    return RCDC_OK;
}

rcdc_status rcdc_sha256_host_ni(const void *const *ptrs, const uint64_t *lens, uint32_t n,
                                uint32_t ways, uint8_t *digests) {
    if (n && (!ptrs || !lens || !digests)) return set_error(RCDC_ERR_INVALID_INPUT, "null argument");
    for (uint32_t i = 0; i < n; i++)
        if (!ptrs[i] && lens[i]) return set_error(RCDC_ERR_INVALID_INPUT, "null buffer");
    if (ways < 1 || ways > 4) return set_error(RCDC_ERR_INVALID_INPUT, "ways must be 1-4");
    host_sha256_ni_many(reinterpret_cast<const uint8_t *const *>(ptrs), lens, n, digests,
                        (int)ways);
    return RCDC_OK;
}

}  // extern "C"
