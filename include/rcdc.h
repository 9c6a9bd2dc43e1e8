/*
 * rcdc.h -- C ABI of librcdc, the MI355X-native content-defined chunker that
 * replaces rustic_core's Rabin CDC hot path.
 *
 * Drop-in point (reference = rustic_core 0.12.0, /root/reference):
 *   crates/core/src/chunker.rs:21-58  ChunkIter::from_config(&ConfigFile, R, size_hint)
 *                                     + Iterator<Item = RusticResult<Vec<u8>>>
 *   crates/core/src/chunker/rabin.rs:82-191  RabinChunkIter::{new, next}
 * called from crates/core/src/archiver/file_archiver.rs:144-160
 * (FileArchiver::backup_reader), one iterator per file on pariter workers
 * (crates/core/src/archiver.rs:195).
 *
 * Contract: every function returns cut offsets (END offset of each chunk,
 * i.e. the prefix sums of the chunk lengths the reference iterator yields)
 * that are bit-identical to what rabin.rs ChunkIter::next produces on the
 * same bytes with the same (poly, min, avg, max).  A Rust `ChunkIter::Gpu`
 * variant slices its buffer at these offsets.
 *
 * Plain C types only (pointers + sizes); no HIP or torch types appear in a
 * signature.  Device pointers are passed as `const void *` / `uint64_t`.
 * All entry points are thread-safe for distinct contexts/streams/plans; one
 * context may be shared by any number of threads (a pool of per-call lanes,
 * see the host-stream section).  A stream or plan is used by one thread at
 * a time.
 */
#ifndef RCDC_H
#define RCDC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RCDC_ABI_VERSION 5u

/* Status codes map onto rustic_core ErrorKind (crates/core/src/error.rs:108-124). */
typedef enum {
    RCDC_OK = 0,
    RCDC_ERR_UNSUPPORTED = 1,   /* ErrorKind::Unsupported  (rabin.rs:22-40)           */
    RCDC_ERR_INVALID_INPUT = 2, /* ErrorKind::InvalidInput (configfile.rs:166-171)     */
    RCDC_ERR_INTERNAL = 3,      /* ErrorKind::Internal     (HIP runtime failures)      */
    RCDC_ERR_INPUT_OUTPUT = 4,  /* ErrorKind::InputOutput  (rabin.rs:131-138,174-180)  */
    RCDC_ERR_CAPACITY = 5,      /* caller's cut buffer too small; counts still valid   */
    RCDC_ERR_VERIFICATION = 6   /* ErrorKind::Verification (decrypt.rs:516-526)       */
} rcdc_status;

typedef struct rcdc_ctx rcdc_ctx;       /* one device + chunker parameters      */
typedef struct rcdc_stream rcdc_stream; /* one file fed in pieces               */
typedef struct rcdc_plan rcdc_plan;     /* a fixed batch layout in device memory */

typedef struct {
    const uint8_t *data; /* host pointer (rcdc_chunk_batch)                */
    uint64_t len;
} rcdc_buf;

/* ---- parameters -------------------------------------------------------- */

/* check_rabin_params -- replaces crates/core/src/chunker/rabin.rs:17-42.
 * avg must be a power of two, min <= avg <= max.  Additionally rejected with
 * RCDC_ERR_UNSUPPORTED: min < 4096 and max > 2^40.  Below 4096 the
 * reference's `min_size -= open_buf_len` (rabin.rs:124, up to 4095 bytes of
 * its 4 KiB read buffer, rabin.rs:12) underflows -- a panic under debug
 * assertions, a read-pattern-dependent wrap in release -- so no bit-exact
 * cut list exists for such parameters.                                     */
rcdc_status rcdc_check_params(uint64_t avg, uint64_t min, uint64_t max);

/* ConfigFile::poly -- replaces crates/core/src/repofile/configfile.rs:165-175
 * (u64::from_str_radix(hex, 16)); RCDC_ERR_INVALID_INPUT on a bad string.   */
rcdc_status rcdc_parse_poly(const char *hex, uint64_t *poly);

/* ---- context ------------------------------------------------------------ */

/* Replaces Rabin64::new_with_polynom(6, &poly) + RabinChunkIter::new
 * (crates/core/src/chunker.rs:29-38, rabin.rs:82-104).  Builds the Rabin64
 * out/mod tables once per context (the reference rebuilds them per file) and
 * uploads them to `device`.  deg(poly) must be in [9, 56].                  */
rcdc_status rcdc_ctx_create(uint64_t poly, uint64_t min, uint64_t avg_pow2,
                            uint64_t max, int device, rcdc_ctx **out);
void rcdc_ctx_destroy(rcdc_ctx *ctx);

/* Message of the last failing call on this thread ("" if none). */
const char *rcdc_last_error(void);

/* Upper bound on the number of chunks of an n-byte stream. */
uint64_t rcdc_max_cuts(const rcdc_ctx *ctx, uint64_t n);

/* ---- independent host streams (per-file parallel path, archiver.rs:195) - */

/* Host-buffer calls (rcdc_chunk_batch, rcdc_stream_feed) may come from many
 * threads at once on one context, as the reference runs one ChunkIter per
 * file on pariter workers (archiver.rs:195).  Each call takes one of the
 * context's lanes -- a HIP stream, two pinned staging slots and a device
 * arena of its own -- for its duration, so concurrent calls overlap instead
 * of serialising; at most RCDC_LANES (environment, default 16) lanes exist,
 * further callers wait for a free one.  The caller's pageable bytes go
 * through the staging slots in 16 MiB blocks, the copy of block k + 1
 * overlapping the DMA of block k.                                          */

/* Chunk n independent host buffers; only the cut offsets come back.  Cuts of
 * stream i are written consecutively to cuts[] in stream order;
 * cut_counts[i] receives the count.  If the total exceeds cuts_cap,
 * RCDC_ERR_CAPACITY is returned with every cut_counts[i] valid and cuts[]
 * untouched (call again with a larger buffer).                            */
rcdc_status rcdc_chunk_batch(rcdc_ctx *ctx, const rcdc_buf *bufs, uint32_t n,
                             uint64_t *cuts, uint64_t cuts_cap,
                             uint64_t *cut_counts);

/* ---- one file fed in pieces (the Read-driven iterator) ------------------ */

/* Replaces the read loop of rabin.rs:110-191: the caller feeds the file in
 * arbitrary pieces (any split gives the same cuts, like the reference's
 * read()-independence).  Cut offsets (absolute, from the start of the file)
 * become final as enough bytes arrive; each call hands out up to `cap` of
 * them (*n_cuts) and keeps the rest queued for the next call -- a call with
 * len = 0 only drains the queue, and rcdc_stream_queued() tells how many
 * wait.  A feed never fails for lack of cut space and never consumes input
 * twice.  is_final = 1 marks EOF (the reference's Ok(0)); the last cut is
 * then the file length.
 * Retention: the stream buffers bytes until rcdc_stream_batch_bytes(ctx)
 * (16 MiB, at least 2 max + 256; environment RCDC_STREAM_BATCH) would be
 * pending, then runs one device pass over the buffered tail plus the new
 * piece, straight from the caller's buffer; afterwards it keeps only the
 * tail after the last final cut (< max bytes).  So at most batch + max
 * bytes are held -- more than the reference's 4 KiB + one chunk, for one
 * device pass per 16 MiB instead of a byte loop per chunk.
 * On an HIP failure the bytes stay buffered and the status is returned;
 * the feed may be retried with len = 0 (same is_final).                    */
rcdc_status rcdc_stream_open(rcdc_ctx *ctx, rcdc_stream **out);
rcdc_status rcdc_stream_feed(rcdc_stream *st, const uint8_t *data,
                             uint64_t len, int is_final, uint64_t *cuts,
                             uint64_t cap, uint64_t *n_cuts);
uint64_t rcdc_stream_queued(const rcdc_stream *st);
uint64_t rcdc_stream_batch_bytes(const rcdc_ctx *ctx);
void rcdc_stream_close(rcdc_stream *st);

/* ---- device-resident batches (the measured hot path) ------------------- */

/* A plan fixes a batch layout: n streams at byte offsets offs[i] (any
 * alignment) with lengths lens[i] inside a device arena of arena_len bytes.
 * It owns the device work lists, per-segment summaries and the cut output.
 * Requires the arena base pointer passed to rcdc_plan_run to be 256-B
 * aligned (hipMalloc / torch allocations are).                             */
rcdc_status rcdc_plan_create(rcdc_ctx *ctx, const uint64_t *offs,
                             const uint64_t *lens, uint32_t n,
                             uint64_t arena_len, rcdc_plan **out);
void rcdc_plan_destroy(rcdc_plan *plan);

/* Enqueue scan + resolve on `hip_stream` (a hipStream_t, or 0 for the
 * context's own stream) over the device arena `d_arena`.  Asynchronous. */
rcdc_status rcdc_plan_run(rcdc_plan *plan, const void *d_arena,
                          void *hip_stream);

/* Complete the last run on the host side: wait for it and, for any long
 * stream whose walk-path fixup overflowed its slots (never seen outside
 * forced tests), re-chunk it on the scan path and write its cuts -- and, if
 * the run was hashed, its digests -- back into the device buffers.  Until
 * this returns the device arena of the run must stay unchanged; after it,
 * the device views below are complete.  rcdc_plan_results and
 * rcdc_plan_digests call it.                                                */
rcdc_status rcdc_plan_finish(rcdc_plan *plan);

/* Finish the last run and copy the results to the host: same layout and
 * capacity rule as rcdc_chunk_batch.                                      */
rcdc_status rcdc_plan_results(rcdc_plan *plan, uint64_t *cuts,
                              uint64_t cuts_cap, uint64_t *cut_counts);

/* Device-side view of the results: stream i's cuts are
 * d_cuts[cut_base[i] .. cut_base[i] + d_counts[i]).  Complete after
 * rcdc_plan_finish; before it, a stream whose walk needs host completion
 * reads d_counts[i] == UINT64_MAX (and its digests are not written).
 * Ordering: a serial run's last kernel is ordered before later work on the
 * run's stream (for hip_stream = 0, before later work on the legacy default
 * stream too).  A pipelined run (rcdc_plan_set_pipeline) ends on a stream
 * of the plan's own and is NOT ordered before the caller's later work on any
 * stream: call rcdc_plan_finish (or synchronise the device) before reading
 * these buffers from device code.                                          */
rcdc_status rcdc_plan_device_results(rcdc_plan *plan, uint64_t *d_cuts,
                                     uint64_t *d_counts,
                                     const uint64_t **cut_base);

/* Crossing window of stream `stream` of the last run, for stitching one
 * stream sliced over GPUs (each rank runs a plan over its slice
 * plus a max + 64 byte halo).  Writes 3 + k words to the device buffer d_out
 * (8-B aligned), asynchronously on hip_stream (0: the context's stream),
 * ordered after the run: [0] the stream's cut count n, [1] j = the index of
 * its first cut >= bound (n if none), [2] that cut (UINT64_MAX if none),
 * [3 + t] cut t for t < k (UINT64_MAX for t >= n).  Cuts are relative to the
 * stream's first byte.  n == UINT64_MAX: the stream needs rcdc_plan_finish
 * (never seen outside forced tests); the caller then reads the host list.   */
rcdc_status rcdc_plan_window(rcdc_plan *plan, uint32_t stream, uint64_t bound, uint32_t k,
                             uint64_t *d_out, void *hip_stream);

/* Pipelined runs: with enable = 1, run k's hashing kernels (scan, walk) go
 * to hashing stream k % 2 of the plan's own (after the caller's earlier
 * work) and its chain kernels (resolve; walk check / fixup / assemble) to a
 * third stream, so run k's chain overlaps run k + 1's hashing; every
 * per-run buffer the chain reads alternates between two sets, and run
 * k + 2's hashing waits for run k's chain.  rcdc_plan_results /
 * rcdc_plan_hash wait for the last chain; a caller that reuses the arena
 * must synchronise the device (or call rcdc_plan_results) first.  The plan
 * then uses three streams: HIP maps a process's streams onto
 * GPU_MAX_HW_QUEUES hardware queues (4 by default), and kernels whose
 * streams share a queue run in order, so a caller that adds streams of its
 * own around a pipelined plan can serialise its chain with the next walk
 * (bench.py runs pipelined plans on the default stream).  enable = 0
 * restores serial runs.  enable = 2: pipelined, and the next run is the
 * last of the sequence: its chain kernels run on every CU instead of beside
 * a next walk (a pipeline flush; one-shot, later runs are narrow again).    */
rcdc_status rcdc_plan_set_pipeline(rcdc_plan *plan, int enable);

/* Scan-kernel geometry chosen by the plan (for profiling / roofline). */
typedef struct {
    uint64_t scanned_bytes;   /* bytes the scan kernel must hash         */
    uint64_t segments;        /* per-lane segments                       */
    uint32_t segment_bytes;   /* S                                        */
    uint32_t work_items;      /* 64-segment wave work items               */
    uint32_t scan_blocks;     /* workgroups of the scan launch            */
    uint32_t walk_pieces;     /* pieces of long streams on the walk path  */
    uint32_t walk_seg_bytes;  /* S of the walk kernel's 64-lane rounds    */
    uint32_t pad;
} rcdc_plan_info;
rcdc_status rcdc_plan_get_info(const rcdc_plan *plan, rcdc_plan_info *info);

/* Kernel timing (HIP events recorded on the launch stream around the scan
 * and the resolve kernel while enabled).  enable = P >= 1 starts a fresh
 * accumulation and times every P-th run from the next one on (P = 1: every
 * run; a larger P samples the runs and keeps the events' own inter-kernel
 * gaps out of most of them); 0 stops recording.  rcdc_plan_kernel_times
 * waits for the timed runs and returns their count and summed device times. */
rcdc_status rcdc_plan_set_timing(rcdc_plan *plan, int enable);
rcdc_status rcdc_plan_kernel_times(rcdc_plan *plan, uint64_t *runs,
                                   double *scan_ms_total,
                                   double *resolve_ms_total);

/* Work counters of the walk path (long streams) of the last run, after it
 * completes: stats[0] 64-lane hashing rounds of rcdc_walk_kernel, [1] its
 * min-zone evaluations (64 windows of 64 bytes), [2] chunks it emitted, [3]
 * 1024-lane rounds of the fixup kernel (1024 x (512 + 64) bytes each), [4]
 * fixup zones, [5] cuts the fixups walked, [6] 64-lane rounds of the
 * boundary check kernel over bytes no walker searched, [7] its zone
 * evaluations, [8] the bytes the walk kernel's rounds hashed (64 x (S + 64)
 * per round; the last round of a search with a known end -- a piece's stop,
 * a chunk's max, EOF -- hashes only the 64-byte units it needs), [9] the
 * same for the check kernel's rounds.  With the environment variable
 * RCDC_WALK_TRACE=1 at plan creation, `trace` (if not NULL) receives 4
 * words per walk piece: wall clock (100 MHz) at the piece's start and end,
 * rounds, chunks; then 4 words per piece boundary (rows of piece 0 unused)
 * from the check kernel: start, end, gap rounds, hop entries -- at most
 * trace_cap words (2 x walk_pieces x 4 in all).  All zero for plans without
 * walked streams.                                                          */
#define RCDC_WALK_STATS 10
rcdc_status rcdc_plan_walk_stats(rcdc_plan *plan, uint64_t *stats, uint64_t *trace,
                                 uint64_t trace_cap);

/* ---- FixedSize chunker (crates/core/src/chunker/fixed_size.rs:41-70) ---- */
/* Cuts every `size` bytes, last chunk short; returns the count.           */
uint64_t rcdc_fixed_cuts(uint64_t n, uint64_t size, uint64_t *cuts,
                         uint64_t cap);

/* ---- SHA-256 blob ids: crypto/hasher.rs:17-19 `hash(&chunk)`, called per
 * chunk by FileArchiver::backup_reader (archiver/file_archiver.rs:151) ---- */

/* One chunk of a device arena: bytes [off, off + len). */
typedef struct {
    uint64_t off;
    uint64_t len;
} rcdc_chunk_ref;

/* SHA-256 of n chunks of a device arena.  d_refs (16-B aligned) and
 * d_digests (32 bytes per chunk, 4-B aligned) are device pointers.
 * Asynchronous on hip_stream (0: the context's stream).                    */
rcdc_status rcdc_sha256_chunks(rcdc_ctx *ctx, const void *d_arena,
                               const rcdc_chunk_ref *d_refs, uint32_t n,
                               uint8_t *d_digests, void *hip_stream);

/* SHA-256 of n buffers in host memory (pack ids: blob/packer.rs:832-834
 * `hash_reader` of each finished pack file), on the calling thread: 16
 * messages side by side in the lanes of AVX-512 registers, a lane taking the
 * next message when its own ends.  digests: 32 bytes per buffer.
 * RCDC_ERR_UNSUPPORTED on a CPU without AVX-512F/BW (no digest written).   */
rcdc_status rcdc_sha256_host(const void *const *ptrs, const uint64_t *lens, uint32_t n,
                             uint8_t *digests);

/* Page-locked host memory for read buffers.  Host-buffer calls
 * (rcdc_stream_feed, rcdc_chunk_batch) whose pieces all lie in such memory
 * copy them to the device by DMA straight from the caller's buffer, with no
 * staging copy.  The reference reads into a Vec (rabin.rs:110-191); this is
 * the buffer a caller's read loop would fill instead.  rcdc_host_free(NULL)
 * is a no-op.                                                              */
rcdc_status rcdc_host_alloc(uint64_t bytes, void **out);
void rcdc_host_free(void *p);

/* Fused blob ids of a plan: after rcdc_plan_run over d_arena (the same
 * pointer), enqueue the SHA-256 of every chunk it found, on the device
 * cut list (no host round trip).  Asynchronous.                           */
rcdc_status rcdc_plan_hash(rcdc_plan *plan, const void *d_arena,
                           void *hip_stream);

/* rcdc_plan_hash for up to 8 plans of one context in a single launch (plan
 * j over d_arenas[j], its last run's arena), so their chunks share the
 * longest-chunk latency floor instead of queueing per stream.            */
rcdc_status rcdc_plan_hash_many(rcdc_plan *const *plans, uint32_t n,
                                const void *const *d_arenas, void *hip_stream);

/* Synchronise and copy the digests to the host: 32 bytes per chunk, in the
 * order of rcdc_plan_results' cuts (whose counts it also writes).          */
rcdc_status rcdc_plan_digests(rcdc_plan *plan, uint8_t *digests,
                              uint64_t cap_chunks, uint64_t *cut_counts);

/* Device view: slot-indexed like rcdc_plan_device_results' d_cuts. */
rcdc_status rcdc_plan_device_digests(rcdc_plan *plan, uint64_t *d_digests);

/* ---- blob encryption: crypto/aespoly1305.rs:88-135 `Key::encrypt_data` /
 * `decrypt_data` (aes256ctr_poly1305aes 0.2.1, the restic format), applied
 * by the packer to every new blob (blob/packer.rs:268-270,
 * backend/decrypt.rs:566-572) -- here to chunks already in HBM. ---------- */

/* One blob.  seal: data [in_off, in_off + len) of d_in becomes
 * nonce || AES-256-CTR ciphertext || Poly1305-AES tag (len + 32 bytes) at
 * out_off of d_out.  open: the sealed blob [in_off, in_off + len) (len >= 32)
 * becomes its len - 32 plaintext bytes at out_off.  Offsets may have any
 * alignment (16-byte aligned outputs store fastest; allow 4 readable bytes
 * after each input).  The nonce is the caller's (rustic draws it at random,
 * :120-121). */
typedef struct {
    uint64_t in_off;
    uint64_t len;
    uint64_t out_off;
    uint8_t nonce[16]; /* seal only; open reads it from the blob */
} rcdc_aead_ref;

/* key: 64 bytes, AES-256 key || Poly1305-AES k || r (aespoly1305.rs:15-24).
 * refs is a HOST array.  Asynchronous on hip_stream (0: the context's
 * stream); calls on one context take turns (the second waits for the
 * first's kernels).                                                         */
rcdc_status rcdc_aead_seal(rcdc_ctx *ctx, const uint8_t *key, const void *d_in,
                           const rcdc_aead_ref *refs, uint32_t n, void *d_out,
                           void *hip_stream);
/* status[i] (host array): 0 = MAC ok, 1 = MAC mismatch or shorter than
 * nonce + tag (ErrorKind::Cryptography, aespoly1305.rs:97-108; the plaintext
 * written is then not to be used), 2 = shorter than 16 bytes (:89-94).
 * Synchronous.                                                              */
rcdc_status rcdc_aead_open(rcdc_ctx *ctx, const uint8_t *key, const void *d_in,
                           const rcdc_aead_ref *refs, uint32_t n, void *d_out,
                           uint32_t *status, void *hip_stream);

/* ---- pack files: blob/packer.rs:615-655 (add_raw), :693-735 (save,
 * write_header) and repofile/packfile.rs (HeaderEntry, PackHeaderRef) -- the
 * packer's byte work for blobs in HBM: each pack is its blobs sealed back to
 * back, then the sealed pack header, then its length (u32 LE). ---------- */

typedef struct {
    uint64_t in_off;           /* the blob's bytes in d_in (as stored: the raw blob, or the
                                  zstd frame of a compressed one)                         */
    uint32_t len;              /* bytes at in_off                                          */
    uint32_t uncompressed_len; /* 0: stored as is (HeaderEntry Data / Tree); else the raw
                                  length of a compressed blob (CompData / CompTree)       */
    uint32_t type;             /* BlobType: 0 data, 1 tree                                 */
    uint32_t pad;
    uint8_t id[32];            /* blob id                                                  */
    uint8_t nonce[16];
} rcdc_pack_blob;              /* 72 B */

typedef struct {
    uint64_t out_off;          /* where the pack file starts in d_out                      */
    uint32_t blob0, nblobs;    /* its blobs, in pack order: blobs[blob0 .. blob0 + nblobs) */
    uint8_t header_nonce[16];
    uint64_t size;             /* out: pack file bytes                                     */
    uint32_t header_len;       /* out: sealed header bytes (the trailing u32)              */
    uint32_t pad;
} rcdc_pack;                   /* 48 B */

/* Build npacks pack files in d_out (out_len bytes).  blobs and packs are HOST
 * arrays; blob_offsets (optional, host, nblobs) receives each blob's offset
 * in its pack (IndexBlob location.offset; its length is len + 32).  Grouping
 * blobs into packs (PackSizer, packer.rs:65-200) and the pack id (SHA-256
 * of the file, packer.rs:833) stay with the caller.  Asynchronous on
 * hip_stream; the outputs of `packs` are set on return.                     */
rcdc_status rcdc_pack_build(rcdc_ctx *ctx, const uint8_t *key, const void *d_in,
                            const rcdc_pack_blob *blobs, uint32_t nblobs, rcdc_pack *packs,
                            uint32_t npacks, void *d_out, uint64_t out_len,
                            uint32_t *blob_offsets, void *hip_stream);

/* The same with blobs sealed already (packer.rs:615-655 add_raw: the packer
 * appends encrypted data): blobs[i].len is the sealed length (>= 32, nonce +
 * ciphertext + tag) of the bytes at in_off, copied into the pack as they are
 * (nonce ignored); only the headers are sealed here.                        */
rcdc_status rcdc_pack_build_raw(rcdc_ctx *ctx, const uint8_t *key, const void *d_in,
                                const rcdc_pack_blob *blobs, uint32_t nblobs, rcdc_pack *packs,
                                uint32_t npacks, void *d_out, uint64_t out_len,
                                uint32_t *blob_offsets, void *hip_stream);

/* rcdc_pack_build_raw over blobs that lie in several device buffers (sealed
 * in different passes, or carried over from an earlier call while their pack
 * was still open, packer.rs:659-671): blob i's bytes are at
 * d_ins[blobs[i].pad] + in_off; pad >= n_ins is InvalidInput.              */
rcdc_status rcdc_pack_build_raw_multi(rcdc_ctx *ctx, const uint8_t *key,
                                      const void *const *d_ins, uint32_t n_ins,
                                      const rcdc_pack_blob *blobs, uint32_t nblobs,
                                      rcdc_pack *packs, uint32_t npacks, void *d_out,
                                      uint64_t out_len, uint32_t *blob_offsets,
                                      void *hip_stream);

/* Device byte ranges gathered into one buffer: bytes [in_off, in_off + len)
 * of d_ins[src] go to out_off of d_out (any alignment).  refs is a HOST
 * array.  Returns once the copy has run (it is ordered on hip_stream).  Used
 * to keep an open pack's sealed blobs alive across ingest calls.           */
typedef struct {
    uint64_t in_off;
    uint64_t out_off;
    uint64_t len;
    uint32_t src;
    uint32_t pad;
} rcdc_copy_ref; /* 32 B */
rcdc_status rcdc_copy_ranges(rcdc_ctx *ctx, const void *const *d_ins, uint32_t n_ins,
                             const rcdc_copy_ref *refs, uint32_t n, void *d_out,
                             void *hip_stream);

/* ---- blob compression: backend/decrypt.rs:478-506 (`encode_all(data,
 * level)` before `Key::encrypt_data` when the repository is version 2,
 * configfile.rs:177-186), applied by the packer's process_data
 * (blob/packer.rs:268-270) -- here to chunks already in HBM.  Each blob
 * becomes one zstd frame (RFC 8878) that any zstd decoder reads back (rustic's
 * decode_all, decrypt.rs:71-95); the bytes are this library's own, not
 * libzstd's (no zstd version promises another's output).               ---- */

/* One blob: bytes [in_off, in_off + len) of d_in become a frame at out_off of
 * d_out, at most rcdc_zstd_bound(len) bytes.  Any alignment. */
typedef struct {
    uint64_t in_off;
    uint64_t len;      /* < 2^32 (decrypt.rs:479-487: the length is a u32) */
    uint64_t out_off;
} rcdc_zstd_ref;

/* Worst-case frame size of a len-byte blob (header + stored blocks):
 * len + 3 per 128 KiB block + 9, + 10 above 2^27 bytes (those frames carry a
 * window descriptor: rustic's decode_all refuses windows above 2^27 + 1, and
 * a single-segment frame's window is its content size). */
uint64_t rcdc_zstd_bound(uint64_t len);

/* Compress n blobs (refs is a HOST array).  level: zstd's range
 * [-131072, 22] (0 = zstd's default, level 3: rustic's choice for version 2);
 * out-of-range -> InvalidInput.  The level picks the parse: <= 1 keys
 * positions on 6 bytes (6-byte minimum match, fastest), 2-3 on 4 bytes,
 * >= 4 also doubles the hash table to 2^12 positions (better ratio on
 * structured data, half the waves per CU).  On return (synchronous)
 * out_lens[i] (host) holds blob i's frame length.  Calls on one context take
 * turns.  The context keeps its scratch after the first call: up to 4 GiB of
 * per-block slots (batches of more than 32768 blocks run in windows) and
 * 1 GiB of per-wave sequence buffers, freed by rcdc_ctx_destroy.  A/B
 * overrides (process environment): RCDC_ZSTD_HLOG (11 / 12), RCDC_ZSTD_KEY
 * (4 / 6).                                                                  */
rcdc_status rcdc_zstd_compress(rcdc_ctx *ctx, int level, const void *d_in,
                               const rcdc_zstd_ref *refs, uint32_t n, void *d_out,
                               uint64_t *out_lens, void *hip_stream);

/* ---- frame check: backend/decrypt.rs:508-529 (`very_data`, on by default:
 * extra_verify, repofile/configfile.rs:198): after compressing a blob the
 * packer decodes it again and compares it with the input.  Here every frame
 * is decoded on the device and compared with its blob in place. ---------- */

/* Frame [frame_off, frame_off + frame_len) of d_frames is expected to decode
 * to [data_off, data_off + data_len) of d_data (allow 4 readable bytes after
 * each range). */
typedef struct {
    uint64_t frame_off;
    uint64_t frame_len;
    uint64_t data_off;
    uint64_t data_len;
} rcdc_zstd_check_ref;

/* Decode n frames (refs is a HOST array) and compare them with their blobs:
 * status[i] (host) = 0 the frame decodes to exactly the blob (RFC 8878: any
 * block and literal type, 1 or 4 Huffman streams, predefined / RLE / FSE /
 * repeat sequence tables, repeat offsets, matches into earlier blocks),
 * 1 it decodes to other bytes or another length (ErrorKind::Verification,
 * decrypt.rs:516-526), 2 malformed or not readable here (a dictionary, a
 * skippable frame, bytes after the frame).  A frame checksum is skipped.
 * Malformed means what decode_all's decoder refuses on the path it would
 * take: one pass when the declared content size fits its first 8 KiB
 * read, otherwise the streaming stage machine (a window above 2^27 + 1
 * bytes is refused there, and empty blocks of any type are skipped).
 * flags bit 0 (RCDC_CHECK_STORED): the "frames" are stored bytes (blobs of an
 * uncompressed repository), compared as they are.  Synchronous.  Calls on one context take turns; the context keeps a
 * 128 KiB literal scratch per resident wave (256 MiB on 256 CUs).          */
rcdc_status rcdc_zstd_check(rcdc_ctx *ctx, const void *d_frames, const void *d_data,
                            const rcdc_zstd_check_ref *refs, uint32_t n, uint32_t flags,
                            uint32_t *status, void *hip_stream);
#define RCDC_CHECK_STORED 1u

/* The FSE coding tables the kernels use (predefined distributions, RFC 8878
 * 3.1.1.3.2.2), copied to out (rcdc_zstd_tables_size() bytes): for tests. */
void rcdc_zstd_tables(void *out);
uint64_t rcdc_zstd_tables_size(void);

/* ---- the backup data path, host memory to host memory (ABI 4, 5) -------
 * FileArchiver::backup_reader (archiver/file_archiver.rs:144-160) for many
 * files: chunk, `hash(&chunk)`, `index.has_data`, Packer::add -- zstd at the
 * repository's level, Key::encrypt_data, extra_verify (backend/decrypt.rs:
 * 478-529) -- PackSizer / should_save (blob/packer.rs:65-200, 659-671), the
 * sealed header (:693-735) and the pack id, SHA-256 of the pack file
 * (hash_reader, :826-836).  One engine per backup (per device): the packer
 * stays open across files and batches, and rcdc_ingest_finish closes the
 * last pack (Packer::finalize, :385-398).
 *
 * Files enter page-locked input slots.  Two ways in:
 *  - a file of known size: rcdc_ingest_reserve hands out space for it (the
 *    node's size; at most batch_bytes), the caller reads the file into it
 *    (the Read of rabin.rs:110-191) and rcdc_ingest_commit hands it over
 *    (fewer bytes than reserved are fine);
 *  - any Read, of any or unknown length (a file larger than a batch, stdin,
 *    a child's stdout: commands/backup.rs:336-346): rcdc_ingest_stream_open,
 *    then pieces -- rcdc_ingest_stream_reserve + rcdc_ingest_commit, each
 *    piece any size up to batch_bytes, the stream's bytes in reservation
 *    order -- then rcdc_ingest_stream_close (EOF).  The size is only a hint
 *    (chunker.rs:22-47, size_hint): cuts never depend on how the bytes were
 *    split into pieces or batches.  The engine carries each stream's open
 *    chunk (at most max bytes) from batch to batch on the device, as
 *    rcdc_stream_feed does for the chunk-only path.
 * Reserve / commit may be called from many threads (archiver.rs:195).  A
 * reservation whose read fails is dropped with rcdc_ingest_cancel (the
 * reference logs and skips the file, archiver.rs:197-203); a stream whose
 * read fails is ended with rcdc_ingest_stream_abort (the chunks it completed
 * before the error stay packed, as the reference's Packer::add calls did).
 * A slot that fills (or whose first file is slot_max_age_ms old) becomes a
 * device batch: H2D, chunking, the short chunks' ids on the device, the long
 * ones' on host threads, zstd + seal + verify of every chunk, then (once the
 * ids are in) dedup in chunk order, packs, D2H and the pack ids on host
 * threads.  Results come back through callbacks: per file (or stream) its
 * cut offsets and chunk ids in file order (the tree's content list), per
 * pack the pack file in host memory (valid during the call), its id and its
 * index entries.  Callbacks run on the engine's threads, one at a time.
 *
 * Memory (rcdc_ingest_footprint gives the exact figures for a config):
 * page-locked in_slots x batch_bytes + out_slots x (batch_bytes + 1/16 +
 * 64 MiB) -- 16.75 GiB at the defaults (4 + 4 slots of 2 GiB) -- and on
 * the device depth x (2 x batch_bytes + max_streams x max + a sealed-blob
 * staging area of ~batch_bytes) plus two batch-sized compression / pack
 * buffers: ~30 GiB at the defaults, about a tenth of an MI355X's HBM.      */
typedef struct rcdc_ingest rcdc_ingest;

typedef struct {
    uint8_t key[64];            /* aespoly1305 Key: AES-256 || Poly1305-AES k || r     */
    int32_t zstd_level;         /* repository version 2: zstd level (0 = zstd's 3)     */
    uint32_t compress;          /* 1: version 2 compression; 0: stored blobs           */
    uint32_t extra_verify;      /* 1: decrypt, decode and compare every blob (default) */
    uint32_t hash_threads;      /* host SHA-256 threads (default 10)                   */
    uint64_t pack_size;         /* PackSizer (configfile.rs:211-231): default 32 MiB,  */
    uint64_t pack_grow_factor;  /*   grow factor 32,                                    */
    uint64_t pack_size_limit;   /*   limit u32::MAX,                                    */
    uint64_t pack_current_size; /*   the repository's data pack bytes so far           */
    uint64_t batch_bytes;       /* input slot / device batch bytes (default 2 GiB)     */
    uint32_t depth;             /* batches in flight on the device (default 4)         */
    uint32_t in_slots;          /* page-locked input slots (default 4)                 */
    uint32_t out_slots;         /* page-locked pack buffers (default 4)                */
    uint32_t max_streams;       /* streams open at once (default 16; each holds a
                                   device carry of max bytes)                          */
    uint64_t long_chunk;        /* chunks above this get their id on the host (2 MiB) */
    uint32_t pack_max_age_ms;   /* should_save's MAX_AGE (packer.rs:63,668-670): an open
                                   pack this old is saved (default 300000 = 5 min)      */
    uint32_t slot_max_age_ms;   /* an open input slot whose first file is this old is
                                   submitted unfilled (default 1000)                   */
} rcdc_ingest_config;

typedef struct {
    uint8_t id[32];
    uint32_t offset;              /* in the pack (IndexBlob location)              */
    uint32_t length;              /* sealed bytes                                  */
    uint32_t uncompressed_length; /* 0: stored as is                               */
    uint32_t type;                /* BlobType: 0 data                              */
} rcdc_ingest_blob;               /* 48 B */

typedef struct {
    const uint8_t *data;          /* the pack file (valid during the callback)     */
    uint64_t size;
    uint64_t seq;                 /* packer order                                  */
    uint8_t id[32];               /* SHA-256 of the pack file                      */
    uint32_t nblobs, header_len;
    const rcdc_ingest_blob *blobs;
} rcdc_ingest_pack;

typedef struct {
    uint64_t tag;                 /* the caller's (rcdc_ingest_commit / _stream_open) */
    uint64_t len;
    uint32_t nchunks, nnew;       /* chunks; those the packer added                */
    const uint64_t *cuts;         /* end offset of each chunk in the file          */
    const uint8_t *ids;           /* 32 B per chunk                                */
} rcdc_ingest_file_result;

typedef struct {
    uint64_t bytes_in, files, chunks, new_blobs, packs, pack_bytes, batches;
    double seconds;               /* first batch submitted .. last pack delivered  */
} rcdc_ingest_stats;

typedef void (*rcdc_ingest_pack_fn)(void *user, const rcdc_ingest_pack *pack);
typedef void (*rcdc_ingest_file_fn)(void *user, const rcdc_ingest_file_result *file);

void rcdc_ingest_config_default(rcdc_ingest_config *cfg);
/* Bytes rcdc_ingest_create allocates for cfg on ctx: page-locked host memory
 * and device memory (the engine's own buffers; the context's scratch and the
 * plans' work lists come on top).                                          */
rcdc_status rcdc_ingest_footprint(const rcdc_ctx *ctx, const rcdc_ingest_config *cfg,
                                  uint64_t *pinned_bytes, uint64_t *device_bytes);
/* Allocates the slots (page-locked and device memory for a full batch
 * each) and starts the engine's threads.  On failure nothing stays
 * allocated.                                                               */
rcdc_status rcdc_ingest_create(rcdc_ctx *ctx, const rcdc_ingest_config *cfg,
                               rcdc_ingest_pack_fn pack_cb, rcdc_ingest_file_fn file_cb,
                               void *user, rcdc_ingest **out);
/* Ids the repository's index already has (Indexer::has): before the first file. */
rcdc_status rcdc_ingest_add_index(rcdc_ingest *ing, const uint8_t *ids, uint64_t n);
/* Space for one file of len bytes (<= batch_bytes); waits for a free slot. */
rcdc_status rcdc_ingest_reserve(rcdc_ingest *ing, uint64_t len, uint8_t **buf, uint64_t *ticket);
/* The file's (or piece's) bytes are in place: its first len bytes (<= the
 * reservation).  tag: the file's (ignored for a stream piece). */
rcdc_status rcdc_ingest_commit(rcdc_ingest *ing, uint64_t ticket, uint64_t tag, uint64_t len);
/* Drop a reservation that will not be committed (its read failed): no
 * result for it, and rcdc_ingest_finish does not wait for it.  For a stream
 * piece: the piece is empty (end the stream with rcdc_ingest_stream_abort). */
rcdc_status rcdc_ingest_cancel(rcdc_ingest *ing, uint64_t ticket);
/* reserve + memcpy + commit of a file already in memory (a file larger than
 * batch_bytes goes in as a stream of pieces). */
rcdc_status rcdc_ingest_add(rcdc_ingest *ing, uint64_t tag, const void *data, uint64_t len);

/* One file (any Read) fed in pieces: ChunkIter::from_config(cfg, reader,
 * size_hint) (chunker.rs:22-47) + its iterator (rabin.rs:110-191).  size_hint
 * is only a hint (0: unknown).  Waits while max_streams streams are closing;
 * RCDC_ERR_UNSUPPORTED if max_streams are open.  *stream: the handle.      */
rcdc_status rcdc_ingest_stream_open(rcdc_ingest *ing, uint64_t tag, uint64_t size_hint,
                                    uint64_t *stream);
/* Space for the stream's next len bytes (<= batch_bytes); commit it with
 * rcdc_ingest_commit(ticket, 0, n).  Consecutive pieces of one stream that
 * land in the same slot are laid out back to back. */
rcdc_status rcdc_ingest_stream_reserve(rcdc_ingest *ing, uint64_t stream, uint64_t len,
                                       uint8_t **buf, uint64_t *ticket);
/* EOF (Ok(0), rabin.rs:164-166): the stream's last chunk ends at its last
 * byte, and its file result (all cuts and ids, in order) follows.  Every
 * piece must be committed or cancelled first.  The handle is then invalid. */
rcdc_status rcdc_ingest_stream_close(rcdc_ingest *ing, uint64_t stream);
/* The stream's read failed: the chunk in progress is dropped, no file
 * result is delivered; chunks it completed before stay packed.  The handle
 * is then invalid. */
rcdc_status rcdc_ingest_stream_abort(rcdc_ingest *ing, uint64_t stream);

/* Submit the partly filled slot now. */
rcdc_status rcdc_ingest_flush(rcdc_ingest *ing);
/* No more files: process everything, close the last pack, wait for every
 * callback; stats (optional) receives the totals.  A verification failure
 * is RCDC_ERR_VERIFICATION.  Every stream must be closed or aborted.       */
rcdc_status rcdc_ingest_finish(rcdc_ingest *ing, rcdc_ingest_stats *stats);
void rcdc_ingest_destroy(rcdc_ingest *ing);

/* ---- one dedup set for several engines (multi-device ingest) ------------
 * The reference has ONE Packer per backup, so a blob is stored once however
 * many file workers found it (archiver.rs:195, blob/packer.rs:304-315, the
 * index check of file_archiver.rs:153).  N engines -- one per GPU, fed by a
 * file router -- keep that property by sharing one id set: an engine packs
 * a chunk only if its insert into the set is the first.  The set is
 * thread-safe (sharded locks).                                             */
typedef struct rcdc_index rcdc_index;
rcdc_status rcdc_index_create(rcdc_index **out);
void rcdc_index_destroy(rcdc_index *idx);       /* after every engine using it */
/* Ids the repository already has (Indexer::has). */
rcdc_status rcdc_index_add(rcdc_index *idx, const uint8_t *ids, uint64_t n);
uint64_t rcdc_index_size(const rcdc_index *idx);
/* Dedup against idx (not the engine's own set) from now on; before the
 * engine's first batch.  Ids already given to rcdc_ingest_add_index move
 * into idx.                                                                */
rcdc_status rcdc_ingest_set_index(rcdc_ingest *ing, rcdc_index *idx);

/* Page-locked and device bytes currently held by all ingest engines of the
 * process (their own buffers, as rcdc_ingest_footprint counts them).        */
void rcdc_ingest_mem_live(uint64_t *pinned_bytes, uint64_t *device_bytes);

/* SHA-256 of one host buffer on the calling thread (SHA extensions when the
 * CPU has them): a pack id (packer.rs:832-834) where latency matters.      */
rcdc_status rcdc_sha256_host_one(const void *data, uint64_t len, uint8_t *digest);
/* SHA-256 of n host buffers on the calling thread, up to `ways` (1-4) of
 * them interleaved on the SHA extensions (one message's rounds are one
 * dependency chain; independent chains fill the unit's idle cycles): more
 * bytes per second per core than rcdc_sha256_host_one at about the same
 * latency per buffer.  Without SHA extensions: one buffer at a time.       */
rcdc_status rcdc_sha256_host_ni(const void *const *ptrs, const uint64_t *lens, uint32_t n,
                                uint32_t ways, uint8_t *digests);

/* ABI version of the loaded library (== RCDC_ABI_VERSION). */
uint32_t rcdc_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* RCDC_H */
