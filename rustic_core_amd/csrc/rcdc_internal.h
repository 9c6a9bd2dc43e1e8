// rcdc_internal.h -- types shared by the HIP kernels and the host runtime.
//
// Data layout in HBM (see DESIGN.md "Data layout"):
//   arena      : caller's bytes; stream i = arena[off_i, off_i + N_i)
//   ScanItem[] : one per 64 consecutive segments of one stream (one wave)
//   Summary[]  : one uint4 per segment {first, last, count, 0}; first/last
//                are positions relative to the segment's first position,
//                0xFFFFFFFF = no candidate
//   item_mask[]: one u64 per ScanItem, bit l = segment l has a candidate
//   StreamDesc[]: resolver input per stream; cuts[] / counts[] its output
#pragma once
#include <stdint.h>

namespace rcdc {

constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr int kWindow = 64;          // Rabin64::new_with_polynom(6, ..) -> 2^6
constexpr uint64_t kRefBufSize = 4096;  // the reference's read buffer (rabin.rs:12): min >= it
constexpr int kScanThreads = 1024;   // 16 waves; one workgroup per CU
constexpr int kScanWaves = kScanThreads / 64;
constexpr int kTableRepl = 32;       // per-lane table copies: bank = lane % 32
constexpr uint32_t kTableBytes = 256u * kTableRepl * 8u;  // 64 KiB per table
constexpr uint32_t kLdsBytes = 2u * kTableBytes;          // OUT + MOD
constexpr uint32_t kUnit = 64;       // bytes per register unit (16 dwords)
constexpr int kDefaultScanCode = 30; // rcdc_scan.hip launch_scan configuration

// One wave of work: segments [sum_idx, sum_idx + nvalid) of one stream.
// Lane l scans bytes [q0 + l*S, q0 + l*S + 64 + S) of the arena and tests
// stream-relative positions pos0 + l*S + r, r in [0, S).
struct ScanItem {
    uint64_t q0;        // arena byte offset of lane 0's first byte (16-aligned)
    uint64_t pos0;      // stream position tested at r = 0 by lane 0
    uint64_t lo, hi;    // positions that matter: [lo, hi)
    uint64_t sum_idx;   // summary index of lane 0
    uint64_t rec_bytes; // buffer-descriptor range from q0 (<= 2^32 - 1)
    uint32_t nvalid;    // lanes with a segment (1..64)
    uint32_t stream;
    uint64_t pad;
};
static_assert(sizeof(ScanItem) == 64, "ScanItem is 64 B");

struct StreamDesc {
    uint64_t off;       // arena offset of byte 0
    uint64_t n;         // stream length
    uint64_t pos0;      // position of segment 0, r = 0
    uint64_t sum_base;  // summary index of segment 0
    uint64_t item_base; // item index of segment 0's item
    uint64_t nseg;      // segments of this stream
    uint64_t cut_base;  // first output slot
    uint64_t cut_cap;   // output slots
};
static_assert(sizeof(StreamDesc) == 64, "StreamDesc is 64 B");

struct ScanParams {
    uint32_t seg_bytes;  // S, multiple of 64
    uint32_t mask;       // avg - 1 (avg <= 2^32)
    uint32_t idx_shift;  // deg - 32: top-byte index from the high word
    uint32_t pad;
};

// Resolver work: one wave hops from `start` until its first cut >= `stop`.
// direct: a whole stream, cuts straight to the stream's output slots;
// otherwise a speculative piece of a long stream (piece_cuts[out_base ..]).
struct ResolveUnit {
    uint64_t start, stop;
    uint64_t out_base;
    uint32_t out_cap;
    uint32_t stream;
    uint32_t direct;
    uint32_t pad;
};
static_assert(sizeof(ResolveUnit) == 40, "ResolveUnit is 40 B");

// One long stream: pieces units[unit0 .. unit0 + npieces).
struct StitchDesc {
    uint32_t stream, unit0, npieces, pad;
};

struct ResolveParams {
    uint64_t min_size, max_size;
    uint32_t seg_bytes;
    uint32_t mask;
    uint32_t shift;  // deg - 8
    uint32_t pad;
};

// ---- walk path (long streams; rcdc_walk.hip) --------------------------------
// A long stream is split into pieces [start, stop).  One wave walks the chunk
// chain of each piece from its start, hashing only what the reference hashes:
// per chunk the 64 min-zone positions and the pure windows from s + min + 64
// to the cut (rabin.rs:127-188 never hashes a chunk's first min bytes).  Piece
// starts other than 0 are assumptions; rcdc_walk_check_kernel finds where the
// true chain meets each piece's chain, rcdc_walk_fixup_kernel walks the rare
// stretches where it does not, rcdc_walk_assemble_kernel writes the result.

// Cut value | kind << 62 in piece lists: what the walker verified before it.
constexpr uint64_t kCutVal = (1ull << 62) - 1;
constexpr uint64_t kKindHit = 0;   // first pure-window hit >= s + min + 64
constexpr uint64_t kKindMax = 1;   // s + max: no hit in [s + min + 64, s + max)
constexpr uint64_t kKindEof = 2;   // N: no hit in [s + min + 64, N) (or N - s <= min)
constexpr uint64_t kKindZone = 3;  // a min-zone / all-zero-prefill cut: nothing scanned
constexpr uint64_t kOpenFlag = 1ull << 32;  // piece status: walk stopped "open"

struct WalkUnit {
    uint64_t start, stop;  // assumed chunk start (exact for piece 0); next piece's start or N
    uint64_t out_base;     // first slot in piece_cuts
    uint32_t out_cap;
    uint32_t stream;
    uint32_t piece;        // index within the stream
    uint32_t unit0;        // unit index of the stream's piece 0
    uint32_t npieces;
    uint32_t nbig;         // the stream's first nbig pieces are Lp long, the rest Ls
};
static_assert(sizeof(WalkUnit) == 48, "WalkUnit is 48 B");

struct WalkParams {
    uint64_t min_size, max_size;
    uint64_t arena_len;
    uint64_t piece_bytes;  // Lp: the (big) piece size
    uint64_t small_bytes;  // Ls: the size of a stream's last (split) pieces
    uint32_t seg_bytes;    // S: bytes per lane per round
    uint32_t mask;         // avg - 1
    uint32_t idx_shift;    // deg - 32
    uint32_t shift;        // deg - 8
    uint32_t nunits;
    uint32_t fix_cap;      // fixup cut slots per boundary
    uint32_t fix_seg;      // S for the fixup walker (latency-bound: smaller rounds)
    uint32_t seed_classes; // queue classes by piece index mod K (seeded starts)
    // kWalkStat* counters (always on: one atomic per piece / fixup boundary)
    unsigned long long *stats;
    // optional per-piece trace (nullptr = off): kTraceWords u64 per unit
    unsigned long long *trace;
    // queue order of the walk kernel: the q-th piece handed out is order[q]
    const uint32_t *order;
    // cost ordering (nullptr = off): the plan's static order (big pieces,
    // then small ones) and the buffer the per-run sort writes `order` into
    const uint32_t *order_in;
    uint32_t *order_out;
    uint32_t nbig_units;   // order_in[0, nbig_units) are big pieces
    uint32_t helpers;      // idle walk waves hash rounds ahead for the busy ones: at
                           // most this many per round of the walker's own (0 = off)
    uint64_t chk_budget;   // bytes of gap hashing a boundary check may do before
                           // it hands the boundary to the fixup kernel
    // Seeded piece starts (this run's buffer set, 2 x nunits words): [0, nunits)
    // a piece's end state when its walker finished, one word published by one
    // atomic store (end_word: kEndOpen | epoch | the open chunk's start or its
    // last cut; position kEndNone: list truncated), [nunits, 2 nunits) the
    // chain start its walker used (kSeed* << 62 | position).  A walker whose
    // previous piece is already done in this run (the word carries this run's
    // epoch) continues that piece's chain instead of assuming a cut at its own
    // start.  One word, so no fences: an acquire would invalidate the XCD's
    // L2 under the other waves' streams.
    uint64_t *wstate;
    uint64_t epoch;        // this run's, 1 .. 2^21 - 1 (the buffers start zeroed)
    uint32_t seed;         // seeding on
    uint32_t early;        // hit rounds stop early, the owed tails spread over the lanes
    // The walk queue counter (ctr[0]) is never reset: every wave of a walk
    // adds 1 per piece it takes and 1 for the failed take that ends it, so a
    // run adds nunits + waves and the next run of the buffer set starts at
    // qbase (mod 2^32).  The walk kernel itself zeroes the chain counters
    // ctr[1..3] and `stats` of its set at its start (no memsets between
    // walks on the hashing queue).
    uint32_t qbase;
    uint32_t flags;        // kWalk* below (A/B switches, all on by default)
    // kWalkKReset: `stats` is slot r % 4 of four (run r); the walk kernel
    // zeroes slot (r + 2) % 4, run r - 2's, whose chain has finished (the
    // run waited for it) and which run r + 2 uses after this run's chain.  A
    // walk cannot zero its own slot: its workgroups run on all XCDs, and one
    // on a busy XCD may start after the others have added their counters.
    unsigned long long *stats_next;
    uint32_t cost_blocks;  // workgroups of the cost kernel (1024 threads; > 256: the old
                           // thousands-of-256-thread grid, A/B via RCDC_COST_BLOCKS)
    uint32_t cost_samples; // 8-byte words the cost kernel samples per piece (16-64;
                           // each pulls a whole cache line: RCDC_COST_SAMPLES A/B)
};
constexpr uint32_t kWalkZoneFast = 1;  // zones on the scan's slide (zone_wave_fast)
constexpr uint32_t kWalkKReset = 2;    // counters reset in the walk kernel, queue by qbase
// kWalkStatic: a wave's first piece (walk) or boundary (check) is its global
// wave index, only later ones come from the queue counter: with one atomic
// per wave at the start, thousands of waves queued on one L2 address (C5:
// 3200 one-piece waves, the median piece 82 us, mostly that wait).  A walk
// then adds exactly nunits to ctr[0] (one failed take per wave that had a
// static piece, one take per dynamic piece).
constexpr uint32_t kWalkStatic = 4;

constexpr uint64_t kEndOpen = 1ull << 63;
constexpr uint64_t kEndPos = (1ull << 42) - 1;  // position bits of an end word
constexpr uint64_t kEndNone = kEndPos;          // position: no usable end state
constexpr uint32_t kEpochShift = 42;            // epoch bits 42..62
__host__ __device__ inline uint64_t end_word(bool open, uint64_t epoch, uint64_t pos) {
    return (open ? kEndOpen : 0ull) | (epoch << kEpochShift) | (pos & kEndPos);
}
__host__ __device__ inline uint64_t end_epoch(uint64_t w) { return (w >> kEpochShift) & ((1ull << 21) - 1); }
constexpr uint64_t kSeedNone = 0;    // speculative: a cut assumed at the piece start
constexpr uint64_t kSeedClosed = 1;  // the chain starts at the previous piece's last cut
constexpr uint64_t kSeedOpen = 2;    // the chain continues the previous piece's open chunk

// WalkParams.stats slots
constexpr int kWalkStatRounds = 0;     // walk kernel: 64-lane hashing rounds
constexpr int kWalkStatZones = 1;      // walk kernel: zone evaluations (64 x 64 slides)
constexpr int kWalkStatChunks = 2;     // walk kernel: chunks emitted (incl. zero-run ones)
constexpr int kWalkStatFixRounds = 3;  // fixup kernel: 1024-lane rounds
constexpr int kWalkStatFixZones = 4;   // fixup kernel: zone evaluations
constexpr int kWalkStatFixCuts = 5;    // fixup kernel: cuts walked
constexpr int kWalkStatChkRounds = 6;  // check kernel: 64-lane rounds over unsearched gaps
constexpr int kWalkStatChkZones = 7;   // check kernel: zone evaluations
constexpr int kWalkStatBytes = 8;      // walk kernel: bytes its rounds hashed (64 x (S + 64) each)
constexpr int kWalkStatChkBytes = 9;   // check kernel: bytes its gap rounds hashed
constexpr int kWalkStats = 10;
// trace per unit: wall clock (100 MHz) at start and end, rounds, chunks
constexpr int kTraceWords = 4;

constexpr int kMaxHops = 13;  // chain steps the check kernel resolves itself

// Per boundary (indexed by the unit of the later piece).
struct BoundRes {
    uint32_t kind;         // kBoundNone / Merged / Fixup / Bad
    uint32_t nhops;        // hops[] cuts before the merge
    uint32_t merge_unit;   // Merged: continue in this unit's list
    int32_t merge_idx;     //   after this index (-1: the whole list)
    uint64_t fix_from;     // Fixup: exact cut the fixup walk starts from
    uint64_t hops[kMaxHops];
};
static_assert(sizeof(BoundRes) == 16 * 8, "BoundRes is 128 B");
constexpr uint32_t kBoundNone = 0, kBoundMerged = 1, kBoundFixup = 2, kBoundEnd = 3;

// Per fixup boundary: cuts in fix_cuts[unit * fix_cap ..].
struct FixRes {
    uint32_t count;
    uint32_t merge_unit;   // 0xFFFFFFFF: ran to N (or overflowed: count > fix_cap)
    int32_t merge_idx;
    uint32_t pad;
};

// ---- blob encryption (rcdc_aead.hip) ---------------------------------------
constexpr uint32_t kAeadUnitBlocks = 4096;  // 16-byte blocks per wave work unit (64 KiB)

struct AeadKeyDev {
    uint32_t rk256[60];    // AES-256 round keys (big-endian column words)
    uint32_t rk128[44];    // AES-128 round keys of Poly1305-AES's k
    uint32_t rpow[65][5];  // r^0 .. r^64, 26-bit limbs (r clamped)
    uint32_t r2j[32][5];   // r^(2^j)
    uint32_t te[256];      // T-table: (2S, S, S, 3S) as a big-endian word
};

constexpr uint32_t kAeadAppendLen = 1;  // seal: write u32 LE (len + 32) after the tag

struct AeadBlob {  // 48 B
    uint64_t in_off;   // seal: plaintext; open: nonce || ct || tag
    uint64_t len;      // plaintext / ciphertext bytes
    uint64_t out_off;  // seal: nonce || ct || tag; open: plaintext (any alignment)
    uint32_t nonce[4]; // the nonce's bytes as 4 little-endian words
    uint32_t flags;    // kAeadAppendLen: a pack header (packfile.rs PackHeaderLength)
    uint32_t pad;
};
static_assert(sizeof(AeadBlob) == 48, "AeadBlob is 48 B");

struct AeadUnit {  // 16 B
    uint32_t blob;
    uint32_t b0, b1;   // block range [b0, b1) of the blob
    uint32_t pad;
};

// ---- blob compression (rcdc_zstd.hip) --------------------------------------
// A blob becomes one zstd frame (RFC 8878): header, then its bytes cut into
// blocks of kZstdBlock, each stored raw, as RLE, or compressed (raw literals +
// sequences coded with the predefined FSE tables).  Matches stay inside their
// block.
constexpr uint32_t kZstdBlock = 128u * 1024u;     // ZSTD_BLOCKSIZE_MAX
// Frames of blobs above kZstdSingleMax bytes are not single-segment: they
// declare a 2^kZstdWindowLog window (rcdc_zstd_frame_kernel)
constexpr uint32_t kZstdSingleMax = 1u << 27;
constexpr uint32_t kZstdWindowLog = 20;
constexpr uint32_t kZstdSlot = kZstdBlock + 64u;  // scratch per block: compressed content
constexpr uint32_t kZstdMaxSeq = kZstdBlock / 4u + 1u;  // matches are >= 4 bytes
constexpr uint32_t kZstdTypeRaw = 0, kZstdTypeRle = 1, kZstdTypeComp = 2;

struct ZstdBlob {  // 32 B
    uint64_t in_off;   // the blob's bytes in the input
    uint64_t out_off;  // where its frame starts in the output
    uint32_t len;
    uint32_t blk0;     // its blocks: [blk0, blk0 + nblk) of this launch
    uint32_t nblk;
    uint32_t pad;
};
static_assert(sizeof(ZstdBlob) == 32, "ZstdBlob is 32 B");

struct ZstdBlk {  // 16 B
    uint32_t blob;
    uint32_t start;    // offset in the blob
    uint32_t len;      // <= kZstdBlock
    uint32_t flags;    // bit 0: the blob's first block, bit 1: its last
};

// FSE compression tables of the predefined distributions (RFC 8878
// 3.1.1.3.2.2) in the layout of zstd's FSE_buildCTable: per symbol
// {deltaFindState, deltaNbBits}, then the state tables; plus the code tables.
struct ZstdFseSym {
    int32_t find;
    uint32_t nbits;
};
struct ZstdTables {
    ZstdFseSym ll[36];
    ZstdFseSym ml[53];
    ZstdFseSym of[32];
    uint16_t llst[64];
    uint16_t mlst[64];
    uint16_t ofst[32];
    uint8_t llcode[64];   // literal length < 64 -> code
    uint8_t mlcode[128];  // match length - 3 < 128 -> code
    uint8_t llbits[36];
    uint8_t mlbits[53];
    uint8_t pad[3];
};
static_assert(sizeof(ZstdTables) % 4 == 0, "ZstdTables is copied as words");

}  // namespace rcdc
