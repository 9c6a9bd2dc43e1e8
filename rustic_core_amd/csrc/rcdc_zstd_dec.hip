// rcdc_zstd_dec.hip -- zstd frames read back on the device: the extra_verify
// check of rustic's packer (backend/decrypt.rs:508-529 `very_data`: after
// compress + seal, decrypt and decompress the blob again and compare it with
// the input; on by default, configfile.rs:198 extra_verify) for blobs in HBM.
//
// rcdc_zstd_check_kernel: one wave per frame (RFC 8878), frames taken from an
// atomic queue in the host's order (longest first).  The wave decodes every
// block the way any conforming decoder does (frame header, raw / RLE /
// compressed blocks; raw / RLE / Huffman / treeless literals with 1 or 4
// streams and direct or FSE-coded weights; predefined / RLE / FSE / repeat
// sequence tables; repeat offsets; matches reaching into earlier blocks) and
// compares what it decodes with the blob's bytes instead of writing it:
//   - a raw or RLE block, or a sequence's literals, is compared with the
//     blob's bytes at the output position (literals decoded into a per-wave
//     scratch first: 4 Huffman streams on lanes 0-3);
//   - a match of offset o at output position p is compared as
//     data[p + i] == data[p - o + i]: by induction everything before p
//     already equals the data, so the data itself stands in for the decoded
//     output and the comparison has no order (overlapping matches included).
// Sequences are decoded 64 at a time by the whole wave (uniform code: every
// lane steps the same FSE states) and lane j keeps sequence j; a prefix sum
// places them and each lane compares its own (sequences longer than 256 bytes
// are compared by the whole wave afterwards).
// Status per frame: 0 = decodes to exactly the blob, 1 = decodes to other
// bytes or another length, 2 = malformed or a feature this reader lacks
// (dictionaries, skippable frames, more than one frame).  A frame checksum,
// when present, is skipped (the blob comparison is the stronger check).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "rcdc_internal.h"

using namespace rcdc;

// RCDC_ZSTD_DBG bit 3: wall-clock sums (100 MHz) over compressed blocks:
// literals section, sequences, whole block; literals, sequences, blocks
__device__ unsigned long long g_zck_prof[8];

namespace {

constexpr uint32_t kCkOk = 0, kCkMismatch = 1, kCkCorrupt = 2;
constexpr uint32_t kCkSeq = 3;  // block-parallel pass: re-check the frame in order
constexpr uint32_t kBlockMax = 128u << 10;

// Predefined distributions (RFC 8878 3.1.1.3.2.2) and code -> (baseline,
// extra bits) of literal and match lengths (3.1.1.3.2.1.1).
__constant__ int16_t kLLNorm[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                    2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
__constant__ int16_t kMLNorm[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                    1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                    1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
__constant__ int16_t kOFNorm[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                    1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
__constant__ uint32_t kLLBase[36] = {0,  1,  2,  3,  4,  5,   6,   7,   8,    9,    10,   11,
                                     12, 13, 14, 15, 16, 18,  20,  22,  24,   28,   32,   40,
                                     48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
__constant__ uint8_t kLLBits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  1,  1,
                                    1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ uint32_t kMLBase[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16,
                                     17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30,
                                     31, 32, 33, 34, 35, 37, 39, 41, 43, 47, 51, 59, 67, 83,
                                     99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
__constant__ uint8_t kMLBits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1,
                                    2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};

struct FseD {  // FSE decoding entry (FSE_decode_t)
    uint8_t sym, nb;
    uint16_t next;
};
struct HufD {
    uint8_t sym, nb;
};

// LDS of one wave (workgroup = one wave).  The Huffman tables live only
// through a block's literals section (its literals are decoded to scratch
// memory) and the LL / ML extras only through its sequences section, so the
// two share bytes: 9984 B per wave, 16 waves per CU by LDS (14464 B and 11
// waves before).  A treeless literals section rebuilds the Huffman table from
// the weights kept in w.
struct DecLds {
    FseD ll[512], ml[512], of[256];
    union {
        struct {
            FseD hw[64];  // FSE table of Huffman weights (log <= 6)
            HufD huf[2048];
        } h;
        // per LL / ML state: the code's baseline | extra bits << 24 (as
        // zstd's ZSTD_seqSymbol), so a sequence's lengths need one LDS read
        // each and no dependent constant-table lookup
        struct {
            uint32_t llx[512], mlx[512];
        } x;
    } u;
    int16_t norm[64];  // (read_ncount's capacity: kNormCap)
    uint16_t nxt[64];  // per symbol: <= 53 (ML), <= 64 by kNormCap
    uint8_t w[256];    // Huffman weights (kept for treeless literals)
    uint32_t pf[8];    // the sequence reader's next group, loaded straight to LDS
};
constexpr uint32_t kNormCap = 64;

__device__ __forceinline__ uint32_t highbit32(uint32_t v) { return 31u - (uint32_t)__clz(v); }

__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __syncthreads();
}

// Frames, blobs and the literal scratch are global memory: loads through a
// global-address-space pointer are global_load (counted by vmcnt only).  A
// generic pointer gives flat_load, which also counts in lgkmcnt, so every
// LDS wait of the sequence loop (its table reads) also waited for the
// bitstream's prefetch loads in flight (r5zpmc ISA: 24 flat loads in the
// decode loop).
template <typename T>
__device__ __forceinline__ const __attribute__((address_space(1))) T *gptr(const T *p) {
    return (const __attribute__((address_space(1))) T *)p;
}

// 4 bytes at any alignment from the aligned dwords that hold them (a dword
// holding a readable byte is readable: allocations are 4-byte granular).
__device__ __forceinline__ uint32_t ld4u(const uint8_t *p) {
    const uint32_t b = (uint32_t)(uintptr_t)p & 3u;
    const auto *w = gptr((const uint32_t *)(p - b));
    const uint32_t lo = w[0];
    const uint32_t hi = w[b ? 1 : 0];
    return __builtin_amdgcn_alignbit(hi, lo, b * 8u);
}

// n (<= 8) little-endian bytes at p; bytes outside [lo, hi) read as 0.
__device__ uint64_t ld8b(const uint8_t *p, const uint8_t *lo, const uint8_t *hi) {
    if (p >= lo && p + 8 <= hi)
        return (uint64_t)ld4u(p) | (uint64_t)ld4u(p + 4) << 32;
    uint64_t v = 0;
    for (int i = 0; i < 8; i++)
        if (p + i >= lo && p + i < hi) v |= (uint64_t)p[i] << (8 * i);
    return v;
}

// Backward bitstream (RFC 8878 4.1): bits [0, pos) unread, read from the top;
// bits below 0 read as zeros (a read that goes below 0 is an overflow).
struct BRev {
    const uint8_t *base;
    int64_t len;
    int64_t pos;
    int64_t cb;      // cache holds bits [cb, cb + 64)
    uint64_t cache;
};

__device__ __forceinline__ void brev_fill(BRev &r) {
    r.cb = ((r.pos - 57) >> 3) << 3;  // arithmetic shift: floor
    r.cache = ld8b(r.base + (r.cb >> 3), r.base, r.base + r.len);
}

// false: empty stream or no end mark
__device__ bool brev_init(BRev &r, const uint8_t *p, int64_t len) {
    r.base = p;
    r.len = len;
    if (len <= 0) return false;
    const uint32_t last = p[len - 1];
    if (last == 0) return false;
    r.pos = 8 * (len - 1) + (int64_t)highbit32(last);
    brev_fill(r);
    return true;
}

__device__ __forceinline__ uint64_t brev_peek(BRev &r, uint32_t n) {
    if (n == 0) return 0;
    const int64_t lo = r.pos - (int64_t)n;
    if (lo < r.cb) brev_fill(r);
    return (r.cache >> (uint32_t)(lo - r.cb)) & ((1ull << n) - 1ull);
}

__device__ __forceinline__ uint64_t brev_bits(BRev &r, uint32_t n) {
    const uint64_t v = brev_peek(r, n);
    r.pos -= n;
    return v;
}

// The same bitstream read through a 64-bit window that slides down 32 bits
// at a time, with the next 4-8 dwords (two 16-byte groups) already loaded or
// in flight: a refill never waits on memory.  Reads are at most 32 bits.
// Invariant: the window holds bits [B, B + 64) and B <= pos (pos - B < 64);
// g0.w is the dword of bits [B - 32, B), then g0.z, g0.y, g0.x, g1.w, ...
struct BRevQ {  // 32-bit positions: the scalar unit has no 64-bit signed compare
    const uint8_t *base;
    int32_t len;
    int32_t pos;
    int32_t B;
    uint64_t acc;
    uint4 g0, g1;
    uint32_t used;  // dwords of the original g0 shifted in (0..3)
    // LDS prefetch (the wave-uniform sequence reader): the group after g0,
    // bytes [nbyte, nbyte + 16), loaded by the global_load_lds of lanes 0-4
    // into pf when g0 was taken and read 4 slides later.  With the dwords
    // loaded into registers and aligned at once, every 4th slide waited for
    // a memory round trip; keeping them in VGPRs spilled (128 VGPRs).
    __attribute__((address_space(3))) uint32_t *pf;
    int32_t nbyte;
};

// A wave-uniform value in a scalar register: the serial sequence decode then
// runs on the scalar unit (a wave64 VALU op takes 4 cycles for one useful
// lane; r5j: 0.7 us per sequence, VALU-issue bound).
__device__ __forceinline__ uint32_t rfl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t rfl64(uint64_t v) {
    return (uint64_t)rfl((uint32_t)v) | (uint64_t)rfl((uint32_t)(v >> 32)) << 32;
}

// 4 bytes at base + byte (any alignment), bytes outside [0, len) as 0; U:
// the reader is wave-uniform (every lane reads the same stream)
template <bool U = false>
__device__ __forceinline__ uint32_t brq_ld4(const uint8_t *base, int64_t len, int64_t byte) {
    uint32_t v = 0;
    if (byte >= 0 && byte + 4 <= len) {
        v = ld4u(base + byte);
    } else {
        for (int i = 0; i < 4; i++)
            if (byte + i >= 0 && byte + i < len) v |= (uint32_t)gptr(base)[byte + i] << (8 * i);
    }
    return U ? rfl(v) : v;
}

// the 16 bytes [byte, byte + 16) as dwords x (lowest) .. w
template <bool U = false>
__device__ __forceinline__ uint4 brq_ld16(const uint8_t *base, int64_t len, int64_t byte) {
    return make_uint4(brq_ld4<U>(base, len, byte), brq_ld4<U>(base, len, byte + 4),
                      brq_ld4<U>(base, len, byte + 8), brq_ld4<U>(base, len, byte + 12));
}

// issue the next group's load into LDS (lanes 0-4, one dword each; no wait)
__device__ __forceinline__ void brq_fetch_lds(BRevQ &r, int32_t byte) {
    r.nbyte = byte;
    if (byte < 0 || byte + 20 > r.len) return;  // (the stream's ends: slow path)
    const uint8_t *a = r.base + byte;
    const uint32_t *w = (const uint32_t *)(a - ((uintptr_t)a & 3u));
    const uint32_t lane = __lane_id();
    if (lane < 5)
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void *)(w + lane), r.pf, 4, 0, 0);
}

// the fetched group, wave-uniform (x lowest)
__device__ __forceinline__ uint4 brq_take_lds(BRevQ &r) {
    if (r.nbyte < 0 || r.nbyte + 20 > r.len) return brq_ld16<true>(r.base, r.len, r.nbyte);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the wave's LDS load has landed
    const uint32_t sh = (uint32_t)((uintptr_t)(r.base + r.nbyte) & 3u) * 8u;
    const uint32_t w0 = r.pf[0], w1 = r.pf[1], w2 = r.pf[2], w3 = r.pf[3], w4 = r.pf[4];
    return make_uint4(rfl(__builtin_amdgcn_alignbit(w1, w0, sh)), rfl(__builtin_amdgcn_alignbit(w2, w1, sh)),
                      rfl(__builtin_amdgcn_alignbit(w3, w2, sh)), rfl(__builtin_amdgcn_alignbit(w4, w3, sh)));
}

template <bool U = false>
__device__ __forceinline__ bool brq_init(BRevQ &r, const uint8_t *p, int64_t len64) {
    if (len64 <= 0 || len64 > (1 << 27)) return false;  // streams of one block
    int32_t len = (int32_t)len64;
    if (U) {
        p = reinterpret_cast<const uint8_t *>(rfl64(reinterpret_cast<uintptr_t>(p)));
        len = (int32_t)rfl((uint32_t)len);
    }
    r.base = p;
    r.len = len;
    const uint32_t last = U ? rfl(p[len - 1]) : p[len - 1];
    if (last == 0) return false;
    r.pos = 8 * (len - 1) + (int32_t)highbit32(last);
    r.B = ((r.pos >> 5) << 5) - 32;  // arithmetic shifts: floor
    const int32_t by = r.B >> 3;
    r.acc = (uint64_t)brq_ld4<U>(p, len, by) | (uint64_t)brq_ld4<U>(p, len, by + 4) << 32;
    r.g0 = brq_ld16<U>(p, len, by - 16);
    if (U && r.pf)
        brq_fetch_lds(r, by - 32);
    else
        r.g1 = brq_ld16<U>(p, len, by - 32);
    r.used = 0;
    return true;
}

template <bool U = false>
__device__ __forceinline__ void brq_slide(BRevQ &r) {
    r.acc = (r.acc << 32) | r.g0.w;
    r.B -= 32;
    r.g0.w = r.g0.z;
    r.g0.z = r.g0.y;
    r.g0.y = r.g0.x;
    if (++r.used == 4) {
        if (U && r.pf) {
            r.g0 = brq_take_lds(r);
            brq_fetch_lds(r, (r.B >> 3) - 32);
        } else {
            r.g0 = r.g1;
            r.g1 = brq_ld16<U>(r.base, r.len, (r.B >> 3) - 32);
        }
        r.used = 0;
    }
}

template <bool U = false>
__device__ __forceinline__ uint32_t brq_peek(BRevQ &r, uint32_t n) {
    if (n == 0) return 0;
    const int32_t lo = r.pos - (int32_t)n;
    if (lo < r.B) brq_slide<U>(r);
    return (uint32_t)((r.acc >> (uint32_t)(lo - r.B)) & ((1ull << n) - 1ull));
}

template <bool U = false>
__device__ __forceinline__ uint32_t brq_bits(BRevQ &r, uint32_t n) {
    const uint32_t v = brq_peek<U>(r, n);
    r.pos -= n;
    return v;
}

// FSE_readNCount: a table description at p (at most `avail` bytes);
// returns its byte length, or -1.  norm[0..*nsym) and *al are set.
__device__ int read_ncount(const uint8_t *p, int64_t avail, uint32_t max_sym, uint32_t max_al,
                           int16_t *norm, uint32_t *nsym, uint32_t *al) {
    if (avail < 1) return -1;
    const uint8_t *end = p + avail;
    int64_t bitpos = 0;  // from p
    auto rd32 = [&](int64_t bp) -> uint32_t {
        const uint64_t v = ld8b(p + (bp >> 3), p, end);
        return (uint32_t)(v >> (bp & 7));
    };
    uint32_t bs = rd32(0);
    int nb = (int)(bs & 0xF) + 5;
    if ((uint32_t)nb > max_al) return -1;
    *al = (uint32_t)nb;
    bitpos = 4;
    int remaining = (1 << nb) + 1;
    int threshold = 1 << nb;
    nb++;
    uint32_t s = 0;
    bool prev0 = false;
    while (remaining > 1 && s <= max_sym) {
        bs = rd32(bitpos);
        if (prev0) {
            uint32_t n0 = s;
            while ((bs & 0xFFFF) == 0xFFFF) {
                n0 += 24;
                bitpos += 16;
                bs = rd32(bitpos);
            }
            while ((bs & 3) == 3) {
                n0 += 3;
                bs >>= 2;
                bitpos += 2;
            }
            n0 += bs & 3;
            bitpos += 2;
            if (n0 > max_sym + 1 || n0 > kNormCap) return -1;
            while (s < n0) norm[s++] = 0;
            if (s > max_sym) break;
            bs = rd32(bitpos);
        }
        const int mx = (2 * threshold - 1) - remaining;
        int count;
        if ((int)(bs & (uint32_t)(threshold - 1)) < mx) {
            count = (int)(bs & (uint32_t)(threshold - 1));
            bitpos += nb - 1;
        } else {
            count = (int)(bs & (uint32_t)(2 * threshold - 1));
            if (count >= threshold) count -= mx;
            bitpos += nb;
        }
        count--;
        remaining -= count < 0 ? -count : count;
        if (s >= kNormCap) return -1;  // (a symbol this table cannot have)
        norm[s++] = (int16_t)count;
        prev0 = count == 0;
        while (remaining < threshold) {
            nb--;
            threshold >>= 1;
        }
        if (bitpos > 8 * avail) return -1;
    }
    if (remaining != 1 || s > max_sym + 1) return -1;
    *nsym = s;
    const int64_t used = (bitpos + 7) >> 3;
    return used > avail ? -1 : (int)used;
}

// FSE_buildDTable from norm[0..nsym) (accuracy al) into t; false if the
// counts do not fill the table.  Uniform code; lane 0 writes.
__device__ bool build_fse(FseD *t, const int16_t *norm, uint32_t nsym, uint32_t al, uint16_t *nxt,
                          uint32_t lane) {
    const uint32_t size = 1u << al, mask = size - 1;
    uint32_t high = size - 1;
    int total = 0;
    for (uint32_t s = 0; s < nsym; s++) total += norm[s] < 0 ? 1 : norm[s];
    if ((uint32_t)total != size) return false;
    for (uint32_t s = 0; s < nsym; s++) {
        if (norm[s] == -1) {
            if (lane == 0) t[high].sym = (uint8_t)s;
            high--;
            if (lane == 0) nxt[s] = 1;
        } else if (lane == 0) {
            nxt[s] = (uint16_t)(norm[s] < 0 ? 0 : norm[s]);
        }
    }
    const uint32_t step = (size >> 1) + (size >> 3) + 3;
    uint32_t pos = 0;
    for (uint32_t s = 0; s < nsym; s++) {
        for (int i = 0; i < norm[s]; i++) {
            if (lane == 0) t[pos].sym = (uint8_t)s;
            do {
                pos = (pos + step) & mask;
            } while (pos > high);
        }
    }
    if (pos != 0) return false;
    wsync();
    if (lane == 0) {
        for (uint32_t u = 0; u < size; u++) {
            const uint32_t s = t[u].sym;
            const uint32_t ns = nxt[s]++;
            const uint32_t nb = al - highbit32(ns);
            t[u].nb = (uint8_t)nb;
            t[u].next = (uint16_t)((ns << nb) - size);
        }
    }
    wsync();
    return true;
}

__device__ bool build_predefined(FseD *t, const int16_t *src, uint32_t nsym, uint32_t al,
                                 int16_t *norm, uint16_t *nxt, uint32_t lane) {
    if (lane < nsym) norm[lane] = src[lane];
    wsync();
    return build_fse(t, norm, nsym, al, nxt, lane);
}

// Frame-walk state of one wave.
struct Dec {
    const uint8_t *data;  // the blob
    uint64_t dlen;
    uint64_t out;         // bytes decoded (= compared) so far
    uint32_t rep[3];
    uint32_t rep_unk;     // bit i: rep[i] unknown (a block checked out of order)
    uint32_t huf_log;     // 0: no Huffman table yet
    uint32_t huf_nw;      // its weights in L.w[0 .. huf_nw)
    uint32_t al_ll, al_ml, al_of;  // 255: no table yet
    uint32_t bad;         // status
    bool block_mode;      // earlier blocks' state unknown: using it -> kCkSeq
    bool prof;            // RCDC_ZSTD_DBG bit 3: phase clocks into g_zck_prof
    bool narrow;          // RCDC_ZSTD_DBG bit 4: 4-byte compare steps only (A/B)
};

// ---- comparisons (the whole wave) -----------------------------------------

// data[p, p+n) == src[0, n) (kind 0) / == byte v (kind 1) / == data[p-o, ..)
// (kind 2); wave-uniform arguments; returns true if equal.
__device__ bool wave_cmp(const uint8_t *a, const uint8_t *b, uint32_t v, int kind, uint64_t n,
                         uint32_t lane) {
    const uint32_t rep4 = v * 0x01010101u;
    bool ok = true;
    for (uint64_t o = (uint64_t)lane * 4u; o < n; o += 256) {
        const uint32_t x = ld4u(a + o);
        const uint32_t y = kind == 1 ? rep4 : ld4u(b + o);
        uint32_t d = x ^ y;
        const uint64_t rem = n - o;
        if (rem < 4) d &= (1u << (8 * rem)) - 1u;
        ok &= d == 0;
    }
    return __builtin_amdgcn_ballot_w64(!ok) == 0;
}

// 16 bytes at any alignment from the 4-5 aligned dwords that hold them.
__device__ __forceinline__ uint4 ld16u(const uint8_t *p) {
    const uint32_t b = (uint32_t)(uintptr_t)p & 3u, sh = b * 8u;
    const auto *w = gptr((const uint32_t *)(p - b));
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[b ? 4 : 3];
    return make_uint4(__builtin_amdgcn_alignbit(w1, w0, sh), __builtin_amdgcn_alignbit(w2, w1, sh),
                      __builtin_amdgcn_alignbit(w3, w2, sh), __builtin_amdgcn_alignbit(w4, w3, sh));
}

// one lane's comparison (kinds as wave_cmp).  16 bytes a step while 16 fit
// (a step's loads stay inside the dwords of [a, a + n), as ld4u's), then 4:
// a lane compares a whole sequence, and the batch waits for its longest, so
// the steps are memory round trips in a chain (text: many sequences of a few
// dozen bytes)
__device__ bool lane_cmp(const uint8_t *a, const uint8_t *b, uint32_t v, int kind, uint32_t n,
                         bool narrow = false) {
    const uint32_t rep4 = v * 0x01010101u;
    uint32_t acc = 0;
    uint32_t o = 0;
    for (; !narrow && o + 16 <= n; o += 16) {
        const uint4 x = ld16u(a + o);
        const uint4 y = kind == 1 ? make_uint4(rep4, rep4, rep4, rep4) : ld16u(b + o);
        acc |= (x.x ^ y.x) | (x.y ^ y.y) | (x.z ^ y.z) | (x.w ^ y.w);
    }
    for (; o < n; o += 4) {
        const uint32_t x = ld4u(a + o);
        const uint32_t y = kind == 1 ? rep4 : ld4u(b + o);
        uint32_t d = x ^ y;
        const uint32_t rem = n - o;
        if (rem < 4) d &= (1u << (8 * rem)) - 1u;
        acc |= d;
    }
    return acc == 0;
}

// ---- literals ---------------------------------------------------------------

// Huffman weights (HUF_readStats) at p (avail bytes) -> L.w[0..*nw), the
// implied last weight appended; returns the description's length or -1.
__device__ int read_huf_weights(const uint8_t *p, int64_t avail, DecLds &L, uint32_t *nw,
                                uint32_t lane) {
    if (avail < 1) return -1;
    const uint32_t hb = p[0];
    uint32_t n = 0;
    int used;
    if (hb >= 128) {
        n = hb - 127;
        used = 1 + (int)((n + 1) / 2);
        if (used > avail) return -1;
        if (lane < n) {
            const uint32_t byte = p[1 + lane / 2];
            L.w[lane] = (uint8_t)((lane & 1) ? (byte & 15u) : (byte >> 4));
        }
        if (lane + 64 < n) {
            const uint32_t k = lane + 64, byte = p[1 + k / 2];
            L.w[k] = (uint8_t)((k & 1) ? (byte & 15u) : (byte >> 4));
        }
        wsync();
    } else {
        // FSE-compressed weights: NCount (log <= 6), then two interleaved
        // states over a backward bitstream (FSE_decompress_usingDTable)
        used = 1 + (int)hb;
        if (used > avail || hb == 0) return -1;
        uint32_t nsym = 0, al = 0;
        const int nc = read_ncount(p + 1, hb, 255, 6, L.norm, &nsym, &al);
        if (nc < 0) return -1;
        wsync();
        if (!build_fse(L.u.h.hw, L.norm, nsym, al, L.nxt, lane)) return -1;
        BRev r;
        if (!brev_init(r, p + 1 + nc, (int64_t)hb - nc)) return -1;
        uint32_t s1 = (uint32_t)brev_bits(r, al), s2 = (uint32_t)brev_bits(r, al);
        for (;;) {
            if (n >= 255) return -1;
            FseD e = L.u.h.hw[s1];
            if (lane == 0) L.w[n] = e.sym;
            n++;
            s1 = e.next + (uint32_t)brev_bits(r, e.nb);
            if (r.pos < 0) {
                if (n >= 255) return -1;
                if (lane == 0) L.w[n] = L.u.h.hw[s2].sym;
                n++;
                break;
            }
            if (n >= 255) return -1;
            e = L.u.h.hw[s2];
            if (lane == 0) L.w[n] = e.sym;
            n++;
            s2 = e.next + (uint32_t)brev_bits(r, e.nb);
            if (r.pos < 0) {
                if (n >= 255) return -1;
                if (lane == 0) L.w[n] = L.u.h.hw[s1].sym;
                n++;
                break;
            }
        }
        wsync();
    }
    // the last weight is implied: the weights fill a power of two
    uint32_t total = 0, ones = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t wi = L.w[i];
        if (wi > 11) return -1;
        total += wi ? (1u << (wi - 1)) : 0u;
        ones += wi == 1u;
    }
    if (total == 0) return -1;
    const uint32_t tl = highbit32(total) + 1;
    if (tl > 11) return -1;
    const uint32_t rest = (1u << tl) - total;
    if (rest & (rest - 1)) return -1;
    // HUF_readStats' tree check: an even number, at least 2, of weight-1
    // symbols (codes of the full table log), the implied last one included.
    // Without it a table whose codes are all shorter than its log decodes,
    // but libzstd calls it corrupt (r6 checker soak, seed 5627)
    ones += rest == 1u;
    if (ones < 2 || (ones & 1u)) return -1;
    wsync();
    if (lane == 0) L.w[n] = (uint8_t)(highbit32(rest) + 1);
    *nw = n + 1;
    wsync();
    return used;
}

// HUF_readDTableX1 from L.w[0..nw) -> L.huf; returns the table log.
__device__ uint32_t build_huf(DecLds &L, uint32_t nw, uint32_t lane) {
    uint32_t cnt[13] = {0};
    uint32_t total = 0;
    for (uint32_t s = 0; s < nw; s++) {
        const uint32_t wi = L.w[s];
        cnt[wi]++;
        total += wi ? (1u << (wi - 1)) : 0u;
    }
    const uint32_t tl = highbit32(total);  // total is a power of two now
    uint32_t start[13];
    uint32_t nx = 0;
    for (uint32_t wi = 1; wi <= tl; wi++) {
        start[wi] = nx;
        nx += cnt[wi] << (wi - 1);
    }
    // symbols of weight wi fill 2^(wi-1) entries each, in symbol order: lane l
    // writes the entries of symbol s with l in the range (all lanes stride)
    for (uint32_t s = 0; s < nw; s++) {
        const uint32_t wi = L.w[s];
        if (!wi) continue;
        const uint32_t len = 1u << (wi - 1), b = start[wi];
        start[wi] += len;
        for (uint32_t k = lane; k < len; k += 64) {
            L.u.h.huf[b + k].sym = (uint8_t)s;
            L.u.h.huf[b + k].nb = (uint8_t)(tl + 1 - wi);
        }
    }
    wsync();
    return tl;
}

// One Huffman stream [p, p+len) -> n symbols at out (one lane).
__device__ bool huf_stream(const DecLds &L, uint32_t tl, const uint8_t *p, int64_t len,
                           uint8_t *out, uint32_t n) {
    BRevQ r;
    r.pf = nullptr;  // (per-lane streams: no LDS prefetch)
    if (n == 0) return len == 0 || (brq_init(r, p, len) && r.pos == 0);
    if (!brq_init(r, p, len)) return false;
    uint32_t i = 0;
    // four symbols per dword store once aligned
    while (i < n && ((uintptr_t)(out + i) & 3u)) {
        const HufD e = L.u.h.huf[brq_peek(r, tl)];
        out[i++] = e.sym;
        r.pos -= e.nb;
    }
    for (; i + 4 <= n; i += 4) {
        uint32_t v = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const HufD e = L.u.h.huf[brq_peek(r, tl)];
            v |= (uint32_t)e.sym << (8 * k);
            r.pos -= e.nb;
        }
        *reinterpret_cast<uint32_t *>(out + i) = v;
    }
    for (; i < n; i++) {
        const HufD e = L.u.h.huf[brq_peek(r, tl)];
        out[i] = e.sym;
        r.pos -= e.nb;
    }
    return r.pos == 0;
}

// ---- blocks -----------------------------------------------------------------

// Compressed block [p, p + bs): literals section then sequences section.
__device__ void check_compressed(Dec &D, DecLds &L, const uint8_t *p, uint32_t bs, uint8_t *scratch,
                                 uint32_t lane) {
    const uint8_t *end = p + bs;
    const uint64_t t0 = D.prof ? wall_clock64() : 0;
    // -- literals section header (3.1.1.3.1.1)
    const uint32_t b0 = p[0];
    const uint32_t ltype = b0 & 3u, sf = (b0 >> 2) & 3u;
    uint32_t regen = 0, csize = 0, hdr = 0, nstreams = 1;
    if (ltype < 2) {
        if (sf == 0 || sf == 2) {
            regen = b0 >> 3;
            hdr = 1;
        } else if (sf == 1) {
            if (bs < 2) { D.bad = kCkCorrupt; return; }
            regen = (b0 >> 4) | ((uint32_t)p[1] << 4);
            hdr = 2;
        } else {
            if (bs < 3) { D.bad = kCkCorrupt; return; }
            regen = (b0 >> 4) | ((uint32_t)p[1] << 4) | ((uint32_t)p[2] << 12);
            hdr = 3;
        }
    } else {
        nstreams = sf == 0 ? 1u : 4u;
        if (sf < 2) {
            if (bs < 3) { D.bad = kCkCorrupt; return; }
            const uint32_t v = b0 | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16);
            regen = (v >> 4) & 0x3FFu;
            csize = (v >> 14) & 0x3FFu;
            hdr = 3;
        } else if (sf == 2) {
            if (bs < 4) { D.bad = kCkCorrupt; return; }
            const uint32_t v = b0 | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
                               ((uint32_t)p[3] << 24);
            regen = (v >> 4) & 0x3FFFu;
            csize = v >> 18;
            hdr = 4;
        } else {
            if (bs < 5) { D.bad = kCkCorrupt; return; }
            const uint64_t v = b0 | ((uint64_t)p[1] << 8) | ((uint64_t)p[2] << 16) |
                               ((uint64_t)p[3] << 24) | ((uint64_t)p[4] << 32);
            regen = (uint32_t)((v >> 4) & 0x3FFFFu);
            csize = (uint32_t)((v >> 22) & 0x3FFFFu);
            hdr = 5;
        }
    }
    if (regen > kBlockMax) { D.bad = kCkCorrupt; return; }
    const uint8_t *lits = nullptr;  // the decoded literals (kind 0) or a byte (kind 1)
    uint32_t lit_byte = 0;
    int lkind = 0;
    const uint8_t *q = p + hdr;
    if (ltype == 0) {
        if (q + regen > end) { D.bad = kCkCorrupt; return; }
        lits = q;
        q += regen;
    } else if (ltype == 1) {
        if (q + 1 > end) { D.bad = kCkCorrupt; return; }
        lit_byte = q[0];
        lkind = 1;
        q += 1;
    } else {
        if (q + csize > end) { D.bad = kCkCorrupt; return; }
        const uint8_t *cs = q;
        int64_t clen = csize;
        if (ltype == 2) {
            uint32_t nw = 0;
            const int tu = read_huf_weights(cs, clen, L, &nw, lane);
            if (tu < 0) { D.bad = kCkCorrupt; return; }
            D.huf_log = build_huf(L, nw, lane);
            D.huf_nw = nw;
            cs += tu;
            clen -= tu;
        } else if (D.huf_log == 0) {  // treeless: the previous block's table
            D.bad = D.block_mode ? kCkSeq : kCkCorrupt;
            return;
        } else {  // its weights: the table's bytes held LL / ML extras since
            build_huf(L, D.huf_nw, lane);
        }
        const uint32_t tl = D.huf_log;
        bool ok = true;
        if (nstreams == 1) {
            if (lane == 0) ok = huf_stream(L, tl, cs, clen, scratch, regen);
        } else {
            if (clen < 6) { D.bad = kCkCorrupt; return; }
            const int64_t s1 = cs[0] | (cs[1] << 8), s2 = cs[2] | (cs[3] << 8),
                          s3 = cs[4] | (cs[5] << 8);
            const int64_t s4 = clen - 6 - s1 - s2 - s3;
            const uint32_t seg = (regen + 3) / 4;
            if (s4 < 0 || 3 * seg > regen) { D.bad = kCkCorrupt; return; }
            if (lane < 4) {
                const int64_t off = 6 + (lane > 0 ? s1 : 0) + (lane > 1 ? s2 : 0) + (lane > 2 ? s3 : 0);
                const int64_t ln = lane == 0 ? s1 : lane == 1 ? s2 : lane == 2 ? s3 : s4;
                const uint32_t n = lane < 3 ? seg : regen - 3 * seg;
                ok = huf_stream(L, tl, cs + off, ln, scratch + lane * seg, n);
            }
        }
        if (__builtin_amdgcn_ballot_w64(!ok)) { D.bad = kCkCorrupt; return; }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        __syncthreads();
        lits = scratch;
        q += csize;
        if (D.prof && lane == 0) {
            atomicAdd(&g_zck_prof[0], wall_clock64() - t0);
            atomicAdd(&g_zck_prof[3], (unsigned long long)regen);
        }
    }
    const uint64_t t1 = D.prof ? wall_clock64() : 0;
    // -- sequences section header (3.1.1.3.2.1)
    if (q >= end) { D.bad = kCkCorrupt; return; }
    uint32_t nseq = q[0];
    if (nseq == 0) {
        q += 1;
    } else if (nseq < 128) {
        q += 1;
    } else if (nseq < 255) {
        if (q + 2 > end) { D.bad = kCkCorrupt; return; }
        nseq = ((nseq - 128) << 8) + q[1];
        q += 2;
    } else {
        if (q + 3 > end) { D.bad = kCkCorrupt; return; }
        nseq = q[1] + ((uint32_t)q[2] << 8) + 0x7F00u;
        q += 3;
    }
    uint64_t litpos = 0;  // literals consumed
    nseq = rfl(nseq);     // wave-uniform (the decode loop's trip count)
    if (nseq) {
        if (q >= end) { D.bad = kCkCorrupt; return; }
        const uint32_t modes = *q++;
        // reserved bits 1-0 must be zero (RFC 8878 3.1.1.3.2.1; libzstd 1.5,
        // the reference's, rejects them, 1.4.8 decodes)
        if (modes & 3u) { D.bad = kCkCorrupt; return; }
        // tables in the order LL, OF, ML
        for (int k = 0; k < 3; k++) {
            const uint32_t mode = (modes >> (6 - 2 * k)) & 3u;
            FseD *t = k == 0 ? L.ll : k == 1 ? L.of : L.ml;
            uint32_t &al = k == 0 ? D.al_ll : k == 1 ? D.al_of : D.al_ml;
            const uint32_t max_sym = k == 0 ? 35u : k == 1 ? 31u : 52u;
            const uint32_t max_al = k == 0 ? 9u : k == 1 ? 8u : 9u;
            if (mode == 0) {
                const int16_t *nrm = k == 0 ? kLLNorm : k == 1 ? kOFNorm : kMLNorm;
                const uint32_t ns = k == 0 ? 36u : k == 1 ? 29u : 53u;
                const uint32_t a = k == 1 ? 5u : 6u;
                if (!build_predefined(t, nrm, ns, a, L.norm, L.nxt, lane)) { D.bad = kCkCorrupt; return; }
                al = a;
            } else if (mode == 1) {
                if (q >= end) { D.bad = kCkCorrupt; return; }
                const uint32_t s = *q++;
                if (s > max_sym) { D.bad = kCkCorrupt; return; }
                if (lane == 0) {
                    t[0].sym = (uint8_t)s;
                    t[0].nb = 0;
                    t[0].next = 0;
                }
                wsync();
                al = 0;
            } else if (mode == 2) {
                uint32_t ns = 0, a = 0;
                const int u = read_ncount(q, end - q, max_sym, max_al, L.norm, &ns, &a);
                if (u < 0) { D.bad = kCkCorrupt; return; }
                wsync();
                if (!build_fse(t, L.norm, ns, a, L.nxt, lane)) { D.bad = kCkCorrupt; return; }
                al = a;
                q += u;
            } else if (al == 255u) {  // repeat: needs an earlier table
                D.bad = D.block_mode ? kCkSeq : kCkCorrupt;
                return;
            }
        }
        for (uint32_t u = lane; u < (1u << D.al_ll); u += 64) {
            const uint32_t c = L.ll[u].sym < 36 ? L.ll[u].sym : 0u;
            L.u.x.llx[u] = kLLBase[c] | (uint32_t)kLLBits[c] << 24;
        }
        for (uint32_t u = lane; u < (1u << D.al_ml); u += 64) {
            const uint32_t c = L.ml[u].sym < 53 ? L.ml[u].sym : 0u;
            L.u.x.mlx[u] = kMLBase[c] | (uint32_t)kMLBits[c] << 24;
        }
        wsync();
        BRevQ r;
        r.pf = (__attribute__((address_space(3))) uint32_t *)L.pf;
        if (!brq_init<true>(r, q, end - q)) { D.bad = kCkCorrupt; return; }
        const uint32_t al_ll = rfl(D.al_ll), al_of = rfl(D.al_of), al_ml = rfl(D.al_ml);
        uint32_t sll = brq_bits<true>(r, al_ll);
        uint32_t sof = brq_bits<true>(r, al_of);
        uint32_t sml = brq_bits<true>(r, al_ml);
        uint32_t r0 = D.rep[0], r1 = D.rep[1], r2 = D.rep[2];
        bool u0 = D.rep_unk & 1u, u1 = (D.rep_unk >> 1) & 1u, u2 = (D.rep_unk >> 2) & 1u;
        bool unk_used = false;
        uint64_t tcmp = 0;  // (phase clocks: the batches' placement + comparisons)
        for (uint32_t s0 = 0; s0 < nseq; s0 += 64) {
            const uint32_t nb = min(64u, nseq - s0);
            uint32_t myll = 0, myml = 0, myoff = 0;
            bool err = false;
            // the decode state is wave-uniform: say so each round (the
            // compare loops below diverge, and the compiler then kept the
            // reader in VGPRs with 64-bit VALU compares per bit read)
            r.pos = (int32_t)rfl((uint32_t)r.pos);
            r.B = (int32_t)rfl((uint32_t)r.B);
            r.acc = rfl64(r.acc);
            r.used = rfl(r.used);
            r.len = (int32_t)rfl((uint32_t)r.len);
            r.base = reinterpret_cast<const uint8_t *>(rfl64(reinterpret_cast<uintptr_t>(r.base)));
            r.g0 = make_uint4(rfl(r.g0.x), rfl(r.g0.y), rfl(r.g0.z), rfl(r.g0.w));
            r.nbyte = (int32_t)rfl((uint32_t)r.nbyte);
            sll = rfl(sll);
            sof = rfl(sof);
            sml = rfl(sml);
            r0 = rfl(r0);
            r1 = rfl(r1);
            r2 = rfl(r2);
            for (uint32_t j = 0; j < nb; j++) {
                // the entries as one dword each (sym | nb << 8 | next << 16),
                // wave-uniform
                // the five reads issued together, then one wait: the
                // scheduler otherwise waited after each (3 LDS round trips
                // per sequence on the critical path)
                const uint32_t veo = reinterpret_cast<const uint32_t *>(L.of)[sof];
                const uint32_t vel = reinterpret_cast<const uint32_t *>(L.ll)[sll];
                const uint32_t vem = reinterpret_cast<const uint32_t *>(L.ml)[sml];
                const uint32_t vxl = L.u.x.llx[sll], vxm = L.u.x.mlx[sml];
                __builtin_amdgcn_sched_barrier(0);
                const uint32_t eo = rfl(veo), el = rfl(vel), em = rfl(vem);
                const uint32_t xl = rfl(vxl), xm = rfl(vxm);
                // (no per-sequence symbol range check: read_ncount bounds every
                // FSE table's symbols by its alphabet, as do the predefined and
                // RLE tables; a repeat table is an earlier one of these)
                const uint32_t ofc = eo & 0xFFu;
                const uint64_t ofv = (1ull << ofc) + brq_bits<true>(r, ofc);
                // ML's then LL's extra bits (<= 16 each) in one read: the
                // decode is bound by the scalar unit's issue rate, and each
                // read is a window check, a 64-bit shift and a mask
                const uint32_t nm = xm >> 24, nl = xl >> 24;
                const uint32_t vx = brq_bits<true>(r, nm + nl);
                const uint32_t ml = (xm & 0xFFFFFFu) + (uint32_t)((uint64_t)vx >> nl);
                const uint32_t ll = (xl & 0xFFFFFFu) + (vx & (uint32_t)((1ull << nl) - 1ull));
                // the repeat-offset history (RFC 8878 3.1.1.5) without
                // branches: the decode is bound by the scalar unit's issue
                // rate, and a branch per case was a good part of a sequence's
                const bool lr = ofv <= 3;  // a repeat code
                const uint32_t idx = (uint32_t)ofv - 1u + (ll == 0 ? 1u : 0u);
                const uint32_t rsel = idx == 1 ? r1 : idx == 2 ? r2 : idx == 0 ? r0 : r0 - 1u;
                const bool usel = idx == 1 ? u1 : idx == 2 ? u2 : u0;
                const uint32_t off = lr ? rsel : (uint32_t)(ofv - 3);
                unk_used |= lr && usel;
                const bool k1 = lr && idx == 0, k2 = lr && idx <= 1;  // r1 / r2 kept
                const uint32_t n2 = k2 ? r2 : r1, n1 = k1 ? r1 : r0;
                const bool nu2 = k2 ? u2 : u1, nu1 = k1 ? u1 : u0, nu0 = k1 ? u0 : false;
                r2 = n2;
                r1 = n1;
                r0 = off;
                u2 = nu2;
                u1 = nu1;
                u0 = nu0;
                if (off == 0) err = true;
                if (s0 + j + 1 < nseq) {
                    // the three state updates (<= 9 + 9 + 8 bits) in one read
                    const uint32_t bl = (el >> 8) & 0xFFu, bm = (em >> 8) & 0xFFu,
                                   bo = (eo >> 8) & 0xFFu;
                    const uint32_t v = brq_bits<true>(r, bl + bm + bo);
                    sll = (el >> 16) + (uint32_t)((uint64_t)v >> (bm + bo));
                    sml = (em >> 16) + ((v >> bo) & ((1u << bm) - 1u));
                    sof = (eo >> 16) + (v & ((1u << bo) - 1u));
                }
                // selects, not a branch on the lane: a divergent branch here
                // made the compiler keep the reader's state in VGPRs
                const bool me = lane == j;
                myll = me ? ll : myll;
                myml = me ? ml : myml;
                myoff = me ? off : myoff;
            }
            if (unk_used) { D.bad = kCkSeq; return; }  // (block mode only)
            if (err || r.pos < 0) { D.bad = kCkCorrupt; return; }
            const uint64_t tc0 = D.prof ? wall_clock64() : 0;
            // place the batch: exclusive prefix sums of ll and ll + ml
            uint64_t incl_l = myll, incl_o = (uint64_t)myll + myml;
            for (uint32_t d = 1; d < 64; d <<= 1) {
                const uint64_t a = __shfl_up(incl_l, d), b = __shfl_up(incl_o, d);
                if (lane >= d) {
                    incl_l += a;
                    incl_o += b;
                }
            }
            const uint64_t lp = litpos + incl_l - myll;             // my literals
            const uint64_t op = D.out + incl_o - myll - myml;       // my output position
            const uint64_t tot_l = __shfl(incl_l, (int)nb - 1), tot_o = __shfl(incl_o, (int)nb - 1);
            const bool mine = lane < nb;
            // uniform verdicts: more literals than decoded or a match before
            // the frame start (malformed), or longer than the blob (mismatch)
            const bool c_lit = litpos + tot_l > regen;
            const bool c_off = __builtin_amdgcn_ballot_w64(mine && (uint64_t)myoff > op + myll) != 0;
            if (c_lit || c_off) { D.bad = kCkCorrupt; return; }
            if (D.out + tot_o > D.dlen) { D.bad = kCkMismatch; return; }
            const bool lng = mine && (uint64_t)myll + myml > 256;
            bool eq = true;
            if (mine && !lng) {
                const uint8_t *dst = D.data + op;
                eq = lane_cmp(dst, lits + lp, lit_byte, lkind, myll, D.narrow) &&
                     lane_cmp(dst + myll, dst + myll - myoff, 0, 2, myml, D.narrow);
            }
            uint64_t longs = __builtin_amdgcn_ballot_w64(lng);
            while (longs) {
                const int L0 = __builtin_ctzll(longs);
                longs &= longs - 1;
                const uint64_t o = __shfl(op, L0), l0 = __shfl(lp, L0);
                const uint32_t a = (uint32_t)__shfl((int)myll, L0), m = (uint32_t)__shfl((int)myml, L0),
                               f = (uint32_t)__shfl((int)myoff, L0);
                const uint8_t *dst = D.data + o;
                const bool e1 = wave_cmp(dst, lits + l0, lit_byte, lkind, a, lane);
                const bool e2 = wave_cmp(dst + a, dst + a - f, 0, 2, m, lane);
                if (lane == (uint32_t)L0) eq = e1 && e2;
            }
            if (__builtin_amdgcn_ballot_w64(!eq)) { D.bad = kCkMismatch; return; }
            if (D.prof) tcmp += wall_clock64() - tc0;
            litpos += tot_l;
            D.out += tot_o;
        }
        if (r.pos != 0) { D.bad = kCkCorrupt; return; }
        if (D.prof && lane == 0) {
            atomicAdd(&g_zck_prof[1], wall_clock64() - t1);
            atomicAdd(&g_zck_prof[4], (unsigned long long)nseq);
            atomicAdd(&g_zck_prof[6], tcmp);
        }
        D.rep[0] = r0;
        D.rep[1] = r1;
        D.rep[2] = r2;
        D.rep_unk = (u0 ? 1u : 0u) | (u1 ? 2u : 0u) | (u2 ? 4u : 0u);
    } else if (q != end) {
        D.bad = kCkCorrupt;
        return;
    }
    // the remaining literals
    const uint64_t rest = regen - litpos;
    if (D.out + rest > D.dlen) { D.bad = kCkMismatch; return; }
    if (!wave_cmp(D.data + D.out, lits + litpos, lit_byte, lkind, rest, lane)) {
        D.bad = kCkMismatch;
        return;
    }
    D.out += rest;
    if (D.prof && lane == 0) {
        atomicAdd(&g_zck_prof[2], wall_clock64() - t0);
        atomicAdd(&g_zck_prof[5], 1ull);
    }
}

// The window a frame asks its decoder for (RFC 8878 3.1.1.1.2; a
// single-segment frame's is its content size) fits the limit of rustic's
// decode_all: the zstd crate's streaming decoder keeps libzstd's default,
// windows up to 2^27 + 1 bytes (ZSTD_WINDOWLOG_LIMIT_DEFAULT; larger ones
// fail with "Frame requires too much memory for decoding").
__device__ __forceinline__ bool window_ok(uint32_t single, uint32_t wd, uint64_t fcs) {
    if (single) return fcs <= (1ull << 27) + 1ull;
    const uint64_t base = 1ull << (10u + (wd >> 3));
    return base + (base >> 3) * (wd & 7u) <= (1ull << 27) + 1ull;
}

// decode_all (decrypt.rs:71-95) reads the decoder through io::copy into a
// Vec, whose first read offers 8 KiB of output (DEFAULT_BUF_SIZE).  A frame
// whose content size is known and fits takes libzstd's one-pass shortcut
// (ZSTD_decompressStream -> ZSTD_decompress_usingDDict): no window limit,
// and an empty compressed block is corrupt.  Other frames go through the
// stage machine: the window limit applies and empty blocks of any type are
// skipped.  The checker follows the path decode_all would take.
constexpr uint64_t kDecodeAllFirstOut = 8192;
__device__ __forceinline__ bool one_pass(uint32_t fcs_len, uint64_t fcs) {
    return fcs_len && fcs <= kDecodeAllFirstOut;
}

// One frame; returns its status.
__device__ uint32_t check_frame(const uint8_t *f, uint64_t flen, const uint8_t *data, uint64_t dlen,
                                DecLds &L, uint8_t *scratch, uint32_t lane, bool prof) {
    const uint8_t *end = f + flen;
    if (flen < 6) return kCkCorrupt;
    const uint32_t magic = f[0] | (f[1] << 8) | (f[2] << 16) | ((uint32_t)f[3] << 24);
    if (magic != 0xFD2FB528u) return kCkCorrupt;
    const uint32_t fhd = f[4];
    const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1u, cksum = (fhd >> 2) & 1u,
                   did_flag = fhd & 3u;
    if (fhd & 8u) return kCkCorrupt;  // reserved bit
    const uint8_t *q = f + 5;
    if (!single) q += 1;  // window descriptor
    const uint32_t did_len = did_flag == 0 ? 0 : did_flag == 1 ? 1 : did_flag == 2 ? 2 : 4;
    if (q + did_len > end) return kCkCorrupt;
    uint32_t did = 0;
    for (uint32_t i = 0; i < did_len; i++) did |= (uint32_t)q[i] << (8 * i);
    if (did) return kCkCorrupt;  // dictionaries: not supported
    q += did_len;
    const uint32_t fcs_len = fcs_flag == 0 ? (single ? 1 : 0) : fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8;
    if (q + fcs_len > end) return kCkCorrupt;
    uint64_t fcs = 0;
    for (uint32_t i = 0; i < fcs_len; i++) fcs |= (uint64_t)q[i] << (8 * i);
    if (fcs_len == 2) fcs += 256;
    q += fcs_len;
    const bool shortcut = one_pass(fcs_len, fcs);
    if (!shortcut && !window_ok(single, single ? 0u : f[5], fcs)) return kCkCorrupt;
    if (fcs_len && fcs != dlen) return kCkMismatch;
    Dec D;
    D.data = data;
    D.dlen = dlen;
    D.out = 0;
    D.rep[0] = 1;
    D.rep[1] = 4;
    D.rep[2] = 8;
    D.rep_unk = 0;
    D.huf_log = 0;
    D.al_ll = D.al_ml = D.al_of = 255u;
    D.bad = kCkOk;
    D.block_mode = false;
    D.prof = prof;
    D.narrow = false;
    for (;;) {
        if (q + 3 > end) return kCkCorrupt;
        const uint32_t bh = q[0] | (q[1] << 8) | ((uint32_t)q[2] << 16);
        q += 3;
        const uint32_t last = bh & 1u, btype = (bh >> 1) & 3u, bsize = bh >> 3;
        if (btype == 3) return kCkCorrupt;
        if (btype == 0) {
            if (bsize > kBlockMax || q + bsize > end) return kCkCorrupt;
            if (D.out + bsize > dlen) return kCkMismatch;
            if (!wave_cmp(data + D.out, q, 0, 0, bsize, lane)) return kCkMismatch;
            D.out += bsize;
            q += bsize;
        } else if (btype == 1) {
            if (bsize > kBlockMax || q + 1 > end) return kCkCorrupt;
            if (D.out + bsize > dlen) return kCkMismatch;
            if (!wave_cmp(data + D.out, nullptr, q[0], 1, bsize, lane)) return kCkMismatch;
            D.out += bsize;
            q += 1;
        } else if (bsize == 0 && !shortcut) {
            // an empty compressed block: the stage machine skips blocks of 0
            // bytes whatever their type (ZSTD_decompressContinue); the one-pass
            // path calls it corrupt, below (r6 checker soak, seeds 8485, 8527)
        } else {
            if (bsize > kBlockMax || bsize == 0 || q + bsize > end) return kCkCorrupt;
            check_compressed(D, L, q, bsize, scratch, lane);
            if (D.bad) return D.bad;
            q += bsize;
        }
        if (last) break;
    }
    if (cksum) q += 4;
    if (q != end) return kCkCorrupt;  // a second frame or trailing bytes
    return D.out == dlen ? kCkOk : kCkMismatch;
}

}  // namespace

// refs: frame_off, frame_len, data_off, data_len (rcdc_zstd_check_ref);
// order: the queue order; ctr: the queue counter (zeroed by the host).
// OCC: waves per SIMD the registers are budgeted for (2: no spills, 3: more
// waves in flight, 4: 128 VGPRs, the 16 waves per CU the LDS now allows;
// RCDC_ZCK_OCC picks, A/B)
template <int OCC>
__global__ __launch_bounds__(64, OCC) void rcdc_zstd_check_kernel(
    const uint8_t *__restrict__ frames, const uint8_t *__restrict__ data,
    const ulonglong4 *__restrict__ refs, const uint32_t *__restrict__ order, uint32_t n,
    uint32_t stored, uint8_t *scratch, uint32_t *__restrict__ status, uint32_t *ctr, uint32_t dbg) {
    __shared__ DecLds L;
    const uint32_t lane = threadIdx.x;
    uint8_t *scr = scratch + (uint64_t)blockIdx.x * (kBlockMax + 64);
    for (;;) {
        uint32_t k = 0;
        if (lane == 0) k = atomicAdd(ctr, 1u);
        k = __builtin_amdgcn_readfirstlane(__shfl(k, 0));
        if (k >= n) break;
        const uint32_t i = order[k];
        const ulonglong4 r = refs[i];
        uint32_t st;
        if (stored)  // plain bytes: equal length and bytes
            st = r.y != r.w ? kCkMismatch
                            : (wave_cmp(data + r.z, frames + r.x, 0, 0, r.w, lane) ? kCkOk : kCkMismatch);
        else
            st = check_frame(frames + r.x, r.y, data + r.z, r.w, L, scr, lane, dbg & 8u);
        if (lane == 0) status[i] = st;
        __syncthreads();  // LDS tables are rebuilt by the next frame
    }
}

// ---- block-parallel pass -----------------------------------------------------
// A thread per frame walks the frame header and block headers and gives each
// block the output position it has when every block but the last decodes to
// Block_Maximum_Size (128 KiB: how zstd encoders cut their input, this one
// included).  A wave per block then checks it at that position; what it
// cannot settle alone -- a repeat offset, Huffman table or FSE table from an
// earlier block, a block of another size, any failure -- marks the frame
// kCkSeq, and those frames are checked again in order (rcdc_zstd_check_kernel).

struct BlkDesc {       // 32 B
    uint64_t content;  // block content: offset in the frames buffer
    uint64_t out;      // output position in the frame
    uint32_t frame;
    uint32_t size;     // Block_Size field
    uint32_t flags;    // type | first << 2 | used << 3
    uint32_t out_len;  // expected decoded bytes
};

__global__ __launch_bounds__(256) void rcdc_zstd_blocks_kernel(
    const uint8_t *__restrict__ frames, const ulonglong4 *__restrict__ refs,
    const uint64_t *__restrict__ blk0, uint32_t n, BlkDesc *__restrict__ blks,
    uint32_t *__restrict__ status) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const ulonglong4 r = refs[i];
    const uint8_t *f = frames + r.x, *end = f + r.y;
    const uint64_t b0 = blk0[i], cap = blk0[i + 1] - b0, dlen = r.w;
    for (uint64_t k = 0; k < cap; k++) blks[b0 + k].flags = 0;
    uint32_t st = kCkOk;
    do {
        if (r.y < 6) { st = kCkCorrupt; break; }
        const uint32_t magic = f[0] | (f[1] << 8) | (f[2] << 16) | ((uint32_t)f[3] << 24);
        const uint32_t fhd = f[4];
        if (magic != 0xFD2FB528u || (fhd & 8u)) { st = kCkCorrupt; break; }
        const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1u, cksum = (fhd >> 2) & 1u,
                       did_flag = fhd & 3u;
        const uint8_t *q = f + 5 + (single ? 0 : 1);
        const uint32_t did_len = did_flag == 0 ? 0 : did_flag == 1 ? 1 : did_flag == 2 ? 2 : 4;
        const uint32_t fcs_len = fcs_flag == 0 ? (single ? 1 : 0) : fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8;
        if (q + did_len + fcs_len > end) { st = kCkCorrupt; break; }
        uint32_t did = 0;
        for (uint32_t j = 0; j < did_len; j++) did |= (uint32_t)q[j] << (8 * j);
        if (did) { st = kCkCorrupt; break; }
        q += did_len;
        uint64_t fcs = 0;
        for (uint32_t j = 0; j < fcs_len; j++) fcs |= (uint64_t)q[j] << (8 * j);
        if (fcs_len == 2) fcs += 256;
        q += fcs_len;
        if (!one_pass(fcs_len, fcs) && !window_ok(single, single ? 0u : f[5], fcs)) {
            st = kCkCorrupt;
            break;
        }
        if (fcs_len && fcs != dlen) { st = kCkMismatch; break; }
        uint64_t k = 0;
        for (;;) {
            if (q + 3 > end) { st = kCkCorrupt; break; }
            const uint32_t bh = q[0] | (q[1] << 8) | ((uint32_t)q[2] << 16);
            q += 3;
            const uint32_t last = bh & 1u, btype = (bh >> 1) & 3u, bsize = bh >> 3;
            const uint64_t csz = btype == 1 ? 1u : bsize;
            if (btype == 3 || bsize > kBlockMax || q + csz > end) { st = kCkCorrupt; break; }
            const uint64_t pos = k * kBlockMax;
            const uint64_t want = last ? (dlen >= pos ? dlen - pos : ~0ull) : kBlockMax;
            if (k >= cap || want > kBlockMax || (btype < 2 && bsize != want)) { st = kCkSeq; break; }
            BlkDesc d;
            d.content = r.x + (uint64_t)(q - f);
            d.out = pos;
            d.frame = i;
            d.size = bsize;
            d.flags = btype | (k == 0 ? 4u : 0u) | 8u;
            d.out_len = (uint32_t)want;
            blks[b0 + k] = d;
            q += csz;
            k++;
            if (last) break;
        }
        if (st) break;
        if (cksum) q += 4;
        if (q != end) st = kCkCorrupt;
    } while (false);
    status[i] = st;
}

template <int OCC>
__global__ __launch_bounds__(64, OCC) void rcdc_zstd_block_check_kernel(
    const uint8_t *__restrict__ frames, const uint8_t *__restrict__ data,
    const ulonglong4 *__restrict__ refs, const BlkDesc *__restrict__ blks, uint64_t nblk,
    uint8_t *scratch, uint32_t *status, uint32_t *ctr, uint32_t dbg) {
    __shared__ DecLds L;
    const uint32_t lane = threadIdx.x;
    uint8_t *scr = scratch + (uint64_t)blockIdx.x * (kBlockMax + 64);
    for (;;) {
        uint32_t k = 0;
        if (lane == 0) k = atomicAdd(ctr, 1u);
        k = __builtin_amdgcn_readfirstlane(__shfl(k, 0));
        if (k >= nblk) break;
        const BlkDesc b = blks[k];
        if (!(b.flags & 8u)) continue;  // an unused slot
        if (__builtin_amdgcn_readfirstlane(((volatile uint32_t *)status)[b.frame]) != kCkOk) continue;
        const ulonglong4 r = refs[b.frame];
        const uint8_t *dat = data + r.z;
        const uint32_t btype = b.flags & 3u;
        uint32_t st = kCkOk;
        if (btype == 0) {
            st = wave_cmp(dat + b.out, frames + b.content, 0, 0, b.out_len, lane) ? kCkOk : kCkSeq;
        } else if (btype == 1) {
            st = wave_cmp(dat + b.out, nullptr, frames[b.content], 1, b.out_len, lane) ? kCkOk : kCkSeq;
        } else {
            Dec D;
            D.data = dat;
            D.dlen = b.out + b.out_len;
            D.out = b.out;
            D.rep[0] = 1;
            D.rep[1] = 4;
            D.rep[2] = 8;
            D.rep_unk = (b.flags & 4u) ? 0u : 7u;
            D.huf_log = 0;
            D.al_ll = D.al_ml = D.al_of = 255u;
            D.bad = kCkOk;
            D.block_mode = true;
            D.prof = dbg & 8u;
            D.narrow = dbg & 16u;
            check_compressed(D, L, frames + b.content, b.size, scr, lane);
            st = (D.bad || D.out != D.dlen) ? kCkSeq : kCkOk;
        }
        if (st != kCkOk && lane == 0) atomicMax(&status[b.frame], kCkSeq);
        __syncthreads();  // LDS tables are rebuilt by the next block
    }
}

namespace rcdc {

uint64_t zstd_check_scratch_bytes(uint32_t grid) { return (uint64_t)grid * (kBlockMax + 64); }

static int zck_occ() {
    // 4: 16 waves per CU (r5z3: text check 27.9 -> 29.1 GiB/s, CSV 47.3 -> 49.9,
    // code 57.6 -> 61.0 against 2 with the same LDS layout)
    static const int o = getenv("RCDC_ZCK_OCC") ? atoi(getenv("RCDC_ZCK_OCC")) : 4;
    return o;
}

static uint32_t zck_dbg() {
    static const uint32_t d = getenv("RCDC_ZSTD_DBG") ? (uint32_t)atoi(getenv("RCDC_ZSTD_DBG")) : 0u;
    return d;
}

void zstd_check_prof_dump() {
    unsigned long long h[8];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_zck_prof), sizeof h) != hipSuccess) return;
    fprintf(stderr, "rcdc zstd check phases (wave-ms, 100 MHz clock): literals %.1f sequences %.1f "
            "(of which placement + compares %.1f) blocks %.1f; literals %llu sequences %llu "
            "compressed blocks %llu\n",
            h[0] / 1e5, h[1] / 1e5, h[6] / 1e5, h[2] / 1e5, h[3], h[4], h[5]);
    memset(h, 0, sizeof h);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_zck_prof), h, sizeof h);
}

uint64_t zstd_blkdesc_bytes() { return sizeof(BlkDesc); }

// Resident check waves per CU the grid is sized for: 16 when the registers
// are budgeted for 4 per SIMD, else 12 (3 per SIMD: the block kernel's ~150
// VGPRs).
uint32_t zstd_check_waves_per_cu() { return zck_occ() == 4 ? 16u : 12u; }

hipError_t launch_zstd_check(const uint8_t *frames, const uint8_t *data, const void *refs,
                             const uint32_t *order, uint32_t n, bool stored, uint8_t *scratch,
                             uint32_t grid, uint32_t *status, uint32_t *ctr, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const uint32_t g = n < grid ? n : grid;
    hipLaunchKernelGGL(zck_occ() == 4   ? rcdc_zstd_check_kernel<4>
                       : zck_occ() == 3 ? rcdc_zstd_check_kernel<3>
                                        : rcdc_zstd_check_kernel<2>,
                       dim3(g), dim3(64), 0, stream, frames, data,
                       (const ulonglong4 *)refs, order, n, stored ? 1u : 0u, scratch, status, ctr,
                       zck_dbg());
    return hipGetLastError();
}

// the block-parallel pass: header walk, then a wave per block
hipError_t launch_zstd_check_blocks(const uint8_t *frames, const uint8_t *data, const void *refs,
                                    const uint64_t *blk0, uint32_t n, void *blks, uint64_t nblk,
                                    uint8_t *scratch, uint32_t grid, uint32_t *status,
                                    uint32_t *ctr, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(rcdc_zstd_blocks_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, frames,
                       (const ulonglong4 *)refs, blk0, n, (BlkDesc *)blks, status);
    const uint32_t g = nblk < grid ? (uint32_t)nblk : grid;
    if (g)
        hipLaunchKernelGGL(zck_occ() == 4   ? rcdc_zstd_block_check_kernel<4>
                           : zck_occ() == 3 ? rcdc_zstd_block_check_kernel<3>
                                            : rcdc_zstd_block_check_kernel<2>,
                           dim3(g), dim3(64), 0, stream, frames, data,
                           (const ulonglong4 *)refs, (const BlkDesc *)blks, nblk, scratch, status,
                           ctr, zck_dbg());
    return hipGetLastError();
}

}  // namespace rcdc

// ---- range copies (pack files from blobs sealed elsewhere: packer.rs
// add_raw, :615-655) -----------------------------------------------------------
// Unit k = {src, dst, len, base} copies len bytes from the device address
// base + src to out + dst (any alignments; base is the unit's own source
// buffer, so one launch gathers from several allocations): the output's
// 16-aligned body in dwordx4 stores of bytes loaded at any alignment (the
// neighbour lane's chunk + v_alignbit), the ragged head and tail byte by byte.

namespace {

typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));


}  // namespace

__global__ __launch_bounds__(256) void rcdc_copy_ranges_kernel(uint8_t *__restrict__ out,
                                                               const ulonglong4 *__restrict__ units,
                                                               uint32_t n) {
    const uint32_t t = threadIdx.x, ln = t & 63u;
    for (uint32_t k = blockIdx.x; k < n; k += gridDim.x) {
        const ulonglong4 u = units[k];  // src, dst, len, source base address
        const uint8_t *s = reinterpret_cast<const uint8_t *>((uintptr_t)(u.w + u.x));
        uint8_t *d = out + u.y;
        const uint64_t len = u.z;
        uint32_t head = (uint32_t)((16u - ((uintptr_t)d & 15u)) & 15u);
        if (head > len) head = (uint32_t)len;
        if (t < head) d[t] = s[t];
        const uint64_t body = (len - head) / 16;
        u32x4v *db = reinterpret_cast<u32x4v *>(d + head);
        // 16-aligned source loads; output chunk i takes aligned chunks i and
        // i + 1 (the neighbour lane's, lane 63 loads its own) funnelled by
        // the unit-uniform byte shift (the zstd copy kernel's scheme)
        const uint8_t *sb = s + head;
        const uint32_t sh = (uint32_t)(uintptr_t)sb & 15u, kk = sh >> 2, rr = (sh & 3u) * 8u;
        const u32x4v *s16 = reinterpret_cast<const u32x4v *>(sb - sh);
        auto funnel = [&](u32x4v A, u32x4v B) {
            uint32_t x0, x1, x2, x3, x4;
            if (kk == 0) {
                x0 = A.x; x1 = A.y; x2 = A.z; x3 = A.w; x4 = B.x;
            } else if (kk == 1) {
                x0 = A.y; x1 = A.z; x2 = A.w; x3 = B.x; x4 = B.y;
            } else if (kk == 2) {
                x0 = A.z; x1 = A.w; x2 = B.x; x3 = B.y; x4 = B.z;
            } else {
                x0 = A.w; x1 = B.x; x2 = B.y; x3 = B.z; x4 = B.w;
            }
            u32x4v v;
            v.x = __builtin_amdgcn_alignbit(x1, x0, rr);
            v.y = __builtin_amdgcn_alignbit(x2, x1, rr);
            v.z = __builtin_amdgcn_alignbit(x3, x2, rr);
            v.w = __builtin_amdgcn_alignbit(x4, x3, rr);
            return v;
        };
        auto nbr = [&](u32x4v A) {
            u32x4v B;
            B.x = __shfl_down(A.x, 1);
            B.y = __shfl_down(A.y, 1);
            B.z = __shfl_down(A.z, 1);
            B.w = __shfl_down(A.w, 1);
            return B;
        };
        uint64_t i0 = 0;
        for (; i0 + 1024 <= body; i0 += 1024) {
            u32x4v A[4], E[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                A[q] = __builtin_nontemporal_load(s16 + i0 + 256 * q + t);
                E[q] = A[q];
                if (sh && ln == 63u) E[q] = __builtin_nontemporal_load(s16 + i0 + 256 * q + t + 1);
            }
#pragma unroll
            for (int q = 0; q < 4; q++) {
                u32x4v v = A[q];
                if (sh) {
                    u32x4v B = nbr(A[q]);
                    if (ln == 63u) B = E[q];
                    v = funnel(A[q], B);
                }
                __builtin_nontemporal_store(v, db + i0 + 256 * q + t);
            }
        }
        for (uint64_t i = i0 + t; i0 < body; i0 += 256, i += 256) {
            // every lane of the wave runs the shuffle; lanes past the body
            // load nothing and store nothing
            const bool on = i < body;
            u32x4v A = {0u, 0u, 0u, 0u};
            if (on) A = __builtin_nontemporal_load(s16 + i);
            u32x4v v = A;
            if (sh) {
                u32x4v B = nbr(A);
                if (on && (ln == 63u || i + 1 >= body)) B = __builtin_nontemporal_load(s16 + i + 1);
                v = funnel(A, B);
            }
            if (on) __builtin_nontemporal_store(v, db + i);
        }
        const uint64_t done = head + 16 * body;
        if (t < len - done) d[done + t] = s[done + t];
    }
}

namespace rcdc {

// A plain copy by the shader, 16 bytes per lane per round, for a host <->
// device transfer through page-locked memory the device maps (zero-copy
// loads or stores over PCIe): the ingest's batch copies, so that HIP's DMA
// queues stay free for the small uploads and read-backs that would wait
// behind them (RCDC_INGEST_KCOPY).  len and both addresses 16-aligned.
__global__ __launch_bounds__(256) void rcdc_stream_copy_kernel(uint4 *__restrict__ dst,
                                                               const uint4 *__restrict__ src,
                                                               uint64_t n16) {
    const uint64_t stride = (uint64_t)gridDim.x * 256u * 4u;
    for (uint64_t i = (uint64_t)blockIdx.x * 1024u + threadIdx.x; i < n16; i += stride) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; u++)
            if (i + u * 256u < n16) v[u] = src[i + u * 256u];
#pragma unroll
        for (int u = 0; u < 4; u++)
            if (i + u * 256u < n16) dst[i + u * 256u] = v[u];
    }
}

hipError_t launch_stream_copy(void *dst, const void *src, uint64_t len, uint32_t blocks,
                              hipStream_t stream) {
    if (!len) return hipSuccess;
    if (((uintptr_t)dst | (uintptr_t)src | len) & 15u) return hipErrorInvalidValue;
    hipLaunchKernelGGL(rcdc_stream_copy_kernel, dim3(blocks), dim3(256), 0, stream, (uint4 *)dst,
                       (const uint4 *)src, len / 16u);
    return hipGetLastError();
}

hipError_t launch_copy_ranges(uint8_t *out, const void *units, uint32_t n, uint32_t cus,
                              hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const uint32_t g = n < cus * 8u ? n : cus * 8u;
    hipLaunchKernelGGL(rcdc_copy_ranges_kernel, dim3(g), dim3(256), 0, stream, out,
                       (const ulonglong4 *)units, n);
    return hipGetLastError();
}

}  // namespace rcdc
