// rcdc_zstd.hip -- blob compression on the device:
// repository version 2 compresses every new blob with zstd before sealing it
// (backend/decrypt.rs:478-506 `encode_all(data, level)`, called by the
// packer's process_data, blob/packer.rs:268-270).  The output is one zstd
// frame per blob (RFC 8878), readable by any zstd decoder -- rustic's
// `decode_all` (decrypt.rs:71-95) included.  The compressed bytes are not
// libzstd's (zstd-sys 2.0.16+zstd.1.5.7 in the reference's Cargo.lock): no
// two zstd versions promise equal output, and the format is the contract.
//
// Frame: magic, single-segment header with the content size, then blocks of
// kZstdBlock bytes.  A block is stored
//   RLE         when all its bytes are equal (not the frame's first block:
//               libzstd avoids that for old decoders; there it becomes one
//               literal + one offset-1 match),
//   compressed  raw literals + sequences coded with the predefined FSE
//               distributions (no table descriptions), when that saves more
//               than zstd's minimum gain (srcSize/64 + 2, ZSTD_minGain),
//   raw         otherwise.
//
// rcdc_zstd_block_kernel: one wave per block (persistent: grid-stride).
//   Match finding is wave-parallel greedy: a step tests 64 positions (lane l
//   at base + l * stride) against a hash table in LDS that holds, per
//   bucket, the last position inserted and its 4 bytes (so a candidate is
//   verified without touching memory); the first verified lane at or after
//   the anchor wins, its match is extended forward and backward by the whole
//   wave (256 bytes per compare), and selection continues after it.  Like
//   zstd_fast, the stride grows while no match is found (1 + run / 256,
//   at most 32), so incompressible blocks cost ~70 steps.  Sequences go to a
//   per-wave scratch; lane 0 then writes the FSE bitstream (last sequence
//   first, as ZSTD_encodeSequences), and only if the block is kept
//   compressed are the literals copied (a lane per short run, the wave per
//   long run).
// rcdc_zstd_frame_kernel: a thread per blob writes the frame header and the
//   output position of every block.
// rcdc_zstd_copy_kernel: a workgroup per block writes the block header and
//   its content (from the input when raw, from the scratch when compressed).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "rcdc_internal.h"

using namespace rcdc;

namespace rcdc {
constexpr uint32_t kZstdNone = 0xFFFFFFFFu;
constexpr int kZstdAccelShift = 8;         // stride = 1 + (bytes since the anchor >> 8)
constexpr uint32_t kZstdMaxStride = 32;
constexpr int kZstdCopyThreads = 256;
}  // namespace rcdc

// RCDC_ZSTD_DBG bit 2: per-phase clock sums (wall clock, 100 MHz) over all
// blocks: RLE check, parse, FSE, literal copy, blocks, sequences
__device__ unsigned long long g_zstd_prof[8];

namespace {

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

__device__ __forceinline__ uint32_t rdl(uint32_t v, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}

__device__ __forceinline__ uint32_t highbit(uint32_t v) { return 31u - (uint32_t)__clz(v); }

// 4 bytes at any alignment from the aligned dwords that hold them (a dword
// that holds a readable byte is readable: allocations are 4-byte granular).
// Branch-free: when aligned, alignbit(hi, lo, 0) is lo whatever hi is, so hi
// is loaded from the dword itself (no exec-masked load, no scalar unit work);
// the aligned pointer comes from p by arithmetic so the loads stay global.
__device__ __forceinline__ uint32_t ld4(const uint8_t *p) {
    const uint32_t b = (uint32_t)(uintptr_t)p & 3u;
    const uint32_t *w = (const uint32_t *)(p - b);
    const uint32_t lo = w[0];
    const uint32_t hi = w[b ? 1 : 0];
    return __builtin_amdgcn_alignbit(hi, lo, b * 8u);
}

// 16 bytes at any alignment (5 aligned dwords when misaligned).
__device__ __forceinline__ uint4 ld16(const uint8_t *p) {
    const uint32_t b = (uint32_t)(uintptr_t)p & 3u, sh = b * 8u;
    const uint32_t *w = (const uint32_t *)(p - b);
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3];
    const uint32_t w4 = w[b ? 4 : 3];
    return make_uint4(__builtin_amdgcn_alignbit(w1, w0, sh), __builtin_amdgcn_alignbit(w2, w1, sh),
                      __builtin_amdgcn_alignbit(w3, w2, sh), __builtin_amdgcn_alignbit(w4, w3, sh));
}

// First differing byte of two 16-byte groups (16 if equal); branch-free: a
// zero word counts as 128 bits, the first differing bit is the minimum.
__device__ __forceinline__ uint32_t first_diff16(uint4 a, uint4 b) {
    const uint32_t x0 = a.x ^ b.x, x1 = a.y ^ b.y, x2 = a.z ^ b.z, x3 = a.w ^ b.w;
    const uint32_t z0 = __builtin_ctzg(x0, 128), z1 = 32u + __builtin_ctzg(x1, 96);
    const uint32_t z2 = 64u + __builtin_ctzg(x2, 64), z3 = 96u + __builtin_ctzg(x3, 32);
    const uint32_t m01 = z0 < z1 ? z0 : z1, m23 = z2 < z3 ? z2 : z3;
    return (m01 < m23 ? m01 : m23) >> 3;
}

// 4 bytes at p where only [p, lim) may be read; missing bytes read as 0.
__device__ __forceinline__ uint32_t ld4_hi(const uint8_t *p, const uint8_t *lim) {
    if (p + 4 <= lim) return ld4(p);
    uint32_t v = 0;
    for (int i = 0; i < 4; i++)
        if (p + i < lim) v |= (uint32_t)p[i] << (8 * i);
    return v;
}

// 4 bytes at p where only [lo, p + 4) may be read; missing bytes read as 0.
__device__ __forceinline__ uint32_t ld4_lo(const uint8_t *p, const uint8_t *lo) {
    if (p >= lo) return ld4(p);
    uint32_t v = 0;
    for (int i = 0; i < 4; i++)
        if (p + i >= lo) v |= (uint32_t)p[i] << (8 * i);
    return v;
}

// Positions are keyed on their first `key` bytes (4 or 6) and matches are at
// least that long (zstd's fast levels use 5-6: on structured data shorter
// matches cost more sequence bits than the literals they replace; 6-byte keys
// pay only with enough buckets).
__device__ __forceinline__ uint64_t key48(uint32_t w, uint32_t w2, uint32_t key) {
    return key == 6   ? (uint64_t)w | (uint64_t)(w2 & 0xFFFFu) << 32
           : key == 5 ? (uint64_t)w | (uint64_t)(w2 & 0xFFu) << 32
                      : (uint64_t)w;
}

template <int HL>
__device__ __forceinline__ uint32_t zhash(uint64_t k) {
    return (uint32_t)((k * 0x9E3779B97F4A7C15ull) >> (64 - HL));
}

// Table entry: position (17 bits) | a 15-bit tag of its 4 bytes << 17, so a
// candidate touches memory only when its tag agrees (random data: ~2^-15).
// A position is at most kZstdBlock - 8, so the empty entry (all ones) is none.
__device__ __forceinline__ uint32_t ztag(uint64_t k) {
    return (uint32_t)((k * 0xC2B2AE3D27D4EB4Full) >> 49);
}
constexpr uint32_t kZstdPosMask = (1u << 17) - 1u;

// Narrow table (levels >= 3): 16-bit entries holding a position's low 16
// bits, twice the buckets in the same LDS (zstd's level-3 tables are 2^16-2^17;
// on structured data the history depth is what pays: CSV rows 0.29 -> 0.21 at
// 2^11 -> 2^12 positions in tests/zstd_model.py).  A bucket names the latest
// position below p with those low bits; candidates are verified on the bytes,
// so an older position 64 KiB away only costs a lost candidate.  0xFFFF is
// empty (a position with those low bits is lost).
constexpr uint32_t kZstdNone16 = 0xFFFFu;
__device__ __forceinline__ uint32_t narrow_cand(uint32_t e, uint32_t p) {
    if (e == kZstdNone16) return kZstdNone;
    const uint32_t c = (p & ~0xFFFFu) | e;
    return c < p ? c : (c >= 0x10000u ? c - 0x10000u : kZstdNone);
}

// key flags (ZstdStrategy.key): key bytes | kZstdRep (repeat codes) |
// kZstdRepCheck (every position also tries the last offset, zstd_fast's
// repcode check: taken before a table match, and one position later wins
// over a table match here)
constexpr uint32_t kZstdRep = 0x100u, kZstdRepCheck = 0x200u, kZstdInsAll = 0x400u,
                   kZstdRep1 = 0x800u, kZstdLazyRep = 0x1000u, kZstdAdaptKey = 0x2000u,
                   kZstdFar = 0x4000u;

// ---- far candidates (levels >= 3): matches into the blob's two previous
// blocks ----------------------------------------------------------------------
// A block's wave keeps only its own 64 KiB of history in LDS; zstd's level 3
// looks back over a 2 MiB window, and structured data repeats at such
// distances (CSV rows whose columns cycle every few hundred KiB).  Blocks stay
// independent: two kernels run before the parse,
//   far_build: per block, a table of 2^13 buckets holding the latest *sampled*
//     position (content-defined: the 8-byte key's hash has bits 20-21 zero, one
//     position in four; zstd's long-distance matcher samples with a rolling
//     hash mask the same way) with a 15-bit tag, in HBM;
//   far_map: per block and 16-byte group, the offset of a sampled position's
//     candidate in the tables of blocks b-1 and b-2 whose first kZstdFarMin
//     bytes agree (0: none);
// and the parse tries p - map[p / 16] beside its own table's candidate,
// keeping the longer match.  A single-segment frame's window is its content,
// so any offset into the blob is valid.  tools/zstd_ldm_model.py: CSV rows
// 0.195 -> 0.145, code lines 0.117 -> 0.108, word text unchanged (1 MiB blobs).
constexpr int kZstdFarLog = 13;
constexpr uint32_t kZstdFarTab = 1u << kZstdFarLog;
constexpr uint32_t kZstdFarGroups = kZstdBlock / 16u;
constexpr uint32_t kZstdFarSample = 3u;  // hash bits 20-21: one position in four

struct FarLayout {
    uint32_t *tab;   // [nblk][kZstdFarTab]: (position + 1) << 15 | tag, 0 empty
    uint32_t *map;   // [nblk][kZstdFarGroups]: offset (blob-relative distance), 0 none
    uint32_t *comp;  // [nblk]: the block looked compressible (its table is built)
    uint32_t *has;   // [nblk]: its map holds an offset
};
__device__ __forceinline__ FarLayout far_layout(uint32_t *far, uint32_t nblk) {
    FarLayout L;
    L.tab = far;
    L.map = far + (size_t)nblk * kZstdFarTab;
    L.comp = L.map + (size_t)nblk * kZstdFarGroups;
    L.has = L.comp + nblk;
    return L;
}

__device__ __forceinline__ uint64_t far_hash(uint64_t k6) { return k6 * 0x9E3779B97F4A7C15ull; }
__device__ __forceinline__ bool far_sampled(uint64_t hv) { return ((hv >> 20) & kZstdFarSample) == 0; }
__device__ __forceinline__ uint32_t far_bucket(uint64_t hv) { return (uint32_t)(hv >> (64 - kZstdFarLog)); }
__device__ __forceinline__ uint32_t far_tag(uint64_t hv) { return (uint32_t)(hv >> 36) & 0x7FFFu; }

// 16 bytes at p where only [p, lim) may be read; missing bytes read as 0.
__device__ __forceinline__ uint4 ld16_lim(const uint8_t *p, const uint8_t *lim) {
    if (p + 20 <= lim) return ld16(p);
    return make_uint4(ld4_hi(p, lim), ld4_hi(p + 4, lim), ld4_hi(p + 8, lim), ld4_hi(p + 12, lim));
}

// The 8 bytes at byte j (0..23) of the 32 bytes u[0..3] (little-endian words).
__device__ __forceinline__ uint64_t bytes8_at(const uint64_t u[4], uint32_t j) {
    const uint32_t i = j >> 3, sh = (j & 7u) * 8u;
    const uint64_t lo = u[i] >> sh, hi = sh ? u[i + 1] << (64u - sh) : 0ull;
    return lo | hi;
}

// The map keeps only candidates whose first kZstdFarMin bytes agree (the
// 8-byte key itself: tools/zstd_ldm_model.py CSV rows 0.143 at 8, 0.156 at
// 12, 0.182 at 16), so a block with none skips the far path.
constexpr uint32_t kZstdFarMin = 8;
constexpr uint32_t kZstdFarDense = 8;  // far path when >= 1/8 of the groups hold an offset

// Equal bytes of a[0..) and b[0..), at most maxlen (wave-uniform result).
// Lane l compares 16 bytes per round (1 KiB per wave round); the last,
// partial groups go byte-safe.
__device__ uint32_t wave_match_fwd(const uint8_t *a, const uint8_t *b, uint32_t maxlen,
                                   const uint8_t *lim) {
    const uint32_t lane = lane_id();
    uint32_t len = 0;
    while (len < maxlen) {
        const uint32_t o = len + lane * 16u;
        uint32_t d = 0;  // first differing byte in this lane's group (16: none)
        if (o + 16 <= maxlen) {
            d = first_diff16(ld16(a + o), ld16(b + o));
        } else if (o < maxlen) {
            d = 16;
            for (uint32_t q = 0; q < 16; q += 4) {
                uint32_t x = ld4_hi(a + o + q, lim) ^ ld4_hi(b + o + q, lim);
                const uint32_t rem = maxlen - o - q;
                if (rem < 4) x |= 0xFFFFFFFFu << (8 * rem);
                if (x) {
                    d = q + ((uint32_t)__builtin_ctz(x) >> 3);
                    break;
                }
            }
        }
        const uint64_t m = __ballot(o < maxlen ? d < 16 : true);
        if (m) {
            const int j = __builtin_ctzll(m);
            len += (uint32_t)j * 16u + rdl(d, j);
            return len < maxlen ? len : maxlen;
        }
        len += 1024;
    }
    return maxlen;
}

// Equal bytes going backward from a[-1] and b[-1], at most maxback; only
// bytes at or after lo may be read.
__device__ uint32_t wave_match_back(const uint8_t *a, const uint8_t *b, uint32_t maxback,
                                    const uint8_t *lo) {
    const uint32_t lane = lane_id();
    uint32_t back = 0;
    while (back < maxback) {
        const uint32_t o = back + lane * 4u;  // bytes a[-o-4 .. -o)
        uint32_t x = 0xFFFFFFFFu;
        if (o < maxback) {
            const uint32_t cnt = maxback - o;  // valid bytes from the top
            x = ld4_lo(a - o - 4, lo) ^ ld4_lo(b - o - 4, lo);
            if (cnt < 4) x |= 0xFFFFFFFFu >> (8 * cnt);
        }
        const uint64_t m = __ballot(x != 0);
        if (m) {
            const int j = __builtin_ctzll(m);
            const uint32_t xj = rdl(x, j);
            back += (uint32_t)j * 4u + ((uint32_t)__builtin_clz(xj) >> 3);
            return back < maxback ? back : maxback;
        }
        back += 256;
    }
    return maxback;
}

// The wave copies n bytes (dword stores once dst is aligned).
__device__ void wave_copy(uint8_t *dst, const uint8_t *src, uint32_t n) {
    const uint32_t lane = lane_id();
    uint32_t head = (uint32_t)((4u - ((uint32_t)(uintptr_t)dst & 3u)) & 3u);
    if (head > n) head = n;
    if (lane < head) dst[lane] = src[lane];
    dst += head;
    src += head;
    n -= head;
    const uint32_t nd = n >> 2;
    for (uint32_t k = lane; k < nd; k += 64) ((uint32_t *)dst)[k] = ld4(src + 4 * k);
    const uint32_t t = nd * 4;
    if (lane < n - t) dst[t + lane] = src[t + lane];
}

// Equal bytes counted down from the top of two 16-byte groups (16 if equal).
__device__ __forceinline__ uint32_t last_eq16(uint4 a, uint4 b) {
    const uint32_t x0 = a.x ^ b.x, x1 = a.y ^ b.y, x2 = a.z ^ b.z, x3 = a.w ^ b.w;
    const uint32_t z3 = __builtin_clzg(x3, 128), z2 = 32u + __builtin_clzg(x2, 96);
    const uint32_t z1 = 64u + __builtin_clzg(x1, 64), z0 = 96u + __builtin_clzg(x0, 32);
    const uint32_t m32 = z3 < z2 ? z3 : z2, m10 = z1 < z0 ? z1 : z0;
    return (m32 < m10 ? m32 : m10) >> 3;
}

// sequence record: literal length | match length << 20 | offset value << 40
// (a repeat code 1-3, or offset + 3)
__device__ __forceinline__ uint64_t seq_pack(uint32_t ll, uint32_t ml, uint32_t off) {
    return (uint64_t)ll | (uint64_t)ml << 20 | (uint64_t)off << 40;
}

struct SeqCodes {
    uint32_t llc, mlc, ofc, ll, mlb, ofv;
};

__device__ __forceinline__ SeqCodes seq_codes(uint64_t s, const ZstdTables &T) {
    SeqCodes c;
    c.ll = (uint32_t)(s & 0xFFFFF);
    const uint32_t ml = (uint32_t)((s >> 20) & 0xFFFFF);
    c.ofv = (uint32_t)(s >> 40);
    c.mlb = ml - 3u;
    c.llc = c.ll < 64 ? T.llcode[c.ll] : highbit(c.ll) + 19u;
    c.mlc = c.mlb < 128 ? T.mlcode[c.mlb] : highbit(c.mlb) + 36u;
    c.ofc = highbit(c.ofv);
    return c;
}

// The FSE tables in VGPRs, for the scalar state chains: lane s holds symbol
// s's {deltaFindState, deltaNbBits}, lane t the state table's entry t.
struct FseRegs {
    uint32_t llF, llN, mlF, mlN, ofF, ofN, llS, mlS, ofS;
};

__device__ FseRegs fse_regs(const ZstdTables &T) {
    const uint32_t l = lane_id();
    FseRegs r;
    r.llF = l < 36 ? (uint32_t)T.ll[l].find : 0u;
    r.llN = l < 36 ? T.ll[l].nbits : 0u;
    r.mlF = l < 53 ? (uint32_t)T.ml[l].find : 0u;
    r.mlN = l < 53 ? T.ml[l].nbits : 0u;
    r.ofF = l < 32 ? (uint32_t)T.of[l].find : 0u;
    r.ofN = l < 32 ? T.of[l].nbits : 0u;
    r.llS = T.llst[l];
    r.mlS = T.mlst[l];
    r.ofS = l < 32 ? T.ofst[l] : 0u;
    return r;
}

// FSE_initCState2 / FSE_encodeSymbol on wave-uniform values (SALU + readlane).
__device__ __forceinline__ uint32_t fse_init_s(uint32_t F, uint32_t N, uint32_t S, uint32_t sym) {
    const uint32_t nb = rdl(N, (int)sym);
    const int32_t f = (int32_t)rdl(F, (int)sym);
    const uint32_t nbo = (nb + (1u << 15)) >> 16;
    const uint32_t v = (nbo << 16) - nb;
    return rdl(S, (int)((int32_t)(v >> nbo) + f));
}

__device__ __forceinline__ uint32_t fse_enc_s(uint32_t F, uint32_t N, uint32_t S, uint32_t sym,
                                              uint32_t st, uint32_t &field) {
    const uint32_t nb = rdl(N, (int)sym);
    const int32_t f = (int32_t)rdl(F, (int)sym);
    const uint32_t nbo = (st + nb) >> 16;
    field = (st & ((1u << nbo) - 1u)) | nbo << 16;
    return rdl(S, (int)((int32_t)(st >> nbo) + f));
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
    return v;
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t o = __shfl_xor(v, d);
        v = o > v ? o : v;
    }
    return v;
}

__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t o = __shfl_xor(v, d);
        v = o < v ? o : v;
    }
    return v;
}

// OR n bits of v (n <= 25) into the LDS bit buffer at bit q.
__device__ __forceinline__ void put_bits(uint32_t *buf, uint32_t q, uint32_t v, uint32_t n) {
    if (!n) return;
    v &= (1u << n) - 1u;
    const uint32_t w = q >> 5, sh = q & 31u;
    atomicOr(&buf[w], v << sh);
    if (sh + n > 32) atomicOr(&buf[w + 1], v >> (32 - sh));
}

// LDS ordering inside the one-wave workgroup: a wave's LDS operations run in
// order, so only the compiler must not move them (no wait for global stores).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint32_t wl(uint32_t v, int lane, uint32_t old) {
    return lane_id() == (uint32_t)lane ? v : old;
}

// FSE_writeNCount of normalized counts nrm[0 .. nsymt) at accuracy log 6
// (RFC 8878 4.1.1), by lane 0; returns the bytes (wave-uniform).
__device__ uint32_t ncount_write(const uint32_t *nrm, uint32_t nsymt, uint8_t *out,
                                 uint32_t cap) {
    uint32_t nbytes = 0;
    if (lane_id() == 0) {
        uint64_t acc = 6u - 5u;  // accuracy log - 5, in 4 bits
        uint32_t nb = 4, o = 0;
        uint32_t remaining = 65, threshold = 64, nbits = 7, sy = 0;
        bool prev0 = false;
        while (sy < nsymt && remaining > 1) {
            if (prev0) {
                uint32_t st0 = sy;
                while (sy < nsymt && nrm[sy] == 0) sy++;
                while (sy >= st0 + 24) {
                    st0 += 24;
                    acc |= (uint64_t)0xFFFF << nb;
                    nb += 16;
                    while (nb >= 8) {
                        if (o < cap) out[o] = (uint8_t)acc;
                        o++;
                        acc >>= 8;
                        nb -= 8;
                    }
                }
                while (sy >= st0 + 3) {
                    st0 += 3;
                    acc |= (uint64_t)3 << nb;
                    nb += 2;
                }
                acc |= (uint64_t)(sy - st0) << nb;
                nb += 2;
            }
            uint32_t count = nrm[sy++];
            const uint32_t mx = (2 * threshold - 1) - remaining;
            remaining -= count;
            count += 1;
            if (count >= threshold) count += mx;
            acc |= (uint64_t)count << nb;
            nb += nbits - (count < mx ? 1u : 0u);
            prev0 = count == 1;
            while (remaining < threshold) {
                nbits--;
                threshold >>= 1;
            }
            while (nb >= 8) {
                if (o < cap) out[o] = (uint8_t)acc;
                o++;
                acc >>= 8;
                nb -= 8;
            }
        }
        if (nb) {
            if (o < cap) out[o] = (uint8_t)acc;
            o++;
        }
        nbytes = o;
    }
    return rdl(nbytes, 0);
}

// FSE_buildCTable of a log-6 table with no low-probability symbols, lane s
// holding symbol s's normalized count an: returns the lane's {find, nbits}
// (symbol s) and state-table entry (state lane).  The spread is position
// (43 k) mod 64 for occurrence k; the state table comes from ranks.
__device__ void fse_build_log6(uint32_t an, uint32_t *lds, uint32_t &F, uint32_t &N,
                               uint32_t &S) {
    const uint32_t lane = lane_id();
    uint32_t *cum = lds + 64, *occ = lds + 128, *pos = lds + 192, *stt = lds + 256;
    uint32_t inc = an;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d);
        if ((int)lane >= d) inc += y;
    }
    const uint32_t c0 = inc - an;  // cumulative count before this symbol
    cum[lane] = c0;
    for (uint32_t j = 0; j < an; j++) occ[c0 + j] = lane;  // occurrence -> symbol
    wave_lds_sync();
    pos[(lane * 43u) & 63u] = occ[lane];  // the spread: step 64/2 + 64/8 + 3
    wave_lds_sync();
    const uint32_t sym = pos[lane];
    uint32_t rank = 0;
    for (uint32_t u = 0; u < lane; u++) rank += pos[u] == sym;
    stt[cum[sym] + rank] = 64u + lane;
    wave_lds_sync();
    S = stt[lane];
    if (an == 0) {
        N = (7u << 16) - 64u;
        F = 0;
    } else if (an == 1) {
        N = (6u << 16) - 64u;
        F = c0 - 1u;
    } else {
        const uint32_t mbo = 6u - (31u - (uint32_t)__clz(an - 1));
        N = (mbo << 16) - (an << mbo);
        F = c0 - an;
    }
    wave_lds_sync();
}

// Per stream (LL, OF, ML): predefined table, or an adaptive one of accuracy
// log 6 (FSE_Compressed mode) when its estimated bits, description included,
// are fewer.  Adaptive counts: rounded shares of 64, present symbols >= 1, the
// difference given to / taken from the largest (tests/zstd_model.py
// fse_normalize).  Log 6 keeps every table at <= 64 entries: one per lane,
// so the scalar state chains read them with v_readlane as the predefined
// ones.  Writes the description (FSE_writeNCount) at out and returns its
// bytes; updates the stream's registers and table log.
__device__ uint32_t fse_choose(uint32_t t, uint32_t nsymt, const uint32_t *hist, uint32_t nseq,
                               uint32_t tlp, uint32_t predN, uint32_t &F, uint32_t &N, uint32_t &S,
                               uint32_t &tl, uint32_t *lds, uint8_t *out, uint32_t cap) {
    const uint32_t lane = lane_id();
    uint32_t *nrm = lds;
    const uint32_t cnt = lane < nsymt ? hist[t * 64 + lane] : 0u;
    // predefined cost: its count c from deltaNbBits (c = ((mbo << 16) - nb) >> mbo, mbo = nb >> 16 + 1)
    float pc = 0.f, ac = 0.f;
    if (cnt) {
        const uint32_t mbo = (predN >> 16) + 1;
        const uint32_t cp = ((mbo << 16) - predN) >> mbo;
        pc = (float)cnt * ((float)tlp - __log2f((float)cp));
    }
    uint32_t an = cnt ? (cnt * 64u + nseq / 2) / nseq : 0u;
    if (cnt && an == 0) an = 1;
    int32_t diff = 64 - (int32_t)wave_sum(an);
    // give to / take from the largest (lowest symbol on ties)
    while (diff != 0) {
        const uint32_t key = wave_max(cnt ? an << 8 | (255u - lane) : 0u);
        const uint32_t big = 255u - (key & 0xFFu);
        if (diff > 0) {
            if (lane == big) an += (uint32_t)diff;
            diff = 0;
        } else {
            if (lane == big) an -= 1;
            diff += 1;
        }
    }
    if (cnt) ac = (float)cnt * (6.f - __log2f((float)an));
    for (int d = 32; d >= 1; d >>= 1) {
        pc += __shfl_xor(pc, d);
        ac += __shfl_xor(ac, d);
    }
    nrm[lane] = an;
    wave_lds_sync();
    // the description (FSE_writeNCount), by lane 0
    const uint32_t nbytes = ncount_write(nrm, nsymt, out, cap);

    if (ac + 8.f * (float)nbytes >= pc || nbytes > cap) return 0;  // predefined
    fse_build_log6(an, lds, F, N, S);
    tl = 6;
    wave_lds_sync();
    return nbytes;
}

// The sequences section after Number_of_Sequences: the modes byte, the
// adaptive tables' descriptions (LL, OF, ML) and the bitstream
// (ZSTD_encodeSequences order: the last sequence first, its states
// initialised from it; then per sequence OF, ML, LL state bits and LL, ML,
// OF extra bits; the final states; the end mark), by the whole wave: 64
// sequences per round, the three state chains stepped as scalar code, every
// field OR-ed into an LDS bit buffer at its prefix-sum position, full words
// stored.  Returns its bytes, or kZstdNone past cap.
__device__ uint32_t wave_fse_sequences(const uint64_t *seqs, uint32_t nseq, const ZstdTables &T,
                                       const FseRegs &R0, uint32_t *buf, uint8_t *out,
                                       uint32_t cap) {
    const uint32_t lane = lane_id();
    // code histograms (LL, OF, ML) for the table choice
    uint32_t *hist = buf + 1024;
    for (uint32_t i = lane; i < 192; i += 64) hist[i] = 0;
    wave_lds_sync();
    for (uint32_t c0 = 0; c0 < nseq; c0 += 64) {
        if (c0 + lane < nseq) {
            const SeqCodes c = seq_codes(seqs[c0 + lane], T);
            atomicAdd(&hist[c.llc], 1u);
            atomicAdd(&hist[64 + c.ofc], 1u);
            atomicAdd(&hist[128 + c.mlc], 1u);
        }
    }
    wave_lds_sync();
    FseRegs R = R0;
    uint32_t tll = 6, tof = 5, tml = 6;
    if (cap < 2) return kZstdNone;
    uint32_t o = 1;
    const uint32_t dl = fse_choose(0, 36, hist, nseq, 6, R0.llN, R.llF, R.llN, R.llS, tll,
                                   buf + 1216, out + o, cap - o);
    o += dl;
    const uint32_t dof = fse_choose(1, 32, hist, nseq, 5, R0.ofN, R.ofF, R.ofN, R.ofS, tof,
                                    buf + 1216, out + o, cap - o);
    o += dof;
    const uint32_t dml = fse_choose(2, 53, hist, nseq, 6, R0.mlN, R.mlF, R.mlN, R.mlS, tml,
                                    buf + 1216, out + o, cap - o);
    o += dml;
    if (lane == 0) out[0] = (uint8_t)((dl ? 2u : 0u) << 6 | (dof ? 2u : 0u) << 4 | (dml ? 2u : 0u) << 2);
    if (o >= cap) return kZstdNone;
    uint8_t *const out0 = out;
    out += o;
    cap -= o;
    // the three state chains run on lanes 0 (OF), 1 (ML), 2 (LL) in VALU over
    // LDS copies of the tables (the scalar unit, shared by the CU's waves, is
    // the parse's bottleneck): buf[256, 832) tables, [832, 1024) the round's
    // symbol codes, [1024, 1216) (the histograms, done) the state fields
    uint32_t *ctN = buf + 256, *ctF = buf + 448, *ctS = buf + 640, *csym = buf + 832,
             *cfld = buf + 1024;
    ctN[lane] = R.ofN;
    ctN[64 + lane] = R.mlN;
    ctN[128 + lane] = R.llN;
    ctF[lane] = R.ofF;
    ctF[64 + lane] = R.mlF;
    ctF[128 + lane] = R.llF;
    ctS[lane] = R.ofS;
    ctS[64 + lane] = R.mlS;
    ctS[128 + lane] = R.llS;
    uint32_t sch = 0;  // lane k < 3: chain k's state
    uint32_t bitpos = 0, wbase = 0;  // bits written; bit index of buf[0] (multiple of 32)
    if (lane == 0) buf[0] = 0;
    wave_lds_sync();
    for (int64_t hi = (int64_t)nseq - 1; hi >= 0; hi -= 64) {
        const uint32_t cnt = hi + 1 < 64 ? (uint32_t)hi + 1 : 64u;
        const bool val = lane < cnt;
        SeqCodes c{0, 0, 0, 0, 0, 0};
        if (val) c = seq_codes(seqs[hi - lane], T);
        const uint32_t nll = val ? T.llbits[c.llc] : 0u, nml = val ? T.mlbits[c.mlc] : 0u;
        if (val) {
            csym[3 * lane] = c.ofc;
            csym[3 * lane + 1] = c.mlc;
            csym[3 * lane + 2] = c.llc;
        }
        wave_lds_sync();
        if (lane < 3) {
            // FSE_initCState2 from the last sequence, then FSE_encodeSymbol
            const uint32_t tb = lane * 64u;
            uint32_t L = 0;
            if ((uint64_t)hi == (uint64_t)nseq - 1) {
                const uint32_t sy = csym[lane], nb = ctN[tb + sy];
                const uint32_t nbo = (nb + (1u << 15)) >> 16;
                const uint32_t v = (nbo << 16) - nb;
                sch = ctS[tb + (uint32_t)((int32_t)(v >> nbo) + (int32_t)ctF[tb + sy])];
                cfld[lane] = 0;
                L = 1;
            }
            for (; L < cnt; L++) {
                const uint32_t sy = csym[3 * L + lane];
                const uint32_t nb = ctN[tb + sy];
                const int32_t f = (int32_t)ctF[tb + sy];
                const uint32_t nbo = (sch + nb) >> 16;
                cfld[3 * L + lane] = (sch & ((1u << nbo) - 1u)) | nbo << 16;
                sch = ctS[tb + (uint32_t)((int32_t)(sch >> nbo) + f)];
            }
        }
        wave_lds_sync();
        uint32_t fOF = 0, fML = 0, fLL = 0;
        if (val) {
            fOF = cfld[3 * lane];
            fML = cfld[3 * lane + 1];
            fLL = cfld[3 * lane + 2];
        }
        const uint32_t total =
            val ? (fOF >> 16) + (fML >> 16) + (fLL >> 16) + nll + nml + c.ofc : 0u;
        uint32_t incl = total;
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(incl, d);
            if ((int)lane >= d) incl += y;
        }
        const uint32_t chunk_bits = rdl(incl, 63);
        const uint32_t start = bitpos - wbase, endbit = start + chunk_bits;
        for (uint32_t w = 1 + lane; w <= (endbit >> 5) + 1; w += 64) buf[w] = 0;
        wave_lds_sync();
        if (val) {
            uint32_t q = start + incl - total;
            put_bits(buf, q, fOF, fOF >> 16);
            q += fOF >> 16;
            put_bits(buf, q, fML, fML >> 16);
            q += fML >> 16;
            put_bits(buf, q, fLL, fLL >> 16);
            q += fLL >> 16;
            put_bits(buf, q, c.ll, nll);
            q += nll;
            put_bits(buf, q, c.mlb, nml);
            q += nml;
            put_bits(buf, q, c.ofv, c.ofc);
        }
        wave_lds_sync();
        const uint32_t full = endbit >> 5;
        if ((wbase >> 3) + full * 4u > cap) return kZstdNone;
        uint8_t *o = out + (wbase >> 3);
        for (uint32_t w = lane; w < full; w += 64) {
            const uint32_t v = buf[w];
            o[4 * w] = (uint8_t)v;
            o[4 * w + 1] = (uint8_t)(v >> 8);
            o[4 * w + 2] = (uint8_t)(v >> 16);
            o[4 * w + 3] = (uint8_t)(v >> 24);
        }
        const uint32_t carry = buf[full];
        wave_lds_sync();
        if (lane == 0) buf[0] = carry;
        wave_lds_sync();
        wbase += full * 32u;
        bitpos += chunk_bits;
    }
    // final states (FSE_flushCState: ML, OF, LL) and the end mark
    const uint32_t start = bitpos - wbase;
    const uint32_t sOF = rdl(sch, 0), sML = rdl(sch, 1), sLL = rdl(sch, 2);
    if (lane == 0) {
        buf[1] = 0;
        put_bits(buf, start, sML, tml);
        put_bits(buf, start + tml, sOF, tof);
        put_bits(buf, start + tml + tof, sLL, tll);
        put_bits(buf, start + tml + tof + tll, 1, 1);
    }
    wave_lds_sync();
    const uint32_t nbytes = (start + tml + tof + tll + 1 + 7) >> 3;  // <= 8
    if ((wbase >> 3) + nbytes > cap) return kZstdNone;
    if (lane < nbytes) out[(wbase >> 3) + lane] = (uint8_t)(buf[lane >> 2] >> (8 * (lane & 3)));
    return (uint32_t)(out - out0) + (wbase >> 3) + nbytes;
}

// ---- literals section (RFC 8878 3.1.1.3.1): raw, RLE or Huffman (4 streams,
// direct 4-bit weights) -------------------------------------------------------

constexpr uint32_t kHufMaxBits = 11;

__device__ __forceinline__ uint32_t byte_of(uint4 v, uint32_t k) {
    const uint32_t w = k < 8 ? (k < 4 ? v.x : v.y) : (k < 12 ? v.z : v.w);
    return (w >> (8 * (k & 3))) & 0xFFu;
}

// Raw/RLE literals header (Size_Format by size: 1, 2 or 3 bytes).
__device__ uint32_t lit_hdr_raw(uint8_t *out, uint32_t type, uint32_t n) {
    if (n < 32) {
        out[0] = (uint8_t)(type | n << 3);
        return 1;
    }
    if (n < 4096) {
        const uint32_t v = type | 1u << 2 | n << 4;
        out[0] = (uint8_t)v;
        out[1] = (uint8_t)(v >> 8);
        return 2;
    }
    const uint32_t v = type | 3u << 2 | n << 4;
    out[0] = (uint8_t)v;
    out[1] = (uint8_t)(v >> 8);
    out[2] = (uint8_t)(v >> 16);
    return 3;
}

// One Huffman stream: literals [a, b) of lbuf, the last one first (as
// HUF_compress1X), then the end mark; rounds of 1024 literals (lane l takes
// 16 of them), codes OR-ed into the LDS bit buffer at prefix-sum positions.
__device__ void huf_stream(const uint8_t *lbuf, uint32_t a, uint32_t b, const uint32_t *code,
                           uint32_t *buf, uint8_t *out) {
    const uint32_t lane = lane_id();
    uint32_t bitpos = 0, wbase = 0;
    if (lane == 0) buf[0] = 0;
    wave_lds_sync();
    const uint32_t len = b - a;
    for (uint32_t t0 = 0; t0 < len; t0 += 1024) {
        const uint32_t tl = t0 + 16u * lane;
        uint32_t cnt = 0, bits = 0;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (tl < len) {
            cnt = len - tl < 16 ? len - tl : 16u;
            // literal b-1-tl is byte 15.  The first stream's last group
            // starts before lbuf, which is the scratch buffer's first byte
            // for wave 0 when its block has no sequences: only bytes at or
            // after lbuf are read (a 16-byte load there faulted, r6 zstd soak)
            const uint8_t *p = lbuf + b - tl - 16;
            if (b - tl >= 16)
                v = ld16(p);
            else
                v = make_uint4(ld4_lo(p, lbuf), ld4_lo(p + 4, lbuf), ld4_lo(p + 8, lbuf),
                               ld4_lo(p + 12, lbuf));
            for (uint32_t k = 0; k < cnt; k++) bits += code[byte_of(v, 15 - k)] >> 16;
        }
        uint32_t incl = bits;
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(incl, d);
            if ((int)lane >= d) incl += y;
        }
        const uint32_t chunk_bits = rdl(incl, 63);
        const uint32_t start = bitpos - wbase, endbit = start + chunk_bits;
        for (uint32_t w = 1 + lane; w <= (endbit >> 5) + 1; w += 64) buf[w] = 0;
        wave_lds_sync();
        uint32_t q = start + incl - bits;
        for (uint32_t k = 0; k < cnt; k++) {
            const uint32_t cd = code[byte_of(v, 15 - k)];
            put_bits(buf, q, cd & 0xFFFFu, cd >> 16);
            q += cd >> 16;
        }
        wave_lds_sync();
        const uint32_t full = endbit >> 5;
        uint8_t *o = out + (wbase >> 3);
        for (uint32_t w = lane; w < full; w += 64) {
            const uint32_t x = buf[w];
            o[4 * w] = (uint8_t)x;
            o[4 * w + 1] = (uint8_t)(x >> 8);
            o[4 * w + 2] = (uint8_t)(x >> 16);
            o[4 * w + 3] = (uint8_t)(x >> 24);
        }
        const uint32_t carry = buf[full];
        wave_lds_sync();
        if (lane == 0) buf[0] = carry;
        wave_lds_sync();
        wbase += full * 32u;
        bitpos += chunk_bits;
    }
    const uint32_t start = bitpos - wbase;
    if (lane == 0) {
        buf[1] = 0;
        put_bits(buf, start, 1, 1);  // end mark
    }
    wave_lds_sync();
    const uint32_t nbytes = (start + 1 + 7) >> 3;
    if (lane < nbytes) out[(wbase >> 3) + lane] = (uint8_t)(buf[lane >> 2] >> (8 * (lane & 3)));
    wave_lds_sync();
}


// Huffman weights of symbols 0 .. n-1 (n <= 255, in wts) as an FSE stream
// (RFC 8878 4.2.1.2): accuracy log 6, NCount description, then two
// interleaved states in FSE_compress_usingCTable order (tests/zstd_model.py
// fse_compress_weights).  Returns the bytes (< 128), or 0 if not codable.
__device__ uint32_t fse_weights(const uint32_t *wts, uint32_t n, uint32_t *lds, uint8_t *out,
                                uint32_t cap) {
    const uint32_t lane = lane_id();
    uint32_t cnt = 0;
    for (uint32_t i = 0; i < n; i++) cnt += wts[i] == lane;  // lane v counts weight v
    if (lane >= 12) cnt = 0;
    if (wave_sum(cnt ? 1u : 0u) < 2) return 0;
    uint32_t an = cnt ? (cnt * 64u + n / 2) / n : 0u;
    if (cnt && an == 0) an = 1;
    int32_t diff = 64 - (int32_t)wave_sum(an);
    while (diff != 0) {
        const uint32_t key = wave_max(cnt ? an << 8 | (255u - lane) : 0u);
        const uint32_t big = 255u - (key & 0xFFu);
        if (diff > 0) {
            if (lane == big) an += (uint32_t)diff;
            diff = 0;
        } else {
            if (lane == big) an -= 1;
            diff += 1;
        }
    }
    uint32_t *nrm = lds;
    nrm[lane] = an;
    wave_lds_sync();
    const uint32_t nb0 = ncount_write(nrm, 12, out, cap);
    uint32_t F, N, S;
    fse_build_log6(an, lds, F, N, S);
    // the stream, as scalar code: the last weight first, two states
    uint64_t acc = 0;
    uint32_t nb = 0, o = nb0;
    auto add = [&](uint32_t v, uint32_t bits) {
        acc |= (uint64_t)(v & ((1u << bits) - 1u)) << nb;
        nb += bits;
    };
    auto flush = [&]() {
        while (nb >= 8) {
            if (lane == 0 && o < cap) out[o] = (uint8_t)acc;
            o++;
            acc >>= 8;
            nb -= 8;
        }
    };
    auto sym_at = [&](uint32_t i) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)wts[i]); };
    auto init = [&](uint32_t sy) { return fse_init_s(F, N, S, sy); };
    auto enc = [&](uint32_t st, uint32_t sy) {
        uint32_t field;
        const uint32_t ns = fse_enc_s(F, N, S, sy, st, field);
        add(field & 0xFFFFu, field >> 16);
        return ns;
    };
    uint32_t ip = n, s1, s2;
    if (n & 1) {
        s1 = init(sym_at(ip - 1));
        s2 = init(sym_at(ip - 2));
        s1 = enc(s1, sym_at(ip - 3));
        ip -= 3;
        flush();
    } else {
        s2 = init(sym_at(ip - 1));
        s1 = init(sym_at(ip - 2));
        ip -= 2;
    }
    if ((n - 2) & 2) {
        s2 = enc(s2, sym_at(ip - 1));
        s1 = enc(s1, sym_at(ip - 2));
        ip -= 2;
        flush();
    }
    while (ip > 0) {
        s2 = enc(s2, sym_at(ip - 1));
        s1 = enc(s1, sym_at(ip - 2));
        s2 = enc(s2, sym_at(ip - 3));
        s1 = enc(s1, sym_at(ip - 4));
        ip -= 4;
        flush();
    }
    add(s2, 6);
    flush();
    add(s1, 6);
    add(1, 1);
    flush();
    if (nb) {
        if (lane == 0 && o < cap) out[o] = (uint8_t)acc;
        o++;
    }
    wave_lds_sync();
    return o < 128 && o <= cap ? o : 0u;
}

// The literals section of a block into out; returns its bytes.  Huffman with
// 4 streams when the literal alphabet fits direct weights (bytes <= 128) and
// it is smaller than raw; RLE when one byte value; raw otherwise.  Code
// lengths: Shannon lengths ceil(log2(n / count)) clamped to 11 bits, the
// Kraft sum repaired (lengthen the shortest code below 11 while above 1) and
// filled (shortest codes first, shorten while the slack allows);
// tests/zstd_model.py restates it.  lds: 2048 words of LDS.
__device__ uint32_t encode_literals(const uint8_t *lbuf, uint32_t nl, uint8_t *out,
                                    uint32_t *lds) {
    const uint32_t lane = lane_id();
    if (nl >= 64) {
        uint32_t *hist = lds, *code = lds + 256, *wts = lds + 512, *st = lds + 768;
        uint32_t *buf = lds + 1024;
        for (uint32_t i = lane; i < 256; i += 64) hist[i] = 0;
        wave_lds_sync();
        for (uint32_t k = lane * 16u; k < nl; k += 1024) {
            const uint4 v = ld16(lbuf + k);
            const uint32_t c = nl - k < 16 ? nl - k : 16u;
            for (uint32_t j = 0; j < c; j++) atomicAdd(&hist[byte_of(v, j)], 1u);
        }
        wave_lds_sync();
        uint32_t c[4], L[4];
        uint32_t mx = 0, ns = 0;
        for (int j = 0; j < 4; j++) {
            c[j] = hist[lane + 64 * j];
            if (c[j]) {
                mx = lane + 64u * j;
                ns++;
            }
        }
        const uint32_t maxsym = wave_max(mx), nsym = wave_sum(ns);
        if (nsym == 1) {  // RLE literals
            const uint32_t h = lit_hdr_raw(out, 1, nl);
            if (lane == 0) out[h] = (uint8_t)maxsym;
            return h + 1;
        }
        // order-0 entropy bound: skip the Huffman work when it cannot pay
        // (random literals: every block of incompressible runs next to zeros)
        float hbits = 0.f;
        for (int j = 0; j < 4; j++)
            if (c[j]) hbits += (float)c[j] * __log2f((float)nl / (float)c[j]);
        for (int d = 32; d >= 1; d >>= 1) hbits += __shfl_xor(hbits, d);
        if (hbits * 0.125f + 64.f < (float)nl) {
            uint32_t k2 = 0;
            for (int j = 0; j < 4; j++) {
                L[j] = 0;
                if (c[j]) {
                    const uint32_t q = (nl + c[j] - 1) / c[j];
                    const uint32_t l = q <= 1 ? 1u : 32u - (uint32_t)__clz(q - 1);
                    L[j] = l > kHufMaxBits ? kHufMaxBits : l;
                    k2 += 2048u >> L[j];
                }
            }
            uint32_t K = wave_sum(k2);
            while (K > 2048u) {  // lengthen the shortest code below 11 (lowest symbol)
                uint32_t key = 0xFFFFFFFFu;
                for (int j = 0; j < 4; j++)
                    if (L[j] && L[j] < kHufMaxBits) {
                        const uint32_t kk = L[j] << 16 | (lane + 64u * j);
                        key = kk < key ? kk : key;
                    }
                key = wave_min(key);
                if (key == 0xFFFFFFFFu) break;
                const uint32_t sym = key & 0xFFFFu, lw = key >> 16;
                for (int j = 0; j < 4; j++) L[j] += (lane + 64u * j == sym) ? 1u : 0u;
                K -= 1024u >> lw;
            }
            for (int j = 0; j < 4; j++) wts[lane + 64 * j] = L[j];
            wave_lds_sync();
            if (K < 2048u && lane == 0) {  // fill the slack, shortest codes first
                for (uint32_t ln = 1; ln <= kHufMaxBits; ln++)
                    for (uint32_t sy = 0; sy <= maxsym; sy++) {
                        uint32_t l = wts[sy];
                        if (l != ln) continue;
                        while (l > 1 && K + (2048u >> l) <= 2048u) {
                            K += 2048u >> l;
                            l--;
                        }
                        wts[sy] = l;
                    }
            }
            K = rdl(K, 0);
            wave_lds_sync();
            if (K == 2048u) {
                uint32_t lm = 0;
                for (int j = 0; j < 4; j++) {
                    L[j] = wts[lane + 64 * j];
                    lm = L[j] > lm ? L[j] : lm;
                }
                const uint32_t M = wave_max(lm);  // the table log
                uint32_t w[4];
                for (int j = 0; j < 4; j++) w[j] = L[j] ? M + 1 - L[j] : 0u;
                // rank starts per weight (HUF_readDTableX1: weights ascending)
                uint32_t acc = 0;
                for (uint32_t x = 1; x <= M; x++) {
                    uint32_t cx = 0;
                    for (int j = 0; j < 4; j++) cx += w[j] == x;
                    cx = wave_sum(cx);
                    if (lane == 0) st[x] = acc;
                    acc += cx << (x - 1);
                }
                wave_lds_sync();
                for (int j = 0; j < 4; j++) wts[lane + 64 * j] = w[j];
                // codes: start[w] >> (w - 1) + rank among the weight's symbols
                uint32_t cd[4] = {0, 0, 0, 0};
                const uint64_t lt = (1ull << lane) - 1ull;
                for (uint32_t x = 1; x <= M; x++) {
                    uint32_t carry = 0;
                    const uint32_t base_x = st[x] >> (x - 1);
                    for (int j = 0; j < 4; j++) {
                        const uint64_t m = __ballot(w[j] == x);
                        if (w[j] == x)
                            cd[j] = (base_x + carry + (uint32_t)__popcll(m & lt)) | (M + 1 - x) << 16;
                        carry += (uint32_t)__popcll(m);
                    }
                }
                for (int j = 0; j < 4; j++) code[lane + 64 * j] = cd[j];
                wave_lds_sync();
                // stream sizes
                const uint32_t seg = (nl + 3) / 4;
                uint32_t sb[4] = {0, 0, 0, 0};
                for (uint32_t k = lane * 16u; k < nl; k += 1024) {
                    const uint4 v = ld16(lbuf + k);
                    const uint32_t cc = nl - k < 16 ? nl - k : 16u;
                    for (uint32_t j = 0; j < cc; j++) {
                        const uint32_t s4 = (k + j) / seg;
                        const uint32_t nb = code[byte_of(v, j)] >> 16;
                        sb[0] += s4 == 0 ? nb : 0u;
                        sb[1] += s4 == 1 ? nb : 0u;
                        sb[2] += s4 == 2 ? nb : 0u;
                        sb[3] += s4 == 3 ? nb : 0u;
                    }
                }
                // tree description: direct 4-bit weights up to symbol 128, else
                // FSE-compressed weights (written now, after the literals header)
                const uint32_t hl = nl < 1024 ? 3u : nl < 16384 ? 4u : 5u;
                uint32_t tree = 1 + (maxsym + 1) / 2;
                if (maxsym > 128) {
                    const uint32_t fw = fse_weights(wts, maxsym, lds + 1536, out + hl + 1, nl);
                    tree = fw ? 1 + fw : 0u;
                }
                uint32_t sbytes[4], comp = tree + 6;
                for (int j = 0; j < 4; j++) {
                    sbytes[j] = (wave_sum(sb[j]) + 1 + 7) >> 3;
                    comp += sbytes[j];
                }
                const uint32_t rawsz = (nl < 32 ? 1u : nl < 4096 ? 2u : 3u) + nl;
                if (tree && hl + comp < rawsz) {
                    if (lane == 0) {
                        const uint64_t hv = hl == 3 ? (2ull | 1ull << 2 | (uint64_t)nl << 4 |
                                                       (uint64_t)comp << 14)
                                            : hl == 4 ? (2ull | 2ull << 2 | (uint64_t)nl << 4 |
                                                         (uint64_t)comp << 18)
                                                      : (2ull | 3ull << 2 | (uint64_t)nl << 4 |
                                                         (uint64_t)comp << 22);
                        for (uint32_t k = 0; k < hl; k++) out[k] = (uint8_t)(hv >> (8 * k));
                        out[hl] = (uint8_t)(maxsym > 128 ? tree - 1 : 127 + maxsym);
                        uint8_t *jt = out + hl + tree;
                        for (int j = 0; j < 3; j++) {
                            jt[2 * j] = (uint8_t)sbytes[j];
                            jt[2 * j + 1] = (uint8_t)(sbytes[j] >> 8);
                        }
                    }
                    // weights of symbols 0 .. maxsym - 1, two per byte, high nibble first
                    if (maxsym <= 128)
                        for (uint32_t k = lane; 2 * k < maxsym; k += 64) {
                            const uint32_t lo = 2 * k + 1 < maxsym ? wts[2 * k + 1] : 0u;
                            out[hl + 1 + k] = (uint8_t)(wts[2 * k] << 4 | lo);
                        }
                    uint8_t *so = out + hl + tree + 6;
                    for (uint32_t j = 0; j < 4; j++) {
                        const uint32_t a = j * seg, bnd = j == 3 ? nl : (j + 1) * seg;
                        huf_stream(lbuf, a, bnd, code, buf, so);
                        so += sbytes[j];
                    }
                    return hl + comp;
                }
            }
        }
    }
    const uint32_t h = lit_hdr_raw(out, 0, nl);
    wave_copy(out + h, lbuf, nl);
    return h + nl;
}

// All n bytes of the block equal to its first?  (wave-uniform; 16-aligned
// 16-byte loads, bytes outside [src, src + n) in the first and last chunk
// masked off (an aligned chunk that holds a readable byte is readable); 4 KiB
// per wave round, four loads in flight per lane; the first round decides
// most non-RLE blocks)
__device__ bool wave_is_rle(const uint8_t *src, uint32_t n, const uint8_t *lim) {
    const uint32_t lane = lane_id();
    const uint32_t b4 = (uint32_t)src[0] * 0x01010101u;
    const uint32_t sb = (uint32_t)(uintptr_t)src & 15u, end = sb + n;
    const uint8_t *s16 = src - sb;
    const uint32_t nch = (end + 15u) >> 4;
    // bytes of the dword at offset p (from s16) that lie in [sb, end)
    auto dmask = [&](uint32_t p) {
        uint32_t m = 0xFFFFFFFFu;
        if (p < sb) m = sb - p >= 4 ? 0u : m << (8 * (sb - p));
        if (p + 4 > end) m = p >= end ? 0u : m & (0xFFFFFFFFu >> (8 * (p + 4 - end)));
        return m;
    };
    auto diff = [&](uint32_t q) {
        const uint4 v = *(const uint4 *)(s16 + 16u * q);
        uint32_t x0 = v.x ^ b4, x1 = v.y ^ b4, x2 = v.z ^ b4, x3 = v.w ^ b4;
        if (q == 0 || q + 1 == nch) {
            x0 &= dmask(16u * q);
            x1 &= dmask(16u * q + 4);
            x2 &= dmask(16u * q + 8);
            x3 &= dmask(16u * q + 12);
        }
        return x0 | x1 | x2 | x3;
    };
    for (uint32_t o = 0; o < nch; o += 256) {
        uint32_t x = 0;
        if (o + 256 <= nch) {
            uint32_t d[4];
#pragma unroll
            for (int u = 0; u < 4; u++) d[u] = diff(o + u * 64u + lane);
            x = d[0] | d[1] | d[2] | d[3];
        } else {
            for (uint32_t q = o + lane; q < nch; q += 64) x |= diff(q);
        }
        if (__ballot(x != 0)) return false;
    }
    return true;
}

}  // namespace

// far_build: a workgroup per block.  The gate is the block kernel's (order-0
// entropy of four 1 KiB windows): random or single-valued samples build no
// table (comp = 0), so incompressible data pays 4 KiB of reads here.  A
// blob's last block has no later block to serve and builds none either.
__global__ __launch_bounds__(256) void rcdc_zstd_far_build_kernel(
    const uint8_t *__restrict__ in, const ZstdBlob *__restrict__ blobs,
    const ZstdBlk *__restrict__ blks, uint32_t nblk, uint32_t *__restrict__ far) {
    __shared__ uint32_t t[kZstdFarTab];
    __shared__ float wnd[4];
    const uint32_t b = blockIdx.x, tid = threadIdx.x;
    const FarLayout L = far_layout(far, nblk);
    const ZstdBlk k = blks[b];
    const ZstdBlob B = blobs[k.blob];
    const uint8_t *src = in + B.in_off + k.start;
    const uint8_t *lim = in + B.in_off + B.len;
    const uint32_t n = k.len;
    // structured data only: each of four 1 KiB windows at 1.5-7 bits per
    // byte (order-0).  Random, already-compressed and constant windows (and
    // blocks mixing them: C3's random and zero runs) have no far matches
    // worth the reads.
    uint32_t comp = 1;
    if (n >= 8192) {
        uint32_t *hs = t;  // 4 windows x 256 counts
        for (uint32_t i = tid; i < 1024; i += 256) hs[i] = 0;
        __syncthreads();
        const uint32_t w0 = tid >> 6, kk = (tid & 63u) * 16u;
        const uint4 v = ld16(src + (((n / 4) * w0) & ~15u) + kk);
        for (uint32_t q = 0; q < 16; q++) atomicAdd(&hs[w0 * 256u + byte_of(v, q)], 1u);
        __syncthreads();
        float e = 0.f;  // wave w0: window w0's entropy (bits over 1024 bytes)
        for (uint32_t i = tid & 63u; i < 256; i += 64) {
            const uint32_t c = hs[w0 * 256u + i];
            if (c) e += (float)c * __log2f(1024.f / (float)c);
        }
        for (int x = 32; x >= 1; x >>= 1) e += __shfl_xor(e, x);
        if ((tid & 63u) == 0) wnd[w0] = e;
        __syncthreads();
        for (uint32_t w = 0; w < 4; w++) comp &= wnd[w] > 1.5f * 1024.f && wnd[w] < 7.0f * 1024.f;
        __syncthreads();
    }
    if (n < 16u) comp = 0;
    if (tid == 0) L.comp[b] = comp;
    if (!comp || (k.flags & 2u)) return;
    for (uint32_t i = tid; i < kZstdFarTab; i += 256) t[i] = 0;
    __syncthreads();
    // 8 positions per thread and round from 16 bytes; positions <= n - 8
    for (uint32_t q = tid * 8u; q + 8u <= n; q += 2048u) {
        const uint4 v = ld16_lim(src + q, lim);
        const uint64_t u[4] = {(uint64_t)v.x | (uint64_t)v.y << 32, (uint64_t)v.z | (uint64_t)v.w << 32,
                               0ull, 0ull};
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) {
            const uint32_t p = q + j;
            const uint64_t hv = far_hash(bytes8_at(u, j));
            if (p + 8u <= n && far_sampled(hv))
                atomicMax(&t[far_bucket(hv)], (p + 1u) << 15 | far_tag(hv));
        }
    }
    __syncthreads();
    uint32_t *dst = L.tab + (size_t)b * kZstdFarTab;
    for (uint32_t i = tid; i < kZstdFarTab; i += 256) dst[i] = t[i];
}

// One 16-byte group of far_map: every load of a round is independent of the
// others in flight -- the group's bytes, then all sampled positions' b-1
// buckets, then the misses' b-2 buckets, then one verification (the last
// hit).  Returns the offset (0: none); *lng: its first 16 bytes agree.
__device__ __forceinline__ uint32_t far_group(const uint8_t *bsrc, const uint8_t *src,
                                              const uint8_t *lim, uint32_t start, uint32_t n,
                                              uint32_t g, bool ok1, bool ok2, const uint32_t *t1,
                                              const uint32_t *t2, bool *lng) {
    const uint32_t p0 = g * 16u;
    const uint4 a = ld16_lim(src + p0, lim), c = ld16_lim(src + p0 + 16u, lim);
    const uint64_t u[4] = {(uint64_t)a.x | (uint64_t)a.y << 32, (uint64_t)a.z | (uint64_t)a.w << 32,
                           (uint64_t)c.x | (uint64_t)c.y << 32, (uint64_t)c.z | (uint64_t)c.w << 32};
    uint32_t bk[16], tg[16], e[16];
    uint32_t smp = 0;
#pragma unroll
    for (uint32_t j = 0; j < 16u; j++) {
        const uint64_t hv = far_hash(bytes8_at(u, j));
        bk[j] = far_bucket(hv);
        tg[j] = far_tag(hv);
        if (far_sampled(hv) && p0 + j + kZstdFarMin <= n) smp |= 1u << j;
    }
#pragma unroll
    for (uint32_t j = 0; j < 16u; j++) e[j] = (ok1 && ((smp >> j) & 1u)) ? t1[bk[j]] : 0u;
    uint32_t hit1 = 0, miss = 0;
#pragma unroll
    for (uint32_t j = 0; j < 16u; j++) {
        const bool h = e[j] && (e[j] & 0x7FFFu) == tg[j];
        hit1 |= (h ? 1u : 0u) << j;
        miss |= ((!h && ((smp >> j) & 1u)) ? 1u : 0u) << j;
    }
    uint32_t hit2 = 0;
    if (ok2 && miss) {
#pragma unroll
        for (uint32_t j = 0; j < 16u; j++)
            if ((miss >> j) & 1u) {
                const uint32_t x = t2[bk[j]];
                if (x && (x & 0x7FFFu) == tg[j]) {
                    e[j] = x;
                    hit2 |= 1u << j;
                }
            }
    }
    *lng = false;
    if (!(hit1 | hit2)) return 0;
    const uint32_t j = 31u - (uint32_t)__clz(hit1 | hit2);  // the last hit
    uint32_t ej = 0;
#pragma unroll
    for (uint32_t i = 0; i < 16u; i++) ej = i == j ? e[i] : ej;
    const uint32_t d = ((hit2 >> j) & 1u) ? 2u : 1u;
    const uint32_t q = start - d * kZstdBlock + (ej >> 15) - 1u;  // blob-relative
    // q + 8 is inside the blob (block b - d ends above it); the next 8
    // bytes are read bounded by the blob's end
    const uint64_t v = (uint64_t)ld4(bsrc + q) | (uint64_t)ld4(bsrc + q + 4) << 32;
    if (v != bytes8_at(u, j)) return 0;
    if (p0 + j + 16u <= n) {
        const uint64_t w = (uint64_t)ld4_hi(bsrc + q + 8, lim) | (uint64_t)ld4_hi(bsrc + q + 12, lim) << 32;
        *lng = w == bytes8_at(u, j + 8);
    }
    return start + p0 + j - q;
}

// far_map: a workgroup per block, a thread per 16-byte group: each sampled
// position looks up the tables of blocks b-1 then b-2 (same blob), verifies
// the 8 key bytes, and the group keeps the last verified offset.  A probe of
// 1/32 of the groups first counts the groups with an offset; below one in
// `dense` the block skips the full map and the far path (data without far
// repeats pays the probe only).  A finer gate was tried: counting only
// 16-byte repeats excluded word text (whose far repeats do not pay: r5p,
// 33.9 -> 27.1 GiB/s at an unchanged ratio) but CSV rows too, whose gain
// comes from many 8-12 byte repeats (0.133 -> 0.198, r5q).
// LDS: the two tables (2 x 32 KiB) are staged in LDS first, so each group's
// ~8 random bucket reads are LDS reads instead of L2 round trips (as L2
// gathers the kernel was 10 % of CSV's compression time, r5z6).
template <bool LDS>
__global__ __launch_bounds__(512) void rcdc_zstd_far_map_kernel(
    const uint8_t *__restrict__ in, const ZstdBlob *__restrict__ blobs,
    const ZstdBlk *__restrict__ blks, uint32_t nblk, uint32_t *__restrict__ far, uint32_t dense) {
    __shared__ uint32_t nlong;
    __shared__ uint4 s_t[LDS ? kZstdFarTab / 2 : 1];  // t1 then t2
    const uint32_t b = blockIdx.x, tid = threadIdx.x;
    const FarLayout L = far_layout(far, nblk);
    const ZstdBlk k = blks[b];
    const uint32_t kidx = k.start / kZstdBlock;
    const bool ok1 = kidx >= 1u && L.comp[b - 1];
    const bool ok2 = kidx >= 2u && L.comp[b - 2];
    if (!L.comp[b] || !(ok1 || ok2) || k.len < 16u) {
        if (tid == 0) L.has[b] = 0;
        return;
    }
    if (tid == 0) nlong = 0;
    __syncthreads();
    const ZstdBlob B = blobs[k.blob];
    const uint8_t *bsrc = in + B.in_off;
    const uint8_t *src = bsrc + k.start;
    const uint8_t *lim = bsrc + B.len;
    const uint32_t n = k.len;
    const uint32_t ng = (n + 15u) / 16u;
    const uint32_t *t1 = L.tab + (size_t)(b - (ok1 ? 1u : 0u)) * kZstdFarTab;
    const uint32_t *t2 = L.tab + (size_t)(b - (ok2 ? 2u : 0u)) * kZstdFarTab;
    const uint32_t nt = blockDim.x;
    if (LDS) {
        constexpr uint32_t q = kZstdFarTab / 4;  // uint4 per table
        const uint4 *g1 = reinterpret_cast<const uint4 *>(t1), *g2 = reinterpret_cast<const uint4 *>(t2);
        for (uint32_t i = tid; i < q; i += nt) {
            if (ok1) s_t[i] = g1[i];
            if (ok2) s_t[q + i] = g2[i];
        }
        __syncthreads();
        t1 = reinterpret_cast<const uint32_t *>(s_t);
        t2 = t1 + kZstdFarTab;
    }
    // the probe: groups tid * 32 (256 of the block's 8192)
    uint32_t np = 0;
    for (uint32_t g = tid * 32u; g < ng; g += nt * 32u) {
        bool lng;
        np += far_group(bsrc, src, lim, k.start, n, g, ok1, ok2, t1, t2, &lng) != 0u;
    }
    if (np) atomicAdd(&nlong, np);
    const uint32_t nprobe = (ng + 31u) / 32u;
    __syncthreads();
    const bool h = nlong * dense >= nprobe;
    if (tid == 0) {
        L.has[b] = h;
        if (h) atomicAdd(&g_zstd_prof[7], 1ull);  // blocks on the far path (RCDC_ZSTD_DBG bit 2)
    }
    if (!h) return;
    uint32_t *map = L.map + (size_t)b * kZstdFarGroups;
    for (uint32_t g = tid; g < ng; g += nt) {
        bool lng;
        map[g] = far_group(bsrc, src, lim, k.start, n, g, ok1, ok2, t1, t2, &lng);
    }
}

// res[b] = {type | rle byte << 8, content bytes}.  HL: hash table of 2^HL
// positions (LDS 4 * 2^HL bytes per wave, 2 * 2^HL when NARROW: more buckets,
// or more waves per CU)
template <int HL, bool NARROW>
__global__ __launch_bounds__(64, (NARROW ? HL - 1 : HL) == 11 ? 4 : 2) void rcdc_zstd_block_kernel(
    const uint8_t *__restrict__ in, const ZstdBlob *__restrict__ blobs,
    const ZstdBlk *__restrict__ blks, uint32_t nblk, const ZstdTables *__restrict__ tabs,
    uint8_t *__restrict__ slots, uint64_t *__restrict__ seqbuf, uint2 *__restrict__ res,
    uint32_t dbg, uint32_t key, uint32_t *__restrict__ queue, uint32_t *__restrict__ far) {
    __shared__ uint32_t table[NARROW ? 1 << (HL - 1) : 1 << HL];
    uint16_t *const t16 = reinterpret_cast<uint16_t *>(table);
    constexpr uint32_t kTabWords = NARROW ? 1u << (HL - 1) : 1u << HL;
    __shared__ ZstdTables T;
    const uint32_t lane = lane_id();
    for (uint32_t i = lane; i < sizeof(ZstdTables) / 4; i += 64)
        ((uint32_t *)&T)[i] = ((const uint32_t *)tabs)[i];
    uint64_t *seqs = seqbuf + (uint64_t)blockIdx.x * kZstdMaxSeq;
    __syncthreads();
    const FseRegs R = fse_regs(T);
    // Blocks [0, S) go by a static stride; the last one to two grids' worth,
    // [S, nblk), are taken from a queue (blocks cost from ~0 to a full parse:
    // a static stride left the last waves running alone).  The queue is 8
    // counters, one per residue x = blockIdx & 7 (its own 64-byte line): set
    // x's k-th take is block S + x + 8k.  Few takes on 8 addresses keep the
    // device-scope atomics off the cheap kernels' path; lane 0's vector atomic
    // is issued as a block starts, so its round trip overlaps the block.
    // Every wave leaves once its set's count passes nblk.
    const uint32_t G = gridDim.x, rounds = nblk / G;
    const uint32_t S = rounds >= 2 ? (rounds - 1) * G : (G < nblk ? G : nblk);
    const uint32_t qx = blockIdx.x & 7u;
    uint32_t nx = 0;
    for (uint32_t b = blockIdx.x; b < nblk; b = b + G < S ? b + G : S + qx + 8u * rdl(nx, 0)) {
        if (b + G >= S && lane == 0) nx = atomicAdd(queue + 16u * qx, 1u);
        const ZstdBlk k = blks[b];
        const ZstdBlob B = blobs[k.blob];
        // candidates are blob-relative (bsrc + c): far ones lie in earlier blocks
        const uint8_t *bsrc = in + B.in_off;
        const uint32_t ks = k.start;
        const uint8_t *src = bsrc + ks;
        const uint8_t *lim = in + B.in_off + B.len;  // readable bytes end
        const uint32_t n = k.len;
        uint8_t *slot = slots + (uint64_t)b * kZstdSlot;
        const uint32_t *fmap = nullptr;  // this block's far offsets per 16-byte group
        if (far) {
            const FarLayout L = far_layout(far, nblk);
            if (L.has[b]) fmap = L.map + (size_t)b * kZstdFarGroups;
        }
        if (n < 16) {  // too small to gain: raw (ZSTD_compressBlock_internal's floor)
            if (lane == 0) res[b] = make_uint2(kZstdTypeRaw, n);
            continue;
        }
        uint32_t nseq = 0, anchor = 0, matched = 0;
        const bool prof = dbg & 4u;
        uint64_t t0 = prof ? wall_clock64() : 0, t1 = t0, t2 = t0, t3 = t0;
        const bool rle = wave_is_rle(src, n, lim);
        if (prof) t1 = wall_clock64();
        if (rle) {
            if (!(k.flags & 1u)) {
                if (lane == 0) res[b] = make_uint2(kZstdTypeRle | (uint32_t)src[0] << 8, 1);
                continue;
            }
            // first block of the frame: one literal, then an offset-1 match
            if (lane == 0) seqs[0] = seq_pack(1, n - 1, 1 + 3);
            nseq = 1;
            anchor = n;
            matched = n - 1;
        } else {
            // incompressible blocks (random runs, already-compressed files):
            // order-0 entropy of four 1 KiB windows spread over the block;
            // all near 8 bits per byte -> stored raw without a parse (the
            // plug-in estimate of random bytes over 4 KiB is ~7.95)
            uint32_t keyb = key & 0xFFu;  // this block's key bytes
            if (n >= 8192) {
                uint32_t *hs = table;
                for (uint32_t i = lane; i < 256; i += 64) hs[i] = 0;
                wave_lds_sync();
                const uint32_t w0 = lane >> 4, k = (lane & 15u) * 64u;  // 16 lanes per window
                const uint32_t base_w = ((n / 4) * w0) & ~15u;
                for (uint32_t j = 0; j < 64; j += 16) {
                    const uint4 v = ld16(src + base_w + k + j);
                    for (uint32_t q = 0; q < 16; q++) atomicAdd(&hs[byte_of(v, q)], 1u);
                }
                wave_lds_sync();
                float hb = 0.f;
                for (uint32_t i = lane; i < 256; i += 64)
                    if (hs[i]) hb += (float)hs[i] * __log2f(4096.f / (float)hs[i]);
                for (int d = 32; d >= 1; d >>= 1) hb += __shfl_xor(hb, d);
                if (hb > 7.9f * 4096.f) {
                    if (lane == 0) res[b] = make_uint2(kZstdTypeRaw, n);
                    continue;
                }
                // kZstdAdaptKey: 5-byte keys unless the sample is numeric
                // (>= 10 % ASCII digits).  Rows of numbers repeat in 4-5
                // byte pieces that cost more sequence bits than their
                // literals; prose's one- and two-word matches pay from 5
                // (tools/zstd_wave_model.py: text 0.384 -> 0.367, CSV rows
                // and code lines unchanged at their 6-byte ratios)
                if (key & kZstdAdaptKey) {
                    const uint32_t dg = lane < 10 ? hs[48 + lane] : 0u;
                    uint32_t sd = dg;
                    for (int d = 32; d >= 1; d >>= 1) sd += __shfl_xor(sd, d);
                    keyb = sd * 10u < 4096u ? 5u : 6u;
                }
            }
            for (uint32_t i = lane; i < kTabWords; i += 64) table[i] = kZstdNone;
            __builtin_amdgcn_wave_barrier();
            const uint32_t ilimit = n - 8;  // last position a match may start at
            uint32_t base = 0;
            uint32_t rep0 = 0, rep1 = 0, rep2 = 0;  // repeat history set in this block (0: unknown)
            while (base <= ilimit) {
                uint32_t stride = 1u + ((base - anchor) >> kZstdAccelShift);
                if (stride > kZstdMaxStride) stride = kZstdMaxStride;
                const uint32_t p = base + lane * stride;
                const bool act = p <= ilimit;
                uint32_t w = 0, wr = 0, wr1 = 0, wr2 = 0, h = 0, tg = 0, c = kZstdNone, fo = 0;
                bool isrep = false, rc = false, rc1 = false, rc2 = false;
                const uint32_t pb = ks + p;  // blob-relative
                if (act) {
                    // the last offsets' 4 bytes load with the position's own
                    rc = (key & kZstdRepCheck) && rep0 != 0u && pb >= rep0;
                    rc1 = (key & kZstdRep1) && rep1 != 0u && pb >= rep1;
                    rc2 = (key & kZstdRep1) && rep2 != 0u && pb >= rep2;
                    if (fmap) fo = fmap[p >> 4];
                    w = ld4(src + p);
                    wr = ld4(bsrc + (rc ? pb - rep0 : pb));
                    wr1 = ld4(bsrc + (rc1 ? pb - rep1 : pb));
                    wr2 = ld4(bsrc + (rc2 ? pb - rep2 : pb));
                    const uint64_t k6 = key48(w, keyb > 4 ? ld4(src + p + 4) : 0u, keyb);
                    h = zhash<HL>(k6);
                    if constexpr (!NARROW) {
                        tg = ztag(k6);
                        const uint32_t e = table[h];
                        if (e != kZstdNone && (e >> 17) == tg) c = ks + (e & kZstdPosMask);
                    }
                }
                if constexpr (NARROW)
                    if (act) {
                        c = narrow_cand(t16[h], p);
                        if (c != kZstdNone) c += ks;
                    }
                if (rc && wr == w) {
                    c = pb - rep0;
                    isrep = true;
                } else if (rc1 && wr1 == w) {  // the step's matches may have moved them
                    c = pb - rep1;
                    isrep = true;
                } else if (rc2 && wr2 == w) {
                    c = pb - rep2;
                    isrep = true;
                }
                // the far map's offset (from the group's sampled position)
                uint32_t cf = !isrep && fo && pb >= fo && n - p - 4 >= 16 ? pb - fo : kZstdNone;
                // no table or repeat candidate: the far one takes the first
                // round trip, so the second (below) is only for lanes whose
                // table candidate fails (RCDC_ZSTD_DBG bit 6: always second)
                if (c == kZstdNone && cf != kZstdNone && !(dbg & 64u)) {
                    c = cf;
                    cf = kZstdNone;
                } else if ((dbg & 128u) && !isrep && cf != kZstdNone) {  // (A/B: far first)
                    const uint32_t t = c;
                    c = cf;
                    cf = t;
                }
                // a candidate's 4 bytes are checked from memory, in the same
                // round trip as its extension: every candidate lane extends
                // its own match by up to 16 bytes each way (most matches end
                // there); longer ones are finished by the wave once selected
                bool ok = false;
                uint32_t fl = 0, bl = 0;
                if (act && c != kZstdNone) {
                    const uint32_t limf = n - p - 4;
                    uint32_t wc;
                    if (limf >= 16) {
                        wc = ld4(bsrc + c);
                        fl = first_diff16(ld16(src + p + 4), ld16(bsrc + c + 4));
                    } else {  // the block's last bytes: independent 4-byte loads
                        uint4 va, vb;
                        wc = ld4(bsrc + c);
                        va.x = ld4_hi(src + p + 4, lim);
                        va.y = ld4_hi(src + p + 8, lim);
                        va.z = ld4_hi(src + p + 12, lim);
                        va.w = 0;
                        vb.x = ld4_hi(bsrc + c + 4, lim);
                        vb.y = ld4_hi(bsrc + c + 8, lim);
                        vb.z = ld4_hi(bsrc + c + 12, lim);
                        vb.w = 0xFFFFFFFFu;
                        fl = first_diff16(va, vb);
                        if (fl > limf) fl = limf;
                    }
                    // 16 bytes before both (the bytes before the anchor are
                    // readable, merely not matchable: clamp)
                    const uint32_t limb = p - anchor < c ? p - anchor : c;
                    if (c >= 16) {
                        bl = last_eq16(ld16(src + p - 16), ld16(bsrc + c - 16));
                        if (bl > limb) bl = limb;
                    }
                    ok = wc == w && (isrep || 4 + fl >= keyb);  // last offset: 4 bytes
                    if (ok && c < 16)
                        while (bl < limb && src[p - 1 - bl] == bsrc[c - 1 - bl]) bl++;
                }
                if (act && cf != kZstdNone && !ok) {  // the far candidate, when the table's fails
                    const uint32_t wf = ld4(bsrc + cf);
                    const uint32_t ff = first_diff16(ld16(src + p + 4), ld16(bsrc + cf + 4));
                    const uint32_t limb = p - anchor < cf ? p - anchor : cf;
                    uint32_t bf = 0;
                    if (cf >= 16) {
                        bf = last_eq16(ld16(src + p - 16), ld16(bsrc + cf - 16));
                        if (bf > limb) bf = limb;
                    }
                    if (wf == w && 4 + ff >= keyb) {
                        if (cf < 16)
                            while (bf < limb && src[p - 1 - bf] == bsrc[cf - 1 - bf]) bf++;
                        c = cf;
                        fl = ff;
                        bl = bf;
                        ok = true;
                    }
                }
                uint64_t m = __ballot(ok);
                // lazy step, per lane in VALU: the next position's match, if
                // it reaches at least two bytes further, wins (zstd's lazy
                // parsers).  Lanes past an accepted match leave m only below
                // it, so the next lane's bit in the round's mask is its bit
                // in m whenever this lane is picked.
                uint32_t tgt = lane;
                {
                    const uint32_t fn = __shfl_down(fl, 1);
                    const bool rn = __shfl_down((uint32_t)isrep, 1) != 0u;
                    const bool okn = lane < 63 && ((m >> (lane + 1)) & 1ull);
                    // the next position's match wins if it reaches two bytes
                    // further (kZstdLazyRep: or if it is a last offset and
                    // this one is not; off: CSV rows 0.194 vs 0.196 but code
                    // lines 0.125 vs 0.119, tools/zstd_wave_model.py)
                    if (stride == 1 && ok && okn &&
                        ((fl < 16 && fn > fl + 1) || ((key & kZstdLazyRep) && rn && !isrep)))
                        tgt = lane + 1;
                }
                // the round's sequences stay in the picked lanes' registers
                // and are stored together after the loop
                uint32_t vll = 0, vml = 0, vof = 0;
                uint64_t sel = 0;
                bool covered = false;  // p strictly inside a selected match
                while (m) {
                    const int j = (int)rdl(tgt, __builtin_ctzll(m));
                    const uint32_t f = rdl(fl, j);
                    uint32_t pj = base + (uint32_t)j * stride;
                    uint32_t cj = rdl(c, j);
                    const uint32_t bb = rdl(bl, j);
                    uint32_t len = 4 + f;
                    if (f == 16 && n - pj > 20)
                        len += wave_match_fwd(src + pj + 20, bsrc + cj + 20, n - pj - 20, lim);
                    const uint32_t mb = pj - anchor < cj ? pj - anchor : cj;
                    uint32_t bk = bb < mb ? bb : mb;
                    if (bb == 16 && mb > 16)
                        bk += wave_match_back(src + pj - 16, bsrc + cj - 16, mb - 16, bsrc);
                    pj -= bk;
                    cj -= bk;
                    len += bk;
                    // offset value: a repeat code when the offset is in the
                    // block-local history (RFC 8878 3.1.2.5; entries from
                    // earlier blocks are unknown here: 0), else offset + 3
                    const uint32_t off = ks + pj - cj, ll = pj - anchor;
                    uint32_t ofv;
                    if (!(key & kZstdRep)) {  // RCDC_ZSTD_REP=0 (A/B): literal offsets only
                        ofv = off + 3;
                    } else if (ll) {
                        if (off == rep0) {
                            ofv = 1;
                        } else if (off == rep1) {
                            ofv = 2;
                            rep1 = rep0;
                            rep0 = off;
                        } else if (off == rep2) {
                            ofv = 3;
                            rep2 = rep1;
                            rep1 = rep0;
                            rep0 = off;
                        } else {
                            ofv = off + 3;
                            rep2 = rep1;
                            rep1 = rep0;
                            rep0 = off;
                        }
                    } else {
                        if (off == rep1) {
                            ofv = 1;
                            rep1 = rep0;
                            rep0 = off;
                        } else if (off == rep2) {
                            ofv = 2;
                            rep2 = rep1;
                            rep1 = rep0;
                            rep0 = off;
                        } else if (rep0 && off == rep0 - 1) {
                            ofv = 3;
                            rep2 = rep1;
                            rep1 = rep0;
                            rep0 = off;
                        } else {
                            ofv = off + 3;
                            rep2 = rep1;
                            rep1 = rep0;
                            rep0 = off;
                        }
                    }
                    const bool me = lane == (uint32_t)j;
                    vll = me ? ll : vll;
                    vml = me ? len : vml;
                    vof = me ? ofv : vof;
                    sel |= 1ull << j;
                    matched += len;
                    covered = covered || (p > pj && p < pj + len);
                    anchor = pj + len;
                    m &= __ballot(p >= anchor);
                }
                // the step's positions into the table, except those inside
                // the matches just taken (a match's own position stays): as
                // zstd's parsers, which skip them, the table then reaches
                // further back (CSV rows 0.31 -> 0.24, code lines 0.136 -> 0.123)
                if (act && (!covered || ((sel >> lane) & 1ull) || (key & kZstdInsAll))) {
                    if constexpr (NARROW) t16[h] = (uint16_t)p;
                    else table[h] = p | tg << 17;
                }
                wave_lds_sync();
                if ((sel >> lane) & 1ull)
                    seqs[nseq + __popcll(sel & ((1ull << lane) - 1ull))] = seq_pack(vll, vml, vof);
                nseq += __popcll(sel);
                const uint32_t next = base + 64u * stride;
                base = next > anchor ? next : anchor;
            }
        }
        if (prof) {
            t2 = wall_clock64();
            if (lane == 0) {
                atomicAdd(&g_zstd_prof[0], t1 - t0);
                atomicAdd(&g_zstd_prof[1], t2 - t1);
                atomicAdd(&g_zstd_prof[4], 1ull);
                atomicAdd(&g_zstd_prof[5], (unsigned long long)nseq);
            }
        }
        if (dbg & 1u) {  // dbg bit 0: measure the parse alone
            if (lane == 0) res[b] = make_uint2(kZstdTypeRaw, n);
            continue;
        }
        if (nseq == 0) {
            // no match: a literals-only block can still pay (Huffman) when the
            // bytes are skewed; an order-0 entropy sample of the first 4 KiB
            // decides before any copy (random blocks end here)
            uint32_t *hs = table;
            for (uint32_t i = lane; i < 256; i += 64) hs[i] = 0;
            wave_lds_sync();
            const uint32_t ns = (n < 4096 ? n : 4096u) & ~15u;  // >= 16; k + 16 <= n
            for (uint32_t k = lane * 16u; k < ns; k += 1024) {
                const uint4 v = ld16(src + k);
                for (uint32_t j = 0; j < 16; j++) atomicAdd(&hs[byte_of(v, j)], 1u);
            }
            wave_lds_sync();
            float hb = 0.f;
            for (uint32_t i = lane; i < 256; i += 64)
                if (hs[i]) hb += (float)hs[i] * __log2f((float)ns / (float)hs[i]);
            for (int d = 32; d >= 1; d >>= 1) hb += __shfl_xor(hb, d);
            if (hb > 7.5f * (float)ns) {
                if (lane == 0) res[b] = make_uint2(kZstdTypeRaw, n);
                continue;
            }
        }
        const uint32_t lits = n - matched;
        // Number_of_Sequences bytes, + the modes byte when there are sequences
        const uint32_t sh = nseq == 0 ? 1u : (nseq < 128 ? 1u : nseq < 0x7F00 ? 2u : 3u) + 1u;
        // zstd keeps a compressed block only if it saves more than minGain
        const uint32_t min_gain = (n >> 6) + 2u;
        const uint32_t keep_below = n - min_gain;
        __threadfence_block();  // lane 0's sequence records, for every lane
        // the literals, gathered into the wave's scratch after its sequences
        // (8 nseq + lits <= 2 kZstdBlock): a lane per short run, the wave per
        // long run, then the tail
        uint8_t *lbuf = (uint8_t *)(seqs + nseq);
        {
            uint32_t src_pos = 0, dst_pos = 0;
            for (uint32_t c = 0; c < nseq; c += 64) {
                const uint32_t i = c + lane;
                uint32_t ll = 0, adv = 0;
                if (i < nseq) {
                    const uint64_t s = seqs[i];
                    ll = (uint32_t)(s & 0xFFFFF);
                    adv = ll + (uint32_t)((s >> 20) & 0xFFFFF);
                }
                // inclusive prefix sums over the 64 sequences
                uint32_t xs = adv, xl = ll;
                for (int d = 1; d < 64; d <<= 1) {
                    const uint32_t ys = __shfl_up(xs, d), yl = __shfl_up(xl, d);
                    if ((int)lane >= d) {
                        xs += ys;
                        xl += yl;
                    }
                }
                const uint32_t sp = src_pos + xs - adv, dp = dst_pos + xl - ll;
                const bool small = ll < 64;
                if (small)
                    for (uint32_t t = 0; t < ll; t++) lbuf[dp + t] = src[sp + t];
                uint64_t big = __ballot(!small);
                while (big) {
                    const int j = __builtin_ctzll(big);
                    big &= big - 1;
                    wave_copy(lbuf + rdl(dp, j), src + rdl(sp, j), rdl(ll, j));
                }
                src_pos = rdl(src_pos + xs, 63);
                dst_pos = rdl(dst_pos + xl, 63);
            }
            wave_copy(lbuf + dst_pos, src + src_pos, n - src_pos);
        }
        __threadfence_block();
        const uint32_t lsz = encode_literals(lbuf, lits, slot, table);
        if (prof && lane == 0) atomicAdd(&g_zstd_prof[6], wall_clock64() - t2);
        const uint32_t bs0 = nseq ? lsz + sh - 1 : lsz + 1;  // after Number_of_Sequences
        uint32_t bsz = nseq ? kZstdNone : 0u;
        if (nseq && bs0 + 1 < keep_below)
            bsz = wave_fse_sequences(seqs, nseq, T, R, table, slot + bs0, keep_below - bs0);
        if (prof) {
            t3 = wall_clock64();
            if (lane == 0) atomicAdd(&g_zstd_prof[2], t3 - t2);
        }
        if (bsz == kZstdNone || bs0 + bsz >= keep_below || (dbg & 2u)) {
            if (lane == 0) res[b] = make_uint2(kZstdTypeRaw, n);
            continue;
        }
        // Number_of_Sequences (the modes byte follows it, written above)
        if (lane == 0) {
            uint8_t *q = slot + lsz;
            if (nseq < 128) {
                q[0] = (uint8_t)nseq;
            } else if (nseq < 0x7F00) {
                q[0] = (uint8_t)((nseq >> 8) + 0x80);
                q[1] = (uint8_t)nseq;
            } else {
                q[0] = 0xFF;
                q[1] = (uint8_t)(nseq - 0x7F00);
                q[2] = (uint8_t)((nseq - 0x7F00) >> 8);
            }
        }
        if (lane == 0) res[b] = make_uint2(kZstdTypeComp, bs0 + bsz);
        if (prof && lane == 0) atomicAdd(&g_zstd_prof[3], wall_clock64() - t3);
    }
}

// A thread per blob: the frame header (magic, descriptor, content size) and
// each block's output position; out_lens[i] = frame bytes.  Blobs up to
// kZstdSingleMax bytes get single-segment frames (the window is the content
// size); larger ones declare a 1 MiB window, above every offset the parse
// emits (< 3 blocks: far candidates reach two blocks back), since rustic's
// decode_all refuses windows above 2^27 + 1 bytes (libzstd's default limit).
__global__ void rcdc_zstd_frame_kernel(const ZstdBlob *__restrict__ blobs, uint32_t nblobs,
                                       const uint2 *__restrict__ res, uint64_t *__restrict__ bpos,
                                       uint8_t *__restrict__ out, uint64_t *__restrict__ out_lens) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nblobs) return;
    const ZstdBlob B = blobs[i];
    uint8_t h[13] = {0x28, 0xB5, 0x2F, 0xFD};
    uint32_t hl;
    if (B.len < 256) {
        h[4] = 0x20;  // FCS_flag 0 + Single_Segment: 1-byte content size
        h[5] = (uint8_t)B.len;
        hl = 6;
    } else if (B.len < 65536 + 256) {
        h[4] = 0x60;  // 2 bytes: size - 256
        const uint32_t v = B.len - 256;
        h[5] = (uint8_t)v;
        h[6] = (uint8_t)(v >> 8);
        hl = 7;
    } else if (B.len <= kZstdSingleMax) {
        h[4] = 0xA0;  // 4 bytes
        for (int j = 0; j < 4; j++) h[5 + j] = (uint8_t)(B.len >> (8 * j));
        hl = 9;
    } else {
        h[4] = 0x80;  // FCS_flag 2 (4 bytes), not single-segment
        h[5] = (uint8_t)((kZstdWindowLog - 10) << 3);  // Window_Descriptor: 2^20, mantissa 0
        for (int j = 0; j < 4; j++) h[6 + j] = (uint8_t)(B.len >> (8 * j));
        hl = 10;
    }
    uint8_t *o = out + B.out_off;
    for (uint32_t j = 0; j < hl; j++) o[j] = h[j];
    uint64_t pos = B.out_off + hl;
    for (uint32_t b = B.blk0; b < B.blk0 + B.nblk; b++) {
        bpos[b] = pos;
        pos += 3u + res[b].y;
    }
    out_lens[i] = pos - B.out_off;
}

// A workgroup per block: 3-byte block header, then the content.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <bool NT, bool AL>
__global__ __launch_bounds__(kZstdCopyThreads) void rcdc_zstd_copy_kernel(
    const uint8_t *__restrict__ in, const ZstdBlob *__restrict__ blobs,
    const ZstdBlk *__restrict__ blks, const uint2 *__restrict__ res,
    const uint64_t *__restrict__ bpos, const uint8_t *__restrict__ slots,
    uint8_t *__restrict__ out) {
    const uint32_t b = blockIdx.x, t = threadIdx.x;
    const ZstdBlk k = blks[b];
    const uint2 r = res[b];
    const uint32_t type = r.x & 0xFF;
    uint8_t *o = out + bpos[b];
    const uint32_t size = type == kZstdTypeRle ? k.len : r.y;
    const uint32_t hdr = ((k.flags >> 1) & 1u) | type << 1 | size << 3;
    if (t < 3) o[t] = (uint8_t)(hdr >> (8 * t));
    o += 3;
    if (type == kZstdTypeRle) {
        if (t == 0) o[0] = (uint8_t)(r.x >> 8);
        return;
    }
    const uint8_t *src = type == kZstdTypeRaw ? in + blobs[k.blob].in_off + k.start
                                              : slots + (uint64_t)b * kZstdSlot;
    const uint32_t n = r.y;
    uint32_t head = (uint32_t)((16u - ((uint32_t)(uintptr_t)o & 15u)) & 15u);
    if (head > n) head = n;
    if (t < head) o[t] = src[t];
    o += head;
    src += head;
    const uint32_t rest = n - head, n16 = rest >> 4;
    // src's byte offset within a dword is the same for every thread: one
    // dwordx4 from the dword-aligned base plus the next dword (which holds
    // byte 15 when misaligned, so nothing past the content is touched)
    const uint32_t sh = ((uint32_t)(uintptr_t)src & 3u) * 8u;
    const uint32_t *w = (const uint32_t *)((uintptr_t)src & ~(uintptr_t)3);
    auto piece = [&](uint32_t q) {
        uint4 a;
        if (NT) {
            const u32x4 x = __builtin_nontemporal_load((const u32x4 *)(w + 4u * q));
            a = make_uint4(x.x, x.y, x.z, x.w);
        } else {
            a = *(const uint4 *)(w + 4u * q);
        }
        uint4 v = a;
        if (sh) {
            const uint32_t e = w[4u * q + 4u];
            v = make_uint4(__builtin_amdgcn_alignbit(a.y, a.x, sh),
                           __builtin_amdgcn_alignbit(a.z, a.y, sh),
                           __builtin_amdgcn_alignbit(a.w, a.z, sh),
                           __builtin_amdgcn_alignbit(e, a.w, sh));
        }
        return v;
    };
    auto put = [&](uint32_t q, uint4 v) {
        if (NT) {
            u32x4 x = {v.x, v.y, v.z, v.w};
            __builtin_nontemporal_store(x, (u32x4 *)(o + 16u * q));
        } else {
            *(uint4 *)(o + 16u * q) = v;
        }
    };
    constexpr uint32_t U = 4, S = U * kZstdCopyThreads;
    uint32_t q0 = 0;
    if (AL) {
        // 16-aligned loads; the next 16 bytes come from the neighbour lane
        // (lane 63 and the last chunk load them), funnelled by the
        // block-uniform byte shift
        const uint32_t sb = (uint32_t)(uintptr_t)src & 15u, kk = sb >> 2, rr = (sb & 3u) * 8u;
        const uint8_t *s16 = src - sb;
        const uint32_t ln = t & 63u;
        auto lda = [&](uint32_t q) {
            const u32x4 x = __builtin_nontemporal_load((const u32x4 *)(s16 + 16u * q));
            return make_uint4(x.x, x.y, x.z, x.w);
        };
        auto funnel = [&](uint4 A, uint4 B) {
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
            return make_uint4(__builtin_amdgcn_alignbit(x1, x0, rr), __builtin_amdgcn_alignbit(x2, x1, rr),
                              __builtin_amdgcn_alignbit(x3, x2, rr), __builtin_amdgcn_alignbit(x4, x3, rr));
        };
        auto nbr = [&](uint4 A) {
            return make_uint4(__shfl_down(A.x, 1), __shfl_down(A.y, 1), __shfl_down(A.z, 1),
                              __shfl_down(A.w, 1));
        };
        for (; q0 + S <= n16; q0 += S) {
            uint4 A[U], E[U];
#pragma unroll
            for (uint32_t u = 0; u < U; u++) {
                const uint32_t q = q0 + u * kZstdCopyThreads + t;
                A[u] = lda(q);
                E[u] = make_uint4(0, 0, 0, 0);
                if (sb && ln == 63u) E[u] = lda(q + 1);  // q + 1 <= n16: holds content bytes
            }
#pragma unroll
            for (uint32_t u = 0; u < U; u++) {
                const uint32_t q = q0 + u * kZstdCopyThreads + t;
                if (sb) {
                    uint4 B = nbr(A[u]);
                    if (ln == 63u) B = E[u];
                    put(q, funnel(A[u], B));
                } else {
                    put(q, A[u]);
                }
            }
        }
        for (uint32_t q = q0 + t; q < n16; q += kZstdCopyThreads) {
            const uint4 A = lda(q);
            if (sb) {
                uint4 B = nbr(A);  // valid when lane + 1 holds q + 1 (< n16)
                if (ln == 63u || q + 1 >= n16) B = lda(q + 1);
                put(q, funnel(A, B));
            } else {
                put(q, A);
            }
        }
    } else {
    for (; q0 + S <= n16; q0 += S) {
        uint4 v[U];
#pragma unroll
        for (uint32_t u = 0; u < U; u++) v[u] = piece(q0 + u * kZstdCopyThreads + t);
#pragma unroll
        for (uint32_t u = 0; u < U; u++) put(q0 + u * kZstdCopyThreads + t, v[u]);
    }
    for (uint32_t q = q0 + t; q < n16; q += kZstdCopyThreads) put(q, piece(q));
    }
    const uint32_t d = n16 * 16u;
    if (t < rest - d) o[d + t] = src[d + t];
}

namespace rcdc {

void zstd_prof_dump() {
    unsigned long long h[8];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_zstd_prof), sizeof h) != hipSuccess) return;
    fprintf(stderr, "rcdc zstd phases (wave-ms, 100 MHz clock): rle %.1f parse %.1f "
            "literals+sequences %.1f (literals %.1f) tail %.1f; blocks %llu sequences %llu; "
            "far-path blocks %llu\n",
            h[0] / 1e5, h[1] / 1e5, h[2] / 1e5, h[6] / 1e5, h[3] / 1e5, h[4], h[5], h[7]);
    memset(h, 0, sizeof h);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_zstd_prof), h, sizeof h);
}

// The parse strategy of a zstd level (decrypt.rs:494 passes the repository's
// level; 0 is zstd's default, level 3).  Like zstd's own fast levels the
// lowest ones key positions on 6 bytes (fewer, longer matches: faster, a
// little larger on text); the default keys on 4 bytes; from level 4 up the
// hash table doubles to 2^12 positions (better ratio on structured data, half
// the waves per CU).  RCDC_ZSTD_KEY (4 or 6) and RCDC_ZSTD_HLOG (11 or 12)
// override for A/B runs; RCDC_ZSTD_REP=0 turns repeat codes off.
struct ZstdStrategy {
    int hlog;
    bool narrow;   // 16-bit table entries (twice the buckets per LDS byte)
    uint32_t key;  // key bytes | kZstdRep | kZstdRepCheck
};

static ZstdStrategy zstd_strategy(int level) {
    static const int ek = getenv("RCDC_ZSTD_KEY") ? atoi(getenv("RCDC_ZSTD_KEY")) : 0;
    static const int eh = getenv("RCDC_ZSTD_HLOG") ? atoi(getenv("RCDC_ZSTD_HLOG")) : 0;
    static const bool rep = !(getenv("RCDC_ZSTD_REP") && atoi(getenv("RCDC_ZSTD_REP")) == 0);
    static const bool rchk =
        !(getenv("RCDC_ZSTD_REPCHK") && atoi(getenv("RCDC_ZSTD_REPCHK")) == 0);
    static const bool insall = getenv("RCDC_ZSTD_INSALL") && atoi(getenv("RCDC_ZSTD_INSALL")) == 1;
    static const bool rep1 = !(getenv("RCDC_ZSTD_REP1") && atoi(getenv("RCDC_ZSTD_REP1")) == 0);
    static const bool lazyrep = getenv("RCDC_ZSTD_LAZYREP") && atoi(getenv("RCDC_ZSTD_LAZYREP")) == 1;
    static const bool farc = !(getenv("RCDC_ZSTD_FAR") && atoi(getenv("RCDC_ZSTD_FAR")) == 0);
    if (level == 0) level = 3;  // ZSTD_CLEVEL_DEFAULT
    ZstdStrategy z{11, false, level <= 1 ? 6u : 4u};
    if (level >= 3) z = ZstdStrategy{level >= 4 ? 13 : 12, true, 6u};
    if (z.narrow) z.key |= kZstdAdaptKey;  // per-block 5 or 6 (RCDC_ZSTD_KEY fixes it)
    if (ek == 4 || ek == 5 || ek == 6) z.key = (uint32_t)ek;
    if (eh == 11) z.hlog = 11, z.narrow = false;
    if (eh == 12 || eh == 13) z.hlog = eh, z.narrow = true;
    if (rep) z.key |= kZstdRep;
    if (rep && rchk) z.key |= kZstdRepCheck;
    if (insall) z.key |= kZstdInsAll;
    if (rep && rchk && rep1) z.key |= kZstdRep1;
    if (lazyrep) z.key |= kZstdLazyRep;
    if (farc && z.narrow) z.key |= kZstdFar;  // levels >= 3 (RCDC_ZSTD_FAR=0: off)
    return z;
}

// LDS per wave: 8 KiB table (16 waves per CU) or 16 KiB (8)
// 32-bit words of the far scratch for nblk blocks (0: far candidates off at
// this level)
uint64_t zstd_far_words(int level, uint64_t nblk) {
    const ZstdStrategy z = zstd_strategy(level);
    return (z.key & kZstdFar) ? nblk * (kZstdFarTab + kZstdFarGroups + 2ull) : 0ull;
}

uint32_t zstd_block_grid(uint32_t cus, int level) {
    const ZstdStrategy z = zstd_strategy(level);
    return cus * ((z.narrow ? z.hlog - 1 : z.hlog) == 11 ? 16u : 8u);
}

hipError_t launch_zstd(const uint8_t *in, uint8_t *out, const ZstdBlob *blobs, uint32_t nblobs,
                       const ZstdBlk *blks, uint32_t nblk, const ZstdTables *tabs, uint8_t *slots,
                       uint64_t *seqbuf, uint32_t grid, uint2 *res, uint64_t *bpos,
                       uint64_t *out_lens, uint32_t *queue, uint32_t *far, int level,
                       hipStream_t stream) {
    if (nblobs == 0) return hipSuccess;
    const ZstdStrategy z = zstd_strategy(level);
    if (!(z.key & kZstdFar)) far = nullptr;
    if (far && nblk) {
        hipLaunchKernelGGL(rcdc_zstd_far_build_kernel, dim3(nblk), dim3(256), 0, stream, in, blobs,
                           blks, nblk, far);
        static const uint32_t dense = getenv("RCDC_ZSTD_FARDENSE")
                                          ? (uint32_t)std::max(atoi(getenv("RCDC_ZSTD_FARDENSE")), 1)
                                          : kZstdFarDense;
        static const bool lds = !(getenv("RCDC_ZSTD_FARLDS") && atoi(getenv("RCDC_ZSTD_FARLDS")) == 0);
        hipLaunchKernelGGL(lds ? rcdc_zstd_far_map_kernel<true> : rcdc_zstd_far_map_kernel<false>,
                           dim3(nblk), dim3(lds ? 512 : 256), 0, stream, in, blobs, blks, nblk, far,
                           dense);
    }
    static const uint32_t dbg = getenv("RCDC_ZSTD_DBG") ? (uint32_t)atoi(getenv("RCDC_ZSTD_DBG")) : 0u;
    // RCDC_ZSTD_DBG bit 4 (16): wait after each kernel and name the one that failed
    auto step = [&](const char *what) -> hipError_t {
        if (!(dbg & 16u)) return hipSuccess;
        const hipError_t e = hipStreamSynchronize(stream);
        if (e != hipSuccess) fprintf(stderr, "rcdc zstd: %s failed: %s\n", what, hipGetErrorString(e));
        return e;
    };
    if (far && nblk)
        if (const hipError_t e = step("far build + far map")) return e;
    const uint32_t g = nblk < grid ? nblk : grid;
    if (g) {
        auto *k = !z.narrow      ? rcdc_zstd_block_kernel<11, false>
                  : z.hlog == 12 ? rcdc_zstd_block_kernel<12, true>
                                 : rcdc_zstd_block_kernel<13, true>;
        hipLaunchKernelGGL(k, dim3(g), dim3(64), 0, stream, in, blobs, blks, nblk, tabs, slots,
                           seqbuf, res, dbg, z.key, queue, far);
        if (const hipError_t e = step("block kernel")) return e;
    }
    hipLaunchKernelGGL(rcdc_zstd_frame_kernel, dim3((nblobs + 255) / 256), dim3(256), 0, stream,
                       blobs, nblobs, res, bpos, out, out_lens);
    if (const hipError_t e = step("frame kernel")) return e;
    // A/B knobs: RCDC_ZSTD_COPY=1 loads dword-aligned dwordx4 + one dword per
    // 16 B instead of 16-aligned loads with a lane shuffle (default, random
    // blocks +13 %); RCDC_ZSTD_NT=0 (with COPY=1) plain loads and stores
    static const bool nt = !(getenv("RCDC_ZSTD_NT") && atoi(getenv("RCDC_ZSTD_NT")) == 0);
    static const bool al = !(getenv("RCDC_ZSTD_COPY") && atoi(getenv("RCDC_ZSTD_COPY")) == 1);
    auto *copy = al   ? rcdc_zstd_copy_kernel<true, true>
                 : nt ? rcdc_zstd_copy_kernel<true, false>
                      : rcdc_zstd_copy_kernel<false, false>;
    if (nblk)
        hipLaunchKernelGGL(copy, dim3(nblk), dim3(kZstdCopyThreads), 0, stream, in, blobs, blks,
                           res, bpos, slots, out);
    if (const hipError_t e = step("copy kernel")) return e;
    return hipGetLastError();
}

}  // namespace rcdc
