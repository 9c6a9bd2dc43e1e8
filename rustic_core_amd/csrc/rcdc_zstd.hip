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

#include "rcdc_internal.h"

using namespace rcdc;

namespace rcdc {
constexpr int kZstdHashLog = 11;           // 2048 buckets x 8 B = 16 KiB of LDS per wave
constexpr uint32_t kZstdNone = 0xFFFFFFFFu;
constexpr int kZstdAccelShift = 8;         // stride = 1 + (bytes since the anchor >> 8)
constexpr uint32_t kZstdMaxStride = 32;
constexpr int kZstdCopyThreads = 256;
}  // namespace rcdc

namespace {

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

__device__ __forceinline__ uint32_t rdl(uint32_t v, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}

__device__ __forceinline__ uint32_t highbit(uint32_t v) { return 31u - (uint32_t)__clz(v); }

// 4 bytes at any alignment from the aligned dwords that hold them (a dword
// that holds a readable byte is readable: allocations are 4-byte granular).
__device__ __forceinline__ uint32_t ld4(const uint8_t *p) {
    const uintptr_t a = (uintptr_t)p & ~(uintptr_t)3;
    const uint32_t sh = ((uint32_t)(uintptr_t)p & 3u) * 8u;
    const uint32_t lo = *(const uint32_t *)a;
    const uint32_t hi = sh ? *(const uint32_t *)(a + 4) : 0u;
    return __builtin_amdgcn_alignbit(hi, lo, sh);
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

__device__ __forceinline__ uint32_t zhash(uint32_t w) {
    return (w * 2654435761u) >> (32 - kZstdHashLog);
}

// Equal bytes of a[0..) and b[0..), at most maxlen (wave-uniform result).
__device__ uint32_t wave_match_fwd(const uint8_t *a, const uint8_t *b, uint32_t maxlen,
                                   const uint8_t *lim) {
    const uint32_t lane = lane_id();
    uint32_t len = 0;
    while (len < maxlen) {
        const uint32_t o = len + lane * 4u;
        uint32_t x = 0xFFFFFFFFu;
        if (o < maxlen) {
            x = ld4_hi(a + o, lim) ^ ld4_hi(b + o, lim);
            const uint32_t rem = maxlen - o;
            if (rem < 4) x |= 0xFFFFFFFFu << (8 * rem);
        }
        const uint64_t m = __ballot(x != 0);
        if (m) {
            const int j = __builtin_ctzll(m);
            const uint32_t xj = rdl(x, j);
            len += (uint32_t)j * 4u + ((uint32_t)__builtin_ctz(xj) >> 3);
            return len < maxlen ? len : maxlen;
        }
        len += 256;
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

struct BitW {
    uint64_t acc;
    uint32_t nb;
    uint8_t *o, *end;
    bool over;
    __device__ void add(uint32_t v, uint32_t bits) {
        acc |= (uint64_t)(v & ((1u << bits) - 1u)) << nb;
        nb += bits;
    }
    __device__ void flush() {
        while (nb >= 8) {
            if (o < end) *o++ = (uint8_t)acc;
            else over = true;
            acc >>= 8;
            nb -= 8;
        }
    }
};

struct FseState {
    uint32_t v;
};

__device__ __forceinline__ void fse_init(FseState &s, const ZstdFseSym *tt, const uint16_t *st,
                                         uint32_t sym) {
    const ZstdFseSym t = tt[sym];
    const uint32_t nbo = (t.nbits + (1u << 15)) >> 16;
    const uint32_t v = (nbo << 16) - t.nbits;
    s.v = st[(int)(v >> nbo) + t.find];
}

__device__ __forceinline__ void fse_enc(BitW &w, FseState &s, const ZstdFseSym *tt,
                                        const uint16_t *st, uint32_t sym) {
    const ZstdFseSym t = tt[sym];
    const uint32_t nbo = (s.v + t.nbits) >> 16;
    w.add(s.v, nbo);
    s.v = st[(int)(s.v >> nbo) + t.find];
}

// sequence record: literal length | match length << 20 | offset << 40
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
    c.ofv = (uint32_t)(s >> 40) + 3u;  // offset_value: never a repeat code
    c.mlb = ml - 3u;
    c.llc = c.ll < 64 ? T.llcode[c.ll] : highbit(c.ll) + 19u;
    c.mlc = c.mlb < 128 ? T.mlcode[c.mlb] : highbit(c.mlb) + 36u;
    c.ofc = highbit(c.ofv);
    return c;
}

// Lane 0: the sequences section's bitstream (ZSTD_encodeSequences order).
// Returns its bytes, or kZstdNone if it would pass `end`.
__device__ uint32_t fse_sequences(const uint64_t *seqs, uint32_t nseq, const ZstdTables &T,
                                  uint8_t *out, uint8_t *end) {
    BitW w{0, 0, out, end, false};
    FseState sll, sml, sof;
    SeqCodes c = seq_codes(seqs[nseq - 1], T);
    fse_init(sml, T.ml, T.mlst, c.mlc);
    fse_init(sof, T.of, T.ofst, c.ofc);
    fse_init(sll, T.ll, T.llst, c.llc);
    w.add(c.ll, T.llbits[c.llc]);
    w.add(c.mlb, T.mlbits[c.mlc]);
    w.flush();
    w.add(c.ofv, c.ofc);
    w.flush();
    for (int64_t i = (int64_t)nseq - 2; i >= 0; i--) {
        c = seq_codes(seqs[i], T);
        fse_enc(w, sof, T.of, T.ofst, c.ofc);
        fse_enc(w, sml, T.ml, T.mlst, c.mlc);
        w.flush();
        fse_enc(w, sll, T.ll, T.llst, c.llc);
        w.add(c.ll, T.llbits[c.llc]);
        w.flush();
        w.add(c.mlb, T.mlbits[c.mlc]);
        w.flush();
        w.add(c.ofv, c.ofc);
        w.flush();
        if (w.over) return kZstdNone;
    }
    w.add(sml.v, 6);
    w.flush();
    w.add(sof.v, 5);
    w.flush();
    w.add(sll.v, 6);
    w.add(1, 1);  // end mark (BIT_closeCStream)
    w.flush();
    if (w.nb) {
        if (w.o < w.end) *w.o++ = (uint8_t)w.acc;
        else w.over = true;
    }
    return w.over ? kZstdNone : (uint32_t)(w.o - out);
}

// All n bytes of the block equal to its first?  (wave-uniform)
__device__ bool wave_is_rle(const uint8_t *src, uint32_t n, const uint8_t *lim) {
    const uint32_t lane = lane_id();
    const uint32_t b4 = (uint32_t)src[0] * 0x01010101u;
    for (uint32_t o = 0; o < n; o += 256) {
        const uint32_t q = o + lane * 4u;
        uint32_t x = 0;
        if (q < n) {
            x = ld4_hi(src + q, lim) ^ b4;
            const uint32_t rem = n - q;
            if (rem < 4) x &= ~(0xFFFFFFFFu << (8 * rem));
        }
        if (__ballot(x != 0)) return false;
    }
    return true;
}

}  // namespace

// res[b] = {type | rle byte << 8, content bytes}
__global__ __launch_bounds__(64) void rcdc_zstd_block_kernel(
    const uint8_t *__restrict__ in, const ZstdBlob *__restrict__ blobs,
    const ZstdBlk *__restrict__ blks, uint32_t nblk, const ZstdTables *__restrict__ tabs,
    uint8_t *__restrict__ slots, uint64_t *__restrict__ seqbuf, uint2 *__restrict__ res) {
    __shared__ uint2 table[1 << kZstdHashLog];
    __shared__ ZstdTables T;
    const uint32_t lane = lane_id();
    for (uint32_t i = lane; i < sizeof(ZstdTables) / 4; i += 64)
        ((uint32_t *)&T)[i] = ((const uint32_t *)tabs)[i];
    uint64_t *seqs = seqbuf + (uint64_t)blockIdx.x * kZstdMaxSeq;
    for (uint32_t b = blockIdx.x; b < nblk; b += gridDim.x) {
        const ZstdBlk k = blks[b];
        const ZstdBlob B = blobs[k.blob];
        const uint8_t *src = in + B.in_off + k.start;
        const uint8_t *lim = in + B.in_off + B.len;  // readable bytes end
        const uint32_t n = k.len;
        uint8_t *slot = slots + (uint64_t)b * kZstdSlot;
        if (n < 16) {  // too small to gain: raw (ZSTD_compressBlock_internal's floor)
            if (lane == 0) res[b] = make_uint2(kZstdTypeRaw, n);
            continue;
        }
        uint32_t nseq = 0, anchor = 0, matched = 0;
        if (wave_is_rle(src, n, lim)) {
            if (!(k.flags & 1u)) {
                if (lane == 0) res[b] = make_uint2(kZstdTypeRle | (uint32_t)src[0] << 8, 1);
                continue;
            }
            // first block of the frame: one literal, then an offset-1 match
            if (lane == 0) seqs[0] = seq_pack(1, n - 1, 1);
            nseq = 1;
            anchor = n;
            matched = n - 1;
        } else {
            for (uint32_t i = lane; i < (1u << kZstdHashLog); i += 64)
                table[i] = make_uint2(kZstdNone, 0);
            __builtin_amdgcn_wave_barrier();
            const uint32_t ilimit = n - 8;  // last position a match may start at
            uint32_t base = 0;
            while (base <= ilimit) {
                uint32_t stride = 1u + ((base - anchor) >> kZstdAccelShift);
                if (stride > kZstdMaxStride) stride = kZstdMaxStride;
                const uint32_t p = base + lane * stride;
                const bool act = p <= ilimit;
                uint32_t w = 0, h = 0;
                uint2 e = make_uint2(kZstdNone, 0);
                if (act) {
                    w = ld4(src + p);
                    h = zhash(w);
                    e = table[h];
                }
                __builtin_amdgcn_wave_barrier();
                if (act) table[h] = make_uint2(p, w);
                __builtin_amdgcn_wave_barrier();
                const bool ok = act && e.x != kZstdNone && e.y == w;
                uint64_t m = __ballot(ok);
                while (m) {
                    const int j = __builtin_ctzll(m);
                    uint32_t pj = base + (uint32_t)j * stride;
                    uint32_t cj = rdl(e.x, j);
                    uint32_t len = 4 + wave_match_fwd(src + pj + 4, src + cj + 4, n - pj - 4, lim);
                    const uint32_t mb = pj - anchor < cj ? pj - anchor : cj;
                    const uint32_t bk = wave_match_back(src + pj, src + cj, mb, src);
                    pj -= bk;
                    cj -= bk;
                    len += bk;
                    if (lane == 0) seqs[nseq] = seq_pack(pj - anchor, len, pj - cj);
                    nseq++;
                    matched += len;
                    anchor = pj + len;
                    m &= __ballot(p >= anchor);
                }
                const uint32_t next = base + 64u * stride;
                base = next > anchor ? next : anchor;
            }
        }
        if (nseq == 0) {
            if (lane == 0) res[b] = make_uint2(kZstdTypeRaw, n);
            continue;
        }
        const uint32_t lits = n - matched;
        const uint32_t lh = lits < 32 ? 1u : lits < 4096 ? 2u : 3u;
        const uint32_t sh = (nseq < 128 ? 1u : nseq < 0x7F00 ? 2u : 3u) + 1u;
        const uint32_t bs0 = lh + lits + sh;
        // zstd keeps a compressed block only if it saves more than minGain
        const uint32_t min_gain = (n >> 6) + 2u;
        const uint32_t keep_below = n - min_gain;
        uint32_t bsz = kZstdNone;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        if (bs0 < keep_below && lane == 0)
            bsz = fse_sequences(seqs, nseq, T, slot + bs0, slot + keep_below);
        bsz = rdl(bsz, 0);
        if (bsz == kZstdNone || bs0 + bsz >= keep_below) {
            if (lane == 0) res[b] = make_uint2(kZstdTypeRaw, n);
            continue;
        }
        // literals section header (Raw_Literals_Block, RFC 8878 3.1.1.3.1.1)
        if (lane == 0) {
            if (lh == 1) {
                slot[0] = (uint8_t)(lits << 3);
            } else if (lh == 2) {
                const uint32_t v = 1u << 2 | lits << 4;
                slot[0] = (uint8_t)v;
                slot[1] = (uint8_t)(v >> 8);
            } else {
                const uint32_t v = 3u << 2 | lits << 4;
                slot[0] = (uint8_t)v;
                slot[1] = (uint8_t)(v >> 8);
                slot[2] = (uint8_t)(v >> 16);
            }
            // sequences section header: Number_of_Sequences, modes (all predefined)
            uint8_t *q = slot + lh + lits;
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
            q[sh - 1] = 0;
        }
        // literals: lane per short run, the wave per long run, then the tail
        uint8_t *lout = slot + lh;
        uint32_t src_pos = 0, dst_pos = 0;
        for (uint32_t c = 0; c < nseq; c += 64) {
            const uint32_t i = c + lane;
            uint32_t ll = 0, adv = 0;
            if (i < nseq) {
                const uint64_t s = seqs[i];
                ll = (uint32_t)(s & 0xFFFFF);
                adv = ll + (uint32_t)((s >> 20) & 0xFFFFF);
            }
            // exclusive prefix sums over the 64 sequences
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
                for (uint32_t t = 0; t < ll; t++) lout[dp + t] = src[sp + t];
            uint64_t big = __ballot(!small);
            while (big) {
                const int j = __builtin_ctzll(big);
                big &= big - 1;
                wave_copy(lout + rdl(dp, j), src + rdl(sp, j), rdl(ll, j));
            }
            src_pos = rdl(src_pos + xs, 63);
            dst_pos = rdl(dst_pos + xl, 63);
        }
        wave_copy(lout + dst_pos, src + src_pos, n - src_pos);
        if (lane == 0) res[b] = make_uint2(kZstdTypeComp, bs0 + bsz);
    }
}

// A thread per blob: the frame header (magic, single-segment descriptor,
// content size) and each block's output position; out_lens[i] = frame bytes.
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
    } else {
        h[4] = 0xA0;  // 4 bytes
        for (int j = 0; j < 4; j++) h[5 + j] = (uint8_t)(B.len >> (8 * j));
        hl = 9;
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
    for (uint32_t q = t; q < n16; q += kZstdCopyThreads) {
        const uint8_t *s = src + 16u * q;
        uint4 v;
        v.x = ld4(s);
        v.y = ld4(s + 4);
        v.z = ld4(s + 8);
        v.w = ld4(s + 12);
        *(uint4 *)(o + 16u * q) = v;
    }
    const uint32_t d = n16 * 16u;
    if (t < rest - d) o[d + t] = src[d + t];
}

namespace rcdc {

uint32_t zstd_block_grid(uint32_t cus) { return cus * 8u; }

hipError_t launch_zstd(const uint8_t *in, uint8_t *out, const ZstdBlob *blobs, uint32_t nblobs,
                       const ZstdBlk *blks, uint32_t nblk, const ZstdTables *tabs, uint8_t *slots,
                       uint64_t *seqbuf, uint32_t grid, uint2 *res, uint64_t *bpos,
                       uint64_t *out_lens, hipStream_t stream) {
    if (nblobs == 0) return hipSuccess;
    const uint32_t g = nblk < grid ? nblk : grid;
    if (g)
        hipLaunchKernelGGL(rcdc_zstd_block_kernel, dim3(g), dim3(64), 0, stream, in, blobs, blks,
                           nblk, tabs, slots, seqbuf, res);
    hipLaunchKernelGGL(rcdc_zstd_frame_kernel, dim3((nblobs + 255) / 256), dim3(256), 0, stream,
                       blobs, nblobs, res, bpos, out, out_lens);
    if (nblk)
        hipLaunchKernelGGL(rcdc_zstd_copy_kernel, dim3(nblk), dim3(kZstdCopyThreads), 0, stream,
                           in, blobs, blks, res, bpos, slots, out);
    return hipGetLastError();
}

}  // namespace rcdc
