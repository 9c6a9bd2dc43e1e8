/*
 * cdc_ref.h -- CPU ORACLE for the rcdc content-defined chunker.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * (or as the timed CPU baseline).  The product path (librcdc.so) never links
 * or calls it.
 *
 * What it restates (reference = /root/reference, rustic_core 0.12.0):
 *   - crates/core/src/chunker/rabin.rs:107-191  ChunkIter::next (cut semantics)
 *   - crates/core/src/chunker/rabin.rs:82-104   ChunkIter::new (split_mask)
 *   - crates/core/src/chunker/rabin.rs:17-42    check_rabin_params
 *   - crates/core/src/chunker/fixed_size.rs:41-70 FixedSize ChunkIter::next
 *   - crates/core/src/chunker.rs:30  Rabin64::new_with_polynom(6, &poly)
 *   - rustic_cdc 0.3.1 Rabin64 (crates.io dependency, Cargo.toml:66,
 *     /root/reference/Cargo.lock:4287-4290; NOT vendored, restated from its
 *     published algorithm -- see SURVEY.md Appendix A)
 *   - rand 0.10 StdRng::seed_from_u64 (PCG32 seed expansion + ChaCha12
 *     keystream, chacha20 0.10.0; Cargo.lock:557-566,3769-3777) to regenerate
 *     the reference tests' input bytes (rabin.rs:343-347).
 *
 * Parity pin: tests/test_oracle_golden.py checks this oracle against every
 * (len, sha256) of the reference snapshots
 *   src/chunker/snapshots/rustic_core__chunker__rabin__tests__chunk_random.snap
 *   src/chunker/snapshots/rustic_core__chunker__fixed_size__tests__chunk-size*.snap
 * plus the chunk_empty / chunk_zeros known answers (rabin.rs:360-385).
 * The min-zone prefill variant (V1 = 63-byte prefill, canonical; A = 64) is
 * NOT distinguished by any reference fixture: "parity unpinned in the
 * min-zone" (DESIGN.md).
 */
#ifndef RCDC_ORACLE_CDC_REF_H
#define RCDC_ORACLE_CDC_REF_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    uint64_t out_table[256]; /* b * x^(8*63) mod P                        */
    uint64_t mod_table[256]; /* ((i << deg) mod P) | (i << deg)           */
    int      degree;         /* deg(P)                                     */
    int      shift;          /* deg(P) - 8                                 */
} cdc_ref_tables;

/* deg(p) = 63 - clz(p); -1 for p == 0 (Polynom64::degree). */
int  cdc_ref_degree(uint64_t p);
/* GF(2) remainder p mod m (Polynom64::modulo). */
uint64_t cdc_ref_modulo(uint64_t p, uint64_t m);
/* Rabin64::new_with_polynom(6, &poly) table construction. */
int  cdc_ref_tables_init(cdc_ref_tables *t, uint64_t poly);

/* check_rabin_params (rabin.rs:17-42): 0 ok, 1 = ErrorKind::Unsupported. */
int  cdc_ref_check_params(uint64_t avg, uint64_t min, uint64_t max);

/* Whole-buffer chunking with the exact semantics of rabin.rs ChunkIter::next.
 * Writes the END offset of every chunk (a prefix sum of chunk lengths) to
 * cuts[] (up to cap entries) and returns the number of chunks (may exceed
 * cap; then only the first cap are written).  prefill64 = 0 -> V1
 * (canonical), 1 -> variant A.  Literal byte-at-a-time restatement: ring
 * window, out/mod tables, reset_and_prefill_window.                       */
size_t cdc_ref_chunk(const cdc_ref_tables *t, const uint8_t *data, size_t n,
                     uint64_t min, uint64_t avg, uint64_t max, int prefill64,
                     uint64_t *cuts, size_t cap);

/* "Reference-equivalent" mode, the CPU baseline of bench.py: the same cuts,
 * but doing the same WORK as rabin.rs:110-191 -- every chunk is materialised
 * as an owned buffer (memcpy of the unhashed min prefix, then one push per
 * hashed byte) fed from a 4 KiB read buffer (BUF_SIZE, rabin.rs:12).       */
size_t cdc_ref_chunk_owned(const cdc_ref_tables *t, const uint8_t *data,
                           size_t n, uint64_t min, uint64_t avg, uint64_t max,
                           uint64_t *cuts, size_t cap);
/* Returned (instead of a count) where rabin.rs:124 `min_size -= open_buf_len`
 * would underflow: min < the up-to-4095 read-ahead bytes (BUF_SIZE,
 * rabin.rs:12).  Reachable only for min < 4096, which librcdc rejects. */
#define CDC_REF_UNDERFLOW ((size_t)-1)
/* Same, with a reader whose every read() returns a pseudo-random 1..want
 * bytes (xorshift64 seeded by read_seed != 0; 0 = full Cursor reads). */
size_t cdc_ref_chunk_owned_reads(const cdc_ref_tables *t, const uint8_t *data,
                                 size_t n, uint64_t min, uint64_t avg,
                                 uint64_t max, uint64_t read_seed,
                                 uint64_t *cuts, size_t cap);

/* Same as cdc_ref_chunk_owned over many independent files with nthreads
 * POSIX threads (per-file parallelism as in archiver.rs:195).  Each file i
 * is data[offs[i] .. offs[i]+lens[i]); cut counts land in counts[i]; cuts
 * are not returned (timing entry point).  Returns total chunks.           */
uint64_t cdc_ref_chunk_many_owned(const cdc_ref_tables *t, const uint8_t *data,
                                  const uint64_t *offs, const uint64_t *lens,
                                  size_t nfiles, uint64_t min, uint64_t avg,
                                  uint64_t max, int nthreads, uint64_t *counts);

/* Same work, and the cut lists too: file i's cut offsets (relative to the
 * file) land in cuts[cut_base[i] .. cut_base[i] + min(counts[i], cut_cap[i])).
 * The parity checker of whole device batches (bench.py, tests).            */
uint64_t cdc_ref_chunk_many_cuts(const cdc_ref_tables *t, const uint8_t *data,
                                 const uint64_t *offs, const uint64_t *lens,
                                 size_t nfiles, uint64_t min, uint64_t avg,
                                 uint64_t max, int nthreads, uint64_t *counts,
                                 uint64_t *cuts, const uint64_t *cut_base,
                                 const uint64_t *cut_cap);

/* FixedSize chunker (fixed_size.rs:41-70): cuts every `size` bytes. */
size_t cdc_ref_fixed(size_t n, uint64_t size, uint64_t *cuts, size_t cap);

/* Per-position candidate test used by the parity tests of the device scan:
 * flags[i] = 1 iff fp(data[p-64 .. p)) & mask == 0 for p = first + i,
 * i < count (p >= 64 required).                                          */
void cdc_ref_candidates(const cdc_ref_tables *t, const uint8_t *data,
                        size_t n, uint64_t mask, size_t first, size_t count,
                        uint8_t *flags);

/* rand 0.10 StdRng::seed_from_u64(seed).fill_bytes(buf[0..n)). */
void cdc_ref_stdrng_fill(uint64_t seed, uint8_t *buf, size_t n);
/* Same keystream, starting at byte offset `skip` (multiple of 64). */
void cdc_ref_stdrng_fill_at(uint64_t seed, uint64_t skip, uint8_t *buf,
                            size_t n);

#ifdef __cplusplus
}
#endif
#endif
