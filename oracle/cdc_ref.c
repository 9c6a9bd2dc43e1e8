/*
 * cdc_ref.c -- CPU ORACLE (test infrastructure only; see cdc_ref.h header).
 *
 * Plain C restatement of the reference's chunking path.  Every function names
 * the reference location it follows.  Nothing here is shipped or called by
 * the product library (rustic_core_amd/csrc -> librcdc.so).
 */
#include "cdc_ref.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* Polynom64 (rustic_cdc 0.3.1, used by rabin.rs:250-315 and table build)    */
/* ------------------------------------------------------------------------ */

int cdc_ref_degree(uint64_t p) { return p ? 63 - __builtin_clzll(p) : -1; }

uint64_t cdc_ref_modulo(uint64_t p, uint64_t m) {
    /* long division over GF(2): while deg(p) >= deg(m) cancel the top term */
    int dm = cdc_ref_degree(m);
    if (dm < 0) return p;
    while (p != 0) {
        int dp = cdc_ref_degree(p);
        if (dp < dm) break;
        p ^= m << (dp - dm);
    }
    return p;
}

/* Rabin64::new_with_polynom(6, &poly) -- chunker.rs:30, SURVEY.md A.1.
 * window = 2^6 = 64 bytes; polynom_shift = deg - 8.                        */
int cdc_ref_tables_init(cdc_ref_tables *t, uint64_t poly) {
    int deg = cdc_ref_degree(poly);
    if (deg < 9 || deg > 56) return 1; /* h << 8 must not overflow u64 */
    t->degree = deg;
    t->shift = deg - 8;
    for (int b = 0; b < 256; b++) {
        /* out_table[b] = b * x^(8*(window-1)) mod P */
        uint64_t h = cdc_ref_modulo((uint64_t)b, poly);
        for (int i = 0; i < 63; i++) h = cdc_ref_modulo(h << 8, poly);
        t->out_table[b] = h;
        /* mod_table[b] = ((b << deg) mod P) | (b << deg) */
        uint64_t p = (uint64_t)b << deg;
        t->mod_table[b] = cdc_ref_modulo(p, poly) | p;
    }
    return 0;
}

/* check_rabin_params -- rabin.rs:17-42 (all three errors are Unsupported). */
int cdc_ref_check_params(uint64_t avg, uint64_t min, uint64_t max) {
    if ((avg & (avg - 1)) != 0) return 1;
    if (min > avg) return 1;
    if (max < avg) return 1;
    return 0;
}

/* ------------------------------------------------------------------------ */
/* Rabin64 rolling state (rustic_cdc RollingHash64 impl)                     */
/* ------------------------------------------------------------------------ */

typedef struct {
    uint8_t  win[64];
    unsigned idx;
    uint64_t hash;
} rabin_state;

/* hash_byte: mod_index from the hash BEFORE the shift. */
static inline void hash_byte(const cdc_ref_tables *t, rabin_state *r,
                             uint8_t b) {
    uint64_t m = (r->hash >> t->shift) & 255;
    r->hash = ((r->hash << 8) | b) ^ t->mod_table[m];
}

/* slide(b) -- called at rabin.rs:187 once per byte after the min prefix. */
static inline void slide(const cdc_ref_tables *t, rabin_state *r, uint8_t b) {
    r->hash ^= t->out_table[r->win[r->idx]];
    r->win[r->idx] = b;
    hash_byte(t, r, b);
    r->idx = (r->idx + 1) & 63;
}

/* reset_and_prefill_window -- called at rabin.rs:149-151 with the 64 bytes
 * vec[len-64 .. len).  V1 (canonical): hash the first 63 items, write their
 * window slots, zero slot 63, window_index = 63; the 64th item is left
 * unconsumed.  Variant A: zero the window and slide all 64 bytes.          */
static void reset_and_prefill(const cdc_ref_tables *t, rabin_state *r,
                              const uint8_t *last64, int prefill64) {
    r->hash = 0;
    if (!prefill64) {
        for (int j = 0; j < 63; j++) {
            r->win[j] = last64[j];
            hash_byte(t, r, last64[j]);
        }
        r->win[63] = 0;
        r->idx = 63;
    } else {
        memset(r->win, 0, sizeof r->win);
        r->idx = 0;
        for (int j = 0; j < 64; j++) slide(t, r, last64[j]);
    }
}

/* ------------------------------------------------------------------------ */
/* ChunkIter::next over a whole in-memory stream (rabin.rs:107-191)         */
/* ------------------------------------------------------------------------ */

size_t cdc_ref_chunk(const cdc_ref_tables *t, const uint8_t *data, size_t n,
                     uint64_t min, uint64_t avg, uint64_t max, int prefill64,
                     uint64_t *cuts, size_t cap) {
    const uint64_t split_mask = avg - 1; /* rabin.rs:92 */
    rabin_state r;
    memset(&r, 0, sizeof r);
    size_t s = 0, nc = 0;
    for (;;) {
        if (s == n) break; /* next() -> None */
        if (n - s < min) { /* rabin.rs:141-147: short read -> final chunk */
            if (nc < cap) cuts[nc] = n;
            nc++;
            break;
        }
        /* vec = data[s .. s+min); prefill from its last 64 bytes */
        reset_and_prefill(t, &r, data + s + min - 64, prefill64);
        size_t L = s + min;
        int finished = 0;
        for (;;) {
            if (L - s >= max) break;                   /* :154 */
            if ((r.hash & split_mask) == 0) break;     /* :158 */
            if (L == n) { finished = 1; break; }        /* :164-166 Ok(0) */
            slide(t, &r, data[L]);                      /* :185-187 */
            L++;
        }
        if (nc < cap) cuts[nc] = L;
        nc++;
        s = L;
        if (finished) break;
    }
    return nc;
}

/* ------------------------------------------------------------------------ */
/* Reference-equivalent work (CPU baseline): owned chunk Vec + 4 KiB buffer  */
/* ------------------------------------------------------------------------ */

typedef struct {
    const uint8_t *src; /* Cursor<Vec<u8>> */
    size_t src_len, src_pos;
    uint8_t buf[4096]; /* BUF_SIZE, rabin.rs:12 */
    size_t buf_len, pos;
    int finished;
    uint64_t short_reads; /* 0: Cursor (full reads); else xorshift state */
} owned_iter;

/* One Read::read of at most `want` bytes.  A Cursor fills the request; with
 * short_reads set every read returns a pseudo-random 1..want bytes (a pipe or
 * stdin reader, commands/backup.rs:339-345), which also shrinks the 4 KiB
 * buffer for good (`self.buf.truncate(size)`, rabin.rs:170). */
static size_t reader_read(owned_iter *it, uint8_t *dst, size_t want) {
    size_t avail = it->src_len - it->src_pos;
    size_t k = want < avail ? want : avail;
    if (it->short_reads && k > 1) {
        uint64_t x = it->short_reads;
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        it->short_reads = x;
        k = 1 + (size_t)(x % k);
    }
    memcpy(dst, it->src + it->src_pos, k);
    it->src_pos += k;
    return k;
}

/* take(want).read_to_end(): loop reads until `want` bytes or EOF */
static size_t cursor_read(owned_iter *it, uint8_t *dst, size_t want) {
    size_t got = 0;
    while (got < want) {
        size_t k = reader_read(it, dst + got, want - got);
        if (k == 0) break;
        got += k;
    }
    return got;
}

/* returns chunk length, 0 at end, CDC_REF_UNDERFLOW where the reference's
 * `min_size -= open_buf_len` (rabin.rs:124) would underflow: up to
 * BUF_SIZE - 1 = 4095 read-ahead bytes (rabin.rs:12) exceed min.  The
 * reference panics there under debug assertions (its test profile) and
 * wraps in release (take(huge) then returns the whole remainder as one
 * chunk, read-pattern dependent), so this mode stops instead of copying
 * past `vec` (which holds max + 8 bytes).  librcdc rejects min < 4096. */
static size_t owned_next(const cdc_ref_tables *t, owned_iter *it,
                         rabin_state *r, uint8_t *vec, uint64_t mask,
                         uint64_t min, uint64_t max) {
    if (it->finished) return 0;
    size_t min_size = min, len = 0;
    size_t open = it->buf_len - it->pos; /* rabin.rs:120-126 */
    if (open > min_size) {
        it->finished = 1;
        return CDC_REF_UNDERFLOW;
    }
    if (open > 0) {
        memcpy(vec, it->buf + it->pos, open);
        len = open;
        it->pos = it->buf_len;
        min_size -= open;
    }
    size_t size = cursor_read(it, vec + len, min_size); /* take().read_to_end */
    len += size;
    if (size < min_size) { /* :141-147 */
        it->finished = 1;
        return len;
    }
    reset_and_prefill(t, r, vec + len - 64, 0);
    for (;;) {
        if (len >= max) break;
        if ((r->hash & mask) == 0) break;
        if (it->buf_len == it->pos) {
            size_t k = reader_read(it, it->buf, it->buf_len); /* :163 */
            if (k == 0) { it->finished = 1; break; }
            it->pos = 0;
            it->buf_len = k; /* buf.truncate(size) */
        }
        uint8_t byte = it->buf[it->pos];
        vec[len++] = byte; /* vec.push(byte) */
        it->pos++;
        slide(t, r, byte);
    }
    return len;
}

size_t cdc_ref_chunk_owned_reads(const cdc_ref_tables *t, const uint8_t *data,
                                 size_t n, uint64_t min, uint64_t avg,
                                 uint64_t max, uint64_t read_seed,
                                 uint64_t *cuts, size_t cap) {
    owned_iter *it = (owned_iter *)calloc(1, sizeof *it);
    it->short_reads = read_seed;
    uint8_t *vec = (uint8_t *)malloc(max + 8);
    rabin_state r;
    memset(&r, 0, sizeof r);
    it->src = data;
    it->src_len = n;
    it->buf_len = sizeof it->buf;
    it->pos = sizeof it->buf;
    size_t nc = 0, off = 0;
    for (;;) {
        size_t len = owned_next(t, it, &r, vec, avg - 1, min, max);
        if (len == 0) break;
        if (len == CDC_REF_UNDERFLOW) { nc = CDC_REF_UNDERFLOW; break; }
        off += len;
        if (nc < cap) cuts[nc] = off;
        nc++;
    }
    free(vec);
    free(it);
    return nc;
}

size_t cdc_ref_chunk_owned(const cdc_ref_tables *t, const uint8_t *data,
                           size_t n, uint64_t min, uint64_t avg, uint64_t max,
                           uint64_t *cuts, size_t cap) {
    return cdc_ref_chunk_owned_reads(t, data, n, min, avg, max, 0, cuts, cap);
}

typedef struct {
    const cdc_ref_tables *t;
    const uint8_t *data;
    const uint64_t *offs, *lens;
    size_t nfiles;
    uint64_t min, avg, max;
    uint64_t *counts;
    /* optional cut lists: file f's cuts go to cuts[cut_base[f] ..], at most
     * cut_cap[f] of them (cdc_ref_chunk_many_cuts) */
    uint64_t *cuts;
    const uint64_t *cut_base, *cut_cap;
    size_t next; /* shared work counter */
    pthread_mutex_t mu;
    uint64_t total;
} many_ctx;

static void *many_worker(void *arg) {
    many_ctx *c = (many_ctx *)arg;
    owned_iter *it = (owned_iter *)calloc(1, sizeof *it);
    uint8_t *vec = (uint8_t *)malloc(c->max + 8);
    uint64_t local = 0;
    for (;;) {
        pthread_mutex_lock(&c->mu);
        size_t f = c->next++;
        pthread_mutex_unlock(&c->mu);
        if (f >= c->nfiles) break;
        /* a fresh iterator per file (file_archiver.rs:144, chunker.rs:30) */
        rabin_state r;
        memset(&r, 0, sizeof r);
        memset(it, 0, sizeof *it);
        it->src = c->data + c->offs[f];
        it->src_len = c->lens[f];
        it->buf_len = sizeof it->buf;
        it->pos = sizeof it->buf;
        uint64_t k = 0, off = 0;
        for (;;) {
            size_t len = owned_next(c->t, it, &r, vec, c->avg - 1, c->min, c->max);
            if (len == 0 || len == CDC_REF_UNDERFLOW) break;
            off += len;
            if (c->cuts && k < c->cut_cap[f]) c->cuts[c->cut_base[f] + k] = off;
            k++;
        }
        if (c->counts) c->counts[f] = k;
        local += k;
    }
    pthread_mutex_lock(&c->mu);
    c->total += local;
    pthread_mutex_unlock(&c->mu);
    free(vec);
    free(it);
    return NULL;
}

uint64_t cdc_ref_chunk_many_owned(const cdc_ref_tables *t, const uint8_t *data,
                                  const uint64_t *offs, const uint64_t *lens,
                                  size_t nfiles, uint64_t min, uint64_t avg,
                                  uint64_t max, int nthreads, uint64_t *counts) {
    many_ctx c;
    memset(&c, 0, sizeof c);
    c.t = t; c.data = data; c.offs = offs; c.lens = lens; c.nfiles = nfiles;
    c.min = min; c.avg = avg; c.max = max; c.counts = counts;
    pthread_mutex_init(&c.mu, NULL);
    if (nthreads < 1) nthreads = 1;
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof *th);
    for (int i = 0; i < nthreads; i++) pthread_create(&th[i], NULL, many_worker, &c);
    for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
    free(th);
    pthread_mutex_destroy(&c.mu);
    return c.total;
}

uint64_t cdc_ref_chunk_many_cuts(const cdc_ref_tables *t, const uint8_t *data,
                                 const uint64_t *offs, const uint64_t *lens,
                                 size_t nfiles, uint64_t min, uint64_t avg,
                                 uint64_t max, int nthreads, uint64_t *counts,
                                 uint64_t *cuts, const uint64_t *cut_base,
                                 const uint64_t *cut_cap) {
    many_ctx c;
    memset(&c, 0, sizeof c);
    c.t = t; c.data = data; c.offs = offs; c.lens = lens; c.nfiles = nfiles;
    c.min = min; c.avg = avg; c.max = max; c.counts = counts;
    c.cuts = cuts; c.cut_base = cut_base; c.cut_cap = cut_cap;
    pthread_mutex_init(&c.mu, NULL);
    if (nthreads < 1) nthreads = 1;
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof *th);
    for (int i = 0; i < nthreads; i++) pthread_create(&th[i], NULL, many_worker, &c);
    for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
    free(th);
    pthread_mutex_destroy(&c.mu);
    return c.total;
}

/* FixedSize -- fixed_size.rs:41-70 */
size_t cdc_ref_fixed(size_t n, uint64_t size, uint64_t *cuts, size_t cap) {
    size_t nc = 0, s = 0;
    while (s < n) {
        size_t e = (n - s < size) ? n : s + size;
        if (nc < cap) cuts[nc] = e;
        nc++;
        s = e;
    }
    return nc;
}

void cdc_ref_candidates(const cdc_ref_tables *t, const uint8_t *data,
                        size_t n, uint64_t mask, size_t first, size_t count,
                        uint8_t *flags) {
    (void)n;
    rabin_state r;
    memset(&r, 0, sizeof r); /* zero window: out_table[0] == 0 */
    size_t p0 = first - 64;
    for (size_t i = p0; i < first; i++) slide(t, &r, data[i]);
    for (size_t i = 0; i < count; i++) {
        flags[i] = (r.hash & mask) == 0;
        if (i + 1 < count) slide(t, &r, data[first + i]);
    }
}

/* ------------------------------------------------------------------------ */
/* rand 0.10 StdRng = ChaCha12                        */
/* ------------------------------------------------------------------------ */

static inline uint32_t rotl32(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }

#define QR(a, b, c, d)                       \
    a += b; d ^= a; d = rotl32(d, 16);       \
    c += d; b ^= c; b = rotl32(b, 12);       \
    a += b; d ^= a; d = rotl32(d, 8);        \
    c += d; b ^= c; b = rotl32(b, 7);

static void chacha12_block(const uint32_t key[8], uint64_t counter,
                           uint8_t out[64]) {
    uint32_t in[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                       key[0], key[1], key[2], key[3], key[4], key[5], key[6],
                       key[7], (uint32_t)counter, (uint32_t)(counter >> 32), 0,
                       0};
    uint32_t x[16];
    memcpy(x, in, sizeof x);
    for (int i = 0; i < 6; i++) { /* 12 rounds = 6 double rounds */
        QR(x[0], x[4], x[8], x[12]);
        QR(x[1], x[5], x[9], x[13]);
        QR(x[2], x[6], x[10], x[14]);
        QR(x[3], x[7], x[11], x[15]);
        QR(x[0], x[5], x[10], x[15]);
        QR(x[1], x[6], x[11], x[12]);
        QR(x[2], x[7], x[8], x[13]);
        QR(x[3], x[4], x[9], x[14]);
    }
    for (int i = 0; i < 16; i++) {
        uint32_t v = x[i] + in[i];
        out[4 * i + 0] = (uint8_t)v;
        out[4 * i + 1] = (uint8_t)(v >> 8);
        out[4 * i + 2] = (uint8_t)(v >> 16);
        out[4 * i + 3] = (uint8_t)(v >> 24);
    }
}

/* SeedableRng::seed_from_u64: PCG32 fills the 32-byte seed, 4 LE bytes each */
static void seed_from_u64(uint64_t state, uint32_t key[8]) {
    const uint64_t MUL = 6364136223846793005ULL;
    const uint64_t INC = 11634580027462260723ULL;
    for (int i = 0; i < 8; i++) {
        state = state * MUL + INC;
        uint32_t xs = (uint32_t)(((state >> 18) ^ state) >> 27);
        uint32_t rot = (uint32_t)(state >> 59);
        key[i] = (xs >> rot) | (xs << ((32 - rot) & 31));
    }
}

void cdc_ref_stdrng_fill_at(uint64_t seed, uint64_t skip, uint8_t *buf,
                            size_t n) {
    uint32_t key[8];
    seed_from_u64(seed, key);
    uint64_t ctr = skip / 64;
    uint8_t blk[64];
    size_t i = 0;
    while (i + 64 <= n) {
        chacha12_block(key, ctr++, buf + i);
        i += 64;
    }
    if (i < n) {
        chacha12_block(key, ctr, blk);
        memcpy(buf + i, blk, n - i);
    }
}

void cdc_ref_stdrng_fill(uint64_t seed, uint8_t *buf, size_t n) {
    cdc_ref_stdrng_fill_at(seed, 0, buf, n);
}
