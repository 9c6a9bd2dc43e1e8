// abi_e2e -- the drop-in C ABI under the caller's load, without Python.
//
// A native restatement of what a Rust `ChunkIter::Gpu` caller does
// (INTEGRATION.md): `--threads` workers (pariter, archiver.rs:195) take files
// one at a time, open an rcdc_stream on one shared rcdc_ctx and feed the
// file in `--read-mib` reads from pageable host memory (rabin.rs:162-182's
// reader), collecting the cut offsets.  Files are generated in host memory
// before the timed region (no disk: the rate is the chunker's, PCIe
// included).  Also measures the box's H2D copy rates (the bound of this
// path) and, with --batch, rcdc_chunk_batch over the same files.
//
// File f, 8-byte word i = splitmix64(f << 40 | i); with --mixed, every 4 MiB
// block b starts with a zero run of splitmix64(f << 40 | 1 << 39 | b) % 4 MiB
// bytes (about half the bytes).  bench.py regenerates the same bytes in
// numpy for the parity check (--dump writes the first files' cuts).
//
// Output: one JSON line.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "../include/rcdc.h"

static uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

static void fill_file(uint8_t *p, uint64_t n, uint64_t f, bool mixed) {
    uint64_t *w = reinterpret_cast<uint64_t *>(p);
    for (uint64_t i = 0; i < n / 8; i++) w[i] = splitmix64(f << 40 | i);
    for (uint64_t i = n / 8 * 8; i < n; i++) p[i] = (uint8_t)(splitmix64(f << 40 | (i / 8)) >> (8 * (i % 8)));
    if (!mixed) return;
    const uint64_t B = 4ull << 20;
    for (uint64_t b = 0; b * B < n; b++) {
        const uint64_t z = splitmix64(f << 40 | 1ull << 39 | b) % B;
        const uint64_t a = b * B, e = std::min(n, a + z);
        memset(p + a, 0, e - a);
    }
}

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static double h2d_rate(bool pinned, uint64_t bytes) {
    void *d = nullptr, *h = nullptr;
    if (hipMalloc(&d, bytes) != hipSuccess) return -1;
    if (pinned) {
        if (hipHostMalloc(&h, bytes, hipHostMallocDefault) != hipSuccess) return -1;
    } else {
        h = malloc(bytes);
    }
    memset(h, 1, bytes);
    (void)hipMemcpy(d, h, bytes, hipMemcpyHostToDevice);
    const double t0 = now();
    for (int r = 0; r < 3; r++) (void)hipMemcpy(d, h, bytes, hipMemcpyHostToDevice);
    const double el = now() - t0;
    if (pinned) (void)hipHostFree(h);
    else free(h);
    (void)hipFree(d);
    return 3.0 * bytes / el / (1ull << 30);
}

// The bound of the ABI paths under the same concurrency:
// `threads` workers take the same files and only copy them to the device,
// each on its own HIP stream.  mode 0: hipMemcpyAsync of each `rd`-byte read
// straight from the pageable file bytes (the runtime stages them); 1: what an
// rcdc lane does -- 4 MiB blocks memcpy'd into one of 4 pinned slots, then an
// async DMA from it, the copies running ahead of the DMA (run_host_pieces,
// kStageBytes / stage_slots); 2: the same DMA pattern from pinned slots
// filled once (the link's own limit at this concurrency, no host copy).
// Returns GiB/s.
static double h2d_concurrent(const std::vector<uint8_t *> &data, uint64_t n, uint64_t rd,
                             int threads, int mode) {
    constexpr int kSlots = 4;
    const uint64_t blk = mode == 0 ? rd : (4ull << 20);
    // per-thread streams, device buffers and pinned slots, allocated before
    // the timed region (as a context's lanes are)
    struct Res {
        hipStream_t s = nullptr;
        void *d = nullptr;
        void *h[kSlots] = {};
        hipEvent_t ev[kSlots] = {};
    };
    std::vector<Res> res(threads);
    int bad = 0;
    for (auto &r : res) {
        if (hipStreamCreateWithFlags(&r.s, hipStreamNonBlocking) != hipSuccess) bad++;
        if (hipMalloc(&r.d, n) != hipSuccess) bad++;
        for (int k = 0; k < kSlots; k++) {
            if (mode && hipHostMalloc(&r.h[k], blk, hipHostMallocDefault) != hipSuccess) bad++;
            if (mode == 2 && r.h[k]) memset(r.h[k], 1, blk);
            (void)hipEventCreateWithFlags(&r.ev[k], hipEventDisableTiming);
        }
    }
    (void)hipDeviceSynchronize();
    std::atomic<int> next{0};
    auto work = [&](Res &r) {
        uint64_t k = 0;
        for (;;) {
            const int f = next++;
            if (f >= (int)data.size() || bad) break;
            for (uint64_t o = 0; o < n; o += blk, k++) {
                const uint64_t len = std::min(blk, n - o);
                const int b = (int)(k % kSlots);
                if (mode) {
                    if (k >= (uint64_t)kSlots) (void)hipEventSynchronize(r.ev[b]);  // slot free
                    if (mode == 1) memcpy(r.h[b], data[f] + o, len);
                    (void)hipMemcpyAsync((uint8_t *)r.d + o, r.h[b], len, hipMemcpyHostToDevice, r.s);
                } else {
                    (void)hipMemcpyAsync((uint8_t *)r.d + o, data[f] + o, len, hipMemcpyHostToDevice,
                                         r.s);
                }
                (void)hipEventRecord(r.ev[b], r.s);
            }
        }
        (void)hipStreamSynchronize(r.s);
    };
    const double t0 = now();
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++) th.emplace_back(work, std::ref(res[t]));
    for (auto &x : th) x.join();
    const double el = now() - t0;
    for (auto &r : res) {
        (void)hipFree(r.d);
        for (int j = 0; j < kSlots; j++) {
            if (r.h[j]) (void)hipHostFree(r.h[j]);
            (void)hipEventDestroy(r.ev[j]);
        }
        (void)hipStreamDestroy(r.s);
    }
    return bad ? -1.0 : (double)data.size() * n / el / (1ull << 30);
}

int main(int argc, char **argv) {
    int threads = 16, files = 32, dump = 0;
    uint64_t file_mib = 256, read_mib = 32;  // 32 MiB reads: stream path 0.92-0.94 of the bound (16 MiB: 0.88)
    bool mixed = false, batch = false;
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        auto next = [&]() { return i + 1 < argc ? argv[++i] : (char *)"0"; };
        if (a == "--threads") threads = atoi(next());
        else if (a == "--files") files = atoi(next());
        else if (a == "--file-mib") file_mib = strtoull(next(), nullptr, 10);
        else if (a == "--read-mib") read_mib = strtoull(next(), nullptr, 10);
        else if (a == "--mixed") mixed = true;
        else if (a == "--batch") batch = true;
        else if (a == "--dump") dump = atoi(next());
    }
    const uint64_t n = file_mib << 20, rd = read_mib << 20;
    std::vector<uint8_t *> data(files);
    {
        std::vector<std::thread> gen;
        for (int t = 0; t < threads; t++)
            gen.emplace_back([&, t]() {
                for (int f = t; f < files; f += threads) {
                    data[f] = (uint8_t *)malloc(n);
                    fill_file(data[f], n, (uint64_t)f, mixed);
                }
            });
        for (auto &g : gen) g.join();
    }
    rcdc_ctx *ctx = nullptr;
    if (rcdc_ctx_create(0x003DA3358B4DC173ull, 512 << 10, 1 << 20, 8 << 20, 0, &ctx)) {
        fprintf(stderr, "ctx: %s\n", rcdc_last_error());
        return 1;
    }
    std::vector<std::vector<uint64_t>> cuts(files);
    std::atomic<int> next_file{0};
    std::atomic<int> errors{0};
    auto worker = [&]() {
        std::vector<uint64_t> buf(n / (512 << 10) + 4);
        for (;;) {
            const int f = next_file++;
            if (f >= files) return;
            rcdc_stream *st = nullptr;
            if (rcdc_stream_open(ctx, &st)) {
                errors++;
                return;
            }
            for (uint64_t o = 0; o < n || o == 0; o += rd) {
                const uint64_t len = std::min(rd, n - o);
                const int fin = o + len >= n;
                uint64_t k = 0;
                if (rcdc_stream_feed(st, data[f] + o, len, fin, buf.data(), buf.size(), &k)) {
                    fprintf(stderr, "feed: %s\n", rcdc_last_error());
                    errors++;
                    break;
                }
                cuts[f].insert(cuts[f].end(), buf.begin(), buf.begin() + (long)k);
                if (fin) break;
            }
            rcdc_stream_close(st);
        }
    };
    // warm-up: lanes and plans for every worker
    {
        next_file = 0;
        const int saved = files;
        files = std::min(files, threads);
        std::vector<std::thread> th;
        for (int t = 0; t < threads; t++) th.emplace_back(worker);
        for (auto &x : th) x.join();
        files = saved;
        for (auto &c : cuts) c.clear();
    }
    next_file = 0;
    const double t0 = now();
    {
        std::vector<std::thread> th;
        for (int t = 0; t < threads; t++) th.emplace_back(worker);
        for (auto &x : th) x.join();
    }
    const double el = now() - t0;
    uint64_t ncuts = 0, xs = 0;
    for (auto &c : cuts) {
        ncuts += c.size();
        for (uint64_t v : c) xs ^= splitmix64(v);
    }
    double batch_gibs = -1;
    if (batch) {
        // rcdc_chunk_batch: each worker chunks groups of 4 files in one call
        std::atomic<int> nf{0};
        auto bw = [&]() {
            std::vector<uint64_t> out(4 * (n / (512 << 10) + 2)), cnt(4);
            for (;;) {
                const int f0 = nf.fetch_add(4);
                if (f0 >= files) return;
                rcdc_buf b[4];
                uint32_t m = 0;
                for (int f = f0; f < files && m < 4; f++, m++) b[m] = {data[f], n};
                if (rcdc_chunk_batch(ctx, b, m, out.data(), out.size(), cnt.data())) errors++;
            }
        };
        const double t1 = now();
        std::vector<std::thread> th;
        for (int t = 0; t < threads; t++) th.emplace_back(bw);
        for (auto &x : th) x.join();
        batch_gibs = (double)files * n / (now() - t1) / (1ull << 30);
    }
    for (int f = 0; f < dump && f < files; f++) {
        char name[64];
        snprintf(name, sizeof name, "abi_e2e_cuts_%d.bin", f);
        FILE *fp = fopen(name, "wb");
        if (fp) {
            fwrite(cuts[f].data(), 8, cuts[f].size(), fp);
            fclose(fp);
        }
    }
    rcdc_ctx_destroy(ctx);
    const double pin = h2d_rate(true, 1ull << 30), pag = h2d_rate(false, 1ull << 30);
    // the concurrent bound: same files, reads and thread count, copies only
    // (twice each, the better pass kept: the first also warms the engines)
    double cb_direct = -1, cb_staged = -1, cb_dma = -1;
    for (int r = 0; r < 2; r++) {
        cb_direct = std::max(cb_direct, h2d_concurrent(data, n, rd, threads, 0));
        cb_staged = std::max(cb_staged, h2d_concurrent(data, n, rd, threads, 1));
        cb_dma = std::max(cb_dma, h2d_concurrent(data, n, rd, threads, 2));
    }
    const double bound = std::max(std::max(cb_direct, cb_staged), cb_dma);
    const double sg = (double)files * n / el / (1ull << 30);
    printf("{\"abi_stream_gibs\": %.2f, \"abi_batch_gibs\": %.2f, \"h2d_pinned_gibs\": %.2f, "
           "\"h2d_pageable_gibs\": %.2f, \"h2d_concurrent_direct_gibs\": %.2f, "
           "\"h2d_concurrent_staged_gibs\": %.2f, \"h2d_concurrent_dma_gibs\": %.2f, "
           "\"h2d_concurrent_bound_gibs\": %.2f, "
           "\"stream_frac_of_bound\": %.3f, \"batch_frac_of_bound\": %.3f, "
           "\"threads\": %d, \"files\": %d, \"file_mib\": %llu, "
           "\"read_mib\": %llu, \"mixed\": %s, \"cuts\": %llu, \"cut_hash\": \"%016llx\", "
           "\"errors\": %d, \"seconds\": %.3f}\n",
           sg, batch_gibs, pin, pag, cb_direct, cb_staged, cb_dma, bound, sg / bound,
           batch_gibs > 0 ? batch_gibs / bound : -1.0, threads, files,
           (unsigned long long)file_mib, (unsigned long long)read_mib, mixed ? "true" : "false",
           (unsigned long long)ncuts, (unsigned long long)xs, errors.load(), el);
    for (auto *p : data) free(p);
    return errors ? 1 : 0;
}
