// Memory-side ceiling of access patterns (no compute): 512 MiB read once.
// mode 0: coalesced (instr i: lane l reads wave_base + i*1024 + l*16)
// mode 1: per-lane segments of S bytes, 16 B per load (v0-like: 4 loads per 64 B)
// mode 2: adjacent-pair 32-B pieces (lanes 2p,2p+1 -> seg 2p then seg 2p+1)
// mode 3: per-lane segments, 64 B burst = 4 back-to-back loads, then next 64 B
// mode 4: per-lane segments, 128 B burst (8 loads)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <int MODE>
__global__ __launch_bounds__(1024) void k(const uint8_t *p, uint64_t bytes, uint32_t S, uint32_t *out) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t gw = (uint64_t)blockIdx.x * 16 + wave;       // global wave
    const uint64_t nw = (uint64_t)gridDim.x * 16;
    const uint64_t per_wave = 64ull * S;                         // bytes per wave-item
    u32x4 acc = {0, 0, 0, 0};
    for (uint64_t item = gw; item * per_wave < bytes; item += nw) {
        const uint8_t *base = p + item * per_wave;
        if constexpr (MODE == 0) {
            for (uint32_t i = 0; i < S / 16; i++)
                acc ^= *(const u32x4 *)(base + (uint64_t)i * 1024 + lane * 16);
        } else if constexpr (MODE == 1) {
            for (uint32_t i = 0; i < S / 16; i++) acc ^= *(const u32x4 *)(base + (uint64_t)lane * S + i * 16);
        } else if constexpr (MODE == 2) {
            const uint64_t va = (uint64_t)(lane & ~1u) * S + (lane & 1u) * 16;
            for (uint32_t i = 0; i < S / 32; i++) {
                acc ^= *(const u32x4 *)(base + va + i * 32);
                acc ^= *(const u32x4 *)(base + va + S + i * 32);
            }
        } else if constexpr (MODE == 3) {
            for (uint32_t i = 0; i < S / 64; i++) {
                const u32x4 *q = (const u32x4 *)(base + (uint64_t)lane * S + i * 64);
                u32x4 a = q[0], b = q[1], c = q[2], d = q[3];
                acc ^= a ^ b ^ c ^ d;
            }
        } else {
            for (uint32_t i = 0; i < S / 128; i++) {
                const u32x4 *q = (const u32x4 *)(base + (uint64_t)lane * S + i * 128);
                u32x4 a = q[0], b = q[1], c = q[2], d = q[3], e = q[4], f = q[5], g = q[6], h = q[7];
                acc ^= a ^ b ^ c ^ d ^ e ^ f ^ g ^ h;
            }
        }
    }
    out[blockIdx.x * 1024 + threadIdx.x] = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
}
template <int MODE>
void run(const uint8_t *p, uint64_t bytes, uint32_t S, uint32_t *out, int cus) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    k<MODE><<<cus, 1024>>>(p, bytes, S, out);
    (void)hipEventRecord(a);
    for (int r = 0; r < 5; r++) k<MODE><<<cus, 1024>>>(p, bytes, S, out);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms; (void)hipEventElapsedTime(&ms, a, b);
    printf("mode %d S %5u: %.1f us  %.0f GB/s\n", MODE, S, ms * 1e3 / 5, bytes * 5 / (ms * 1e-3) / 1e9);
}
int main() {
    hipDeviceProp_t pr; (void)hipGetDeviceProperties(&pr, 0);
    const uint64_t bytes = 512ull << 20;
    uint8_t *p; (void)hipMalloc(&p, bytes + (1 << 20));
    (void)hipMemset(p, 1, bytes);
    uint32_t *out; (void)hipMalloc(&out, pr.multiProcessorCount * 1024 * 4);
    int cus = pr.multiProcessorCount;
    for (uint32_t S : {1024u, 2048u, 4096u}) {
        run<0>(p, bytes, S, out, cus); run<1>(p, bytes, S, out, cus); run<2>(p, bytes, S, out, cus);
        run<3>(p, bytes, S, out, cus); run<4>(p, bytes, S, out, cus);
    }
    return 0;
}
