// Byte-step throughput of the Rabin64 slide (no global memory): data bytes
// from registers, OUT/MOD tables in LDS (32 lane-private copies), NC chains
// per lane, WAVES waves per CU.  LDSMODE 0: real LDS lookups; 1: lookups
// faked by one v_xor (keeps the dependency chain, no LDS); CHK 0/1: candidate
// test on/off (h kept alive through the output).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define STEPS 4096
constexpr uint32_t kA = 0xF0, kB = 0xCC, kC = 0xAA;
__device__ __forceinline__ uint32_t in_vgpr(uint32_t x) {
    uint32_t r; asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "s"(x)); return r; }
template <int LDSMODE>
__device__ __forceinline__ uint2 lk(const uint8_t *tab, uint32_t a) {
    if constexpr (LDSMODE == 1) return make_uint2(a ^ 0x1234567u, a ^ 0x89ABCDu);
    else return *reinterpret_cast<const uint2 *>(tab + a);
}
template <int K, int LDSMODE>
__device__ __forceinline__ void slide(uint32_t &h0, uint32_t &h1, uint32_t dn, uint32_t dold,
                                      const uint8_t *tab, uint32_t lwo, uint32_t lwm, uint32_t kff00) {
    const uint2 o = lk<LDSMODE>(tab, __builtin_amdgcn_perm(dold, lwo, 0x0C0C0000u | ((4u + K) << 8)));
    const uint32_t a1x = __builtin_amdgcn_alignbit(h1, h0, 24) ^ o.y;
    const uint32_t am = __builtin_amdgcn_bitop3_b32(a1x >> 13, kff00, lwm, (kA & kB) | kC);
    const uint2 m = lk<LDSMODE>(tab, am);
    h0 = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_perm(h0, dn, 0x06050400u | K), o.x, m.x, kA ^ kB ^ kC);
    h1 = a1x ^ m.y;
}

// g-form: g = h ^ out[next outgoing byte]; MOD index straight from g1.
template <int K, int LDSMODE>
__device__ __forceinline__ uint32_t slideg(uint32_t &g0, uint32_t &g1, uint32_t dn, uint32_t dold,
                                           const uint8_t *tab, uint32_t lwo, uint32_t lwm, uint32_t kff00) {
    const uint32_t am = __builtin_amdgcn_bitop3_b32(g1 >> 5, kff00, lwm, (kA & kB) | kC);
    const uint2 m = lk<LDSMODE>(tab, am);
    const uint2 o = lk<LDSMODE>(tab, __builtin_amdgcn_perm(dold, lwo, 0x0C0C0000u | ((4u + K) << 8)));
    const uint32_t a1 = __builtin_amdgcn_alignbit(g1, g0, 24);
    const uint32_t h0 = __builtin_amdgcn_perm(g0, dn, 0x06050400u | K) ^ m.x;
    g0 = h0 ^ o.x;
    g1 = __builtin_amdgcn_bitop3_b32(a1, m.y, o.y, kA ^ kB ^ kC);
    return h0;
}
template <int NC, int WAVES, int LDSMODE, int CHK, bool GF>
__global__ __launch_bounds__(WAVES * 64, 1) void kern(const uint64_t *gtab, uint32_t *out, uint32_t seed) {
    __shared__ __attribute__((aligned(16))) uint8_t tab[131072];
    for (uint32_t i = threadIdx.x; i < 256 * 32; i += WAVES * 64) {
        const uint32_t e = i / 32, c = i % 32;
        *reinterpret_cast<uint2 *>(tab + e * 256 + c * 8) = make_uint2((uint32_t)gtab[e], (uint32_t)(gtab[e] >> 32));
        *reinterpret_cast<uint2 *>(tab + 65536 + e * 256 + c * 8) = make_uint2((uint32_t)gtab[256 + e], (uint32_t)(gtab[256 + e] >> 32));
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t lwo = (lane & 31) * 8, lwm = lwo | 65536;
    const uint32_t kff00 = in_vgpr(0xFF00u), mask = in_vgpr(0xFFFFFu);
    uint32_t h0[NC], h1[NC], d[NC][4], hk[NC];
    uint64_t any = 0;
    uint16_t acc16[NC]; uint32_t acc32[NC];
    for (int c = 0; c < NC; c++) { acc16[c] = 0xFFFF; acc32[c] = ~0u; }
#pragma unroll
    for (int c = 0; c < NC; c++) {
        h0[c] = threadIdx.x * 0x9E3779B1u + c + seed; h1[c] = (threadIdx.x * 77u + c) & 0x1FFFFF;
        for (int j = 0; j < 4; j++) d[c][j] = (threadIdx.x + 1) * 0x01000193u * (j + 1 + c) ^ seed;
    }
    for (int s = 0; s < STEPS / 16; s++) {
#pragma unroll
        for (int b = 0; b < 16; b++) {
#pragma unroll
            for (int c = 0; c < NC; c++) {
                const uint32_t dn = d[c][b >> 2], dold = d[c][(b >> 2) ^ 1];
                if constexpr (GF) {
                    uint32_t hv;
                    switch (b & 3) {
                        case 0: hv = slideg<0, LDSMODE>(h0[c], h1[c], dn, dold, tab, lwo, lwm, kff00); break;
                        case 1: hv = slideg<1, LDSMODE>(h0[c], h1[c], dn, dold, tab, lwo, lwm, kff00); break;
                        case 2: hv = slideg<2, LDSMODE>(h0[c], h1[c], dn, dold, tab, lwo, lwm, kff00); break;
                        default: hv = slideg<3, LDSMODE>(h0[c], h1[c], dn, dold, tab, lwo, lwm, kff00); break;
                    }
                    hk[c] = hv;
                } else {
                switch (b & 3) {
                    case 0: slide<0, LDSMODE>(h0[c], h1[c], dn, dold, tab, lwo, lwm, kff00); break;
                    case 1: slide<1, LDSMODE>(h0[c], h1[c], dn, dold, tab, lwo, lwm, kff00); break;
                    case 2: slide<2, LDSMODE>(h0[c], h1[c], dn, dold, tab, lwo, lwm, kff00); break;
                    default: slide<3, LDSMODE>(h0[c], h1[c], dn, dold, tab, lwo, lwm, kff00); break;
                }
                hk[c] = h0[c];
                }
                if constexpr (CHK == 1) any |= __builtin_amdgcn_ballot_w64((hk[c] & mask) == 0u);
                if constexpr (CHK == 2) any |= __builtin_amdgcn_ballot_w64((uint16_t)hk[c] == 0);
                if constexpr (CHK == 3) acc16[c] = __builtin_elementwise_min(acc16[c], (uint16_t)hk[c]);
                if constexpr (CHK == 5) acc32[c] = __builtin_elementwise_min(acc32[c], hk[c] << 12);
                if constexpr (CHK == 6) acc32[c] = __builtin_elementwise_min(acc32[c], hk[c]);
            }
        }
#pragma unroll
        for (int c = 0; c < NC; c++) {
            if constexpr (CHK == 3) { any |= __builtin_amdgcn_ballot_w64(acc16[c] == 0); acc16[c] = 0xFFFF; }
            if constexpr (CHK >= 5) { any |= __builtin_amdgcn_ballot_w64(acc32[c] == 0); acc32[c] = ~0u; }
        }
#pragma unroll
        for (int c = 0; c < NC; c++)
            for (int j = 0; j < 4; j++) d[c][j] = __builtin_amdgcn_alignbit(d[c][j], h0[c], 7);
    }
    uint32_t acc = (uint32_t)any;
#pragma unroll
    for (int c = 0; c < NC; c++) acc ^= h0[c] ^ h1[c] ^ hk[c];
    out[blockIdx.x * WAVES * 64 + threadIdx.x] = acc;
}
template <int NC, int WAVES, int LDSMODE, int CHK, bool GF = false>
void run(const uint64_t *gt, uint32_t *out, int cus) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    kern<NC, WAVES, LDSMODE, CHK, GF><<<cus, WAVES * 64>>>(gt, out, 1);
    (void)hipEventRecord(a);
    kern<NC, WAVES, LDSMODE, CHK, GF><<<cus, WAVES * 64>>>(gt, out, 2);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms; (void)hipEventElapsedTime(&ms, a, b);
    const double bytes_per_cu = (double)WAVES * 64 * NC * STEPS;
    const double ns_per_wavestep = ms * 1e6 / (WAVES * NC * (double)STEPS);
    printf("GF %d NC %d waves %2d lds %d chk %d: %.3f ms, %.3f ns/wave-step/CU -> %.0f GB/s chip\n", (int)GF, NC, WAVES, LDSMODE, CHK, ms,
           ns_per_wavestep, bytes_per_cu * cus / (ms * 1e-3) / 1e9);
}

// OUT value supplied by the caller (prefetched PD bytes ahead).
template <int K, int LDSMODE>
__device__ __forceinline__ void slide_po(uint32_t &h0, uint32_t &h1, uint32_t dn, uint2 o,
                                         const uint8_t *tab, uint32_t lwm, uint32_t kff00) {
    const uint32_t a1x = __builtin_amdgcn_alignbit(h1, h0, 24) ^ o.y;
    const uint32_t am = __builtin_amdgcn_bitop3_b32(a1x >> 13, kff00, lwm, (kA & kB) | kC);
    const uint2 m = lk<LDSMODE>(tab, am);
    h0 = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_perm(h0, dn, 0x06050400u | K), o.x, m.x, kA ^ kB ^ kC);
    h1 = a1x ^ m.y;
}
template <int K, int LDSMODE>
__device__ __forceinline__ uint32_t slideg_po(uint32_t &g0, uint32_t &g1, uint32_t dn, uint2 o,
                                              const uint8_t *tab, uint32_t lwm, uint32_t kff00) {
    const uint32_t am = __builtin_amdgcn_bitop3_b32(g1 >> 5, kff00, lwm, (kA & kB) | kC);
    const uint2 m = lk<LDSMODE>(tab, am);
    const uint32_t a1 = __builtin_amdgcn_alignbit(g1, g0, 24);
    const uint32_t h0 = __builtin_amdgcn_perm(g0, dn, 0x06050400u | K) ^ m.x;
    g0 = h0 ^ o.x;
    g1 = __builtin_amdgcn_bitop3_b32(a1, m.y, o.y, kA ^ kB ^ kC);
    return h0;
}
template <int K>
__device__ __forceinline__ uint2 oload(uint32_t dold, const uint8_t *tab, uint32_t lwo) {
    return *reinterpret_cast<const uint2 *>(tab + __builtin_amdgcn_perm(dold, lwo, 0x0C0C0000u | ((4u + K) << 8)));
}
__device__ __forceinline__ uint2 oload_b(int b, uint32_t dold, const uint8_t *tab, uint32_t lwo) {
    switch (b & 3) { case 0: return oload<0>(dold, tab, lwo); case 1: return oload<1>(dold, tab, lwo);
                     case 2: return oload<2>(dold, tab, lwo); default: return oload<3>(dold, tab, lwo); }
}
// NC = 1 only; CHK 3 (min3_u16 per 16) ; PD = prefetch distance (bytes)
template <int WAVES, bool GF, int PD>
__global__ __launch_bounds__(WAVES * 64, 1) void kernp(const uint64_t *gtab, uint32_t *out, uint32_t seed) {
    __shared__ __attribute__((aligned(16))) uint8_t tab[131072];
    for (uint32_t i = threadIdx.x; i < 256 * 32; i += WAVES * 64) {
        const uint32_t e = i / 32, c = i % 32;
        *reinterpret_cast<uint2 *>(tab + e * 256 + c * 8) = make_uint2((uint32_t)gtab[e], (uint32_t)(gtab[e] >> 32));
        *reinterpret_cast<uint2 *>(tab + 65536 + e * 256 + c * 8) = make_uint2((uint32_t)gtab[256 + e], (uint32_t)(gtab[256 + e] >> 32));
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t lwo = (lane & 31) * 8, lwm = lwo | 65536;
    const uint32_t kff00 = in_vgpr(0xFF00u);
    uint64_t any = 0;
    uint32_t h0 = threadIdx.x * 0x9E3779B1u + seed, h1 = (threadIdx.x * 77u) & 0x1FFFFF, d[4];
    for (int j = 0; j < 4; j++) d[j] = (threadIdx.x + 1) * 0x01000193u * (j + 1) ^ seed;
    uint32_t hk = 0;
    for (int s = 0; s < STEPS / 16; s++) {
        uint16_t acc = 0xFFFF;
        uint2 ob[16];
        if constexpr (PD > 0) {
#pragma unroll
            for (int b = 0; b < PD; b++) ob[b] = oload_b(b, d[(b >> 2) ^ 1], tab, lwo);
        }
#pragma unroll
        for (int b = 0; b < 16; b++) {
            const uint32_t dn = d[b >> 2];
            uint2 o;
            if constexpr (PD > 0) {
                if (b + PD < 16) ob[b + PD] = oload_b(b + PD, d[((b + PD) >> 2) ^ 1], tab, lwo);
                o = ob[b];
            } else {
                o = oload_b(b, d[(b >> 2) ^ 1], tab, lwo);
            }
            uint32_t hv;
            switch (b & 3) {
                case 0: hv = GF ? slideg_po<0, 0>(h0, h1, dn, o, tab, lwm, kff00) : (slide_po<0, 0>(h0, h1, dn, o, tab, lwm, kff00), h0); break;
                case 1: hv = GF ? slideg_po<1, 0>(h0, h1, dn, o, tab, lwm, kff00) : (slide_po<1, 0>(h0, h1, dn, o, tab, lwm, kff00), h0); break;
                case 2: hv = GF ? slideg_po<2, 0>(h0, h1, dn, o, tab, lwm, kff00) : (slide_po<2, 0>(h0, h1, dn, o, tab, lwm, kff00), h0); break;
                default: hv = GF ? slideg_po<3, 0>(h0, h1, dn, o, tab, lwm, kff00) : (slide_po<3, 0>(h0, h1, dn, o, tab, lwm, kff00), h0); break;
            }
            hk ^= hv;
            acc = __builtin_elementwise_min(acc, (uint16_t)hv);
        }
        any |= __builtin_amdgcn_ballot_w64(acc == 0);
        for (int j = 0; j < 4; j++) d[j] = __builtin_amdgcn_alignbit(d[j], h0, 7);
    }
    out[blockIdx.x * WAVES * 64 + threadIdx.x] = h0 ^ h1 ^ hk ^ (uint32_t)any;
}
template <int WAVES, bool GF, int PD>
void runp(const uint64_t *gt, uint32_t *out, int cus) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    kernp<WAVES, GF, PD><<<cus, WAVES * 64>>>(gt, out, 1);
    (void)hipEventRecord(a);
    kernp<WAVES, GF, PD><<<cus, WAVES * 64>>>(gt, out, 2);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms; (void)hipEventElapsedTime(&ms, a, b);
    const double ns = ms * 1e6 / (WAVES * (double)STEPS);
    printf("prefetch GF %d PD %d waves %2d: %.3f ms, %.3f ns/wave-step/CU -> %.0f GB/s chip\n", (int)GF, PD, WAVES, ms, ns,
           (double)WAVES * 64 * STEPS * cus / (ms * 1e-3) / 1e9);
}
int main() {
    hipDeviceProp_t pr; (void)hipGetDeviceProperties(&pr, 0);
    int cus = pr.multiProcessorCount;
    uint64_t ht[512];
    for (int i = 0; i < 512; i++) ht[i] = (0x9E3779B97F4A7C15ull * (i + 1)) & 0x1FFFFFFFFFFFFFull;
    uint64_t *gt; (void)hipMalloc(&gt, sizeof ht); (void)hipMemcpy(gt, ht, sizeof ht, hipMemcpyHostToDevice);
    uint32_t *out; (void)hipMalloc(&out, cus * 1024 * 4 * 4);
    run<1, 16, 0, 3>(gt, out, cus); run<1, 16, 0, 3, true>(gt, out, cus);
    runp<16, false, 0>(gt, out, cus); runp<16, false, 2>(gt, out, cus); runp<16, false, 4>(gt, out, cus);
    runp<16, true, 0>(gt, out, cus); runp<16, true, 2>(gt, out, cus); runp<16, true, 4>(gt, out, cus);
    runp<8, false, 4>(gt, out, cus); runp<8, true, 4>(gt, out, cus);
    runp<12, false, 4>(gt, out, cus); runp<12, true, 4>(gt, out, cus);
    return 0;
}
