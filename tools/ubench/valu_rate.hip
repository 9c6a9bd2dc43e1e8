// Microbenchmark: wave64 VALU throughput per instruction kind on gfx950.
// 16 waves/CU, 8 independent chains per lane, unrolled; prints ns per
// wave-instruction per CU -> cycles per instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 2048
#define CHAINS 8
template <int OP>
__global__ __launch_bounds__(1024) void k(uint32_t *out, uint32_t seed) {
    uint32_t r[CHAINS];
#pragma unroll
    for (int i = 0; i < CHAINS; i++) r[i] = threadIdx.x * 7 + i + seed;
    uint32_t s1 = seed * 3 + 1, s2 = seed ^ 0x5bd1e995;
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
#pragma unroll
            for (int i = 0; i < CHAINS; i++) {
                uint32_t x = r[i];
                if constexpr (OP == 0) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(x) : "v"(r[(i + 1) % CHAINS]));
                if constexpr (OP == 1) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x) : "v"(r[(i + 1) % CHAINS]), "s"(s1));
                if constexpr (OP == 2) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(r[(i + 1) % CHAINS]), "v"(r[(i + 2) % CHAINS]));
                if constexpr (OP == 3) asm volatile("v_alignbit_b32 %0, %0, %1, 24" : "+v"(x) : "v"(r[(i + 1) % CHAINS]));
                if constexpr (OP == 4) asm volatile("v_lshl_or_b32 %0, %0, 8, %1" : "+v"(x) : "v"(r[(i + 1) % CHAINS]));
                if constexpr (OP == 5) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(x) : "v"(r[(i + 1) % CHAINS]));
                if constexpr (OP == 6) asm volatile("v_lshrrev_b32 %0, 13, %0" : "+v"(x));
                if constexpr (OP == 7) asm volatile("v_and_b32 %0, %1, %0" : "+v"(x) : "s"(s2));
                if constexpr (OP == 8) asm volatile("v_cmp_eq_u16 vcc, 0, %0" :: "v"(x) : "vcc");
                if constexpr (OP == 9) asm volatile("v_cmp_eq_u32 vcc, 0, %0" :: "v"(x) : "vcc");
                if constexpr (OP == 10) asm volatile("v_xor_b32 %0, %1, %0\n\tv_perm_b32 %0, %0, %1, %2" : "+v"(x) : "v"(r[(i + 1) % CHAINS]), "s"(s1));
                r[i] = x;
            }
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < CHAINS; i++) acc ^= r[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
template <int OP>
double run(uint32_t *d, int cus, int ninstr) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    k<OP><<<cus, 1024>>>(d, 1);
    hipEventRecord(a);
    k<OP><<<cus, 1024>>>(d, 2);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    double winstr = (double)cus * 16 * ITERS * 8 * CHAINS * ninstr;  // wave-instructions
    double per_cu_ns = ms * 1e6 / (winstr / cus);
    return per_cu_ns;  // ns per wave-instruction per CU
}
int main() {
    hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
    int cus = p.multiProcessorCount;
    uint32_t *d; hipMalloc(&d, cus * 1024 * 4);
    const char *names[] = {"v_xor_b32", "v_perm_b32", "v_bitop3_b32", "v_alignbit_b32", "v_lshl_or_b32",
                           "v_pk_add_u16", "v_lshrrev_b32", "v_and_b32(sgpr)", "v_cmp_eq_u16", "v_cmp_eq_u32", "xor+perm pair"};
    double r[11];
    r[0] = run<0>(d, cus, 1); r[1] = run<1>(d, cus, 1); r[2] = run<2>(d, cus, 1); r[3] = run<3>(d, cus, 1);
    r[4] = run<4>(d, cus, 1); r[5] = run<5>(d, cus, 1); r[6] = run<6>(d, cus, 1); r[7] = run<7>(d, cus, 1);
    r[8] = run<8>(d, cus, 1); r[9] = run<9>(d, cus, 1); r[10] = run<10>(d, cus, 2);
    printf("CUs %d clock %d MHz\n", cus, p.clockRate / 1000);
    for (int i = 0; i < 11; i++)
        printf("%-18s %.4f ns per wave-instr per CU  -> %.2f cyc/instr/SIMD @2.1GHz\n", names[i], r[i], r[i] * 4 * 2.1);
    return 0;
}
