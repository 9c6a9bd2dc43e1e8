#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 1024
#define CHAINS 8
template <int OP>
__global__ __launch_bounds__(1024) void k(uint32_t *out, uint32_t seed) {
    uint32_t r[CHAINS];
    uint64_t q[CHAINS];
#pragma unroll
    for (int i = 0; i < CHAINS; i++) { r[i] = threadIdx.x * 7 + i + seed; q[i] = r[i] * 0x9E3779B97F4A7C15ull; }
    uint32_t s1 = seed * 3 + 1, s2 = seed ^ 0x5bd1e995;
    uint64_t m64 = 0x5555555555555555ull ^ seed;
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
#pragma unroll
            for (int i = 0; i < CHAINS; i++) {
                uint32_t x = r[i];
                if constexpr (OP == 0) { asm volatile("v_and_b32 %0, %1, %0" : "+v"(x) : "v"(r[(i + 1) % CHAINS])); }
                if constexpr (OP == 1) { asm volatile("v_or_b32 %0, %1, %0" : "+v"(x) : "v"(r[(i + 1) % CHAINS])); }
                if constexpr (OP == 2) { asm volatile("v_and_b32 %0, 0xff00, %0" : "+v"(x)); }
                if constexpr (OP == 3) { asm volatile("v_xor_b32 %0, %2, %0" : "+v"(x) : "v"(r[(i + 1) % CHAINS]), "s"(s2)); }
                if constexpr (OP == 4) { asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x6a" : "+v"(x) : "v"(r[(i + 1) % CHAINS]), "s"(s1)); }
                if constexpr (OP == 5) { asm volatile("v_lshrrev_b32 %0, 5, %0" : "+v"(x)); }
                if constexpr (OP == 6) { asm volatile("v_bfe_u32 %0, %0, 13, 8" : "+v"(x)); }
                if constexpr (OP == 7) { asm volatile("v_mul_u32_u24 %0, 0x1000, %0" : "+v"(x)); }
                if constexpr (OP == 8) { asm volatile("v_min_u32 %0, %1, %0" : "+v"(x) : "v"(r[(i + 1) % CHAINS])); }
                if constexpr (OP == 9) { asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(r[(i + 1) % CHAINS]), "v"(r[(i + 2) % CHAINS])); }
                if constexpr (OP == 10) { asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(r[(i + 1) % CHAINS])); }
                if constexpr (OP == 11) { asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(x) : "v"(r[(i + 1) % CHAINS]), "s"(m64)); }
                if constexpr (OP == 12) { asm volatile("v_xor_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(x) : "v"(r[(i + 1) % CHAINS])); }
                if constexpr (OP == 13) { asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(x) : "v"(r[(i + 1) % CHAINS])); }
                if constexpr (OP == 14) { asm volatile("v_min_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0" : "+v"(x) : "v"(r[(i + 1) % CHAINS])); }
                if constexpr (OP == 15) { asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(x) : "v"(r[(i + 1) % CHAINS])); }
                if constexpr (OP == 16) { asm volatile("v_xor_b32_dpp %0, %1, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(x) : "v"(r[(i + 1) % CHAINS])); }
                if constexpr (OP == 17) { asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(x), "+v"(r[(i + 1) % CHAINS])); }
                if constexpr (OP == 18) { asm volatile("v_permlane16_swap_b32 %0, %1" : "+v"(x), "+v"(r[(i + 1) % CHAINS])); }
                if constexpr (OP == 19) { asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x) : "v"(r[(i + 1) % CHAINS]), "v"(r[(i + 2) % CHAINS])); }
                if constexpr (OP == 20) { asm volatile("v_alignbit_b32 %0, %0, %1, %2" : "+v"(x) : "v"(r[(i + 1) % CHAINS]), "v"(r[(i + 2) % CHAINS])); }
                if constexpr (OP == 21) { asm volatile("v_add_u32 %0, %1, %0" : "+v"(x) : "v"(r[(i + 1) % CHAINS])); }
                if constexpr (OP == 22) { asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(r[(i + 1) % CHAINS]), "v"(r[(i + 2) % CHAINS])); }
                if constexpr (OP == 23) { asm volatile("v_lshl_add_u32 %0, %0, 8, %1" : "+v"(x) : "v"(r[(i + 1) % CHAINS])); }
                if constexpr (OP == 24) { asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(x) : "v"(r[(i + 1) % CHAINS]), "v"(r[(i + 2) % CHAINS])); }
                if constexpr (OP == 25) { asm volatile("v_lshlrev_b64 %0, 8, %0" : "+v"(q[i])); }
                if constexpr (OP == 26) { asm volatile("v_lshl_add_u64 %0, %0, 8, %1" : "+v"(q[i]) : "v"(q[(i+1)%CHAINS])); }
                if constexpr (OP == 27) { asm volatile("v_cmp_eq_u32_e64 %2, 0, %0" : "+v"(x) : "v"(r[(i + 1) % CHAINS]), "s"(m64)); }
                if constexpr (OP == 28) { asm volatile("v_cmp_gt_u32 vcc, 0x1000, %0" : "+v"(x) :: "vcc"); }
                if constexpr (OP == 29) { asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x) : "v"(r[(i + 1) % CHAINS]), "s"(s1)); }
                r[i] = x;
            }
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < CHAINS; i++) acc ^= r[i] ^ (uint32_t)q[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
template <int OP>
double run(uint32_t *d, int cus) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    k<OP><<<cus, 1024>>>(d, 1);
    (void)hipEventRecord(a);
    k<OP><<<cus, 1024>>>(d, 2);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms; (void)hipEventElapsedTime(&ms, a, b);
    double winstr = 16.0 * ITERS * 8 * CHAINS;  // wave-instructions per CU
    return ms * 1e6 / winstr;
}
int main() {
    hipDeviceProp_t p; (void)hipGetDeviceProperties(&p, 0);
    int cus = p.multiProcessorCount;
    uint32_t *d; (void)hipMalloc(&d, cus * 1024 * 4);
    double base = run<0>(d, cus);
    { double t = run<0>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_and_b32 vgpr", t, t / base); }
    { double t = run<1>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_or_b32 vgpr", t, t / base); }
    { double t = run<2>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_and_b32 literal", t, t / base); }
    { double t = run<3>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_xor_b32 sgpr", t, t / base); }
    { double t = run<4>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_bitop3 sgpr", t, t / base); }
    { double t = run<5>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_lshrrev (ref)", t, t / base); }
    { double t = run<6>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_bfe_u32", t, t / base); }
    { double t = run<7>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_mul_u32_u24", t, t / base); }
    { double t = run<8>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_min_u32", t, t / base); }
    { double t = run<9>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_min3_u32", t, t / base); }
    { double t = run<10>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_cndmask vcc", t, t / base); }
    { double t = run<11>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_cndmask_e64 s", t, t / base); }
    { double t = run<12>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_xor sdwa byte1", t, t / base); }
    { double t = run<13>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_mov sdwa->byte1", t, t / base); }
    { double t = run<14>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_min_u32 sdwa w0", t, t / base); }
    { double t = run<15>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_mov dpp qperm", t, t / base); }
    { double t = run<16>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_xor dpp qperm", t, t / base); }
    { double t = run<17>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_permlane32_swap", t, t / base); }
    { double t = run<18>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_permlane16_swap", t, t / base); }
    { double t = run<19>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_perm vgpr sel", t, t / base); }
    { double t = run<20>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_alignbit vgpr", t, t / base); }
    { double t = run<21>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_add_u32", t, t / base); }
    { double t = run<22>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_add3_u32", t, t / base); }
    { double t = run<23>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_lshl_add_u32", t, t / base); }
    { double t = run<24>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_xad_u32", t, t / base); }
    { double t = run<25>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_lshlrev_b64", t, t / base); }
    { double t = run<26>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_lshl_add_u64", t, t / base); }
    { double t = run<27>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_cmp_eq_u32 (e64 s)", t, t / base); }
    { double t = run<28>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_cmp_gt_u32 vcc", t, t / base); }
    { double t = run<29>(d, cus); printf("%-22s %.4f ns/wave-instr/CU  (%.2f x v_and vgpr)\n", "v_perm sgpr sel", t, t / base); }
    return 0;
}
