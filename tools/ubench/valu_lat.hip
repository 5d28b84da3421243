// valu_lat.hip -- issue rate and dependent latency of the VALU forms the fill uses
// (gfx950, one wave64 alone on a CU).  Each test runs N unrolled blocks of
// inline asm and reports shader cycles (s_memtime) per instruction.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

__global__ void k(unsigned long long *out, int n) {
    int a = threadIdx.x, b = threadIdx.x * 3, c = 7, d = 9, e = 11, f = 13, g = 15, h = 17;
    unsigned long long t0, t1;
    int idx = 0;
#define TEST(body)                                                            \
    t0 = __builtin_amdgcn_s_memtime();                                        \
    for (int i = 0; i < n; ++i) {                                             \
        asm volatile(REP64(body) : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) :: "vcc", "s34", "s35", "s36", "s37"); \
    }                                                                         \
    t1 = __builtin_amdgcn_s_memtime();                                        \
    if (threadIdx.x == 0) out[idx] = t1 - t0;                                 \
    idx++;
    // 0: independent adds (8 chains) -- 8 instr per body
    TEST("v_add_u32 %0, %0, %1\n v_add_u32 %1, %1, %2\n v_add_u32 %2, %2, %3\n v_add_u32 %3, %3, %4\n v_add_u32 %4, %4, %5\n v_add_u32 %5, %5, %6\n v_add_u32 %6, %6, %7\n v_add_u32 %7, %7, %0\n")
    // 1: dependent add chain -- 8 instr
    TEST("v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n")
    // 2: dependent max3 chain -- 8 instr
    TEST("v_max3_i32 %0, %0, %1, %2\n v_max3_i32 %0, %0, %1, %2\n v_max3_i32 %0, %0, %1, %2\n v_max3_i32 %0, %0, %1, %2\n v_max3_i32 %0, %0, %1, %2\n v_max3_i32 %0, %0, %1, %2\n v_max3_i32 %0, %0, %1, %2\n v_max3_i32 %0, %0, %1, %2\n")
    // 3: cmp_sdwa -> vcc -> addc, 4 pairs back to back (8 instr)
    TEST("v_cmp_eq_u32_sdwa vcc, %1, %2 src0_sel:BYTE_0 src1_sel:BYTE_1\n v_addc_co_u32_e32 %3, vcc, %3, %4, vcc\n v_cmp_eq_u32_sdwa vcc, %1, %2 src0_sel:BYTE_1 src1_sel:BYTE_1\n v_addc_co_u32_e32 %5, vcc, %5, %4, vcc\n v_cmp_eq_u32_sdwa vcc, %1, %2 src0_sel:BYTE_2 src1_sel:BYTE_1\n v_addc_co_u32_e32 %6, vcc, %6, %4, vcc\n v_cmp_eq_u32_sdwa vcc, %1, %2 src0_sel:BYTE_3 src1_sel:BYTE_1\n v_addc_co_u32_e32 %7, vcc, %7, %4, vcc\n")
    // 4: cmp to two SGPR pairs, then two addc_e64 (8 instr)
    TEST("v_cmp_eq_u32_sdwa s[34:35], %1, %2 src0_sel:BYTE_0 src1_sel:BYTE_1\n v_cmp_eq_u32_sdwa s[36:37], %1, %2 src0_sel:BYTE_1 src1_sel:BYTE_1\n v_addc_co_u32_e64 %3, vcc, %3, %4, s[34:35]\n v_addc_co_u32_e64 %5, vcc, %5, %4, s[36:37]\n v_cmp_eq_u32_sdwa s[34:35], %1, %2 src0_sel:BYTE_2 src1_sel:BYTE_1\n v_cmp_eq_u32_sdwa s[36:37], %1, %2 src0_sel:BYTE_3 src1_sel:BYTE_1\n v_addc_co_u32_e64 %6, vcc, %6, %4, s[34:35]\n v_addc_co_u32_e64 %7, vcc, %7, %4, s[36:37]\n")
    // 5: independent cmp_sdwa only (8)
    TEST("v_cmp_eq_u32_sdwa vcc, %1, %2 src0_sel:BYTE_0 src1_sel:BYTE_1\n v_cmp_eq_u32_sdwa vcc, %1, %2 src0_sel:BYTE_1 src1_sel:BYTE_1\n v_cmp_eq_u32_sdwa vcc, %1, %2 src0_sel:BYTE_2 src1_sel:BYTE_1\n v_cmp_eq_u32_sdwa vcc, %1, %2 src0_sel:BYTE_3 src1_sel:BYTE_1\n v_cmp_eq_u32_sdwa vcc, %1, %2 src0_sel:BYTE_0 src1_sel:BYTE_2\n v_cmp_eq_u32_sdwa vcc, %1, %2 src0_sel:BYTE_1 src1_sel:BYTE_2\n v_cmp_eq_u32_sdwa vcc, %1, %2 src0_sel:BYTE_2 src1_sel:BYTE_2\n v_cmp_eq_u32_sdwa vcc, %1, %2 src0_sel:BYTE_3 src1_sel:BYTE_2\n")
    // 6: dpp mov dependent chain (8)
    TEST("v_mov_b32_dpp %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf\n s_nop 1\n v_mov_b32_dpp %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf\n s_nop 1\n v_mov_b32_dpp %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf\n s_nop 1\n v_mov_b32_dpp %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf\n s_nop 1\n v_mov_b32_dpp %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf\n s_nop 1\n v_mov_b32_dpp %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf\n s_nop 1\n v_mov_b32_dpp %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf\n s_nop 1\n v_mov_b32_dpp %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf\n s_nop 1\n")
    // 7: independent dpp movs (8)
    TEST("v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %2, %3 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %4, %5 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %6, %7 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %1, %0 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %3, %2 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %5, %4 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %7, %6 wave_shr:1 row_mask:0xf bank_mask:0xf\n")
    // 8: xor_sdwa + min_u32 + sub (VCC-free match), 2 cells interleaved (6 instr) + 2 adds
    TEST("v_xor_b32_sdwa %3, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_1\n v_xor_b32_sdwa %5, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_1\n v_min_u32 %3, 1, %3\n v_min_u32 %5, 1, %5\n v_sub_u32 %6, %6, %3\n v_sub_u32 %7, %7, %5\n v_add_u32 %0, %0, %1\n v_add_u32 %4, %4, %1\n")
    // 9: the fill's cell: cmp+addc (vcc) + max3 + add, chain over 2 cells (8 instr)
    TEST("v_cmp_eq_u32_sdwa vcc, %1, %2 src0_sel:BYTE_0 src1_sel:BYTE_1\n v_addc_co_u32_e32 %3, vcc, %3, %4, vcc\n v_max3_i32 %5, %3, %5, %0\n v_add_u32 %0, %5, %6\n v_cmp_eq_u32_sdwa vcc, %1, %2 src0_sel:BYTE_0 src1_sel:BYTE_2\n v_addc_co_u32_e32 %7, vcc, %7, %4, vcc\n v_max3_i32 %5, %7, %5, %0\n v_add_u32 %0, %5, %6\n")
    if (threadIdx.x == 0) out[63] = a + b + c + d + e + f + g + h;
}

int main() {
    unsigned long long *d, h[64];
    (void)hipMalloc(&d, 64 * 8);
    const int n = 1000;
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, n);
        (void)hipDeviceSynchronize();
    }
    (void)hipMemcpy(h, d, 64 * 8, hipMemcpyDeviceToHost);
    const char *names[] = {"indep add", "dep add", "dep max3", "cmp->vcc->addc x4", "cmp->sgpr x2 ->addc_e64",
                           "indep cmp_sdwa", "dep dpp (+s_nop1)", "indep dpp", "xor_sdwa/min/sub (vcc-free)",
                           "fill cell x2 (cmp,addc,max3,add)"};
    for (int i = 0; i < 10; ++i)
        printf("%-36s %6.2f shader-clk per instr (s_memtime ticks %llu)\n", names[i],
               (double)h[i] / (n * 64.0 * 8.0), h[i]);
    return 0;
}
