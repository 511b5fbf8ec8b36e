// issue_probe4.hip -- issue rates of VALU forms with a wave-uniform (SGPR)
// operand on gfx950: VOP2 v_xor_b32 with an SGPR src0, v_bitop3 with the SGPR
// first or last, v_mov from an SGPR, against all-VGPR forms.  8 independent
// instructions per group, 8 waves per SIMD.
//   hipcc -O3 --offload-arch=gfx950 -o tools/ab/issue_probe4 tools/issue_probe4.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define CLOB "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27"
#define G8(I0, I1, I2, I3, I4, I5, I6, I7) I0 "\n" I1 "\n" I2 "\n" I3 "\n" I4 "\n" I5 "\n" I6 "\n" I7 "\n"

template <int K>
__global__ __launch_bounds__(512) void probe(unsigned* out, int iters, unsigned s) {
    for (int i = 0; i < iters; ++i) {
        if (K == 0)   // VOP2, all VGPR
            asm volatile(".rept 32\n" G8("v_xor_b32 v10, v20, v21", "v_xor_b32 v11, v21, v22", "v_xor_b32 v12, v22, v23",
                                         "v_xor_b32 v13, v23, v24", "v_xor_b32 v14, v24, v25", "v_xor_b32 v15, v25, v26",
                                         "v_xor_b32 v16, v26, v27", "v_xor_b32 v17, v27, v20") ".endr\n" ::: CLOB);
        if (K == 1)   // VOP2 with SGPR src0
            asm volatile(".rept 32\n" G8("v_xor_b32 v10, %0, v21", "v_xor_b32 v11, %0, v22", "v_xor_b32 v12, %0, v23",
                                         "v_xor_b32 v13, %0, v24", "v_xor_b32 v14, %0, v25", "v_xor_b32 v15, %0, v26",
                                         "v_xor_b32 v16, %0, v27", "v_xor_b32 v17, %0, v20") ".endr\n" :: "s"(s) : CLOB);
        if (K == 2)   // bitop3, SGPR first
            asm volatile(".rept 32\n" G8("v_bitop3_b32 v10, %0, v21, v22 bitop3:0x96", "v_bitop3_b32 v11, %0, v22, v23 bitop3:0x96",
                                         "v_bitop3_b32 v12, %0, v23, v24 bitop3:0x96", "v_bitop3_b32 v13, %0, v24, v25 bitop3:0x96",
                                         "v_bitop3_b32 v14, %0, v25, v26 bitop3:0x96", "v_bitop3_b32 v15, %0, v26, v27 bitop3:0x96",
                                         "v_bitop3_b32 v16, %0, v27, v20 bitop3:0x96", "v_bitop3_b32 v17, %0, v20, v21 bitop3:0x96")
                         ".endr\n" :: "s"(s) : CLOB);
        if (K == 3)   // bitop3, all VGPR
            asm volatile(".rept 32\n" G8("v_bitop3_b32 v10, v27, v21, v22 bitop3:0x96", "v_bitop3_b32 v11, v20, v22, v23 bitop3:0x96",
                                         "v_bitop3_b32 v12, v21, v23, v24 bitop3:0x96", "v_bitop3_b32 v13, v22, v24, v25 bitop3:0x96",
                                         "v_bitop3_b32 v14, v23, v25, v26 bitop3:0x96", "v_bitop3_b32 v15, v24, v26, v27 bitop3:0x96",
                                         "v_bitop3_b32 v16, v25, v27, v20 bitop3:0x96", "v_bitop3_b32 v17, v26, v20, v21 bitop3:0x96")
                         ".endr\n" ::: CLOB);
        if (K == 4)   // v_mov from an SGPR
            asm volatile(".rept 32\n" G8("v_mov_b32 v10, %0", "v_mov_b32 v11, %0", "v_mov_b32 v12, %0", "v_mov_b32 v13, %0",
                                         "v_mov_b32 v14, %0", "v_mov_b32 v15, %0", "v_mov_b32 v16, %0", "v_mov_b32 v17, %0")
                         ".endr\n" :: "s"(s) : CLOB);
        if (K == 5)   // VOP2 xor with a literal
            asm volatile(".rept 32\n" G8("v_xor_b32 v10, 0x63636363, v21", "v_xor_b32 v11, 0x63636363, v22", "v_xor_b32 v12, 0x63636363, v23",
                                         "v_xor_b32 v13, 0x63636363, v24", "v_xor_b32 v14, 0x63636363, v25", "v_xor_b32 v15, 0x63636363, v26",
                                         "v_xor_b32 v16, 0x63636363, v27", "v_xor_b32 v17, 0x63636363, v20") ".endr\n" ::: CLOB);
        if (K == 6)   // v_and_b32 / v_or_b32 mix with SGPR src0 (VOP2)
            asm volatile(".rept 32\n" G8("v_and_b32 v10, %0, v21", "v_or_b32 v11, %0, v22", "v_and_b32 v12, %0, v23",
                                         "v_or_b32 v13, %0, v24", "v_and_b32 v14, %0, v25", "v_or_b32 v15, %0, v26",
                                         "v_and_b32 v16, %0, v27", "v_or_b32 v17, %0, v20") ".endr\n" :: "s"(s) : CLOB);
        if (K == 7)   // v_lshrrev_b32 (VOP2) by an inline constant
            asm volatile(".rept 32\n" G8("v_lshrrev_b32 v10, 8, v21", "v_lshrrev_b32 v11, 8, v22", "v_lshrrev_b32 v12, 8, v23",
                                         "v_lshrrev_b32 v13, 8, v24", "v_lshrrev_b32 v14, 8, v25", "v_lshrrev_b32 v15, 8, v26",
                                         "v_lshrrev_b32 v16, 8, v27", "v_lshrrev_b32 v17, 8, v20") ".endr\n" ::: CLOB);
        if (K == 8)   // v_bfe_u32
            asm volatile(".rept 32\n" G8("v_bfe_u32 v10, v21, 8, 8", "v_bfe_u32 v11, v22, 8, 8", "v_bfe_u32 v12, v23, 8, 8",
                                         "v_bfe_u32 v13, v24, 8, 8", "v_bfe_u32 v14, v25, 8, 8", "v_bfe_u32 v15, v26, 8, 8",
                                         "v_bfe_u32 v16, v27, 8, 8", "v_bfe_u32 v17, v20, 8, 8") ".endr\n" ::: CLOB);
        if (K == 9)   // v_and_or_b32 (VOP3, all VGPR)
            asm volatile(".rept 32\n" G8("v_and_or_b32 v10, v27, v21, v22", "v_and_or_b32 v11, v20, v22, v23", "v_and_or_b32 v12, v21, v23, v24",
                                         "v_and_or_b32 v13, v22, v24, v25", "v_and_or_b32 v14, v23, v25, v26", "v_and_or_b32 v15, v24, v26, v27",
                                         "v_and_or_b32 v16, v25, v27, v20", "v_and_or_b32 v17, v26, v20, v21") ".endr\n" ::: CLOB);
    }
    if (threadIdx.x == 0) out[blockIdx.x] = iters;
}

template <class F>
float timeit(F f) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    f();
    hipDeviceSynchronize();
    hipEventRecord(a);
    f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    unsigned* out;
    hipMalloc(&out, 4 * 65536);
    const int blocks = cus * 4, iters = 2000;
    const double instr = (double)blocks * 8 * iters * 32 * 8;
    auto rep = [&](const char* name, float ms) {
        printf("%-40s %8.3f ms  %6.1f lane-ops/clk/CU (2.4 GHz)\n", name, ms, instr * 64 / (ms * 1e-3) / 2.4e9 / cus);
    };
    const unsigned s = 0x0f0f0f0fu;
    for (int r = 0; r < 2; ++r) {
        rep("v_xor_b32 (VOP2) all VGPR", timeit([&] { probe<0><<<blocks, 512>>>(out, iters, s); }));
        rep("v_xor_b32 (VOP2) SGPR src0", timeit([&] { probe<1><<<blocks, 512>>>(out, iters, s); }));
        rep("v_bitop3 SGPR first operand", timeit([&] { probe<2><<<blocks, 512>>>(out, iters, s); }));
        rep("v_bitop3 all VGPR", timeit([&] { probe<3><<<blocks, 512>>>(out, iters, s); }));
        rep("v_mov_b32 from SGPR", timeit([&] { probe<4><<<blocks, 512>>>(out, iters, s); }));
        rep("v_xor_b32 (VOP2) literal src0", timeit([&] { probe<5><<<blocks, 512>>>(out, iters, s); }));
        rep("v_and/v_or (VOP2) SGPR src0", timeit([&] { probe<6><<<blocks, 512>>>(out, iters, s); }));
        rep("v_lshrrev_b32 const", timeit([&] { probe<7><<<blocks, 512>>>(out, iters, s); }));
        rep("v_bfe_u32 const", timeit([&] { probe<8><<<blocks, 512>>>(out, iters, s); }));
        rep("v_and_or_b32 all VGPR", timeit([&] { probe<9><<<blocks, 512>>>(out, iters, s); }));
    }
    return 0;
}
