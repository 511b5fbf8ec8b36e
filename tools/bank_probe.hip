// bank_probe.hip -- does a VALU instruction whose two VGPR sources sit in the
// same register bank (v_n and v_m with n % 4 == m % 4) issue slower on gfx950?
// Each wave runs 64 x 32 independent instructions of one kind with either
// same-bank or different-bank source pairs; the kernel time at 8 waves per
// SIMD gives the issue rate.  hipcc -O3 --offload-arch=gfx950 -o tools/bank_probe tools/bank_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CLOB "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", \
             "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33"
// (the probes only read v20..v31: their values do not matter)

// 8 independent instructions: dst v10..v17 (rotating), sources from v20..v27
// same bank: (v20, v24) (v21, v25) (v22, v26) (v23, v27): n and n + 4
// diff bank: (v20, v21) (v21, v22) (v22, v23) (v23, v24)
#define BODY(OP, A0, B0, A1, B1, A2, B2, A3, B3)                    \
    OP " v10, " A0 ", " B0 "\n" OP " v11, " A1 ", " B1 "\n"         \
    OP " v12, " A2 ", " B2 "\n" OP " v13, " A3 ", " B3 "\n"         \
    OP " v14, " A0 ", " B0 "\n" OP " v15, " A1 ", " B1 "\n"         \
    OP " v16, " A2 ", " B2 "\n" OP " v17, " A3 ", " B3 "\n"

template <int K>
__global__ __launch_bounds__(512) void probe(unsigned* out, int iters) {
    for (int i = 0; i < iters; ++i) {
        if (K == 0)
            asm volatile(".rept 32\n" BODY("v_xor_b32", "v20", "v24", "v21", "v25", "v22", "v26", "v23", "v27") ".endr\n" ::: CLOB);
        if (K == 1)
            asm volatile(".rept 32\n" BODY("v_xor_b32", "v20", "v21", "v21", "v22", "v22", "v23", "v23", "v24") ".endr\n" ::: CLOB);
        if (K == 2)
            asm volatile(".rept 32\n" BODY("v_add_u32", "v20", "v24", "v21", "v25", "v22", "v26", "v23", "v27") ".endr\n" ::: CLOB);
        if (K == 3)
            asm volatile(".rept 32\n" BODY("v_add_u32", "v20", "v21", "v21", "v22", "v22", "v23", "v23", "v24") ".endr\n" ::: CLOB);
    }
    if (threadIdx.x == 0) out[blockIdx.x] = iters;
}

// v_alignbit_b32 d, a, b, s with a, b distinct: same bank vs different
template <int K>
__global__ __launch_bounds__(512) void probe3(unsigned* out, int iters) {
    for (int i = 0; i < iters; ++i) {
        if (K == 0)
            asm volatile(".rept 32\n"
                         "v_alignbit_b32 v10, v20, v24, 16\n v_alignbit_b32 v11, v21, v25, 16\n"
                         "v_alignbit_b32 v12, v22, v26, 16\n v_alignbit_b32 v13, v23, v27, 16\n"
                         "v_alignbit_b32 v14, v20, v24, 16\n v_alignbit_b32 v15, v21, v25, 16\n"
                         "v_alignbit_b32 v16, v22, v26, 16\n v_alignbit_b32 v17, v23, v27, 16\n"
                         ".endr\n" ::: CLOB);
        if (K == 1)
            asm volatile(".rept 32\n"
                         "v_alignbit_b32 v10, v20, v21, 16\n v_alignbit_b32 v11, v21, v22, 16\n"
                         "v_alignbit_b32 v12, v22, v23, 16\n v_alignbit_b32 v13, v23, v24, 16\n"
                         "v_alignbit_b32 v14, v20, v21, 16\n v_alignbit_b32 v15, v21, v22, 16\n"
                         "v_alignbit_b32 v16, v22, v23, 16\n v_alignbit_b32 v17, v23, v24, 16\n"
                         ".endr\n" ::: CLOB);
        if (K == 2)   // rotation form: both sources the same register
            asm volatile(".rept 32\n"
                         "v_alignbit_b32 v10, v20, v20, 16\n v_alignbit_b32 v11, v21, v21, 16\n"
                         "v_alignbit_b32 v12, v22, v22, 16\n v_alignbit_b32 v13, v23, v23, 16\n"
                         "v_alignbit_b32 v14, v24, v24, 16\n v_alignbit_b32 v15, v25, v25, 16\n"
                         "v_alignbit_b32 v16, v26, v26, 16\n v_alignbit_b32 v17, v27, v27, 16\n"
                         ".endr\n" ::: CLOB);
    }
    if (threadIdx.x == 0) out[blockIdx.x] = iters;
}

// v_perm_b32 / v_bitop3_b32 with the third operand in an SGPR vs a VGPR
template <int K>
__global__ __launch_bounds__(512) void probe_sop(unsigned* out, int iters, unsigned sel) {
    for (int i = 0; i < iters; ++i) {
        if (K == 0)
            asm volatile(".rept 32\n"
                         "v_perm_b32 v10, v20, v21, %0\n v_perm_b32 v11, v21, v22, %0\n"
                         "v_perm_b32 v12, v22, v23, %0\n v_perm_b32 v13, v23, v24, %0\n"
                         "v_perm_b32 v14, v24, v25, %0\n v_perm_b32 v15, v25, v26, %0\n"
                         "v_perm_b32 v16, v26, v27, %0\n v_perm_b32 v17, v27, v20, %0\n"
                         ".endr\n" :: "s"(sel) : CLOB);
        if (K == 1)
            asm volatile("v_mov_b32 v28, %0\n.rept 32\n"
                         "v_perm_b32 v10, v20, v21, v28\n v_perm_b32 v11, v21, v22, v28\n"
                         "v_perm_b32 v12, v22, v23, v28\n v_perm_b32 v13, v23, v24, v28\n"
                         "v_perm_b32 v14, v24, v25, v28\n v_perm_b32 v15, v25, v26, v28\n"
                         "v_perm_b32 v16, v26, v27, v28\n v_perm_b32 v17, v27, v20, v28\n"
                         ".endr\n" :: "s"(sel) : CLOB, "v28");
        if (K == 2)
            asm volatile(".rept 32\n"
                         "v_bitop3_b32 v10, v20, v21, %0 bitop3:0xca\n v_bitop3_b32 v11, v21, v22, %0 bitop3:0xca\n"
                         "v_bitop3_b32 v12, v22, v23, %0 bitop3:0xca\n v_bitop3_b32 v13, v23, v24, %0 bitop3:0xca\n"
                         "v_bitop3_b32 v14, v24, v25, %0 bitop3:0xca\n v_bitop3_b32 v15, v25, v26, %0 bitop3:0xca\n"
                         "v_bitop3_b32 v16, v26, v27, %0 bitop3:0xca\n v_bitop3_b32 v17, v27, v20, %0 bitop3:0xca\n"
                         ".endr\n" :: "s"(sel) : CLOB);
        if (K == 3)
            asm volatile("v_mov_b32 v28, %0\n.rept 32\n"
                         "v_bitop3_b32 v10, v20, v21, v28 bitop3:0xca\n v_bitop3_b32 v11, v21, v22, v28 bitop3:0xca\n"
                         "v_bitop3_b32 v12, v22, v23, v28 bitop3:0xca\n v_bitop3_b32 v13, v23, v24, v28 bitop3:0xca\n"
                         "v_bitop3_b32 v14, v24, v25, v28 bitop3:0xca\n v_bitop3_b32 v15, v25, v26, v28 bitop3:0xca\n"
                         "v_bitop3_b32 v16, v26, v27, v28 bitop3:0xca\n v_bitop3_b32 v17, v27, v20, v28 bitop3:0xca\n"
                         ".endr\n" :: "s"(sel) : CLOB, "v28");
    }
    if (threadIdx.x == 0) out[blockIdx.x] = iters;
}

// v_bitop3_b32 with three VGPR sources (the S-box gates of aes_bs_sbox.h):
// K 0 three banks, 1 two sources in one bank, 2 all three in one bank
template <int K>
__global__ __launch_bounds__(512) void probe_b3(unsigned* out, int iters) {
    for (int i = 0; i < iters; ++i) {
        if (K == 0)
            asm volatile(".rept 32\n"
                         "v_bitop3_b32 v10, v20, v21, v22 bitop3:0x96\n v_bitop3_b32 v11, v21, v22, v23 bitop3:0x96\n"
                         "v_bitop3_b32 v12, v22, v23, v24 bitop3:0x96\n v_bitop3_b32 v13, v23, v24, v25 bitop3:0x96\n"
                         "v_bitop3_b32 v14, v24, v25, v26 bitop3:0x96\n v_bitop3_b32 v15, v25, v26, v27 bitop3:0x96\n"
                         "v_bitop3_b32 v16, v26, v27, v28 bitop3:0x96\n v_bitop3_b32 v17, v27, v28, v29 bitop3:0x96\n"
                         ".endr\n" ::: CLOB);
        if (K == 1)
            asm volatile(".rept 32\n"
                         "v_bitop3_b32 v10, v20, v24, v21 bitop3:0x96\n v_bitop3_b32 v11, v21, v25, v22 bitop3:0x96\n"
                         "v_bitop3_b32 v12, v22, v26, v23 bitop3:0x96\n v_bitop3_b32 v13, v23, v27, v24 bitop3:0x96\n"
                         "v_bitop3_b32 v14, v24, v28, v25 bitop3:0x96\n v_bitop3_b32 v15, v25, v29, v26 bitop3:0x96\n"
                         "v_bitop3_b32 v16, v26, v30, v27 bitop3:0x96\n v_bitop3_b32 v17, v27, v31, v28 bitop3:0x96\n"
                         ".endr\n" ::: CLOB);
        if (K == 2)
            asm volatile(".rept 32\n"
                         "v_bitop3_b32 v10, v20, v24, v28 bitop3:0x96\n v_bitop3_b32 v11, v21, v25, v29 bitop3:0x96\n"
                         "v_bitop3_b32 v12, v22, v26, v30 bitop3:0x96\n v_bitop3_b32 v13, v23, v27, v31 bitop3:0x96\n"
                         "v_bitop3_b32 v14, v20, v24, v28 bitop3:0x96\n v_bitop3_b32 v15, v21, v25, v29 bitop3:0x96\n"
                         "v_bitop3_b32 v16, v22, v26, v30 bitop3:0x96\n v_bitop3_b32 v17, v23, v27, v31 bitop3:0x96\n"
                         ".endr\n" ::: CLOB);
    }
    if (threadIdx.x == 0) out[blockIdx.x] = iters;
}

// Dependent chains: C independent chains of v_bitop3 (VGPR sources, three
// banks) per wave, each instruction reading its chain's previous result;
// C = 1 / 2 / 4 / 8.  With W waves per SIMD this shows how much independent
// work per wave the VALU needs to issue at its rate.
template <int C>
__global__ __launch_bounds__(256) void probe_chain(unsigned* out, int iters) {
    for (int i = 0; i < iters; ++i) {
        if (C == 1)
            asm volatile(".rept 256\n v_bitop3_b32 v10, v10, v21, v22 bitop3:0x96\n .endr\n" ::: CLOB);
        if (C == 2)
            asm volatile(".rept 128\n v_bitop3_b32 v10, v10, v21, v22 bitop3:0x96\n"
                         " v_bitop3_b32 v11, v11, v22, v23 bitop3:0x96\n .endr\n" ::: CLOB);
        if (C == 4)
            asm volatile(".rept 64\n v_bitop3_b32 v10, v10, v21, v22 bitop3:0x96\n"
                         " v_bitop3_b32 v11, v11, v22, v23 bitop3:0x96\n"
                         " v_bitop3_b32 v12, v12, v23, v24 bitop3:0x96\n"
                         " v_bitop3_b32 v13, v13, v24, v25 bitop3:0x96\n .endr\n" ::: CLOB);
        if (C == 8)
            asm volatile(".rept 32\n v_bitop3_b32 v10, v10, v21, v22 bitop3:0x96\n"
                         " v_bitop3_b32 v11, v11, v22, v23 bitop3:0x96\n"
                         " v_bitop3_b32 v12, v12, v23, v24 bitop3:0x96\n"
                         " v_bitop3_b32 v13, v13, v24, v25 bitop3:0x96\n"
                         " v_bitop3_b32 v14, v14, v25, v26 bitop3:0x96\n"
                         " v_bitop3_b32 v15, v15, v26, v27 bitop3:0x96\n"
                         " v_bitop3_b32 v16, v16, v27, v28 bitop3:0x96\n"
                         " v_bitop3_b32 v17, v17, v28, v29 bitop3:0x96\n .endr\n" ::: CLOB);
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
    const int blocks = cus * 4, iters = 2000;   // 4 x 512 threads = 32 waves per CU = 8 per SIMD
    const double instr = (double)blocks * 8 * iters * 32 * 8;   // wave instructions
    auto rep = [&](const char* name, float ms) {
        // lane-ops per clock per CU at the nominal 2.4 GHz
        printf("%-34s %8.3f ms  %6.1f lane-ops/clk/CU (2.4 GHz)\n", name, ms,
               instr * 64 / (ms * 1e-3) / 2.4e9 / cus);
    };
    if (getenv("BANK_PROBE_B3")) {   // the 3-source and dependency-chain probes only
        for (int r = 0; r < 2; ++r) {
            rep("v_bitop3 3 VGPRs, three banks", timeit([&] { probe_b3<0><<<blocks, 512>>>(out, iters); }));
            rep("v_bitop3 3 VGPRs, two in one bank", timeit([&] { probe_b3<1><<<blocks, 512>>>(out, iters); }));
            rep("v_bitop3 3 VGPRs, all in one bank", timeit([&] { probe_b3<2><<<blocks, 512>>>(out, iters); }));
            // 256-thread workgroups: W waves per SIMD = blocks per CU
            for (int w : {1, 2, 4, 8}) {
                const double ins = (double)cus * w * 4 * iters * 256;   // wave instructions
                auto rc = [&](const char* name, float ms) {
                    printf("%-22s %d waves/SIMD %8.3f ms  %6.1f lane-ops/clk/CU (2.4 GHz)\n", name, w, ms,
                           ins * 64 / (ms * 1e-3) / 2.4e9 / cus);
                };
                rc("bitop3 chains x1", timeit([&] { probe_chain<1><<<cus * w, 256>>>(out, iters); }));
                rc("bitop3 chains x2", timeit([&] { probe_chain<2><<<cus * w, 256>>>(out, iters); }));
                rc("bitop3 chains x4", timeit([&] { probe_chain<4><<<cus * w, 256>>>(out, iters); }));
                rc("bitop3 chains x8", timeit([&] { probe_chain<8><<<cus * w, 256>>>(out, iters); }));
            }
        }
        return 0;
    }
    for (int r = 0; r < 2; ++r) {
        rep("v_xor_b32 same-bank sources", timeit([&] { probe<0><<<blocks, 512>>>(out, iters); }));
        rep("v_xor_b32 different-bank sources", timeit([&] { probe<1><<<blocks, 512>>>(out, iters); }));
        rep("v_add_u32 same-bank sources", timeit([&] { probe<2><<<blocks, 512>>>(out, iters); }));
        rep("v_add_u32 different-bank sources", timeit([&] { probe<3><<<blocks, 512>>>(out, iters); }));
        rep("v_alignbit same-bank sources", timeit([&] { probe3<0><<<blocks, 512>>>(out, iters); }));
        rep("v_alignbit different-bank sources", timeit([&] { probe3<1><<<blocks, 512>>>(out, iters); }));
        rep("v_alignbit one source twice", timeit([&] { probe3<2><<<blocks, 512>>>(out, iters); }));
        rep("v_perm selector in an SGPR", timeit([&] { probe_sop<0><<<blocks, 512>>>(out, iters, 0x05040100u); }));
        rep("v_perm selector in a VGPR", timeit([&] { probe_sop<1><<<blocks, 512>>>(out, iters, 0x05040100u); }));
        rep("v_bitop3 third operand in an SGPR", timeit([&] { probe_sop<2><<<blocks, 512>>>(out, iters, 0x0f0f0f0fu); }));
        rep("v_bitop3 third operand in a VGPR", timeit([&] { probe_sop<3><<<blocks, 512>>>(out, iters, 0x0f0f0f0fu); }));
    }
    return 0;
}
