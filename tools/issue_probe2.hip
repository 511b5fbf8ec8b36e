// issue_probe2.hip -- VALU issue rate on gfx950 for the instruction shapes of
// the bitsliced AES (aes_bs8.h): v_bitop3 with three VGPR sources (same or
// different register banks), with an SGPR source, VOP2 v_xor, and the
// Boyar-Peralta S-box itself, at 1..8 waves per SIMD.  Not part of libtlsgpu.
//   hipcc -O3 --offload-arch=gfx950 -I tlslite-ng_amd/csrc -o issue_probe2 tools/issue_probe2.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "aes_bs.h"

// MODE 0: bitop3 x[c] = f(x[c], y, z)  (y, z shared)
// MODE 1: bitop3 x[c] = f(x[c], x[c+1], x[c+2])  (ring of chains)
// MODE 2: bitop3 x[c] = f(x[c], y, s)  (s an SGPR)
// MODE 3: v_xor_b32 x[c] ^= y
template <int MODE, int CH, int B, int R>
__global__ void probe(uint32_t* out, uint64_t* cyc, uint32_t seed) {
    uint32_t x[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = seed + threadIdx.x * 7 + c;
    const uint32_t y = seed * 3 + threadIdx.x, z = seed ^ threadIdx.x;
    const uint32_t sg = __builtin_amdgcn_readfirstlane(seed * 5);
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int b = 0; b < B; ++b)
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                if (MODE == 0)
                    asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x[c]) : "v"(y), "v"(z));
                else if (MODE == 1)
                    asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96"
                                 : "+v"(x[c]) : "v"(x[(c + 1) % CH]), "v"(x[(c + 2) % CH]));
                else if (MODE == 2)
                    asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x[c]) : "v"(y), "s"(sg));
                else
                    asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
            }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) acc ^= x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

// The S-box circuit on NS independent rows per iteration (compiler-scheduled).
template <int NS, int R>
__global__ void sbox_probe(uint32_t* out, uint64_t* cyc, uint32_t seed) {
    uint32_t x[NS][8];
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int b = 0; b < 8; ++b) x[s][b] = seed * (b + 1) + threadIdx.x * 13 + s;
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int s = 0; s < NS; ++s) tg::bs::sbox(x[s]);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t acc = 0;
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int b = 0; b < 8; ++b) acc ^= x[s][b];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

static void report(const char* name, int w, float ms, const uint64_t* h, int nw, double instr) {
    double mean = 0;
    for (int i = 0; i < nw; ++i) mean += h[i];
    mean /= nw;
    const double lane_ops = instr * 64 * nw;
    printf("%-34s waves/SIMD %d: %.3f ms, %5.1f cyc/instr per wave, %6.1f lane-ops/clk/CU @2.4GHz\n", name, w,
           ms, mean / instr, lane_ops / (ms * 1e-3 * 2.4e9 * 256));
}

template <class K>
static void launch(const char* name, K kern, int w, double instr, uint32_t* d_out, uint64_t* d_cyc) {
    const int blocks = 256 * w, threads = 256;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, d_out, d_cyc, 1u);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, d_out, d_cyc, 2u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    static uint64_t h[256 * 8 * 4];
    hipMemcpy(h, d_cyc, blocks * 4 * 8, hipMemcpyDeviceToHost);
    report(name, w, ms, h, blocks * 4, instr);
}

int main() {
    uint32_t* d_out;
    uint64_t* d_cyc;
    hipMalloc(&d_out, 256 * 8 * 256 * 4);
    hipMalloc(&d_cyc, 256 * 8 * 4 * 8);
    const int ws[] = {1, 2, 4, 6, 8};
    for (int w : ws) {
        launch("bitop3 vvv shared y,z ILP8", probe<0, 8, 64, 256>, w, 8.0 * 64 * 256, d_out, d_cyc);
        launch("bitop3 vvv ring ILP8", probe<1, 8, 64, 256>, w, 8.0 * 64 * 256, d_out, d_cyc);
        launch("bitop3 vvs ILP8", probe<2, 8, 64, 256>, w, 8.0 * 64 * 256, d_out, d_cyc);
        launch("xor vv ILP8", probe<3, 8, 64, 256>, w, 8.0 * 64 * 256, d_out, d_cyc);
        launch("bitop3 vvv shared ILP2", probe<0, 2, 256, 256>, w, 2.0 * 256 * 256, d_out, d_cyc);
        launch("sbox x1 (84 gates)", sbox_probe<1, 512>, w, 84.0 * 512, d_out, d_cyc);
        launch("sbox x2", sbox_probe<2, 256>, w, 84.0 * 2 * 256, d_out, d_cyc);
        launch("sbox x4", sbox_probe<4, 128>, w, 84.0 * 4 * 128, d_out, d_cyc);
    }
    return 0;
}
