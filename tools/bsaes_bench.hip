// bsaes_bench.hip -- throughput probe of the bitsliced AES-CTR core
// (csrc/aes_bs.h): each lane produces NCH chunks of 32 keystream blocks and
// folds them into one accumulator; lane 0..63 results are checked on the host
// against the same core run on the CPU.  Not part of libtlsgpu.
//   hipcc -O3 --offload-arch=gfx950 -I tlslite-ng_amd/csrc -o bsaes_bench tools/bsaes_bench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <type_traits>
#include "aes_bs.h"

template <int NR, int NCH, int SCHED, int W, int MASKS>
__global__ __launch_bounds__(256, W) void bs_kernel(const uint32_t* __restrict__ rkp,
                                                 const uint32_t* __restrict__ s1, uint4* out) {
    using KM = typename std::conditional<MASKS != 0, tg::bs::BsKeyMasks, tg::bs::BsKey>::type;
    const KM key{MASKS ? rkp + 4 * (NR + 2) : rkp};
    const uint32_t rk0w = rkp[4 * (NR + 1) + 3];
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t s1w[3] = {s1[3 * gid], s1[3 * gid + 1], s1[3 * gid + 2]};
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (int j = 0; j < NCH; ++j) {
        uint32_t w[4][32];
        tg::bs::ctr32<NR, SCHED & 1, KM, 2, (SCHED & 2) != 0>(key, rk0w, s1w, 2u + 32u * j, w);
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            acc.x ^= w[0][i] + i; acc.y ^= w[1][i]; acc.z ^= w[2][i]; acc.w ^= w[3][i];
        }
    }
    out[gid] = acc;
}

int main(int argc, char** argv) {
    const int nthreads = argc > 1 ? atoi(argv[1]) : 256 * 1024;
    constexpr int NR = 10, NCH = 8;
    static uint32_t h_rk[4 * 12 + 1408];   // rk' words, rk0, then the plane masks
    srand(1);
    for (int i = 0; i < 4 * 12; ++i) h_rk[i] = (uint32_t)rand() * 2654435761u;
    for (int r = 0; r <= NR; ++r)
        for (int k = 0; k < 16; ++k)
            for (int b = 0; b < 8; ++b)
                h_rk[4 * (NR + 2) + (16 * r + k) * 8 + b] = tg::bs::bitmask(h_rk[4 * r + k / 4], 8 * (k % 4) + b);
    uint32_t* h_s1 = (uint32_t*)malloc(12 * (size_t)nthreads);
    for (int i = 0; i < 3 * nthreads; ++i) h_s1[i] = (uint32_t)rand() * 40503u ^ i;
    uint32_t *d_rk, *d_s1; uint4* d_out;
    hipMalloc(&d_rk, sizeof h_rk); hipMalloc(&d_s1, 12 * (size_t)nthreads);
    hipMalloc(&d_out, 16 * (size_t)nthreads);
    hipMemcpy(d_rk, h_rk, sizeof h_rk, hipMemcpyHostToDevice);
    hipMemcpy(d_s1, h_s1, 12 * (size_t)nthreads, hipMemcpyHostToDevice);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    int dev; hipGetDevice(&dev); hipDeviceProp_t p; hipGetDeviceProperties(&p, dev);
    uint4* h_out = (uint4*)malloc(16 * (size_t)nthreads);
    const tg::bs::BsKey key{h_rk};
    int fails = 0;
    auto run = [&](const char* name, void (*kern)(const uint32_t*, const uint32_t*, uint4*)) {
        hipLaunchKernelGGL(kern, dim3(nthreads / 256), dim3(256), 0, 0, d_rk, d_s1, d_out);
        hipDeviceSynchronize();
        float best = 1e9;
        for (int it = 0; it < 5; ++it) {
            hipEventRecord(a);
            hipLaunchKernelGGL(kern, dim3(nthreads / 256), dim3(256), 0, 0, d_rk, d_s1, d_out);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
        }
        hipMemcpy(h_out, d_out, 16 * (size_t)nthreads, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int g = 0; g < 64; ++g) {
            uint4 acc = make_uint4(0, 0, 0, 0);
            for (int j = 0; j < NCH; ++j) {
                uint32_t w[4][32];
                tg::bs::ctr32<NR>(key, h_rk[4 * (NR + 1) + 3], h_s1 + 3 * g, 2u + 32u * j, w);
                for (int i = 0; i < 32; ++i) { acc.x ^= w[0][i] + i; acc.y ^= w[1][i]; acc.z ^= w[2][i]; acc.w ^= w[3][i]; }
            }
            if (memcmp(&acc, &h_out[g], 16)) ++bad;
        }
        fails += bad != 0;
        const double blocks = (double)nthreads * NCH * 32;
        printf("%-28s %d lanes x %d chunks: %.3f ms, %7.1f GB/s keystream, %.2f CU-clk/block @2.4GHz, host check %s\n",
               name, nthreads, NCH, best, blocks * 16 / best / 1e6,
               best * 1e-3 * 2.4e9 * p.multiProcessorCount / blocks, bad ? "FAIL" : "ok");
    };
    run("sbox-all sched0 w2", bs_kernel<NR, NCH, 0, 2, 0>);
    run("by-column sched1 w2", bs_kernel<NR, NCH, 1, 2, 0>);
    run("sbox-all sched0 w2 masks", bs_kernel<NR, NCH, 0, 2, 1>);
    run("by-column sched1 w2 masks", bs_kernel<NR, NCH, 1, 2, 1>);
    run("sbox-all fenced w2 masks", bs_kernel<NR, NCH, 2, 2, 1>);
    run("sbox-all fenced w3 masks", bs_kernel<NR, NCH, 2, 3, 1>);
    return fails != 0;
}
