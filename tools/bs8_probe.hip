// bs8_probe.hip -- throughput probe of the 8-block bitsliced AES core
// (csrc/aes_bs8.h): each lane runs NB batches of 8 keystream blocks from its
// own first-state planes and folds them into one accumulator (no payload, no
// GHASH), for several occupancies.  Lanes 0..63 are checked on the host.
// Not part of libtlsgpu.
//   hipcc -O3 --offload-arch=gfx950 -I tlslite-ng_amd/csrc -o bs8_probe tools/bs8_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "aes_bs8.h"

constexpr int NR = 10, NB = 16;

// Ablations of one batch (8 blocks per lane), for cost attribution:
// MODE 1: the NR-1 middle rounds only (S-boxes + mix_round);
// MODE 2: as 1 without the round-key XORs (a zero-key functor: constants);
// MODE 3: as 1 with the round keys held in VGPRs (opaque copies);
// MODE 4: S-boxes only (4 per round);
// MODE 5: mix_round only;
// MODE 6: to_blocks only.
struct ZeroKey {
    __device__ uint32_t operator()(int, int, int) const { return 0; }
};
struct VKey {
    uint32_t v[32];
    __device__ uint32_t operator()(int, int i, int b) const { return v[8 * i + b]; }
};

template <int MODE, int W>
__global__ __launch_bounds__(256, W) void k_abl(const uint32_t* __restrict__ planes,
                                                const uint32_t* __restrict__ rec, uint4* out) {
    const tg::bs8::KeyPlanes km{planes};
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t s[4][8];
#pragma unroll
    for (int e = 0; e < 32; ++e) s[e >> 3][e & 7] = rec[32 * (gid >> 3) + e];
    VKey vk;
    if (MODE == 3) {
#pragma unroll
        for (int e = 0; e < 32; ++e) {
            vk.v[e] = planes[e];
            asm volatile("" : "+v"(vk.v[e]));
        }
    }
    for (uint32_t beta = 0; beta < NB; ++beta) {
        if (MODE == 6) {
            uint32_t w[4][8];
            tg::bs8::to_blocks(s, w);
#pragma unroll
            for (int e = 0; e < 32; ++e) s[e >> 3][e & 7] = w[e & 3][e >> 2] + e;
            continue;
        }
#pragma unroll 1
        for (int r = 1; r < NR + 1; ++r) {
            if (MODE != 5) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    tg::bs::sbox(s[i]);
                    TG_BS8_FENCE();
                }
            }
            if (MODE == 1 || MODE == 5) tg::bs8::mix_round(s, km, r);
            if (MODE == 2) tg::bs8::mix_round(s, ZeroKey{}, r);
            if (MODE == 3) tg::bs8::mix_round(s, vk, r);
        }
    }
    uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int e = 0; e < 32; e += 4) {
        acc.x ^= s[e >> 3][e & 7]; acc.y ^= s[e >> 3][(e & 7) + 1];
        acc.z ^= s[e >> 3][(e & 7) + 2]; acc.w ^= s[e >> 3][(e & 7) + 3];
    }
    out[gid] = acc;
}

template <int W, int T>
__global__ __launch_bounds__(T, W) void k_bs8(const uint32_t* __restrict__ planes,
                                              const uint32_t* __restrict__ rec, uint4* out) {
    const tg::bs8::KeyPlanes km{planes};
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t lane[6], kmask;
    tg::bs8::lane_consts(2u + (gid & 7u), lane, kmask);
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (uint32_t beta = 0; beta < NB; ++beta) {
        uint32_t s[4][8], w[4][8];
#pragma unroll
        for (int e = 0; e < 32; ++e) s[e >> 3][e & 7] = rec[32 * (gid >> 3) + e];
#pragma unroll
        for (int b = 0; b < 6; ++b) s[3][b] ^= lane[b];
        tg::bs8::ctr_planes<6, 16>(s, kmask, beta);
        tg::bs8::encrypt<NR>(s, km, w);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            acc.x ^= w[0][j] + j; acc.y ^= w[1][j]; acc.z ^= w[2][j]; acc.w ^= w[3][j];
        }
    }
    out[gid] = acc;
}

int main(int argc, char** argv) {
    const int nthreads = argc > 1 ? atoi(argv[1]) : 256 * 2048;
    static uint32_t h_planes[32 * (NR + 1)];
    srand(7);
    uint32_t rkw[60];
    for (int i = 0; i < 60; ++i) rkw[i] = (uint32_t)rand() * 2654435761u;
    for (int e = 0; e < 32 * (NR + 1); ++e) h_planes[e] = tg::bs8::mask_word(rkw, e);
    const size_t nrec = nthreads / 8;
    uint32_t* h_rec = (uint32_t*)malloc(4 * 32 * nrec);
    for (size_t i = 0; i < 32 * nrec; ++i) h_rec[i] = (uint32_t)rand() * 40503u ^ (uint32_t)i;
    uint32_t *d_planes, *d_rec;
    uint4* d_out;
    hipMalloc(&d_planes, sizeof h_planes);
    hipMalloc(&d_rec, 4 * 32 * nrec);
    hipMalloc(&d_out, 16 * (size_t)nthreads);
    hipMemcpy(d_planes, h_planes, sizeof h_planes, hipMemcpyHostToDevice);
    hipMemcpy(d_rec, h_rec, 4 * 32 * nrec, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    int dev;
    hipGetDevice(&dev);
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, dev);
    uint4* h_out = (uint4*)malloc(16 * (size_t)nthreads);
    int fails = 0;
    auto run = [&](const char* name, void (*kern)(const uint32_t*, const uint32_t*, uint4*), int T) {
        hipLaunchKernelGGL(kern, dim3(nthreads / T), dim3(T), 0, 0, d_planes, d_rec, d_out);
        hipDeviceSynchronize();
        float best = 1e9;
        for (int it = 0; it < 5; ++it) {
            hipEventRecord(a);
            hipLaunchKernelGGL(kern, dim3(nthreads / T), dim3(T), 0, 0, d_planes, d_rec, d_out);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (ms < best) best = ms;
        }
        hipMemcpy(h_out, d_out, 16 * (size_t)nthreads, hipMemcpyDeviceToHost);
        int bad = 0;
        const tg::bs8::KeyPlanes km{h_planes};
        for (int g = 0; g < 64; ++g) {
            uint32_t lane[6], kmask;
            tg::bs8::lane_consts(2u + (g & 7u), lane, kmask);
            uint4 acc = make_uint4(0, 0, 0, 0);
            for (uint32_t beta = 0; beta < NB; ++beta) {
                uint32_t s[4][8], w[4][8];
                for (int e = 0; e < 32; ++e) s[e >> 3][e & 7] = h_rec[32 * (g >> 3) + e];
                for (int bb = 0; bb < 6; ++bb) s[3][bb] ^= lane[bb];
                tg::bs8::ctr_planes<6, 16>(s, kmask, beta);
                tg::bs8::encrypt<NR>(s, km, w);
                for (int j = 0; j < 8; ++j) {
                    acc.x ^= w[0][j] + j; acc.y ^= w[1][j]; acc.z ^= w[2][j]; acc.w ^= w[3][j];
                }
            }
            if (memcmp(&acc, &h_out[g], 16)) ++bad;
        }
        fails += bad != 0;
        const double blocks = (double)nthreads * NB * 8;
        printf("%-22s %d lanes x %d batches: %.3f ms, %7.1f GB/s keystream, %.2f CU-clk/block @2.4GHz, host %s\n",
               name, nthreads, NB, best, blocks * 16 / best / 1e6,
               best * 1e-3 * 2.4e9 * p.multiProcessorCount / blocks, bad ? "FAIL" : "ok");
    };
    run("bs8 256thr W=2", k_bs8<2, 256>, 256);
    run("bs8 256thr W=4", k_bs8<4, 256>, 256);
    run("bs8 256thr W=5", k_bs8<5, 256>, 256);
    auto abl = [&](const char* name, void (*kern)(const uint32_t*, const uint32_t*, uint4*)) {
        hipLaunchKernelGGL(kern, dim3(nthreads / 256), dim3(256), 0, 0, d_planes, d_rec, d_out);
        hipDeviceSynchronize();
        float best = 1e9;
        for (int it = 0; it < 5; ++it) {
            hipEventRecord(a);
            hipLaunchKernelGGL(kern, dim3(nthreads / 256), dim3(256), 0, 0, d_planes, d_rec, d_out);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (ms < best) best = ms;
        }
        const double blocks = (double)nthreads * NB * 8;
        printf("%-34s %.3f ms, %.2f CU-clk/block @2.4GHz\n", name, best,
               best * 1e-3 * 2.4e9 * p.multiProcessorCount / blocks);
    };
    abl("abl 10 rounds (sbox+mix) W4", k_abl<1, 4>);
    abl("abl 10 rounds no key W4", k_abl<2, 4>);
    abl("abl 10 rounds VGPR key W4", k_abl<3, 4>);
    abl("abl 40 sboxes only W4", k_abl<4, 4>);
    abl("abl 10 mix only W4", k_abl<5, 4>);
    abl("abl to_blocks only W4", k_abl<6, 4>);
    abl("abl 10 rounds (sbox+mix) W6", k_abl<1, 6>);
    abl("abl 10 rounds no key W6", k_abl<2, 6>);
    abl("abl 40 sboxes only W6", k_abl<4, 6>);
    abl("abl 10 mix only W6", k_abl<5, 6>);
    return fails;
}
