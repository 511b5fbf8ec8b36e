// chacha_probe.hip -- ChaCha20 keystream rate vs blocks interleaved per lane
// (ILP) and waves per SIMD, to size the ChaCha kernel's inner loop.
//   hipcc -O3 --offload-arch=gfx950 -o chacha_probe tools/chacha_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ uint32_t rotl(uint32_t v, int c) { return __builtin_amdgcn_alignbit(v, v, 32 - c); }
#define QR(a, b, c, d)                          \
    a += b; d ^= a; d = rotl(d, 16);            \
    c += d; b ^= c; b = rotl(b, 12);            \
    a += b; d ^= a; d = rotl(d, 8);             \
    c += d; b ^= c; b = rotl(b, 7);

template <int P, int W>
__global__ __launch_bounds__(256, W) void k_chacha(uint32_t* out, uint32_t seed, int nblk) {
    uint32_t acc = 0;
    const uint32_t k0 = seed, k1 = seed * 3, k2 = seed * 5, k3 = seed * 7;
    for (int blk = 0; blk < nblk; blk += P) {
        uint32_t x[P][16];
#pragma unroll
        for (int p = 0; p < P; ++p) {
            x[p][0] = 0x61707865u; x[p][1] = 0x3320646eu; x[p][2] = 0x79622d32u; x[p][3] = 0x6b206574u;
            x[p][4] = k0; x[p][5] = k1; x[p][6] = k2; x[p][7] = k3;
            x[p][8] = k0 ^ 1; x[p][9] = k1 ^ 1; x[p][10] = k2 ^ 1; x[p][11] = k3 ^ 1;
            x[p][12] = blk + p; x[p][13] = threadIdx.x; x[p][14] = blockIdx.x; x[p][15] = seed;
        }
#pragma unroll
        for (int r = 0; r < 10; ++r) {
#pragma unroll
            for (int p = 0; p < P; ++p) {
                QR(x[p][0], x[p][4], x[p][8], x[p][12]); QR(x[p][1], x[p][5], x[p][9], x[p][13]);
                QR(x[p][2], x[p][6], x[p][10], x[p][14]); QR(x[p][3], x[p][7], x[p][11], x[p][15]);
            }
#pragma unroll
            for (int p = 0; p < P; ++p) {
                QR(x[p][0], x[p][5], x[p][10], x[p][15]); QR(x[p][1], x[p][6], x[p][11], x[p][12]);
                QR(x[p][2], x[p][7], x[p][8], x[p][13]); QR(x[p][3], x[p][4], x[p][9], x[p][14]);
            }
        }
#pragma unroll
        for (int p = 0; p < P; ++p)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc ^= x[p][q];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int P, int W>
void run(uint32_t* buf, int cus) {
    const int nblk = 64;
    hipLaunchKernelGGL((k_chacha<P, W>), dim3(cus * 16), dim3(256), 0, 0, buf, 7u, nblk);
    hipDeviceSynchronize();
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    float best = 1e9;
    for (int it = 0; it < 3; ++it) {
        hipEventRecord(a);
        hipLaunchKernelGGL((k_chacha<P, W>), dim3(cus * 16), dim3(256), 0, 0, buf, 7u, nblk);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
    }
    const double blocks = (double)cus * 16 * 256 * nblk;
    printf("P=%d minW=%d: %.3f ms  %.2f CU-clk/block @2.4GHz  %.0f GB/s keystream\n", P, W, best,
           best * 1e-3 * 2.4e9 * cus / blocks, blocks * 64 / best / 1e6);
}

int main() {
    int dev; hipGetDevice(&dev); hipDeviceProp_t p; hipGetDeviceProperties(&p, dev);
    uint32_t* buf; hipMalloc(&buf, (size_t)p.multiProcessorCount * 16 * 256 * 4);
    const int cus = p.multiProcessorCount;
    run<1, 1>(buf, cus); run<1, 4>(buf, cus); run<1, 8>(buf, cus);
    run<2, 1>(buf, cus); run<2, 3>(buf, cus); run<2, 4>(buf, cus);
    run<4, 1>(buf, cus); run<4, 2>(buf, cus);
    return 0;
}
