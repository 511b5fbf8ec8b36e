// chacha_sdwa_probe.hip -- does an SDWA word-swap XOR pair (two full-rate
// VOP2 ops) beat XOR + v_alignbit (one full-rate + one half-rate op) for
// ChaCha's rotations by 16?  Measures bare instruction streams and the full
// double round with rot16 done either way.
//   hipcc -O3 --offload-arch=gfx950 -o chacha_sdwa_probe tools/chacha_sdwa_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ uint32_t rotl(uint32_t v, int c) { return __builtin_amdgcn_alignbit(v, v, 32 - c); }
// rotl16(a ^ d) as two SDWA XORs: the high word of t gets (a^d).lo, then
// the low word gets (a^d).hi with the high word preserved.
__device__ __forceinline__ uint32_t xor_rot16(uint32_t a, uint32_t d) {
    uint32_t t;
    asm("v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0"
        : "=v"(t) : "v"(a), "v"(d));
    asm("v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1"
        : "+v"(t) : "v"(a), "v"(d));
    return t;
}
#define QR0(a, b, c, d)                         \
    a += b; d ^= a; d = rotl(d, 16);            \
    c += d; b ^= c; b = rotl(b, 12);            \
    a += b; d ^= a; d = rotl(d, 8);             \
    c += d; b ^= c; b = rotl(b, 7);
#define QR1(a, b, c, d)                         \
    a += b; d = xor_rot16(a, d);                \
    c += d; b ^= c; b = rotl(b, 12);            \
    a += b; d ^= a; d = rotl(d, 8);             \
    c += d; b ^= c; b = rotl(b, 7);

template <int MODE, int W>
__global__ __launch_bounds__(256, W) void k_chacha(uint32_t* out, uint32_t seed, int nblk) {
    uint32_t acc = 0;
    const uint32_t k0 = seed, k1 = seed * 3, k2 = seed * 5, k3 = seed * 7;
    for (int blk = 0; blk < nblk; ++blk) {
        uint32_t x[16];
        x[0] = 0x61707865u; x[1] = 0x3320646eu; x[2] = 0x79622d32u; x[3] = 0x6b206574u;
        x[4] = k0; x[5] = k1; x[6] = k2; x[7] = k3;
        x[8] = k0 ^ 1; x[9] = k1 ^ 1; x[10] = k2 ^ 1; x[11] = k3 ^ 1;
        x[12] = blk; x[13] = threadIdx.x; x[14] = blockIdx.x; x[15] = seed;
#pragma unroll
        for (int r = 0; r < 10; ++r) {
            if (MODE == 0) {
                QR0(x[0], x[4], x[8], x[12]); QR0(x[1], x[5], x[9], x[13]);
                QR0(x[2], x[6], x[10], x[14]); QR0(x[3], x[7], x[11], x[15]);
                QR0(x[0], x[5], x[10], x[15]); QR0(x[1], x[6], x[11], x[12]);
                QR0(x[2], x[7], x[8], x[13]); QR0(x[3], x[4], x[9], x[14]);
            } else {
                QR1(x[0], x[4], x[8], x[12]); QR1(x[1], x[5], x[9], x[13]);
                QR1(x[2], x[6], x[10], x[14]); QR1(x[3], x[7], x[11], x[15]);
                QR1(x[0], x[5], x[10], x[15]); QR1(x[1], x[6], x[11], x[12]);
                QR1(x[2], x[7], x[8], x[13]); QR1(x[3], x[4], x[9], x[14]);
            }
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) acc ^= x[q];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// Bare streams: 8 independent chains, 64 ops each of (xor + alignbit) or
// (two SDWA xors).
template <int MODE>
__global__ __launch_bounds__(256, 4) void k_stream(uint32_t* out, uint32_t seed, int iters) {
    uint32_t v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = seed * (i + 3) + threadIdx.x;
    const uint32_t a = seed ^ blockIdx.x;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int s = 0; s < 32; ++s)
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (MODE == 0) { v[i] ^= a; v[i] = rotl(v[i], 16); }
                else if (MODE == 1) v[i] = xor_rot16(a, v[i]);
                else { v[i] ^= a; v[i] += a; }
            }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc ^= v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int MODE, int W>
void run(uint32_t* buf, int cus) {
    const int nblk = 64;
    hipLaunchKernelGGL((k_chacha<MODE, W>), dim3(cus * 16), dim3(256), 0, 0, buf, 7u, nblk);
    hipDeviceSynchronize();
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    float best = 1e9;
    for (int it = 0; it < 5; ++it) {
        hipEventRecord(a);
        hipLaunchKernelGGL((k_chacha<MODE, W>), dim3(cus * 16), dim3(256), 0, 0, buf, 7u, nblk);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
    }
    const double blocks = (double)cus * 16 * 256 * nblk;
    printf("double rounds rot16=%s minW=%d: %.3f ms  %.1f CU-clk/block @2.4GHz  %.0f GB/s keystream\n",
           MODE ? "sdwa-pair" : "xor+alignbit", W, best, best * 1e-3 * 2.4e9 * cus / blocks,
           blocks * 64 / best / 1e6);
}

template <int MODE>
void run_stream(uint32_t* buf, int cus) {
    const int iters = 256;
    hipLaunchKernelGGL((k_stream<MODE>), dim3(cus * 16), dim3(256), 0, 0, buf, 7u, iters);
    hipDeviceSynchronize();
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    float best = 1e9;
    for (int it = 0; it < 5; ++it) {
        hipEventRecord(a);
        hipLaunchKernelGGL((k_stream<MODE>), dim3(cus * 16), dim3(256), 0, 0, buf, 7u, iters);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
    }
    const double ops = (double)cus * 16 * 256 * iters * 32 * 8 * 2;   // lane-ops
    printf("stream %s: %.3f ms  %.1f lane-ops/clk/CU @2.4GHz\n",
           MODE == 0 ? "xor+alignbit" : MODE == 1 ? "sdwa xor pair" : "xor+add", best,
           ops / (best * 1e-3 * 2.4e9 * cus));
}

int main() {
    int dev; hipGetDevice(&dev); hipDeviceProp_t p; hipGetDeviceProperties(&p, dev);
    uint32_t* buf; hipMalloc(&buf, (size_t)p.multiProcessorCount * 16 * 256 * 4);
    const int cus = p.multiProcessorCount;
    run_stream<2>(buf, cus); run_stream<0>(buf, cus); run_stream<1>(buf, cus);
    run<0, 2>(buf, cus); run<1, 2>(buf, cus);
    run<0, 4>(buf, cus); run<1, 4>(buf, cus);
    run<0, 8>(buf, cus); run<1, 8>(buf, cus);
    return 0;
}
