// microbench.hip -- instruction-rate and access-pattern probes for the AEAD
// kernels' design decisions on gfx950 (run on the GPU box; results are
// recorded in DESIGN.md).  Not part of libtlsgpu.
//
//   hipcc -O3 --offload-arch=gfx950 -o microbench tools/microbench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                                \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);     \
            return 1;                                                           \
        }                                                                       \
    } while (0)

constexpr int ITERS = 4096;
constexpr int CH = 8;  // independent chains per lane

// Each op is applied CH-way independently, ITERS times.
#define OP_KERNEL(name, T, init, body)                                          \
    __global__ void name(T* out, uint32_t seed) {                               \
        T x[CH];                                                                \
        for (int c = 0; c < CH; ++c) x[c] = (T)(init);                           \
        uint32_t s = seed + threadIdx.x;                                        \
        for (int it = 0; it < ITERS; ++it) {                                    \
            _Pragma("unroll") for (int c = 0; c < CH; ++c) { body; }             \
        }                                                                       \
        T acc = 0;                                                              \
        for (int c = 0; c < CH; ++c) acc += x[c];                               \
        out[blockIdx.x * blockDim.x + threadIdx.x] = acc;                       \
    }

#define N1 x[(c + 1) & 7]
#define N2 x[(c + 2) & 7]
#define ASM2(ins) asm volatile(ins " %0, %0, %1" : "+v"(x[c]) : "v"(N1))
#define ASM3(ins) asm volatile(ins " %0, %0, %1, %2" : "+v"(x[c]) : "v"(N1), "v"(N2))
OP_KERNEL(k_add_u32, uint32_t, c + seed + threadIdx.x, ASM2("v_add_u32"))
OP_KERNEL(k_xor_b32, uint32_t, c + seed + threadIdx.x, ASM2("v_xor_b32"))
OP_KERNEL(k_add3_u32, uint32_t, c + seed + threadIdx.x, ASM3("v_add3_u32"))
OP_KERNEL(k_or3_b32, uint32_t, c + seed + threadIdx.x, ASM3("v_or3_b32"))
OP_KERNEL(k_alignbit, uint32_t, c + seed + threadIdx.x, ASM3("v_alignbit_b32"))
OP_KERNEL(k_perm, uint32_t, c + seed + threadIdx.x, ASM3("v_perm_b32"))
OP_KERNEL(k_bfe, uint32_t, c + seed + threadIdx.x, ASM3("v_bfe_u32"))
OP_KERNEL(k_lshl_or, uint32_t, c + seed + threadIdx.x, ASM3("v_lshl_or_b32"))
OP_KERNEL(k_and_or, uint32_t, c + seed + threadIdx.x, ASM3("v_and_or_b32"))
OP_KERNEL(k_mul_u24, uint32_t, c + seed + threadIdx.x, ASM2("v_mul_u32_u24"))
OP_KERNEL(k_mad_u24, uint32_t, c + seed + threadIdx.x, ASM3("v_mad_u32_u24"))
OP_KERNEL(k_mul_hi_u24, uint32_t, c + seed + threadIdx.x, ASM2("v_mul_hi_u32_u24"))
OP_KERNEL(k_mul_lo_u32, uint32_t, c + seed + threadIdx.x, ASM2("v_mul_lo_u32"))
OP_KERNEL(k_mul_hi_u32, uint32_t, c + seed + threadIdx.x, ASM2("v_mul_hi_u32"))
OP_KERNEL(k_fma_f32, float, c + seed + threadIdx.x, ASM3("v_fma_f32"))
OP_KERNEL(k_pk_fma_f32, double, c + seed + threadIdx.x, ASM3("v_pk_fma_f32"))
OP_KERNEL(k_fma_f64, double, c + seed + threadIdx.x, ASM3("v_fma_f64"))
OP_KERNEL(k_bitop3, uint32_t, c + seed + threadIdx.x, asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x[c]) : "v"(N1), "v"(N2)))
OP_KERNEL(k_xor_sdwa, uint32_t, c + seed + threadIdx.x, asm volatile("v_xor_b32_sdwa %0, %0, %1 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1" : "+v"(x[c]) : "v"(N1)))
OP_KERNEL(k_lshrrev, uint32_t, c + seed + threadIdx.x, ASM2("v_lshrrev_b32"))
OP_KERNEL(k_and_b32, uint32_t, c + seed + threadIdx.x, ASM2("v_and_b32"))
OP_KERNEL(k_xad_u32, uint32_t, c + seed + threadIdx.x, ASM3("v_xad_u32"))
OP_KERNEL(k_pk_rot16, uint32_t, c + seed + threadIdx.x, asm volatile("v_pk_add_u16 %0, %1, 0 op_sel:[1,1] op_sel_hi:[0,0]" : "=v"(x[c]) : "v"(N1)))
OP_KERNEL(k_pk_add_u16, uint32_t, c + seed + threadIdx.x, ASM2("v_pk_add_u16"))
OP_KERNEL(k_cndmask, uint32_t, c + seed + threadIdx.x, asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[c]) : "v"(N1)))
OP_KERNEL(k_add_u64, uint64_t, c + seed + threadIdx.x, asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(x[c]) : "v"(N1)))

__global__ void k_mad_u64_u32(uint64_t* out, uint32_t seed) {
    uint64_t x[CH];
    uint32_t y[CH];
    for (int c = 0; c < CH; ++c) { x[c] = c + seed + threadIdx.x; y[c] = x[c] * 3; }
    for (int it = 0; it < ITERS; ++it) {
        _Pragma("unroll") for (int c = 0; c < CH; ++c)
            asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(x[c]) : "v"(y[c]), "v"(y[(c + 1) & 7]) : "vcc");
    }
    uint64_t acc = 0;
    for (int c = 0; c < CH; ++c) acc += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

#define QR(a, b, c, d)                                              \
    a += b; d ^= a; d = __builtin_amdgcn_alignbit(d, d, 16);        \
    c += d; b ^= c; b = __builtin_amdgcn_alignbit(b, b, 20);        \
    a += b; d ^= a; d = __builtin_amdgcn_alignbit(d, d, 24);        \
    c += d; b ^= c; b = __builtin_amdgcn_alignbit(b, b, 25);
__global__ void k_chacha_only(uint32_t* out, uint32_t seed) {
    uint32_t acc = 0;
    const uint32_t k0 = seed, k1 = seed * 3, k2 = seed * 5, k3 = seed * 7;
    for (int blk = 0; blk < 64; ++blk) {
        uint32_t x0 = 0x61707865u, x1 = 0x3320646eu, x2 = 0x79622d32u, x3 = 0x6b206574u;
        uint32_t x4 = k0, x5 = k1, x6 = k2, x7 = k3, x8 = k0 ^ 1, x9 = k1 ^ 1, x10 = k2 ^ 1, x11 = k3 ^ 1;
        uint32_t x12 = blk, x13 = threadIdx.x, x14 = blockIdx.x, x15 = seed;
#pragma unroll
        for (int r = 0; r < 10; ++r) {
            QR(x0, x4, x8, x12); QR(x1, x5, x9, x13); QR(x2, x6, x10, x14); QR(x3, x7, x11, x15);
            QR(x0, x5, x10, x15); QR(x1, x6, x11, x12); QR(x2, x7, x8, x13); QR(x3, x4, x9, x14);
        }
        acc ^= x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7 ^ x8 ^ x9 ^ x10 ^ x11 ^ x12 ^ x13 ^ x14 ^ x15;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
#undef QR

// LDS random-lookup rate: T-table style, per-lane replicated (conflict-free)
// vs shared random (conflicted), and 16-byte entries (ds_read_b128).
__global__ void k_lds_b32(uint32_t* out, uint32_t seed, int replicated) {
    __shared__ uint32_t t[256 * 32];
    for (int e = threadIdx.x; e < 256 * 32; e += blockDim.x) t[e] = e * 2654435761u;
    __syncthreads();
    uint32_t x[4] = {seed + threadIdx.x, seed * 3 + threadIdx.x, seed * 5 + threadIdx.x,
                     seed * 7 + threadIdx.x};
    const uint32_t lane = threadIdx.x & 31;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            uint32_t idx = (x[c] >> 8) & 0xff;
            x[c] ^= replicated ? t[idx * 32 + lane] : t[(idx * 33 + (x[c] & 31)) & 8191];
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x[0] ^ x[1] ^ x[2] ^ x[3];
}

__global__ void k_lds_b128(uint4* out, uint32_t seed) {
    __shared__ uint4 t[4096];
    for (int e = threadIdx.x; e < 4096; e += blockDim.x) t[e] = make_uint4(e, e * 3, e * 5, e * 7);
    __syncthreads();
    uint4 y = make_uint4(seed + threadIdx.x, seed, seed ^ threadIdx.x, 7);
    for (int it = 0; it < ITERS / 4; ++it) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            uint32_t w = j < 4 ? y.x : j < 8 ? y.y : j < 12 ? y.z : y.w;
            uint4 v = t[j * 256 + ((w >> (8 * (j & 3))) & 0xff)];
            y.x ^= v.x; y.y ^= v.y; y.z ^= v.z; y.w ^= v.w;
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = y;
}

// Streaming copy of n records of L bytes: lane-per-record (each lane walks its
// own record in 16-byte steps) vs coalesced (a wave walks contiguous 1 KiB).
__global__ void k_copy_lane_per_record(const uint4* in, uint4* out, uint64_t n, uint32_t L16) {
    uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const uint4* src = in + r * L16;
    uint4* dst = out + r * L16;
    for (uint32_t j = 0; j < L16; j += 4) {
        uint4 a = src[j], b = src[j + 1], c = src[j + 2], d = src[j + 3];
        dst[j] = a; dst[j + 1] = b; dst[j + 2] = c; dst[j + 3] = d;
    }
}

__global__ void k_copy_coalesced(const uint4* in, uint4* out, uint64_t total16) {
    uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total16; i += stride)
        out[i] = in[i];
}

template <typename K, typename... A>
float time_kernel(K k, dim3 g, dim3 b, A... a) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k, g, b, 0, 0, a...);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k, g, b, 0, 0, a...);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 3;
}

int main() {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    printf("device %s CUs %d clock %d kHz\n", p.gcnArchName, cus, p.clockRate);
    const dim3 g(cus * 8), b(256);
    void* buf;
    CHECK(hipMalloc(&buf, (size_t)cus * 8 * 256 * 16));
    const double lane_ops = (double)cus * 8 * 256 * ITERS * CH;
    const double peak_clk = 2.4e9;
#define RUN(k, T)                                                                         \
    {                                                                                     \
        float ms = time_kernel(k, g, b, (T*)buf, 7u);                                     \
        double rate = lane_ops / (ms / 1e3);                                              \
        printf("%-16s %8.3f ms  %7.2f Tops/s  %6.2f lane-ops/clk/CU (@2.4GHz)\n", #k, ms,   \
               rate / 1e12, rate / peak_clk / cus);                                       \
    }
    RUN(k_add_u32, uint32_t);
    RUN(k_xor_b32, uint32_t);
    RUN(k_add3_u32, uint32_t);
    RUN(k_or3_b32, uint32_t);
    RUN(k_alignbit, uint32_t);
    RUN(k_perm, uint32_t);
    RUN(k_bfe, uint32_t);
    RUN(k_lshl_or, uint32_t);
    RUN(k_and_or, uint32_t);
    RUN(k_mul_u24, uint32_t);
    RUN(k_mad_u24, uint32_t);
    RUN(k_mul_hi_u24, uint32_t);
    RUN(k_mul_lo_u32, uint32_t);
    RUN(k_mul_hi_u32, uint32_t);
    RUN(k_mad_u64_u32, uint64_t);
    RUN(k_add_u64, uint64_t);
    RUN(k_bitop3, uint32_t);
    RUN(k_pk_rot16, uint32_t);
    RUN(k_pk_add_u16, uint32_t);
    RUN(k_cndmask, uint32_t);
    RUN(k_xor_sdwa, uint32_t);
    RUN(k_lshrrev, uint32_t);
    RUN(k_and_b32, uint32_t);
    RUN(k_xad_u32, uint32_t);
    // ChaCha20 block function alone (no memory), 4 and 8 waves per SIMD
    for (int bs : {256, 512, 1024}) {
        float ms = time_kernel(k_chacha_only, dim3(cus * 4), dim3(bs), (uint32_t*)buf, 7u);
        double blocks = (double)cus * 4 * bs * 64;
        printf("chacha-only blockDim %4d %8.3f ms  %6.2f CU-clk/block (@2.4GHz)  %7.1f GB/s keystream\n",
               bs, ms, (ms / 1e3) * 2.4e9 * cus / blocks, blocks * 64 / (ms / 1e3) / 1e9);
    }
    RUN(k_fma_f32, float);
    RUN(k_pk_fma_f32, double);
    RUN(k_fma_f64, double);
    {
        for (int rep = 1; rep >= 0; --rep) {
            float ms = time_kernel(k_lds_b32, g, b, (uint32_t*)buf, 7u, rep);
            double look = (double)cus * 8 * 256 * ITERS * 4;
            printf("lds_b32 %-10s %8.3f ms  %6.2f lookups/clk/CU\n", rep ? "replicated" : "random",
                   ms, look / (ms / 1e3) / peak_clk / cus);
        }
        float ms = time_kernel(k_lds_b128, g, b, (uint4*)buf, 7u);
        double look = (double)cus * 8 * 256 * (ITERS / 4) * 16;
        printf("lds_b128 random  %8.3f ms  %6.2f lookups/clk/CU\n", ms, look / (ms / 1e3) / peak_clk / cus);
    }
    CHECK(hipFree(buf));
    // streaming patterns, 8 GiB in + 8 GiB out
    const uint64_t n = 1 << 19, L = 16384;
    void *in, *out;
    CHECK(hipMalloc(&in, n * L));
    CHECK(hipMalloc(&out, n * L));
    CHECK(hipMemset(in, 1, n * L));
    float ms = time_kernel(k_copy_lane_per_record, dim3(n / 256), dim3(256), (const uint4*)in,
                           (uint4*)out, n, (uint32_t)(L / 16));
    printf("copy lane-per-record: %8.3f ms  %7.1f GB/s (r+w)\n", ms, 2.0 * n * L / (ms / 1e3) / 1e9);
    ms = time_kernel(k_copy_coalesced, dim3(cus * 16), dim3(256), (const uint4*)in, (uint4*)out,
                     n * L / 16);
    printf("copy coalesced:       %8.3f ms  %7.1f GB/s (r+w)\n", ms, 2.0 * n * L / (ms / 1e3) / 1e9);
    CHECK(hipFree(in));
    CHECK(hipFree(out));
    return 0;
}
