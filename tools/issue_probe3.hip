// issue_probe3.hip -- VALU issue rate on gfx950 for the instruction shapes of
// the ChaCha20-Poly1305 kernels (chacha_poly.hip, poly1305.h): v_add_u32,
// v_xor_b32, v_alignbit_b32 (rotate), v_mad_u64_u32 (Poly1305 limb products),
// v_lshl_add_u64 (64-bit address math) and a full ChaCha double round on 4
// independent columns, at 1..8 waves per SIMD.  Not part of libtlsgpu.
//   hipcc -O3 --offload-arch=gfx950 -o issue_probe3 tools/issue_probe3.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

// MODE 0: v_add_u32 x[c] += y      MODE 1: v_alignbit x[c] = rot(x[c], 7)
// MODE 2: v_mad_u64_u32 a[c] = x[c] * y + a[c] (64-bit accumulators)
// MODE 3: v_lshl_add_u64 a[c] = (a[c] << 2) + b
// MODE 4: v_perm_b32 (byte rotate)   MODE 5: v_alignbyte_b32
// MODE 6: v_lshl_or_b32              MODE 7: v_lshrrev_b32
// MODE 8: v_xad_u32 (a ^ b) + c      MODE 9: v_add3_u32
// MODE 10: v_mul_u32_u24             MODE 11: v_mad_u32_u24
// MODE 12: v_mul_lo_u32              MODE 13: v_mul_hi_u32
// MODE 14: v_lshlrev_b32             MODE 15: v_or_b32
// MODE 16: v_pk_add_u16 half swap    MODE 17: v_add_co_u32_e32
// MODE 18: v_bitop3 with an inline constant   MODE 19: v_and_b32
template <int MODE, int CH, int B, int R>
__global__ void probe(uint32_t* out, uint64_t* cyc, uint32_t seed) {
    uint32_t x[CH];
    uint64_t a[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        x[c] = seed + threadIdx.x * 7 + c;
        a[c] = (uint64_t)x[c] * 3;
    }
    const uint32_t y = seed * 3 + threadIdx.x;
    const uint64_t bb = (uint64_t)y << 20;
    const uint32_t z = seed ^ threadIdx.x, sel = 0x02010003u + (seed & 0x100u);
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int b = 0; b < B; ++b)
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                if (MODE == 0)
                    asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
                else if (MODE == 1)
                    asm volatile("v_alignbit_b32 %0, %0, %0, 25" : "+v"(x[c]));
                else if (MODE == 2)
                    asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a[c]) : "v"(x[c]), "v"(y) : "vcc");
                else if (MODE == 3)
                    asm volatile("v_lshl_add_u64 %0, %0, 2, %1" : "+v"(a[c]) : "v"(bb));
                else if (MODE == 4)
                    asm volatile("v_perm_b32 %0, %0, %0, %1" : "+v"(x[c]) : "v"(sel));
                else if (MODE == 5)
                    asm volatile("v_alignbyte_b32 %0, %0, %0, 3" : "+v"(x[c]));
                else if (MODE == 6)
                    asm volatile("v_lshl_or_b32 %0, %0, 7, %1" : "+v"(x[c]) : "v"(y));
                else if (MODE == 7)
                    asm volatile("v_lshrrev_b32 %0, 25, %0" : "+v"(x[c]));
                else if (MODE == 8)
                    asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(y), "v"(z));
                else if (MODE == 9)
                    asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(y), "v"(z));
                else if (MODE == 10)
                    asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x[c]) : "v"(y));
                else if (MODE == 11)
                    asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(x[c]) : "v"(y), "v"(z));
                else if (MODE == 12)
                    asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
                else if (MODE == 13)
                    asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
                else if (MODE == 14)
                    asm volatile("v_lshlrev_b32 %0, 7, %0" : "+v"(x[c]));
                else if (MODE == 15)
                    asm volatile("v_or_b32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
                else if (MODE == 16)
                    asm volatile("v_pk_add_u16 %0, %0, 0 op_sel:[1,0] op_sel_hi:[0,1]" : "+v"(x[c]));
                else if (MODE == 17)
                    asm volatile("v_add_co_u32_e32 %0, vcc, %0, %1" : "+v"(x[c]) : "v"(y) : "vcc");
                else if (MODE == 18)
                    asm volatile("v_bitop3_b32 %0, %0, %1, 15 bitop3:0x96" : "+v"(x[c]) : "v"(y));
                else
                    asm volatile("v_and_b32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
            }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) acc ^= x[c] ^ (uint32_t)a[c] ^ (uint32_t)(a[c] >> 32);
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

__device__ __forceinline__ uint32_t rotl(uint32_t v, int c) { return __builtin_amdgcn_alignbit(v, v, 32 - c); }
#define QR(a, b, c, d)                                  \
    a += b; d ^= a; d = rotl(d, 16);                    \
    c += d; b ^= c; b = rotl(b, 12);                    \
    a += b; d ^= a; d = rotl(d, 8);                     \
    c += d; b ^= c; b = rotl(b, 7);

__device__ __forceinline__ uint32_t rot16p(uint32_t v) { return __builtin_amdgcn_perm(v, v, 0x01000302u); }
__device__ __forceinline__ uint32_t rot8p(uint32_t v) { return __builtin_amdgcn_perm(v, v, 0x02010003u); }
#define QRP(a, b, c, d)                                 \
    a += b; d ^= a; d = rot16p(d);                      \
    c += d; b ^= c; b = rotl(b, 12);                    \
    a += b; d ^= a; d = rot8p(d);                       \
    c += d; b ^= c; b = rotl(b, 7);

// R double rounds of one ChaCha state (4 independent QRs per half round;
// 96 VALU per double round).
template <int R, bool PERM>
__global__ void chacha_probe(uint32_t* out, uint64_t* cyc, uint32_t seed) {
    uint32_t x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = seed * (i + 1) + threadIdx.x;
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < R; ++r) {
        if (PERM) {
            QRP(x[0], x[4], x[8], x[12]);
            QRP(x[1], x[5], x[9], x[13]);
            QRP(x[2], x[6], x[10], x[14]);
            QRP(x[3], x[7], x[11], x[15]);
            QRP(x[0], x[5], x[10], x[15]);
            QRP(x[1], x[6], x[11], x[12]);
            QRP(x[2], x[7], x[8], x[13]);
            QRP(x[3], x[4], x[9], x[14]);
        } else {
            QR(x[0], x[4], x[8], x[12]);
            QR(x[1], x[5], x[9], x[13]);
            QR(x[2], x[6], x[10], x[14]);
            QR(x[3], x[7], x[11], x[15]);
            QR(x[0], x[5], x[10], x[15]);
            QR(x[1], x[6], x[11], x[12]);
            QR(x[2], x[7], x[8], x[13]);
            QR(x[3], x[4], x[9], x[14]);
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc ^= x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}


// Forced instruction order (inline asm keeps it): one ChaCha half round on 4
// columns, INTERLEAVED = step k of all four QRs back to back (independent
// neighbours), else QR after QR (dependent neighbours).  ROT: 0 = alignbit,
// 1 = lshlrev + lshrrev + or.
#define A_ADD(x, y) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(y))
#define A_XOR(x, y) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(y))
template <int ROT>
__device__ __forceinline__ void a_rot(uint32_t& x, uint32_t& t, int n) {
    if (ROT == 0) {
        switch (n) {
        case 16: asm volatile("v_alignbit_b32 %0, %0, %0, 16" : "+v"(x)); break;
        case 12: asm volatile("v_alignbit_b32 %0, %0, %0, 20" : "+v"(x)); break;
        case 8: asm volatile("v_alignbit_b32 %0, %0, %0, 24" : "+v"(x)); break;
        default: asm volatile("v_alignbit_b32 %0, %0, %0, 25" : "+v"(x)); break;
        }
    } else {
        switch (n) {
        case 16: asm volatile("v_lshrrev_b32 %1, 16, %0\n v_lshlrev_b32 %0, 16, %0\n v_or_b32 %0, %0, %1" : "+v"(x), "=&v"(t)); break;
        case 12: asm volatile("v_lshrrev_b32 %1, 20, %0\n v_lshlrev_b32 %0, 12, %0\n v_or_b32 %0, %0, %1" : "+v"(x), "=&v"(t)); break;
        case 8: asm volatile("v_lshrrev_b32 %1, 24, %0\n v_lshlrev_b32 %0, 8, %0\n v_or_b32 %0, %0, %1" : "+v"(x), "=&v"(t)); break;
        default: asm volatile("v_lshrrev_b32 %1, 25, %0\n v_lshlrev_b32 %0, 7, %0\n v_or_b32 %0, %0, %1" : "+v"(x), "=&v"(t)); break;
        }
    }
}

template <int ROT, bool INTERLEAVED>
__device__ __forceinline__ void a_half(uint32_t* a[4], uint32_t* b[4], uint32_t* c[4], uint32_t* d[4], uint32_t* t) {
    const int rots[4] = {16, 12, 8, 7};
    if (INTERLEAVED) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const bool ad = (s & 1) == 0;   // steps 0, 2: a += b, d ^= a, rot d; 1, 3: c += d, b ^= c, rot b
#pragma unroll
            for (int q = 0; q < 4; ++q) { if (ad) A_ADD(*a[q], *b[q]); else A_ADD(*c[q], *d[q]); }
#pragma unroll
            for (int q = 0; q < 4; ++q) { if (ad) A_XOR(*d[q], *a[q]); else A_XOR(*b[q], *c[q]); }
#pragma unroll
            for (int q = 0; q < 4; ++q) a_rot<ROT>(ad ? *d[q] : *b[q], t[q], rots[s]);
        }
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const bool ad = (s & 1) == 0;
                if (ad) { A_ADD(*a[q], *b[q]); A_XOR(*d[q], *a[q]); a_rot<ROT>(*d[q], t[q], rots[s]); }
                else { A_ADD(*c[q], *d[q]); A_XOR(*b[q], *c[q]); a_rot<ROT>(*b[q], t[q], rots[s]); }
            }
    }
}

template <int R, int ROT, bool INTERLEAVED>
__global__ void chacha_asm_probe(uint32_t* out, uint64_t* cyc, uint32_t seed) {
    uint32_t x[16], t[4];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = seed * (i + 1) + threadIdx.x;
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < R; ++r) {
        uint32_t* a1[4] = {&x[0], &x[1], &x[2], &x[3]};
        uint32_t* b1[4] = {&x[4], &x[5], &x[6], &x[7]};
        uint32_t* c1[4] = {&x[8], &x[9], &x[10], &x[11]};
        uint32_t* d1[4] = {&x[12], &x[13], &x[14], &x[15]};
        a_half<ROT, INTERLEAVED>(a1, b1, c1, d1, t);
        uint32_t* b2[4] = {&x[5], &x[6], &x[7], &x[4]};
        uint32_t* c2[4] = {&x[10], &x[11], &x[8], &x[9]};
        uint32_t* d2[4] = {&x[15], &x[12], &x[13], &x[14]};
        a_half<ROT, INTERLEAVED>(a1, b2, c2, d2, t);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc ^= x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

// alternating cheap / expensive ops on independent chains
template <int R>
__global__ void mix_probe(uint32_t* out, uint64_t* cyc, uint32_t seed) {
    uint32_t x[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) x[c] = seed + threadIdx.x * 7 + c;
    const uint32_t y = seed * 3 + threadIdx.x;
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int b = 0; b < 64; ++b) {
#pragma unroll
            for (int c = 0; c < 8; c += 2) {
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
                asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[c + 1]) : "v"(y));
                asm volatile("v_alignbit_b32 %0, %0, %0, 25" : "+v"(x[(c + 2) & 7]));
            }
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) acc ^= x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}


// S independent ChaCha states per thread (column+diagonal double rounds,
// compiler-scheduled): ILP 4 S per wave.
template <int R, int S>
__global__ void chacha_multi_probe(uint32_t* out, uint64_t* cyc, uint32_t seed) {
    uint32_t x[S][16];
#pragma unroll
    for (int q = 0; q < S; ++q)
#pragma unroll
        for (int i = 0; i < 16; ++i) x[q][i] = seed * (i + 1) + threadIdx.x + 77 * q;
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int q = 0; q < S; ++q) {
            QR(x[q][0], x[q][4], x[q][8], x[q][12]);
            QR(x[q][1], x[q][5], x[q][9], x[q][13]);
            QR(x[q][2], x[q][6], x[q][10], x[q][14]);
            QR(x[q][3], x[q][7], x[q][11], x[q][15]);
        }
#pragma unroll
        for (int q = 0; q < S; ++q) {
            QR(x[q][0], x[q][5], x[q][10], x[q][15]);
            QR(x[q][1], x[q][6], x[q][11], x[q][12]);
            QR(x[q][2], x[q][7], x[q][8], x[q][13]);
            QR(x[q][3], x[q][4], x[q][9], x[q][14]);
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t acc = 0;
#pragma unroll
    for (int q = 0; q < S; ++q)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc ^= x[q][i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

static void report(const char* name, int w, float ms, const uint64_t* h, int nw, double instr) {
    double mean = 0;
    for (int i = 0; i < nw; ++i) mean += h[i];
    mean /= nw;
    const double lane_ops = instr * 64 * nw;
    printf("%-30s waves/SIMD %d: %.3f ms, %5.1f cyc/instr per wave, %6.1f lane-ops/clk/CU @2.4GHz\n", name, w,
           ms, mean / instr, lane_ops / (ms * 1e-3 * 2.4e9 * 256));
}

template <class K>
static void launch(const char* name, K kern, int w, double instr, uint32_t* d_out, uint64_t* d_cyc) {
    const int blocks = 256 * w, threads = 256;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, d_out, d_cyc, 1u);
    (void)hipDeviceSynchronize();
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, d_out, d_cyc, 2u);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    static uint64_t h[256 * 8 * 4];
    (void)hipMemcpy(h, d_cyc, blocks * 4 * 8, hipMemcpyDeviceToHost);
    report(name, w, ms, h, blocks * 4, instr);
}

int main() {
    uint32_t* d_out;
    uint64_t* d_cyc;
    if (hipMalloc(&d_out, 256 * 8 * 256 * 4) != hipSuccess || hipMalloc(&d_cyc, 256 * 8 * 4 * 8) != hipSuccess)
        return 1;
    const int ws[] = {2, 3, 4, 6, 8};
    for (int w : ws) {
        launch("chacha 1 state", chacha_multi_probe<1024, 1>, w, 96.0 * 1024, d_out, d_cyc);
        launch("chacha 2 states", chacha_multi_probe<512, 2>, w, 96.0 * 1024, d_out, d_cyc);
        launch("chacha 3 states", chacha_multi_probe<342, 3>, w, 96.0 * 1026, d_out, d_cyc);
    }
    return 0;
}
