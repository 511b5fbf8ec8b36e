// issue_probe.hip -- VALU issue rate on gfx950 as a function of ILP, waves per
// SIMD and straight-line code size (bitsliced AES design question).  Each
// wave times its own instruction stream with s_memtime (shader clock).
//   hipcc -O3 --offload-arch=gfx950 -o issue_probe tools/issue_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

// CH independent chains, body of B bitop3 per chain, repeated R times
template <int CH, int B, int R>
__global__ void probe(uint32_t* out, uint64_t* cyc, uint32_t seed) {
    uint32_t x[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = seed + threadIdx.x * 7 + c;
    const uint32_t y = seed * 3 + threadIdx.x, z = seed ^ threadIdx.x;
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int b = 0; b < B; ++b)
#pragma unroll
            for (int c = 0; c < CH; ++c)
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x[c]) : "v"(y), "v"(z));
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) acc ^= x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int CH, int B, int R>
void run(const char* name, int waves_per_simd, uint32_t* d_out, uint64_t* d_cyc) {
    const int cus = 256, threads = 256;   // 4 waves per block = 1 per SIMD
    const int blocks = cus * waves_per_simd;
    hipLaunchKernelGGL((probe<CH, B, R>), dim3(blocks), dim3(threads), 0, 0, d_out, d_cyc, 1u);
    hipDeviceSynchronize();
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL((probe<CH, B, R>), dim3(blocks), dim3(threads), 0, 0, d_out, d_cyc, 2u);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    static uint64_t h[256 * 16 * 4];
    const int nw = blocks * 4;
    hipMemcpy(h, d_cyc, nw * 8, hipMemcpyDeviceToHost);
    double mean = 0;
    for (int i = 0; i < nw; ++i) mean += h[i];
    mean /= nw;
    const double instr = (double)CH * B * R;
    const double lane_ops = instr * 64 * nw;
    printf("%-34s waves/SIMD %d: %.3f ms, %.1f cyc/instr per wave (s_memtime), %.1f lane-ops/clk/CU @2.4GHz\n",
           name, waves_per_simd, ms, mean / instr, lane_ops / (ms * 1e-3 * 2.4e9 * cus));
}

int main() {
    uint32_t* d_out; uint64_t* d_cyc;
    hipMalloc(&d_out, 256 * 16 * 256 * 4); hipMalloc(&d_cyc, 256 * 16 * 4 * 8);
    for (int w = 1; w <= 4; w *= 2) {
        run<1, 64, 2048>("ILP1 loop body 64", w, d_out, d_cyc);
        run<2, 32, 2048>("ILP2 loop body 64", w, d_out, d_cyc);
        run<4, 16, 2048>("ILP4 loop body 64", w, d_out, d_cyc);
        run<8, 8, 2048>("ILP8 loop body 64", w, d_out, d_cyc);
        run<8, 256, 64>("ILP8 loop body 2048", w, d_out, d_cyc);
        run<8, 1024, 16>("ILP8 loop body 8192", w, d_out, d_cyc);
        run<16, 512, 16>("ILP16 loop body 8192", w, d_out, d_cyc);
    }
    return 0;
}
