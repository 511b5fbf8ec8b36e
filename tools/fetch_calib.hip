// fetch_calib.hip -- calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE on
// gfx950 for the access shapes of the AEAD kernels: one copy kernel per
// shape moves exactly BYTES bytes (2^18 records of 16 KiB) from src to dst.
// tools/traffic.sh runs it under the same --pmc passes as bench.py, and
// tools/traffic_summary.py divides the known byte count by the counters to
// get each shape's factor.  Not part of libtlsgpu.
//   hipcc -O3 --offload-arch=gfx950 -o fetch_calib tools/fetch_calib.hip
// Shapes (per wave instruction, 16 B per lane):
//   coalesced  1 KiB contiguous
//   octet      8 records x 128 B (aes_gcm_bs8.hip: lane 8q + l of record q;
//              chacha_poly.hip tiled_blocks since round 2)
//   tile64     16 records x 64 B (chacha_poly.hip tiled_blocks in round 1)
//   lane       64 records x 16 B (lane per record, no tile)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr uint64_t REC = 16384, NREC = 1u << 18, BYTES = REC * NREC;

__global__ void k_coalesced(const uint4* __restrict__ s, uint4* __restrict__ d) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < BYTES / 16) d[i] = s[i];
}

// one wave per 8 records; slot j of 64: lane l of record q copies block 8 j + l
__global__ void k_octet(const uint8_t* __restrict__ s, uint8_t* __restrict__ d) {
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63u, q = lane >> 3, l = lane & 7u;
    const uint64_t rec = 8 * wave + q;
    if (rec >= NREC) return;
    for (uint32_t j = 0; j < REC / 128; ++j) {
        const uint64_t o = rec * REC + 128u * j + 16u * l;
        *reinterpret_cast<uint4*>(d + o) = *reinterpret_cast<const uint4*>(s + o);
    }
}

// one wave per 16 records: lane L copies chunk L % 4 of record 16 w + L / 4
__global__ void k_tile64(const uint8_t* __restrict__ s, uint8_t* __restrict__ d) {
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t rec = 16 * wave + (lane >> 2);
    if (rec >= NREC) return;
    for (uint32_t j = 0; j < REC / 64; ++j) {
        const uint64_t o = rec * REC + 64u * j + 16u * (lane & 3u);
        *reinterpret_cast<uint4*>(d + o) = *reinterpret_cast<const uint4*>(s + o);
    }
}

// lane per record: 64 records x 16 B per instruction
__global__ void k_lane(const uint8_t* __restrict__ s, uint8_t* __restrict__ d) {
    const uint64_t rec = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (rec >= NREC) return;
    for (uint32_t j = 0; j < REC / 16; ++j) {
        const uint64_t o = rec * REC + 16u * j;
        *reinterpret_cast<uint4*>(d + o) = *reinterpret_cast<const uint4*>(s + o);
    }
}

int main() {
    uint8_t *s = nullptr, *d = nullptr;
    if (hipMalloc(&s, BYTES) != hipSuccess || hipMalloc(&d, BYTES) != hipSuccess) return 1;
    (void)hipMemset(s, 0x5a, BYTES);
    (void)hipMemset(d, 0, BYTES);
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL(k_coalesced, dim3(BYTES / 16 / 256), dim3(256), 0, 0, (const uint4*)s, (uint4*)d);
    hipLaunchKernelGGL(k_octet, dim3(NREC / 8 * 64 / 256), dim3(256), 0, 0, s, d);
    hipLaunchKernelGGL(k_tile64, dim3(NREC / 16 * 64 / 256), dim3(256), 0, 0, s, d);
    hipLaunchKernelGGL(k_lane, dim3(NREC / 256), dim3(256), 0, 0, s, d);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("fetch_calib: 4 copies of %llu bytes each\n", (unsigned long long)BYTES);
    return 0;
}
