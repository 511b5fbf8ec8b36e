// aes_bs.h -- bitsliced building blocks for gfx950 shared by the 8-block
// bitsliced AES (aes_bs8.h): the plane mask of a bit, v_bitop3 / v_perm
// wrappers, and the S-box circuit (aes_bs_sbox.h).
//
// Restates the SubBytes of Rijndael.encrypt (tlslite/utils/rijndael.py:
// 995-1038) on bit planes so that it runs on the VALU instead of LDS table
// lookups: Boyar and Peralta's circuit, its four XNORs dropped, i.e. every
// S-box output is S(x) ^ 0x63, the 0x63 folded into the next round key
// (MixColumns maps a column of equal bytes c to itself, so MC(y ^ c) =
// MC(y) ^ c).
//
// Usable from host code too (the CPU unit test compiles it with g++).
#pragma once
#include <stdint.h>
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#endif

#if defined(__HIPCC__)
#define TG_BS_HD __host__ __device__ __forceinline__
#define TG_BS_MF __host__ __device__ __forceinline__
#else
#define TG_BS_HD static inline
#define TG_BS_MF inline
#endif

namespace tg {
namespace bs {

// Plane mask of bit p of word w: 0 or ~0.
TG_BS_HD uint32_t bitmask(uint32_t w, int p) { return (uint32_t)((int32_t)(w << (31 - p)) >> 31); }

// One full-rate v_bitop3_b32: bit i of the result = bit (4 a_i + 2 b_i + c_i) of tt.
#if defined(__HIP_DEVICE_COMPILE__)
#define bop3(a, b, c, tt) __builtin_amdgcn_bitop3_b32((a), (b), (c), (tt))
#else
TG_BS_HD uint32_t bop3(uint32_t a, uint32_t b, uint32_t c, uint32_t tt) {
    uint32_t r = 0;
    for (int k = 0; k < 8; ++k)
        if ((tt >> k) & 1) r |= ((k & 4) ? a : ~a) & ((k & 2) ? b : ~b) & ((k & 1) ? c : ~c);
    return r;
}
#endif
TG_BS_HD uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return bop3(a, b, c, 0x96); }

// v_perm_b32: byte i of the result = byte sel_i of (hi:lo) (0..3 = lo, 4..7 = hi).
TG_BS_HD uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_perm(hi, lo, sel);
#else
    const uint64_t v = ((uint64_t)hi << 32) | lo;
    uint32_t r = 0;
    for (int i = 0; i < 4; ++i) r |= (uint32_t)((v >> (8 * ((sel >> (8 * i)) & 7))) & 0xff) << (8 * i);
    return r;
#endif
}

// In-place S-box (without the affine constant 0x63) on the planes of one byte,
// x[b] = bit b: Boyar & Peralta's 113-gate circuit covered by 72 two- and
// three-input gates (tools/gen_bs_sbox.py).
#include "aes_bs_sbox.h"

}  // namespace bs
}  // namespace tg
