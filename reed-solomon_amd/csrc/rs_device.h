// rs_device.h -- device helpers shared by rs_kernels.hip and the hiprtc-specialised kernels
// (rs_jit.cpp embeds this file's text into every generated source; keep it self-contained).
#pragma once
#ifndef RS_JIT_SOURCE
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// gamma's minimal polynomial is x^8 + x^4 + x^3 + x^2 + 1: gamma^8 = 0x1D in gamma-basis
// coordinates (host-checked against Gamma8::red).
__device__ __forceinline__ uint32_t xt8(uint32_t m) {
    // multiply 4 packed GF(256) bytes by gamma; the per-byte reduction top * 0x1D is formed with a
    // packed 16-bit multiply (a 24-bit multiply would drop byte 3's carry)
    const uint32_t top = (m >> 7) & 0x01010101u;
    const u16x2 red = __builtin_bit_cast(u16x2, top) * (u16x2){0x1D, 0x1D};
    return ((m << 1) & 0xFEFEFEFEu) ^ __builtin_bit_cast(uint32_t, red);
}

__device__ __forceinline__ uint32_t xt16(uint32_t m) {
    // multiply 2 packed GF(2^16) words by alpha (x^16 = x^5 + x^3 + x^2 + 1)
    const uint32_t top = (m >> 15) & 0x00010001u;
    return ((m << 1) & 0xFFFEFFFEu) ^ (__umul24(top, 0x2Du)  /* top < 2^17 */);
}

// 16-entry nibble table: T[e] = XOR of m_j over the set bits j of e.
__device__ __forceinline__ u32x16 build16(uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3) {
    const uint32_t a = m0 ^ m1, b = m2 ^ m0, c = m2 ^ m1, d = m2 ^ a;
    return (u32x16){0u, m0, m1, a, m2, b, c, d, m3, m3 ^ m0, m3 ^ m1, m3 ^ a, m3 ^ m2, m3 ^ b, m3 ^ c, m3 ^ d};
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

__device__ __forceinline__ uint32_t lds_lookup4(const uint32_t* lt, uint32_t x) {
    return lt[x & 255u] ^ lt[256 + ((x >> 8) & 255u)] ^ lt[512 + ((x >> 16) & 255u)] ^ lt[768 + (x >> 24)];
}

// 8-byte (m<=8) / 4-byte (m=16) column slices; `avail` = bytes of the symbol left from col.
template <int W>
__device__ __forceinline__ void load_slice(uint32_t (&x)[W / 4], const uint8_t* p, int64_t avail) {
    if (avail >= W) {
        if constexpr (W == 8) {
            const u32x2 v = *reinterpret_cast<const u32x2*>(p);
            x[0] = v.x;
            x[1] = v.y;
        } else {
            x[0] = *reinterpret_cast<const uint32_t*>(p);
        }
    } else {
#pragma unroll
        for (int d = 0; d < W / 4; ++d) x[d] = 0;
        for (int b = 0; b < avail; ++b) x[b >> 2] |= uint32_t(p[b]) << (8 * (b & 3));
    }
}

template <int W>
__device__ __forceinline__ void store_slice(uint8_t* p, const uint32_t (&x)[W / 4], int64_t avail) {
    if (avail >= W) {
        if constexpr (W == 8) {
            *reinterpret_cast<u32x2*>(p) = (u32x2){x[0], x[1]};
        } else {
            *reinterpret_cast<uint32_t*>(p) = x[0];
        }
    } else {
        for (int b = 0; b < avail; ++b) p[b] = uint8_t(x[b >> 2] >> (8 * (b & 3)));
    }
}

