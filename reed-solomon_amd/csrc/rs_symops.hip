// rs_symops.hip -- CDNA4 (gfx950) kernels of rsg_symbol_ops: chains of gf_add / gf_mul / gf_madd (reference
// src/rs/gf65536.c:155-219) on one target symbol each, applied in order, many chains per launch.
//
// k_symop_consts runs first: for every op that multiplies, the 16 packed constants c * alpha^i (one thread per
// constant, 64 B per op), computed once per call instead of per wave and op on the scalar unit.
// k_symbol_chains then takes one workgroup of W waves per (256 * DW byte column span, chain): the target's DW
// dwords per lane stay in registers across the chain, every op reads its source once (sources are loaded a
// group of ops ahead of their use), the constants arrive by one scalar load per op, and the target is written
// once. With W waves per workgroup a chain is cut into W slices of consecutive ops, one per wave, each applied
// from zero (wave 0 from the target); a chain that scales its target multiplies each slice's result by the
// product of the later slices' scale factors (records the host appends, rs_symops.hpp); the W results are XORed
// through LDS: the latency of a long chain is paid W times in parallel instead of once in series.
// c * x on two packed words is bit-sliced: XOR over the bits i of x of c alpha^i, the lane mask of bit i in
// each 16-bit half being the half's sign after a packed shift left by 15 - i -- three VALU per bit and dword
// (packed shift, packed arithmetic shift, one v_bitop3 for the masked XOR).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rs_symops.hpp"

namespace rsamd {

__global__ void __launch_bounds__(256) k_symop_consts(const SymOpRec* __restrict__ ops, uint64_t n_ops,
                                                      uint32_t* __restrict__ consts) {
    const uint64_t t = uint64_t(blockIdx.x) * 256u + threadIdx.x;
    const uint64_t o = t >> 4;
    const uint32_t i = uint32_t(t & 15u);
    if (o >= n_ops) return;
    const uint32_t kind = ops[o].kind;
    if (kind != kSymMadd && kind != kSymScale) return;
    uint32_t c = ops[o].coef;
    for (uint32_t j = 0; j < i; ++j) c = (c << 1) ^ ((c >> 15) ? 0x1002Du : 0u);  // c * alpha, x^16 + x^5 + x^3 + x^2 + 1
    consts[16 * o + i] = c | (c << 16);
}

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));

// r ^ c x (r = 0 for a plain product)
__device__ __forceinline__ uint32_t madd_packed(uint32_t r, uint32_t x, const uint32_t (&K)[16]) {
    const u16x2 v = __builtin_bit_cast(u16x2, x);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const u16x2 up = v << static_cast<unsigned short>(15 - i);                   // bit i of each half to bit 15
        const s16x2 m = __builtin_bit_cast(s16x2, up) >> static_cast<short>(15);     // 0xffff where it was set
        r = __builtin_amdgcn_bitop3_b32(r, __builtin_bit_cast(uint32_t, m), K[i], 0x78);  // r ^ (m & K[i])
    }
    return r;
}

constexpr int kSymOpGroup = 4;  // ops whose sources are loaded together

template <int DW>
__global__ void __launch_bounds__(64 * kSymMaxWaves) k_symbol_chains(const SymChain* __restrict__ chains,
                                                                     const SymOpRec* __restrict__ ops,
                                                                     const uint32_t* __restrict__ consts,
                                                                     uint64_t nwords) {
    extern __shared__ uint32_t part[];  // [W - 1][DW][64]: the slice sums of waves 1 .. W - 1 (none for W = 1,
                                        // so single-wave launches keep full occupancy)
    const SymChain ch = chains[blockIdx.y];
    const uint32_t nw = blockDim.x >> 6;
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
    const uint32_t lane = threadIdx.x & 63u;
    const bool split = nw > 1 && (ch.flags & kChainSplit);
    const uint64_t nd = nwords / 2;  // whole dwords; an odd word count leaves one 16-bit word at dword nd
    const bool odd = nwords & 1;
    const uint64_t d0 = uint64_t(blockIdx.x) * (64 * DW) + lane;
    // this wave's ops: a slice of a split chain, the whole chain on wave 0, nothing otherwise
    uint32_t start = ch.start, end = ch.start + ch.count;
    if (split) {
        const uint32_t len = (ch.count + nw - 1) / nw;
        start = ch.start + min(w * len, ch.count);
        end = ch.start + min((w + 1) * len, ch.count);
    } else if (w) {
        start = end;
    }
    uint32_t acc[DW];
    auto load = [&](const uint8_t* p, uint32_t (&v)[DW]) {
#pragma unroll
        for (int j = 0; j < DW; ++j) {
            const uint64_t d = d0 + 64u * j;
            v[j] = d < nd ? reinterpret_cast<const uint32_t*>(p)[d]
                          : (odd && d == nd ? uint32_t(reinterpret_cast<const uint16_t*>(p)[2 * d]) : 0u);
        }
    };
    if (w == 0) {
        load(ch.a, acc);
    } else {
#pragma unroll
        for (int j = 0; j < DW; ++j) acc[j] = 0u;
    }
    auto loads_src = [&](uint32_t o) {
        const uint32_t k = ops[o].kind;
        return k == kSymXor || k == kSymMadd;
    };
    // sources go in by groups of kSymOpGroup ops; group g + 1's loads are issued before group g's work, so
    // up to two groups of loads are in flight against one wait per group
    auto load_group = [&](uint32_t g0, uint32_t (&x)[kSymOpGroup][DW]) {
#pragma unroll
        for (int q = 0; q < kSymOpGroup; ++q)
            if (g0 + q < end && loads_src(g0 + q)) load(ops[g0 + q].b, x[q]);
    };
    auto apply = [&](uint32_t o, const uint32_t (&xs)[DW]) {
        const uint32_t kind = ops[o].kind;
        if (kind == kSymXor) {
#pragma unroll
            for (int j = 0; j < DW; ++j) acc[j] ^= xs[j];
        } else if (kind == kSymMadd || kind == kSymScale) {
            uint32_t K[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) K[i] = consts[16u * o + i];  // uniform: one s_load_dwordx16 (as SGPR
                                                                      // operands: VGPR copies measured 5-30 % slower)
            if (kind == kSymMadd) {
#pragma unroll
                for (int j = 0; j < DW; ++j) acc[j] = madd_packed(acc[j], xs[j], K);
            } else {
#pragma unroll
                for (int j = 0; j < DW; ++j) acc[j] = madd_packed(0u, acc[j], K);
            }
        } else if (kind == kSymZero) {
#pragma unroll
            for (int j = 0; j < DW; ++j) acc[j] = 0u;
        }
    };
    auto run_group = [&](uint32_t g0, const uint32_t (&x)[kSymOpGroup][DW]) {
#pragma unroll
        for (int q = 0; q < kSymOpGroup; ++q)
            if (g0 + q < end) apply(g0 + q, x[q]);
    };
    uint32_t xa[kSymOpGroup][DW], xb[kSymOpGroup][DW];
    load_group(start, xa);
    for (uint32_t g0 = start; g0 < end; g0 += 2 * kSymOpGroup) {
        load_group(g0 + kSymOpGroup, xb);
        run_group(g0, xa);
        load_group(g0 + 2 * kSymOpGroup, xa);
        run_group(g0 + kSymOpGroup, xb);
    }
    if (split && (ch.flags & kChainAffine)) {  // times the scale factors of the slices after this one
        const uint32_t o = ch.comb + w, kind = ops[o].kind;
        if (kind == kSymScale) {
            uint32_t K[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) K[i] = consts[16u * o + i];
#pragma unroll
            for (int j = 0; j < DW; ++j) acc[j] = madd_packed(0u, acc[j], K);
        } else if (kind == kSymZero) {
#pragma unroll
            for (int j = 0; j < DW; ++j) acc[j] = 0u;
        }
    }
    if (nw > 1) {  // every wave reaches the barrier (uniform per workgroup: nw, split)
        if (split && w) {
#pragma unroll
            for (int j = 0; j < DW; ++j) part[((w - 1) * DW + j) * 64 + lane] = acc[j];
        }
        __syncthreads();
        if (split && w == 0) {
            for (uint32_t v = 1; v < nw; ++v) {
#pragma unroll
                for (int j = 0; j < DW; ++j) acc[j] ^= part[((v - 1) * DW + j) * 64 + lane];
            }
        }
    }
    if (w) return;
#pragma unroll
    for (int j = 0; j < DW; ++j) {
        const uint64_t d = d0 + 64u * j;
        if (d < nd)
            reinterpret_cast<uint32_t*>(ch.a)[d] = acc[j];
        else if (odd && d == nd)
            reinterpret_cast<uint16_t*>(ch.a)[2 * d] = uint16_t(acc[j]);
    }
}

hipError_t launch_symop_consts(const SymOpRec* ops, uint64_t n_ops, uint32_t* consts, hipStream_t st) {
    if (!n_ops) return hipSuccess;
    const uint64_t blocks = (n_ops * 16 + 255) / 256;
    if (blocks > 0x7FFFFFFFu) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_symop_consts, dim3(unsigned(blocks)), dim3(256), 0, st, ops, n_ops, consts);
    return hipGetLastError();
}

hipError_t launch_symbol_chains(const SymChain* chains, const SymOpRec* ops, const uint32_t* consts,
                                uint32_t n_chains, uint64_t nwords, hipStream_t st, int dw, int waves) {
    if (!n_chains || !nwords) return hipSuccess;
    if (waves < 1 || waves > kSymMaxWaves) return hipErrorInvalidValue;
    const dim3 block(64u * unsigned(waves));
    const size_t lds = size_t(waves - 1) * size_t(dw) * 64 * sizeof(uint32_t);
    const uint64_t nd = nwords / 2 + (nwords & 1);
    const uint64_t spans = (nd + 64 * uint64_t(dw) - 1) / (64 * uint64_t(dw));
    if (spans > 0x7FFFFFFFu || n_chains > 65535u) return hipErrorInvalidValue;
    const dim3 grid(unsigned(spans), n_chains);
    if (dw == 1)
        hipLaunchKernelGGL(k_symbol_chains<1>, grid, block, lds, st, chains, ops, consts, nwords);
    else if (dw == 2)
        hipLaunchKernelGGL(k_symbol_chains<2>, grid, block, lds, st, chains, ops, consts, nwords);
    else if (dw == 4)
        hipLaunchKernelGGL(k_symbol_chains<4>, grid, block, lds, st, chains, ops, consts, nwords);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace rsamd
