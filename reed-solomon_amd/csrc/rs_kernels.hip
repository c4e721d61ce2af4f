// rs_kernels.hip -- CDNA4 (gfx950) kernels of the Reed-Solomon engine.
//
// Every encode and decode is one GF(2^16)-linear map applied independently to each 16-bit word
// column of a stripe:  out_p = sum_i C[p][i] * in_i.  The kernels
// stream the K input symbols of a stripe once from HBM, keep R output accumulators per lane in
// VGPRs and write each output once: algorithmic traffic (K + R) * S bytes per stripe.
//
// GF multiply-add without per-word table gathers: for each input word x a lane builds, in
// registers, the 16-entry nibble tables T[e] = (e-th combination of x * basis^j). A coefficient c
// then contributes T_lo[c & 15] ^ T_hi[c >> 4] (m <= 8) -- two uniform-index register reads
// (s_set_gpr_idx) and one 3-input XOR per dword, shared by all 64 lanes because the coefficient
// is wave-uniform. No MFMA: GF(2) arithmetic is XOR, not a dense numeric contraction.
//
//  * m <= 8 (all positions in GF(256), e.g. k+r <= 255): words are moved to GF(256)^2 coordinates
//    (x = x0 + x1*alpha, x_h in the gamma = alpha^257 polynomial basis) through LDS byte tables,
//    so multiplication by a GF(256) coefficient is byte-wise; 8 multiples by gamma^j come from
//    xtime on 4 packed bytes; two nibble tables; coordinates are mapped back before the store.
//  * m = 16 (general): multiples x * alpha^j (j < 16) by 16-bit xtime on packed words, four
//    nibble tables, no coordinate change.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>

#include "rs_device.h"
#include "rs_kernels.hpp"
#include "gen/cs16t_off.h"

namespace rsamd {

// ------------------------------------------------------------------------------------ m <= 8
// Block = 256 lanes x 8 bytes = 2 KiB of columns of one stripe, RT outputs of tile blockIdx.y.
// MODE 0: nibble tables in VGPRs read with a wave-uniform index (s_set_gpr_idx), 1 xor3 / output.
// MODE 1: the 8 gamma-multiples masked by the coefficient's bits (SGPR masks), 8 bitop3 / output.
template <int RT, int MODE>
__global__ void __launch_bounds__(256) k_apply_m8(ApplyArgs a) {
    __shared__ uint32_t lt[2048];  // [0,1024): L byte tables, [1024,2048): L^-1 byte tables
    for (int i = threadIdx.x; i < 2048; i += 256) lt[i] = a.ltab[i];
    __syncthreads();

    const int64_t bid = blockIdx.x;
    const int64_t local = bid / a.nchunks;  // launch-local stripe
    const int64_t stripe = RS_STRIPE(a.ids, local);
    const int64_t col = (bid - local * a.nchunks) * 2048 + int64_t(threadIdx.x) * 8;
    const int64_t avail = a.nbytes - col;
    const int tile = blockIdx.y;
    const uint8_t* src = a.src + stripe * a.src_stripe + col;
    const uint32_t* cf = a.coef + size_t(tile) * a.K * (RT / 4);

    uint32_t acc[RT][2];
#pragma unroll
    for (int p = 0; p < RT; ++p) acc[p][0] = acc[p][1] = 0;

    if (avail > 0) {
        uint32_t nxt[2];
        if (a.K > 0) load_slice<8>(nxt, src + int64_t(a.in_idx[0]) * a.src_sym, avail);
        for (int i = 0; i < a.K; ++i) {
            const uint32_t x[2] = {nxt[0], nxt[1]};
            if (i + 1 < a.K) load_slice<8>(nxt, src + int64_t(a.in_idx[i + 1]) * a.src_sym, avail);
            uint32_t m[2][8];
#pragma unroll
            for (int v = 0; v < 2; ++v) {
                m[v][0] = lds_lookup4(lt, x[v]);
#pragma unroll
                for (int j = 1; j < 8; ++j) m[v][j] = xt8(m[v][j - 1]);
            }
            const uint32_t* c = cf + size_t(i) * (RT / 4);
            if constexpr (MODE == 0) {
                const u32x16 Tl0 = build16(m[0][0], m[0][1], m[0][2], m[0][3]);
                const u32x16 Th0 = build16(m[0][4], m[0][5], m[0][6], m[0][7]);
                const u32x16 Tl1 = build16(m[1][0], m[1][1], m[1][2], m[1][3]);
                const u32x16 Th1 = build16(m[1][4], m[1][5], m[1][6], m[1][7]);
#pragma unroll
                for (int q = 0; q < RT / 4; ++q) {
                    const uint32_t w = c[q];
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        const uint32_t lo = (w >> (8 * b)) & 15u, hi = (w >> (8 * b + 4)) & 15u;
                        acc[4 * q + b][0] = xor3(acc[4 * q + b][0], Tl0[lo], Th0[hi]);
                        acc[4 * q + b][1] = xor3(acc[4 * q + b][1], Tl1[lo], Th1[hi]);
                    }
                }
            } else {
#pragma unroll
                for (int q = 0; q < RT / 4; ++q) {
                    const uint32_t w = c[q];
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            const uint32_t mask = 0u - ((w >> (8 * b + j)) & 1u);
                            acc[4 * q + b][0] ^= m[0][j] & mask;
                            acc[4 * q + b][1] ^= m[1][j] & mask;
                        }
                    }
                }
            }
        }
    }
    if (avail <= 0) return;
    uint8_t* dst = a.dst + stripe * a.dst_stripe + col;
    const int rows = min(RT, a.R - tile * RT);
#pragma unroll
    for (int p = 0; p < RT; ++p) {
        if (p < rows) {
            uint32_t y[2] = {lds_lookup4(lt + 1024, acc[p][0]), lds_lookup4(lt + 1024, acc[p][1])};
            store_slice<8>(dst + int64_t(a.out_idx[tile * RT + p]) * a.dst_sym, y, avail);
        }
    }
}

// ------------------------------------------------------------------------------ m <= 8, asm
// Same math as k_apply_m8<32, 0>, but the (output x nibble) lookups are one hand-scheduled block
// (csrc/gen_asm.py): the wave enters gpr-index mode once per half, reads pre-split table indices
// from SGPRs filled by SMEM loads, and retargets the index with one s_set_gpr_idx_idx per lookup
// pair, so each output costs 2 SALU + 4 VALU instead of ~12 SALU with compiler lowering (the
// scalar unit, shared by the CU's four SIMDs, was the bottleneck). Tables and accumulators are
// pinned to fixed VGPRs by the constraints below.
// One input step of k_apply_m8_idx: LDS coordinate lookup, then the asm block (multiples, tables,
// 32 outputs x 2 dwords of indexed XORs).
template <int ABL>
__device__ __forceinline__ void m8_asm_step(uint32_t y0, uint32_t y1, const uint32_t* cp, u32x16& a0l, u32x16& a0h,
                                            u32x16& a1l, u32x16& a1h) {
    const uint32_t k1d = 0x1D1D1D1Du;  // VGPR operand: an SGPR operand would halve the bitop3 rate
    uint32_t t0, t1, t2, t3;
    u32x16 Tl0, Th0, Tl1, Th1;
#define RS_M8_IDX_OPERANDS                                                                                     \
    : "+{v[72:87]}"(a0l), "+{v[88:103]}"(a0h), "+{v[104:119]}"(a1l), "+{v[120:135]}"(a1h), "=&{v[8:23]}"(Tl0),        \
      "=&{v[24:39]}"(Th0), "=&{v[40:55]}"(Tl1), "=&{v[56:71]}"(Th1), [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2),  \
      [t3] "=&v"(t3)                                                                                                  \
    : [y0] "v"(y0), [y1] "v"(y1), [cp] "s"(cp), [kfe] "s"(0xFEFEFEFEu), [k1d] "v"(k1d)                                               \
    : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55", "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68", "s69", "s70", "s71"
    // ABL: 0 production ("split"), 1..6 timing ablations / alternative schedules (csrc/gen_asm.py)
    if constexpr (ABL == 0) {
        asm volatile(
#include "gen/m8_idx_asm.inc"
            RS_M8_IDX_OPERANDS);
    } else if constexpr (ABL == 1) {
        asm volatile(
#include "gen/m8_idx_asm_noidx.inc"
            RS_M8_IDX_OPERANDS);
    } else if constexpr (ABL == 2) {
        asm volatile(
#include "gen/m8_idx_asm_build.inc"
            RS_M8_IDX_OPERANDS);
    } else if constexpr (ABL == 3) {
        asm volatile(
#include "gen/m8_idx_asm_look.inc"
            RS_M8_IDX_OPERANDS);
    } else if constexpr (ABL == 4) {
        asm volatile(
#include "gen/m8_idx_asm_nop.inc"
            RS_M8_IDX_OPERANDS);
    } else if constexpr (ABL == 5) {
        asm volatile(
#include "gen/m8_idx_asm_split_mul.inc"
            RS_M8_IDX_OPERANDS);
    } else {
        asm volatile(
#include "gen/m8_idx_asm_plain.inc"
            RS_M8_IDX_OPERANDS);
    }
#undef RS_M8_IDX_OPERANDS
}


template <int ABL>
__device__ __forceinline__ void m8_idx_step(const uint32_t* lt, const uint32_t (&x)[2], const uint32_t* cp,
                                            u32x16& a0l, u32x16& a0h, u32x16& a1l, u32x16& a1h) {
    m8_asm_step<ABL>(lds_lookup4(lt, x[0]), lds_lookup4(lt, x[1]), cp, a0l, a0h, a1l, a1h);
}

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));

// Input loop with a PD-deep load ring (PD x 512 B in flight per wave: HBM latency under full load
// is microseconds). Slot indices are fetched four at a time through SMEM (in_idx is padded). FULL: the
// whole 2 KiB chunk lies inside the symbol (decided per block), so loads carry no bounds checks.
template <bool FULL, int ABL, int PD>
__device__ __forceinline__ void m8_idx_body(const ApplyArgs& a, const int32_t* __restrict__ in_idx, const uint32_t* lt,
                                            const uint8_t* src, int64_t avail, const uint32_t* cbase, u32x16& a0l,
                                            u32x16& a0h, u32x16& a1l, u32x16& a1h) {
    auto load = [&](uint32_t (&dst)[2], int32_t slot) {
        const uint8_t* p = src + int64_t(slot) * a.src_sym;
        if constexpr (FULL) {
            const u32x2 v = *reinterpret_cast<const u32x2*>(p);
            dst[0] = v.x;
            dst[1] = v.y;
        } else {
            load_slice<8>(dst, p, avail);
        }
    };
    const int K = a.K;
    uint32_t ring[PD][2];
    int32_t sl[PD];
#pragma unroll
    for (int q = 0; q < PD / 4; ++q) {
        const i32x4 v = *reinterpret_cast<const i32x4*>(in_idx + 4 * q);
        sl[4 * q] = v.x, sl[4 * q + 1] = v.y, sl[4 * q + 2] = v.z, sl[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int j = 0; j < PD; ++j) {
        ring[j][0] = ring[j][1] = 0;
        if (j < K) load(ring[j], sl[j]);
    }
    for (int i = 0; i < K; i += PD) {
#pragma unroll
        for (int q = 0; q < PD / 4; ++q) {
            const i32x4 v = *reinterpret_cast<const i32x4*>(in_idx + i + PD + 4 * q);
            sl[4 * q] = v.x, sl[4 * q + 1] = v.y, sl[4 * q + 2] = v.z, sl[4 * q + 3] = v.w;
        }
        const uint32_t* cp = cbase + size_t(i) * 64;
#pragma unroll
        for (int j = 0; j < PD; ++j) {
            if (i + j < K) {
                const uint32_t x[2] = {ring[j][0], ring[j][1]};
                if (i + j + PD < K) load(ring[j], sl[j]);
                m8_idx_step<ABL>(lt, x, cp + 64 * j, a0l, a0h, a1l, a1h);
            }
        }
    }
}

// ------------------------------------------------------------------ m <= 8, asm + LDS-DMA ring
// Input staging for full 2 KiB chunks: each input's chunk is copied HBM -> LDS by two
// global_load_lds_dwordx4 (1 KiB, 16 B per lane) issued by one wave of the block (wave i % 4 owns
// input i), RING_B batches of 4 inputs ahead. Completion: the issuing wave's counted
// s_waitcnt vmcnt, then a raw s_barrier (one per batch); readers ds_read_b64 their 8 bytes.
// Ring slot of input i = i % (4 * (RING_B + 1)): batch b + RING_B reuses batch b - 1's slots, which
// every wave finished reading before the barrier that ended round b - 1.
// wait until at most n of this wave's DMA instructions are outstanding (n even, 0..2*RING_B)
__device__ __forceinline__ void wait_vm_dyn(int n) {
    if (n <= 0)
        wait_vm<0>();
    else if (n <= 2)
        wait_vm<2>();
    else if (n <= 4)
        wait_vm<4>();
    else
        wait_vm<6>();
}

__device__ __forceinline__ uint64_t stamp_now() {
    uint64_t v;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");
    return v;
}

template <int ABL, bool STAMP = false>
__device__ __forceinline__ void m8_lds_body(const ApplyArgs& a, const int32_t* __restrict__ in_idx, uint32_t* lds,
                                            const uint8_t* chunk_src, const uint32_t* cbase, u32x16& a0l,
                                            u32x16& a0h, u32x16& a1l, u32x16& a1h) {
    const uint32_t* lt = lds;
    uint32_t* ring = lds + 2048;
    const int K = a.K;
    const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x) >> 6);
    const int lane = threadIdx.x & 63;
    const uint32_t ring_lds = uint32_t(reinterpret_cast<uintptr_t>(ring));
    const uint8_t* gl = chunk_src + 16 * lane;
    auto issue = [&](int i) {  // wave-uniform: only the owning wave calls
        const uint8_t* g = gl + int64_t(sload(in_idx + i)) * a.src_sym;
        const uint32_t dst = ring_lds + uint32_t(i % RING_SLOTS) * 2048u;
        dma16(g, dst);
        dma16(g + 1024, dst + 1024);
    };
    const int nb = (K + 3) / 4;
    // outstanding DMA instructions of this wave for batches [lo, hi]
    auto mine = [&](int lo, int hi) {
        int c = 0;
        for (int b = lo; b <= hi; ++b)
            if (b < nb && 4 * b + wave < K) c += 2;
        return c;
    };
    uint64_t ph[4] = {0, 0, 0, 0}, t0 = 0, t1 = 0;  // STAMP: prologue+coords, asm, wait+barrier, total
    if constexpr (STAMP) t0 = stamp_now();
    const uint64_t tstart = t0;
    for (int b = 0; b < RING_B; ++b)
        if (4 * b + wave < K) issue(4 * b + wave);
    wait_vm_dyn(mine(1, RING_B - 1));
    asm volatile("s_barrier" ::: "memory");
    for (int b = 0; b < nb; ++b) {
        if constexpr (STAMP) t0 = stamp_now();
        const int ib = 4 * (b + RING_B) + wave;
        if (ib < K) issue(ib);
        // the batch's 4 inputs: ring reads and coordinate lookups first (one LDS latency for all
        // four; slots past K hold stale bytes and are not used), then the 4 asm steps
        uint32_t y[4][2];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const u32x2 v = *reinterpret_cast<const u32x2*>(
                reinterpret_cast<const uint8_t*>(ring) + ((4 * b + j) % RING_SLOTS) * 2048 + 8 * threadIdx.x);
            y[j][0] = lds_lookup4(lt, v.x);
            y[j][1] = lds_lookup4(lt, v.y);
        }
        if constexpr (STAMP) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            t1 = stamp_now();
            ph[0] += t1 - t0;
            t0 = t1;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = 4 * b + j;
            if (i < K) m8_asm_step<ABL>(y[j][0], y[j][1], cbase + size_t(i) * 64, a0l, a0h, a1l, a1h);
        }
        if constexpr (STAMP) {
            t1 = stamp_now();
            ph[1] += t1 - t0;
            t0 = t1;
        }
        wait_vm_dyn(mine(b + 2, b + RING_B));
        asm volatile("s_barrier" ::: "memory");
        if constexpr (STAMP) {
            t1 = stamp_now();
            ph[2] += t1 - t0;
        }
    }
    if constexpr (STAMP) {
        ph[3] = stamp_now() - tstart;
        if (lane == 0) {
            uint64_t* o = a.stamps + (int64_t(blockIdx.y) * gridDim.x + blockIdx.x) * 16 + wave * 4;
            o[0] = ph[0], o[1] = ph[1], o[2] = ph[2], o[3] = ph[3];
        }
    }
}

// Full 2 KiB chunks only (a.nchunks = full chunks per symbol); the tail chunk goes to k_apply_m8_idx.
template <int ABL, bool STAMP = false>
__global__ void __launch_bounds__(256) k_apply_m8_lds(ApplyArgs a, const int32_t* __restrict__ in_idx) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[2048 + RING_SLOTS * 512];
    for (int i = threadIdx.x; i < 2048; i += 256) lds[i] = a.ltab[i];
    __syncthreads();

    const int64_t bid = blockIdx.x;
    const int64_t local = bid / a.nchunks;  // launch-local stripe
    const int64_t stripe = RS_STRIPE(a.ids, local);
    const int64_t chunk0 = (bid - local * a.nchunks) * 2048;
    const int64_t col = chunk0 + int64_t(threadIdx.x) * 8;
    const int64_t avail = a.nbytes - col;
    const int tile = blockIdx.y;
    const uint32_t* cbase = a.idx + size_t(tile) * a.K * 64;

    u32x16 a0l = 0, a0h = 0, a1l = 0, a1h = 0;
    m8_lds_body<ABL, STAMP>(a, in_idx, lds, a.src + stripe * a.src_stripe + chunk0, cbase, a0l, a0h, a1l, a1h);
    uint8_t* dst = a.dst + stripe * a.dst_stripe + col;
    const int rows = min(32, a.R - tile * 32);
#pragma unroll
    for (int p = 0; p < 32; ++p) {
        if (p < rows) {
            const uint32_t v0 = p < 16 ? a0l[p & 15] : a0h[p & 15];
            const uint32_t v1 = p < 16 ? a1l[p & 15] : a1h[p & 15];
            uint32_t y[2] = {lds_lookup4(lds + 1024, v0), lds_lookup4(lds + 1024, v1)};
            store_slice<8>(dst + int64_t(a.out_idx[tile * 32 + p]) * a.dst_sym, y, avail);
        }
    }
}

// ------------------------------------------------------- m <= 8, one dword per lane (V = 1)
// Same algorithm as k_apply_m8_lds with 4 bytes per lane per step: tables (32 VGPRs) and 32
// accumulators (32 VGPRs) take half the registers, so 5 waves share each SIMD instead of 3 (the
// V = 2 kernel is bound by each wave's own issue rate, not by the VALU pipe). Block = 256 lanes x 4 B
// = one 1 KiB column chunk; each input's chunk is one global_load_lds_dwordx4 (1 KiB) issued by
// wave i % 4, RING_B batches ahead, one s_barrier per batch of 4 inputs.
template <int ABL>
__device__ __forceinline__ void m8_v1_step(uint32_t y, const uint32_t* cp, u32x16& a0, u32x16& a1) {
    const uint32_t k1d = 0x1D1D1D1Du;
    uint32_t t0, t1;
    u32x16 Tl, Th;
#define RS_M8_V1_OPERANDS                                                                                  \
    : "+{v[40:55]}"(a0), "+{v[56:71]}"(a1), "=&{v[8:23]}"(Tl), "=&{v[24:39]}"(Th), [t0] "=&v"(t0), [t1] "=&v"(t1) \
    : [y0] "v"(y), [cp] "s"(cp), [k1d] "v"(k1d)                                                                 \
    : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55", \
      "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68", "s69", "s70", "s71"
    if constexpr (ABL == 0) {
        asm volatile(
#include "gen/m8_idx_asm_v1.inc"
            RS_M8_V1_OPERANDS);
#ifdef RS_AMD_DIAG
    } else if constexpr (ABL == 7) {  // timing ablation: one SMEM round trip per step (wrong results)
        asm volatile(
#include "gen/m8_idx_asm_v1_nohi.inc"
            RS_M8_V1_OPERANDS);
#endif
    } else {
        asm volatile(
#include "gen/m8_idx_asm_v1_plain.inc"
            RS_M8_V1_OPERANDS);
    }
#undef RS_M8_V1_OPERANDS
}

// One-table input step (gen_asm.py v1h): multiples y g^0..3, one nibble table, low-nibble lookups into
// A = (a0, a1), high-nibble lookups of the same table into B = (b0, b1); the output is A + g^4 B.
__device__ __forceinline__ void m8_v1h_step(uint32_t y, const uint32_t* cp, u32x16& a0, u32x16& a1, u32x16& b0,
                                            u32x16& b1) {
    const uint32_t k1d = 0x1D1D1D1Du;
    u32x16 T;
    asm volatile(
#include "gen/m8_idx_asm_v1h.inc"
        : "+{v[24:39]}"(a0), "+{v[40:55]}"(a1), "+{v[56:71]}"(b0), "+{v[72:87]}"(b1), "=&{v[8:23]}"(T)
        : [y0] "v"(y), [cp] "s"(cp), [k1d] "v"(k1d)
        : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55",
          "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68", "s69", "s70", "s71");
}

// V = 1 generic kernel (rs_device.h:m8_v1_run): per input, multiples + tables + 64 gpr-indexed
// lookups with SMEM-fed indices. ABL 0: two tables (production v1), 1: v1 without gpr-index mode
// (timing only), 2: the one-table step (m8_v1h_step, two accumulator sets). The matrix-specialised
// variant is rs_jit.cpp's rs_v1jit.
template <int ABL>
__global__ void __launch_bounds__(256) k_apply_m8_v1(V1Args a) {
    if constexpr (ABL >= 2 && ABL <= 4) {  // inputs converted 1 (ABL 2), 2 (3) or 4 (4) at a time
        __shared__ __attribute__((aligned(16))) uint32_t lds[V1H_LDS_WORDS];
        m8_v1_run<2, ABL == 2 ? 1 : ABL == 3 ? 2 : 4>(a, lds, [&](uint32_t y, int, int, u32x16& a0, u32x16& a1, u32x16& b0, u32x16& b1,
                                 const uint32_t* rec) { m8_v1h_step(y, rec, a0, a1, b0, b1); });
    } else if constexpr (ABL == 6) {  // the production step over a.cpb column chunks per workgroup (inputs
                                      // converted two at a time: 91 VGPRs, 5 waves/SIMD)
        __shared__ __attribute__((aligned(16))) uint32_t lds[V1_LDS_WORDS];
        m8_v1_run<1, 2, false, true>(a, lds, [&](uint32_t y, int, int, u32x16& a0, u32x16& a1, const uint32_t* rec) {
            m8_v1_step<0>(y, rec, a0, a1);
        });
    } else if constexpr (ABL == 5) {  // diagnostic: the production step with s_memtime phase stamps
        __shared__ __attribute__((aligned(16))) uint32_t lds[V1_LDS_WORDS];
        m8_v1_run<1, 4, true>(a, lds, [&](uint32_t y, int, int, u32x16& a0, u32x16& a1, const uint32_t* rec) {
            m8_v1_step<0>(y, rec, a0, a1);
        });
    } else {
        __shared__ __attribute__((aligned(16))) uint32_t lds[V1_LDS_WORDS];
        m8_v1_run(a, lds, [&](uint32_t y, int, int, u32x16& a0, u32x16& a1, const uint32_t* rec) {
            m8_v1_step<ABL>(y, rec, a0, a1);
        });
    }
}

#ifdef RS_AMD_DIAG  // option-only per-stripe solve kernels (m8_ps_kernel 1 / 2): diagnostic build only
// Per-stripe V = 1 apply without the LDS input ring, for the short solves of rsg_decode_batch (K = t <= r
// inputs per stripe; at C3 32). The ring kernel's four waves of a 1 KiB chunk meet at a barrier every 4
// inputs and wait for DMA bookkeeping: at K = 32 its waves spent a third of their time parked
// (SQ_WAIT_ANY, profiles/r4/ps8_pmc.txt). Here the four waves of a block share only the coordinate tables:
// each loads its own 256-byte column of the inputs straight into registers, 8 inputs ahead, and runs the
// same input step (gen_asm.py v1) and output stage as k_apply_m8_v1.
__global__ void __launch_bounds__(256) k_apply_m8_ps_w(V1Args a) {
    __shared__ uint32_t lt[2048];
    for (int i = threadIdx.x; i < 2048; i += 256) lt[i] = a.ltab[i];
    __syncthreads();
    const int64_t bid = blockIdx.x;
    const int64_t local = bid / a.nchunks;  // launch-local stripe
    const int64_t stripe = RS_STRIPE(a.ids, local);
    const int64_t col = (bid - local * a.nchunks) * 1024 + int64_t(threadIdx.x) * 4;
    const int tile = blockIdx.y;
    const int K = sload(a.ps_kr + 2 * local), R = sload(a.ps_kr + 2 * local + 1);
    if (tile * 32 >= R) return;  // uniform over the block
    const int32_t* in_idx = a.in_idx + local * a.ps_in;
    const uint32_t* idxb = a.idx + local * a.ps_idx + size_t(tile) * K * 64;
    const uint8_t* src = a.src + (a.src_local ? local : stripe) * a.src_stripe + col;
    auto ld = [&](int i) { return *reinterpret_cast<const uint32_t*>(src + int64_t(sload(in_idx + i)) * a.src_sym); };
    u32x16 a0 = 0, a1 = 0;
    uint32_t cur[8], nxt[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) cur[j] = j < K ? ld(j) : 0u;
    for (int i0 = 0; i0 < K; i0 += 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) nxt[j] = i0 + 8 + j < K ? ld(i0 + 8 + j) : 0u;
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (i0 + j < K) m8_v1_step<0>(lds_lookup4(lt, cur[j]), idxb + size_t(i0 + j) * 64, a0, a1);
#pragma unroll
        for (int j = 0; j < 8; ++j) cur[j] = nxt[j];
    }
    m8_v1_store<1>(a, lt, a.dst + stripe * a.dst_stripe + col, a.out_idx + local * a.ps_out + tile * 32,
                   min(32, R - tile * 32), a0, a1, a0, a1);
}

// The same with two dwords per lane (the "split" input step of k_apply_m8_idx / _lds, gen_asm.py): each
// index switch serves two lookups, half the V = 1 kernel's SALU per byte, at 3 waves per SIMD. A block's
// four waves cover a 2 KiB column chunk; the last chunk of a symbol may be partial (FULL = false: loads
// and stores bounded by the symbol size).
template <bool FULL>
__device__ __forceinline__ void m8_ps_w2_body(const V1Args& a, const uint32_t* lt, int64_t local, int64_t stripe,
                                              int64_t col, int tile, int K, int R) {
    const int64_t avail = FULL ? 8 : a.nchunks - col;  // nchunks carries the symbol size here (see launcher)
    const int32_t* in_idx = a.in_idx + local * a.ps_in;
    const uint32_t* idxb = a.idx + local * a.ps_idx + size_t(tile) * K * 64;
    const uint8_t* src = a.src + (a.src_local ? local : stripe) * a.src_stripe + col;
    auto ld = [&](uint32_t (&x)[2], int i) {
        const uint8_t* p = src + int64_t(sload(in_idx + i)) * a.src_sym;
        if constexpr (FULL) {
            const u32x2 v = *reinterpret_cast<const u32x2*>(p);
            x[0] = v.x;
            x[1] = v.y;
        } else {
            load_slice<8>(x, p, avail);
        }
    };
    u32x16 a0l = 0, a0h = 0, a1l = 0, a1h = 0;
    uint32_t cur[4][2], nxt[4][2];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        cur[j][0] = cur[j][1] = 0;
        if (j < K) ld(cur[j], j);
    }
    for (int i0 = 0; i0 < K; i0 += 4) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            nxt[j][0] = nxt[j][1] = 0;
            if (i0 + 4 + j < K) ld(nxt[j], i0 + 4 + j);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (i0 + j < K) m8_idx_step<0>(lt, cur[j], idxb + size_t(i0 + j) * 64, a0l, a0h, a1l, a1h);
#pragma unroll
        for (int j = 0; j < 4; ++j) cur[j][0] = nxt[j][0], cur[j][1] = nxt[j][1];
    }
    uint8_t* dst = a.dst + stripe * a.dst_stripe + col;
    const int32_t* out = a.out_idx + local * a.ps_out + tile * 32;
    const int rows = min(32, R - tile * 32);
#pragma unroll
    for (int p = 0; p < 32; ++p) {
        if (p < rows) {
            uint8_t* d = dst + int64_t(sload(out + p)) * a.dst_sym;
            uint32_t y[2] = {lds_lookup4(lt + 1024, p < 16 ? a0l[p & 15] : a0h[p & 15]),
                             lds_lookup4(lt + 1024, p < 16 ? a1l[p & 15] : a1h[p & 15])};
            if (a.xor_dst) {  // V1Args::xor_dst
                uint32_t old[2];
                if constexpr (FULL) {
                    const u32x2 v = *reinterpret_cast<const u32x2*>(d);
                    old[0] = v.x;
                    old[1] = v.y;
                } else {
                    load_slice<8>(old, d, avail);
                }
                y[0] ^= old[0];
                y[1] ^= old[1];
            }
            if constexpr (FULL)
                *reinterpret_cast<u32x2*>(d) = (u32x2){y[0], y[1]};
            else
                store_slice<8>(d, y, avail);
        }
    }
}

// grid (n_sel * chunks of 2 KiB, tiles); a.nchunks = the symbol size in bytes
__global__ void __launch_bounds__(256) k_apply_m8_ps_w2(V1Args a) {
    __shared__ uint32_t lt[2048];
    for (int i = threadIdx.x; i < 2048; i += 256) lt[i] = a.ltab[i];
    __syncthreads();
    const int64_t S = a.nchunks, nch = (S + 2047) / 2048;
    const int64_t bid = blockIdx.x;
    const int64_t local = bid / nch;
    const int64_t chunk0 = (bid - local * nch) * 2048;
    const int64_t stripe = RS_STRIPE(a.ids, local);
    const int tile = blockIdx.y;
    const int K = sload(a.ps_kr + 2 * local), R = sload(a.ps_kr + 2 * local + 1);
    if (tile * 32 >= R) return;  // uniform over the block
    const int64_t col = chunk0 + int64_t(threadIdx.x) * 8;
    if (chunk0 + 2048 <= S)
        m8_ps_w2_body<true>(a, lt, local, stripe, col, tile, K, R);
    else
        m8_ps_w2_body<false>(a, lt, local, stripe, col, tile, K, R);
}
#endif  // RS_AMD_DIAG

template <int ABL, int PD>
__global__ void __launch_bounds__(256) k_apply_m8_idx(ApplyArgs a, const int32_t* __restrict__ in_idx) {
    __shared__ uint32_t lt[2048];
    for (int i = threadIdx.x; i < 2048; i += 256) lt[i] = a.ltab[i];
    __syncthreads();

    const int64_t bid = blockIdx.x;
    const int64_t local = bid / a.nchunks;  // launch-local stripe
    const int64_t stripe = RS_STRIPE(a.ids, local);
    const int64_t chunk0 = (a.chunk_base + bid - local * a.nchunks) * 2048;
    const int64_t col = chunk0 + int64_t(threadIdx.x) * 8;
    const int64_t avail = a.nbytes - col;
    const int tile = blockIdx.y;
    const uint8_t* src = a.src + stripe * a.src_stripe + col;
    const uint32_t* cbase = a.idx + size_t(tile) * a.K * 64;

    u32x16 a0l = 0, a0h = 0, a1l = 0, a1h = 0;
    if (chunk0 + 2048 <= a.nbytes)
        m8_idx_body<true, ABL, PD>(a, in_idx, lt, src, avail, cbase, a0l, a0h, a1l, a1h);
    else if (avail > 0)
        m8_idx_body<false, ABL, PD>(a, in_idx, lt, src, avail, cbase, a0l, a0h, a1l, a1h);
    if (avail <= 0) return;
    uint8_t* dst = a.dst + stripe * a.dst_stripe + col;
    const int rows = min(32, a.R - tile * 32);
#pragma unroll
    for (int p = 0; p < 32; ++p) {
        if (p < rows) {
            const uint32_t v0 = p < 16 ? a0l[p & 15] : a0h[p & 15];
            const uint32_t v1 = p < 16 ? a1l[p & 15] : a1h[p & 15];
            uint32_t y[2] = {lds_lookup4(lt + 1024, v0), lds_lookup4(lt + 1024, v1)};
            store_slice<8>(dst + int64_t(a.out_idx[tile * 32 + p]) * a.dst_sym, y, avail);
        }
    }
}

// ------------------------------------------------------------------------------------ m = 16
// Block = 256 lanes x 4 bytes = 1 KiB of columns, RT outputs of tile blockIdx.y.
template <int RT>
__global__ void __launch_bounds__(256) k_apply_m16(ApplyArgs a) {
    const int64_t bid = blockIdx.x;
    const int64_t local = bid / a.nchunks;  // launch-local stripe
    const int64_t stripe = RS_STRIPE(a.ids, local);
    const int64_t col = (a.chunk_base + bid - local * a.nchunks) * 1024 + int64_t(threadIdx.x) * 4;
    const int64_t avail = a.nbytes - col;
    if (avail <= 0) return;
    const int tile = blockIdx.y;
    const uint8_t* src = a.src + stripe * a.src_stripe + col;
    const uint32_t* cf = a.coef + size_t(tile) * a.K * (RT / 2);

    uint32_t acc[RT];
#pragma unroll
    for (int p = 0; p < RT; ++p) acc[p] = 0;

    uint32_t nxt[1];
    if (a.K > 0) load_slice<4>(nxt, src + int64_t(a.in_idx[0]) * a.src_sym, avail);
    for (int i = 0; i < a.K; ++i) {
        const uint32_t x = nxt[0];
        if (i + 1 < a.K) load_slice<4>(nxt, src + int64_t(a.in_idx[i + 1]) * a.src_sym, avail);
        uint32_t m[16];
        m[0] = x;
#pragma unroll
        for (int j = 1; j < 16; ++j) m[j] = xt16(m[j - 1]);
        const u32x16 T0 = build16(m[0], m[1], m[2], m[3]);
        const u32x16 T1 = build16(m[4], m[5], m[6], m[7]);
        const u32x16 T2 = build16(m[8], m[9], m[10], m[11]);
        const u32x16 T3 = build16(m[12], m[13], m[14], m[15]);
        const uint32_t* c = cf + size_t(i) * (RT / 2);
#pragma unroll
        for (int q = 0; q < RT / 2; ++q) {
            const uint32_t w = c[q];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint32_t cc = w >> (16 * h);
                const int p = 2 * q + h;
                acc[p] = xor3(acc[p], T0[cc & 15u], T1[(cc >> 4) & 15u]);
                acc[p] = xor3(acc[p], T2[(cc >> 8) & 15u], T3[(cc >> 12) & 15u]);
            }
        }
    }
    uint8_t* dst = a.dst + stripe * a.dst_stripe + col;
    const int rows = min(RT, a.R - tile * RT);
#pragma unroll
    for (int p = 0; p < RT; ++p) {
        if (p < rows) {
            uint32_t y[1] = {acc[p]};
            store_slice<4>(dst + int64_t(a.out_idx[tile * RT + p]) * a.dst_sym, y, avail);
        }
    }
}

// --------------------------------------------- m = 16, hand-scheduled step, one dword per lane
// Same block structure as m8_v1_run (1 KiB column chunk, inputs staged HBM -> LDS by DMA, one
// s_barrier per batch of 4 inputs), 64 outputs per tile, no coordinate change. Per input the step
// (csrc/gen_asm.py m16_v1) forms x * alpha^j (j < 16), four nibble tables in v[8:71] and 256
// lookups, each one s_set_gpr_idx_idx + one v_xor (record: [tile][K + 1][64] dwords of packed
// byte indices; s[40:55] carries the current plane from one step to the next).
template <int ABL>
__device__ __forceinline__ void m16_v1_step(uint32_t y, const uint32_t* cp, u32x16& plane, u32x16& a0, u32x16& a1,
                                            u32x16& a2, u32x16& a3) {
    const uint32_t k2d = 0x002D002Du;
    uint32_t t0, t1;
    u32x16 T0, T1, T2, T3;
#define RS_M16_V1_OPERANDS                                                                                    \
    : "+{v[72:87]}"(a0), "+{v[88:103]}"(a1), "+{v[104:119]}"(a2), "+{v[120:135]}"(a3), "=&{v[8:23]}"(T0),        \
      "=&{v[24:39]}"(T1), "=&{v[40:55]}"(T2), "=&{v[56:71]}"(T3), [t0] "=&v"(t0), [t1] "=&v"(t1),               \
      "+{s[40:55]}"(plane)                                                                                       \
    : [y0] "v"(y), [cp] "s"(cp), [k2d] "v"(k2d)                                                                 \
    : "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68", "s69", "s70", "s71", \
      "s72", "s73", "s74"
    if constexpr (ABL == 0) {
        asm volatile(
#include "gen/m8_idx_asm_m16_v1.inc"
            RS_M16_V1_OPERANDS);
    } else {
        asm volatile(
#include "gen/m8_idx_asm_m16_v1_plain.inc"
            RS_M16_V1_OPERANDS);
    }
#undef RS_M16_V1_OPERANDS
}

template <int ABL>
__global__ void __launch_bounds__(256) k_apply_m16_v1(V1Args a) {
    __shared__ __attribute__((aligned(16))) uint32_t ring[RING_SLOTS * 256];
    int64_t unit = blockIdx.x;
    int tile = blockIdx.y;
    if (a.units) {  // XCD-aware order: workgroup b runs on XCD b % 8
        const int64_t slot = blockIdx.x >> 3;
        tile = int(slot % a.tiles);
        unit = (slot / a.tiles) * 8 + (blockIdx.x & 7);
        if (unit >= a.units) return;  // padding of the last group of 8 units
    }
    const int64_t local = unit / a.nchunks;  // launch-local stripe
    const int64_t stripe = RS_STRIPE(a.ids, local);
    const int64_t chunk0 = (unit - local * a.nchunks) * 1024;
    const int slice = blockIdx.z;
    // per-stripe plans (rsg_decode_batch, GF(2^16) route): this stripe's K, R, lists and records
    int Kp = a.K, Rp = a.R;
    const int32_t* in_list = a.in_idx;
    const int32_t* out_list = a.out_idx;
    const uint32_t* idxb = a.idx;
    if (a.ps_kr) {
        Kp = sload(a.ps_kr + 2 * local);
        Rp = sload(a.ps_kr + 2 * local + 1);
        in_list += local * a.ps_in;
        out_list += local * a.ps_out;
        idxb += local * a.ps_idx;
        if (tile * 64 >= Rp) return;  // the stripe has fewer row tiles than the launch
    }
    // split-K: this workgroup takes inputs [i0, i0 + K) of the full list
    const int i0 = a.kslices > 1 ? int(int64_t(Kp) * slice / a.kslices) : 0;
    const int K = a.kslices > 1 ? int(int64_t(Kp) * (slice + 1) / a.kslices) - i0 : Kp;
    const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x) >> 6);
    const int lane = threadIdx.x & 63;
    const uint32_t ring_lds = uint32_t(reinterpret_cast<uintptr_t>(ring));
    const uint8_t* gl = a.src + (a.src_local ? local : stripe) * a.src_stripe + chunk0 + 16 * lane;
    const int32_t* in_idx = in_list + i0;
    auto issue = [&](int i) { dma16(gl + int64_t(sload(in_idx + i)) * a.src_sym, ring_lds + uint32_t(i % RING_SLOTS) * 1024u); };
    const int nb = (K + 3) / 4;
    auto mine = [&](int lo, int hi) {  // this wave's outstanding DMA instructions for batches [lo, hi]
        int c = 0;
        for (int b = lo; b <= hi; ++b)
            if (b < nb && 4 * b + wave < K) c += 1;
        return c;
    };
    auto wait_mine = [&](int n) {
        if (n <= 0)
            wait_vm<0>();
        else if (n == 1)
            wait_vm<1>();
        else if (n == 2)
            wait_vm<2>();
        else
            wait_vm<3>();
    };
    u32x16 a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    for (int b = 0; b < RING_B; ++b)
        if (4 * b + wave < K) issue(4 * b + wave);
    wait_mine(mine(1, RING_B - 1));
    asm volatile("s_barrier" ::: "memory");
    // records: [tile][K + 1][64] packed table indices (one padding record: the last step prefetches)
    const uint32_t* rec = idxb + (size_t(tile) * (Kp + 1) + i0) * 64;
    u32x16 plane;  // plane 0 of the next step's record, requested one step ahead (s[40:55] in the asm)
    asm volatile("s_load_dwordx16 %0, %1, 0x0" : "={s[40:55]}"(plane) : "s"(rec) : "memory");
    for (int b = 0; b < nb; ++b) {
        const int ib = 4 * (b + RING_B) + wave;
        if (ib < K) issue(ib);
        uint32_t y[4];  // slots past K hold stale bytes and are not used
#pragma unroll
        for (int j = 0; j < 4; ++j) y[j] = ring[((4 * b + j) % RING_SLOTS) * 256 + threadIdx.x];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = 4 * b + j;
            if (i < K) m16_v1_step<ABL>(y[j], rec + size_t(i) * 64, plane, a0, a1, a2, a3);
        }
        wait_mine(mine(b + 2, b + RING_B));
        asm volatile("s_barrier" ::: "memory");
    }
    const int rows = min(64, Rp - tile * 64);
    if (a.kslices > 1) {  // partial products: [slice][stripe][tile * 64 + p][chunk dwords]
        const int64_t nloc = a.units ? a.units / a.nchunks : gridDim.x / a.nchunks;
        const int64_t rpad = int64_t(a.units ? a.tiles : gridDim.y) * 64, cw = a.nchunks * 256;
        uint32_t* part = a.partial + ((slice * nloc + local) * rpad + tile * 64) * cw + (chunk0 >> 2) + threadIdx.x;
#pragma unroll
        for (int p = 0; p < 64; ++p)
            if (p < rows) part[p * cw] = p < 16 ? a0[p & 15] : p < 32 ? a1[p & 15] : p < 48 ? a2[p & 15] : a3[p & 15];
        return;
    }
    uint8_t* dst = a.dst + stripe * a.dst_stripe + chunk0 + int64_t(threadIdx.x) * 4;
#pragma unroll
    for (int p = 0; p < 64; ++p) {
        if (p < rows) {
            const uint32_t v = p < 16 ? a0[p & 15] : p < 32 ? a1[p & 15] : p < 48 ? a2[p & 15] : a3[p & 15];
            *reinterpret_cast<uint32_t*>(dst + int64_t(sload(out_list + tile * 64 + p)) * a.dst_sym) = v;
        }
    }
}

// Split-K reduction: output row `row` of launch-local stripe blockIdx.y, dwords [0, cw) of the full
// 1 KiB chunks = XOR of the kslices partials.
__global__ void __launch_bounds__(256) k_xor_slices(V1Args a, int64_t nloc, int64_t rpad, int64_t cw) {
    const int64_t local = blockIdx.y;
    const int64_t e = int64_t(blockIdx.x) * 256 + threadIdx.x;  // row * cw + dword
    if (e >= int64_t(a.R) * cw) return;
    const int64_t row = e / cw, c = e - row * cw;
    uint32_t v = 0;
    for (int sl = 0; sl < a.kslices; ++sl) v ^= a.partial[((sl * nloc + local) * rpad + row) * cw + c];
    const int64_t stripe = RS_STRIPE(a.ids, local);
    *reinterpret_cast<uint32_t*>(a.dst + stripe * a.dst_stripe + int64_t(a.out_idx[row]) * a.dst_sym + 4 * c) = v;
}

// ------------------------------------------------------------------------ synthetic inputs
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Information region of stripe s = k symbols of S bytes; byte b = byte (b & 7) of
// mix64(seed ^ s*G ^ (b>>3)*Q + G)  (tests/_util.py:gen_info, oracle/gen_golden.c:gen_byte).
__global__ void k_gen_info(uint8_t* base, int64_t stripe_stride, int64_t sym_stride, int64_t S, int64_t words_per_stripe,
                           int64_t stripe0, int64_t n_stripes, uint64_t seed) {
    const int64_t total = words_per_stripe * n_stripes;
    for (int64_t g = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; g < total; g += int64_t(gridDim.x) * blockDim.x) {
        const int64_t s = g / words_per_stripe;
        const int64_t q = g - s * words_per_stripe;
        const uint64_t x = seed ^ (uint64_t(stripe0 + s) * 0x9E3779B97F4A7C15ull) ^ (uint64_t(q) * 0xC2B2AE3D27D4EB4Full);
        const uint64_t v = mix64(x + 0x9E3779B97F4A7C15ull);
        const int64_t b = q * 8, sym = b / S, off = b - sym * S;
        *reinterpret_cast<uint64_t*>(base + s * stripe_stride + sym * sym_stride + off) = v;
    }
}

// Order-independent, position-sensitive 64-bit fingerprint of symbols [sym0, sym0+nsym) of each
// stripe (S % 8 == 0): out[s] ^= mix64(word ^ mix64(sym << 40 | offset)).
__global__ void k_fingerprint(const uint8_t* base, int64_t stripe_stride, int64_t sym_stride, int64_t S, int sym0,
                              int nsym, int64_t n_stripes, unsigned long long* out) {
    const int64_t wps = (S / 8) * nsym;
    const int64_t s = blockIdx.y;
    if (s >= n_stripes) return;
    uint64_t h = 0;
    for (int64_t q = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; q < wps; q += int64_t(gridDim.x) * blockDim.x) {
        const int64_t sym = q / (S / 8), off = (q - sym * (S / 8)) * 8;
        const uint64_t w = *reinterpret_cast<const uint64_t*>(base + s * stripe_stride + (sym0 + sym) * sym_stride + off);
        h ^= mix64(w ^ mix64((uint64_t(sym0 + sym) << 40) | uint64_t(off)));
    }
    for (int o = 32; o > 0; o >>= 1) h ^= __shfl_xor(h, o);
    if ((threadIdx.x & 63) == 0) atomicXor(out + s, (unsigned long long)h);
}

// ------------------------------------------- m = 16 cyclotomic syndromes (k_cs16, gen_asm.py cs16a/b)
// Block = 4 waves on one 1 KiB column chunk of one stripe (one dword per lane), one tile of 4 syndrome
// cosets (64 accumulators per lane; 152 VGPRs, 3 waves per SIMD). Per input group (a cyclotomic coset
// of up to 16 slots) the step builds four subset tables and runs 4 x 16 gpr-index switches, each feeding
// four XORs (the circulant structure of alpha^(s L 2^a), see gen_asm.py), and loads the next group's
// inputs with raw buffer loads (empty slots read out of range, i.e. zero). Then the needed syndromes of
// each coset, S_(s 2^b) = sum_t nb_((t + b) mod 16) * u_t, are formed with log / exp gathers and stored.
typedef uint32_t u32x4s __attribute__((ext_vector_type(4)));

#define RS_CS16_OPERANDS                                                                                      \
    : "+{v[72:87]}"(a0), "+{v[88:103]}"(a1), "+{v[104:119]}"(a2), "+{v[120:135]}"(a3), "+{v[8:23]}"(T0),        \
      "+{v[24:39]}"(T1), "+{v[40:55]}"(T2), "+{v[56:71]}"(T3), "+{v[136:151]}"(ld), "+{s[40:55]}"(ra),           \
      "+{s[56:71]}"(rb), "+{s[76:91]}"(goff), [t0] "=&v"(t0), [t1] "=&v"(t1)                                     \
    : [cp] "s"(cp), [gp] "s"(gp), [rsrc] "s"(rsrc), [lane] "v"(lane)                                           \
    : "s72", "s73", "memory"

// one group step; B selects the record buffer (A: this record in s[40:55], B: in s[56:71])
template <bool B>
__device__ __forceinline__ void cs16_step(const uint32_t* cp, const uint32_t* gp, u32x4s rsrc, uint32_t lane,
                                          u32x16& ld, u32x16& ra, u32x16& rb, u32x16& goff, u32x16& T0, u32x16& T1,
                                          u32x16& T2, u32x16& T3, u32x16& a0, u32x16& a1, u32x16& a2, u32x16& a3) {
    uint32_t t0, t1;
    if constexpr (!B) {
        asm volatile(
#include "gen/m8_idx_asm_cs16a.inc"
            RS_CS16_OPERANDS);
    } else {
        asm volatile(
#include "gen/m8_idx_asm_cs16b.inc"
            RS_CS16_OPERANDS);
    }
}
#undef RS_CS16_OPERANDS

// S = sum_t nb_((t + B) mod 16) * u_t on both packed words, without tables: nb_k = sum_q bit_q(nb_k) alpha^q,
// so S = sum_q alpha^q w_q with w_q = XOR of the u_t whose nb_((t + B) mod 16) has bit q (a fixed XOR
// network for each B), then Horner in alpha over q (x * alpha on packed words: shift, carry * 0x2D).
// nb = the GF(2^16) normal basis of reference gf65536.c:21-57 (facts).
__device__ constexpr uint16_t kNb16[16] = {2048, 2880, 7129, 30616, 2643, 6897, 29685, 7378,
                                           30100, 2743, 20193, 36223, 24055, 41458, 41014, 61451};

template <int B>
__device__ __forceinline__ uint32_t nb_combine(const u32x16& u) {
    uint32_t w[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        w[q] = 0;
#pragma unroll
        for (int t = 0; t < 16; ++t)
            if ((kNb16[(t + B) & 15] >> q) & 1) w[q] ^= u[t];
    }
    uint32_t s = w[15];
#pragma unroll
    for (int q = 14; q >= 0; --q) s = (((s << 1) & 0xFFFEFFFEu) ^ (((s >> 15) & 0x10001u) * 0x2Du)) ^ w[q];
    return s;
}

// needed syndromes / outputs of local coset c from its 16 accumulators u (both words of the lane's dword)
__device__ __forceinline__ void cs16_finish(const Cs16Args& a, const u32x16& u, int c, int tile, uint8_t* out) {
    const int e0 = sload(a.fin_off + tile * (a.cw + 1) + c), e1 = sload(a.fin_off + tile * (a.cw + 1) + c + 1);
    for (int e = e0; e < e1; ++e) {
        const int32_t ent = sload(a.fin + int64_t(tile) * a.fin_stride + e);
        const int64_t j = ent >> 8;
        uint32_t v = 0;
        switch ((ent >> 4) & 15) {  // wave-uniform
        case 0: v = nb_combine<0>(u); break;
        case 1: v = nb_combine<1>(u); break;
        case 2: v = nb_combine<2>(u); break;
        case 3: v = nb_combine<3>(u); break;
        case 4: v = nb_combine<4>(u); break;
        case 5: v = nb_combine<5>(u); break;
        case 6: v = nb_combine<6>(u); break;
        case 7: v = nb_combine<7>(u); break;
        case 8: v = nb_combine<8>(u); break;
        case 9: v = nb_combine<9>(u); break;
        case 10: v = nb_combine<10>(u); break;
        case 11: v = nb_combine<11>(u); break;
        case 12: v = nb_combine<12>(u); break;
        case 13: v = nb_combine<13>(u); break;
        case 14: v = nb_combine<14>(u); break;
        default: v = nb_combine<15>(u); break;
        }
        *reinterpret_cast<uint32_t*>(out + j * a.dst_sym) = v;
    }
}

// Block -> (tile, launch-local stripe, lane's column byte) of k_cs16 / k_bs16; false: nothing to do.
// XCD-aware: consecutive slots on one XCD (workgroup b runs on XCD b % 8) walk the tiles of one unit.
// colw 1024: block = 4 waves on the four 256-byte quarters of a 1 KiB unit, one tile per block.
// colw 256: every wave is one (256-byte unit, tile) pair of the flattened sequence unit * ntiles +
// tile, 4 consecutive pairs per block (no idle waves when ntiles % 4 != 0), and XCD x runs the
// contiguous 1/8 of the blocks [x nb / 8, (x + 1) nb / 8) in order (nb = gridDim.x, a multiple of 8): the
// ~32 blocks of a unit run together on one XCD and sweep its input groups in step, so the XCD's L2
// serves the repeats.
__device__ __forceinline__ bool cs16_unit(const Cs16Args& a, int& tile, int64_t& local, uint32_t& col) {
    const int64_t slot = blockIdx.x >> 3;
    int64_t unit;
    if (a.colw == 1024) {
        tile = int(slot % a.ntiles);
        unit = (slot / a.ntiles) * 8 + (blockIdx.x & 7);
        col = uint32_t(threadIdx.x * 4u);
    } else {
        const int64_t lb = int64_t(blockIdx.x & 7) * (gridDim.x >> 3) + slot;
        const int64_t wv = lb * 4 + __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
        unit = wv / a.ntiles;
        tile = int(wv - unit * a.ntiles);
        col = uint32_t((threadIdx.x & 63u) * 4u);
    }
    if (unit >= a.units || tile >= a.ntiles) return false;
    local = unit / a.nchunks;
    col += uint32_t((unit - local * a.nchunks) * a.colw);
    return true;
}

__global__ void __launch_bounds__(256) k_cs16(Cs16Args a) {
    int tile;
    int64_t local;
    uint32_t col;
    if (!cs16_unit(a, tile, local, col)) return;
    const int64_t stripe = RS_STRIPE(a.ids, local);
    const uint64_t base = uint64_t(reinterpret_cast<uintptr_t>(a.src + stripe * a.src_stripe));
    // raw buffer V#: base, stride 0, num_records = the inputs' byte range, 32-bit data format
    const u32x4s rsrc = {uint32_t(base), uint32_t(base >> 32) & 0xFFFFu, a.in_bytes, 0x20000u};
    const uint32_t* rec = a.rec + size_t(tile) * size_t(a.ngroups + 2) * 16;  // [tile][ngroups + 2][16]
    const uint32_t* goffs = a.goff;  // [ngroups + 3][16] slot byte offsets (0x80000000 = empty)
    u32x16 a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    u32x16 T0 = 0, T1 = 0, T2 = 0, T3 = 0;  // entry 0 of each table stays zero
    u32x16 ld, ra, rb, goff;
    uint32_t t0;
    // prologue: group 0's inputs in flight, group 1's offsets and group 0's record requested
    asm volatile(
#include "gen/m8_idx_asm_cs16_pro.inc"
        : "=&{v[136:151]}"(ld), "=&{s[76:91]}"(goff), "=&{s[40:55]}"(ra), [t0] "=&v"(t0)
        : [g0] "s"(goffs), [r0] "s"(rec), [rsrc] "s"(rsrc), [lane] "v"(col)
        : "memory");
    rb = 0;
    for (int g = 0; g < a.ngroups; g += 2) {  // ngroups is padded to even on the host
        cs16_step<false>(rec + size_t(g) * 16, goffs + size_t(g + 2) * 16, rsrc, col, ld, ra, rb, goff, T0, T1, T2,
                         T3, a0, a1, a2, a3);
        cs16_step<true>(rec + size_t(g + 1) * 16, goffs + size_t(g + 3) * 16, rsrc, col, ld, ra, rb, goff, T0, T1,
                        T2, T3, a0, a1, a2, a3);
    }
    // the last step's prefetches (padding group / records) must land before these registers are reused
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)"
                 : "+{v[136:151]}"(ld), "+{s[40:55]}"(ra), "+{s[56:71]}"(rb), "+{s[76:91]}"(goff)
                 :
                 : "memory");
    uint8_t* out = a.dst + local * a.dst_stripe + col;
    cs16_finish(a, a0, 0, tile, out);
    cs16_finish(a, a1, 1, tile, out);
    cs16_finish(a, a2, 2, tile, out);
    cs16_finish(a, a3, 3, tile, out);
}

// k_cs16t: k_cs16 without gpr-indexed VALU (gen_asm.py cs16t_kernel). The circulant of each (group,
// syndrome coset) is run as four code blocks chosen by z's nibbles, XORing raw inputs into fixed
// accumulator registers at full rate; the blocks are threaded by code offsets in the records
// ([tile][ngroups + 2][16] uint32, block p = 4c + n of the step). Tiles of kCs16tCw = 4 cosets, no
// subset tables and no load ring: 16 inputs + 16 pair sums + 64 accumulators = v[0:95], 5 waves per
// SIMD to cover each wave's jumps and loads (the lane's column is recomputed per step from its id). The whole group loop is one asm statement: between steps, scalar
// and vector loads are still filling the record, slot-offset and input registers, which
// compiler-visible code must never copy. Same block layout and finish as k_cs16.
#if RS_CS16T_R2 && RS_CS16T_CW == 4
static_assert(kCs16tF == 0 && kCs16tR == 16 && kCs16tAcc == 32, "k_cs16t's register operands");
#define RS_CS16T_WAVES 5
#elif RS_CS16T_R2 && RS_CS16T_CW == 3  // inputs + pair sums + 48 accumulators = v[0:79], 6 waves
static_assert(kCs16tF == 0 && kCs16tR == 16 && kCs16tAcc == 32, "k_cs16t's register operands");
#define RS_CS16T_WAVES 6
#else  // raw inputs only: 16 inputs + 64 accumulators = v[0:79], 6 waves per SIMD
static_assert(kCs16tCw == 4 && kCs16tF == 0 && kCs16tAcc == 16, "k_cs16t's register operands");
#define RS_CS16T_WAVES 6
#endif

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RS_CS16T_WAVES))) k_cs16t(Cs16Args a) {
    int tile;
    int64_t local;
    uint32_t col;
    if (!cs16_unit(a, tile, local, col)) return;
    const int64_t stripe = RS_STRIPE(a.ids, local);
    const uint64_t sbase = uint64_t(reinterpret_cast<uintptr_t>(a.src + stripe * a.src_stripe));
    const u32x4s rsrc = {uint32_t(sbase), uint32_t(sbase >> 32) & 0xFFFFu, a.in_bytes, 0x20000u};
    const uint32_t* rec = a.rec + size_t(tile) * size_t(a.ngroups + 2) * (4 * kCs16tCw);  // [tile][ngroups + 2][4 cw]
    const uint32_t* goffs = a.goff;                                                      // [ngroups + 3][16]
    // the wave's byte column (lane 0's); every VGPR is taken inside the loop, so the lanes' columns are
    // formed there from their ids, and again here after it
    const uint32_t colbase = __builtin_amdgcn_readfirstlane(col - (threadIdx.x & 63u) * 4u);
    u32x16 a0 = 0, a1 = 0, a2 = 0;
#if RS_CS16T_CW == 4
    u32x16 a3 = 0;
#endif
    asm volatile(
#include "gen/m8_idx_asm_cs16t_kernel.inc"
#if RS_CS16T_R2 && RS_CS16T_CW == 4
        : "+{v[32:47]}"(a0), "+{v[48:63]}"(a1), "+{v[64:79]}"(a2), "+{v[80:95]}"(a3)
#elif RS_CS16T_R2
        : "+{v[32:47]}"(a0), "+{v[48:63]}"(a1), "+{v[64:79]}"(a2)
#else
        : "+{v[16:31]}"(a0), "+{v[32:47]}"(a1), "+{v[48:63]}"(a2), "+{v[64:79]}"(a3)
#endif
        : [g0] "s"(goffs), [g2] "s"(goffs + 32), [r0] "s"(rec), [ng] "s"(a.ngroups), [rsrc] "s"(rsrc),
          [colbase] "s"(colbase)
        : "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15",
#if RS_CS16T_R2
          "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31",
#endif
          "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55",
          "s72", "s73", "s74", "s75", "s76", "s77", "s78", "s79", "s80", "s81", "s82", "s83", "s84", "s85", "s86", "s87",
          "s88", "s89", "s90", "s91", "s92", "s93", "s94", "s95", "s96", "s97", "s98", "scc", "memory");
    const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    uint8_t* out = a.dst + local * a.dst_stripe + (colbase + lane * 4u);
    cs16_finish(a, a0, 0, tile, out);
    cs16_finish(a, a1, 1, tile, out);
    cs16_finish(a, a2, 2, tile, out);
#if RS_CS16T_CW == 4
    cs16_finish(a, a3, 3, tile, out);
#endif
}

// m = 16 binary accumulation (k_bs16, gen_asm.py bs16): the syndrome route's encode second stage. Same
// block / tile / input scheme as k_cs16 (the inputs are the D syndromes of a stripe, 16 per group), but
// every (coset, table, accumulator) has its own gpr-index switch: the coefficients S_j -> output coset
// are Frobenius-structured along the coset (finish as k_cs16), not along the inputs.
__device__ __forceinline__ void bs16_step(const uint32_t* cp, const uint32_t* gp, u32x4s rsrc, uint32_t lane,
                                          u32x16& ld, u32x16& ra, u32x16& rb, u32x16& goff, u32x16& T0, u32x16& T1,
                                          u32x16& T2, u32x16& T3, u32x16& a0, u32x16& a1, u32x16& a2, u32x16& a3) {
    uint32_t t0, t1;
    asm volatile(
#include "gen/m8_idx_asm_bs16.inc"
        : "+{v[72:87]}"(a0), "+{v[88:103]}"(a1), "+{v[104:119]}"(a2), "+{v[120:135]}"(a3), "+{v[8:23]}"(T0),
          "+{v[24:39]}"(T1), "+{v[40:55]}"(T2), "+{v[56:71]}"(T3), "+{v[136:151]}"(ld), "+{s[40:55]}"(ra),
          "+{s[56:71]}"(rb), "+{s[76:91]}"(goff), [t0] "=&v"(t0), [t1] "=&v"(t1)
        : [cp] "s"(cp), [gp] "s"(gp), [rsrc] "s"(rsrc), [lane] "v"(lane)
        : "s72", "s73", "memory");
}

__global__ void __launch_bounds__(256) k_bs16(Cs16Args a) {
    int tile;
    int64_t local;
    uint32_t col;
    if (!cs16_unit(a, tile, local, col)) return;
    const int64_t stripe = RS_STRIPE(a.ids, local);
    const uint64_t base = uint64_t(reinterpret_cast<uintptr_t>(a.src + stripe * a.src_stripe));
    const u32x4s rsrc = {uint32_t(base), uint32_t(base >> 32) & 0xFFFFu, a.in_bytes, 0x20000u};
    const uint32_t* rec = a.rec + size_t(tile) * size_t(a.ngroups + 2) * 64;  // [tile][ngroups + 2][4][16]
    const uint32_t* goffs = a.goff;
    u32x16 a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    u32x16 T0 = 0, T1 = 0, T2 = 0, T3 = 0;
    u32x16 ld, ra, rb, goff;
    uint32_t t0;
    asm volatile(
#include "gen/m8_idx_asm_cs16_pro.inc"
        : "=&{v[136:151]}"(ld), "=&{s[76:91]}"(goff), "=&{s[40:55]}"(ra), [t0] "=&v"(t0)
        : [g0] "s"(goffs), [r0] "s"(rec), [rsrc] "s"(rsrc), [lane] "v"(col)
        : "memory");
    rb = 0;
    for (int g = 0; g < a.ngroups; ++g)
        bs16_step(rec + size_t(g) * 64, goffs + size_t(g + 2) * 16, rsrc, col, ld, ra, rb, goff, T0, T1, T2, T3, a0, a1,
                  a2, a3);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)"
                 : "+{v[136:151]}"(ld), "+{s[40:55]}"(ra), "+{s[56:71]}"(rb), "+{s[76:91]}"(goff)
                 :
                 : "memory");
    uint8_t* out = a.dst + stripe * a.dst_stripe + col;  // outputs go to the caller's stripes
    cs16_finish(a, a0, 0, tile, out);
    cs16_finish(a, a1, 1, tile, out);
    cs16_finish(a, a2, 2, tile, out);
    cs16_finish(a, a3, 3, tile, out);
}

hipError_t launch_cs16t(const Cs16Args& a, hipStream_t st) {
    if (a.units <= 0 || a.ntiles <= 0) return hipSuccess;
    const int64_t blocks = a.colw == 1024 ? (a.units + 7) / 8 * 8 * a.ntiles : (a.units * a.ntiles + 31) / 32 * 8;
    if (blocks > int64_t(0x7fffffff)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_cs16t, dim3(unsigned(blocks)), dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_bs16(const Cs16Args& a, hipStream_t st) {
    if (a.units <= 0 || a.ntiles <= 0) return hipSuccess;
    const int64_t blocks = a.colw == 1024 ? (a.units + 7) / 8 * 8 * a.ntiles : (a.units * a.ntiles + 31) / 32 * 8;
    if (blocks > int64_t(0x7fffffff)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_bs16, dim3(unsigned(blocks)), dim3(256), 0, st, a);
    return hipGetLastError();
}

// slot lists -> byte offsets for k_cs16 (slot * sym; -1 -> 0x80000000, out of the V#'s range)
__global__ void k_cs16_goff(const int32_t* slots, uint32_t* goff, int n, int64_t sym) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) goff[i] = slots[i] < 0 ? 0x80000000u : uint32_t(int64_t(slots[i]) * sym);
}

hipError_t launch_cs16_goff(const int32_t* slots, uint32_t* goff, int n, int64_t sym, hipStream_t st) {
    hipLaunchKernelGGL(k_cs16_goff, dim3(unsigned((n + 255) / 256)), dim3(256), 0, st, slots, goff, n, sym);
    return hipGetLastError();
}

hipError_t launch_cs16(const Cs16Args& a, hipStream_t st) {
    if (a.units <= 0 || a.ntiles <= 0) return hipSuccess;
    const int64_t blocks = a.colw == 1024 ? (a.units + 7) / 8 * 8 * a.ntiles : (a.units * a.ntiles + 31) / 32 * 8;
    if (blocks > int64_t(0x7fffffff)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_cs16, dim3(unsigned(blocks)), dim3(256), 0, st, a);
    return hipGetLastError();
}

// ---------------------------------------------------- symbol-wide ops (gf_add / gf_mul / gf_madd)
// Eight words (16 bytes) per lane, reference src/rs/gf65536.c:155-219: add a ^= b; mul a = c * a; madd
// a ^= c * b, products through the log / exp tables with zero words skipped (lc = log c, c != 0, 1).
// nw is a multiple of 8 (the callers' staging is padded with zero words: a zero word of b adds nothing,
// a zero word of a stays zero under mul); 16-byte accesses also suit operands read across PCIe.
__global__ void __launch_bounds__(256) k_symbol_op(uint16_t* a, const uint16_t* b, int op, uint32_t lc, int64_t nw,
                                                   const uint16_t* __restrict__ logt, const uint16_t* __restrict__ expt) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const int64_t nu = nw / 8;
    for (int64_t u = int64_t(blockIdx.x) * 256 + threadIdx.x; u < nu; u += int64_t(gridDim.x) * 256) {
        u32x4 va = reinterpret_cast<u32x4*>(a)[u];
        const u32x4 src = op == 1 ? va : reinterpret_cast<const u32x4*>(b)[u];
        u32x4 v = src;
        if (op != 0) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                uint32_t r = 0;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const uint32_t x = (src[q] >> (16 * h)) & 0xFFFFu;
                    if (x) {
                        const uint32_t e = logt[x] + lc;
                        r |= uint32_t(expt[e >= 65535u ? e - 65535u : e]) << (16 * h);
                    }
                }
                v[q] = r;
            }
        }
        reinterpret_cast<u32x4*>(a)[u] = op == 1 ? v : (va ^ v);
    }
}

hipError_t launch_symbol_op(uint16_t* a, const uint16_t* b, int op, uint32_t lc, int64_t nw, const uint16_t* logt,
                            const uint16_t* expt, hipStream_t st) {
    if (nw <= 0) return hipSuccess;
    if (nw % 8 || (uintptr_t(a) | uintptr_t(b)) % 16) return hipErrorInvalidValue;
    const unsigned grid = unsigned(std::min<int64_t>((nw / 8 + 255) / 256, 4096));
    hipLaunchKernelGGL(k_symbol_op, dim3(grid), dim3(256), 0, st, a, b, op, lc, nw, logt, expt);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------ launchers
V1Args v1_args(const ApplyArgs& a, int64_t nchunks_1k, const int32_t* boff) {
    V1Args v{};
    v.src = a.src;
    v.src_stripe = a.src_stripe;
    v.src_sym = a.src_sym;
    v.in_idx = a.in_idx;
    v.dst = a.dst;
    v.dst_stripe = a.dst_stripe;
    v.dst_sym = a.dst_sym;
    v.out_idx = a.out_idx;
    v.ltab = a.ltab;
    v.idx = a.idx;
    v.boff = boff;
    v.K = a.K;
    v.R = a.R;
    v.nchunks = nchunks_1k;
    v.ids = a.ids;
    v.nslots = a.nslots;
    v.slot_err = a.slot_err;
    return v;
}

// Columns past the last full 2 KiB chunk of every symbol (rows of all tiles), register-ring kernel.
void launch_m8_tail(const ApplyArgs& a, int64_t n_stripes, unsigned tiles, hipStream_t st) {
    if (a.nbytes % 2048 == 0) return;
    ApplyArgs t = a;
    t.chunk_base = a.nbytes / 2048;
    t.nchunks = 1;
    hipLaunchKernelGGL((k_apply_m8_idx<0, 4>), dim3(unsigned(n_stripes), tiles), dim3(256), 0, st, t, a.in_idx);
}

template <int RT>
static hipError_t launch_m8(const ApplyArgs& a, int64_t n_stripes, hipStream_t st) {
    dim3 grid(unsigned(n_stripes * a.nchunks), unsigned((a.R + RT - 1) / RT));
    // Release build: the generic GF(256) kernels are the V = 1 ones (mode 20: one nibble table per input,
    // k_apply_m8_v1<2>, the default; mode 18: two tables, k_apply_m8_v1<0>, the per-stripe solve's kernel)
    // and the register-ring tail kernel. Every other family is an option-only A/B or ablation and lives in
    // the diagnostic build (make diag): 0 / 1 compiler-indexed table / SGPR-mask kernels, 2 the LDS-DMA
    // kernel, 3 / 4 register ring 4 / 8 over whole symbols, 10..17 LDS-DMA ablations and stamps, 19 / 21 V = 1
    // ablation and stamps.
    if (RT == 32 && a.idx && (a.mode == 18 || a.mode == 19 || a.mode == 20 || a.mode == 21)) {
        const int64_t full = (a.nbytes / 2048) * 2;  // 1 KiB chunks up to the last full 2 KiB boundary
        if (full > 0) {
            V1Args v = v1_args(a, full, nullptr);
            v.kslices = a.mode != 19 && a.mode != 21 ? m8_kslices(a, n_stripes, nullptr) : 1;
            v.stamps = a.stamps;
            v.partial = a.scratch;
            dim3 g(unsigned(n_stripes * full), grid.y, unsigned(v.kslices));
#ifdef RS_AMD_DIAG
            if (a.mode == 19)
                hipLaunchKernelGGL((k_apply_m8_v1<1>), g, dim3(256), 0, st, v);
            else if (a.mode == 21)
                hipLaunchKernelGGL((k_apply_m8_v1<5>), g, dim3(256), 0, st, v);
            else
#else
            if (a.mode == 19 || a.mode == 21) return hipErrorInvalidValue;
#endif
            if (a.mode == 20)
                hipLaunchKernelGGL((k_apply_m8_v1<2>), g, dim3(256), 0, st, v);
            else
                hipLaunchKernelGGL((k_apply_m8_v1<0>), g, dim3(256), 0, st, v);
            if (v.kslices > 1) {
                const int64_t cw = full * 256, rows = int64_t(a.R) * cw;
                hipLaunchKernelGGL(k_xor_slices, dim3(unsigned((rows + 255) / 256), unsigned(n_stripes)), dim3(256),
                                   0, st, v, int64_t(n_stripes), int64_t(grid.y) * 32, cw);
            }
        }
        launch_m8_tail(a, n_stripes, grid.y, st);
        return hipGetLastError();
    }
#ifdef RS_AMD_DIAG
    if (RT == 32 && a.mode >= 2 && a.idx) {
        // mode 2: LDS-DMA ring over full chunks + register-ring tail; 3 / 4: register ring 4 / 8 only;
        // 10..16: the LDS-DMA kernel with asm variant ABL = mode - 9 (timing ablations, wrong results except
        // 14 = "full" schedule): 10 no index switching, 11 multiples + tables only, 12 lookups only, 13 loads
        // only, 14 split schedule with the multiply-based xtime, 15 no gpr-index mode; 17 stamps
        if (a.mode == 2 || (a.mode >= 10 && a.mode <= 15) || a.mode == 17) {
            ApplyArgs f = a;
            f.nchunks = a.nbytes / 2048;
            if (f.nchunks > 0) {
                dim3 g(unsigned(n_stripes * f.nchunks), grid.y);
                switch (a.mode) {
                case 14: hipLaunchKernelGGL((k_apply_m8_lds<5>), g, dim3(256), 0, st, f, a.in_idx); break;
                case 10: hipLaunchKernelGGL((k_apply_m8_lds<1>), g, dim3(256), 0, st, f, a.in_idx); break;
                case 11: hipLaunchKernelGGL((k_apply_m8_lds<2>), g, dim3(256), 0, st, f, a.in_idx); break;
                case 12: hipLaunchKernelGGL((k_apply_m8_lds<3>), g, dim3(256), 0, st, f, a.in_idx); break;
                case 13: hipLaunchKernelGGL((k_apply_m8_lds<4>), g, dim3(256), 0, st, f, a.in_idx); break;
                case 15: hipLaunchKernelGGL((k_apply_m8_lds<6>), g, dim3(256), 0, st, f, a.in_idx); break;
                case 17:  // the LDS-DMA kernel with s_memtime phase counters (needs a.stamps)
                    if (!a.stamps) return hipErrorInvalidValue;
                    hipLaunchKernelGGL((k_apply_m8_lds<0, true>), g, dim3(256), 0, st, f, a.in_idx);
                    break;
                default: hipLaunchKernelGGL((k_apply_m8_lds<0>), g, dim3(256), 0, st, f, a.in_idx); break;
                }
            }
            if (a.nbytes % 2048) {
                ApplyArgs t = a;
                t.chunk_base = f.nchunks;
                t.nchunks = 1;
                dim3 g(unsigned(n_stripes), grid.y);
                hipLaunchKernelGGL((k_apply_m8_idx<0, 4>), g, dim3(256), 0, st, t, a.in_idx);
            }
        } else if (a.mode == 4) {
            hipLaunchKernelGGL((k_apply_m8_idx<0, 8>), grid, dim3(256), 0, st, a, a.in_idx);
        } else if (a.mode == 16) {  // loads only, register ring 4 (timing ablation, wrong results)
            hipLaunchKernelGGL((k_apply_m8_idx<4, 4>), grid, dim3(256), 0, st, a, a.in_idx);
        } else {
            hipLaunchKernelGGL((k_apply_m8_idx<0, 4>), grid, dim3(256), 0, st, a, a.in_idx);
        }
    } else if (a.mode == 1)
        hipLaunchKernelGGL((k_apply_m8<RT, 1>), grid, dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL((k_apply_m8<RT, 0>), grid, dim3(256), 0, st, a);
    return hipGetLastError();
#else
    return hipErrorInvalidValue;  // no other generic GF(256) family in the release build
#endif
}

template <int RT>
static hipError_t launch_m16(const ApplyArgs& a, int64_t n_stripes, hipStream_t st) {
    if (RT == 64 && a.idx && (a.mode == 0 || a.mode == 1)) {
        // hand-scheduled kernel over the full 1 KiB chunks (mode 1: fixed-register timing ablation),
        // the compiled kernel over the rest of each symbol
        const int64_t full = a.nbytes / 1024;
        const unsigned tiles = unsigned((a.R + 63) / 64);
        if (full > 0) {
            V1Args v = v1_args(a, full, nullptr);
            v.kslices = m16_kslices(a, n_stripes, nullptr);
            v.partial = a.scratch;
            // XCD-aware order only with units to spread over all 8 XCDs (a single stripe's tiles and
            // slices would otherwise all land on one XCD)
            const int64_t units = n_stripes * full;
            v.units = (v.kslices == 1 && units >= 64) ? units : 0;
            v.tiles = int(tiles);
            dim3 g = v.units ? dim3(unsigned((units + 7) / 8 * 8 * tiles), 1, 1)
                             : dim3(unsigned(units), tiles, unsigned(v.kslices));
#ifdef RS_AMD_DIAG
            if (a.mode == 1)  // fixed-register timing ablation (wrong results)
                hipLaunchKernelGGL((k_apply_m16_v1<1>), g, dim3(256), 0, st, v);
            else
#endif
                hipLaunchKernelGGL((k_apply_m16_v1<0>), g, dim3(256), 0, st, v);
            if (v.kslices > 1) {
                const int64_t cw = full * 256, rows = int64_t(a.R) * cw;
                hipLaunchKernelGGL(k_xor_slices, dim3(unsigned((rows + 255) / 256), unsigned(n_stripes)), dim3(256), 0,
                                   st, v, int64_t(n_stripes), int64_t(tiles) * 64, cw);
            }
        }
        if (a.nbytes % 1024) {
            ApplyArgs t = a;
            t.chunk_base = full;
            t.nchunks = 1;
            hipLaunchKernelGGL(k_apply_m16<64>, dim3(unsigned(n_stripes), tiles), dim3(256), 0, st, t);
        }
        return hipGetLastError();
    }
    dim3 grid(unsigned(n_stripes * a.nchunks), unsigned((a.R + RT - 1) / RT));
    hipLaunchKernelGGL(k_apply_m16<RT>, grid, dim3(256), 0, st, a);
    return hipGetLastError();
}

int m16_kslices(const ApplyArgs& a, int64_t n_stripes, int64_t* scratch_bytes) {
    // split K when the grid would leave most CUs idle (one workgroup walks all K inputs serially):
    // aim for >= 512 workgroups, slices of >= 64 inputs, at most 32 slices, within the scratch
    // (RS_AMD_KSLICES overrides the slice cap for experiments; target = 16 workgroups per slice cap)
    static const int64_t cap = [] {
        const char* e = std::getenv("RS_AMD_KSLICES");
        const long v = e ? std::atol(e) : 32;
        return int64_t(v >= 2 && v <= 256 ? v : 32);
    }();
    const int64_t full = a.nbytes / 1024, tiles = (a.R + 63) / 64;
    const int64_t blocks = n_stripes * full * tiles;
    if (blocks <= 0 || blocks >= 256) return 1;
    int64_t s = std::min<int64_t>({(16 * cap + blocks - 1) / blocks, int64_t(a.K) / 64, cap});
    const int64_t per = n_stripes * tiles * 64 * full * 1024;  // partial bytes per slice
    if (!scratch_bytes) s = std::min<int64_t>(s, per > 0 ? a.scratch_bytes / per : 0);
    if (s < 2) return 1;
    if (scratch_bytes) *scratch_bytes = s * per;
    return int(s);
}

int m8_kslices(const ApplyArgs& a, int64_t n_stripes, int64_t* scratch_bytes) {
    // the generic V = 1 kernel on small grids (e.g. one 64 KiB stripe of a per-call decode before its
    // pattern is specialised: 64 workgroups each walking all K inputs): up to 16 input slices of >= 16
    // inputs, aiming for >= 512 workgroups, within the scratch
    const int64_t full = (a.nbytes / 2048) * 2, tiles = (a.R + 31) / 32;
    const int64_t blocks = n_stripes * full * tiles;
    if (blocks <= 0 || blocks >= 256 || a.ids) return 1;
    int64_t s = std::min<int64_t>({(512 + blocks - 1) / blocks, int64_t(a.K) / 16, 16});
    const int64_t per = n_stripes * tiles * 32 * full * 1024;  // partial bytes per slice
    if (!scratch_bytes) s = std::min<int64_t>(s, per > 0 ? a.scratch_bytes / per : 0);
    if (s < 2) return 1;
    if (scratch_bytes) *scratch_bytes = s * per;
    return int(s);
}

int apply_tile_rows(int m, int R) {
    if (m <= 8) return R <= 4 ? 4 : R <= 8 ? 8 : R <= 16 ? 16 : 32;
    return R <= 16 ? 16 : R <= 32 ? 32 : 64;  // 64 measured best for C5 (RT 32: -3 %, RT 16: -22 %)
}

int64_t apply_chunk_bytes(int m) { return m <= 8 ? 2048 : 1024; }

hipError_t launch_apply(int m, int rt, ApplyArgs a, int64_t n_stripes, hipStream_t st) {
    a.nchunks = (a.nbytes + apply_chunk_bytes(m) - 1) / apply_chunk_bytes(m);
    if (n_stripes <= 0 || a.R <= 0 || a.nchunks == 0) return hipSuccess;
    if (m <= 8) {
        switch (rt) {
        case 4: return launch_m8<4>(a, n_stripes, st);
        case 8: return launch_m8<8>(a, n_stripes, st);
        case 16: return launch_m8<16>(a, n_stripes, st);
        case 32: return launch_m8<32>(a, n_stripes, st);
        }
    } else {
        switch (rt) {
        case 16: return launch_m16<16>(a, n_stripes, st);
        case 32: return launch_m16<32>(a, n_stripes, st);
        case 64: return launch_m16<64>(a, n_stripes, st);
        }
    }
    return hipErrorInvalidValue;
}

hipError_t launch_gen_info(uint8_t* base, int64_t stripe_stride, int64_t sym_stride, int64_t S, int k, int64_t stripe0,
                           int64_t n_stripes, uint64_t seed, hipStream_t st) {
    const int64_t wps = int64_t(k) * S / 8;
    hipLaunchKernelGGL(k_gen_info, dim3(4096), dim3(256), 0, st, base, stripe_stride, sym_stride, S, wps, stripe0,
                       n_stripes, seed);
    return hipGetLastError();
}

hipError_t launch_fingerprint(const uint8_t* base, int64_t stripe_stride, int64_t sym_stride, int64_t S, int sym0,
                              int nsym, int64_t n_stripes, unsigned long long* out, hipStream_t st) {
    hipError_t e = hipMemsetAsync(out, 0, size_t(n_stripes) * 8, st);
    if (e != hipSuccess) return e;
    const int64_t wps = (S / 8) * nsym;
    unsigned gx = unsigned(std::min<int64_t>((wps + 255) / 256, 64));
    hipLaunchKernelGGL(k_fingerprint, dim3(gx, unsigned(n_stripes)), dim3(256), 0, st, base, stripe_stride, sym_stride,
                       S, sym0, nsym, n_stripes, out);
    return hipGetLastError();
}

// ------------------------------------------------------- per-stripe decode plans (m <= 8)
// One workgroup per stripe builds that stripe's decode matrix from the closed form (SURVEY.md a-16,
// same evaluation as gf16.cpp:solve_matrix): with E = erased slots, survivors Q, erased information
// slots P,
//   lp[q] = sum_{e in E} log(X_q + X_e),  ld[p] = sum_{e in E, e != p} log(X_p + X_e),
//   C[p][q] = alpha^(lp[q] - ld[p] - log(X_p + X_q))
// and writes it straight into the V = 1 kernel's form: per (tile, survivor) a 64-dword record of the
// coefficients' gamma-basis nibbles, plus the slot lists and (K, R). Every C[p][q] lies in GF(256), so
// its exponent is a multiple of 257 and g8[exponent / 257] is its gamma-basis byte.
__global__ void __launch_bounds__(256) k_plan_m8(PlanArgs a) {
    __shared__ uint16_t qe[256], ee[256], pe[256];
    __shared__ int32_t qs[256], ps[256];
    __shared__ uint32_t lp[256], ld[256];
    __shared__ int cnt[4][3];
    const int64_t s = blockIdx.x;
    const int j = threadIdx.x, lane = j & 63, w = j >> 6;
    const bool valid = j < a.n;
    const bool er = valid && a.masks[s * a.n + j] != 0;
    const uint64_t be = __ballot(er), bq = __ballot(valid && !er), bp = __ballot(er && j < a.k);
    const uint64_t below = (uint64_t(1) << lane) - 1;
    if (lane == 0) {
        cnt[w][0] = __popcll(be);
        cnt[w][1] = __popcll(bq);
        cnt[w][2] = __popcll(bp);
    }
    __syncthreads();
    int oe = 0, oq = 0, op = 0, t = 0, K = 0, R = 0;
    for (int v = 0; v < 4; ++v) {
        if (v < w) oe += cnt[v][0], oq += cnt[v][1], op += cnt[v][2];
        t += cnt[v][0], K += cnt[v][1], R += cnt[v][2];
    }
    const uint16_t xj = valid ? a.elem[j] : 0;
    if (er) {
        ee[oe + __popcll(be & below)] = xj;
        if (j < a.k) {
            const int i = op + __popcll(bp & below);
            pe[i] = xj;
            ps[i] = j;
        }
    } else if (valid) {
        const int i = oq + __popcll(bq & below);
        qe[i] = xj;
        qs[i] = j;
    }
    __syncthreads();
    constexpr uint32_t N = 65535u;
    for (int q = j; q < K; q += 256) {
        uint32_t acc = 0;
        for (int e = 0; e < t; ++e) acc += a.logt[qe[q] ^ ee[e]];
        lp[q] = acc % N;
    }
    for (int p = j; p < R; p += 256) {
        uint32_t acc = 0;
        for (int e = 0; e < t; ++e)
            if (ee[e] != pe[p]) acc += a.logt[pe[p] ^ ee[e]];  // elements are distinct: skips p itself
        ld[p] = acc % N;
    }
    __syncthreads();
    if (j == 0) {
        a.kr[2 * s] = K;
        a.kr[2 * s + 1] = R;
    }
    int32_t* pin = a.pin + s * a.in_stride;
    for (int q = j; q < a.in_stride; q += 256) pin[q] = q < K ? qs[q] : 0;
    int32_t* pout = a.pout + s * a.out_stride;
    for (int p = j; p < a.out_stride; p += 256) pout[p] = p < R ? ps[p] : 0;
    uint32_t* rec = a.pidx + s * a.idx_stride;
    const int ntiles = (R + 31) / 32;
    for (int e = j; e < ntiles * K * 32; e += 256) {
        const int tile = e / (K * 32), rem = e - tile * K * 32, i = rem >> 5, jj = rem & 31;
        const int row = tile * 32 + jj;
        uint32_t b = 0;
        if (row < R) {
            const uint32_t L = (lp[i] + 2 * N - ld[row] - a.logt[pe[row] ^ qe[i]]) % N;
            b = a.g8[L / 257u];
        }
        uint32_t* r = rec + (size_t(tile) * K + i) * 64;
        r[jj] = b & 15u;
        r[32 + jj] = b >> 4;
    }
}

// Syndrome-route plans (SynPlanArgs). With E the erased slots (t <= r) and P(x) = prod_{e in E}(x + X_e),
// the reference's evaluator / Forney steps (reed_solomon.c:186-336) solve the t x t Vandermonde system
// sum_{e in E} X_e^j d_e = S_j, j < t, over the syndromes of fft_transform_cycl (fft.c:39-100, erased
// slots read as zero). Its inverse is W[p][j] = q_{p,j} / Q_p(X_p), q_p the coefficients of
// Q_p(x) = P(x) / (x + X_p) (Lagrange): the same linear map, so results are bit-identical. Erased slots are
// never zeroed: the masked fixed pass reads them as zero and the solve stores c (default), or the plain pass
// sees their old contents g, the solve yields g + c and the apply XORs that into g (V1Args::xor_dst, option
// m8_syn_masked 0). Erased repair slots only shift their own unknowns.
// Byte of lookup L in a packed k_apply_m8_pf record (gen_asm.py ps8pf_kernel): L = 8 m + 2 k + d sits in byte
// k of dword 2 m + d, so one s_lshr_b64 of a dword pair brings the next byte of both dwords down.
__device__ __forceinline__ int pf_byte(int L) { return 4 * (2 * (L >> 3) + (L & 1)) + ((L & 7) >> 1); }

// The stripe's pattern as bit words for the masked fixed pass: wave w's ballot covers slots 64w .. 64w + 63.
__device__ __forceinline__ void plan_mask_words(const SynPlanArgs& a, int64_t s, int w, int lane, uint64_t bits) {
    if (!a.mbits || lane != 0) return;
    uint32_t* o = a.mbits + s * a.mw;
    if (2 * w < a.mw) o[2 * w] = uint32_t(bits);
    if (2 * w + 1 < a.mw) o[2 * w + 1] = uint32_t(bits >> 32);
}

__global__ void __launch_bounds__(256) k_plan_syn_m8(SynPlanArgs a) {
    __shared__ uint16_t ee[256], pe[256];
    __shared__ int32_t ps[256];
    __shared__ uint16_t cf[2][257];
    __shared__ int cnt[4][2];
    constexpr uint32_t N = 65535u;
    const int64_t s = blockIdx.x;
    const int j = threadIdx.x, lane = j & 63, w = j >> 6;
    const bool valid = j < a.n;
    const bool er = valid && a.masks[s * a.n + j] != 0;
    const uint64_t be = __ballot(er), bp = __ballot(er && j < a.k);
    const uint64_t below = (uint64_t(1) << lane) - 1;
    plan_mask_words(a, s, w, lane, be);
    if (lane == 0) {
        cnt[w][0] = __popcll(be);
        cnt[w][1] = __popcll(bp);
    }
    __syncthreads();
    int oe = 0, op = 0, t = 0, R = 0;
    for (int v = 0; v < 4; ++v) {
        if (v < w) oe += cnt[v][0], op += cnt[v][1];
        t += cnt[v][0], R += cnt[v][1];
    }
    if (er) {
        const uint16_t xj = a.elem[j];
        ee[oe + __popcll(be & below)] = xj;
        if (j < a.k) {
            const int i = op + __popcll(bp & below);
            pe[i] = xj;
            ps[i] = j;
        }
    }
    auto gmul = [&](uint32_t x, uint32_t y) -> uint32_t {
        return (x && y) ? a.expt[(uint32_t(a.logt[x]) + a.logt[y]) % N] : 0u;
    };
    // P(x) = prod (x + X_e), coefficients cf[.][0..t]
    if (j <= 256) cf[0][j] = j == 0 ? 1 : 0;
    if (j == 0) cf[0][256] = 0;
    __syncthreads();
    int cur = 0;
    for (int e = 0; e < t; ++e) {
        const uint32_t xe = ee[e];
        if (j <= e + 1) cf[cur ^ 1][j] = uint16_t((j ? cf[cur][j - 1] : 0u) ^ (j <= e ? gmul(xe, cf[cur][j]) : 0u));
        __syncthreads();
        cur ^= 1;
    }
    if (j == 0) {
        a.kr[2 * s] = t;
        a.kr[2 * s + 1] = R;
    }
    int32_t* pin = a.pin + s * a.in_stride;
    for (int q = j; q < a.in_stride; q += 256) pin[q] = q < t ? int32_t(s * a.r + q) : 0;
    int32_t* pout = a.pout + s * a.out_stride;
    for (int p = j; p < a.out_stride; p += 256) pout[p] = p < R ? ps[p] : 0;
    // row j of the records: synthetic division of P by (x + X_p), q_{t-1} = 1, q_{i-1} = c_i + X_p q_i
    uint32_t* rec = a.pidx + s * a.idx_stride;
    const int ntiles = (R + 31) / 32;
    if (j < ntiles * 32) {
        const int tile = j >> 5, jj = j & 31;
        uint32_t* r0 = rec + size_t(tile) * t * 64;
        if (j < R) {
            const uint32_t xp = pe[j];
            uint32_t ld = 0;  // log prod_{e != p} (X_p + X_e)
            for (int e = 0; e < t; ++e)
                if (ee[e] != xp) ld += a.logt[xp ^ ee[e]];
            ld %= N;
            uint32_t q = 1;
            for (int i = t - 1; i >= 0; --i) {
                uint32_t b = 0;
                if (q) b = a.g8[((uint32_t(a.logt[q]) + N - ld) % N) / 257u];
                if (a.pidx8) {
                    uint8_t* r8 = a.pidx8 + s * a.idx8_stride + (size_t(tile) * t + i) * 64;
                    r8[pf_byte(jj)] = uint8_t(b & 15u);
                    r8[pf_byte(32 + jj)] = uint8_t(b >> 4);
                } else {
                    r0[size_t(i) * 64 + jj] = b & 15u;
                    r0[size_t(i) * 64 + 32 + jj] = b >> 4;
                }
                if (i > 0) q = cf[cur][i] ^ gmul(xp, q);
            }
        } else if (a.pidx8) {
            for (int i = 0; i < t; ++i) {
                uint8_t* r8 = a.pidx8 + s * a.idx8_stride + (size_t(tile) * t + i) * 64;
                r8[pf_byte(jj)] = r8[pf_byte(32 + jj)] = 0;
            }
        } else {
            for (int i = 0; i < t; ++i) r0[size_t(i) * 64 + jj] = r0[size_t(i) * 64 + 32 + jj] = 0u;
        }
    }
}

// Re-encode plans (SynPlanArgs, syn_route 2). The codec's fixed pass computes, for every repair slot P,
//   S'_P = (G rcv_info)_P + rcv_P          (G the encode matrix: [G | I] on the bit-plane XOR kernel)
// which is zero for a codeword. With d the differences on the erased slots (the masked pass reads them as zero,
// d_Q = c_Q; the plain pass reads their old contents g, d_Q = g_Q + c_Q), S'_P = sum_{Q in E_i} G[P][Q] d_Q for
// every surviving repair slot P. The first t_i = |E_i| of them (R', in slot order; t <= r leaves enough)
// give a square system, and because G[P][Q] = L_E(Y_Q) / (L_E'(X_P) (X_P + Y_Q)) (gf16.cpp:solve_matrix, E
// = the repair positions) is a scaled Cauchy matrix, its inverse is again of that form:
//   W[Q][P] = L_T(X_P) / ((X_P + Y_Q) L_T'(Y_Q)),   T = E_i + (repair slots not in R'), |T| = r,
// i.e. solve_matrix with targets T, emitted rows E_i, sources R' -- the same evaluation as k_plan_m8.
// d = W S'_{R'} is then stored into the erased information slots (masked pass) or XORed into them
// (V1Args::xor_dst, plain pass). A t_i x t_i solve from
// t_i rows of a pattern-independent pass over k + r inputs whose matrix is G plus an identity, against the
// syndrome route's t_i x t solve after a pass of r x (k + r) Vandermonde rows.
__global__ void __launch_bounds__(256) k_plan_reenc_m8(SynPlanArgs a) {
    __shared__ uint16_t tx[256], px[256], qx[256];
    __shared__ int32_t ps[256], qs[256];
    __shared__ uint32_t lp[256], ld[256];
    __shared__ int cnt[4][3];
    constexpr uint32_t N = 65535u;
    const int64_t s = blockIdx.x;
    const int j = threadIdx.x, lane = j & 63, w = j >> 6;
    const bool valid = j < a.n;
    const bool er = valid && a.masks[s * a.n + j] != 0;
    const bool inf_er = er && j < a.k, rep_ok = valid && j >= a.k && !er;
    const uint64_t bp = __ballot(inf_er), bq = __ballot(rep_ok);
    const uint64_t below = (uint64_t(1) << lane) - 1;
    plan_mask_words(a, s, w, lane, __ballot(er));
    if (lane == 0) {
        cnt[w][0] = __popcll(bp);
        cnt[w][1] = __popcll(bq);
    }
    __syncthreads();
    int op = 0, oq = 0, R = 0;
    for (int v = 0; v < 4; ++v) {
        if (v < w) op += cnt[v][0], oq += cnt[v][1];
        R += cnt[v][0];
    }
    const uint16_t xj = valid ? a.elem[j] : 0;
    const int qi = oq + __popcll(bq & below);  // rank among the surviving repair slots
    if (inf_er) {
        const int i = op + __popcll(bp & below);
        px[i] = xj;
        ps[i] = j;
    }
    const bool in_rp = rep_ok && qi < R;  // one of the first R survivors: a source of the solve
    if (in_rp) {
        qx[qi] = xj;
        qs[qi] = j - a.k;
    }
    const bool in_t = inf_er || (valid && j >= a.k && !in_rp);
    const uint64_t bt = __ballot(in_t);
    if (lane == 0) cnt[w][2] = __popcll(bt);
    __syncthreads();
    int ot = 0, T = 0;
    for (int v = 0; v < 4; ++v) {
        if (v < w) ot += cnt[v][2];
        T += cnt[v][2];
    }
    if (in_t) tx[ot + __popcll(bt & below)] = xj;
    __syncthreads();
    // log L_T(Y_q) for the sources, log L_T'(X_p) for the emitted rows (solve_matrix's lp / ld)
    if (j < R) {
        uint32_t sp = 0, sd = 0;
        for (int e = 0; e < T; ++e) {
            sp += a.logt[qx[j] ^ tx[e]];
            if (tx[e] != px[j]) sd += a.logt[px[j] ^ tx[e]];
        }
        lp[j] = sp % N;
        ld[j] = sd % N;
    }
    if (j == 0) {
        a.kr[2 * s] = R;  // K = R: t_i inputs, t_i outputs
        a.kr[2 * s + 1] = R;
    }
    __syncthreads();
    int32_t* pin = a.pin + s * a.in_stride;
    for (int q = j; q < a.in_stride; q += 256) pin[q] = q < R ? int32_t(s * a.r + qs[q]) : 0;
    int32_t* pout = a.pout + s * a.out_stride;
    for (int p = j; p < a.out_stride; p += 256) pout[p] = p < R ? ps[p] : 0;
    // row j of the V = 1 records [tile][K][64]: gamma-basis byte of W[j][q] split into nibbles
    uint32_t* rec = a.pidx + s * a.idx_stride;
    const int ntiles = (R + 31) / 32;
    if (j < ntiles * 32) {
        const int tile = j >> 5, jj = j & 31;
        uint32_t* r0 = rec + size_t(tile) * R * 64;
        for (int q = 0; q < R; ++q) {
            uint32_t b = 0;
            if (j < R) b = a.g8[((lp[q] + 2 * N - ld[j] - a.logt[px[j] ^ qx[q]]) % N) / 257u];
            if (a.pidx8) {
                uint8_t* r8 = a.pidx8 + s * a.idx8_stride + (size_t(tile) * R + q) * 64;
                r8[pf_byte(jj)] = uint8_t(b & 15u);
                r8[pf_byte(32 + jj)] = uint8_t(b >> 4);
                continue;
            }
            r0[size_t(q) * 64 + jj] = b & 15u;
            r0[size_t(q) * 64 + 32 + jj] = b >> 4;
        }
    }
}

// Per-stripe solve with every load issued ahead of its use (m8_ps_kernel 9 / 10 / 11; 10 = NB 2 is the default,
// and 12 / 13 = NB 12 / 13 are its diagnostic timing ablations). The ring kernel's waves spend
// about half their cycles waiting (SMEM record halves fetched inside each step, a slot read per batch, one
// barrier per 4 inputs; profiles/r4/ps8_route2.md); here each wave runs its own 256-byte column with no
// barrier after the table copy, and the whole input loop is one asm statement (gen_asm.py ps8pf_kernel) in
// which the next input's packed record (one SMEM load of 16 dwords) and coordinate-table reads are issued a
// step ahead and the raw inputs four inputs ahead, so each step waits once for loads issued a step earlier.
// Records are the plan kernels' packed form (SynPlanArgs::pidx8); same math as k_apply_m8_v1<0>, same
// output stage. The coordinate tables must sit at LDS address 0: lt is the kernel's only LDS array. Reads
// past the stripe's lists: records up to K (one record of prefetch; the record array has room), slot entries
// up to K + 18 (blocks of 8, two ahead; the host requires K + 19 <= ps_in), raw inputs of the zero-padded slots
// (slot 0, a valid offset); all are drained before the asm statement ends.
// NB = 1: two nibble tables per input (gen_asm.py ps8pf_kernel, 78 VGPRs, 6 waves per SIMD); NB = 2: one table
// over y gamma^0..3 with the high-nibble lookups in a second accumulator set (ps8pf1_kernel: 4 multiples and a
// table less per input, 5 waves per SIMD), the output stage adding gamma^4 times it through a third LDS table.
// NB = 4 (ps8pf1c_kernel, launched as 14; diagnostic build, option m8_syn_coord): NB = 2 over inputs the fixed
// pass stored in coordinates already (rs_xj masked form 2, which converts its outputs with the same LDS tables):
// no coordinate reads per step, but the pass's conversion costs more than the solve saves.
// NB = 3 (ps8pf2_kernel): NB = 2 with the multiples y gamma^1..3 read from three more coordinate tables
// (gamma^j L(x) = L(gamma^j x) is linear in x's bytes: table j entry = xt8^j of table 0's) instead of computed;
// LDS: tables j = 0..3 at dword 1024 j, L^-1 at 4096, the gamma^4 table at 5120. NB = 2 issues fastest (the
// loop is VALU-issue bound), so 9 and 11 are diagnostic-build only.
template <int NB>
__global__ void __launch_bounds__(256) k_apply_m8_pf(V1Args a) {
    constexpr int G4 = 2048;  // NB >= 2: gamma^4 folded into L^-1 (m8_v1_out), G4 dwords after the L^-1 base
    constexpr int LINV = NB == 3 ? 3072 : 0;  // the output stage's table base: L^-1 at LINV + 1024
    __shared__ uint32_t lt[NB == 3 ? 6144 : NB == 1 ? 2048 : 3072];
    if (uint32_t(reinterpret_cast<uintptr_t>(lt)) != 0u) __builtin_trap();  // folded away: lt is at 0
    if constexpr (NB == 3) {
        for (int i = threadIdx.x; i < 1024; i += 256) {
            uint32_t v = a.ltab[i];
            lt[i] = v;
#pragma unroll
            for (int j = 1; j < 4; ++j) lt[1024 * j + i] = v = xt8(v);
            lt[4096 + i] = a.ltab[1024 + i];
        }
    } else {  // NB = 2 / 12 / 13: the gamma^4 table comes precomputed after L and L^-1 (device_tables)
        for (int i = threadIdx.x; i < (NB == 1 ? 2048 : 3072); i += 256) lt[i] = a.ltab[i];
    }
    if constexpr (NB == 3) {
        __syncthreads();
        for (int i = threadIdx.x; i < 1024; i += 256)
            lt[LINV + G4 + i] = lt[LINV + 1024 + (i & ~255) + gmul_g4(i & 255)];
    }
    __syncthreads();
    const int64_t bid = blockIdx.x;
    const int64_t local = bid / a.nchunks;  // launch-local stripe
    const int64_t stripe = RS_STRIPE(a.ids, local);
    const int64_t chunk = bid - local * a.nchunks;
    const int tile = blockIdx.y;
    const int K = sload(a.ps_kr + 2 * local), R = sload(a.ps_kr + 2 * local + 1);
    if (tile * 32 >= R || K <= 0) return;  // uniform over the block
    const uint32_t col = uint32_t(chunk * 1024) + threadIdx.x * 4u;
    const uint64_t sbase = uint64_t(reinterpret_cast<uintptr_t>(a.src + (a.src_local ? local : stripe) * a.src_stripe));
    const uint32_t nrec = a.src_bytes > 0 && a.src_bytes < 0xFFFFFFFFll ? uint32_t(a.src_bytes) : 0xFFFFFFFFu;
    const u32x4s rsrc = {uint32_t(sbase), uint32_t(sbase >> 32) & 0xFFFFu, nrec, 0x20000u};
    const uint32_t* rec = a.idx + local * a.ps_idx + size_t(tile) * size_t(K) * 16;
    const int32_t* pin = a.in_idx + local * a.ps_in;
    // the output stage's operands are formed after the loop (nothing of the kernel's own lives across it)
#define RS_PF_DST a.dst + stripe * a.dst_stripe + chunk * 1024 + int64_t(threadIdx.x) * 4, \
                  a.out_idx + local * a.ps_out + tile * 32, min(32, R - tile * 32)
    // stored outputs (the masked pass): the SGPR-addressed store stage; XORed outputs (and the diagnostic output
    // ablation) through m8_v1_store
#ifdef RS_AMD_DIAG
    const bool plain_store = !a.xor_dst && !(a.ablate & 2);
#else
    const bool plain_store = !a.xor_dst;
#endif
#define RS_PF_STORE(LT)                                                                                           \
    if (plain_store)                                                                                              \
        m8_v1h_store<G4>(a, LT, a.dst + stripe * a.dst_stripe + chunk * 1024, threadIdx.x * 4u,                   \
                         a.out_idx + local * a.ps_out + tile * 32, min(32, R - tile * 32), a0, a1, b0, b1);       \
    else                                                                                                          \
        m8_v1_store<2, 0, G4>(a, LT, RS_PF_DST, a0, a1, b0, b1)
#define RS_PF_IN                                                                                                  \
    [rec] "s"(rec), [pin] "s"(pin), [nk] "s"(K), [sym] "s"(uint32_t(a.src_sym)), [rsrc] "s"(rsrc), [col] "v"(col)
#define RS_PF_SGPRS                                                                                               \
    "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55",   \
        "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68", "s69", "s70", "s71", \
        "s72", "s73", "s74", "s76", "s77", "s78", "s79", "s80", "s81", "s82", "s83", "s84", "s85", "s86", "s87", "s88", \
        "s89", "s90", "s91", "s92", "s93", "s94", "s95", "s96", "s97", "scc", "memory"
    if constexpr (NB == 1) {
        u32x16 a0, a1;
        asm volatile(
#include "gen/m8_idx_asm_ps8pf_kernel.inc"
            : "=&{v[32:47]}"(a0), "=&{v[48:63]}"(a1)
            : RS_PF_IN
            : "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15",
              "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30",
              "v31", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", RS_PF_SGPRS);
        m8_v1_store<1>(a, lt, RS_PF_DST, a0, a1, a0, a1);
    } else if constexpr (NB == 2 || NB == 4 || NB == 12 || NB == 13) {
        u32x16 a0, a1, b0, b1;
#define RS_PF1_OPS                                                                                                \
    : "=&{v[16:31]}"(a0), "=&{v[32:47]}"(a1), "=&{v[48:63]}"(b0), "=&{v[64:79]}"(b1)                               \
    : RS_PF_IN                                                                                                     \
    : "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v80", \
      "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", RS_PF_SGPRS
        if constexpr (NB == 2) {
            asm volatile(
#include "gen/m8_idx_asm_ps8pf1_kernel.inc"
                RS_PF1_OPS);
        } else if constexpr (NB == 4) {  // inputs already in coordinates (the fixed pass's masked form 2)
            asm volatile(
#include "gen/m8_idx_asm_ps8pf1c_kernel.inc"
                RS_PF1_OPS);
#ifdef RS_AMD_DIAG
        } else if constexpr (NB == 12) {  // timing ablation: no index switches (wrong results)
            asm volatile(
#include "gen/m8_idx_asm_ps8pf1_noswitch.inc"
                RS_PF1_OPS);
        } else {  // timing ablation: no gpr-index mode (wrong results)
            asm volatile(
#include "gen/m8_idx_asm_ps8pf1_plain.inc"
                RS_PF1_OPS);
#endif
        }
#undef RS_PF1_OPS
        RS_PF_STORE(lt);
    } else {
        u32x16 a0, a1, b0, b1;
        asm volatile(
#include "gen/m8_idx_asm_ps8pf2_kernel.inc"
            : "=&{v[16:31]}"(a0), "=&{v[32:47]}"(a1), "=&{v[48:63]}"(b0), "=&{v[64:79]}"(b1)
            : RS_PF_IN
            : "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15",
              "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94",
              "v95", "v96", "v97", "v98", "v99", "v100", RS_PF_SGPRS);
        RS_PF_STORE(lt + LINV);
    }
#undef RS_PF_STORE
#undef RS_PF_DST
#undef RS_PF_IN
#undef RS_PF_SGPRS
}

// Columns [col0, nbytes) (< 1 KiB) of every stripe under per-stripe plans: one lane per dword,
// coefficients from the nibble records, multiplication by masked gamma-multiples.
__global__ void __launch_bounds__(256) k_apply_m8_ps_tail(V1Args a, int64_t col0, int64_t nbytes) {
    __shared__ uint32_t lt[2048];
    for (int i = threadIdx.x; i < 2048; i += 256) lt[i] = a.ltab[i];
    __syncthreads();
    const int64_t local = blockIdx.x;
    const int64_t stripe = RS_STRIPE(a.ids, local);
    const int tile = blockIdx.y;
    int K = a.K, R = a.R;
    const int32_t* in_idx = a.in_idx;
    const int32_t* out_idx = a.out_idx;
    const uint32_t* idxb = a.idx;
    if (a.ps_kr) {
        K = a.ps_kr[2 * local];
        R = a.ps_kr[2 * local + 1];
        in_idx += local * a.ps_in;
        out_idx += local * a.ps_out;
        idxb += local * a.ps_idx;
    }
    const int64_t col = col0 + int64_t(threadIdx.x) * 4;
    const int64_t avail = nbytes - col;
    if (tile * 32 >= R || avail <= 0) return;
    const int rows = min(32, R - tile * 32);
    const uint8_t* src = a.src + stripe * a.src_stripe + col;
    uint32_t acc[32];
#pragma unroll
    for (int p = 0; p < 32; ++p) acc[p] = 0;
    for (int i = 0; i < K; ++i) {
        uint32_t x[1];
        load_slice<4>(x, src + int64_t(in_idx[i]) * a.src_sym, avail);
        uint32_t m[8];
        m[0] = lds_lookup4(lt, x[0]);
#pragma unroll
        for (int b = 1; b < 8; ++b) m[b] = xt8(m[b - 1]);
        const uint32_t* r = idxb + (size_t(tile) * K + i) * 64;
#pragma unroll
        for (int p = 0; p < 32; ++p) {
            if (p < rows) {
                const uint32_t c = r[p] | (r[32 + p] << 4);
#pragma unroll
                for (int b = 0; b < 8; ++b) acc[p] ^= m[b] & (0u - ((c >> b) & 1u));
            }
        }
    }
    uint8_t* dst = a.dst + stripe * a.dst_stripe + col;
#pragma unroll
    for (int p = 0; p < 32; ++p) {
        if (p < rows) {
            uint8_t* d = dst + int64_t(out_idx[tile * 32 + p]) * a.dst_sym;
            uint32_t y[1] = {lds_lookup4(lt + 1024, acc[p])};
            if (a.xor_dst) {  // see V1Args::xor_dst
                uint32_t old[1];
                load_slice<4>(old, d, avail);
                y[0] ^= old[0];
            }
            store_slice<4>(d, y, avail);
        }
    }
}

// ------------------------------------------------------------ GF(2^16) plans on the device
// lp[q] = sum_e log(Y_q + X_e), ld[p] = sum_{e != p} log(X_p + X_e) (solve_matrix's log-sums): 16
// lanes per item, each summing every 16th target, then a shuffle reduction (sums < 2^32 for d <= 65535)
__global__ void __launch_bounds__(256) k_plan16_sums(Plan16Args a) {
    const int64_t i = (int64_t(blockIdx.x) * 256 + threadIdx.x) >> 4;
    const int part = int(threadIdx.x & 15);
    constexpr uint32_t N = 65535u;
    uint32_t acc = 0;
    if (i < a.K) {
        const uint16_t y = a.src_el[i];
        for (int e = part; e < a.d; e += 16) acc += a.logt[y ^ a.tgt_el[e]];
    } else if (i < int64_t(a.K) + a.R) {
        const int self = a.emit[i - a.K];
        const uint16_t x = a.tgt_el[self];
        for (int e = part; e < a.d; e += 16)
            if (e != self) acc += a.logt[x ^ a.tgt_el[e]];
    }
    for (int o = 8; o; o >>= 1) acc += __shfl_xor(acc, o, 16);
    if (part == 0) {
        if (i < a.K)
            a.lp[i] = acc % N;
        else if (i < int64_t(a.K) + a.R)
            a.ld[i - a.K] = acc % N;
    }
}

// Coefficient (row, i) = alpha^(lp[i] - ld[row] - log(X_row + Y_i)), written into the coefficient tiles
// and, for 64-row tiles, the packed index records. Grid (row blocks, sources): consecutive lanes take
// consecutive rows of one source, so tile writes are contiguous and record bytes share one record.
__global__ void __launch_bounds__(256) k_plan16_fill(Plan16Args a) {
    const int row = int(blockIdx.x) * 256 + int(threadIdx.x), i = int(blockIdx.y);
    if (row >= a.R) return;
    constexpr uint32_t N = 65535u;
    const uint32_t L = (a.lp[i] + 2 * N - a.ld[row] - a.logt[a.tgt_el[a.emit[row]] ^ a.src_el[i]]) % N;
    const uint32_t c = a.expt[L];
    const int t = row / a.rt, j = row - t * a.rt;
    reinterpret_cast<uint16_t*>(a.coef)[(int64_t(t) * a.K + i) * a.rt + j] = uint16_t(c);
    if (a.rec) {  // k_apply_m16_v1 record byte of (plane n, output j): see rs_api.cpp:build_plan
        const int t64 = row >> 6, j64 = row & 63;
        uint8_t* r = a.rec + (int64_t(t64) * (a.K + 1) + i) * 256;
        for (int n = 0; n < 4; ++n)
            r[4 * (16 * n + 2 * (j64 >> 3) + (j64 & 1)) + ((j64 & 7) >> 1)] = uint8_t(16 * n + ((c >> (4 * n)) & 15u));
    }
}

hipError_t launch_plan_m16(const Plan16Args& a, hipStream_t st) {
    const int64_t nsum = (int64_t(a.K) + a.R) * 16;
    if (a.K > 65535) return hipErrorInvalidValue;  // grid y of the fill (K <= k + r <= 65535)
    if (nsum > 0) hipLaunchKernelGGL(k_plan16_sums, dim3(unsigned((nsum + 255) / 256)), dim3(256), 0, st, a);
    if (a.R > 0 && a.K > 0)
        hipLaunchKernelGGL(k_plan16_fill, dim3(unsigned((a.R + 255) / 256), unsigned(a.K)), dim3(256), 0, st, a);
    return hipGetLastError();
}

// dst row j = src row rows[j] (16-byte units; the per-call decode packs the restored rows for one D2H)
__global__ void __launch_bounds__(256) k_gather_rows(uint8_t* dst, int64_t dpitch, const uint8_t* src, int64_t spitch,
                                                     const int32_t* rows, int64_t units) {
    const int64_t u = int64_t(blockIdx.x) * 256 + threadIdx.x;
    if (u >= units) return;
    const int64_t j = blockIdx.y;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    reinterpret_cast<u32x4*>(dst + j * dpitch)[u] = reinterpret_cast<const u32x4*>(src + int64_t(rows[j]) * spitch)[u];
}

hipError_t launch_gather_rows(uint8_t* dst, int64_t dpitch, const uint8_t* src, int64_t spitch, const int32_t* rows,
                              int64_t nrows, int64_t width, hipStream_t st) {
    const int64_t units = (width + 15) / 16;
    if (nrows <= 0 || units <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_gather_rows, dim3(unsigned((units + 255) / 256), unsigned(nrows)), dim3(256), 0, st, dst,
                       dpitch, src, spitch, rows, units);
    return hipGetLastError();
}

// Re-encode decode (rs_api.cpp run_reenc): row p of stripe s of dst ^= row p of stripe s of src, S bytes
// as 4-byte words (blockIdx.y = row, blockIdx.z = stripe).
__global__ void __launch_bounds__(256) k_xor_rows(uint8_t* dst, int64_t dst_stripe, int64_t dst_sym, const uint8_t* src,
                                                  int64_t src_stripe, int64_t src_sym, int64_t words) {
    const int64_t w = int64_t(blockIdx.x) * 256 + threadIdx.x;
    if (w >= words) return;
    const int64_t p = blockIdx.y, s = blockIdx.z;
    uint32_t* d = reinterpret_cast<uint32_t*>(dst + s * dst_stripe + p * dst_sym) + w;
    *d ^= reinterpret_cast<const uint32_t*>(src + s * src_stripe + p * src_sym)[w];
}

hipError_t launch_xor_rows(uint8_t* dst, int64_t dst_stripe, int64_t dst_sym, const uint8_t* src, int64_t src_stripe,
                           int64_t src_sym, int64_t nrows, int64_t S, int64_t n_stripes, hipStream_t st) {
    if (nrows <= 0 || n_stripes <= 0 || S <= 0) return hipSuccess;
    if ((S | dst_stripe | dst_sym | src_stripe | src_sym) % 4 || (uintptr_t(dst) | uintptr_t(src)) % 4 ||
        nrows > 65535 || n_stripes > 65535)
        return hipErrorInvalidValue;
    const int64_t words = S / 4;
    hipLaunchKernelGGL(k_xor_rows, dim3(unsigned((words + 255) / 256), unsigned(nrows), unsigned(n_stripes)), dim3(256),
                       0, st, dst, dst_stripe, dst_sym, src, src_stripe, src_sym, words);
    return hipGetLastError();
}

// 16-byte stores of whole rows across PCIe into page-locked host memory (posted writes; visible to
// the host once the stream's completion event has been waited on)
__global__ void __launch_bounds__(256) k_put_rows(uint8_t* dst, int64_t dpitch, const uint8_t* src, int64_t spitch,
                                                  const int32_t* rows, int64_t units) {
    const int64_t u = int64_t(blockIdx.x) * 256 + threadIdx.x;
    if (u >= units) return;
    const int64_t i = rows ? rows[blockIdx.y] : int64_t(blockIdx.y);
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    reinterpret_cast<u32x4*>(dst + i * dpitch)[u] = reinterpret_cast<const u32x4*>(src + i * spitch)[u];
}

hipError_t launch_put_rows(uint8_t* dst, int64_t dpitch, const uint8_t* src, int64_t spitch, const int32_t* rows,
                           int64_t nrows, int64_t width, hipStream_t st) {
    const int64_t units = width / 16;
    if (nrows <= 0 || units <= 0) return hipSuccess;
    if ((width & 15) || (dpitch & 15) || (spitch & 15) || (uintptr_t(dst) & 15) || (uintptr_t(src) & 15))
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_put_rows, dim3(unsigned((units + 255) / 256), unsigned(nrows)), dim3(256), 0, st, dst, dpitch,
                       src, spitch, rows, units);
    return hipGetLastError();
}

// ------------------------------------------- per-stripe GF(2^16) decode plans (Ps16Args, rs_kernels.hpp)
// One workgroup per selected stripe: the erased slots in slot order (ee, and the information ones as rows
// pe / pout), the coefficients of P(x) = prod (x + X_e), and the erased information slots zeroed.
__global__ void __launch_bounds__(256) k_plan16_ps(Ps16Args a) {
    constexpr int Q = kPs16MaxR / 4 + 2;
    __shared__ uint16_t ee[kPs16MaxR];
    __shared__ uint16_t sub[4][2][Q];                           // per-wave sub-products (double buffer)
    __shared__ uint16_t hv[kPs16MaxR + 4], hl[kPs16MaxR + 4];  // halves P01, P23: values, logs
    __shared__ int cnt[4][2];
    constexpr uint32_t N = 65535u;
    constexpr uint16_t kZeroLog = 0xFFFF;
    const int64_t s = blockIdx.x;
    const int j = threadIdx.x, lane = j & 63, w = j >> 6;
    const uint64_t below = (uint64_t(1) << lane) - 1;
    const uint8_t* mask = a.masks + s * a.n;
    uint16_t* pe = a.pe + s * a.out_stride;
    int32_t* pout = a.pout + s * a.out_stride;
    int t = 0, R = 0;  // block-uniform running counts
    for (int c0 = 0; c0 < a.n; c0 += 256) {
        const int i = c0 + j;
        const bool er = i < a.n && mask[i] != 0;
        const bool info = er && i < a.k;
        const uint64_t be = __ballot(er), bp = __ballot(info);
        if (lane == 0) {
            cnt[w][0] = __popcll(be);
            cnt[w][1] = __popcll(bp);
        }
        __syncthreads();
        int oe = t, op = R, te = 0, tp = 0;
        for (int v = 0; v < 4; ++v) {
            if (v < w) oe += cnt[v][0], op += cnt[v][1];
            te += cnt[v][0];
            tp += cnt[v][1];
        }
        if (er) {
            const uint16_t x = a.elem[i];
            const int ie = oe + __popcll(be & below);
            if (ie < a.r) ee[ie] = x;  // t <= r: checked by the host
            if (info) {
                const int ip = op + __popcll(bp & below);
                pe[ip] = x;
                pout[ip] = i;
            }
        }
        t += te;
        R += tp;
        __syncthreads();  // cnt is rewritten by the next chunk
    }
    t = min(t, a.r);
    for (int p = R + j; p < a.out_stride; p += 256) pe[p] = 0, pout[p] = 0;
    if (j == 0) {
        a.kr[2 * s] = t;
        a.kr[2 * s + 1] = R;
    }
    uint16_t* eg = a.ee + s * a.r;
    for (int e = j; e < t; e += 256) eg[e] = ee[e];
    auto lg = [&](uint32_t x) -> uint16_t { return x ? a.logt[x] : kZeroLog; };
    auto emul = [&](uint16_t la, uint16_t lb) -> uint32_t {  // product from logs (kZeroLog: zero)
        return (la == kZeroLog || lb == kZeroLog) ? 0u : uint32_t(a.expt[(uint32_t(la) + lb) % N]);
    };
    // P(x) = prod (x + X_e) as a product tree: wave w multiplies out its quarter of E one linear factor at
    // a time (wave-synchronous, no block barrier), then the halves P01 = P0 P1, P23 = P2 P3 and P = P01 P23
    // (one output coefficient per thread, products through the logs of the factors' coefficients).
    const int q0 = t * w / 4, m = t * (w + 1) / 4 - q0;
    for (int i = lane; i <= m; i += 64) sub[w][0][i] = i == 0 ? 1 : 0;
    __builtin_amdgcn_wave_barrier();
    int cur = 0;
    for (int e = 0; e < m; ++e) {  // (x + X_e) * B: new[i] = B[i - 1] + X_e B[i]
        const uint16_t lx = lg(ee[q0 + e]);
        const uint16_t* o = sub[w][cur];
        uint16_t* nw = sub[w][cur ^ 1];
        for (int i = lane; i <= e + 1; i += 64)
            nw[i] = uint16_t((i ? o[i - 1] : 0u) ^ (i <= e ? emul(lx, lg(o[i])) : 0u));
        __builtin_amdgcn_wave_barrier();
        cur ^= 1;
    }
    // logs of the sub-products into their free halves
    for (int i = lane; i <= m; i += 64) sub[w][cur ^ 1][i] = lg(sub[w][cur][i]);
    __syncthreads();
    int mq[4], cq[4];
    for (int v = 0; v < 4; ++v) {
        mq[v] = t * (v + 1) / 4 - t * v / 4;
        cq[v] = mq[v] & 1;  // buffer holding sub-product v's values (cur after mq[v] toggles)
    }
    const int d01 = mq[0] + mq[1], d23 = mq[2] + mq[3];
    for (int o = j; o <= d01 + 1 + d23; o += 256) {  // level 1: hv[0 .. d01] = P01, hv[d01 + 1 ..] = P23
        const int A = o <= d01 ? 0 : 2, oo = o <= d01 ? o : o - d01 - 1;
        const uint16_t* la = sub[A][cq[A] ^ 1];
        const uint16_t* lb = sub[A + 1][cq[A + 1] ^ 1];
        uint32_t acc = 0;
        for (int x = max(0, oo - mq[A + 1]); x <= min(oo, mq[A]); ++x) acc ^= emul(la[x], lb[oo - x]);
        hv[o] = uint16_t(acc);
        hl[o] = lg(acc);
    }
    __syncthreads();
    uint16_t* cg = a.cf + s * (int64_t(a.r) + 1);
    for (int o = j; o <= t; o += 256) {  // level 2: P = P01 * P23
        uint32_t acc = 0;
        for (int x = max(0, o - d23); x <= min(o, d01); ++x) acc ^= emul(hl[x], hl[d01 + 1 + o - x]);
        cg[o] = uint16_t(acc);
    }
    // zero the erased information slots of the stripe (16-byte stores; S and strides are multiples of 16)
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    uint8_t* sb = a.base + int64_t(a.ids[s]) * a.stripe_stride;
    const int64_t units = a.S / 16;
    const u32x4 z = {0u, 0u, 0u, 0u};
    for (int p = 0; p < R; ++p) {
        u32x4* d = reinterpret_cast<u32x4*>(sb + int64_t(pout[p]) * a.symbol_stride);
        for (int64_t x = j; x < units; x += 256) d[x] = z;
    }
}

// The records of W (k_apply_m16_v1 format, see rs_api.cpp:build_plan): one wave per (stripe, 64-row
// tile), one lane per row p. ld = log prod_{e != p} (X_p + X_e); then the synthetic division of P by
// (x + X_p) from the top, q_{t-1} = 1, q_{i-1} = cf_i + X_p q_i, emits W[p][i] = q_i / prod for i = t-1 .. 0;
// the wave packs the 64 rows' index bytes of input i in LDS and stores the 256-byte record.
// Both products of q_i (by X_p and by 1 / prod) come from one set of per-lane nibble tables in LDS, a
// dword per entry (low half X_p * v, high half v / prod; lane-contiguous, so conflict-free): four LDS
// reads and three XORs a step instead of dependent log / exp gathers from L2.
__global__ void __launch_bounds__(256) k_plan16_ps_rec(Ps16Args a) {
    __shared__ uint32_t buf[4][2][64];
    __shared__ uint32_t tab[4][64][64];  // [wave][16 * nibble position + nibble value][lane]
    __shared__ uint16_t cfl[kPs16MaxR + 1];
    constexpr uint32_t N = 65535u;
    const int64_t s = blockIdx.x / a.tblocks;
    const int wave = int(threadIdx.x >> 6), lane = int(threadIdx.x & 63);
    const int tile = int(blockIdx.x - s * a.tblocks) * 4 + wave;
    const int t = a.kr[2 * s], R = a.kr[2 * s + 1];
    const uint16_t* cf = a.cf + s * (int64_t(a.r) + 1);
    for (int i = int(threadIdx.x); i <= t; i += 256) cfl[i] = cf[i];
    __syncthreads();  // the only block barrier: waves without rows leave after it
    if (tile * 64 >= R) return;
    const int row = tile * 64 + lane;
    const bool live = row < R;
    const uint16_t* ee = a.ee + s * a.r;
    const uint32_t xp = live ? a.pe[s * a.out_stride + row] : 0u;
    uint32_t ld = 0;
    if (live) {
        for (int e = 0; e < t; ++e) {
            const uint32_t x = ee[e];
            if (x != xp) ld += a.logt[xp ^ x];
        }
        ld %= N;
    }
    const uint32_t inv = live ? uint32_t(a.expt[(N - ld) % N]) : 0u;
    // tables: base_b = X_p alpha^b | (alpha^b / prod) << 16 (both halves times alpha per bit), entry (j, v)
    // = XOR of base_{4j + bit} over the set bits of v
    uint32_t* tw = &tab[wave][0][0];
    uint32_t base = xp | (inv << 16);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        uint32_t b4[4];
#pragma unroll
        for (int bit = 0; bit < 4; ++bit) {
            b4[bit] = base;
            base = ((base << 1) & 0xFFFEFFFEu) ^ (((base >> 15) & 0x10001u) * 0x2Du);
        }
        uint32_t e[16];
        e[0] = 0;
#pragma unroll
        for (int v = 1; v < 16; ++v) e[v] = e[v & (v - 1)] ^ b4[__builtin_ctz(v)];
#pragma unroll
        for (int v = 0; v < 16; ++v) tw[(16 * j + v) * 64 + lane] = e[v];
    }
    __builtin_amdgcn_wave_barrier();
    const uint32_t* tl = tw + lane;
    uint32_t* rec = a.rec + s * a.rec_stride + size_t(tile) * size_t(t + 1) * 64;
    uint8_t* lb = reinterpret_cast<uint8_t*>(&buf[wave][0][0]);
    const int slot0 = 4 * (2 * (lane >> 3) + (lane & 1)) + ((lane & 7) >> 1);  // byte of plane 0
    uint32_t q = 1;
    for (int i = t - 1; i >= 0; --i) {
        const uint32_t pr = tl[(q & 15u) * 64] ^ tl[(16 + ((q >> 4) & 15u)) * 64] ^ tl[(32 + ((q >> 8) & 15u)) * 64] ^
                            tl[(48 + (q >> 12)) * 64];
        const uint32_t c = pr >> 16;  // q_i / prod
        uint8_t* b = lb + (i & 1) * 256;
#pragma unroll
        for (int n = 0; n < 4; ++n) b[64 * n + slot0] = uint8_t(16 * n + ((c >> (4 * n)) & 15u));
        __builtin_amdgcn_wave_barrier();
        rec[size_t(i) * 64 + lane] = reinterpret_cast<const uint32_t*>(b)[lane];
        if (i > 0) q = uint32_t(cfl[i]) ^ (pr & 0xFFFFu);
    }
}

// ---------------------------------------------- GF(2^16) per-stripe re-encode plans (m16_ps 2)
// The fixed pass is the codec's encode route over every information slot of the stripe range (erased ones
// zeroed here first), + the received repair rows: S'_P = (G rcv_info)_P + rcv_P = sum_{Q in E} G[P][Q] c_Q
// for each surviving repair slot P. The first t_info of them (R', slot order) give a square Cauchy system
// whose inverse is again scaled Cauchy (k_plan_reenc_m8, gf16.cpp:solve_matrix):
//   W'[Q][P] = L_T(X_P) / ((X_P + X_Q) L_T'(X_Q)),   T = E + (repair slots not in R'),  |T| = r.
// k_plan16_reenc: one workgroup per stripe -- E (rows: pe, pout), R' (sources: qe, pin), T (into ee), K = R
// = t_info, and the erased information slots zeroed.
__global__ void __launch_bounds__(256) k_plan16_reenc(Ps16Args a) {
    __shared__ int cnt[4][3];
    const int64_t s = blockIdx.x;
    const int j = threadIdx.x, lane = j & 63, w = j >> 6;
    const uint64_t below = (uint64_t(1) << lane) - 1;
    const uint8_t* mask = a.masks + s * a.n;
    uint16_t* pe = a.pe + s * a.out_stride;
    int32_t* pout = a.pout + s * a.out_stride;
    uint16_t* qe = a.qe + s * a.in_stride;
    int32_t* pin = a.pin + s * a.in_stride;
    uint16_t* tx = a.ee + s * a.r;
    int R = 0, Q = 0, T = 0;  // block-uniform running counts: erased info, surviving repair, T
    for (int c0 = 0; c0 < a.n; c0 += 256) {
        const int i = c0 + j;
        const bool valid = i < a.n;
        const bool er = valid && mask[i] != 0;
        const bool inf_er = er && i < a.k, rep_ok = valid && i >= a.k && !er;
        const uint64_t bp = __ballot(inf_er), bq = __ballot(rep_ok);
        if (lane == 0) {
            cnt[w][0] = __popcll(bp);
            cnt[w][1] = __popcll(bq);
        }
        __syncthreads();
        int op = R, oq = Q, tp = 0, tq = 0;
        for (int v = 0; v < 4; ++v) {
            if (v < w) op += cnt[v][0], oq += cnt[v][1];
            tp += cnt[v][0];
            tq += cnt[v][1];
        }
        // every information slot precedes every repair slot: t_info is final for this chunk's repair slots
        const int rall = R + tp;
        const uint16_t x = valid ? a.elem[i] : 0;
        if (inf_er) {
            const int ip = op + __popcll(bp & below);
            pe[ip] = x;
            pout[ip] = i;
        }
        const int qi = oq + __popcll(bq & below);
        const bool src = rep_ok && qi < rall;
        if (src) {
            qe[qi] = x;
            pin[qi] = i - a.k;
        }
        const bool in_t = inf_er || (valid && i >= a.k && !src);
        const uint64_t bt = __ballot(in_t);
        __syncthreads();  // cnt[.][0..1] read by every wave
        if (lane == 0) cnt[w][2] = __popcll(bt);
        __syncthreads();
        int ot = T, tt = 0;
        for (int v = 0; v < 4; ++v) {
            if (v < w) ot += cnt[v][2];
            tt += cnt[v][2];
        }
        if (in_t) {
            const int it = ot + __popcll(bt & below);
            if (it < a.r) tx[it] = x;  // |T| = r for a pattern with t <= r (checked by the host)
        }
        R += tp;
        Q += tq;
        T += tt;
        __syncthreads();  // cnt is rewritten by the next chunk
    }
    for (int p = R + j; p < a.out_stride; p += 256) pe[p] = 0, pout[p] = 0;
    for (int q = R + j; q < a.in_stride; q += 256) qe[q] = 0, pin[q] = 0;
    if (j == 0) {
        a.kr[2 * s] = R;  // K = R: t_info sources, t_info rows
        a.kr[2 * s + 1] = R;
    }
    // zero the erased information slots (the fixed pass reads every information slot)
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    uint8_t* sb = a.base + int64_t(a.ids[s]) * a.stripe_stride;
    const int64_t units = a.S / 16;
    const u32x4 z = {0u, 0u, 0u, 0u};
    for (int p = 0; p < R; ++p) {
        u32x4* d = reinterpret_cast<u32x4*>(sb + int64_t(pout[p]) * a.symbol_stride);
        for (int64_t x = j; x < units; x += 256) d[x] = z;
    }
}

// The log sums: lq[q] = sum_{e in T} log(X_q + X_e) for the sources, lr[p] = sum_{e in T, e != p} log(X_p +
// X_e) for the rows; lblocks workgroups per stripe, one sum per thread, T staged in LDS, gathers unrolled.
__global__ void __launch_bounds__(256) k_plan16_reenc_logs(Ps16Args a) {
    __shared__ uint16_t tx[kPs16MaxR];
    constexpr uint32_t N = 65535u;
    const int64_t s = blockIdx.x / a.lblocks;
    const int blk = int(blockIdx.x - s * a.lblocks);
    const int R = a.kr[2 * s];
    const uint16_t* tg = a.ee + s * a.r;
    for (int e = threadIdx.x; e < a.r; e += 256) tx[e] = tg[e];
    __syncthreads();
    const int item = blk * 256 + int(threadIdx.x);  // [0, R): sources, [R, 2R): rows
    if (item >= 2 * R) return;
    const bool row = item >= R;
    const int idx = row ? item - R : item;
    const uint32_t x = row ? a.pe[s * a.out_stride + idx] : a.qe[s * a.in_stride + idx];
    uint32_t sum = 0;
    int e = 0;
    for (; e + 8 <= a.r; e += 8) {
        uint32_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint32_t d = x ^ tx[e + u];
            v[u] = d ? uint32_t(a.logt[d]) : 0u;  // d = 0 only for a row's own element (excluded)
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) sum += v[u];
    }
    for (; e < a.r; ++e) {
        const uint32_t d = x ^ tx[e];
        sum += d ? uint32_t(a.logt[d]) : 0u;
    }
    if (row)
        a.lr[s * a.out_stride + idx] = sum % N;
    else
        a.lq[s * a.in_stride + idx] = sum % N;
}

// The records of W' (k_apply_m16_v1 format, as k_plan16_ps_rec): one wave per (stripe, 64-row tile), one
// lane per row p, four sources per step (independent gathers): W'[p][q] = alpha^(lq[q] - lr[p] - log(X_p +
// X_q)); the wave packs the 64 rows' index bytes of source q in LDS and stores the 256-byte record.
__global__ void __launch_bounds__(256) k_plan16_reenc_rec(Ps16Args a) {
    __shared__ uint32_t buf[4][4][64];
    constexpr uint32_t N = 65535u;
    const int64_t s = blockIdx.x / a.tblocks;
    const int wave = int(threadIdx.x >> 6), lane = int(threadIdx.x & 63);
    const int tile = int(blockIdx.x - s * a.tblocks) * 4 + wave;
    const int R = a.kr[2 * s];
    if (tile * 64 >= R) return;  // no block barrier below
    const int row = tile * 64 + lane;
    const bool live = row < R;
    const uint32_t xp = live ? a.pe[s * a.out_stride + row] : 0u;
    const uint32_t lrp = live ? a.lr[s * a.out_stride + row] : 0u;
    const uint16_t* qe = a.qe + s * a.in_stride;
    const uint32_t* lq = a.lq + s * a.in_stride;
    uint32_t* rec = a.rec + s * a.rec_stride + size_t(tile) * size_t(R + 1) * 64;
    uint8_t* lb = reinterpret_cast<uint8_t*>(&buf[wave][0][0]);
    const int slot0 = 4 * (2 * (lane >> 3) + (lane & 1)) + ((lane & 7) >> 1);  // byte of plane 0
    for (int q0 = 0; q0 < R; q0 += 4) {
        uint32_t c[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int q = min(q0 + u, R - 1);
            const uint32_t lg = uint32_t(a.logt[xp ^ qe[q]]);  // X_p != X_q: rows are information slots
            c[u] = live ? uint32_t(a.expt[(lq[q] + 2 * N - lrp - lg) % N]) : 0u;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            uint8_t* b = lb + u * 256;
#pragma unroll
            for (int n = 0; n < 4; ++n) b[64 * n + slot0] = uint8_t(16 * n + ((c[u] >> (4 * n)) & 15u));
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (q0 + u < R) rec[size_t(q0 + u) * 64 + lane] = reinterpret_cast<const uint32_t*>(lb + u * 256)[lane];
        __builtin_amdgcn_wave_barrier();  // buf is rewritten by the next step
    }
}

hipError_t launch_plan16_reenc(const Ps16Args& a, int64_t n_sel, hipStream_t st) {
    if (n_sel <= 0) return hipSuccess;
    if (a.r > kPs16MaxR || a.lblocks <= 0 || (a.S & 15) || (a.symbol_stride & 15) || (a.stripe_stride & 15) ||
        (uintptr_t(a.base) & 15))
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_plan16_reenc, dim3(unsigned(n_sel)), dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_plan16_reenc_rec(const Ps16Args& a, int64_t n_sel, hipStream_t st) {
    if (n_sel <= 0 || a.tblocks <= 0 || a.lblocks <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_plan16_reenc_logs, dim3(unsigned(n_sel * a.lblocks)), dim3(256), 0, st, a);
    hipLaunchKernelGGL(k_plan16_reenc_rec, dim3(unsigned(n_sel * a.tblocks)), dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_plan16_ps(const Ps16Args& a, int64_t n_sel, hipStream_t st) {
    if (n_sel <= 0) return hipSuccess;
    if (a.r > kPs16MaxR || (a.S & 15) || (a.symbol_stride & 15) || (a.stripe_stride & 15) ||
        (uintptr_t(a.base) & 15))
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_plan16_ps, dim3(unsigned(n_sel)), dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_plan16_ps_rec(const Ps16Args& a, int64_t n_sel, hipStream_t st) {
    if (n_sel <= 0 || a.tblocks <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_plan16_ps_rec, dim3(unsigned(n_sel * a.tblocks)), dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_apply_m16_ps(const V1Args& v, int64_t n_sel, int64_t nbytes, int tiles, hipStream_t st) {
    const int64_t full = nbytes / 1024;
    if (n_sel <= 0 || tiles <= 0 || full <= 0) return hipSuccess;
    if (nbytes % 1024 || !v.ps_kr) return hipErrorInvalidValue;
    V1Args f = v;
    f.nchunks = full;
    f.kslices = 1;
    f.units = n_sel * full;  // XCD-aware order: a unit's tiles back to back on one XCD
    f.tiles = tiles;
    hipLaunchKernelGGL((k_apply_m16_v1<0>), dim3(unsigned((f.units + 7) / 8 * 8 * tiles)), dim3(256), 0, st, f);
    return hipGetLastError();
}

// drop-in path over registered caller symbols: whole rows between per-symbol host addresses (mapped,
// read / written across PCIe) and the device staging stripe
__global__ void __launch_bounds__(256) k_gather_ptrs(uint8_t* dst, int64_t dpitch, const uint64_t* ptrs,
                                                     const int32_t* rows, int64_t off, int64_t units) {
    const int64_t u = int64_t(blockIdx.x) * 256 + threadIdx.x;
    if (u >= units) return;
    const int64_t i = rows ? rows[blockIdx.y] : int64_t(blockIdx.y);
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    reinterpret_cast<u32x4*>(dst + i * dpitch + off)[u] = reinterpret_cast<const u32x4*>(uintptr_t(ptrs[i]) + off)[u];
}

__global__ void __launch_bounds__(256) k_scatter_ptrs(const uint64_t* ptrs, const uint8_t* src, int64_t spitch,
                                                      const int32_t* rows, int64_t off, int64_t units) {
    const int64_t u = int64_t(blockIdx.x) * 256 + threadIdx.x;
    if (u >= units) return;
    const int64_t i = rows ? rows[blockIdx.y] : int64_t(blockIdx.y);
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    reinterpret_cast<u32x4*>(uintptr_t(ptrs[i]) + off)[u] = reinterpret_cast<const u32x4*>(src + i * spitch + off)[u];
}

hipError_t launch_gather_ptrs(uint8_t* dst, int64_t dpitch, const uint64_t* ptrs, const int32_t* rows, int64_t nrows,
                              int64_t off, int64_t width, hipStream_t st) {
    const int64_t units = width / 16;
    if (nrows <= 0 || units <= 0) return hipSuccess;
    if ((width & 15) || (off & 15) || (dpitch & 15) || (uintptr_t(dst) & 15) || nrows > 65535) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_gather_ptrs, dim3(unsigned((units + 255) / 256), unsigned(nrows)), dim3(256), 0, st, dst, dpitch,
                       ptrs, rows, off, units);
    return hipGetLastError();
}

hipError_t launch_scatter_ptrs(const uint64_t* ptrs, const uint8_t* src, int64_t spitch, const int32_t* rows,
                               int64_t nrows, int64_t off, int64_t width, hipStream_t st) {
    const int64_t units = width / 16;
    if (nrows <= 0 || units <= 0) return hipSuccess;
    if ((width & 15) || (off & 15) || (spitch & 15) || (uintptr_t(src) & 15) || nrows > 65535) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_scatter_ptrs, dim3(unsigned((units + 255) / 256), unsigned(nrows)), dim3(256), 0, st, ptrs, src,
                       spitch, rows, off, units);
    return hipGetLastError();
}

hipError_t launch_plan_m8(const PlanArgs& a, int64_t n_sel, hipStream_t st) {
    if (n_sel <= 0) return hipSuccess;
    if (a.n > 256) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_plan_m8, dim3(unsigned(n_sel)), dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_plan_syn_m8(const SynPlanArgs& a, int64_t n_sel, hipStream_t st, int kind) {
    if (n_sel <= 0) return hipSuccess;
    if (kind == 2)
        hipLaunchKernelGGL(k_plan_reenc_m8, dim3(unsigned(n_sel)), dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL(k_plan_syn_m8, dim3(unsigned(n_sel)), dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_apply_m8_ps(const V1Args& v, int64_t n_sel, int64_t nbytes, int tiles, hipStream_t st, int kernel,
                              int cpb) {
    if (n_sel <= 0 || tiles <= 0) return hipSuccess;
    if (kernel >= 9 && kernel <= 14) {  // prefetching solves (14: kernel 10 on coordinate inputs) (two / one nibble tables / one table with read
                                        // multiples): packed records, whole 1 KiB chunks only
        if (nbytes % 1024 || v.src_sym > 0xFFFFFFFFll) return hipErrorInvalidValue;
        V1Args f = v;
        f.nchunks = nbytes / 1024;
#ifdef RS_AMD_DIAG  // the two-table (9) and read-multiples (11) forms: measured slower than 10, DESIGN.md 9.1
        if (kernel == 9)
            hipLaunchKernelGGL(k_apply_m8_pf<1>, dim3(unsigned(n_sel * f.nchunks), unsigned(tiles)), dim3(256), 0, st, f);
        else if (kernel == 12 || kernel == 13)  // timing ablations of kernel 10 (wrong results)
            hipLaunchKernelGGL(kernel == 12 ? k_apply_m8_pf<12> : k_apply_m8_pf<13>,
                               dim3(unsigned(n_sel * f.nchunks), unsigned(tiles)), dim3(256), 0, st, f);
        else if (kernel == 11)
            hipLaunchKernelGGL(k_apply_m8_pf<3>, dim3(unsigned(n_sel * f.nchunks), unsigned(tiles)), dim3(256), 0, st, f);
        else if (kernel == 14)  // coordinate inputs (option m8_syn_coord)
            hipLaunchKernelGGL(k_apply_m8_pf<4>, dim3(unsigned(n_sel * f.nchunks), unsigned(tiles)), dim3(256), 0, st, f);
        else
#else
        if (kernel != 10) return hipErrorInvalidValue;
#endif
            hipLaunchKernelGGL(k_apply_m8_pf<2>, dim3(unsigned(n_sel * f.nchunks), unsigned(tiles)), dim3(256), 0, st, f);
        return hipGetLastError();
    }
#ifndef RS_AMD_DIAG
    // release build: the prefetching solve (10, above; the default), the LDS-ring solve (0, one column chunk per
    // workgroup) and its one-table variant (3)
    if ((kernel != 0 && kernel != 3) || cpb > 1) return hipErrorInvalidValue;
#else
    if (kernel == 2) {  // two dwords per lane over 2 KiB chunks, the last one partial: no tail launch
        V1Args f = v;
        f.nchunks = nbytes;
        hipLaunchKernelGGL(k_apply_m8_ps_w2, dim3(unsigned(n_sel * ((nbytes + 2047) / 2048)), unsigned(tiles)),
                           dim3(256), 0, st, f);
        return hipGetLastError();
    }
#endif
    const int64_t full = nbytes / 1024;
    if (full > 0) {
        V1Args f = v;
        f.nchunks = full;
        // the production ring kernel (0) walks cpb chunks per block (k_apply_m8_v1<6>); the others one
        f.cpb = kernel == 0 ? std::max(1, std::min<int>(cpb, int(full))) : 1;
        const int64_t blocks = n_sel * ((full + f.cpb - 1) / f.cpb);
        if (kernel == 3)
            hipLaunchKernelGGL((k_apply_m8_v1<2>), dim3(unsigned(blocks), unsigned(tiles)), dim3(256), 0, st, f);
#ifdef RS_AMD_DIAG  // option-only A/B kernels (1, 2, 4, 5, cpb > 1), the ablation (6) and the stamps (7)
        else if (kernel == 1)
            hipLaunchKernelGGL(k_apply_m8_ps_w, dim3(unsigned(n_sel * full), unsigned(tiles)), dim3(256), 0, st, f);
        else if (kernel == 4)
            hipLaunchKernelGGL((k_apply_m8_v1<3>), dim3(unsigned(blocks), unsigned(tiles)), dim3(256), 0, st, f);
        else if (kernel == 5)
            hipLaunchKernelGGL((k_apply_m8_v1<4>), dim3(unsigned(blocks), unsigned(tiles)), dim3(256), 0, st, f);
        else if (kernel == 6)  // timing ablation: fixed table registers, no index switches (wrong results)
            hipLaunchKernelGGL((k_apply_m8_v1<1>), dim3(unsigned(blocks), unsigned(tiles)), dim3(256), 0, st, f);
        else if (kernel == 7)  // the production kernel with phase stamps into f.stamps
            hipLaunchKernelGGL((k_apply_m8_v1<5>), dim3(unsigned(blocks), unsigned(tiles)), dim3(256), 0, st, f);
        else if (kernel == 8)  // timing ablation: one record round trip per input step (wrong results)
            hipLaunchKernelGGL((k_apply_m8_v1<7>), dim3(unsigned(blocks), unsigned(tiles)), dim3(256), 0, st, f);
        else if (f.cpb > 1)
            hipLaunchKernelGGL((k_apply_m8_v1<6>), dim3(unsigned(blocks), unsigned(tiles)), dim3(256), 0, st, f);
#endif
        else
            hipLaunchKernelGGL((k_apply_m8_v1<0>), dim3(unsigned(blocks), unsigned(tiles)), dim3(256), 0, st, f);
    }
    if (nbytes % 1024)
        hipLaunchKernelGGL(k_apply_m8_ps_tail, dim3(unsigned(n_sel), unsigned(tiles)), dim3(256), 0, st, v,
                           full * 1024, nbytes);
    return hipGetLastError();
}

}  // namespace rsamd
