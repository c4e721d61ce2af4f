// rs_device.h -- device helpers shared by rs_kernels.hip and the hiprtc-specialised kernels
// (rs_jit.cpp embeds this file's text into every generated source; keep it self-contained).
#pragma once
#ifndef RS_JIT_SOURCE
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rs_v1args.h"
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


// ------------------------------------------------------------- LDS-DMA input ring (m <= 8)
// Inputs are copied HBM -> LDS by global_load_lds_dwordx4 (16 B per lane, 1 KiB per wave
// instruction), RING_B batches of 4 inputs ahead of use; slot of input i = i % RING_SLOTS.
constexpr int RING_B = 3;
constexpr int RING_SLOTS = 4 * (RING_B + 1);

__device__ __forceinline__ void dma16(const uint8_t* g, uint32_t lds_byte) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(g), "s"(lds_byte)
        : "memory");
}

// Wave-uniform read of an index table that no kernel writes (slot and offset arrays) through the
// scalar cache. The compiler cannot prove these arrays unaliased with the kernels' global stores,
// so a plain read becomes a global_load + s_waitcnt vmcnt(0) -- which also drains every LDS-DMA
// in flight.
__device__ __forceinline__ int32_t sload(const int32_t* p) {
    int32_t v;
    asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
    return v;
}

// Diagnostic builds with checked launches: a slot index outside [0, nslots) is recorded in a.slot_err (vector
// stores of the wave's first lane: what, list position, value, block) and the access it would address is
// redirected to slot 0 (loads) or skipped (stores); release and hiprtc builds compile nothing.
#if defined(RS_AMD_DIAG) && !defined(RS_JIT_SOURCE)
__device__ __noinline__ bool rs_slot_fail(int32_t* err, int what, int pos, int32_t slot) {
    if (err && (threadIdx.x & 63) == 0) {
        err[0] = what;
        err[1] = pos;
        err[2] = slot;
        err[3] = int32_t(blockIdx.x);
    }
    return false;
}
#define RS_SLOT_OK(a, slot, what, pos) \
    ((a).nslots <= 0 || (uint32_t(slot) < uint32_t((a).nslots)) || rs_slot_fail((a).slot_err, (what), (pos), (slot)))
#else
#define RS_SLOT_OK(a, slot, what, pos) true
#endif

template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ------------------------------------------ m <= 8, one dword per lane per input step (V = 1)
constexpr int V1_LDS_WORDS = 2048 + RING_SLOTS * 256;
// NB = 2 (one-table step, gen_asm.py v1h): a third 1024-dword table after the ring, L^-1 of (gamma^4 x) per
// coordinate byte, so the output stage converts A + gamma^4 B as L^-1(A) ^ G4(B)
constexpr int V1H_G4 = V1_LDS_WORDS;
constexpr int V1H_LDS_WORDS = V1_LDS_WORDS + 1024;

// gamma^4 * v for one GF(256) byte in gamma-basis coordinates (xt8's reduction, four times)
__device__ __forceinline__ uint32_t gmul_g4(uint32_t v) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v = ((v << 1) & 0xFEu) ^ ((v >> 7) * 0x1Du);
    return v;
}

// Output p of the tile in GF(2^16) words: accumulator a0[p] / a1[p - 16] (GF(256)^2 coordinates) through
// L^-1; NB = 2 adds gamma^4 times b0[p] / b1[p - 16] through the G4 table.
template <int NB, int G4 = V1H_G4>
__device__ __forceinline__ uint32_t m8_v1_out(const uint32_t* lt, int p, const u32x16& a0, const u32x16& a1,
                                              const u32x16& b0, const u32x16& b1) {
    uint32_t w = lds_lookup4(lt + 1024, p < 16 ? a0[p & 15] : a1[p & 15]);
    if constexpr (NB == 2) w ^= lds_lookup4(lt + G4, p < 16 ? b0[p & 15] : b1[p & 15]);
    return w;
}

typedef int32_t i32x16s __attribute__((ext_vector_type(16)));

// The 32 output slots of a tile (out[0..31], 16-byte aligned, read-only) into SGPRs: two SMEM loads and
// one wait, instead of one scalar round trip per output. The outputs are early-clobber: the second load
// reads the base after the first was issued, and SMEM does not interlock its results, so a base placed
// inside o0 could be overwritten in flight and the second load would fetch from o0's data as an address
// (round 4's illegal-address fault: s_load_dwordx16 s[8:23], s[10:11] then s_load_dwordx16 s[72:87],
// s[10:11], 0x40 -- DESIGN.md section 7; scripts/isa_hazards.py checks every kernel for this class).
__device__ __forceinline__ void sload32(const int32_t* out, i32x16s& o0, i32x16s& o1) {
    asm volatile("s_load_dwordx16 %0, %2, 0x0\n\ts_load_dwordx16 %1, %2, 0x40\n\ts_waitcnt lgkmcnt(0)"
                 : "=&s"(o0), "=&s"(o1)
                 : "s"(out)
                 : "memory");
}

// The V = 1 kernels' outputs: row p of the tile back to GF(2^16) words (m8_v1_out) and stored to
// dst + out[p] * dst_sym, or XORed into it (V1Args::xor_dst: every old value is loaded first, so the
// wave waits on one round of loads while it converts its outputs).
template <int NB, int LBX = 0, int G4 = V1H_G4>
__device__ __forceinline__ void m8_v1_store(const V1Args& a, const uint32_t* lt, uint8_t* dst, const int32_t* out,
                                            int rows, const u32x16& a0, const u32x16& a1, const u32x16& b0,
                                            const u32x16& b1) {
    i32x16s o0, o1;
    sload32(out, o0, o1);
    auto slot = [&](int p) { return p < 16 ? o0[p & 15] : o1[p & 15]; };
    auto at = [&](int p) { return reinterpret_cast<uint32_t*>(dst + int64_t(slot(p)) * a.dst_sym); };
    // diagnostic builds: a slot outside the codec's range is recorded and its store (and old-value load)
    // skipped, so a violation never writes another slot's data; release builds: always true
    auto ok = [&](int p) { return RS_SLOT_OK(a, slot(p), 2, p); };
#if defined(RS_AMD_DIAG) && !defined(RS_JIT_SOURCE)
    if (a.ablate & 2) {  // timing ablation: raw accumulators, no L^-1 conversion (wrong results)
#pragma unroll
        for (int p = 0; p < 32; ++p)
            if (p < rows && ok(p)) *at(p) = p < 16 ? a0[p & 15] : a1[p & 15];
        return;
    }
#endif
    if (a.xor_dst) {  // g ^ (W S), in rounds of LB loads (NB = 2 holds twice the accumulators)
        constexpr int LB = LBX ? LBX : NB == 2 ? 16 : 32;
#pragma unroll
        for (int p0 = 0; p0 < 32; p0 += LB) {
            uint32_t old[LB];
#pragma unroll
            for (int q = 0; q < LB; ++q) old[q] = p0 + q < rows && ok(p0 + q) ? *at(p0 + q) : 0u;
#pragma unroll
            for (int q = 0; q < LB; ++q)
                if (p0 + q < rows && ok(p0 + q)) *at(p0 + q) = m8_v1_out<NB, G4>(lt, p0 + q, a0, a1, b0, b1) ^ old[q];
        }
        return;
    }
    // Outputs are stored from p = 31 down in groups of 8: a group past the tile's rows is skipped (one uniform
    // branch), and in the group holding row rows - 1 every p >= rows goes to that row's address first, so that
    // output's own store (same lane, same address, later in program order) is the one that stays; each group is
    // straight-line code with 32 LDS reads in flight.
    const int32_t slast = sload(out + (rows - 1));
#pragma unroll
    for (int p0 = 24; p0 >= 0; p0 -= 8) {
        if (p0 >= rows) continue;  // a whole group past the tile's rows (uniform): not converted
        uint32_t w[8];
#pragma unroll
        for (int q = 7; q >= 0; --q) w[q] = m8_v1_out<NB, G4>(lt, p0 + q, a0, a1, b0, b1);
#pragma unroll
        for (int q = 7; q >= 0; --q) {
            const int32_t sl = p0 + q < rows ? slot(p0 + q) : slast;
            if (RS_SLOT_OK(a, sl, 2, p0 + q)) *reinterpret_cast<uint32_t*>(dst + int64_t(sl) * a.dst_sym) = w[q];
        }
    }
}

// The one-table solves' store stage (k_apply_m8_pf, stored outputs): output p = L^-1(A_p) ^ G4(B_p) as eight LDS
// reads folded by three-input XORs (v_bitop3: 4 VALU instead of 7), stored at base + slot * dst_sym + voff with the
// row address formed in SGPRs (base and the slots are uniform) and the lane's byte offset as the store's VGPR
// offset, so a store costs no VALU. Same order and same-address rule as m8_v1_store's store path.
template <int G4>
__device__ __forceinline__ uint32_t m8_v1h_out(const uint32_t* lt, uint32_t x, uint32_t y) {
    const uint32_t* li = lt + 1024;
    const uint32_t* g = lt + G4;
    const uint32_t r0 = li[x & 255u], r1 = li[256 + ((x >> 8) & 255u)], r2 = li[512 + ((x >> 16) & 255u)],
                   r3 = li[768 + (x >> 24)];
    const uint32_t r4 = g[y & 255u], r5 = g[256 + ((y >> 8) & 255u)], r6 = g[512 + ((y >> 16) & 255u)],
                   r7 = g[768 + (y >> 24)];
    uint32_t w = __builtin_amdgcn_bitop3_b32(r0, r1, r2, 0x96);
    w = __builtin_amdgcn_bitop3_b32(w, r3, r4, 0x96);
    w = __builtin_amdgcn_bitop3_b32(w, r5, r6, 0x96);
    return w ^ r7;
}

template <int G4>
__device__ __forceinline__ void m8_v1h_store(const V1Args& a, const uint32_t* lt, uint8_t* base, uint32_t voff,
                                             const int32_t* out, int rows, const u32x16& a0, const u32x16& a1,
                                             const u32x16& b0, const u32x16& b1) {
    i32x16s o0, o1;
    sload32(out, o0, o1);
    auto slot = [&](int p) { return p < 16 ? o0[p & 15] : o1[p & 15]; };
    const int32_t slast = sload(out + (rows - 1));
#pragma unroll
    for (int p0 = 24; p0 >= 0; p0 -= 8) {
        if (p0 >= rows) continue;  // a whole group past the tile's rows (uniform): not converted
        uint32_t w[8];
#pragma unroll
        for (int q = 7; q >= 0; --q) {
            const int p = p0 + q;
            w[q] = m8_v1h_out<G4>(lt, p < 16 ? a0[p & 15] : a1[p & 15], p < 16 ? b0[p & 15] : b1[p & 15]);
        }
#pragma unroll
        for (int q = 7; q >= 0; --q) {
            const int32_t sl = p0 + q < rows ? slot(p0 + q) : slast;
            if (!RS_SLOT_OK(a, sl, 2, p0 + q)) continue;  // diagnostic builds: recorded, not stored
            uint8_t* d = base + int64_t(uint32_t(sl)) * a.dst_sym;  // slots >= 0
            asm volatile("global_store_dword %0, %1, %2" ::"v"(voff), "v"(w[q]), "s"(d) : "memory");
        }
    }
}

// Block = 256 lanes x 4 B = one 1 KiB column chunk of one stripe, 32 output rows of tile
// blockIdx.y. Per batch of 4 inputs: wave (i % 4) issues input i's DMA RING_B batches ahead; every
// wave reads its 4 dwords from the ring, maps them to GF(256)^2 coordinates (LDS byte tables) and
// runs `step(y, i, tile, acc0_15, acc16_31, record)` per input (record: the plan's 64-dword nibble
// record of (tile, input)); one s_barrier per batch. Outputs go back through L^-1 into 4-byte
// stores. With per-stripe plans (a.ps_kr) K, R, the slot lists and the records are the stripe's own.
// NB = 2: the step also takes the second accumulator set (step(y, i, tile, a0, a1, b0, b1, record)) and
// lds must hold V1H_LDS_WORDS. CB (1, 2 or 4): inputs converted to coordinates per LDS round trip.
// STAMP (diagnostic kernels): per wave, s_memtime cycles of [0] table setup, [1] ring prologue, [2] input
// steps (with their conversions), [3] DMA waits + barriers, [4] output stage, [5] total, [6] / [7] start /
// end time, into a.stamps[((blockIdx.y * gridDim.x + blockIdx.x) * 4 + wave) * 8 + ...].
__device__ __forceinline__ uint64_t v1_stamp() {
    uint64_t v;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");
    return v;
}

template <int NB = 1, int CB = 4, bool STAMP = false, bool MULTI = false, class Step>
__device__ __forceinline__ void m8_v1_run(const V1Args& a, uint32_t* lds, Step&& step) {
    uint64_t ph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, ts = 0;
    if constexpr (STAMP) ph[6] = ts = v1_stamp();
    const uint32_t* lt = lds;
    uint32_t* ring = lds + 2048;
    // block -> (launch-local stripe, its chunks [cbeg, cend)): MULTI kernels walk a.cpb column chunks of the
    // stripe, so the table setup is paid once and each next chunk's ring prologue is in flight during the
    // current chunk's output stage (a separate instantiation: the chunk loop costs registers)
    const int cpb = MULTI && a.cpb > 1 ? a.cpb : 1;
    const int64_t ngrp = (a.nchunks + cpb - 1) / cpb;
    const int64_t bid = blockIdx.x;
    const int64_t local = bid / ngrp;  // launch-local stripe
    const int64_t stripe = RS_STRIPE(a.ids, local);
    const int64_t cbeg = (bid - local * ngrp) * cpb;
    const int64_t cend = MULTI ? min(cbeg + int64_t(cpb), a.nchunks) : cbeg + 1;
    const int tile = blockIdx.y;
    int K = a.K, R = a.R;
    const int32_t* in_idx = a.in_idx;
    const int32_t* out_idx = a.out_idx;
    const uint32_t* idxb = a.idx;
    // split-K (small grids, one plan for all stripes, one chunk per block): this workgroup takes inputs
    // [i0, i0 + K) of the list and leaves its partial outputs for k_xor_slices
    const int slice = blockIdx.z;
    const int kfull = a.K;
    int i0 = 0;
    if (a.kslices > 1 && !a.ps_kr) {
        i0 = int(int64_t(a.K) * slice / a.kslices);
        K = int(int64_t(a.K) * (slice + 1) / a.kslices) - i0;
        in_idx += i0;
    }
    if (a.ps_kr) {  // this stripe's own plan
        K = sload(a.ps_kr + 2 * local);
        R = sload(a.ps_kr + 2 * local + 1);
        if (tile * 32 >= R) return;  // uniform over the block: no barrier is left waiting
        in_idx += local * a.ps_in;
        out_idx += local * a.ps_out;
        idxb += local * a.ps_idx;
    }
    const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x) >> 6);
    const int lane = threadIdx.x & 63;
    const int rows = min(32, R - tile * 32);
    const uint32_t ring_lds = uint32_t(reinterpret_cast<uintptr_t>(ring));
    // wave-uniform base of the current chunk (SGPRs); the lane's 16-byte offset is added per DMA, so the
    // chunk loop carries no 64-bit per-lane pointer
    const uint8_t* gsb = a.src + stripe * a.src_stripe + cbeg * 1024;
    auto issue = [&](int i) {
        int32_t s = sload(in_idx + i);
        if (!RS_SLOT_OK(a, s, 1, i)) s = 0;  // diagnostic builds: record, read slot 0 instead
        dma16(gsb + int64_t(s) * a.src_sym + 16 * lane, ring_lds + uint32_t(i % RING_SLOTS) * 1024u);
    };
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
    // the prologue's wait after an output stage: that stage's `pend` stores are newer than the prologue's
    // DMAs and may still be in flight (vmcnt counts both, in issue order)
    auto wait_pro = [&](int n, int pend) {
        if (pend == 32) {
            if (n <= 0)
                wait_vm<32>();
            else if (n == 1)
                wait_vm<33>();
            else
                wait_vm<34>();
        } else {
            wait_mine(n);
        }
    };
    u32x16 a0 = 0, a1 = 0, b0 = 0, b1 = 0;
    auto lap = [&](int k) {
        if constexpr (STAMP) {
            const uint64_t t = v1_stamp();
            ph[k] += t - ts;
            ts = t;
        }
    };
    // the ring prologue's DMAs go out first, then the coordinate tables are copied into LDS: the two
    // latencies overlap (the ring area and the tables are disjoint)
    for (int b = 0; b < RING_B; ++b)
        if (4 * b + wave < K) issue(4 * b + wave);
#if defined(RS_AMD_DIAG) && !defined(RS_JIT_SOURCE)
    if (!(a.ablate & 1))  // timing ablation: the tables are not copied (wrong results)
#endif
        for (int i = threadIdx.x; i < 2048; i += 256) lds[i] = a.ltab[i];
    if constexpr (NB == 2) {
        __syncthreads();
        for (int i = threadIdx.x; i < 1024; i += 256) lds[V1H_G4 + i] = lds[1024 + (i & ~255) + gmul_g4(i & 255)];
    }
    __syncthreads();
    lap(0);
    int pend = 0;
    for (int64_t c = cbeg; c < cend; ++c) {
        const int64_t chunk0 = c * 1024;
        wait_pro(mine(1, RING_B - 1), pend);
        asm volatile("s_barrier" ::: "memory");
        lap(1);
        for (int b = 0; b < nb; ++b) {
            const int ib = 4 * (b + RING_B) + wave;
            if (ib < K) issue(ib);
            // the batch's inputs in coordinates (slots past K hold stale bytes and are not used), CB at a
            // time (one LDS latency per CB inputs; each converted input held across the steps before its own
            // costs a VGPR)
            uint32_t y[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (j % CB == 0) {
#pragma unroll
                    for (int q = j; q < j + CB; ++q)
                        y[q] = lds_lookup4(lt, ring[((4 * b + q) % RING_SLOTS) * 256 + threadIdx.x]);
                }
                const int i = 4 * b + j;
                if (i < K) {
                    const uint32_t* rec = idxb + (size_t(tile) * (a.ps_kr ? K : kfull) + i0 + i) * 64;
                    if constexpr (NB == 2)
                        step(y[j], i, tile, a0, a1, b0, b1, rec);
                    else
                        step(y[j], i, tile, a0, a1, rec);
                }
            }
            lap(2);
            wait_mine(mine(b + 2, b + RING_B));
            asm volatile("s_barrier" ::: "memory");
            lap(3);
        }
        if (a.kslices > 1 && !a.ps_kr) {  // partial products (L^-1 is GF(2)-linear: XOR of converted partials)
            const int64_t nloc = gridDim.x / a.nchunks, rpad = int64_t(gridDim.y) * 32, cw = a.nchunks * 256;
            uint32_t* part = a.partial + ((slice * nloc + local) * rpad + tile * 32) * cw + (chunk0 >> 2) + threadIdx.x;
#pragma unroll
            for (int p = 0; p < 32; ++p)
                if (p < rows) part[p * cw] = m8_v1_out<NB>(lt, p, a0, a1, b0, b1);
            return;
        }
        // every wave has read the whole ring (last barrier): the next chunk's prologue may refill it now
        if (MULTI && c + 1 < cend) {
            gsb += 1024;
            for (int b = 0; b < RING_B; ++b)
                if (4 * b + wave < K) issue(4 * b + wave);
        }
        m8_v1_store<NB, MULTI ? 8 : 0>(a, lt, a.dst + stripe * a.dst_stripe + chunk0 + int64_t(threadIdx.x) * 4,
                                        out_idx + tile * 32, rows, a0, a1, b0, b1);
        if constexpr (MULTI) {
            pend = rows;
            // zero the accumulators where the input step keeps them (NB = 1: v[40:71], gen_asm.py v1)
            asm volatile(
                "v_mov_b32 v40, 0\n\tv_mov_b32 v41, 0\n\tv_mov_b32 v42, 0\n\tv_mov_b32 v43, 0\n\t"
                "v_mov_b32 v44, 0\n\tv_mov_b32 v45, 0\n\tv_mov_b32 v46, 0\n\tv_mov_b32 v47, 0\n\t"
                "v_mov_b32 v48, 0\n\tv_mov_b32 v49, 0\n\tv_mov_b32 v50, 0\n\tv_mov_b32 v51, 0\n\t"
                "v_mov_b32 v52, 0\n\tv_mov_b32 v53, 0\n\tv_mov_b32 v54, 0\n\tv_mov_b32 v55, 0\n\t"
                "v_mov_b32 v56, 0\n\tv_mov_b32 v57, 0\n\tv_mov_b32 v58, 0\n\tv_mov_b32 v59, 0\n\t"
                "v_mov_b32 v60, 0\n\tv_mov_b32 v61, 0\n\tv_mov_b32 v62, 0\n\tv_mov_b32 v63, 0\n\t"
                "v_mov_b32 v64, 0\n\tv_mov_b32 v65, 0\n\tv_mov_b32 v66, 0\n\tv_mov_b32 v67, 0\n\t"
                "v_mov_b32 v68, 0\n\tv_mov_b32 v69, 0\n\tv_mov_b32 v70, 0\n\tv_mov_b32 v71, 0"
                : "=&{v[40:55]}"(a0), "=&{v[56:71]}"(a1));
        }
        lap(4);
    }
    if constexpr (STAMP) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lap(4);
        ph[7] = ts;
        ph[5] = ts - ph[6];
        if (lane == 0) {
            uint64_t* o = a.stamps + ((int64_t(blockIdx.y) * gridDim.x + blockIdx.x) * 4 + wave) * 8;
#pragma unroll
            for (int k = 0; k < 8; ++k) o[k] = ph[k];
        }
    }
}
