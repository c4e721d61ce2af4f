// rs_symops.hpp -- device records and launcher of rsg_symbol_ops (kernels in rs_symops.hip, host side in
// rs_refops.cpp). Kept apart from rs_kernels.hpp so that the coding kernels' source hash (srchash.py, the key
// of the PMC traffic records) does not move with this surface.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rsamd {

// An op in canonical form (the host folds RSG_OP_* and the self-source cases, reference gf65536.c:155-219):
//   kSymXor   a ^= b               kSymMadd  a ^= coef * b   (coef not 0, 1)
//   kSymScale a = coef * a         (coef not 0, 1; also a ^= c a, i.e. (1 + c) a)
//   kSymZero  a = 0                (gf_mul by 0, a ^= a)       kSymNop   nothing (gf_mul by 1, madd by 0)
enum : uint32_t { kSymNop = 0, kSymXor = 1, kSymMadd = 2, kSymScale = 3, kSymZero = 4 };

// a chain: the ops of one target, ops[start, start + count) in order. kChainSplit: its ops may run as W slices of
// consecutive ops on W waves (wave 0 from the target, the others from zero) whose results are XORed. Every op is
// affine in the target (a = m a + b), so that is exact once each slice's result is multiplied by the product of
// the scale factors of the slices after it; kChainAffine: the chain scales (kSymScale / kSymZero ops) and those
// W products are the records ops[comb + w] (kinds kSymScale / kSymZero / kSymNop), else they are all 1.
struct SymChain {
    uint8_t* a;
    uint32_t start, count;
    uint32_t flags, comb;
};
constexpr uint32_t kChainSplit = 1u, kChainAffine = 2u;
constexpr int kSymMaxWaves = 8;  // waves per chain (workgroup size / 64)
struct SymOpRec {
    const uint8_t* b;  // source (kSymXor / kSymMadd), else null
    uint32_t coef, kind;
};

// Bytes of device scratch the launch needs after the records for n_ops ops (the multiply constants).
inline size_t symbol_chains_scratch(uint64_t n_ops) { return size_t(n_ops) * 64; }

// k_symop_consts: the 16 constants coef * alpha^i (both 16-bit halves) of every multiplying op of ops[0, n_ops)
// into consts[16 op + i] (64 B per op), once per call instead of once per wave and op on the scalar unit
hipError_t launch_symop_consts(const SymOpRec* ops, uint64_t n_ops, uint32_t* consts, hipStream_t st);
// k_symbol_chains<dw> over n_chains chains of nwords 16-bit words (dw dwords per lane: 256 * dw bytes of a
// symbol per wave; `waves` per chain and column span, 1..kSymMaxWaves); `ops` / `consts` indexed by the chains'
// op ranges
hipError_t launch_symbol_chains(const SymChain* chains, const SymOpRec* ops, const uint32_t* consts,
                                uint32_t n_chains, uint64_t nwords, hipStream_t st, int dw, int waves);

}  // namespace rsamd
