// rs_jit.hpp -- coding-matrix-specialised kernels compiled at run time with hiprtc.
//
// For m <= 8 codes the generic kernels spend most of their issue slots deciding, per
// (output, input), which precomputed multiples to XOR (wave-uniform coefficient bits -> SALU
// work or masks). Baking the matrix into the code turns every (output, input) pair into 1-2
// straight-line 3-input XORs with no scalar work at all. One kernel per matrix, cached in memory
// and on disk (RS_AMD_JIT_CACHE, default <lib dir>/jit_cache).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace rsamd {

struct JitModule;

struct JitKernel {
    std::shared_ptr<JitModule> mod;
    hipFunction_t fn = nullptr;
    std::string name;
};

// Largest matrix (K * R) the specialiser accepts; bigger ones stay on the generic kernels.
constexpr int64_t kJitMaxPairs = 8192;
constexpr int kJitMaxRows = 32;

bool jit_supported(int m, int K, int R);
// Builds (or fetches) the kernel for an m <= 8 matrix M[R][K] (GF(2^16) values in GF(256)).
// Returns 0 and leaves `out` empty when the shape is not supported; RS_ERR_DEVICE on failure.
int jit_build(const std::vector<uint16_t>& M, int K, int R, const std::vector<int32_t>& in_slots,
              const std::vector<int32_t>& out_slots, std::unique_ptr<JitKernel>& out);
// Compiles into the disk cache only (no GPU needed).
int jit_precompile(const std::vector<uint16_t>& M, int K, int R, const std::vector<int32_t>& in_slots,
                   const std::vector<int32_t>& out_slots);
int jit_launch(const JitKernel& k, const uint8_t* src, int64_t src_stripe, int64_t src_sym, uint8_t* dst,
               int64_t dst_stripe, int64_t dst_sym, int64_t n_stripes, int64_t nbytes, const uint32_t* ltab,
               hipStream_t st);
// Source text of the specialised kernel (exposed for tests / offline inspection).
std::string jit_source(const std::vector<uint16_t>& M, int K, int R, const std::vector<int32_t>& in_slots,
                       const std::vector<int32_t>& out_slots);

}  // namespace rsamd
