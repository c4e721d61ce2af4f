// rs_jit.hpp -- coding-matrix-specialised V = 1 kernels compiled at run time with hiprtc.
//
// The generic m <= 8 kernels pick each (output, input) nibble table entry with gpr-index mode: an
// s_set_gpr_idx_idx plus an indexed v_xor, which issues at half rate. With the matrix known, the
// lookups of input i become a block of fixed-register v_xor (zero nibbles dropped) followed by
// s_setpc_b64; the kernel's generic loop (rs_device.h:m8_v1_run) builds the nibble tables and
// s_swappc_b64's into block i. 64 lookups per input = 260 B, so a 128-input tile's blocks
// (33 KB) stay resident in the instruction cache. One kernel per matrix, cached in memory and on
// disk (RS_AMD_JIT_CACHE, default <lib dir>/jit_cache).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "rs_v1args.h"

namespace rsamd {

struct JitModule;

struct JitKernel {
    std::shared_ptr<JitModule> mod;
    hipFunction_t fn = nullptr;
    int32_t* d_boff = nullptr;  // [ntiles][K] block byte offsets (device)
    int device = 0;
    int ntiles = 0;
    std::string name;
    ~JitKernel();
};

// Largest number of lookup blocks (tiles x inputs) per kernel: 256 x 260 B = 66 KB of blocks.
constexpr int kJitMaxBlocks = 256;

bool jit_supported(int m, int K, int R);
// cg: [R][K] coefficients in GF(256) gamma-basis coordinates (Gamma8::coord of the GF(2^16) entry).
// Builds (or fetches) the kernel; RS_ERR_DEVICE-style nonzero on failure, `out` empty if unsupported.
int jit_build(const std::vector<uint8_t>& cg, int K, int R, std::unique_ptr<JitKernel>& out);
// Compiles into the disk cache only (no GPU needed).
int jit_precompile(const std::vector<uint8_t>& cg, int K, int R);
// Launches over `nchunks_1k` full 1 KiB column chunks of every stripe (v.boff is filled in here).
int jit_launch(const JitKernel& k, V1Args v, int64_t n_stripes, hipStream_t st);
// Shared hiprtc machinery (also used by rs_xj.cpp): code object from the disk cache (file
// <prefix>_<hash>.co) or compiled; module per (device, source hash), loaded once.
int jit_code(const std::string& src, const char* prefix, uint64_t h, std::vector<char>& code);
uint64_t jit_hash(const std::string& s);
int jit_module(const std::string& src, const char* prefix, std::shared_ptr<JitModule>& out, uint64_t* hash);
hipModule_t jit_module_handle(const JitModule& m);
// Source text of the specialised kernel and the per-block byte offsets (tests / inspection).
std::string jit_source(const std::vector<uint8_t>& cg, int K, int R, std::vector<int32_t>* boff);

}  // namespace rsamd
