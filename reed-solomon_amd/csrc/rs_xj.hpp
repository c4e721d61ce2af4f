// rs_xj.hpp -- bit-plane XOR kernels: matrix-specialised m <= 8 encode/decode compiled at run time.
//
// Every coefficient c of a GF(256)-valued coding matrix is split into 8 bit-planes over a fixed basis
// {beta_t} of GF(256):  c = sum_t b_t(c) beta_t.  Then
//     out_p = sum_i c_{p,i} x_i = sum_t beta_t * u_{p,t},   u_{p,t} = XOR of x_i over {i : b_t(c_{p,i}) = 1},
// so the K x R matrix apply becomes a pure XOR network on raw GF(2^16) words (8R accumulators), and
// field multiplication happens once per OUTPUT (8 constant multiplies, Horner in alpha^-1) instead of
// once per input. The XOR network uses four-Russians tables: per group of 4 inputs the 11 non-trivial
// subset XORs are built once, so one v_bitop3 (3-input XOR) adds two groups (8 inputs) to an
// accumulator. All register indices are fixed by the matrix, so the kernel is generated per coding
// matrix (hiprtc) and cached in memory and on disk, like rs_jit.hpp.
//
// Work per 256-byte column of a stripe at k=128, r=32 (two roles of 16 outputs): 4096 XOR3 (rows) +
// 2 x 352 table XORs + 32 x ~88 finish ops ~= 7500 VALU, against ~18000 for the per-input
// multiple / nibble-table kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace rsamd {

struct JitModule;

// Kernel arguments of rs_xj (plain data; mirrored in the generated source).
struct XJArgs {
    const uint8_t* src;  // stripe 0 of the input layout
    int64_t src_stripe;
    uint8_t* dst;
    int64_t dst_stripe;
    int32_t src_sym, dst_sym;  // symbol strides (slot * stride < 2^31)
    const int32_t* ids;        // optional [n_stripes] stripe indices; null = 0..n-1
    const uint16_t* tab;       // persistent form (fin = 1): device table T[w] = gamma * w (set by xj_launch);
                               // coordinate outputs (masked form 2): the 1024-dword L byte tables (ApplyArgs::ltab)
    uint32_t nchunks, ncols;   // chunks per stripe (set by xj_launch); persistent form: chunks in the launch
    uint32_t dst_local;        // 1: dst indexed by the launch-local stripe (ids only select the source)
    // masked kernels (xj_build(..., masked)): input slot i of launch-local stripe s reads the zero buffer when
    // bit i % 32 of masks[s * mask_words + i / 32] is set. The fields trail the struct, so unmasked kernels
    // (whose generated source declares only the fields above) read the same prefix.
    uint32_t mask_words;
    const uint32_t* masks;
    const uint8_t* zero;       // zero bytes, at least as many as a symbol has (an erased slot's column c reads
                               // zero + c, so the reads of different columns spread over the memory channels)
};

struct XjKernel {
    std::shared_ptr<JitModule> mod;
    hipFunction_t fn = nullptr;
    int device = 0;
    int roles = 0;  // waves per column (opr outputs each)
    int pairs = 0;  // > 0: persistent kernel (LDS finish), columns per workgroup in flight, grid <= CUs
    int cpb = 1;    // consecutive 256-byte columns per workgroup (column loop), grid.x = chunks / cpb
    bool masked = false;  // per-stripe input masks (XJArgs::masks)
    bool coord = false;   // outputs stored in GF(256)^2 coordinates (masked form 2; XJArgs::tab = the L tables)
    std::string name;
    // wave instructions per 256-byte column, all role waves together, counted in the generated asm
    // (the XOR network, the finish once per role, loads / stores / addressing); the compiler's few
    // prologue instructions are not included
    uint64_t valu_per_col = 0, salu_per_col = 0;
};

constexpr int kXjMaxRoles = 16;     // 1024-thread blocks
constexpr int kXjMaxWork = 6144;    // K * R bound (instruction-cache footprint of the XOR network)
constexpr int kXjChunk = 256;       // column bytes per block (64 lanes x 4 B)

// Host-side decomposition (no GPU): basis bits of a GF(256) element and the finish map.
// Finish = Horner over a power basis {z^j} of GF(2^16): out = sum_j z^j v_j, v_j = XOR of the u_t whose
// beta_t has z-coordinate j. horner 1: z = alpha (packed-16 shift + sign-mask reduction, 3 ops per
// step), coordinates = raw bits; horner 0: z = alpha^-1 (mask/shift/multiply, 4 ops per step).
// beta_t is the reduced basis of GF(256) whose coordinates at pivots[t] form the identity; the pivot set
// minimises the finish cost.
struct XjBasis {
    int horner;            // 1: z = alpha, 0: z = alpha^-1
    int pivots[8];         // z-coordinate j carrying bit t
    uint16_t beta_y[8];    // beta_t in z-coordinates
    uint16_t ycoord(uint16_t x) const;  // x = sum_j y_j z^j
    uint8_t bits(uint16_t c) const;     // b_t(c), c in GF(256)
    explicit XjBasis(int horner);

   private:
    uint16_t inv_row_[16];  // row j of the inverse of [z^0 .. z^15] over GF(2)
};
const XjBasis& xj_basis(int horner);
int xj_horner(bool env_knobs = false);  // generation setting (RS_XJ_HORNER, default 0)

bool xj_supported(int m, int K, int R);
int xj_outputs_per_role();  // generation setting (RS_XJ_OPR, default 16)
int xj_roles(int R);         // waves per column for R outputs
int xj_max_roles(int R);     // role waves that fit one CU at the layout's VGPR footprint
int xj_fin();                // generation setting (RS_XJ_FIN, default 0)
int xj_pairs(int R);         // columns per workgroup (1 unless the LDS-table finish is on)
// M: R x K GF(2^16) matrix (entries in GF(256)); in_slots[K] / out_slots[R] symbol slots.
// env_knobs: honour the RS_XJ_* generation knobs (inspection / emulator tests; the launched kernels never do)
// masked: 1 the per-stripe input-mask form (XjConfig::masked, XJArgs::masks), default layout only; 2 the same
// with the outputs stored in GF(256)^2 coordinates (XjConfig::coord)
std::string xj_source(const std::vector<uint16_t>& M, int K, int R, const std::vector<int32_t>& in_slots,
                      const std::vector<int32_t>& out_slots, bool env_knobs = false, int masked = 0);
int xj_build(const std::vector<uint16_t>& M, int K, int R, const std::vector<int32_t>& in_slots,
             const std::vector<int32_t>& out_slots, std::unique_ptr<XjKernel>& out, int masked = 0);
int xj_precompile(const std::vector<uint16_t>& M, int K, int R, const std::vector<int32_t>& in_slots,
                  const std::vector<int32_t>& out_slots, int masked = 0);
// Launches over the first `nchunks` 256-byte column chunks of every stripe.
int xj_launch(const XjKernel& k, const XJArgs& a, int64_t n_stripes, int64_t nchunks, hipStream_t st);

}  // namespace rsamd
