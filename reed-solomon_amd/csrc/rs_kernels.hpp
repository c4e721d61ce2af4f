// rs_kernels.hpp -- launch interface of the HIP kernels (rs_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rs_v1args.h"

namespace rsamd {

// out[stripe][out_idx[p]] = sum_i C[p][i] * in[stripe][in_idx[i]]   for p < R, per 16-bit word.
struct ApplyArgs {
    const uint8_t* src;      // stripe 0 of the input layout
    int64_t src_stripe;      // bytes between stripes
    int64_t src_sym;         // bytes between symbols
    const int32_t* in_idx;   // [K] input symbol indices (device)
    uint8_t* dst;
    int64_t dst_stripe;
    int64_t dst_sym;
    const int32_t* out_idx;  // [R] output symbol indices (device)
    const uint32_t* coef;    // [ntiles][K][RT/4] gamma-basis bytes (m<=8) | [ntiles][K][RT/2] u16 (m=16)
    const uint32_t* idx;     // m<=8, RT=32, mode 2: [ntiles][K][64] pre-split nibble indices (lo, hi per output)
    const uint32_t* ltab;    // m<=8: [2048] LDS coordinate tables (L bytes 0..3, L^-1 bytes 0..3)
    int32_t K;
    int32_t R;
    int64_t nbytes;          // symbol size (even)
    int64_t nchunks;         // filled by launch_apply
    int64_t chunk_base;      // first column chunk (tail launches)
    int32_t mode;            // m<=8 inner loop: 0 = register nibble tables (compiler indexing),
                             //   1 = SGPR-masked multiples, 2 = hand-scheduled gpr-index block (RT=32)
    uint64_t* stamps;        // mode 17 (instrumented): [blocks * 4 waves][4] phase cycle counters
    const int32_t* ids;      // optional [n_stripes] stripe indices (per-stripe erasure patterns); null = 0..n-1
    uint32_t* scratch;       // m = 16 split-K partials (codec-owned), scratch_bytes long; may be null
    int64_t scratch_bytes;
    int32_t nslots;          // diagnostic builds: slot indices lie in [0, nslots) (V1Args::nslots); 0 = unchecked
    int32_t* slot_err;       // its violation record (V1Args::slot_err)
};
// input slices of the split-K m = 16 launch over n_stripes (1 = no split) and the scratch it needs
int m16_kslices(const ApplyArgs& a, int64_t n_stripes, int64_t* scratch_bytes);
// the same for the generic GF(256) V = 1 kernel (m8 mode 18, 32-row tiles)
int m8_kslices(const ApplyArgs& a, int64_t n_stripes, int64_t* scratch_bytes);

// Per-stripe decode plans (k_plan_m8): one per selected stripe, from its erasure mask.
struct PlanArgs {
    const uint8_t* masks;  // [n_sel][n] 1 = erased
    const uint16_t* elem;  // [n] X_j = alpha^position of slot j
    const uint16_t* logt;  // [65536] discrete log (entry 0 unused)
    const uint8_t* g8;     // [255] gamma-basis byte of alpha^(257 e)
    int32_t k, r, n;       // n = k + r <= 256
    int32_t* kr;           // [n_sel][2] survivors K, erased information slots R
    int32_t* pin;          // [n_sel][in_stride] survivor slots, zero-padded
    int32_t* pout;         // [n_sel][out_stride] erased information slots, zero-padded
    uint32_t* pidx;        // [n_sel][idx_stride] V = 1 nibble records, (tile * K + i) * 64
    int64_t in_stride, out_stride, idx_stride;
};
hipError_t launch_plan_m8(const PlanArgs& a, int64_t n_sel, hipStream_t st);

// Syndrome route of rsg_decode_batch (m <= 8): per selected stripe, the t_info x t matrix W that maps
// the first t syndromes S_j = sum_i X_i^j rcv_i to the erased information symbols (V = 1 nibble
// records; inputs are syndrome slots local * r + j of the syndrome scratch), and zeroes the stripe's
// erased information slots (the syndrome pass reads every slot).
struct SynPlanArgs {
    const uint8_t* masks;  // [n_sel][n] 1 = erased
    const uint16_t* elem;  // [n] X_j = alpha^position of slot j
    const uint16_t* logt;  // [65536] discrete log
    const uint16_t* expt;  // [65536] alpha^e, e < 65536
    const uint8_t* g8;     // [255] gamma-basis byte of alpha^(257 e)
    int32_t k, r, n;
    int32_t* kr;           // [n_sel][2] inputs t, erased information slots R
    int32_t* pin;          // [n_sel][in_stride] syndrome slots
    int32_t* pout;         // [n_sel][out_stride] erased information slots
    uint32_t* pidx;        // [n_sel][idx_stride] V = 1 nibble records
    int64_t in_stride, out_stride, idx_stride;
    uint32_t* mbits;       // [n_sel][mw] the pattern as bit words (slot i: bit i % 32 of word i / 32), for the
    int32_t mw;            // masked fixed pass (XJArgs::masks)
    // non-null: records in k_apply_m8_pf's packed form instead ([n_sel][idx8_stride bytes], per (tile, input)
    // 64 bytes: lookup L = 8 m + 2 k + d in byte k of dword 2 m + d; L < 32 the low nibble of output L, else
    // the high nibble of output L - 32)
    uint8_t* pidx8;
    int64_t idx8_stride;
};
// kind 1: syndrome-route solves (k_plan_syn_m8); 2: re-encode solves (k_plan_reenc_m8)
hipError_t launch_plan_syn_m8(const SynPlanArgs& a, int64_t n_sel, hipStream_t st, int kind = 1);

// One GF(2^16) coding matrix built on the device (gf16.cpp:solve_matrix's evaluation) straight into
// the m = 16 kernels' formats: coefficient tiles (k_apply_m16) and, if rec != null, the packed index
// records of k_apply_m16_v1 (rt = 64). coef / rec must be zeroed by the caller.
struct Plan16Args {
    const uint16_t* src_el;  // [K] source elements Y_q
    const uint16_t* tgt_el;  // [d] all target elements X_e
    const int32_t* emit;     // [R] emitted target indices (matrix rows)
    const uint16_t* logt;    // [65536] discrete log
    const uint16_t* expt;    // [65536] alpha^i, i < 65535 (entry 65535 = 1)
    uint32_t* lp;            // [K] scratch
    uint32_t* ld;            // [R] scratch
    uint32_t* coef;          // [ntiles][K][rt / 2]
    uint8_t* rec;            // [ceil(R / 64)][K + 1][256] or null
    int32_t K, d, R, rt;
};
hipError_t launch_plan_m16(const Plan16Args& a, hipStream_t st);
// Per-stripe GF(2^16) decode (rsg_decode_batch, the syndrome route with a plan per stripe). With E the
// stripe's erased slots (t <= r) and P(x) = prod_{e in E} (x + X_e), the reference's evaluator / Forney
// restore (reed_solomon.c:186-336) solves sum_{e in E} X_e^j d_e = S_j, j < t, over the syndromes of all
// k + r slots (fft.c:39-100, erased slots read as zero). Its inverse row for erased information slot p is
// W[p][j] = q_{p,j} / prod_{e != p} (X_p + X_e), q_p = P(x) / (x + X_p) (Lagrange; the same linear map,
// so results are bit-identical).
constexpr int kPs16MaxR = 4096;  // r bound of the path (P's product tree lives in LDS)
struct Ps16Args {
    const uint8_t* masks;  // [n_sel][n] 1 = erased
    const uint16_t* elem;  // [n] X_i = alpha^position of slot i
    const uint16_t* logt;  // [65536] discrete log
    const uint16_t* expt;  // [65536] alpha^e, e < 65535
    int32_t k, r, n;
    int32_t* kr;           // [n_sel][2] t, R (erased information slots)
    uint16_t* ee;          // [n_sel][r] erased elements X_e, slot order
    uint16_t* pe;          // [n_sel][out_stride] elements of the erased information slots (rows), zero-padded
    int32_t* pout;         // [n_sel][out_stride] erased information slots, zero-padded
    uint16_t* cf;          // [n_sel][r + 1] coefficients of P (cf[t] = 1)
    int64_t out_stride;    // row tiles * 64
    uint32_t* rec;         // [n_sel][rec_stride] k_apply_m16_v1 records of W: [tile][t + 1][64] dwords
    int64_t rec_stride;
    int32_t tblocks;       // workgroups (4 tiles each) per stripe of the record build
    uint8_t* base;         // stripes: the erased information slots are zeroed (the syndromes read every slot)
    int64_t stripe_stride, symbol_stride, S;
    const int32_t* ids;    // [n_sel] stripe indices
    // re-encode variant (k_plan16_reenc*): sources = the first t_info surviving repair slots R'
    int32_t* pin;          // [n_sel][in_stride] their rows in the fixed pass's output (repair slot - k)
    uint16_t* qe;          // [n_sel][in_stride] their elements X_q
    uint32_t* lq;          // [n_sel][in_stride] log L_T(X_q)
    uint32_t* lr;          // [n_sel][out_stride] log L_T'(X_p) of the rows (T = E + repair slots not in R')
    int64_t in_stride;
    int32_t lblocks;       // workgroups per stripe of the log sums
};
// lists, P and the zeroing (one workgroup per stripe), then the records (tblocks workgroups per stripe)
hipError_t launch_plan16_ps(const Ps16Args& a, int64_t n_sel, hipStream_t st);
hipError_t launch_plan16_ps_rec(const Ps16Args& a, int64_t n_sel, hipStream_t st);
// the re-encode variant: lists + T + zeroing (one workgroup per stripe), the log sums (lblocks per stripe),
// the records of W' (tblocks per stripe)
hipError_t launch_plan16_reenc(const Ps16Args& a, int64_t n_sel, hipStream_t st);
hipError_t launch_plan16_reenc_rec(const Ps16Args& a, int64_t n_sel, hipStream_t st);
// k_apply_m16_v1 in per-stripe mode over the full 1 KiB chunks (v.ps_* set, tiles = the largest stripe's)
hipError_t launch_apply_m16_ps(const V1Args& v, int64_t n_sel, int64_t nbytes, int tiles, hipStream_t st);
// V = 1 kernel over the full 1 KiB chunks + per-stripe tail kernel, plans in v.ps_* (n_sel stripes);
// kernel = option m8_ps_kernel, cpb = column chunks per block of the ring kernels (option m8_ps_cpb)
hipError_t launch_apply_m8_ps(const V1Args& v, int64_t n_sel, int64_t nbytes, int tiles, hipStream_t st,
                              int kernel = 0, int cpb = 1);

// dst row j = src row rows[j] for j < nrows, `width` bytes each (16-byte aligned rows, padded pitch)
hipError_t launch_gather_rows(uint8_t* dst, int64_t dpitch, const uint8_t* src, int64_t spitch, const int32_t* rows,
                              int64_t nrows, int64_t width, hipStream_t st);
// dst row rows[j] = src row rows[j] (same slot, different pitch): the per-call decode writes its
// restored rows straight into the caller's page-locked stripe (dst a device-visible host address);
// rows == nullptr: rows 0 .. nrows - 1
hipError_t launch_put_rows(uint8_t* dst, int64_t dpitch, const uint8_t* src, int64_t spitch, const int32_t* rows,
                           int64_t nrows, int64_t width, hipStream_t st);
// registered caller symbols (rs_api.cpp, drop-in path): bytes [off, off + width) of dst row i = those of
// the symbol at device-visible address ptrs[i], for the rows i in rows[0 .. nrows) (rows null: 0 .. nrows
// - 1), and back (scatter). 16-byte units: addresses, pitch, offset and width multiples of 16.
hipError_t launch_gather_ptrs(uint8_t* dst, int64_t dpitch, const uint64_t* ptrs, const int32_t* rows, int64_t nrows,
                              int64_t off, int64_t width, hipStream_t st);
hipError_t launch_scatter_ptrs(const uint64_t* ptrs, const uint8_t* src, int64_t spitch, const int32_t* rows,
                               int64_t nrows, int64_t off, int64_t width, hipStream_t st);
// row p of stripe s of dst ^= the same row of src (p < nrows, S bytes, 4-byte aligned; the re-encode decode)
hipError_t launch_xor_rows(uint8_t* dst, int64_t dst_stripe, int64_t dst_sym, const uint8_t* src, int64_t src_stripe,
                           int64_t src_sym, int64_t nrows, int64_t S, int64_t n_stripes, hipStream_t st);

// m = 16 cyclotomic syndromes (k_cs16, the reference's fft_transform_cycl structure, src/rs/fft.c:39-100):
// S_j = sum_i X_i^j in_i for the needed j, inputs grouped by cyclotomic coset (16 slots at positions
// L * 2^a), syndromes by coset s (16 normal-basis accumulators each, 4 cosets per wave = one tile).
struct Cs16Args {
    const uint8_t* src;       // stripe 0 of the input layout
    int64_t src_stripe, src_sym;
    const uint32_t* goff;     // [ngroups + 3][16] byte offset (slot * src_sym) of the input at position
                              // L_g * 2^a; 0x80000000 = no input there (loads out of range: zero)
    uint32_t in_bytes;        // inputs' byte range past the stripe base (< 2^31; the V#'s num_records)
    const uint32_t* rec;      // [ntiles][ngroups + 2][16] packed gpr-index records (gen_asm.py cs16a/b)
    const int32_t* fin;       // [ntiles][fin_stride] needed syndromes: local coset | b << 4 | j << 8
    const int32_t* fin_off;   // [ntiles][cw + 1] entries of local coset c: [fin_off[c], fin_off[c + 1])
    int32_t cw = 4;           // syndrome cosets per tile (k_cs16 / k_bs16: 4; k_cs16t: kCs16tCw)
    int32_t fin_stride;
    uint8_t* dst;             // syndrome j of launch-local stripe s at dst + s * dst_stripe + j * dst_sym
    int64_t dst_stripe, dst_sym;
    const uint16_t* logt;     // [65536] discrete log
    const uint16_t* expt;     // [65536] alpha^e, e < 65535
    uint32_t nblog[16];       // log of the GF(2^16) normal basis elements nb_t
    int32_t ngroups, ntiles;  // ngroups even (padded with empty groups)
    int64_t nchunks;          // columns (colw bytes) per symbol
    int64_t units;            // n_stripes * nchunks
    int32_t colw;             // 1024: block = 4 waves on one 1 KiB column, one tile; 256: every wave one
                              // (256-byte column, tile) pair, 4 consecutive pairs per block (rs_kernels.hip)
    const int32_t* ids;       // optional [n_stripes] stripe indices (inputs only)
};
hipError_t launch_cs16(const Cs16Args& a, hipStream_t st);
// the same syndromes by threaded code blocks (k_cs16t): tiles of cw = kCs16tCw cosets, records
// [ntiles][ngroups + 2][4 cw] uint32 block offsets (gen/cs16t_off.h), one group per step
hipError_t launch_cs16t(const Cs16Args& a, hipStream_t st);
// binary accumulation with per-accumulator indices (k_bs16): records [ntiles][ngroups + 2][4][64] bytes,
// finish entries' j = output slot, written at dst + stripe * dst_stripe + j * dst_sym
hipError_t launch_bs16(const Cs16Args& a, hipStream_t st);
// goff[i] = slots[i] * sym (0x80000000 for slots[i] < 0), i < n
hipError_t launch_cs16_goff(const int32_t* slots, uint32_t* goff, int n, int64_t sym, hipStream_t st);

// symbol-wide word ops over nw words (a multiple of 8; a, b 16-byte aligned): op 0 a ^= b, 1 a = c * a,
// 2 a ^= c * b (lc = log c; logt / expt: discrete log and alpha^i tables, i < 65535)
hipError_t launch_symbol_op(uint16_t* a, const uint16_t* b, int op, uint32_t lc, int64_t nw, const uint16_t* logt,
                            const uint16_t* expt, hipStream_t st);
int apply_tile_rows(int m, int R);
// V = 1 kernel arguments from an ApplyArgs (nchunks_1k full 1 KiB chunks; boff for the JIT kernel)
V1Args v1_args(const ApplyArgs& a, int64_t nchunks_1k, const int32_t* boff);
// the register-ring kernel over the columns past the last full 2 KiB chunk (no-op if none)
void launch_m8_tail(const ApplyArgs& a, int64_t n_stripes, unsigned tiles, hipStream_t st);
int64_t apply_chunk_bytes(int m);
hipError_t launch_apply(int m, int rt, ApplyArgs a, int64_t n_stripes, hipStream_t st);
hipError_t launch_gen_info(uint8_t* base, int64_t stripe_stride, int64_t sym_stride, int64_t S, int k, int64_t stripe0,
                           int64_t n_stripes, uint64_t seed, hipStream_t st);
hipError_t launch_fingerprint(const uint8_t* base, int64_t stripe_stride, int64_t sym_stride, int64_t S, int sym0,
                              int nsym, int64_t n_stripes, unsigned long long* out, hipStream_t st);

}  // namespace rsamd
