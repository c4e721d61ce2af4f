/*
 * rs_amd/rsg.h -- batched, device-resident Reed-Solomon engine API (librs_amd.so).
 *
 * The per-call drop-in API (rs/reed_solomon.h) codes one stripe held in host memory. This API codes
 * many stripes that already live in HBM: a stripe is k information + r repair symbols of
 * `symbol_size` bytes, addressed as  base + stripe * stripe_stride + symbol * symbol_stride.
 * It is what the reference's rs_generate_repair_symbols (src/rs/reed_solomon.c:338-441) and
 * rs_restore_symbols (src/rs/reed_solomon.c:443-559) become when the buffers are device-resident;
 * results are bit-identical, stripe by stripe, under the reference's contract that erased slots hold
 * zeros on entry (reed_solomon.h:64). Erased slots are never read here, so with garbage in them this
 * library still restores the true symbols, where the reference (whose syndromes read every slot,
 * fft.c:68-75) would not: parity for non-zeroed erased slots is by design, not with the reference.
 *
 * Plain C ABI: device pointers, sizes, `stream` is a hipStream_t (NULL = default stream).
 * Calls only enqueue work; synchronise the stream before reading results.
 * Alignment: base pointers, strides and symbol_size must be multiples of 8 bytes for the m<=8
 * kernels and 4 bytes for m = 16 (symbol_size must be even in any case).
 * Return codes are those of rs/reed_solomon.h (0, 1, RS_ERR_INVALID, RS_ERR_DEVICE, 100).
 */
#ifndef RS_AMD_RSG_H
#define RS_AMD_RSG_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rsg_codec rsg_codec_t;

/* Builds the (k, r) code on `device` (positions as reference cc_select_cosets) and uploads the
 * encode matrix. */
int rsg_codec_create(int device, uint16_t k, uint16_t r, rsg_codec_t** out);
void rsg_codec_destroy(rsg_codec_t* c);
/* Subfield degree m of the code (8 => GF(256) kernels, 16 => general kernels). */
int rsg_codec_subfield(const rsg_codec_t* c);

/* Options (every value gives identical results, they choose kernels and plans). The release library
 * accepts only values that select a parity-tested production path; the values marked [diag] are option-only
 * A/B families, overlap variants and layouts that exist only in the diagnostic build (make diag,
 * librs_amd_diag.so) -- the release library returns RS_ERR_INVALID for them:
 *   "jit"          matrix-specialised GF(256) kernels (hiprtc, cached on disk): 0 off, 1 every eligible
 *                  matrix, 2 the encode matrix and decode matrices from their dec_jit_uses-th launch
 *                  (default)
 *   "dec_jit_uses" launches of >= 1 MiB before a decode plan is specialised under jit = 2 (default 2)
 *   "xj"           specialised family: 1 bit-plane XOR kernels (default), 0 nibble-table kernels (rs_v1jit,
 *                  also the default for matrices the XOR kernel rejects)
 *   "m8_mode"      GF(256) kernel without specialisation: 20 one dword per lane, one nibble table per
 *                  input, two accumulator sets, gpr-index lookups (default); 18 the same with two tables
 *                  and one accumulator set; [diag] 2 two dwords per lane, 0 register tables with compiler
 *                  indexing, 1 masked multiples, 3, 4, 14 other register layouts of the gpr-index kernels
 *   "batch_plans"  rsg_decode_batch: 0 host plans per distinct pattern; 1 device-built plans (GF(256):
 *                  per stripe; GF(2^16): see m16_ps); 2 device plans past 16 distinct patterns for GF(256)
 *                  codes and past one pattern for GF(2^16) codes (default)
 *   "syn_route"    GF(256) device-plan decodes (S a multiple of 2 KiB): 2 the re-encode differences
 *                  [G | I] of every slot on the bit-plane XOR kernel (each stripe's erased slots read as
 *                  zero), then a per-stripe t_info x t_info solve from the first t_info surviving repair rows
 *                  that stores the erased information symbols (default); 1 syndromes of every slot on that
 *                  kernel, then a t_info x t solve; 0 survivor matrices. Erased slots may hold anything.
 *   "m8_syn_overlap" 0 one stream (default); [diag] 1 that route's plans + fixed pass of the next chunk on a
 *                  codec stream beside this chunk's solve (two buffer sets)
 *   "m8_ps_kernel" that route's per-stripe solve kernel: 10 the prefetching solve (one asm loop, packed
 *                  records, every load a step ahead, one nibble table; default), 0 LDS input ring, 3 the ring
 *                  kernel with one nibble table; [diag] 9 / 11 the prefetching solve with two tables / with its
 *                  multiples read from LDS, 1 one dword per lane without the ring, 2 two dwords per lane,
 *                  4 / 5 the one-table kernel converting 2 / 4 inputs per LDS round trip. Survivor plans and
 *                  symbol sizes with a partial 1 KiB chunk take 0.
 *   "m8_syn_masked" 1 the fixed pass reads each stripe's erased slots as zero and the solve stores (default);
 *                  0 the pass reads the slots as they are and the solve XORs its result into them
 *   "m8_syn_scratch_mib" fixed-pass scratch per chunk of stripes (MiB, default 1024; sets the launch count)
 *   "m8_syn_coord" 0 the solve converts its inputs (default); [diag] 1 with the masked pass and solve 10: the
 *                  pass stores its outputs in GF(256)^2 coordinates and the solve reads them as they are
 *   "m8_ps_cpb"    1 KiB column chunks per workgroup of solve kernel 0: 1 (default); [diag] 2-64 walk a
 *                  stripe's chunks in one workgroup (table setup once, next chunk's ring prologue under the
 *                  outputs)
 *   "m16_ps"       GF(2^16) rsg_decode_batch with per-stripe patterns (S a multiple of 1 KiB, r <= 4096):
 *                  1 one syndrome pass over all slots + a device-built t_info x t solve per stripe; 2 the
 *                  encode route over the information slots + the received repair rows, then a t_info x
 *                  t_info Cauchy solve per stripe; 3 (default) 2 when the batch's largest pattern needs at
 *                  least 13/16 r syndromes, else 1; 0 one plan per pattern rebuilt on the stream
 *   "m16_ps_chunk" / "m16_ps_rec_mib"  stripes / record MiB per chunk of that path (0 / 1024 defaults)
 *   "m16_ps_overlap" 1 (default) the next chunk's syndrome pass runs on a codec stream beside this chunk's
 *                  solve (two syndrome buffers); 0 both on the caller's stream
 *   "m16_cs_overlap" 0 serial (default); [diag] 1 the one-pattern syndrome route runs >= 16 stripes in 4
 *                  chunks, each chunk's syndromes on that codec stream beside the previous chunk's second stage
 *   "m16_mode"     GF(2^16) dense kernels: 0 hand-scheduled gpr-index kernel for > 32 outputs (default),
 *                  2 the compiled kernel
 *   "m16_plans"    GF(2^16) dense matrices: 0 built on the host, 1 on the device, 2 on the device from 64K
 *                  coefficients (default); rebuilds the encode plan
 *   "m16_route"    GF(2^16) syndrome route (cyclotomic k_cs16 + second stage): 1 matrices with >= 64
 *                  inputs (default), 0 never, 2 every matrix
 *   "m16_route_min_bytes"  bytes a dense decode plan with t > 64 moves before it switches to the route
 *                  (default 1 GiB; 0 = at once)
 *   "m16_reenc"    GF(2^16) decodes without repair erasures and t >= 0.9 r by re-encoding: 1 (default), 0
 *   "m16_cs_col"   route kernels' block layout: 256 bytes per column unit (default); [diag] 1024
 *   "m16_cs_thread" route syndromes: 1 k_cs16t, threaded code blocks at full VALU rate (default); 0 k_cs16,
 *                  gpr-indexed subset-table lookups
 * The timing ablations (wrong results: m8_mode 10-13, 15, 16, 19; m8_ps_kernel 6, 8; "m8_ps_ablate"; m16_mode
 * 1) and the s_memtime stamps (m8_mode 17, 21; m8_ps_kernel 7; "stamp_buffer") exist only in the diagnostic
 * build too.
 * Returns RS_ERR_INVALID for unknown names or values. */
int rsg_set_option(rsg_codec_t* c, const char* name, int64_t value);
/* Device scratch of a codec only grows with the launches it serves, and is reused by later calls: the
 * GF(2^16) per-stripe routes of rsg_decode_batch keep two record sets of up to m16_ps_rec_mib (1 GiB each by
 * default) and two syndrome buffers of up to 1 GiB (the re-encode variant: one 1 GiB fixed-pass buffer plus
 * the encode route's 1 GiB syndrome buffer); the GF(256) fixed pass one buffer of up to 1 GiB (two with
 * m8_syn_overlap); the route / re-encode decodes up to 1 GiB each; the host pipelines two 256 MiB batch
 * buffers.
 * rsg_codec_trim waits for the codec's outstanding work on that scratch and frees it: every buffer above,
 * the stripe-id lists, the route's slot-offset tables, the GF(2^16) many-pattern batch plan with its records
 * (up to 256 MiB) and pinned staging, and the host-pipeline buffers. What survives: the cached encode /
 * decode plans, the per-codec streams and events, and two small tables (slot elements, 2 (k + r) bytes;
 * the per-stripe route's input list, 4 (r + 16) bytes). Later calls grow the scratch again. */
int rsg_codec_trim(rsg_codec_t* c);
/* Name of the kernel the last encode/decode launched (diagnostics). */
const char* rsg_last_kernel(const rsg_codec_t* c);
/* Wave-instructions (VALU, SALU) the hand-scheduled GF(2^16) kernels issued in the last rsg_encode /
 * rsg_decode: their generated steps' instruction counts times the steps run (0 for the other kernels).
 * bench.py divides them by the launch time for the compute roofline of m = 16 codes. */
int rsg_last_work(const rsg_codec_t* c, uint64_t* valu, uint64_t* salu);

/* Repair symbols of n_stripes stripes: info at d_info (k symbols per stripe), repair written to
 * d_rep (r symbols per stripe). */
int rsg_encode(rsg_codec_t* c, const void* d_info, uint64_t info_stripe_stride, uint64_t info_symbol_stride,
               void* d_rep, uint64_t rep_stripe_stride, uint64_t rep_symbol_stride, uint64_t n_stripes,
               uint64_t symbol_size, void* stream);

/* Restores, in place, the erased information symbols of n_stripes stripes of k + r symbols that share
 * one erasure pattern (is_erased[k + r] in host memory, exactly t entries true). Erased slots are not
 * read; erased repair slots are not written (reference src/rs/reed_solomon.c:299-336). */
int rsg_decode(rsg_codec_t* c, void* d_rcv, uint64_t stripe_stride, uint64_t symbol_stride, uint64_t n_stripes,
               uint64_t symbol_size, const bool* is_erased, uint16_t t, void* stream);

/* Per-stripe erasure patterns: is_erased is [n_stripes][k + r] in host memory (stripe s lost the
 * symbols flagged in row s). With few distinct patterns (<= 16, or option batch_plans = 0) stripes are
 * grouped by pattern and each pattern is decoded by one launch over its stripes (host-built plans,
 * 16 most recent cached). With more (m <= 8 codes; batch_plans = 1 forces it) every stripe's decode
 * matrix is built on the device from its mask and one launch applies each stripe's own matrix.
 * Returns RS_ERR_CANNOT_RESTORE without writing anything if any stripe has more than r erasures;
 * stripes without erased information symbols are left untouched. Synchronises `stream` once
 * (upload of the stripe lists / masks). */
int rsg_decode_batch(rsg_codec_t* c, void* d_rcv, uint64_t stripe_stride, uint64_t symbol_stride, uint64_t n_stripes,
                     uint64_t symbol_size, const bool* is_erased, void* stream);

/* Host-memory batches (stripes arriving from a file or socket): the same operations on stripes in
 * HOST memory, pipelined over two streams (H2D -> kernel -> D2H per batch of up to 256 MiB, batches
 * overlapped). Synchronous: results are in host memory on return. Pinned memory (hipHostMalloc /
 * hipHostRegister) runs at PCIe rate; pageable memory works, slower. Any even symbol_size and byte
 * strides. rsg_decode_host copies only surviving symbols in and only the restored information symbols
 * out. */
int rsg_encode_host(rsg_codec_t* c, const void* h_info, uint64_t info_stripe_stride, uint64_t info_symbol_stride,
                    void* h_rep, uint64_t rep_stripe_stride, uint64_t rep_symbol_stride, uint64_t n_stripes,
                    uint64_t symbol_size);
int rsg_decode_host(rsg_codec_t* c, void* h_rcv, uint64_t stripe_stride, uint64_t symbol_stride, uint64_t n_stripes,
                    uint64_t symbol_size, const bool* is_erased, uint16_t t);

/* Synthetic inputs: fills the k information symbols of stripes [stripe0, stripe0 + n) with the
 * counter-based generator of tests/_util.py:gen_info (symbol_size % 8 == 0). */
int rsg_fill_info(void* d_base, uint64_t stripe_stride, uint64_t symbol_stride, uint64_t symbol_size, uint16_t k,
                  uint64_t stripe0, uint64_t n_stripes, uint64_t seed, void* stream);
/* Per-stripe 64-bit fingerprint of symbols [sym0, sym0 + nsym) into d_out[n_stripes] (device). */
int rsg_fingerprint(const void* d_base, uint64_t stripe_stride, uint64_t symbol_stride, uint64_t symbol_size,
                    uint32_t sym0, uint32_t nsym, uint64_t n_stripes, uint64_t* d_out, void* stream);

/* ---- host-only helpers (no GPU needed; used by tests and integration code) ---- */
/* Coding matrix in GF(2^16): encode when is_erased == NULL (rows = r repair, cols = k info), else the
 * decode matrix (rows = erased information slots, cols = surviving slots). Any output pointer may be
 * NULL to query sizes first. */
int rsg_coding_matrix(uint16_t k, uint16_t r, const bool* is_erased, uint16_t t, uint16_t* matrix, uint32_t* rows,
                      uint32_t* cols, int32_t* in_slots, int32_t* out_slots);
/* Compiles the matrix-specialised kernel for the encode (is_erased == NULL) or decode matrix into the
 * on-disk JIT cache without touching a GPU (0 also when the matrix is not JIT-eligible). */
int rsg_jit_precompile(uint16_t k, uint16_t r, const bool* is_erased, uint16_t t);
/* Generated source of the bit-plane XOR kernel (rs_xj) for the encode (is_erased == NULL) or decode
 * matrix; *len = full length, buf gets at most cap - 1 bytes + NUL. RS_ERR_INVALID when not eligible. */
int rsg_xj_source(uint16_t k, uint16_t r, const bool* is_erased, uint16_t t, char* buf, size_t cap, size_t* len);
/* Bit-plane basis of the XOR kernels: pivots[8], beta_y[8] (alpha^-j coordinates of beta_t) and the
 * 8 bit-plane bits of each GF(256) element indexed by its gamma-basis byte (bits256[256]). */
int rsg_xj_basis(int32_t* pivots, uint16_t* beta_y, uint8_t* bits256);
/* GF(256)^2 coordinate tables used by the m <= 8 kernels (lbyte/ibyte: 2 x 256 entries each). */
int rsg_gamma_tables(uint16_t* lbyte, uint16_t* ibyte, uint8_t* red);
/* GF(2^16) syndrome route of the encode (is_erased == NULL) or decode matrix:
 * the k_cs16 plan -- groups [ngroups][16] input slots (-1 = none), records [ntiles][ngroups + 2][64]
 * bytes, finish lists [ntiles][fin_stride] and [ntiles][5] -- and the second-stage matrix m2 [R][D]
 * (out = m2 * syndromes). info = {D, ngroups, ntiles, fin_stride, R}; arrays may be NULL. Host only. */
int rsg_route_dump(uint16_t k, uint16_t r, const bool* is_erased, uint16_t t, int32_t* info, int32_t* groups,
                   uint8_t* rec, int32_t* fin, int32_t* fin_off, uint16_t* m2);
/* The same plan as k_cs16t runs it: info = {cw (cosets per tile), ntiles, fin_stride, nblocks}; records
 * [ntiles][ngroups + 2][4 cw] code-block offsets, finish lists [ntiles][fin_stride] and [ntiles][cw + 1],
 * and the block table [nblocks] (offset of block (c, n, v) at (4c + n) * 16 + v). Host only. */
int rsg_route_dump_t(uint16_t k, uint16_t r, const bool* is_erased, uint16_t t, int32_t* info, uint32_t* rec,
                     int32_t* fin, int32_t* fin_off, uint32_t* blocks);
/* Symbol data from symbol_create of >= 16 KiB (page-aligned whole pages of its own): 1 when it is page-locked
 * and mapped (hipHostRegister, done by the first rs_* call that moves it; symbol_create itself makes no HIP
 * call), 0 when it is not (not used yet, or the registration was refused: such symbols go by the staging
 * path); -1 for any other pointer. */
int rsg_symbol_registered(const void* data);
/* Counters of the library-allocated symbol pages since process start (rs_hostmem.cpp). A block whose
 * registration cannot be undone (hipHostUnregister fails, or the runtime still reports the range) is
 * "stuck": it stays mapped, out of circulation and counted against the pinned cap. */
typedef struct rsg_symbol_stats {
    uint64_t live;                /* symbols in registrable pages, not destroyed */
    uint64_t live_registered;     /* of those, page-locked and mapped */
    uint64_t idle_blocks;         /* destroyed blocks parked in the idle pool (registration kept) */
    uint64_t idle_bytes;
    uint64_t idle_reuses;         /* symbol_create calls served from the idle pool */
    uint64_t registrations;       /* successful hipHostRegister calls */
    uint64_t register_failures;   /* refused by the runtime, range already known, or no device pointer */
    uint64_t unregistrations;     /* hipHostUnregister succeeded and the runtime forgot the range */
    uint64_t unregister_failures;
    uint64_t retired_blocks;      /* memory returned to the OS, address range kept reserved (never reused) */
    uint64_t stuck_blocks;
    uint64_t stuck_bytes;
    uint64_t pinned_bytes;        /* page-locked bytes of arenas, slabs and registered symbols */
} rsg_symbol_stats_t;
int rsg_symbol_stats(rsg_symbol_stats_t* out);
/* Idle-pool cap in bytes (default 1 GiB, RS_AMD_SYM_POOL_MB); bytes < 0 only queries. Returns the previous
 * cap. Blocks destroyed past the cap are unregistered and retired. */
int64_t rsg_symbol_pool_cap(int64_t bytes);
/* The k_bs16 second stage of the GF(2^16) route for the encode (is_erased NULL) or decode matrix, when it
 * applies (encode: the repair cosets; decode: an erased set closed under x -> x^(2^d), d < 16): records
 * [ntiles][ngroups + 2][4][64] bytes, finish lists [ntiles][fin_stride] (local coset | rotation << 4 |
 * output slot << 8) and [ntiles][5]. info = {applies, D, ngroups, ntiles, fin_stride, d}; arrays may be
 * NULL and are written only when it applies. Host only. */
int rsg_bs16_dump(uint16_t k, uint16_t r, const bool* is_erased, uint16_t t, int32_t* info, uint8_t* rec,
                  int32_t* fin, int32_t* fin_off);
/* Source of the masked (masked = 1), masked with outputs in GF(256)^2 coordinates (2, the form the default
 * prefetching solve reads) or plain (0) XOR kernel of the GF(256) per-stripe route's fixed pass over all
 * k + r slots: route 1 the r syndromes, 2 the re-encode differences [G | I]. The masked forms read every
 * slot whose bit is set in its stripe's mask words as zero. RS_ERR_INVALID when the route does not apply
 * (m = 16 codes, K * R past the XOR kernel's bound). Host only (emulator tests). */
int rsg_xj_fixed_source(uint16_t k, uint16_t r, int route, int masked, char* buf, size_t cap, size_t* len);
/* Compiles the masked fixed-pass kernel of that route into the JIT cache, like rsg_jit_precompile (0 when the
 * route does not apply). Host only. */
int rsg_xj_fixed_precompile(uint16_t k, uint16_t r, int route);
/* Batched symbol operations: the reference's gf_add / gf_mul / gf_madd (rs/gf65536.h:146-167,
 * src/rs/gf65536.c:155-219) over many symbols in ONE call, asynchronous on `stream` -- the form a loop of
 * gf_* calls takes on the GPU (each gf_* call of rs/gf65536.h is one synchronous round trip, ~15 us).
 *   RSG_OP_ADD   a ^= b            RSG_OP_MUL   a = coef * a            RSG_OP_MADD  a ^= coef * b
 * All symbols are `symbol_size` bytes (little-endian GF(2^16) words; an odd last byte is not touched, as
 * the reference's Release build) at device-accessible addresses (hipMalloc memory, or the device address
 * of page-locked host memory), 4-byte aligned. Ops on the same target `a` are applied in array order
 * (b == a reads the target's current value); ops on different targets run in parallel, so no op may read
 * (as b) another op's target, and targets may not overlap: RS_ERR_INVALID, nothing queued. The op array is
 * copied before the call returns (the caller may reuse it); synchronise `stream` before reading results.
 * `device` is the HIP device the symbols live on (the caller's current device is restored). */
enum { RSG_OP_ADD = 0, RSG_OP_MUL = 1, RSG_OP_MADD = 2 };
typedef struct rsg_symbol_op {
    void* a;        /* target symbol, read and written */
    const void* b;  /* source symbol (RSG_OP_ADD / RSG_OP_MADD; ignored for RSG_OP_MUL) */
    uint16_t coef;  /* GF(2^16) coefficient (RSG_OP_MUL / RSG_OP_MADD) */
    uint16_t op;    /* RSG_OP_* */
    uint32_t reserved;
} rsg_symbol_op_t;
int rsg_symbol_ops(int device, const rsg_symbol_op_t* ops, uint64_t n_ops, uint64_t symbol_size, void* stream);
const char* rsg_version(void);
/* 1 when checked launches are on (environment RS_AMD_CHECK set and not "0" at the first call of the
 * process), else 0. In checked mode every launch group is followed by a device wait and an error read: a
 * device fault is reported on stderr at the call that queued it (its kernel, the code's k / r, the plan's
 * K / R and slot ranges, stripes and symbol size) and the call returns RS_ERR_DEVICE; plans' slot lists
 * are bounds-checked on the host before their first launch (RS_ERR_INVALID). Diagnosis only: each
 * launch then costs a device round trip. Host only. */
int rsg_check_enabled(void);

#ifdef __cplusplus
}
#endif
#endif
