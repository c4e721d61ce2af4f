// rs_v1args.h -- kernel-argument block of the V = 1 m <= 8 kernels, shared by host code, the AOT
// kernels and the hiprtc sources (rs_jit.cpp embeds this text ahead of rs_device.h). Plain data only.
#pragma once
#ifndef RS_JIT_SOURCE
#include <stdint.h>
#endif

// Kernel arguments of the V = 1 kernels (AOT k_apply_m8_v1 and the hiprtc-specialised rs_v1jit).
struct V1Args {
    const uint8_t* src;      // stripe 0 of the input layout
    int64_t src_stripe, src_sym;
    const int32_t* in_idx;   // [K (+16 pad)] input symbol slots
    uint8_t* dst;
    int64_t dst_stripe, dst_sym;
    const int32_t* out_idx;  // [ntiles * 32] output symbol slots
    const uint32_t* ltab;    // [3072] GF(256)^2 coordinate byte tables (L, L^-1, L^-1 of gamma^4 x)
    const uint32_t* idx;     // AOT: [ntiles][K][64] nibble indices (lo p, hi 32 + p)
    const int32_t* boff;     // JIT: [ntiles][K] byte offset of each input's lookup block
    int32_t K, R;
    int64_t nchunks;         // 1 KiB column chunks per symbol processed by this launch
    const int32_t* ids;      // optional [n_stripes] stripe indices; null = 0..n-1
    // per-stripe plans (rsg_decode_batch with device-built decode matrices), indexed by the
    // launch-local stripe s: K, R = ps_kr[2s], ps_kr[2s + 1]; in_idx, out_idx and idx advance by
    // s * ps_in / ps_out / ps_idx elements. Null = one plan for every stripe (K, R above).
    const int32_t* ps_kr;
    int64_t ps_in, ps_out, ps_idx;
    // split-K (k_apply_m16_v1 on small grids): blockIdx.z = input slice of kslices; each slice XORs
    // its partial products into partial[slice][stripe][tile * 64 + row][chunk dwords], which
    // k_xor_slices reduces into the outputs. kslices <= 1: direct stores.
    int32_t kslices;
    uint32_t* partial;
    // k_apply_m16_v1 block order (XCD-aware): units = n_stripes * nchunks (stripe, chunk) pairs, unit u
    // on XCD u % 8 with its `tiles` row tiles dispatched back to back there, so they share that XCD's
    // L2 copy of the unit's inputs. units == 0: grid (units, tiles) in the plain order.
    int64_t units;
    int32_t tiles;
    // k_apply_m16_v1 per-stripe mode (ps_kr set): nonzero = inputs come from the launch-local stripe
    // (src + local * src_stripe: a per-stripe scratch, e.g. syndromes), outputs from ids (RS_STRIPE)
    int32_t src_local;
    // nonzero: each output is XORed into its destination instead of stored (the GF(256) per-stripe
    // syndrome route: the erased slots still hold their old contents g, the syndromes saw them, and the
    // solve yields g + c, so g ^ (W S) = c without a pass that zeroes the slots first)
    int32_t xor_dst;
    // diagnostic builds only (k_apply_m8_v1<5>): per wave, 8 s_memtime phase counters (m8_v1_run STAMP)
    uint64_t* stamps;
    // m8_v1_run: column chunks per block (<= 1: one; the grid's x then covers n_stripes * ceil(nchunks / cpb)
    // blocks). Not combined with split-K.
    int32_t cpb;
    // diagnostic builds (RS_AMD_DIAG) under checked launches (RS_AMD_CHECK): slot indices read from in_idx /
    // out_idx must lie in [0, nslots) (the codec's k + r); a violation is recorded in slot_err ({1 in / 2 out,
    // list position, value, block}) and the access goes to slot 0 (loads) or is skipped (stores) instead of
    // faulting; the host reports it after the launch. nslots 0 = unchecked.
    int32_t nslots;
    int32_t* slot_err;
    // diagnostic builds only (option m8_ps_ablate; timing ablations with wrong results): bit 1 skips the
    // coordinate-table copy into LDS, bit 2 stores the accumulators without the L^-1 conversion
    int32_t ablate;
    // k_apply_m8_pf: bytes of the input buffer from src (the buffer resource's range; 0 = unchecked)
    int64_t src_bytes;
};

// Stripe processed by launch-local stripe `s`: ids[s] when a stripe-id list is given.
#define RS_STRIPE(ids, s) ((ids) ? int64_t((ids)[(s)]) : int64_t(s))

