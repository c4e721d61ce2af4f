// rs_api.cpp -- the batched device API (rs_amd/rsg.h): codec lifetime and options, the launch
// dispatcher run_plan (bit-plane XOR kernels, JIT kernels, generic gpr-index kernels, the GF(2^16)
// route), rsg_encode / rsg_decode, the host-memory pipelines and the host-only inspection calls.
//
// Every encode/decode runs on the GPU through rs_kernels.hip; there is no CPU compute path for
// symbol data in this library. The reference API shims live in rs_dropin.cpp / rs_hostmem.cpp /
// rs_refops.cpp, per-stripe batches in rs_batch.cpp, the GF(2^16) route in rs_route16.cpp.
#include "rs_core.hpp"

using namespace rsamd;

#ifdef RS_AMD_DIAG
#define RSG_VERSION "rs_amd 0.2 (gfx950, DIAGNOSTIC build: timing ablations enabled)"
#else
#define RSG_VERSION "rs_amd 0.2 (gfx950)"
#endif

extern "C" int rsg_codec_create(int device, uint16_t k, uint16_t r, rsg_codec_t** out) {
    rsamd::CallerDevice caller_device;
    if (!out) return RS_ERR_INVALID;
    *out = nullptr;
    if (uint32_t(k) + r > kN) return RS_ERR_INVALID;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device || device < 0) {
        std::fprintf(stderr, "librs_amd: no HIP device %d (found %d)\n", device, ndev);
        return RS_ERR_DEVICE;
    }
    HIP_TRY(hipSetDevice(device));
    auto c = std::make_unique<rsg_codec>();
    c->device = device;
    c->k = k;
    c->r = r;
    try {
        c->positions = code_positions(k, r);
    } catch (...) {
        return RS_ERR_INVALID;
    }
    c->m = subfield_degree(c->positions);
    int rc = device_tables(device, &c->d_ltab);
    if (rc) return rc;
    if ((rc = make_plan(c.get(), nullptr, c->enc, nullptr))) return rc;
    HIP_TRY(hipStreamSynchronize(nullptr));  // the encode plan is complete before any stream uses it
    *out = c.release();
    return 0;
}

extern "C" void rsg_codec_destroy(rsg_codec_t* c) {
    rsamd::CallerDevice caller_device;
    delete c;
}

extern "C" int rsg_codec_subfield(const rsg_codec_t* c) { return c ? (c->m <= 8 ? 8 : 16) : 0; }

extern "C" int rsg_set_option(rsg_codec_t* c, const char* name, int64_t value) {
    rsamd::CallerDevice caller_device;
    if (!c || !name) return RS_ERR_INVALID;
    // The release build accepts only knobs that select a parity-tested production path:
    // option-only A/B families, overlap variants and block layouts are diagnostic-build knobs (make diag).
    if (!std::strcmp(name, "m8_mode")) {
        if (value < 0 || (value > 4 && value < 10) || value > 21) return RS_ERR_INVALID;
#ifndef RS_AMD_DIAG  // 18 / 20: the V = 1 kernels; the rest are A/B families, ablations (wrong results), stamps
        if (value != 18 && value != 20) return RS_ERR_INVALID;
#endif
        c->m8_mode = int(value);
        return 0;
    }
#ifdef RS_AMD_DIAG
    if (!std::strcmp(name, "stamp_buffer")) {  // device pointer, [blocks * 4][4] uint64 (mode 17)
        c->stamps = reinterpret_cast<uint64_t*>(static_cast<uintptr_t>(value));
        return 0;
    }
#endif
    if (!std::strcmp(name, "xj")) {
        if (value < 0 || value > 1) return RS_ERR_INVALID;
        c->xj = int(value);
        return 0;
    }
    if (!std::strcmp(name, "dec_jit_uses")) {
        if (value < 1 || value > (int64_t(1) << 30)) return RS_ERR_INVALID;
        c->dec_jit_uses = int(value);
        return 0;
    }
    if (!std::strcmp(name, "jit")) {
        if (value < 0 || value > 2) return RS_ERR_INVALID;
        c->jit = int(value);
        return 0;
    }
    if (!std::strcmp(name, "m16_mode")) {
        if (value < 0 || value > 2) return RS_ERR_INVALID;
#ifndef RS_AMD_DIAG  // 1: timing ablation with wrong results, diagnostic build only
        if (value == 1) return RS_ERR_INVALID;
#endif
        c->m16_mode = int(value);
        return 0;
    }
    if (!std::strcmp(name, "m16_plans")) {
        if (value < 0 || value > 2) return RS_ERR_INVALID;
        c->m16_plans = int(value);
        c->dec.clear();  // plans are rebuilt under the new setting: decode plans on use, encode now
        c->dec_lru.clear();
        if (c->m > 8) {
            HIP_TRY(hipSetDevice(c->device));
            HIP_TRY(hipDeviceSynchronize());  // the old encode plan may still be in use
            std::unique_ptr<DevPlan> e;
            if (int rc = make_plan(c, nullptr, e, nullptr)) return rc;
            HIP_TRY(hipStreamSynchronize(nullptr));
            c->enc = std::move(e);
        }
        return 0;
    }
    if (!std::strcmp(name, "m16_route")) {  // new plans follow the setting; cached ones are dropped
        if (value < 0 || value > 2) return RS_ERR_INVALID;
        if (c->m16_route != int(value)) {
            c->m16_route = int(value);
            c->dec.clear();
            c->dec_lru.clear();
            if (c->m > 8) {
                HIP_TRY(hipSetDevice(c->device));
                HIP_TRY(hipDeviceSynchronize());  // the old encode plan may still be in use
                std::unique_ptr<DevPlan> e;
                if (int rc = make_plan(c, nullptr, e, nullptr)) return rc;
                HIP_TRY(hipStreamSynchronize(nullptr));
                c->enc = std::move(e);
            }
        }
        return 0;
    }
    if (!std::strcmp(name, "m16_cs_thread")) {  // k_cs16t (1) or k_cs16 (0) syndromes (results identical)
        if (value < 0 || value > 1) return RS_ERR_INVALID;
        c->m16_cs_thread = int(value);
        return 0;
    }
    if (!std::strcmp(name, "m16_cs_col")) {  // k_cs16 / k_bs16 block layout (results identical)
        if (value != 256 && value != 1024) return RS_ERR_INVALID;
#ifndef RS_AMD_DIAG
        if (value != 256) return RS_ERR_INVALID;  // 1024: A/B layout, diagnostic build
#endif
        c->m16_cs_col = int(value);
        return 0;
    }
    if (!std::strcmp(name, "m16_reenc")) {  // decode patterns built from now on
        if (value < 0 || value > 1) return RS_ERR_INVALID;
        c->m16_reenc = int(value);
        c->dec.clear();
        c->dec_lru.clear();
        return 0;
    }
    if (!std::strcmp(name, "m16_ps")) {  // rsg_decode_batch of GF(2^16) codes: per-stripe route plans
        if (value < 0 || value > 3) return RS_ERR_INVALID;
        c->m16_ps = int(value);
        return 0;
    }
    if (!std::strcmp(name, "m16_ps_overlap")) {  // its syndrome pass of the next chunk beside this chunk's solve
        if (value < 0 || value > 1) return RS_ERR_INVALID;
        c->ps_overlap = int(value);
        return 0;
    }
    if (!std::strcmp(name, "m16_cs_overlap")) {  // one-pattern syndrome route: syndromes beside the second stage
        if (value < 0 || value > 1) return RS_ERR_INVALID;
#ifndef RS_AMD_DIAG
        if (value) return RS_ERR_INVALID;  // measured slower: diagnostic build
#endif
        c->cs_overlap = int(value);
        return 0;
    }
    if (!std::strcmp(name, "m16_ps_chunk")) {  // its stripes per chunk (0 = sized by m16_ps_rec_mib)
        if (value < 0 || value > 65535) return RS_ERR_INVALID;
        c->ps_chunk = value;
        return 0;
    }
    if (!std::strcmp(name, "m8_syn_scratch_mib")) {  // GF(256) per-stripe route: fixed-pass scratch per chunk
        if (value < 1 || value > 4095) return RS_ERR_INVALID;
        c->syn_scratch_mib = value;
        return 0;
    }
    if (!std::strcmp(name, "m16_ps_rec_mib")) {  // its record bytes per chunk
        if (value < 1 || value > 4096) return RS_ERR_INVALID;
        c->ps_rec_mib = value;
        return 0;
    }
    if (!std::strcmp(name, "m16_route_min_bytes")) {
        if (value < 0) return RS_ERR_INVALID;
        c->route_min_bytes = value;
        c->dec.clear();
        c->dec_lru.clear();
        return 0;
    }
    // the per-stripe fixed pass's form follows these options: a change rebuilds it at the next call
    auto syn_reform = [c]() {
        if (c->syn && c->syn->xj && hipSetDevice(c->device) == hipSuccess)
            (void)hipDeviceSynchronize();  // the old pass may still be queued (on the codec's device)
        c->syn.reset();
        c->syn_failed = false;
    };
    if (!std::strcmp(name, "m8_ps_kernel")) {  // per-stripe GF(256) solve kernel (results identical)
        if (value < 0 || value > 13) return RS_ERR_INVALID;
#ifndef RS_AMD_DIAG  // 10: the prefetching kernel (default); 0 / 3: the ring kernels; 9, 11: other prefetching
                     // forms and 1, 2, 4, 5: A/B kernels (diagnostic build); 6, 8, 12, 13: ablations (wrong
                     // results); 7: stamps
        if (value != 0 && value != 3 && value != 10) return RS_ERR_INVALID;
#endif
        if ((int(value) == 10) != (c->m8_ps_kernel == 10)) syn_reform();  // the coordinate form goes with 10
        c->m8_ps_kernel = int(value);
        return 0;
    }
    if (!std::strcmp(name, "m8_syn_masked")) {  // per-stripe fixed pass masked (1) or plain + XOR solve (0)
        if (value < 0 || value > 1) return RS_ERR_INVALID;
        if (int(value) != c->m8_syn_masked) syn_reform();
        c->m8_syn_masked = int(value);
        return 0;
    }
    if (!std::strcmp(name, "m8_syn_coord")) {  // fixed pass stores coordinates for solve 10 (1) or not (0)
        if (value < 0 || value > 1) return RS_ERR_INVALID;
#ifndef RS_AMD_DIAG
        if (value) return RS_ERR_INVALID;  // measured slower: diagnostic build
#endif
        if (int(value) != c->m8_syn_coord) syn_reform();
        c->m8_syn_coord = int(value);
        return 0;
    }
    if (!std::strcmp(name, "m8_ps_cpb")) {  // per-stripe GF(256) solve: column chunks per workgroup
        if (value < 1 || value > 64) return RS_ERR_INVALID;
#ifndef RS_AMD_DIAG
        if (value != 1) return RS_ERR_INVALID;  // k_apply_m8_v1<6>: measured slower past 2, diagnostic build
#endif
        c->m8_ps_cpb = int(value);
        return 0;
    }
#ifdef RS_AMD_DIAG
    if (!std::strcmp(name, "inject_fail_group")) {  // failure injection: rsg_decode_batch's grouping path
        if (value < -1 || value > 65535) return RS_ERR_INVALID;
        c->inject_fail_group = value;
        return 0;
    }
    if (!std::strcmp(name, "m8_ps_ablate")) {  // timing ablations of the per-stripe solve (wrong results)
        if (value < 0 || value > 3) return RS_ERR_INVALID;
        c->m8_ps_ablate = int(value);
        return 0;
    }
#endif
    if (!std::strcmp(name, "m8_syn_overlap")) {  // GF(256) per-stripe syndrome route: overlapped chunks
        if (value < 0 || value > 1) return RS_ERR_INVALID;
#ifndef RS_AMD_DIAG
        if (value) return RS_ERR_INVALID;  // measured no faster (profiles/r4/ps8_route2.md): diagnostic build
#endif
        c->m8_syn_overlap = int(value);
        return 0;
    }
    if (!std::strcmp(name, "syn_route")) {  // 0 survivor plans, 1 syndromes, 2 re-encode differences
        if (value < 0 || value > 2) return RS_ERR_INVALID;
        if (c->syn && int(value) != c->syn_route) {  // the fixed pass's plan changes with it
            HIP_TRY(hipSetDevice(c->device));
            HIP_TRY(hipDeviceSynchronize());
            c->syn.reset();
            c->syn_failed = false;
        }
        c->syn_route = int(value);
        return 0;
    }
    if (!std::strcmp(name, "batch_plans")) {
        if (value < 0 || value > 2) return RS_ERR_INVALID;
        c->batch_plans = int(value);
        return 0;
    }
    return RS_ERR_INVALID;
}

extern "C" int rsg_codec_trim(rsg_codec_t* c) {
    rsamd::CallerDevice caller_device;
    if (!c) return RS_ERR_INVALID;
    HIP_TRY(hipSetDevice(c->device));
    // the launches that may still read the scratch: the last batch / route call's (scratch_ev), the side
    // and syndrome streams, the host pipelines' streams, the staged list copies
    if (c->scratch_pending) HIP_TRY(hipEventSynchronize(c->scratch_ev));
    c->scratch_pending = false;
    if (c->stage_pending) HIP_TRY(hipEventSynchronize(c->stage_ev));
    c->stage_pending = false;
    for (hipStream_t s : {c->ps_side, c->ps_synst, c->hs[0], c->hs[1]})
        if (s) HIP_TRY(hipStreamSynchronize(s));
    auto drop = [](void*& p, size_t& cap) {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    };
    drop(c->d_cs, c->cs_cap);
    drop(c->d_reenc, c->reenc_cap);
    drop(c->d_syn, c->syn_cap);
    drop(c->d_ps_rec, c->ps_rec_cap);
    drop(c->d_ps_small, c->ps_small_cap);
    drop(c->d_partial, c->partial_cap);
    drop(c->d_masks, c->masks_cap);
    drop(c->d_kr, c->kr_cap);
    drop(c->d_pin, c->pin_cap);
    drop(c->d_pout, c->pout_cap);
    drop(c->d_pidx, c->pidx_cap);
    drop(c->d_mbits, c->mbits_cap);
    {
        size_t zc = size_t(c->zero_cap);
        drop(c->d_zero, zc);
        c->zero_cap = 0;
    }
    size_t ids_bytes = c->ids_cap * 4;  // ids_cap counts entries
    drop(reinterpret_cast<void*&>(c->d_ids), ids_bytes);
    c->ids_cap = 0;
    for (int i = 0; i < 2; ++i) drop(c->d_goff[i], c->goff_cap[i]);
    // the GF(2^16) many-pattern batch plan: its staging slots' last uploads first, then the plan (its
    // destructor guards its own blob), the records it pointed into, and the pinned staging
    for (int i = 0; i < 2; ++i) {
        if (c->bp16_rec_pending[i]) HIP_TRY(hipEventSynchronize(c->bp16_ev[i]));
        c->bp16_rec_pending[i] = false;
    }
    if (c->bp16) {
        c->bp16->d_idx = nullptr;  // a view into d_bp16_rec
        c->bp16.reset();
    }
    size_t none = 0;
    drop(c->d_bp16, none);
    drop(c->d_bp16_rec, none);
    for (int i = 0; i < 2; ++i) {
        if (c->h_bp16[i]) (void)hipHostFree(c->h_bp16[i]);
        c->h_bp16[i] = nullptr;
    }
    for (int i = 0; i < 2; ++i) {
        if (c->hbuf[i]) (void)hipFree(c->hbuf[i]);
        c->hbuf[i] = nullptr;
    }
    c->hbuf_cap = 0;
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    c->h_stage = nullptr;
    c->stage_cap = 0;
    HIP_TRY(hipGetLastError());
    return 0;
}

extern "C" const char* rsg_last_kernel(const rsg_codec_t* c) { return c ? c->last_kernel.c_str() : "none"; }

namespace rsamd {

int run_plan_body(rsg_codec_t* c, DevPlan& p, const uint8_t* src, int64_t src_stripe, int64_t src_sym,
                  uint8_t* dst, int64_t dst_stripe, int64_t dst_sym, uint64_t n_stripes, uint64_t S,
                  hipStream_t st, const int32_t* d_ids, bool dst_local);

bool check_mode() {
    static const bool on = [] {
        const char* e = std::getenv("RS_AMD_CHECK");
        return e && *e && std::strcmp(e, "0") != 0;
    }();
    return on;
}

static void slot_range(const std::vector<int32_t>& v, size_t n, int64_t& lo, int64_t& hi) {
    lo = INT64_MAX;
    hi = INT64_MIN;
    for (size_t i = 0; i < std::min(n, v.size()); ++i) lo = std::min<int64_t>(lo, v[i]), hi = std::max<int64_t>(hi, v[i]);
}

int check_plan_slots(const rsg_codec_t* c, const DevPlan& p) {
    const int64_t n = p.slot_bound ? int64_t(p.slot_bound) : int64_t(c->k) + c->r;
    int64_t ilo, ihi, olo, ohi;
    slot_range(p.in_slots, size_t(p.K), ilo, ihi);
    slot_range(p.out_slots, size_t(p.R), olo, ohi);
    if ((p.K && (ilo < 0 || ihi >= n)) || (p.R && (olo < 0 || ohi >= n))) {
        std::fprintf(stderr,
                     "librs_amd: RS_AMD_CHECK: plan K=%d R=%d has slots outside [0, %lld): in [%lld, %lld], out [%lld, %lld]\n",
                     p.K, p.R, static_cast<long long>(n), static_cast<long long>(ilo), static_cast<long long>(ihi),
                     static_cast<long long>(olo), static_cast<long long>(ohi));
        return RS_ERR_INVALID;
    }
    return 0;
}

int check_launch(const rsg_codec_t* c, const DevPlan* p, const char* where, uint64_t n_stripes, uint64_t S) {
    const hipError_t sync = hipDeviceSynchronize();
    const hipError_t last = hipGetLastError();
    const hipError_t e = sync != hipSuccess ? sync : last;
    if (e == hipSuccess && c && c->d_slot_err) {  // diagnostic builds: a device-side slot check fired
        int32_t rec[4] = {0, 0, 0, 0};
        if (hipMemcpy(rec, c->d_slot_err, sizeof rec, hipMemcpyDeviceToHost) == hipSuccess && rec[0]) {
            std::fprintf(stderr,
                         "librs_amd: RS_AMD_CHECK: %s slot list entry %d = %d outside [0, %d) in block %d after %s: "
                         "kernel %s, plan K=%d R=%d\n",
                         rec[0] == 1 ? "input" : "output", rec[1], rec[2], p && p->slot_bound ? p->slot_bound : c->k + c->r,
                         rec[3], where, c->last_kernel.c_str(), p ? p->K : 0, p ? p->R : 0);
            (void)hipMemset(c->d_slot_err, 0, sizeof rec);
            return RS_ERR_DEVICE;
        }
    }
    if (e == hipSuccess) return 0;
    int64_t ilo = 0, ihi = -1, olo = 0, ohi = -1;
    if (p) {
        slot_range(p->in_slots, size_t(p->K), ilo, ihi);
        slot_range(p->out_slots, size_t(p->R), olo, ohi);
    }
    std::fprintf(stderr,
                 "librs_amd: RS_AMD_CHECK: device error '%s' after %s: kernel %s, code k=%d r=%d, plan K=%d R=%d, "
                 "in slots [%lld, %lld], out slots [%lld, %lld], %llu stripes x %llu bytes\n",
                 hipGetErrorString(e), where, c ? c->last_kernel.c_str() : "-", c ? c->k : 0, c ? c->r : 0,
                 p ? p->K : 0, p ? p->R : 0, static_cast<long long>(ilo), static_cast<long long>(ihi),
                 static_cast<long long>(olo), static_cast<long long>(ohi), static_cast<unsigned long long>(n_stripes),
                 static_cast<unsigned long long>(S));
    return RS_ERR_DEVICE;
}

int run_plan(rsg_codec_t* c, DevPlan& p, const uint8_t* src, int64_t src_stripe, int64_t src_sym, uint8_t* dst,
             int64_t dst_stripe, int64_t dst_sym, uint64_t n_stripes, uint64_t S, hipStream_t st,
             const int32_t* d_ids, bool dst_local) {
    if (p.R == 0 || n_stripes == 0 || S == 0) return 0;
    if (check_mode() && !p.slots_checked) {
        if (int rc = check_plan_slots(c, p)) return rc;
        p.slots_checked = true;
    }
    const int rc = run_plan_body(c, p, src, src_stripe, src_sym, dst, dst_stripe, dst_sym, n_stripes, S, st, d_ids,
                                 dst_local);
    const int rc2 = p.note_use(st);  // after the launches (also a failed call's partial ones)
    if (!rc && !rc2) RS_CHECKPOINT(c, &p, "run_plan", n_stripes, S);
    return rc ? rc : rc2;
}

int run_plan_body(rsg_codec_t* c, DevPlan& p, const uint8_t* src, int64_t src_stripe, int64_t src_sym,
                  uint8_t* dst, int64_t dst_stripe, int64_t dst_sym, uint64_t n_stripes, uint64_t S,
                  hipStream_t st, const int32_t* d_ids, bool dst_local) {
    if (int rc = p.order_after_build(st)) return rc;
    if (p.reenc) {  // in place: src == dst is the stripe (rsg_decode); the parent checked the launch fits
        if (src != dst || src_stripe != dst_stripe || src_sym != dst_sym || d_ids || dst_local) return RS_ERR_INVALID;
        return run_reenc(c, p, dst, dst_stripe, dst_sym, n_stripes, S, st);
    }
    if (p.route_ok && !d_ids && !dst_local && S % 1024 == 0 && int64_t(S) < (int64_t(1) << 31)) {
        int64_t max_in = 0;  // the route's 31-bit offsets (run_plan_body's p.cs branch)
        for (int32_t v : p.in_slots) max_in = std::max<int64_t>(max_in, v);
        const int64_t D = int64_t(std::count(p.erased.begin(), p.erased.end(), uint8_t(1)));
        const bool fits = max_in * src_sym + int64_t(S) < (int64_t(1) << 31) && D * int64_t(S) < (int64_t(1) << 31);
        if (fits && !p.route) {
            p.route_bytes += n_stripes * uint64_t(p.K + p.R) * S;
            if (p.route_bytes >= uint64_t(c->route_min_bytes)) {
                std::unique_ptr<bool[]> er(new bool[p.erased.size()]);
                for (size_t i = 0; i < p.erased.size(); ++i) er[i] = p.erased[i] != 0;
                // the re-encode decode runs in place (its launch layout) with 31-bit offsets over all slots
                const bool in_place = src == dst && src_stripe == dst_stripe && src_sym == dst_sym &&
                                      (c->k + c->r) * src_sym < (int64_t(1) << 31) &&
                                      int64_t(c->r) * int64_t(S) < (int64_t(1) << 31);
                if (int rc = make_plan_route(c, er.get(), in_place, p.route, st)) return rc;
            }
        }
        if (fits && p.route)
            return run_plan(c, *p.route, src, src_stripe, src_sym, dst, dst_stripe, dst_sym, n_stripes, S, st, d_ids,
                            dst_local);
    }
    if (p.cs) {
        HIP_TRY(hipSetDevice(c->device));
        // both stages index their inputs with 31-bit byte offsets (the second stage reads D syndrome rows)
        if (!d_ids && !dst_local && S % 1024 == 0 && p.cs->max_slot * src_sym + int64_t(S) < (int64_t(1) << 31) &&
            int64_t(p.cs->D) * int64_t(S) < (int64_t(1) << 31))
            return run_cs(c, p, src, src_stripe, src_sym, dst, dst_stripe, dst_sym, n_stripes, S, st);
        if (p.cs->kind == 1) return RS_ERR_INVALID;  // a second stage runs only inside its route (run_cs)
        if (!p.dense) {  // launches the route does not cover run the plain matrix plan
            std::unique_ptr<bool[]> er;
            if (!p.erased.empty()) {
                er.reset(new bool[p.erased.size()]);
                for (size_t i = 0; i < p.erased.size(); ++i) er[i] = p.erased[i] != 0;
            }
            if (int rc = make_plan_dense(c, er.get(), p.dense, st)) return rc;
        }
        return run_plan(c, *p.dense, src, src_stripe, src_sym, dst, dst_stripe, dst_sym, n_stripes, S, st, d_ids,
                        dst_local);
    }
    const int64_t align = p.m == 8 ? 8 : 4;
    if ((S & 1) || (uintptr_t(src) % align) || (uintptr_t(dst) % align) || (src_stripe % align) ||
        (src_sym % align) || (dst_stripe % align) || (dst_sym % align))
        return RS_ERR_INVALID;
    HIP_TRY(hipSetDevice(c->device));
    // a decode plan is specialised (hiprtc) after dec_jit_uses launches that each move at least
    // kJitMinBytes: a compile costs far more than tiny launches (one C1 / C2 stripe per call) can recover
    if (uint64_t(p.K + p.R) * S * n_stripes >= kJitMinBytes) ++p.uses;
    const bool policy = p.m == 8 && p.d_idx &&
                        (c->jit == 1 || (c->jit == 2 && (&p == c->enc.get() || &p == c->syn.get() ||
                                                          p.uses >= c->dec_jit_uses)));
    // bit-plane XOR kernel: slot * stride must fit the kernel's 32-bit scalar offsets
    int64_t max_in = 0, max_out = 0;
    for (int32_t v : p.in_slots) max_in = std::max<int64_t>(max_in, v);
    for (int j = 0; j < p.R; ++j) max_out = std::max<int64_t>(max_out, p.out_slots[size_t(j)]);
    const bool xj_ok = policy && c->xj && !p.xj_failed && xj_supported(p.m, p.K, p.R) && S >= 2048 &&
                       (max_in + 1) * src_sym < (int64_t(1) << 31) && (max_out + 1) * dst_sym < (int64_t(1) << 31);
    if (xj_ok && !p.xj) {
        if (xj_build(p.matrix, p.K, p.R, p.in_slots, p.out_slots, p.xj) || !p.xj) {
            std::fprintf(stderr, "librs_amd: XOR kernel unavailable for a %dx%d matrix; using the next kernel\n", p.R,
                         p.K);
            p.xj_failed = true;
            p.xj.reset();
        }
    }
    if (dst_local && !(xj_ok && p.xj)) return RS_ERR_INVALID;  // only the XOR kernel indexes dst locally
    const bool jit_ok = policy && !(xj_ok && p.xj) && !p.jit_failed && jit_supported(8, p.K, p.R);
    if (jit_ok && !p.jit) {
        const Gamma8& g = gamma8();
        std::vector<uint8_t> cg(p.matrix.size());
        for (size_t e = 0; e < cg.size(); ++e) cg[e] = uint8_t(g.coord(p.matrix[e]));
        if (jit_build(cg, p.K, p.R, p.jit) || !p.jit) {
            std::fprintf(stderr, "librs_amd: JIT kernel unavailable for a %dx%d matrix; using the generic kernel\n",
                         p.R, p.K);
            p.jit_failed = true;
            p.jit.reset();
        }
    }
    ApplyArgs a{};
    a.src = src;
    a.src_stripe = src_stripe;
    a.src_sym = src_sym;
    a.in_idx = p.d_in;
    a.dst = dst;
    a.dst_stripe = dst_stripe;
    a.dst_sym = dst_sym;
    a.out_idx = p.d_out;
    a.coef = p.d_coef;
    a.idx = p.d_idx;
    a.ltab = c->d_ltab;
    a.K = p.K;
    a.R = p.R;
    a.nbytes = int64_t(S);
    a.mode = p.m == 8 ? c->m8_mode : c->m16_mode;
    a.stamps = c->stamps;
    a.ids = d_ids;
#ifdef RS_AMD_DIAG
    if (check_mode()) {  // device-side slot checks (m8_v1_run) with a violation record read by check_launch
        if (!c->d_slot_err) {
            HIP_TRY(hipMalloc(reinterpret_cast<void**>(&c->d_slot_err), 16));
            HIP_TRY(hipMemset(c->d_slot_err, 0, 16));
        }
        a.nslots = p.slot_bound ? p.slot_bound : int32_t(c->k) + c->r;  // codec (or syndrome / staging) slots
        a.slot_err = c->d_slot_err;
    }
#endif
    const bool m8_generic = p.m == 8 && p.d_idx && (a.mode == 18 || a.mode == 20 || a.mode == 21) && !(xj_ok && p.xj) && !(jit_ok && p.jit);
    if ((p.m == 16 && p.rt == 64 && p.d_idx && a.mode < 2) || m8_generic) {  // split-K scratch for small grids
        int64_t need = 0;
        if ((m8_generic ? m8_kslices(a, int64_t(n_stripes), &need) : m16_kslices(a, int64_t(n_stripes), &need)) > 1) {
            if (int rc = scratch_acquire(c, st)) return rc;
            if (int rc = grow(&c->d_partial, c->partial_cap, size_t(need))) return rc;
            a.scratch = static_cast<uint32_t*>(c->d_partial);
            a.scratch_bytes = int64_t(c->partial_cap);
        }
    }
    const int nt32 = (p.R + 31) / 32;
    if (xj_ok && p.xj) {
        XJArgs x{};
        x.src = src;
        x.src_stripe = src_stripe;
        x.dst = dst;
        x.dst_stripe = dst_stripe;
        x.src_sym = int32_t(src_sym);
        x.dst_sym = int32_t(dst_sym);
        x.ids = d_ids;
        x.dst_local = dst_local ? 1u : 0u;
        c->last_kernel = p.xj->name;
        // 256-byte column chunks up to the last full 2 KiB boundary; the rest by the generic tail kernel
        int rc = xj_launch(*p.xj, x, int64_t(n_stripes), (a.nbytes / 2048) * (2048 / kXjChunk), st);
        if (rc) return rc;
        const uint64_t cols = n_stripes * uint64_t(a.nbytes / 2048) * (2048 / kXjChunk);
        c->work_valu += cols * p.xj->valu_per_col;
        c->work_salu += cols * p.xj->salu_per_col;
        launch_m8_tail(a, int64_t(n_stripes), unsigned(nt32), st);
        HIP_TRY(hipGetLastError());
        return 0;
    }
    if (jit_ok && p.jit) {
        const int64_t full = (a.nbytes / 2048) * 2;  // 1 KiB chunks up to the last full 2 KiB boundary
        c->last_kernel = p.jit->name;
        if (full > 0) {
            int rc = jit_launch(*p.jit, v1_args(a, full, nullptr), int64_t(n_stripes), st);
            if (rc) return rc;
        }
        launch_m8_tail(a, int64_t(n_stripes), unsigned(nt32), st);
        HIP_TRY(hipGetLastError());
        return 0;
    }
    // gpr-index kernel families (modes >= 2) always tile 32 rows
    const int rt = p.m == 8 && a.mode >= 2 ? 32 : p.rt;
    c->last_kernel = p.m == 8 ? (std::string("apply_m8_rt") + std::to_string(rt) + "_mode" + std::to_string(a.mode))
                     : (rt == 64 && p.d_idx && a.mode < 2) ? std::string(a.mode ? "apply_m16_v1_plain" : "apply_m16_v1")
                                                             : (std::string("apply_m16_rt") + std::to_string(rt));
    HIP_TRY(launch_apply(p.m, rt, a, int64_t(n_stripes), st));
    if (p.m == 16 && rt == 64 && p.d_idx && a.mode < 2) {  // k_apply_m16_v1 over the full 1 KiB chunks
        const uint64_t steps = n_stripes * (S / 1024) * uint64_t((p.R + 63) / 64) * 4 * uint64_t(p.K);
        c->work_valu += steps * kValu_m16_v1;
        c->work_salu += steps * kSalu_m16_v1;
    }
    if (a.scratch) return scratch_release(c, st);  // split-K partials in flight on st
    return 0;
}

}  // namespace rsamd

extern "C" int rsg_last_work(const rsg_codec_t* c, uint64_t* valu, uint64_t* salu) {
    if (!c) return RS_ERR_INVALID;
    if (valu) *valu = c->work_valu;
    if (salu) *salu = c->work_salu;
    return 0;
}

extern "C" int rsg_encode(rsg_codec_t* c, const void* d_info, uint64_t info_stripe_stride, uint64_t info_symbol_stride,
                          void* d_rep, uint64_t rep_stripe_stride, uint64_t rep_symbol_stride, uint64_t n_stripes,
                          uint64_t symbol_size, void* stream) {
    rsamd::CallerDevice caller_device;
    if (!c) return RS_ERR_INVALID;
    c->work_valu = c->work_salu = 0;
    return run_plan(c, *c->enc, static_cast<const uint8_t*>(d_info), int64_t(info_stripe_stride),
                    int64_t(info_symbol_stride), static_cast<uint8_t*>(d_rep), int64_t(rep_stripe_stride),
                    int64_t(rep_symbol_stride), n_stripes, symbol_size, static_cast<hipStream_t>(stream));
}

namespace rsamd {

int decode_plan(rsg_codec_t* c, const bool* is_erased, uint16_t t, DevPlan** out, hipStream_t st) {
    const size_t n = size_t(c->k) + c->r;
    if (t > c->r) return RS_ERR_CANNOT_RESTORE;
    std::vector<uint8_t> key(n);
    size_t cnt = 0;
    for (size_t i = 0; i < n; ++i) cnt += (key[i] = is_erased[i] ? 1 : 0);
    if (cnt != t) return RS_ERR_INVALID;
    auto it = c->dec.find(key);
    if (it == c->dec.end()) {
        std::unique_ptr<DevPlan> p;
        if (int rc = make_plan(c, is_erased, p, st)) return rc;
        if (c->dec_lru.size() >= 16) {
            auto old = c->dec.find(c->dec_lru.front());
            if (old != c->dec.end()) {
                old->second->guard_before_release(st);
                c->dec.erase(old);
            }
            c->dec_lru.erase(c->dec_lru.begin());
        }
        c->dec_lru.push_back(key);
        it = c->dec.emplace(key, std::move(p)).first;
    }
    *out = it->second.get();
    return 0;
}

}  // namespace rsamd

extern "C" int rsg_decode(rsg_codec_t* c, void* d_rcv, uint64_t stripe_stride, uint64_t symbol_stride,
                          uint64_t n_stripes, uint64_t symbol_size, const bool* is_erased, uint16_t t, void* stream) {
    rsamd::CallerDevice caller_device;
    if (!c || !is_erased) return RS_ERR_INVALID;
    c->work_valu = c->work_salu = 0;
    if (t > c->r) return RS_ERR_CANNOT_RESTORE;
    DevPlan* p = nullptr;
    int rc = decode_plan(c, is_erased, t, &p, static_cast<hipStream_t>(stream));
    if (rc) return rc;
    uint8_t* base = static_cast<uint8_t*>(d_rcv);
    return run_plan(c, *p, base, int64_t(stripe_stride), int64_t(symbol_stride), base, int64_t(stripe_stride),
                    int64_t(symbol_stride), n_stripes, symbol_size, static_cast<hipStream_t>(stream));
}

namespace rsamd {

// rsg_decode_batch scratch: wait until the previous call's launches are done with it / mark this one's
int scratch_acquire(rsg_codec_t* c, hipStream_t st) {
    // work queued earlier on the same stream runs first anyway; another stream's is waited for
    if (c->scratch_pending && c->scratch_stream != st) HIP_TRY(hipEventSynchronize(c->scratch_ev));
    c->scratch_pending = false;
    return 0;
}
int scratch_release(rsg_codec_t* c, hipStream_t st) {
    if (!c->scratch_ev) HIP_TRY(hipEventCreateWithFlags(&c->scratch_ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(c->scratch_ev, st));
    c->scratch_pending = true;
    c->scratch_stream = st;
    return 0;
}

// A route that fails after its first launch returns with work still queued (on st, and on the codec's side
// and syndrome streams for the per-stripe routes) and without marking the scratch busy: join those streams
// into st and mark the scratch as used by st, so the next call (on any stream) waits for the orphaned kernels
// before it overwrites lists, records or syndromes they may still read. Best effort: rc, the call's own
// error, is what gets reported.
int scratch_fence(rsg_codec_t* c, hipStream_t st, int rc) {
    if (!rc) return 0;
    for (hipStream_t s : {c->ps_side, c->ps_synst}) {
        if (!s) continue;
        hipEvent_t e = nullptr;
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess) {
            if (hipEventRecord(e, s) == hipSuccess) (void)hipStreamWaitEvent(st, e, 0);
            (void)hipEventDestroy(e);
        }
    }
    (void)scratch_release(c, st);
    (void)hipGetLastError();
    return rc;
}

// ---------------------------------------------------------------- host-memory batches (PCIe)
// Stripes in host memory: batches of stripes alternate over two streams, each H2D -> kernel -> D2H,
// so one batch's kernel overlaps the other's copies and H2D overlaps D2H. Pinned host memory
// (hipHostMalloc / hipHostRegister) runs the copies at PCIe rate; pageable memory works, slower.
constexpr size_t kHostBatchBytes = size_t(256) << 20;  // device buffer per stream

int host_pipe_reserve(rsg_codec_t* c, size_t bytes) {
    HIP_TRY(hipSetDevice(c->device));
    for (int i = 0; i < 2; ++i)
        if (!c->hs[i]) HIP_TRY(hipStreamCreateWithFlags(&c->hs[i], hipStreamNonBlocking));
    if (bytes > c->hbuf_cap) {
        for (int i = 0; i < 2; ++i) {
            if (c->hbuf[i]) (void)hipFree(c->hbuf[i]);
            c->hbuf[i] = nullptr;
        }
        c->hbuf_cap = 0;
        for (int i = 0; i < 2; ++i) HIP_TRY(hipMalloc(reinterpret_cast<void**>(&c->hbuf[i]), bytes));
        c->hbuf_cap = bytes;
    }
    return 0;
}

}  // namespace rsamd

extern "C" int rsg_encode_host(rsg_codec_t* c, const void* h_info, uint64_t info_stripe_stride,
                               uint64_t info_symbol_stride, void* h_rep, uint64_t rep_stripe_stride,
                               uint64_t rep_symbol_stride, uint64_t n_stripes, uint64_t symbol_size) {
    rsamd::CallerDevice caller_device;
    if (!c || (n_stripes && (!h_info || !h_rep))) return RS_ERR_INVALID;
    const uint64_t S = symbol_size, k = c->k, r = c->r;
    if (S & 1) return RS_ERR_INVALID;
    if (!n_stripes || !S || !r) return 0;
    const uint64_t P = (S + 15) & ~uint64_t(15), per = (k + r) * P;
    const uint64_t B = std::max<uint64_t>(1, std::min<uint64_t>(n_stripes, kHostBatchBytes / per));
    if (int rc = host_pipe_reserve(c, size_t(B * per))) return rc;
    const bool reg_in = info_stripe_stride == k * info_symbol_stride, reg_out = rep_stripe_stride == r * rep_symbol_stride;
    const uint8_t* hi = static_cast<const uint8_t*>(h_info);
    uint8_t* ho = static_cast<uint8_t*>(h_rep);
    for (uint64_t s0 = 0, it = 0; s0 < n_stripes; s0 += B, ++it) {
        const uint64_t nb = std::min(B, n_stripes - s0);
        hipStream_t st = c->hs[it & 1];
        uint8_t* d_info = c->hbuf[it & 1];  // [nb][k][P] then [nb][r][P]
        uint8_t* d_rep = d_info + nb * k * P;
        if (reg_in)
            HIP_TRY(hipMemcpy2DAsync(d_info, P, hi + s0 * info_stripe_stride, info_symbol_stride, S, nb * k,
                                     hipMemcpyHostToDevice, st));
        else
            for (uint64_t b = 0; b < nb; ++b)
                HIP_TRY(hipMemcpy2DAsync(d_info + b * k * P, P, hi + (s0 + b) * info_stripe_stride, info_symbol_stride,
                                         S, k, hipMemcpyHostToDevice, st));
        if (int rc = rsg_encode(c, d_info, k * P, P, d_rep, r * P, P, nb, S, st)) return rc;
        if (reg_out)
            HIP_TRY(hipMemcpy2DAsync(ho + s0 * rep_stripe_stride, rep_symbol_stride, d_rep, P, S, nb * r,
                                     hipMemcpyDeviceToHost, st));
        else
            for (uint64_t b = 0; b < nb; ++b)
                HIP_TRY(hipMemcpy2DAsync(ho + (s0 + b) * rep_stripe_stride, rep_symbol_stride, d_rep + b * r * P, P, S,
                                         r, hipMemcpyDeviceToHost, st));
    }
    HIP_TRY(hipStreamSynchronize(c->hs[0]));
    HIP_TRY(hipStreamSynchronize(c->hs[1]));
    return 0;
}

extern "C" int rsg_decode_host(rsg_codec_t* c, void* h_rcv, uint64_t stripe_stride, uint64_t symbol_stride,
                               uint64_t n_stripes, uint64_t symbol_size, const bool* is_erased, uint16_t t) {
    rsamd::CallerDevice caller_device;
    if (!c || !is_erased || (n_stripes && !h_rcv)) return RS_ERR_INVALID;
    if (t > c->r) return RS_ERR_CANNOT_RESTORE;
    const uint64_t S = symbol_size, n = uint64_t(c->k) + c->r;
    if (S & 1) return RS_ERR_INVALID;
    std::vector<int> lost;  // restored (erased information) slots
    uint16_t cnt = 0;
    for (uint64_t i = 0; i < n; ++i)
        if (is_erased[i]) {
            ++cnt;
            if (i < c->k) lost.push_back(int(i));
        }
    if (cnt != t) return RS_ERR_INVALID;
    if (!n_stripes || !S || lost.empty()) return 0;
    const uint64_t P = (S + 15) & ~uint64_t(15), per = n * P;
    const uint64_t B = std::max<uint64_t>(1, std::min<uint64_t>(n_stripes, kHostBatchBytes / per));
    if (int rc = host_pipe_reserve(c, size_t(B * per))) return rc;
    // surviving slots in runs of consecutive slots: with rows packed in host and device memory
    // (symbol_stride == S == P) a run of every stripe of a batch is one strided copy, erased slots are
    // never transferred (the decoder does not read them)
    std::vector<std::pair<uint64_t, uint64_t>> runs;  // [first slot, count)
    for (uint64_t i = 0; i < n;) {
        if (is_erased[i]) {
            ++i;
            continue;
        }
        uint64_t j = i;
        while (j < n && !is_erased[j]) ++j;
        runs.emplace_back(i, j - i);
        i = j;
    }
    const bool packed_rows = symbol_stride == S && S == P;
    uint8_t* h = static_cast<uint8_t*>(h_rcv);
    for (uint64_t s0 = 0, it = 0; s0 < n_stripes; s0 += B, ++it) {
        const uint64_t nb = std::min(B, n_stripes - s0);
        hipStream_t st = c->hs[it & 1];
        uint8_t* d = c->hbuf[it & 1];  // [nb][k + r][P]
        if (packed_rows)
            for (const auto& run : runs)
                HIP_TRY(hipMemcpy2DAsync(d + run.first * P, n * P, h + s0 * stripe_stride + run.first * S, stripe_stride,
                                         run.second * S, nb, hipMemcpyHostToDevice, st));
        else
            for (const auto& run : runs)  // per slot: the slot of every stripe of the batch
                for (uint64_t i = run.first; i < run.first + run.second; ++i)
                    HIP_TRY(hipMemcpy2DAsync(d + i * P, n * P, h + s0 * stripe_stride + i * symbol_stride,
                                             stripe_stride, S, nb, hipMemcpyHostToDevice, st));
        if (int rc = rsg_decode(c, d, n * P, P, nb, S, is_erased, t, st)) return rc;
        for (int i : lost)  // restored slot i of every stripe of the batch: one strided copy
            HIP_TRY(hipMemcpy2DAsync(h + s0 * stripe_stride + uint64_t(i) * symbol_stride, stripe_stride,
                                     d + uint64_t(i) * P, n * P, S, nb, hipMemcpyDeviceToHost, st));
    }
    HIP_TRY(hipStreamSynchronize(c->hs[0]));
    HIP_TRY(hipStreamSynchronize(c->hs[1]));
    return 0;
}

extern "C" int rsg_fill_info(void* d_base, uint64_t stripe_stride, uint64_t symbol_stride, uint64_t symbol_size,
                             uint16_t k, uint64_t stripe0, uint64_t n_stripes, uint64_t seed, void* stream) {
    rsamd::CallerDevice caller_device;
    if (symbol_size % 8 || symbol_stride % 8 || stripe_stride % 8 || uintptr_t(d_base) % 8) return RS_ERR_INVALID;
    if (!n_stripes || !k) return 0;
    HIP_TRY(launch_gen_info(static_cast<uint8_t*>(d_base), int64_t(stripe_stride), int64_t(symbol_stride),
                            int64_t(symbol_size), k, int64_t(stripe0), int64_t(n_stripes), seed,
                            static_cast<hipStream_t>(stream)));
    return 0;
}

extern "C" int rsg_fingerprint(const void* d_base, uint64_t stripe_stride, uint64_t symbol_stride,
                               uint64_t symbol_size, uint32_t sym0, uint32_t nsym, uint64_t n_stripes, uint64_t* d_out,
                               void* stream) {
    rsamd::CallerDevice caller_device;
    if (symbol_size % 8 || symbol_stride % 8 || stripe_stride % 8 || uintptr_t(d_base) % 8) return RS_ERR_INVALID;
    if (!n_stripes) return 0;
    HIP_TRY(launch_fingerprint(static_cast<const uint8_t*>(d_base), int64_t(stripe_stride), int64_t(symbol_stride),
                               int64_t(symbol_size), int(sym0), int(nsym), int64_t(n_stripes),
                               reinterpret_cast<unsigned long long*>(d_out), static_cast<hipStream_t>(stream)));
    return 0;
}

extern "C" int rsg_coding_matrix(uint16_t k, uint16_t r, const bool* is_erased, uint16_t t, uint16_t* matrix,
                                 uint32_t* rows, uint32_t* cols, int32_t* in_slots, int32_t* out_slots) {
    if (uint32_t(k) + r > kN) return RS_ERR_INVALID;
    if (is_erased) {
        if (t > r) return RS_ERR_CANNOT_RESTORE;
        size_t cnt = 0;
        for (size_t i = 0; i < size_t(k) + r; ++i) cnt += is_erased[i] ? 1 : 0;
        if (cnt != t) return RS_ERR_INVALID;
    }
    std::vector<uint16_t> pos = code_positions(k, r), M;
    std::vector<int32_t> in, outs;
    codec_matrix(pos, k, r, is_erased, M, in, outs);
    if (rows) *rows = uint32_t(outs.size());
    if (cols) *cols = uint32_t(in.size());
    copy_out(matrix, M);
    copy_out(in_slots, in);
    copy_out(out_slots, outs);
    return 0;
}

extern "C" int rsg_jit_precompile(uint16_t k, uint16_t r, const bool* is_erased, uint16_t t) {
    if (uint32_t(k) + r > kN) return RS_ERR_INVALID;
    std::vector<uint16_t> pos = code_positions(k, r), M;
    if (subfield_degree(pos) > 8) return 0;
    std::vector<int32_t> in, outs;
    if (is_erased) {
        size_t cnt = 0;
        for (size_t i = 0; i < size_t(k) + r; ++i) cnt += is_erased[i] ? 1 : 0;
        if (cnt != t || t > r) return RS_ERR_INVALID;
    }
    codec_matrix(pos, k, r, is_erased, M, in, outs);
    if (xj_supported(8, int(in.size()), int(outs.size())))
        return xj_precompile(M, int(in.size()), int(outs.size()), in, outs);
    const Gamma8& g = gamma8();
    std::vector<uint8_t> cg(M.size());
    for (size_t e = 0; e < cg.size(); ++e) cg[e] = uint8_t(g.coord(M[e]));
    return jit_precompile(cg, int(in.size()), int(outs.size()));
}

extern "C" int rsg_xj_source(uint16_t k, uint16_t r, const bool* is_erased, uint16_t t, char* buf, size_t cap,
                             size_t* len) {
    if (uint32_t(k) + r > kN) return RS_ERR_INVALID;
    std::vector<uint16_t> pos = code_positions(k, r), M;
    if (subfield_degree(pos) > 8) return RS_ERR_INVALID;
    if (is_erased) {
        size_t cnt = 0;
        for (size_t i = 0; i < size_t(k) + r; ++i) cnt += is_erased[i] ? 1 : 0;
        if (cnt != t || t > r) return RS_ERR_INVALID;
    }
    std::vector<int32_t> in, outs;
    codec_matrix(pos, k, r, is_erased, M, in, outs);
    if (!xj_supported(8, int(in.size()), int(outs.size()))) return RS_ERR_INVALID;
    const std::string src = xj_source(M, int(in.size()), int(outs.size()), in, outs, true);
    if (len) *len = src.size();
    if (buf && cap) {
        const size_t n = std::min(cap - 1, src.size());
        std::memcpy(buf, src.data(), n);
        buf[n] = 0;
    }
    return 0;
}

extern "C" int rsg_xj_basis(int32_t* pivots, uint16_t* beta_y, uint8_t* bits256) {
    const XjBasis& B = xj_basis(xj_horner(true));  // inspection API: honours RS_XJ_HORNER like rsg_xj_source
    if (pivots)
        for (int t = 0; t < 8; ++t) pivots[t] = B.pivots[t];
    if (beta_y)
        for (int t = 0; t < 8; ++t) beta_y[t] = B.beta_y[t];
    if (bits256) {
        const Gamma8& g = gamma8();
        for (int b = 0; b < 256; ++b) bits256[b] = B.bits(g.to_elem[b]);
    }
    return 0;
}

extern "C" int rsg_gamma_tables(uint16_t* lbyte, uint16_t* ibyte, uint8_t* red) {
    const Gamma8& g = gamma8();
    if (lbyte) std::memcpy(lbyte, g.lbyte, sizeof(g.lbyte));
    if (ibyte) std::memcpy(ibyte, g.ibyte, sizeof(g.ibyte));
    if (red) *red = g.red;
    return 0;
}

extern "C" const char* rsg_version(void) { return RSG_VERSION; }

extern "C" int rsg_check_enabled(void) { return rsamd::check_mode() ? 1 : 0; }
