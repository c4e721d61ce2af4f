// rs_batch.cpp -- rsg_decode_batch: one erasure pattern per stripe (SURVEY f-2).
// Stripes sharing a pattern share a plan and a launch; past kHostPlanGroups patterns the decode
// matrices are built on the device (GF(256): the syndrome route or survivor plans; GF(2^16): the
// per-stripe syndrome route or one plan rebuilt on the stream per pattern).
#include "rs_core.hpp"

using namespace rsamd;

namespace rsamd {

// The host lists of a batch call (stripe ids, erasure masks) reach the device through the codec's pinned
// staging: one copy per list queued on the caller's stream, and the call returns without waiting for
// them (it used to synchronise the caller's whole stream). The staging is grow-only and guarded by an event:
// the next call that overwrites it waits for the previous call's copies only.
struct ListPart {
    void* dst;
    const void* src;
    size_t bytes;
};
int stage_lists(rsg_codec_t* c, hipStream_t st, std::initializer_list<ListPart> parts) {
    size_t total = 0;
    for (const ListPart& q : parts) total += (q.bytes + 255) & ~size_t(255);
    if (c->stage_pending) HIP_TRY(hipEventSynchronize(c->stage_ev));
    c->stage_pending = false;
    if (total > c->stage_cap) {
        if (c->h_stage) HIP_TRY(hipHostFree(c->h_stage));
        c->h_stage = nullptr;
        c->stage_cap = 0;
        HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&c->h_stage), std::max<size_t>(total, 4096), hipHostMallocDefault));
        c->stage_cap = std::max<size_t>(total, 4096);
    }
    if (!c->stage_ev) HIP_TRY(hipEventCreateWithFlags(&c->stage_ev, hipEventDisableTiming));
    size_t off = 0;
    for (const ListPart& q : parts) {
        if (q.bytes) {
            std::memcpy(c->h_stage + off, q.src, q.bytes);
            HIP_TRY(hipMemcpyAsync(q.dst, c->h_stage + off, q.bytes, hipMemcpyHostToDevice, st));
        }
        off += (q.bytes + 255) & ~size_t(255);
    }
    HIP_TRY(hipEventRecord(c->stage_ev, st));
    c->stage_pending = true;
    return 0;
}

// Distinct patterns beyond which rsg_decode_batch builds the decode matrices on the device (the
// host plan cache holds 16; past it every pattern would cost a host build, an upload and a launch).
constexpr size_t kHostPlanGroups = 16;

// The fixed r x (k + r) matrix of the GF(256) per-stripe route over every slot: route 1 the r syndromes,
// H[j][i] = X_i^j (reed_solomon.c:443-559); route 2 the re-encode differences [G | I] (k_plan_reenc_m8), G the
// encode matrix, I on the repair slots.
std::vector<uint16_t> syn_fixed_matrix(const std::vector<uint16_t>& positions, int k, int r, int route) {
    const int n = k + r;
    std::vector<uint16_t> H(size_t(r) * n);
    if (route == 2) {
        std::vector<uint16_t> G;
        std::vector<int32_t> gi, go;
        codec_matrix(positions, uint16_t(k), uint16_t(r), nullptr, G, gi, go);  // r x k
        for (int p = 0; p < r; ++p) {
            for (int i = 0; i < k; ++i) H[size_t(p) * n + i] = G[size_t(p) * k + i];
            H[size_t(p) * n + k + p] = 1;
        }
    } else {
        const Field& F = field();
        for (int j = 0; j < r; ++j)
            for (int i = 0; i < n; ++i) H[size_t(j) * n + i] = F.exp[(uint64_t(positions[i]) * j) % kN];
    }
    return H;
}

// Syndrome route eligibility: the r x (k + r) syndrome matrix H[j][i] = X_i^j runs on its bit-plane XOR
// kernel (built once per codec), which covers whole 2 KiB column blocks only.
bool syn_prepare(rsg_codec_t* c, uint64_t S, int64_t symbol_stride) {
    const int n = int(c->k) + c->r;
    if (!c->syn_route || c->syn_failed || !c->xj || c->jit == 0 || c->m > 8 || S % 2048 || !xj_supported(8, n, c->r) ||
        int64_t(n) * symbol_stride >= (int64_t(1) << 31) || int64_t(c->r) * int64_t(S) >= (int64_t(1) << 31))
        return false;
    if (!c->syn) {
        std::vector<uint16_t> H = syn_fixed_matrix(c->positions, c->k, c->r, c->syn_route);
        std::vector<int32_t> in(n), out(c->r);
        for (int i = 0; i < n; ++i) in[size_t(i)] = i;
        for (int j = 0; j < c->r; ++j) out[size_t(j)] = j;
        std::unique_ptr<DevPlan> p;
        if (build_plan(c->device, 8, std::move(H), n, c->r, std::move(in), std::move(out), p, nullptr) || !p ||
            hipStreamSynchronize(nullptr) != hipSuccess) {
            c->syn_failed = true;
            return false;
        }
        // the masked form (default): each stripe's erased slots read as zero (XJArgs::masks); option m8_syn_coord
        // (diagnostic): with the prefetching solve 10 (whose slot lists need 19 entries past K: K <= min(k, r) or
        // r), its outputs stored in coordinates (form 2), which the solve then reads as they are
        const int kmax = c->syn_route == 2 ? std::min<int>(c->k, c->r) : int(c->r);
        const bool coord = c->m8_syn_masked && c->m8_syn_coord && c->m8_ps_kernel == 10 && kmax + 3 <= n;
        if (xj_build(p->matrix, p->K, p->R, p->in_slots, p->out_slots, p->xj, c->m8_syn_masked ? (coord ? 2 : 1) : 0) ||
            !p->xj) {
            std::fprintf(stderr, "librs_amd: syndrome XOR kernel unavailable; per-stripe survivor plans\n");
            c->syn_failed = true;
            return false;
        }
        c->syn = std::move(p);
    }
    return true;
}

// The masked fixed pass of one chunk of the syndrome / re-encode route: the r rows of every selected stripe
// into the chunk-local scratch, each stripe's erased slots (bits of its mask words) read as zero, so the
// per-stripe solve yields the erased information symbols themselves and stores them.
static int syn_fixed_pass(rsg_codec_t* c, const uint8_t* base, int64_t stripe_stride, int64_t symbol_stride,
                          uint8_t* syn, int64_t per, uint64_t S, int64_t cn, const int32_t* d_ids,
                          const uint32_t* d_mbits, uint32_t mw, hipStream_t st) {
    DevPlan& p = *c->syn;
    if (int rc = p.order_after_build(st)) return rc;
    XJArgs x{};
    x.src = base;
    x.src_stripe = stripe_stride;
    x.dst = syn;
    x.dst_stripe = per;
    x.src_sym = int32_t(symbol_stride);
    x.dst_sym = int32_t(S);
    x.ids = d_ids;
    x.dst_local = 1u;
    if (p.xj->masked) {
        x.mask_words = mw;
        x.masks = d_mbits;
        x.zero = static_cast<const uint8_t*>(c->d_zero);
    }
    if (p.xj->coord) x.tab = reinterpret_cast<const uint16_t*>(c->d_ltab);  // its outputs' coordinate tables
    c->last_kernel = p.xj->name;
    const int rc = xj_launch(*p.xj, x, cn, int64_t(S / 2048) * (2048 / kXjChunk), st);
    const int rc2 = p.note_use(st);
    if (!rc && !rc2) RS_CHECKPOINT(c, &p, "per-stripe fixed pass (rs_xj)", uint64_t(cn), S);
    return rc ? rc : rc2;
}

// Nonzero bytes of [p, p + len): an erasure pattern's set entries (a bool is erased when nonzero, as in
// reed_solomon.c's `if (is_erased[i])`). Vectorises; the 32-bit partial sums cannot overflow.
size_t count_nonzero(const uint8_t* p, size_t len) {
    size_t c = 0;
    for (size_t i0 = 0; i0 < len; i0 += 4096) {
        const size_t e = std::min(len, i0 + 4096);
        uint32_t cc = 0;
        for (size_t i = i0; i < e; ++i) cc += p[i] != 0;
        c += cc;
    }
    return c;
}

// 64-bit hash of [p, p + len) (four independent multiply-xor lanes over 8-byte words, then the tail)
uint64_t hash_bytes(const uint8_t* p, size_t len) {
    constexpr uint64_t kM = 0x9E3779B97F4A7C15ull;
    uint64_t h[4] = {len, kM, ~len, kM ^ len};
    size_t i = 0;
    for (; i + 32 <= len; i += 32)
        for (int l = 0; l < 4; ++l) {
            uint64_t w;
            std::memcpy(&w, p + i + 8 * l, 8);
            h[l] = (h[l] ^ w) * kM;
            h[l] ^= h[l] >> 29;
        }
    uint64_t r = h[0] ^ (h[1] * 3) ^ (h[2] * 5) ^ (h[3] * 7);
    for (; i < len; ++i) r = (r ^ p[i]) * kM;
    return r ^ (r >> 31);
}

// rsg_decode_batch for m <= 8 codes with device-built plans: k_plan_m8 turns each selected stripe's
// erasure mask into its decode matrix (nibble records of the V = 1 kernel), then one V = 1 launch (+
// the tail kernel) applies every stripe's own plan. Stripes without erased information slots are
// skipped; the caller has validated every pattern.
int decode_batch_device_plans(rsg_codec_t* c, uint8_t* base, int64_t stripe_stride, int64_t symbol_stride,
                              uint64_t n_stripes, uint64_t S, const bool* is_erased, const int32_t* tr,
                              hipStream_t st) {
    const size_t n = size_t(c->k) + c->r;
    if ((S & 1) || (uintptr_t(base) % 8) || (stripe_stride % 8) || (symbol_stride % 8)) return RS_ERR_INVALID;
    std::vector<int32_t> ids;
    for (uint64_t s = 0; s < n_stripes; ++s)
        if (tr[2 * s + 1]) ids.push_back(int32_t(s));
    if (ids.empty()) return 0;
    std::vector<uint8_t> masks(ids.size() * n);
    for (size_t j = 0; j < ids.size(); ++j) {
        const uint8_t* e = reinterpret_cast<const uint8_t*>(is_erased + size_t(ids[j]) * n);
        for (size_t i = 0; i < n; ++i) masks[j * n + i] = e[i] != 0;
    }
    int rc = scratch_acquire(c, st);
    if (rc) return rc;
    const uint16_t* logt = nullptr;
    const uint8_t* g8 = nullptr;
    rc = plan_tables(c->device, &logt, &g8);
    if (rc) return rc;
    if (!c->d_elem) {
        const Field& F = field();
        std::vector<uint16_t> el(n);
        for (size_t i = 0; i < n; ++i) el[i] = F.exp[c->positions[i]];
        if ((rc = upload(reinterpret_cast<void**>(&c->d_elem), el.data(), n * 2))) return rc;
    }
    const int64_t nsel = int64_t(ids.size());
    const int tiles = (std::min<int>(c->k, c->r) + 31) / 32;  // erased information slots <= min(k, r)
    const int64_t in_stride = int64_t(n) + 16, out_stride = int64_t(tiles) * 32, idx_stride = int64_t(tiles) * n * 64;
    // plans are built and applied in chunks of stripes: at most 256 MiB of nibble records at a time
    const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(nsel, (int64_t(256) << 20) / (idx_stride * 4)));
    size_t ids_bytes = c->ids_cap * 4;  // ids_cap counts entries
    rc = grow(reinterpret_cast<void**>(&c->d_ids), ids_bytes, ids.size() * 4);
    c->ids_cap = ids_bytes / 4;
    if (rc) return rc;
    if ((rc = grow(&c->d_masks, c->masks_cap, masks.size()))) return rc;
    if ((rc = grow(&c->d_kr, c->kr_cap, size_t(chunk) * 8))) return rc;
    if ((rc = grow(&c->d_pin, c->pin_cap, size_t(chunk * in_stride) * 4))) return rc;
    if ((rc = grow(&c->d_pout, c->pout_cap, size_t(chunk * out_stride) * 4))) return rc;
    if ((rc = grow(&c->d_pidx, c->pidx_cap, size_t(chunk * idx_stride) * 4))) return rc;
    const bool syn = syn_prepare(c, S, symbol_stride);
    // the masked fixed pass takes each stripe's pattern as bit words ([chunk][mw]), written by the plan kernels
    const uint32_t mw = uint32_t((n + 31) / 32);
    if (syn) {
        if (S > c->zero_cap) {  // one symbol of zeros: erased slots' columns read it column for column
            if (c->d_zero) (void)hipFree(c->d_zero);
            c->d_zero = nullptr;
            c->zero_cap = 0;
            HIP_TRY(hipMalloc(&c->d_zero, S));
            // zeroed on the launch stream and waited for: later calls may come on other streams (once per growth)
            HIP_TRY(hipMemsetAsync(c->d_zero, 0, S, st));
            HIP_TRY(hipStreamSynchronize(st));
            c->zero_cap = S;
        }
    }
    if ((rc = stage_lists(c, st, {{c->d_ids, ids.data(), ids.size() * 4}, {c->d_masks, masks.data(), masks.size()}})))
        return rc;
    if (syn) {
        // syndrome / re-encode route: the per-stripe solves (k_plan_syn_m8 / k_plan_reenc_m8), the masked
        // fixed pass's r outputs of every selected stripe into scratch (XOR kernel, dst indexed by the
        // chunk-local stripe; erased slots read as zero, so nothing needs zeroing first), then the per-stripe
        // solves from those stored into the erased information slots. Option m8_syn_overlap (diagnostic build): plans
        // and fixed pass of chunk i + 1 run on the codec's syndrome stream beside chunk i's solve on the caller's
        // stream, two buffer sets alternating.
        const uint16_t* expt = nullptr;
        if ((rc = plan_tables(c->device, &logt, &g8, &expt))) return rc;
        const int64_t per = int64_t(c->r) * int64_t(S);
        int64_t sch = std::max<int64_t>(1, std::min<int64_t>(chunk, (c->syn_scratch_mib << 20) / per));
        const bool ovl = c->m8_syn_overlap && nsel > sch / 2;
        if (ovl) sch = std::max<int64_t>(1, std::min<int64_t>(sch, (nsel + 3) / 4));  // at least 4 chunks
        const int nset = ovl ? 2 : 1;
        if ((rc = grow(&c->d_syn, c->syn_cap, size_t(nset * sch * per)))) return rc;
        if ((rc = grow(&c->d_kr, c->kr_cap, size_t(nset * sch) * 8))) return rc;
        if ((rc = grow(&c->d_pin, c->pin_cap, size_t(nset * sch * in_stride) * 4))) return rc;
        if ((rc = grow(&c->d_pout, c->pout_cap, size_t(nset * sch * out_stride) * 4))) return rc;
        if ((rc = grow(&c->d_pidx, c->pidx_cap, size_t(nset * sch * idx_stride) * 4))) return rc;
        if ((rc = grow(&c->d_mbits, c->mbits_cap, size_t(nset * sch) * mw * 4))) return rc;
        // the prefetching solves (m8_ps_kernel 9-11) need whole 1 KiB chunks, 32-bit input offsets, and slot lists
        // 19 entries longer than K: their slot blocks of 8 are loaded up to two blocks ahead (K + 18 at most;
        // in_stride = n + 16, K <= min(k, r) on the re-encode route, <= r on the syndrome route)
        const int kmax = c->syn_route == 2 ? std::min<int>(c->k, c->r) : int(c->r);
        const bool pf = c->m8_ps_kernel >= 9 && S % 1024 == 0 && uint64_t(sch) * uint64_t(per) <= 0xFFFFFFFFull &&
                        int64_t(kmax) + 19 <= in_stride;
        hipStream_t sy = st;
        if (ovl) {
            if ((rc = overlap_objects(c))) return rc;
            sy = c->ps_synst;
            HIP_TRY(hipEventRecord(c->ps_ev_entry, st));  // the stripes' earlier writers on st come first
            HIP_TRY(hipStreamWaitEvent(sy, c->ps_ev_entry, 0));
        }
        for (int64_t c0 = 0, ci = 0; c0 < nsel; c0 += sch, ++ci) {
            const int64_t cn = std::min(sch, nsel - c0);
            const int set = ovl ? int(ci & 1) : 0;
            if (ovl && ci >= 2) HIP_TRY(hipStreamWaitEvent(sy, c->ps_ev_used[set], 0));  // chunk ci - 2's solve read it
            SynPlanArgs pa{};
            pa.masks = static_cast<const uint8_t*>(c->d_masks) + size_t(c0) * n;
            pa.elem = c->d_elem;
            pa.logt = logt;
            pa.expt = expt;
            pa.g8 = g8;
            pa.k = c->k;
            pa.r = c->r;
            pa.n = int32_t(n);
            pa.kr = static_cast<int32_t*>(c->d_kr) + 2 * set * sch;
            pa.pin = static_cast<int32_t*>(c->d_pin) + set * sch * in_stride;
            pa.pout = static_cast<int32_t*>(c->d_pout) + set * sch * out_stride;
            pa.pidx = static_cast<uint32_t*>(c->d_pidx) + set * sch * idx_stride;
            pa.in_stride = in_stride;
            pa.out_stride = out_stride;
            pa.idx_stride = idx_stride;
            pa.mbits = static_cast<uint32_t*>(c->d_mbits) + size_t(set * sch) * mw;
            pa.mw = int32_t(mw);
            if (pf) {  // packed records for k_apply_m8_pf, in the same buffer (a quarter of its stride)
                pa.pidx8 = reinterpret_cast<uint8_t*>(pa.pidx);
                pa.idx8_stride = idx_stride * 4;
            }
            HIP_TRY(launch_plan_syn_m8(pa, cn, sy, c->syn_route));
            uint8_t* syn = static_cast<uint8_t*>(c->d_syn) + set * sch * per;
            if ((rc = syn_fixed_pass(c, base, stripe_stride, symbol_stride, syn, per, S, cn, c->d_ids + c0, pa.mbits,
                                     mw, sy)))
                return rc;
            if (ovl) {
                HIP_TRY(hipEventRecord(c->ps_ev_syn[set], sy));
                HIP_TRY(hipStreamWaitEvent(st, c->ps_ev_syn[set], 0));
            }
            V1Args v{};
            v.src = syn;
            v.src_stripe = 0;  // input slots of the plan are local * r + j, relative to this set's buffer
            v.src_sym = int64_t(S);
            v.in_idx = pa.pin;
            v.dst = base;
            v.dst_stripe = stripe_stride;
            v.dst_sym = symbol_stride;
            v.out_idx = pa.pout;
            v.ltab = c->d_ltab;
            v.idx = pa.pidx;
            v.ids = c->d_ids + c0;
            v.ps_kr = pa.kr;
            v.ps_in = in_stride;
            v.ps_out = out_stride;
            v.ps_idx = idx_stride;
            // masked fixed pass: the erased slots read as zero, the solve yields them; plain pass: the solve yields
            // g + c for old contents g, XORed into the slots
            v.xor_dst = c->syn->xj->masked ? 0 : 1;
#ifdef RS_AMD_DIAG
            v.ablate = c->m8_ps_ablate & 3;
#endif
            v.stamps = c->stamps;  // diagnostic builds, m8_ps_kernel 7
            v.src_bytes = cn * per;
            // the coordinate-output pass pairs only with the prefetching solve on coordinate inputs (14)
            const int kern = c->syn->xj->coord ? 14 : pf ? c->m8_ps_kernel : c->m8_ps_kernel >= 9 ? 0 : c->m8_ps_kernel;
            if (c->syn->xj->coord && !pf) return RS_ERR_INVALID;  // not reached: the route needs whole 2 KiB chunks
            HIP_TRY(launch_apply_m8_ps(v, cn, int64_t(S), tiles, st, kern, c->m8_ps_cpb));
            RS_CHECKPOINT(c, c->syn.get(), "per-stripe GF(256) solve (apply_m8_ps, syndrome / re-encode route)", uint64_t(cn), S);
            if (ovl) HIP_TRY(hipEventRecord(c->ps_ev_used[set], st));
        }
        c->last_kernel = std::string(c->syn_route == 2 ? "reenc_xj" : "syn_xj") + (pf ? "+apply_m8_pf" : "+apply_m8_v1_ps") +
                         (ovl ? "(overlap)" : "");
        return scratch_release(c, st);
    }
    for (int64_t c0 = 0; c0 < nsel; c0 += chunk) {
        const int64_t cn = std::min(chunk, nsel - c0);
        PlanArgs pa{};
        pa.masks = static_cast<const uint8_t*>(c->d_masks) + size_t(c0) * n;
        pa.elem = c->d_elem;
        pa.logt = logt;
        pa.g8 = g8;
        pa.k = c->k;
        pa.r = c->r;
        pa.n = int32_t(n);
        pa.kr = static_cast<int32_t*>(c->d_kr);
        pa.pin = static_cast<int32_t*>(c->d_pin);
        pa.pout = static_cast<int32_t*>(c->d_pout);
        pa.pidx = static_cast<uint32_t*>(c->d_pidx);
        pa.in_stride = in_stride;
        pa.out_stride = out_stride;
        pa.idx_stride = idx_stride;
        HIP_TRY(launch_plan_m8(pa, cn, st));
        V1Args v{};
        v.src = base;
        v.src_stripe = stripe_stride;
        v.src_sym = symbol_stride;
        v.in_idx = pa.pin;
        v.dst = base;
        v.dst_stripe = stripe_stride;
        v.dst_sym = symbol_stride;
        v.out_idx = pa.pout;
        v.ltab = c->d_ltab;
        v.idx = pa.pidx;
        v.ids = c->d_ids + c0;
        v.ps_kr = pa.kr;
        v.ps_in = in_stride;
        v.ps_out = out_stride;
        v.ps_idx = idx_stride;
        // survivor plans carry the 64-dword records: the prefetching solve (9) does not take them
        HIP_TRY(launch_apply_m8_ps(v, cn, int64_t(S), tiles, st, c->m8_ps_kernel >= 9 ? 0 : c->m8_ps_kernel,
                                   c->m8_ps_cpb));
        RS_CHECKPOINT(c, nullptr, "per-stripe GF(256) survivor plans (apply_m8_ps)", uint64_t(cn), S);
    }
    c->last_kernel = "apply_m8_v1_ps";
    return scratch_release(c, st);
}

// rsg_decode_batch, GF(2^16) codes past kHostPlanGroups patterns: the codec's one batch plan is rebuilt
// on the stream for every pattern by k_plan16_sums / k_plan16_fill -- the same evaluation and formats as
// build_plan_m16_device, so results are identical -- instead of a cached plan per pattern (allocations,
// synchronous uploads and, past 16 patterns, an eviction that frees device memory). Launches on one
// stream are ordered, so the plan of the next pattern is written after the previous apply has read it;
// only the host staging needs a ring (two pinned buffers, each guarded by the event after its copies).
size_t al16(size_t v) { return (v + 15) & ~size_t(15); }

int batch_plan_m16(rsg_codec_t* c, const bool* er, int slot, hipStream_t st, DevPlan** out) {
    const Field& F = field();
    const size_t n = size_t(c->k) + c->r, r = c->r;
    std::vector<uint16_t> targets, sources;
    std::vector<int> emit;
    std::vector<int32_t> in, outs;
    codec_lists(c->positions, c->k, c->r, er, targets, emit, sources, in, outs);
    const int K = int(sources.size()), R = int(emit.size()), d = int(targets.size());
    if (R == 0 || size_t(K) > n || size_t(d) > r) return RS_ERR_INVALID;
    const size_t o_x = al16(n * 2), o_emit = o_x + al16(r * 2), o_lp = o_emit + al16(r * 4), o_ld = o_lp + al16(n * 4);
    const size_t dev_bytes = o_ld + al16(r * 4);
    const size_t o_in = o_lp, o_out = o_in + al16((n + 16) * 4), host_bytes = o_out + al16((r + 64) * 4);
    const size_t rec_cap = ((r + 63) / 64) * (n + 1) * 256;
    if (!c->bp16) {
        auto p = std::make_unique<DevPlan>();
        p->device = c->device;
        p->m = 16;
        HIP_TRY(hipMalloc(reinterpret_cast<void**>(&p->d_coef), (r + 64) * n * 2));
        HIP_TRY(hipMalloc(reinterpret_cast<void**>(&p->d_in), (n + 16) * 4));
        HIP_TRY(hipMalloc(reinterpret_cast<void**>(&p->d_out), (r + 64) * 4));
        if (!c->d_bp16) HIP_TRY(hipMalloc(&c->d_bp16, dev_bytes));
        if (!c->d_bp16_rec && rec_cap <= (size_t(256) << 20)) HIP_TRY(hipMalloc(&c->d_bp16_rec, rec_cap));
        for (int i = 0; i < 2; ++i) {
            if (!c->h_bp16[i])
                HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&c->h_bp16[i]), host_bytes, hipHostMallocDefault));
            if (!c->bp16_ev[i]) HIP_TRY(hipEventCreateWithFlags(&c->bp16_ev[i], hipEventDisableTiming));
        }
        c->bp16 = std::move(p);
    }
    DevPlan& p = *c->bp16;
    p.K = K;
    p.R = R;
    p.rt = apply_tile_rows(16, R);
    p.ntiles = (R + p.rt - 1) / p.rt;
    const size_t coef_bytes = size_t(p.ntiles) * size_t(K) * size_t(p.rt / 2) * 4;
    const size_t rec_bytes = size_t(p.ntiles) * size_t(K + 1) * 256;
    const bool records = p.rt == 64 && c->d_bp16_rec && rec_bytes <= (size_t(256) << 20);
    p.d_idx = records ? static_cast<uint32_t*>(c->d_bp16_rec) : nullptr;
    p.in_slots = in;
    p.out_slots = outs;
    p.out_slots.resize(std::max(size_t(p.ntiles) * p.rt, size_t((R + 31) / 32) * 32), 0);
    p.uses = 0;
    // stage the lists (the copies that last used this buffer are complete once its event is)
    if (c->bp16_rec_pending[slot]) HIP_TRY(hipEventSynchronize(c->bp16_ev[slot]));
    uint8_t* h = c->h_bp16[slot];
    uint16_t* hy = reinterpret_cast<uint16_t*>(h);
    uint16_t* hx = reinterpret_cast<uint16_t*>(h + o_x);
    int32_t* he = reinterpret_cast<int32_t*>(h + o_emit);
    int32_t* hin = reinterpret_cast<int32_t*>(h + o_in);
    int32_t* hout = reinterpret_cast<int32_t*>(h + o_out);
    for (int q = 0; q < K; ++q) hy[q] = F.exp[sources[size_t(q)]];
    for (int e = 0; e < d; ++e) hx[e] = F.exp[targets[size_t(e)]];
    for (int j = 0; j < R; ++j) he[j] = emit[size_t(j)];
    for (int q = 0; q < K + 16; ++q) hin[q] = q < K ? in[size_t(q)] : 0;
    for (size_t j = 0; j < p.out_slots.size(); ++j) hout[j] = p.out_slots[j];
    HIP_TRY(hipMemcpyAsync(c->d_bp16, h, o_lp, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(p.d_in, hin, size_t(K + 16) * 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(p.d_out, hout, p.out_slots.size() * 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipEventRecord(c->bp16_ev[slot], st));
    c->bp16_rec_pending[slot] = true;
    HIP_TRY(hipMemsetAsync(p.d_coef, 0, coef_bytes, st));
    if (records) HIP_TRY(hipMemsetAsync(p.d_idx, 0, rec_bytes, st));
    const uint16_t *logt = nullptr, *expt = nullptr;
    const uint8_t* g8 = nullptr;
    if (int rc = plan_tables(c->device, &logt, &g8, &expt)) return rc;
    uint8_t* dt = static_cast<uint8_t*>(c->d_bp16);
    Plan16Args a{};
    a.src_el = reinterpret_cast<const uint16_t*>(dt);
    a.tgt_el = reinterpret_cast<const uint16_t*>(dt + o_x);
    a.emit = reinterpret_cast<const int32_t*>(dt + o_emit);
    a.logt = logt;
    a.expt = expt;
    a.lp = reinterpret_cast<uint32_t*>(dt + o_lp);
    a.ld = reinterpret_cast<uint32_t*>(dt + o_ld);
    a.coef = p.d_coef;
    a.rec = records ? reinterpret_cast<uint8_t*>(p.d_idx) : nullptr;
    a.K = K;
    a.d = d;
    a.R = R;
    a.rt = p.rt;
    HIP_TRY(launch_plan_m16(a, st));
    *out = &p;
    return 0;
}

// rsg_decode_batch, GF(2^16) codes with per-stripe patterns: the reference's decode split
// (reed_solomon.c:527-549) into its pattern-independent part -- the syndromes S_j (j < D, D = the largest
// t of the batch) of all k + r slots of every stripe, one k_cs16 pass with a fixed plan (cached per D) --
// and the per-pattern part: each stripe's t_info x t solve W (k_plan16_ps / k_plan16_ps_rec build it on
// the device from the stripe's mask, straight into k_apply_m16_v1 records), applied to that stripe's
// first t syndromes by k_apply_m16_v1 in per-stripe mode. Erased information slots are zeroed first (the
// syndromes read every slot); garbage in an erased repair slot only shifts that slot's own unknown,
// which is never written.
bool ps16_eligible(const rsg_codec_t* c, uint64_t S, int64_t stripe_stride, int64_t symbol_stride,
                   const void* base) {
    const int64_t n = int64_t(c->k) + c->r;
    return c->m > 8 && c->m16_ps && c->r <= kPs16MaxR && S % 1024 == 0 && int64_t(S) < (int64_t(1) << 31) &&
           (n - 1) * symbol_stride + int64_t(S) < (int64_t(1) << 31) && int64_t(c->r) * int64_t(S) < (int64_t(1) << 31) &&
           (stripe_stride % 16) == 0 && (symbol_stride % 16) == 0 && (uintptr_t(base) % 16) == 0 &&
           symbol_stride >= int64_t(S);
}

int ps16_syn_plan(rsg_codec_t* c, int D, hipStream_t st, DevPlan** out) {
    auto it = c->ps_syn.find(D);
    if (it == c->ps_syn.end()) {
        if (c->ps_syn.size() >= 4) {  // small LRU: batches usually share a few D values
            const int old = c->ps_syn_lru.front();
            c->ps_syn_lru.erase(c->ps_syn_lru.begin());
            auto o = c->ps_syn.find(old);
            if (o != c->ps_syn.end()) {
                o->second->guard_before_release(st);
                c->ps_syn.erase(o);
            }
        }
        const int n = int(c->k) + c->r;
        std::vector<int32_t> all(static_cast<size_t>(n));
        for (int i = 0; i < n; ++i) all[size_t(i)] = i;
        auto p = std::make_unique<DevPlan>();
        p->device = c->device;
        p->m = 16;
        p->K = n;
        p->R = D;
        p->in_slots = all;
        if (int rc = build_cs16(*p, c->positions, all, D, st)) return rc;
        it = c->ps_syn.emplace(D, std::move(p)).first;
    } else {
        c->ps_syn_lru.erase(std::find(c->ps_syn_lru.begin(), c->ps_syn_lru.end(), D));
    }
    c->ps_syn_lru.push_back(D);
    *out = it->second.get();
    return 0;
}

// m16_ps 2 (or 3 for patterns near r): the re-encode variant below, when the codec's encode is the GF(2^16)
// route (run_cs) and its launches fit (31-bit offsets over the information slots and the r fixed-pass rows)
bool ps16_reenc_eligible(const rsg_codec_t* c, int tmax, int64_t symbol_stride, uint64_t S) {
    // 3 (default): when the syndrome route would compute at least 13/16 r syndromes -- at C5 (256 stripes,
    // t erasures anywhere) the two cross between t = 768 (20.1 vs 21.2 ms) and t = 1024 (29.5 vs 26.2 ms)
    const int D = std::min<int>(c->r, (tmax + 31) / 32 * 32);
    const bool want = c->m16_ps == 2 || (c->m16_ps == 3 && 16 * D >= 13 * c->r);
    const DevPlan* E = c->enc.get();
    return want && E && E->cs && E->cs->kind == 0 && E->second && E->second->cs &&
           E->cs->max_slot * symbol_stride + int64_t(S) < (int64_t(1) << 31) &&
           int64_t(E->cs->D) * int64_t(S) < (int64_t(1) << 31) && int64_t(c->r) * int64_t(S) < (int64_t(1) << 31);
}

// The re-encode variant (option m16_ps 2): the pattern-independent part is the codec's encode route over
// the information slots of a contiguous range of stripes (erased ones zeroed first), + the received repair
// rows (launch_xor_rows), i.e. S' = [G | I] rcv, which run_reenc uses for one pattern; the per-pattern part
// is each stripe's t_info x t_info Cauchy solve W' from its first t_info surviving repair rows (k_plan16_reenc*,
// see rs_kernels.hip), applied by k_apply_m16_v1 in per-stripe mode. Against the syndrome route: the fixed
// pass reads k instead of k + r slots, the solve t_info instead of t inputs, and W' has a closed form (no
// synthetic division). ids: the selected stripes (ascending), sel_masks their masks.
int decode_batch_m16_ps_reenc(rsg_codec_t* c, uint8_t* base, int64_t stripe_stride, int64_t symbol_stride,
                              uint64_t S, const std::vector<int32_t>& ids, const uint8_t* sel_masks, int rmax,
                              hipStream_t st) {
    const int64_t k = c->k, r = c->r, n = k + r;
    DevPlan& E = *c->enc;
    int rc = 0;
    if ((rc = E.order_after_build(st))) return rc;  // its records are read directly (run_cs)
    if ((rc = scratch_acquire(c, st))) return rc;
    const uint16_t *logt = nullptr, *expt = nullptr;
    const uint8_t* g8 = nullptr;
    if ((rc = plan_tables(c->device, &logt, &g8, &expt))) return rc;
    if (!c->d_elem) {
        const Field& F = field();
        std::vector<uint16_t> el(static_cast<size_t>(n));
        for (int64_t i = 0; i < n; ++i) el[size_t(i)] = F.exp[c->positions[size_t(i)]];
        if ((rc = upload(reinterpret_cast<void**>(&c->d_elem), el.data(), size_t(n) * 2))) return rc;
    }
    const int64_t nsel = int64_t(ids.size());
    const int tiles = (rmax + 63) / 64;
    const int64_t out_stride = int64_t(tiles) * 64, in_stride = out_stride + 16;
    const int64_t rec_stride = int64_t(tiles) * (rmax + 1) * 64;  // dwords
    const int64_t per = r * int64_t(S);                            // fixed-pass bytes per stripe
    // chunks of selected stripes: at most m16_ps_rec_mib of records, and a stripe range (the fixed pass runs
    // over every stripe of it) of at most 1 GiB of fixed-pass output
    const int64_t cap_sel = std::max<int64_t>(
        1, std::min<int64_t>({(int64_t(c->ps_rec_mib) << 20) / (rec_stride * 4), 65535,
                              c->ps_chunk > 0 ? c->ps_chunk : int64_t(1) << 40}));
    const int64_t cap_range = std::max<int64_t>(1, (int64_t(1) << 30) / per);
    std::vector<std::pair<int64_t, int64_t>> chunks;  // [i0, i1) of ids
    for (int64_t i0 = 0; i0 < nsel;) {
        int64_t i1 = i0 + 1;
        while (i1 < nsel && i1 - i0 < cap_sel && ids[size_t(i1)] - ids[size_t(i0)] < cap_range) ++i1;
        chunks.emplace_back(i0, i1);
        i0 = i1;
    }
    int64_t chunk = 0, range = 0;
    for (auto& ch : chunks) {
        chunk = std::max(chunk, ch.second - ch.first);
        range = std::max<int64_t>(range, ids[size_t(ch.second - 1)] - ids[size_t(ch.first)] + 1);
    }
    auto al = [](int64_t b) { return (b + 255) / 256 * 256; };
    const int64_t o_kr = 0, o_ee = al(chunk * 8), o_pe = o_ee + al(chunk * r * 2),
                  o_po = o_pe + al(chunk * out_stride * 2), o_qe = o_po + al(chunk * out_stride * 4),
                  o_pi = o_qe + al(chunk * in_stride * 2), o_lq = o_pi + al(chunk * in_stride * 4),
                  o_lr = o_lq + al(chunk * in_stride * 4), small = o_lr + al(chunk * out_stride * 4);
    size_t ids_bytes = c->ids_cap * 4;
    rc = grow(reinterpret_cast<void**>(&c->d_ids), ids_bytes, ids.size() * 4);
    c->ids_cap = ids_bytes / 4;
    if (rc) return rc;
    if ((rc = grow(&c->d_masks, c->masks_cap, size_t(nsel * n)))) return rc;
    if ((rc = grow(&c->d_reenc, c->reenc_cap, size_t(range * per)))) return rc;
    const int64_t rec_set = al(chunk * rec_stride * 4);
    if ((rc = grow(&c->d_ps_rec, c->ps_rec_cap, size_t(2 * rec_set)))) return rc;
    if ((rc = grow(&c->d_ps_small, c->ps_small_cap, size_t(2 * small)))) return rc;
    if (!c->ps_side) HIP_TRY(hipStreamCreateWithFlags(&c->ps_side, hipStreamNonBlocking));
    for (hipEvent_t* e : {&c->ps_ev_zero[0], &c->ps_ev_zero[1], &c->ps_ev_plan[0], &c->ps_ev_plan[1]})
        if (!*e) HIP_TRY(hipEventCreateWithFlags(e, hipEventDisableTiming));
    if ((rc = stage_lists(c, st, {{c->d_ids, ids.data(), ids.size() * 4}, {c->d_masks, sel_masks, size_t(nsel * n)}})))
        return rc;
    Ps16Args pa{};
    pa.elem = c->d_elem;
    pa.logt = logt;
    pa.expt = expt;
    pa.k = c->k;
    pa.r = c->r;
    pa.n = int32_t(n);
    pa.out_stride = out_stride;
    pa.in_stride = in_stride;
    pa.rec_stride = rec_stride;
    pa.tblocks = (tiles + 3) / 4;
    pa.lblocks = (2 * rmax + 255) / 256;
    pa.base = base;
    pa.stripe_stride = stripe_stride;
    pa.symbol_stride = symbol_stride;
    pa.S = int64_t(S);
    uint8_t* y = static_cast<uint8_t*>(c->d_reenc);
    std::string fixed;
    for (size_t ci = 0; ci < chunks.size(); ++ci) {
        const int64_t i0 = chunks[ci].first, cn = chunks[ci].second - i0;
        const int64_t s0 = ids[size_t(i0)], ns = ids[size_t(i0 + cn - 1)] - s0 + 1;
        const int set = int(ci & 1);
        uint8_t* sm = static_cast<uint8_t*>(c->d_ps_small) + set * small;
        pa.kr = reinterpret_cast<int32_t*>(sm + o_kr);
        pa.ee = reinterpret_cast<uint16_t*>(sm + o_ee);
        pa.pe = reinterpret_cast<uint16_t*>(sm + o_pe);
        pa.pout = reinterpret_cast<int32_t*>(sm + o_po);
        pa.qe = reinterpret_cast<uint16_t*>(sm + o_qe);
        pa.pin = reinterpret_cast<int32_t*>(sm + o_pi);
        pa.lq = reinterpret_cast<uint32_t*>(sm + o_lq);
        pa.lr = reinterpret_cast<uint32_t*>(sm + o_lr);
        pa.rec = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(c->d_ps_rec) + set * rec_set);
        pa.masks = static_cast<const uint8_t*>(c->d_masks) + size_t(i0) * size_t(n);
        pa.ids = c->d_ids + i0;
        // lists + zeroing on st (after chunk ci - 2's apply, which read the same set, and ahead of the fixed
        // pass, whose first kernels then do not queue behind the side stream's wide log-sum grid); the log
        // sums and records on the side stream, beside the fixed pass (its wait on ev_zero orders it after
        // everything earlier on st, chunk ci - 2's apply included)
        HIP_TRY(launch_plan16_reenc(pa, cn, st));
        HIP_TRY(hipEventRecord(c->ps_ev_zero[set], st));
        HIP_TRY(hipStreamWaitEvent(c->ps_side, c->ps_ev_zero[set], 0));
        HIP_TRY(launch_plan16_reenc_rec(pa, cn, c->ps_side));
        HIP_TRY(hipEventRecord(c->ps_ev_plan[set], c->ps_side));
        // the fixed pass over the stripe range, + the received repair rows
        uint8_t* b = base + s0 * stripe_stride;
        if ((rc = run_cs(c, E, b, stripe_stride, symbol_stride, y, per, int64_t(S), uint64_t(ns), S, st))) return rc;
        fixed = c->last_kernel;
        HIP_TRY(launch_xor_rows(y, per, int64_t(S), b + k * symbol_stride, stripe_stride, symbol_stride, r, int64_t(S),
                                ns, st));
        HIP_TRY(hipStreamWaitEvent(st, c->ps_ev_plan[set], 0));
        V1Args v{};
        // stripe ids index the range's rows: stripe s at y + (s - s0) * per (the base itself is never read)
        v.src = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(y) - uintptr_t(s0 * per));
        v.src_stripe = per;
        v.src_sym = int64_t(S);
        v.in_idx = pa.pin;
        v.dst = base;
        v.dst_stripe = stripe_stride;
        v.dst_sym = symbol_stride;
        v.out_idx = pa.pout;
        v.idx = pa.rec;
        v.ids = c->d_ids + i0;
        v.ps_kr = pa.kr;
        v.ps_in = in_stride;
        v.ps_out = out_stride;
        v.ps_idx = rec_stride;
        v.K = rmax;
        v.R = rmax;
        HIP_TRY(launch_apply_m16_ps(v, cn, int64_t(S), tiles, st));
        RS_CHECKPOINT(c, &E, "per-stripe GF(2^16) re-encode solve (apply_m16_ps)", uint64_t(cn), S);
    }
    if ((rc = E.note_use(st))) return rc;
    c->last_kernel = "ps16r+" + fixed + "+xor+apply_m16_v1_ps";
    return scratch_release(c, st);
}

// tr: per stripe, t (erasures) and R (erased information slots), counted by rsg_decode_batch
int decode_batch_m16_ps(rsg_codec_t* c, uint8_t* base, int64_t stripe_stride, int64_t symbol_stride,
                        uint64_t n_stripes, uint64_t S, const bool* is_erased, const int32_t* tr,
                        hipStream_t st) {
    const size_t n = size_t(c->k) + c->r;
    std::vector<int32_t> ids;
    std::vector<uint8_t> masks;
    int tmax = 0, rmax = 0;
    for (uint64_t s = 0; s < n_stripes; ++s) {
        const int t = tr[2 * s], R = tr[2 * s + 1];
        if (!R) continue;
        tmax = std::max(tmax, t);
        rmax = std::max(rmax, R);
        ids.push_back(int32_t(s));
    }
    if (ids.empty()) return 0;
    // the selected stripes' masks: the caller's array itself when every stripe is selected
    const uint8_t* mask_src = reinterpret_cast<const uint8_t*>(is_erased);
    if (ids.size() != n_stripes) {
        masks.resize(ids.size() * n);
        for (size_t i = 0; i < ids.size(); ++i)
            std::memcpy(masks.data() + i * n, is_erased + size_t(ids[i]) * n, n);
        mask_src = masks.data();
    }
    if (ps16_reenc_eligible(c, tmax, symbol_stride, S))
        return decode_batch_m16_ps_reenc(c, base, stripe_stride, symbol_stride, S, ids, mask_src, rmax, st);
    int rc = scratch_acquire(c, st);
    if (rc) return rc;
    const uint16_t *logt = nullptr, *expt = nullptr;
    const uint8_t* g8 = nullptr;
    if ((rc = plan_tables(c->device, &logt, &g8, &expt))) return rc;
    if (!c->d_elem) {
        const Field& F = field();
        std::vector<uint16_t> el(n);
        for (size_t i = 0; i < n; ++i) el[i] = F.exp[c->positions[i]];
        if ((rc = upload(reinterpret_cast<void**>(&c->d_elem), el.data(), n * 2))) return rc;
    }
    // D: the batch's largest t rounded up to a multiple of 32 (fewer distinct cached syndrome plans)
    const int D = std::min<int>(c->r, (tmax + 31) / 32 * 32);
    DevPlan* syn = nullptr;
    if ((rc = ps16_syn_plan(c, D, st, &syn))) return rc;
    if ((rc = syn->order_after_build(st))) return rc;
    const DevPlan::Cs& cs = *syn->cs;
    const int64_t nsel = int64_t(ids.size());
    const int tiles = (rmax + 63) / 64;
    const int64_t out_stride = int64_t(tiles) * 64;
    const int64_t rec_stride = int64_t(tiles) * (D + 1) * 64;  // dwords
    const int64_t per = int64_t(D) * int64_t(S);                // syndrome bytes per stripe
    // chunks of stripes, at most m16_ps_rec_mib of records each: larger chunks measured faster (C5, 256
    // stripes: 48 MiB 0.260, 160 MiB 0.204, 1024 MiB 0.184 ms a stripe; option m16_ps_chunk caps it)
    int64_t chunk = std::max<int64_t>(
        1, std::min<int64_t>({nsel, (int64_t(1) << 30) / per, (int64_t(c->ps_rec_mib) << 20) / (rec_stride * 4), 65535}));
    if (c->ps_chunk > 0) chunk = std::min<int64_t>(chunk, c->ps_chunk);
    const int64_t nchunk = (nsel + chunk - 1) / chunk;
    chunk = (nsel + nchunk - 1) / nchunk;  // even chunks (no small tail chunk)
    // small per-stripe arrays in one buffer: kr [2] i32, ee [r] u16, pe [out_stride] u16, pout
    // [out_stride] i32, cf [r + 1] u16 (each part 256-byte aligned)
    auto al = [](int64_t b) { return (b + 255) / 256 * 256; };
    const int64_t o_kr = 0, o_ee = al(chunk * 8), o_pe = o_ee + al(chunk * c->r * 2),
                  o_po = o_pe + al(chunk * out_stride * 2), o_cf = o_po + al(chunk * out_stride * 4),
                  small = o_cf + al(chunk * (int64_t(c->r) + 1) * 2);
    size_t ids_bytes = c->ids_cap * 4;
    rc = grow(reinterpret_cast<void**>(&c->d_ids), ids_bytes, ids.size() * 4);
    c->ids_cap = ids_bytes / 4;
    if (rc) return rc;
    if ((rc = grow(&c->d_masks, c->masks_cap, ids.size() * n))) return rc;
    const bool ovl = c->ps_overlap && nchunk > 1;
    if ((rc = grow(&c->d_cs, c->cs_cap, size_t((ovl ? 2 : 1) * chunk * per)))) return rc;
    // two sets of plan buffers: chunk i + 1's plans are built on the side stream while chunk i runs
    const int64_t rec_set = al(chunk * rec_stride * 4);
    if ((rc = grow(&c->d_ps_rec, c->ps_rec_cap, size_t(2 * rec_set)))) return rc;
    if ((rc = grow(&c->d_ps_small, c->ps_small_cap, size_t(2 * small)))) return rc;
    if (!c->ps_side) HIP_TRY(hipStreamCreateWithFlags(&c->ps_side, hipStreamNonBlocking));
    if (ovl && !c->ps_synst) HIP_TRY(hipStreamCreateWithFlags(&c->ps_synst, hipStreamNonBlocking));
    for (hipEvent_t* e : {&c->ps_ev_entry, &c->ps_ev_zero[0], &c->ps_ev_zero[1], &c->ps_ev_plan[0], &c->ps_ev_plan[1],
                          &c->ps_ev_used[0], &c->ps_ev_used[1], &c->ps_ev_syn[0], &c->ps_ev_syn[1]})
        if (!*e) HIP_TRY(hipEventCreateWithFlags(e, hipEventDisableTiming));
    const int ngo = (cs.ngroups + 3) * 16;
    if ((rc = grow(&c->d_goff[0], c->goff_cap[0], size_t(ngo) * 4))) return rc;
    if ((rc = stage_lists(c, st, {{c->d_ids, ids.data(), ids.size() * 4}, {c->d_masks, mask_src, ids.size() * n}})))
        return rc;
    HIP_TRY(launch_cs16_goff(cs.groups, static_cast<uint32_t*>(c->d_goff[0]), ngo, symbol_stride, st));
    Ps16Args pa{};
    pa.elem = c->d_elem;
    pa.logt = logt;
    pa.expt = expt;
    pa.k = c->k;
    pa.r = c->r;
    pa.n = int32_t(n);
    pa.out_stride = out_stride;
    pa.rec_stride = rec_stride;
    pa.tblocks = (tiles + 3) / 4;
    pa.base = base;
    pa.stripe_stride = stripe_stride;
    pa.symbol_stride = symbol_stride;
    pa.S = int64_t(S);
    Cs16Args ca{};
    ca.src = base;
    ca.src_stripe = stripe_stride;
    ca.src_sym = symbol_stride;
    ca.goff = static_cast<const uint32_t*>(c->d_goff[0]);
    ca.in_bytes = uint32_t(cs.max_slot * symbol_stride + int64_t(S));
    const bool thr = c->m16_cs_thread && cs.rec_t;
    ca.rec = thr ? cs.rec_t : cs.rec;
    ca.fin = thr ? cs.fin_t : cs.fin;
    ca.fin_off = thr ? cs.fin_off_t : cs.fin_off;
    ca.fin_stride = thr ? cs.fin_stride_t : cs.fin_stride;
    ca.cw = thr ? kCs16tCw : 4;
    ca.dst_stripe = per;
    ca.dst_sym = int64_t(S);
    ca.logt = logt;
    ca.expt = expt;
    for (int q = 0; q < 16; ++q) ca.nblog[q] = cs.nblog[q];
    ca.ngroups = cs.ngroups;
    ca.ntiles = thr ? cs.ntiles_t : cs.ntiles;
    ca.colw = c->m16_cs_col == 1024 ? 1024 : 256;
    ca.nchunks = int64_t(S) / ca.colw;
    if (!c->d_ps_in) {  // the apply's shared input list: input j = syndrome j of the stripe (j < r, + padding)
        std::vector<int32_t> in_list(size_t(c->r) + 16);
        for (size_t j = 0; j < in_list.size(); ++j) in_list[j] = int32_t(j);
        if ((rc = upload(reinterpret_cast<void**>(&c->d_ps_in), in_list.data(), in_list.size() * 4))) return rc;
    }
    // the side stream starts after the caller's earlier work on st (the plans zero erased slots)
    HIP_TRY(hipEventRecord(c->ps_ev_entry, st));
    HIP_TRY(hipStreamWaitEvent(c->ps_side, c->ps_ev_entry, 0));
    // overlap: the syndrome passes on their own stream into two buffers, chunk ci's after chunk ci - 2's solve
    // has read the same buffer; the solve of chunk ci waits for its syndromes and its records
    hipStream_t sy = ovl ? c->ps_synst : st;
    if (ovl) HIP_TRY(hipStreamWaitEvent(sy, c->ps_ev_entry, 0));
    for (int64_t c0 = 0, ci = 0; c0 < nsel; c0 += chunk, ++ci) {
        const int64_t cn = std::min(chunk, nsel - c0);
        const int set = int(ci & 1);
        uint8_t* sm = static_cast<uint8_t*>(c->d_ps_small) + set * small;
        pa.kr = reinterpret_cast<int32_t*>(sm + o_kr);
        pa.ee = reinterpret_cast<uint16_t*>(sm + o_ee);
        pa.pe = reinterpret_cast<uint16_t*>(sm + o_pe);
        pa.pout = reinterpret_cast<int32_t*>(sm + o_po);
        pa.cf = reinterpret_cast<uint16_t*>(sm + o_cf);
        pa.rec = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(c->d_ps_rec) + set * rec_set);
        pa.masks = static_cast<const uint8_t*>(c->d_masks) + size_t(c0) * n;
        pa.ids = c->d_ids + c0;
        // plans of this chunk on the side stream, once chunk ci - 2 (same buffer set) has been applied
        if (ci >= 2) HIP_TRY(hipStreamWaitEvent(c->ps_side, c->ps_ev_used[set], 0));
        HIP_TRY(launch_plan16_ps(pa, cn, c->ps_side));
        HIP_TRY(hipEventRecord(c->ps_ev_zero[set], c->ps_side));
        HIP_TRY(launch_plan16_ps_rec(pa, cn, c->ps_side));  // runs beside this chunk's syndrome pass
        HIP_TRY(hipEventRecord(c->ps_ev_plan[set], c->ps_side));
        // syndromes (after the zeroing: they read every slot), then the apply (after the records)
        HIP_TRY(hipStreamWaitEvent(sy, c->ps_ev_zero[set], 0));
        if (ovl && ci >= 2) HIP_TRY(hipStreamWaitEvent(sy, c->ps_ev_used[set], 0));
        uint8_t* csb = static_cast<uint8_t*>(c->d_cs) + (ovl ? set * chunk * per : 0);
        ca.dst = csb;
        ca.ids = c->d_ids + c0;
        ca.units = cn * ca.nchunks;
        const uint64_t steps = uint64_t(ca.units) * uint64_t(ca.colw / 256) * uint64_t(ca.ntiles) * uint64_t(cs.ngroups);
        if (thr) {
            HIP_TRY(launch_cs16t(ca, sy));
            c->work_valu += uint64_t(ca.units) * uint64_t(ca.colw / 256) * cs.valu_t;
            c->work_salu += steps * kSaluStepCs16t;
        } else {
            HIP_TRY(launch_cs16(ca, sy));
            c->work_valu += steps * kValu_cs16a;
            c->work_salu += steps * kSalu_cs16a;
        }
        if (ovl) {
            HIP_TRY(hipEventRecord(c->ps_ev_syn[set], sy));
            HIP_TRY(hipStreamWaitEvent(st, c->ps_ev_syn[set], 0));
        }
        HIP_TRY(hipStreamWaitEvent(st, c->ps_ev_plan[set], 0));
        V1Args v{};
        v.src = csb;
        v.src_stripe = per;
        v.src_sym = int64_t(S);
        v.src_local = 1;
        v.in_idx = c->d_ps_in;
        v.dst = base;
        v.dst_stripe = stripe_stride;
        v.dst_sym = symbol_stride;
        v.out_idx = pa.pout;
        v.idx = pa.rec;
        v.ids = c->d_ids + c0;
        v.ps_kr = pa.kr;
        v.ps_in = 0;
        v.ps_out = out_stride;
        v.ps_idx = rec_stride;
        v.K = D;
        v.R = rmax;
        HIP_TRY(launch_apply_m16_ps(v, cn, int64_t(S), tiles, st));
        RS_CHECKPOINT(c, syn, "per-stripe GF(2^16) syndrome solve (apply_m16_ps)", uint64_t(cn), S);
        HIP_TRY(hipEventRecord(c->ps_ev_used[set], st));
    }
    if ((rc = syn->note_use(st))) return rc;
    c->last_kernel = thr ? "ps16+cs16t+apply_m16_v1_ps" : "ps16+cs16+apply_m16_v1_ps";
    return scratch_release(c, st);
}

}  // namespace rsamd

extern "C" int rsg_decode_batch(rsg_codec_t* c, void* d_rcv, uint64_t stripe_stride, uint64_t symbol_stride,
                                uint64_t n_stripes, uint64_t symbol_size, const bool* is_erased, void* stream) {
    rsamd::CallerDevice caller_device;
    if (!c || (!is_erased && n_stripes)) return RS_ERR_INVALID;
    const size_t n = size_t(c->k) + c->r;
    // validate every stripe first (nothing is written when one pattern cannot be restored), then group
    // the stripes that share a pattern: one plan and one launch (over a stripe-id list) per pattern.
    // Patterns are keyed by a hash and compared byte for byte; groups keep first-occurrence order.
    struct Group {
        const uint8_t* key;
        std::vector<int32_t> ids;
    };
    std::vector<Group> groups;
    std::unordered_map<uint64_t, std::vector<size_t>> by_hash;
    std::vector<int32_t> tr(size_t(n_stripes) * 2);  // per stripe: t, R
    // The groups matter only while a host-plan route can still be taken: once their count passes the
    // point where a device-plan route takes over, the remaining stripes are validated, not grouped
    // (at 4096 all-distinct patterns the hashing and per-group lists were ~0.5 ms of host time).
    const bool dev_m8 = c->m <= 8 && n <= 256 && (c->batch_plans == 1 || c->batch_plans == 2);
    const bool dev_m16 = c->m > 8 && (c->batch_plans == 1 || c->batch_plans == 2) &&
                         ps16_eligible(c, symbol_size, int64_t(stripe_stride), int64_t(symbol_stride), d_rcv);
    const size_t group_cap = (dev_m8 || dev_m16) && c->batch_plans == 1 ? 0
                             : dev_m8                                     ? kHostPlanGroups
                             : dev_m16                                    ? 1
                                                                          : SIZE_MAX;
    for (uint64_t s = 0; s < n_stripes; ++s) {
        const uint8_t* e = reinterpret_cast<const uint8_t*>(is_erased + s * n);
        const size_t R = count_nonzero(e, c->k), t = R + count_nonzero(e + c->k, c->r);
        if (t > c->r) return RS_ERR_CANNOT_RESTORE;
        tr[2 * s] = int32_t(t);
        tr[2 * s + 1] = int32_t(R);
        if (!R) continue;  // nothing to restore (erased repair slots are never written)
        if (s > uint64_t(INT32_MAX)) return RS_ERR_INVALID;
        if (groups.size() > group_cap) continue;
        std::vector<size_t>& cand = by_hash[hash_bytes(e, n)];
        size_t g = 0;
        while (g < cand.size() && std::memcmp(groups[cand[g]].key, e, n)) ++g;
        if (g == cand.size()) {
            cand.push_back(groups.size());
            groups.push_back(Group{e, {}});
        }
        groups[cand[g]].ids.push_back(int32_t(s));
    }
    if (groups.empty() || !symbol_size) return 0;
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (dev_m8 && (c->batch_plans == 1 || groups.size() > kHostPlanGroups))
        return scratch_fence(c, st,
                      decode_batch_device_plans(c, static_cast<uint8_t*>(d_rcv), int64_t(stripe_stride),
                                                int64_t(symbol_stride), n_stripes, symbol_size, is_erased, tr.data(), st));
    // GF(2^16): more than one pattern -> per-stripe plans on the syndrome route (one shared syndrome pass)
    if (dev_m16 && (c->batch_plans == 1 || groups.size() > 1))
        return scratch_fence(c, st,
                      decode_batch_m16_ps(c, static_cast<uint8_t*>(d_rcv), int64_t(stripe_stride),
                                          int64_t(symbol_stride), n_stripes, symbol_size, is_erased, tr.data(), st));
    std::vector<int32_t> ids;
    std::vector<size_t> first;
    for (auto& g : groups) {
        first.push_back(ids.size());
        ids.insert(ids.end(), g.ids.begin(), g.ids.end());
    }
    if (int rc = scratch_acquire(c, st)) return rc;
    // from here on every failure goes through scratch_fence(): group kernels launched before it may still read
    // d_ids, so the scratch is marked busy on st and the next call (on any stream) waits for them
    const int rc = [&]() -> int {
        if (ids.size() > c->ids_cap) {
            if (c->d_ids) (void)hipFree(c->d_ids);
            c->d_ids = nullptr;
            c->ids_cap = 0;
            HIP_TRY(hipMalloc(&c->d_ids, ids.size() * 4));
            c->ids_cap = ids.size();
        }
        if (int e = stage_lists(c, st, {{c->d_ids, ids.data(), ids.size() * 4}})) return e;
        uint8_t* base = static_cast<uint8_t*>(d_rcv);
        // GF(2^16) codes with many patterns: one plan rebuilt on the stream per pattern (batch_plan_m16)
        const bool stream_plans = c->m > 8 && c->m16_plans != 0 &&
                                  (c->batch_plans == 1 || (c->batch_plans == 2 && groups.size() > kHostPlanGroups));
        size_t gi = 0;
        for (auto& g : groups) {
            std::unique_ptr<bool[]> er(new bool[n]);
            uint16_t t = 0;
            for (size_t i = 0; i < n; ++i) t = uint16_t(t + (er[i] = g.key[i] != 0));
            DevPlan* p = nullptr;
#ifdef RS_AMD_DIAG
            if (int64_t(gi) == c->inject_fail_group) return RS_ERR_DEVICE;  // failure injection (tests)
#endif
            int e = stream_plans ? batch_plan_m16(c, er.get(), int(gi & 1), st, &p) : decode_plan(c, er.get(), t, &p, st);
            if (e) return e;
            // a pattern shared by every stripe, in order: no stripe-id list (the GF(2^16) route and the re-encode
            // decode cover only that form)
            const bool all = g.ids.size() == n_stripes && g.ids.front() == 0 && g.ids.back() == int32_t(n_stripes - 1);
            e = run_plan(c, *p, base, int64_t(stripe_stride), int64_t(symbol_stride), base, int64_t(stripe_stride),
                         int64_t(symbol_stride), g.ids.size(), symbol_size, st, all ? nullptr : c->d_ids + first[gi]);
            if (e) return e;
            ++gi;
        }
        return 0;
    }();
    return rc ? scratch_fence(c, st, rc) : scratch_release(c, st);
}

extern "C" int rsg_xj_fixed_precompile(uint16_t k, uint16_t r, int route) {
    if (uint32_t(k) + r > kN || (route != 1 && route != 2)) return RS_ERR_INVALID;
    const std::vector<uint16_t> pos = code_positions(k, r);
    const int n = int(k) + r;
    if (subfield_degree(pos) > 8 || !xj_supported(8, n, r)) return 0;
    std::vector<int32_t> in(static_cast<size_t>(n)), out(static_cast<size_t>(r));
    for (int i = 0; i < n; ++i) in[size_t(i)] = i;
    for (int j = 0; j < r; ++j) out[size_t(j)] = j;
    return xj_precompile(syn_fixed_matrix(pos, k, r, route), n, r, in, out, 1);  // the codec's default form
}

extern "C" int rsg_xj_fixed_source(uint16_t k, uint16_t r, int route, int masked, char* buf, size_t cap, size_t* len) {
    if (uint32_t(k) + r > kN || (route != 1 && route != 2)) return RS_ERR_INVALID;
    const std::vector<uint16_t> pos = code_positions(k, r);
    if (subfield_degree(pos) > 8) return RS_ERR_INVALID;
    const int n = int(k) + r;
    if (!xj_supported(8, n, r)) return RS_ERR_INVALID;
    std::vector<int32_t> in(static_cast<size_t>(n)), out(static_cast<size_t>(r));
    for (int i = 0; i < n; ++i) in[size_t(i)] = i;
    for (int j = 0; j < r; ++j) out[size_t(j)] = j;
    const std::string src = xj_source(syn_fixed_matrix(pos, k, r, route), n, r, in, out, true, masked);
    if (len) *len = src.size();
    if (buf && cap) {
        const size_t m = std::min(cap - 1, src.size());
        std::memcpy(buf, src.data(), m);
        buf[m] = 0;
    }
    return 0;
}
