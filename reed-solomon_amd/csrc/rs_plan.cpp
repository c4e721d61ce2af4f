// rs_plan.cpp -- device plans: per-device constant tables, recycled plan memory (PlanMemPool), the
// packed coding-matrix plans of the apply kernels (host-built build_plan, device-built
// build_plan_m16_device) and the position lists every plan starts from.
#include "rs_core.hpp"

using namespace rsamd;

namespace rsamd {

struct DeviceTables {
    uint32_t* d_ltab = nullptr;  // 3072 dwords, see ApplyArgs::ltab (+ the gamma^4 table of the one-table solves)
    uint16_t* d_log = nullptr;   // [65536] discrete log (device-built plans)
    uint16_t* d_exp = nullptr;   // [65536] alpha^i (entry 65535 = 1)
    uint8_t* d_g8 = nullptr;     // [256] gamma-basis byte of alpha^(257 e), e < 255
};

std::mutex g_dev_mu;
std::map<int, DeviceTables> g_dev;

int device_tables(int device, const uint32_t** out) {
    std::lock_guard<std::mutex> lk(g_dev_mu);
    DeviceTables& t = g_dev[device];
    if (!t.d_ltab) {
        const Gamma8& g = gamma8();
        std::vector<uint32_t> h(3072);
        for (int b = 0; b < 256; ++b) {
            h[b] = g.lbyte[0][b];
            h[256 + b] = g.lbyte[1][b];
            h[512 + b] = uint32_t(g.lbyte[0][b]) << 16;
            h[768 + b] = uint32_t(g.lbyte[1][b]) << 16;
            h[1024 + b] = g.ibyte[0][b];
            h[1280 + b] = g.ibyte[1][b];
            h[1536 + b] = uint32_t(g.ibyte[0][b]) << 16;
            h[1792 + b] = uint32_t(g.ibyte[1][b]) << 16;
        }
        // [2048, 3072): L^-1 of gamma^4 times each coordinate byte (the device's gmul_g4 / V1H_G4 table), so the
        // one-table solves copy it instead of building it per workgroup
        for (int i = 0; i < 1024; ++i) {
            uint32_t v = uint32_t(i & 255);
            for (int j = 0; j < 4; ++j) v = ((v << 1) & 0xFEu) ^ ((v >> 7) * 0x1Du);
            h[2048 + i] = h[1024 + (i & ~255) + v];
        }
        void* p = nullptr;
        HIP_TRY(hipMalloc(&p, h.size() * 4));
        HIP_TRY(hipMemcpy(p, h.data(), h.size() * 4, hipMemcpyHostToDevice));
        t.d_ltab = static_cast<uint32_t*>(p);
    }
    *out = t.d_ltab;
    return 0;
}

// log / gamma-byte tables of the device plan builder (k_plan_m8)
int plan_tables(int device, const uint16_t** logt, const uint8_t** g8, const uint16_t** expt) {
    std::lock_guard<std::mutex> lk(g_dev_mu);
    DeviceTables& t = g_dev[device];
    if (!t.d_log) {
        const Field& F = field();
        const Gamma8& g = gamma8();
        std::vector<uint8_t> gb(256, 0);
        for (uint32_t e = 0; e < 255; ++e) gb[e] = g.coord(F.exp[257u * e]);
        std::vector<uint16_t> ex(65536);
        for (uint32_t e = 0; e < 65536; ++e) ex[e] = F.exp[e % kN];
        void* pl = nullptr;
        void* pe = nullptr;
        void* pg = nullptr;
        HIP_TRY(hipMalloc(&pl, 65536 * 2));
        HIP_TRY(hipMemcpy(pl, F.log, 65536 * 2, hipMemcpyHostToDevice));
        HIP_TRY(hipMalloc(&pe, 65536 * 2));
        HIP_TRY(hipMemcpy(pe, ex.data(), 65536 * 2, hipMemcpyHostToDevice));
        HIP_TRY(hipMalloc(&pg, 256));
        HIP_TRY(hipMemcpy(pg, gb.data(), 256, hipMemcpyHostToDevice));
        t.d_log = static_cast<uint16_t*>(pl);
        t.d_exp = static_cast<uint16_t*>(pe);
        t.d_g8 = static_cast<uint8_t*>(pg);
    }
    *logt = t.d_log;
    *g8 = t.d_g8;
    if (expt) *expt = t.d_exp;
    return 0;
}

// device scratch that only grows (freed with its owner)
int grow(void** p, size_t& cap, size_t bytes) {
    if (bytes <= cap) return 0;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    cap = 0;
    HIP_TRY(hipMalloc(p, std::max<size_t>(bytes, 256)));
    cap = bytes;
    return 0;
}

// Recycled plan memory. A new decode pattern used to cost a hipMalloc + hipHostMalloc for its plan
// and, once the plan cache was full, a hipFree + hipHostFree for the evicted one: calls that
// synchronise with the device or (un)pin pages, ~0.25 ms apiece, more than the launch they serve.
// Released plan buffers go to per-size-class free lists instead: a device buffer together with an
// event recorded after the last launch that used it (handed out again once that event has
// completed), a pinned staging buffer once its upload has completed.
struct PlanMemPool {
    struct Dev {
        void* p;
        int device;
        hipEvent_t guard;  // null: idle
    };
    std::mutex mu;
    std::multimap<size_t, Dev> dev;
    std::multimap<size_t, void*> host;
    size_t dev_bytes = 0, host_bytes = 0;
    static constexpr size_t kDevCap = size_t(512) << 20, kHostCap = size_t(64) << 20;
    static size_t cls(size_t b) {
        size_t c = 4096;
        while (c < b) c <<= 1;
        return c;
    }
};
PlanMemPool& plan_pool() {
    static PlanMemPool* p = new PlanMemPool;  // never destroyed: plans may outlive static destructors
    return *p;
}

int pool_dev_acquire(size_t bytes, int device, void** out, size_t* cap) {
    PlanMemPool& P = plan_pool();
    const size_t c = PlanMemPool::cls(bytes);
    {
        std::lock_guard<std::mutex> lk(P.mu);
        auto range = P.dev.equal_range(c);
        for (auto it = range.first; it != range.second; ++it) {
            if (it->second.device != device) continue;
            if (it->second.guard) {
                const hipError_t q = hipEventQuery(it->second.guard);
                (void)hipGetLastError();  // an ignored status must not surface at the next launch check
                if (q == hipErrorNotReady) continue;  // still in use
                if (q != hipSuccess) {  // unexpected: wait for the last launch the hard way
                    static bool once = false;
                    if (!once) std::fprintf(stderr, "librs_amd: plan pool: event query: %s\n", hipGetErrorString(q));
                    once = true;
                    (void)hipEventSynchronize(it->second.guard);
                    (void)hipGetLastError();
                }
                (void)hipEventDestroy(it->second.guard);
            }
            *out = it->second.p;
            *cap = c;
            P.dev_bytes -= c;
            P.dev.erase(it);
            return 0;
        }
    }
    HIP_TRY(hipMalloc(out, c));
    *cap = c;
    return 0;
}

// takes ownership of guard; the current device is `device`
void pool_dev_release(void* p, size_t cap, int device, hipEvent_t guard) {
    if (!p) return;
    PlanMemPool& P = plan_pool();
    {
        std::lock_guard<std::mutex> lk(P.mu);
        if (P.dev_bytes + cap <= PlanMemPool::kDevCap) {
            P.dev.emplace(cap, PlanMemPool::Dev{p, device, guard});
            P.dev_bytes += cap;
            return;
        }
    }
    if (guard) {
        (void)hipEventSynchronize(guard);
        (void)hipEventDestroy(guard);
    }
    (void)hipFree(p);
    (void)hipGetLastError();
}

int pool_host_acquire(size_t bytes, void** out, size_t* cap) {
    PlanMemPool& P = plan_pool();
    const size_t c = PlanMemPool::cls(bytes);
    {
        std::lock_guard<std::mutex> lk(P.mu);
        auto it = P.host.find(c);
        if (it != P.host.end()) {
            *out = it->second;
            *cap = c;
            P.host_bytes -= c;
            P.host.erase(it);
            return 0;
        }
    }
    HIP_TRY(hipHostMalloc(out, c, hipHostMallocDefault));
    *cap = c;
    return 0;
}

void pool_host_release(void* p, size_t cap) {  // the copies reading p have completed
    if (!p) return;
    PlanMemPool& P = plan_pool();
    {
        std::lock_guard<std::mutex> lk(P.mu);
        if (P.host_bytes + cap <= PlanMemPool::kHostCap) {
            P.host.emplace(cap, p);
            P.host_bytes += cap;
            return;
        }
    }
    (void)hipHostFree(p);
    (void)hipGetLastError();
}

DevPlan::~DevPlan() {
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(device);
    if (ready) {  // the build may still be in flight: its buffers must outlive it
        (void)hipEventSynchronize(ready);
        (void)hipEventDestroy(ready);
    }
    pool_host_release(h_stage, stage_cap);
    if (blob && !multi_stream && recorded != launches) {  // launches past the guard: wait for them
        (void)hipDeviceSynchronize();
        if (used) (void)hipEventDestroy(used);
        used = nullptr;
    } else if (used && hipEventQuery(used) == hipSuccess) {  // last launch done: no guard to carry
        (void)hipEventDestroy(used);
        used = nullptr;
    }
    (void)hipGetLastError();
    if (blob && !multi_stream) {
        // a guard may outlive its stream (a drop-in context's streams die after its codecs): the
        // pool then sees an odd query status and waits on the event before reusing the buffer
        pool_dev_release(blob, blob_cap, device, used);
        used = nullptr;
    } else if (blob) {
        (void)hipFree(blob);
    } else {
        (void)hipFree(d_in);
        (void)hipFree(d_out);
        (void)hipFree(d_coef);
        (void)hipFree(d_idx);
    }
    if (used) (void)hipEventDestroy(used);
    (void)hipSetDevice(cur);
    (void)hipGetLastError();  // teardown statuses are not the next launch's error
}

int upload(void** dst, const void* src, size_t bytes) {
    HIP_TRY(hipMalloc(dst, std::max<size_t>(bytes, 16)));
    if (bytes) HIP_TRY(hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice));
    return 0;
}

int build_plan(int device, int m, std::vector<uint16_t> M, int K, int R, std::vector<int32_t> in_slots,
               std::vector<int32_t> out_slots, std::unique_ptr<DevPlan>& out, hipStream_t st) {
    auto p = std::make_unique<DevPlan>();
    p->device = device;
    p->m = m <= 8 ? 8 : 16;
    p->K = K;
    p->R = R;
    p->rt = apply_tile_rows(p->m, std::max(R, 1));
    p->ntiles = (R + p->rt - 1) / p->rt;
    const int rt = p->rt;
    std::vector<uint32_t> coef;
    if (p->m == 8) {
        const Gamma8& g = gamma8();
        coef.assign(size_t(p->ntiles) * K * (rt / 4), 0);
        for (int t = 0; t < p->ntiles; ++t)
            for (int i = 0; i < K; ++i)
                for (int j = 0; j < rt; ++j) {
                    const int row = t * rt + j;
                    if (row >= R) continue;
                    const uint32_t c = g.coord(M[size_t(row) * K + i]);
                    coef[(size_t(t) * K + i) * (rt / 4) + j / 4] |= c << (8 * (j % 4));
                }
    } else {
        coef.assign(size_t(p->ntiles) * K * (rt / 2), 0);
        for (int t = 0; t < p->ntiles; ++t)
            for (int i = 0; i < K; ++i)
                for (int j = 0; j < rt; ++j) {
                    const int row = t * rt + j;
                    if (row >= R) continue;
                    const uint32_t c = M[size_t(row) * K + i];
                    coef[(size_t(t) * K + i) * (rt / 2) + j / 2] |= c << (16 * (j % 2));
                }
    }
    out_slots.resize(std::max(size_t(p->ntiles) * rt, size_t((R + 31) / 32) * 32), 0);  // padded rows: never stored
    int rc;
    PlanBlob blob;
    size_t o_idx = SIZE_MAX;
    if (p->m == 8) {
        // gpr-index kernels (k_apply_m8_idx / _lds / _v1), 32-row tiles whatever p->rt is: record per
        // (tile, input) = 64 dwords, [j] = low, [32 + j] = high nibble of output j's coefficient
        const Gamma8& g = gamma8();
        const int nt32 = (R + 31) / 32;
        std::vector<uint32_t> idx(size_t(nt32) * K * 64, 0);
        for (int t = 0; t < nt32; ++t)
            for (int i = 0; i < K; ++i)
                for (int j = 0; j < 32 && t * 32 + j < R; ++j) {
                    const uint32_t c = g.coord(M[size_t(t * 32 + j) * K + i]);
                    idx[(size_t(t) * K + i) * 64 + j] = c & 15;
                    idx[(size_t(t) * K + i) * 64 + 32 + j] = c >> 4;
                }
        o_idx = blob.add(idx.data(), idx.size() * 4);
    } else if (rt == 64 && size_t(p->ntiles) * (K + 1) * 256 <= (size_t(256) << 20)) {
        // k_apply_m16_v1: per (tile, input) 256 byte-sized table indices packed in 64 dwords (16 per
        // nibble plane n; output j's index 16n + nibble n in byte (j % 8) / 2 of the plane's dword
        // 2 (j / 8) + j % 2, the order the kernel's s_lshr_b64 extraction walks); one padding record. (One index
        // per dword would save the kernel's byte shifts but quadruples the record stream: measured
        // 13.4 vs 23.6 GB/s at C5.)
        std::vector<uint32_t> idx(size_t(p->ntiles) * (K + 1) * 64, 0);
        for (int t = 0; t < p->ntiles; ++t)
            for (int i = 0; i < K; ++i) {
                uint8_t* rec = reinterpret_cast<uint8_t*>(idx.data() + (size_t(t) * (K + 1) + i) * 64);
                for (int n = 0; n < 4; ++n)
                    for (int j = 0; j < 64; ++j) {  // plane dword 2 (j / 8) + j % 2, byte (j % 8) / 2
                        const int row = t * 64 + j;
                        const uint32_t c = row < R ? M[size_t(row) * K + i] : 0;
                        const int dw = 16 * n + 2 * (j / 8) + (j % 2), by = (j % 8) / 2;
                        rec[4 * dw + by] = uint8_t(16 * n + ((c >> (4 * n)) & 15u));
                    }
            }
        o_idx = blob.add(idx.data(), idx.size() * 4);
    }
    in_slots.resize(in_slots.size() + 16, 0);  // kernels read slot indices in vectors past the end
    const size_t o_in = blob.add(in_slots.data(), in_slots.size() * 4);
    const size_t o_out = blob.add(out_slots.data(), out_slots.size() * 4);
    const size_t o_coef = blob.add(coef.data(), coef.size() * 4);
    if ((rc = blob.upload(*p, st)) || (rc = PlanBlob::finish(*p))) return rc;
    if (o_idx != SIZE_MAX) p->d_idx = PlanBlob::at<uint32_t>(*p, o_idx);
    p->d_in = PlanBlob::at<int32_t>(*p, o_in);
    p->d_out = PlanBlob::at<int32_t>(*p, o_out);
    p->d_coef = PlanBlob::at<uint32_t>(*p, o_coef);
    p->matrix = std::move(M);
    in_slots.resize(size_t(K));
    p->in_slots = std::move(in_slots);
    p->out_slots = std::move(out_slots);
    out = std::move(p);
    return 0;
}

// ============================================================================ codec
// m = 16 plan built on the device (k_plan16_*): same kernels' formats as build_plan, from the target
// / source position lists instead of a host matrix (a C5 decode plan is 4M coefficients and 16 MiB of
// index records: tens of ms on the host, well under one on the GPU). Synchronous, like build_plan.
int build_plan_m16_device(int device, const std::vector<uint16_t>& targets, const std::vector<int>& emit,
                          const std::vector<uint16_t>& sources, std::vector<int32_t> in_slots,
                          std::vector<int32_t> out_slots, std::unique_ptr<DevPlan>& out, hipStream_t st) {
    const Field& F = field();
    const int K = int(sources.size()), R = int(emit.size()), d = int(targets.size());
    auto p = std::make_unique<DevPlan>();
    p->device = device;
    p->m = 16;
    p->K = K;
    p->R = R;
    p->rt = apply_tile_rows(16, std::max(R, 1));
    p->ntiles = (R + p->rt - 1) / p->rt;
    const uint16_t *logt = nullptr, *expt = nullptr;
    const uint8_t* g8 = nullptr;
    int rc = plan_tables(device, &logt, &g8, &expt);
    if (rc) return rc;
    const size_t coef_bytes = size_t(p->ntiles) * K * (p->rt / 2) * 4;
    const size_t rec_bytes = size_t(p->ntiles) * (K + 1) * 256;
    const bool records = p->rt == 64 && rec_bytes <= (size_t(256) << 20);
    std::vector<uint16_t> y(static_cast<size_t>(K)), x(static_cast<size_t>(d));
    for (int q = 0; q < K; ++q) y[size_t(q)] = F.exp[sources[size_t(q)]];
    for (int e = 0; e < d; ++e) x[size_t(e)] = F.exp[targets[size_t(e)]];
    // one allocation: [in][out][y][x][emit] uploaded on the caller's stream, then [lp][ld][coef][records]
    // zeroed and filled on the device there too (the build's temporaries y .. ld stay with the plan:
    // freeing them here would wait for the device)
    out_slots.resize(std::max(size_t(p->ntiles) * p->rt, size_t((R + 31) / 32) * 32), 0);
    in_slots.resize(in_slots.size() + 16, 0);
    PlanBlob blob;
    const size_t o_in = blob.add(in_slots.data(), in_slots.size() * 4);
    const size_t o_out = blob.add(out_slots.data(), out_slots.size() * 4);
    const size_t o_y = blob.add(y.data(), y.size() * 2), o_x = blob.add(x.data(), x.size() * 2);
    const size_t o_emit = blob.add(emit.data(), emit.size() * 4);
    const size_t up = blob.host.size();
    const size_t o_lp = blob.add(nullptr, size_t(K) * 4), o_ld = blob.add(nullptr, size_t(R) * 4);
    const size_t o_coef = blob.add(nullptr, coef_bytes);
    const size_t o_idx = records ? blob.add(nullptr, rec_bytes) : SIZE_MAX;
    if ((rc = blob.upload(*p, st))) return rc;
    HIP_TRY(hipMemsetAsync(PlanBlob::at<uint8_t>(*p, up), 0, blob.total - up, st));
    p->d_in = PlanBlob::at<int32_t>(*p, o_in);
    p->d_out = PlanBlob::at<int32_t>(*p, o_out);
    p->d_coef = PlanBlob::at<uint32_t>(*p, o_coef);
    if (records) p->d_idx = PlanBlob::at<uint32_t>(*p, o_idx);
    Plan16Args a{};
    a.src_el = PlanBlob::at<const uint16_t>(*p, o_y);
    a.tgt_el = PlanBlob::at<const uint16_t>(*p, o_x);
    a.emit = PlanBlob::at<const int32_t>(*p, o_emit);
    a.logt = logt;
    a.expt = expt;
    a.lp = PlanBlob::at<uint32_t>(*p, o_lp);
    a.ld = PlanBlob::at<uint32_t>(*p, o_ld);
    a.coef = p->d_coef;
    a.rec = records ? reinterpret_cast<uint8_t*>(p->d_idx) : nullptr;
    a.K = K;
    a.d = d;
    a.R = R;
    a.rt = p->rt;
    HIP_TRY(launch_plan_m16(a, st));
    if ((rc = PlanBlob::finish(*p))) return rc;
    in_slots.resize(size_t(K));
    p->in_slots = std::move(in_slots);
    p->out_slots = std::move(out_slots);
    out = std::move(p);
    return 0;
}

// Target / source position lists of the encode (erased == NULL) or decode matrix, and their slots.
void codec_lists(const std::vector<uint16_t>& pos, uint16_t k, uint16_t r, const bool* erased,
                 std::vector<uint16_t>& targets, std::vector<int>& emit, std::vector<uint16_t>& sources,
                 std::vector<int32_t>& in_slots, std::vector<int32_t>& out_slots) {
    const size_t n = size_t(k) + r;
    targets.clear();
    emit.clear();
    sources.clear();
    in_slots.clear();
    out_slots.clear();
    if (!erased) {
        // encode: solve the r repair positions from the k information positions
        for (size_t i = 0; i < k; ++i) sources.push_back(pos[i]), in_slots.push_back(int32_t(i));
        for (size_t p = 0; p < r; ++p) targets.push_back(pos[k + p]), emit.push_back(int(p)), out_slots.push_back(int32_t(p));
    } else {
        for (size_t i = 0; i < n; ++i) {
            if (erased[i]) {
                if (i < k) emit.push_back(int(targets.size())), out_slots.push_back(int32_t(i));
                targets.push_back(pos[i]);
            } else {
                sources.push_back(pos[i]);
                in_slots.push_back(int32_t(i));
            }
        }
    }
}

int codec_matrix(const std::vector<uint16_t>& pos, uint16_t k, uint16_t r, const bool* erased,
                 std::vector<uint16_t>& M, std::vector<int32_t>& in_slots, std::vector<int32_t>& out_slots) {
    std::vector<uint16_t> targets, sources;
    std::vector<int> emit;
    codec_lists(pos, k, r, erased, targets, emit, sources, in_slots, out_slots);
    M = solve_matrix(targets, emit, sources);
    return 0;
}

}  // namespace rsamd
