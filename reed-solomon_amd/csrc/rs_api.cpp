// rs_api.cpp -- C ABI of librs_amd.so: the reference's drop-in API (rs/reed_solomon.h,
// memory/*.h, scalar gf/cc helpers) and the batched device API (rs_amd/rsg.h).
//
// Every encode/decode runs on the GPU through rs_kernels.hip; there is no CPU compute path for
// symbol data in this library.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <string>
#include <vector>

#include "gen/asm_counts.h"
#include "gen/cs16t_off.h"
#include "gf16.hpp"
#include "rs_jit.hpp"
#include "rs_kernels.hpp"
#include "rs_pool.hpp"
#include "rs_xj.hpp"
#include <thread>
#include <unistd.h>
#include <sys/mman.h>

extern "C" {
#include <memory/seq.h>
#include <rs/cyclotomic_coset.h>
#include <rs/fft.h>
#include <rs/gf65536.h>
#include <rs/reed_solomon.h>
#include <rs_amd/rsg.h>
}

using namespace rsamd;

#ifdef RS_AMD_DIAG
#define RSG_VERSION "rs_amd 0.2 (gfx950, DIAGNOSTIC build: timing ablations enabled)"
#else
#define RSG_VERSION "rs_amd 0.2 (gfx950)"
#endif

static int hip_fail(hipError_t e, const char* what) {
    std::fprintf(stderr, "librs_amd: %s failed: %s\n", what, hipGetErrorString(e));
    return RS_ERR_DEVICE;
}

#define HIP_TRY(expr)                                      \
    do {                                                   \
        hipError_t _e = (expr);                            \
        if (_e != hipSuccess) return hip_fail(_e, #expr);  \
    } while (0)

// ============================================================================ device plans
namespace {

struct DeviceTables {
    uint32_t* d_ltab = nullptr;  // 2048 dwords, see ApplyArgs::ltab
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
        std::vector<uint32_t> h(2048);
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
        void* p = nullptr;
        HIP_TRY(hipMalloc(&p, h.size() * 4));
        HIP_TRY(hipMemcpy(p, h.data(), h.size() * 4, hipMemcpyHostToDevice));
        t.d_ltab = static_cast<uint32_t*>(p);
    }
    *out = t.d_ltab;
    return 0;
}

// log / gamma-byte tables of the device plan builder (k_plan_m8)
int plan_tables(int device, const uint16_t** logt, const uint8_t** g8, const uint16_t** expt = nullptr) {
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

// A coding matrix resident on one device, packed for the kernels.
struct DevPlan {
    int device = 0;
    int m = 16, rt = 0, K = 0, R = 0, ntiles = 0;
    int32_t* d_in = nullptr;
    int32_t* d_out = nullptr;
    uint32_t* d_coef = nullptr;
    uint32_t* d_idx = nullptr;  // m8, rt 32: pre-split nibble indices; m16, rt 64: table indices (asm kernels)
    std::vector<uint16_t> matrix;  // R x K, GF(2^16)
    std::vector<int32_t> in_slots, out_slots;
    std::unique_ptr<JitKernel> jit;  // matrix-specialised kernel, if built
    bool jit_failed = false;         // compile failed once: stay on the generic kernels
    std::unique_ptr<XjKernel> xj;    // bit-plane XOR kernel (rs_xj.hpp), if built
    bool xj_failed = false;
    // GF(2^16) syndrome route (k_cs16, then `second`): set when this plan applies its matrix as
    //   out = M2 * S,  S_j = sum_i X_i^j in_i (j < D)  -- the reference's own factorisation (syndromes by
    // the cyclotomic FFT, evaluator + Forney). The arrays live in this plan's blob; `dense` is the
    // plain matrix plan, built on demand for launches the route does not cover (stripe-id lists,
    // symbol sizes that are not a multiple of 1 KiB).
    struct Cs {
        int kind = 0;  // 0: k_cs16 syndromes into scratch, then `second`; 1: k_bs16 straight into the outputs
        int D = 0, ngroups = 0, ntiles = 0, fin_stride = 0;
        int64_t max_slot = 0;       // largest input slot (the loads' byte range)
        int32_t* groups = nullptr;  // [ngroups + 2][16] input slots, -1 = none
        uint32_t* rec = nullptr;
        // k_cs16t (kind 0): tiles of kCs16tCw cosets, records [ntiles_t][ngroups + 2][4 kCs16tCw] block
        // offsets, its finish lists, and its VALU per column unit (sum over tiles and groups of its blocks)
        uint32_t* rec_t = nullptr;
        int32_t* fin_t = nullptr;
        int32_t* fin_off_t = nullptr;
        int ntiles_t = 0, fin_stride_t = 0;
        uint64_t valu_t = 0;
        int32_t* fin = nullptr;
        int32_t* fin_off = nullptr;
        uint32_t nblog[16] = {};
        std::vector<int32_t> h_groups;  // host copy of `groups` (re-encode plans mask it)
    };
    std::unique_ptr<Cs> cs;
    std::unique_ptr<DevPlan> second, dense;
    // Decode by re-encoding (no repair symbol erased, t close to r): with U the surviving information
    // slots, e = D_Rep (y + G_U u) -- G_U u is the codec's encode route (k_cs16 + k_bs16) over U only
    // (`groups` = the encode plan's groups with the erased slots masked), y the received repair symbols,
    // D_Rep the decode matrix's repair columns (t x r, dense). Exact: D_U = D_Rep G_U over GF(2^16).
    struct Reenc {
        int32_t* groups = nullptr;  // in this plan's blob
        std::unique_ptr<DevPlan> drep;
    };
    std::unique_ptr<Reenc> reenc;
    // decode plans of route-eligible GF(2^16) patterns start dense: `route` is built once route_bytes
    // (bytes moved by this plan's launches) reaches the codec's route_min_bytes
    bool route_ok = false;
    uint64_t route_bytes = 0;
    std::unique_ptr<DevPlan> route;
    std::vector<uint8_t> erased;  // the pattern (empty: encode), to build `dense`
    int64_t uses = 0;                // launches of this plan (JIT policy)
    void* blob = nullptr;            // set: d_in / d_out / d_coef / d_idx are views into this one allocation
    size_t blob_cap = 0;             // its size class (plan_pool)
    // stream-ordered build: the upload (and device fill) ran on `built_on`; `ready` marks its end, so a
    // launch on another stream waits for it; the pinned source of the upload lives until then
    hipEvent_t ready = nullptr;
    hipStream_t built_on = nullptr;
    void* h_stage = nullptr;
    size_t stage_cap = 0;
    // the guard that keeps the memory from being reused before the last launch is done: `used`, recorded
    // on the launch stream after the first 16 launches and then after every 64th (a record costs
    // microseconds of host time, which small launches would feel every call; recording at release
    // instead is unsafe, as the caller's stream may be gone by then). A plan released with launches
    // after its last record waits for the device; one launched on more than one stream is released
    // with hipFree (device-synchronous) instead of to the pool.
    hipEvent_t used = nullptr;
    hipStream_t used_on = nullptr;
    bool launched = false, multi_stream = false;
    int64_t launches = 0, recorded = 0;  // launches so far / covered by `used`
    int note_use(hipStream_t st) {
        if (launched && used_on != st) multi_stream = true;
        used_on = st;
        launched = true;
        if (++launches <= 16 || launches % 64 == 0) return record_guard(st);
        return 0;
    }
    int record_guard(hipStream_t st) {
        if (!used) HIP_TRY(hipEventCreateWithFlags(&used, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(used, st));
        recorded = launches;
        return 0;
    }
    // before a release from a call on stream st (cache eviction): a plan whose launches all ran on st
    // gets its guard there -- st is alive, and it orders after them -- instead of a device wait
    // The plans this one owns (second stage, dense twin, route, re-encode D_Rep) are launched by its
    // calls too, so they get the same treatment: without it their destructors would wait for the device.
    void guard_before_release(hipStream_t st) {
        if (launched && !multi_stream && recorded != launches && used_on == st) (void)record_guard(st);
        for (DevPlan* q : {second.get(), dense.get(), route.get(), reenc ? reenc->drep.get() : nullptr})
            if (q) q->guard_before_release(st);
    }
    // called before a launch on stream st: orders it after the build, releases the build's resources
    // once the build is complete
    int order_after_build(hipStream_t st) {
        if (!ready) return 0;
        const hipError_t q = hipEventQuery(ready);
        (void)hipGetLastError();  // NotReady is a status, not an error of the next launch
        if (q == hipSuccess) {
            (void)hipEventDestroy(ready);
            ready = nullptr;
            pool_host_release(h_stage, stage_cap);
            h_stage = nullptr;
            return 0;
        }
        if (st != built_on && hipStreamWaitEvent(st, ready, 0) != hipSuccess) return RS_ERR_DEVICE;
        return 0;
    }
    ~DevPlan() {
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
};

// A plan's device arrays in one allocation, filled by one copy (a new decode pattern then costs one
// hipMalloc + one upload instead of four of each, and one hipFree when the cache evicts it).
struct PlanBlob {
    std::vector<uint8_t> host;  // the uploaded prefix: every part added with a source
    size_t total = 0;           // prefix + device-only parts (src = null, added after the prefix)
    size_t add(const void* src, size_t bytes) {  // offset of a 256-byte aligned part
        const size_t o = (total + 255) & ~size_t(255);
        total = o + std::max<size_t>(bytes, 16);
        if (src) {
            host.resize(total, 0);
            if (bytes) std::memcpy(host.data() + o, src, bytes);
        }
        return o;
    }
    // Allocates the plan's buffer and uploads the prefix on stream st, from a pinned copy the plan keeps
    // until the copy is done (no null-stream copy: a new pattern must not stall unrelated streams).
    int upload(DevPlan& p, hipStream_t st) {
        if (int rc = pool_dev_acquire(total, p.device, &p.blob, &p.blob_cap)) return rc;
        p.built_on = st;
        if (host.empty()) return 0;
        if (int rc = pool_host_acquire(host.size(), &p.h_stage, &p.stage_cap)) return rc;
        std::memcpy(p.h_stage, host.data(), host.size());
        HIP_TRY(hipMemcpyAsync(p.blob, p.h_stage, host.size(), hipMemcpyHostToDevice, st));
        return 0;
    }
    // marks the end of the plan's build work queued on its stream
    static int finish(DevPlan& p) {
        HIP_TRY(hipEventCreateWithFlags(&p.ready, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(p.ready, p.built_on));
        return 0;
    }
    template <class T>
    static T* at(DevPlan& p, size_t o) { return reinterpret_cast<T*>(static_cast<uint8_t*>(p.blob) + o); }
};

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

}  // namespace

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

struct rsg_codec {
    int device = 0;
    uint16_t k = 0, r = 0;
    int m = 16;
    std::vector<uint16_t> positions;
    const uint32_t* d_ltab = nullptr;
    std::unique_ptr<DevPlan> enc;
    std::map<std::vector<uint8_t>, std::unique_ptr<DevPlan>> dec;
    std::vector<std::vector<uint8_t>> dec_lru;
    int m8_mode = 18;
    int m16_mode = 0;  // m = 16 kernels: 0 hand-scheduled (64-row tiles), 1 its timing ablation, 2 compiled
    int m16_plans = 2;  // m = 16 plans: 0 host, 1 device (build_plan_m16_device), 2 device above 64K coefficients
    int m16_route = 1;  // m = 16 matrices with K >= 64: 1 syndrome route (k_cs16 + D x R apply), 0 dense, 2 all
    // a decode pattern with t > 64 erasures starts on the dense device-built plan and moves to the
    // syndrome route once its launches have moved this many bytes ((K + R) * S per stripe): that route
    // plan's host build (~16 ms at C5, t = 1024) pays only over a few hundred stripes; 0 = route at once
    // (option m16_route_min_bytes). Patterns with t <= 64 take the route at once (cheap build).
    int64_t route_min_bytes = int64_t(1) << 30;
    // wave-instructions issued by the hand-scheduled GF(2^16) kernels of the last rsg_encode / rsg_decode
    // (their generated steps' VALU / SALU counts times the steps run; rsg_last_work)
    uint64_t work_valu = 0, work_salu = 0;
    void* d_cs = nullptr;  // syndrome route scratch: [chunk][D][S]
    void* d_reenc = nullptr;  // re-encode decode scratch: [chunk][r][S] (G_U u + y)
    size_t reenc_cap = 0;
    int m16_reenc = 1;  // option m16_reenc: 0 keeps full-pattern decodes on the plain route
    // rsg_decode_batch of GF(2^16) codes with per-stripe patterns (decode_batch_m16_ps): 1 = the syndrome
    // route with a device-built plan per stripe (default), 0 = a plan per distinct pattern
    int m16_ps = 1;
    std::map<int, std::unique_ptr<DevPlan>> ps_syn;  // k_cs16 plans over all k + r slots, keyed by D
    std::vector<int> ps_syn_lru;
    void *d_ps_rec = nullptr, *d_ps_small = nullptr;  // per-stripe records / lists of decode_batch_m16_ps
    int32_t* d_ps_in = nullptr;                       // its shared input list 0 .. r + 15
    hipStream_t ps_side = nullptr;                    // plan kernels of the next chunk run here
    hipStream_t ps_synst = nullptr;                   // option m16_ps_overlap: the syndrome passes run here
    hipEvent_t ps_ev_entry = nullptr, ps_ev_zero[2] = {nullptr, nullptr}, ps_ev_plan[2] = {nullptr, nullptr},
               ps_ev_used[2] = {nullptr, nullptr}, ps_ev_syn[2] = {nullptr, nullptr};
    int ps_overlap = 1;  // 1: chunk i + 1's syndrome pass beside chunk i's solve (two syndrome buffers)
    // option m16_cs_overlap: the same for the one-pattern syndrome route (run_cs); off by default: C5 in four
    // overlapped chunks measured 77.5-78.3 GB/s against 80.6-80.7 serial (profiles/r3_cs_overlap_ab.log)
    int cs_overlap = 0;
    int64_t ps_chunk = 0;   // option m16_ps_chunk: max stripes per chunk (0 = by ps_rec_mib)
    int64_t ps_rec_mib = 1024;  // records per chunk (MiB); larger chunks keep k_cs16 busier (measured 48-1024)
    size_t ps_rec_cap = 0, ps_small_cap = 0;
    int m16_cs_thread = 1;  // option m16_cs_thread: 1 k_cs16t (threaded blocks), 0 k_cs16 (gpr-index lookups)
    int m16_cs_col = 256;  // option m16_cs_col: the route kernels' block layout (256 or 1024 bytes, rs_kernels.hip)
    size_t cs_cap = 0;
    void* d_goff[2] = {nullptr, nullptr};  // syndrome route: input slots as byte offsets (per stage)
    size_t goff_cap[2] = {0, 0};
    int jit = 2;  // 0 off, 1 every eligible plan, 2 encode plans + decode plans from their 2nd use
    int dec_jit_uses = 2;  // jit = 2: decode plans are specialised from this many launches on
    int xj = 1;   // specialised kernel family: 1 bit-plane XOR kernels (rs_xj), 0 nibble-table rs_v1jit
    uint64_t* stamps = nullptr;  // device buffer for mode 17 (instrumented timing)
    int32_t* d_ids = nullptr;    // stripe-id lists of rsg_decode_batch
    size_t ids_cap = 0;
    // rsg_decode_batch with device-built per-stripe plans (k_plan_m8): 0 = host plans per distinct
    // pattern, 1 = device plans, 2 = device plans when more than kHostPlanGroups patterns (default)
    int batch_plans = 2;
    // device-plan decodes of m <= 8 codes: 1 = syndrome route (fixed r x (k + r) syndrome matrix on the
    // XOR kernel, then a per-stripe t_info x t solve), 0 = per-stripe survivor matrices (k_plan_m8)
    int syn_route = 1;
    std::unique_ptr<DevPlan> syn;  // syndrome matrix S_j = sum_i X_i^j rcv_i, j < r
    bool syn_failed = false;
    void* d_syn = nullptr;  // [chunk][r][S] syndromes
    size_t syn_cap = 0;
    uint16_t* d_elem = nullptr;  // [k + r] slot elements alpha^position
    void *d_masks = nullptr, *d_kr = nullptr, *d_pin = nullptr, *d_pout = nullptr, *d_pidx = nullptr;
    size_t masks_cap = 0, kr_cap = 0, pin_cap = 0, pout_cap = 0, pidx_cap = 0;
    void* d_partial = nullptr;  // split-K partial products of small m = 16 launches
    size_t partial_cap = 0;
    // rsg_decode_batch for GF(2^16) codes with many patterns: one reusable device plan, rebuilt on the
    // stream for each pattern (batch_plan_m16); its lists go through two pinned staging buffers
    std::unique_ptr<DevPlan> bp16;
    void* d_bp16 = nullptr;      // [y: n u16][x: r u16][emit: r i32][lp: n u32][ld: r u32]
    void* d_bp16_rec = nullptr;  // index records (the plan's d_idx when the pattern uses them)
    uint8_t* h_bp16[2] = {nullptr, nullptr};
    hipEvent_t bp16_ev[2] = {nullptr, nullptr};
    bool bp16_rec_pending[2] = {false, false};
    // the scratch above is reused by every rsg_decode_batch call: the event marks the end of the last
    // call's launches (which may be on another stream) and is waited for before the next overwrite
    hipEvent_t scratch_ev = nullptr;
    bool scratch_pending = false;
    hipStream_t scratch_stream = nullptr;
    // rsg_encode_host / rsg_decode_host: two streams, each with its own device batch buffer
    hipStream_t hs[2] = {nullptr, nullptr};
    uint8_t* hbuf[2] = {nullptr, nullptr};
    size_t hbuf_cap = 0;
    ~rsg_codec() {
        (void)hipSetDevice(device);
        if (scratch_ev) (void)hipEventDestroy(scratch_ev);
        if (ps_side) (void)hipStreamSynchronize(ps_side), (void)hipStreamDestroy(ps_side);
        if (ps_synst) (void)hipStreamSynchronize(ps_synst), (void)hipStreamDestroy(ps_synst);
        for (hipEvent_t e : {ps_ev_entry, ps_ev_zero[0], ps_ev_zero[1], ps_ev_plan[0], ps_ev_plan[1], ps_ev_used[0],
                             ps_ev_used[1], ps_ev_syn[0], ps_ev_syn[1]})
            if (e) (void)hipEventDestroy(e);
        if (bp16) bp16->d_idx = nullptr;  // d_bp16_rec, freed below
        for (int i = 0; i < 2; ++i) {
            if (bp16_ev[i]) (void)hipEventDestroy(bp16_ev[i]);
            if (h_bp16[i]) (void)hipHostFree(h_bp16[i]);
        }
        for (int i = 0; i < 2; ++i) {
            if (hs[i]) (void)hipStreamDestroy(hs[i]);
            if (hbuf[i]) (void)hipFree(hbuf[i]);
        }
        for (void* p : {static_cast<void*>(d_ids), static_cast<void*>(d_elem), d_masks, d_kr, d_pin, d_pout, d_pidx,
                        d_partial, d_syn, d_bp16, d_bp16_rec, d_cs, d_reenc, d_goff[0], d_goff[1], d_ps_rec,
                        d_ps_small, static_cast<void*>(d_ps_in)})
            if (p) (void)hipFree(p);
    }
    std::string last_kernel = "none";
};

// Target / source position lists of the encode (erased == NULL) or decode matrix, and their slots.
static void codec_lists(const std::vector<uint16_t>& pos, uint16_t k, uint16_t r, const bool* erased,
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

static int codec_matrix(const std::vector<uint16_t>& pos, uint16_t k, uint16_t r, const bool* erased,
                        std::vector<uint16_t>& M, std::vector<int32_t>& in_slots, std::vector<int32_t>& out_slots) {
    std::vector<uint16_t> targets, sources;
    std::vector<int> emit;
    codec_lists(pos, k, r, erased, targets, emit, sources, in_slots, out_slots);
    M = solve_matrix(targets, emit, sources);
    return 0;
}

// The device plan of the encode (erased == NULL) or decode matrix: GF(2^16) codes with large matrices
// are built on the device, everything else from the host matrix.
static const std::vector<uint16_t>* normal_repr_tables();  // [li][d]: alpha^d in the normal basis of GF(2^(1 << li))
static uint16_t normal_basis_element(int m, int i);          // i-th element of the normal basis of GF(2^m)

// Second stage of the syndrome route: out_p = sum_{j < D} M2[p][j] S_j for the emitted targets p, with
// E = all D targets. This is the reference's evaluator + Forney restore (reed_solomon.c:186-336, the same
// for encode, E = repair positions, and decode, E = erased positions):
//   Omega = S * Lambda_E mod x^D,  out_p = F_p * sum_{i < D} X_p^-i Omega_i,  F_p = X_p / Lambda_E'(X_p^-1)
// so M2[p][j] = F_p x^j sum_{d = 0}^{D - 1 - j} Lambda_d x^d with x = X_p^-1 (O(D) per row).
static std::vector<uint16_t> syndrome_solve_matrix(const std::vector<uint16_t>& targets, const std::vector<int>& emit) {
    const Field& F = field();
    const size_t D = targets.size(), R = emit.size();
    std::vector<uint16_t> lam(D + 1, 0);  // Lambda_E(x) = prod (1 + X_e x), reference _rs_get_locator_poly
    lam[0] = 1;
    for (size_t d = 0; d < D; ++d) {
        const uint16_t xe = F.exp[targets[d]];
        for (size_t i = d + 1; i > 0; --i) lam[i] ^= F.mul(lam[i - 1], xe);
    }
    std::vector<uint16_t> M(R * D), pw(D), q(D);
    for (size_t r = 0; r < R; ++r) {
        const uint16_t pos = targets[size_t(emit[r])];
        const uint16_t x = F.exp[(kN - pos) % kN];  // X_p^-1
        pw[0] = 1;
        for (size_t d = 1; d < D; ++d) pw[d] = F.mul(pw[d - 1], x);
        uint16_t dl = 0;  // Lambda'(x) = sum over odd i of Lambda_i x^(i - 1)
        for (size_t i = 1; i <= D; i += 2) dl ^= F.mul(lam[i], pw[i - 1]);
        const uint16_t fp = F.div(F.exp[pos], dl);
        uint16_t acc = 0;  // q[m] = sum_{d <= m} Lambda_d x^d
        for (size_t d = 0; d < D; ++d) q[d] = acc ^= F.mul(lam[d], pw[d]);
        for (size_t j = 0; j < D; ++j) M[r * D + j] = F.mul(F.mul(fp, pw[j]), q[D - 1 - j]);
    }
    return M;
}

// The syndrome route's k_cs16 plan: input groups (the codec's cyclotomic cosets, a slot per coset
// element, -1 where the slot is not an input), syndrome cosets of j < D in tiles of 8, gpr-index records
// and the finish lists (gen_asm.py cs16, rs_kernels.hip:k_cs16).
struct CsHost {
    int D = 0, ngroups = 0, ntiles = 0, fin_stride = 1;
    std::vector<int32_t> groups, fin, fin_off;
    std::vector<uint8_t> rec;
    // k_cs16t (gen_asm.py cs16t): its own tiling (kCs16tCw cosets per tile) and block-offset records
    int ntiles_t = 0, fin_stride_t = 1;
    std::vector<int32_t> fin_t, fin_off_t;
    std::vector<uint32_t> rec_t;
    uint64_t valu_t = 0;
};

static CsHost cs16_host(const std::vector<uint16_t>& pos, const std::vector<int32_t>& in_slots, int D) {
    const size_t n = pos.size();
    std::vector<char> is_in(n, 0);
    for (int32_t v : in_slots) is_in[size_t(v)] = 1;
    // groups: runs of slots whose positions double (a coset in cc_cosets_to_positions order), <= 16
    std::vector<int32_t> groups;
    std::vector<uint16_t> lead;
    for (size_t i = 0; i < n;) {
        size_t j = i + 1;
        while (j < n && j - i < 16 && pos[j] == uint16_t((uint32_t(pos[j - 1]) << 1) % kN)) ++j;
        bool any = false;
        for (size_t a = i; a < j; ++a) any |= is_in[a] != 0;
        if (any) {
            for (size_t a = 0; a < 16; ++a) groups.push_back(i + a < j && is_in[i + a] ? int32_t(i + a) : -1);
            lead.push_back(pos[i]);
        }
        i = j;
    }
    // the kernel steps two groups per iteration (record buffers alternate) and prefetches the inputs of
    // the next group and the slot offsets of the one after: pad to an even count, plus 3 empty groups
    const int ng = int(lead.size()) + int(lead.size() & 1);
    groups.resize(size_t(ng + 3) * 16, -1);
    // syndrome cosets: j < D grouped by s * 2^b (mod N), s the smallest member
    std::vector<uint16_t> cs_s;
    std::vector<std::vector<std::pair<int, int>>> cs_need;  // (b, j)
    std::vector<char> seen(size_t(D), 0);
    for (int j = 0; j < D; ++j) {
        if (seen[size_t(j)]) continue;
        cs_s.push_back(uint16_t(j));
        cs_need.emplace_back();
        for (int b = 0; b < 16; ++b) {
            const uint32_t jj = uint32_t((uint64_t(j) << b) % kN);
            if (jj < uint32_t(D) && !seen[jj]) {
                seen[jj] = 1;
                cs_need.back().emplace_back(b, int(jj));
            }
        }
    }
    const std::vector<uint16_t>& rep = normal_repr_tables()[4];
    const int C = int(cs_s.size()), nlead = int(lead.size());
    // finish lists of tiles of cw cosets: entry = local coset | b << 4 | j << 8, coset c's entries at
    // [fin_off[tile][c], fin_off[tile][c + 1])
    auto finish_lists = [&](int cw, int& ntiles, int& fin_stride, std::vector<int32_t>& fin, std::vector<int32_t>& fin_off) {
        ntiles = (C + cw - 1) / cw;
        fin_stride = 1;
        for (int t = 0; t < ntiles; ++t) {
            int cnt = 0;
            for (int c = cw * t; c < std::min(C, cw * t + cw); ++c) cnt += int(cs_need[size_t(c)].size());
            fin_stride = std::max(fin_stride, cnt);
        }
        fin.assign(size_t(ntiles) * size_t(fin_stride), 0);
        fin_off.assign(size_t(ntiles) * size_t(cw + 1), 0);
        for (int t = 0; t < ntiles; ++t) {
            int e = 0;
            for (int cl = 0; cl < cw; ++cl) {
                const int c = cw * t + cl;
                fin_off[size_t(t) * size_t(cw + 1) + size_t(cl)] = e;
                if (c < C)
                    for (auto& bj : cs_need[size_t(c)])
                        fin[size_t(t) * size_t(fin_stride) + size_t(e++)] = cl | (bj.first << 4) | (bj.second << 8);
            }
            fin_off[size_t(t) * size_t(cw + 1) + size_t(cw)] = e;
        }
    };
    constexpr int CW = 4;  // syndrome cosets per wave (k_cs16 tile)
    int ntiles = 0, fin_stride = 0;
    std::vector<int32_t> fin, fin_off;
    finish_lists(CW, ntiles, fin_stride, fin, fin_off);
    // records [tile][ng + 2][CW cosets][16 byte indices]; padding groups keep index 0 (table entry 0 = 0)
    std::vector<uint8_t> rec(size_t(ntiles) * size_t(ng + 2) * CW * 16, 0);
    for (int t = 0; t < ntiles; ++t)
        for (int cl = 0; cl < CW && CW * t + cl < C; ++cl)
            for (int g = 0; g < nlead; ++g) {
                const uint32_t z = rep[(uint64_t(cs_s[size_t(CW * t + cl)]) * lead[size_t(g)]) % kN];
                uint8_t* r = rec.data() + ((size_t(t) * size_t(ng + 2) + size_t(g)) * CW + size_t(cl)) * 16;
                for (int tp = 0; tp < 16; ++tp) {  // bit d of e(t') = bit (t' - d) mod 16 of z
                    uint8_t v = 0;
                    for (int d = 0; d < 4; ++d) v = uint8_t(v | (((z >> ((tp - d + 16) % 16)) & 1u) << d));
                    r[tp] = v;
                }
            }
    // k_cs16t (gen_asm.py cs16t): tiles of kCs16tCw cosets, records [tile][ng + 2][4 kCs16tCw] block
    // offsets, entry p = 4c + n the block (c, n, nibble n of z). Every entry names a block of its own
    // position (padding: the empty block v = 0), so every step's chain runs all its blocks and returns.
    constexpr int CWT = kCs16tCw, NBT = 4 * kCs16tCw;
    CsHost h;
    finish_lists(CWT, h.ntiles_t, h.fin_stride_t, h.fin_t, h.fin_off_t);
    std::vector<uint32_t> rec_t(size_t(h.ntiles_t) * size_t(ng + 2) * NBT);
    for (size_t i = 0; i < rec_t.size(); ++i) rec_t[i] = kCs16tOff[(i % NBT) * 16];
    for (int t = 0; t < h.ntiles_t; ++t)
        for (int cl = 0; cl < CWT && CWT * t + cl < C; ++cl)
            for (int g = 0; g < nlead; ++g) {
                const uint32_t z = rep[(uint64_t(cs_s[size_t(CWT * t + cl)]) * lead[size_t(g)]) % kN];
                uint32_t* rt = rec_t.data() + (size_t(t) * size_t(ng + 2) + size_t(g)) * NBT;
                for (int nb = 0; nb < 4; ++nb) rt[4 * cl + nb] = kCs16tOff[(4 * cl + nb) * 16 + ((z >> (4 * nb)) & 15u)];
            }
    // zero nibbles cost no jump: an entry naming the empty block (p, 0) is replaced by entry p + 1, so the
    // previous block jumps straight to block p + 1 (whose tail reads entry p + 2); the last position
    // keeps its block, the one that returns. Padding groups become a single jump.
    for (size_t row = 0; row < rec_t.size() / NBT; ++row) {
        uint32_t* rt = rec_t.data() + row * NBT;
        for (int p = NBT - 2; p >= 0; --p)
            if (rt[p] == kCs16tOff[p * 16]) rt[p] = rt[p + 1];
    }
    uint64_t valu_t = 0;  // the step's own VALU (pair sums, lane, address adds) and its blocks', every step of every tile
    constexpr int NBLK = int(sizeof(kCs16tOff) / sizeof(kCs16tOff[0]));
    std::unordered_map<uint32_t, int> off_block;  // code offset -> block index (4c + n) * 16 + v
    for (int b = 0; b < NBLK; ++b) off_block[kCs16tOff[b]] = b;
    for (int t = 0; t < h.ntiles_t; ++t)
        for (int g = 0; g < ng; ++g) {
            valu_t += uint64_t(kValu_cs16t);
            const uint32_t* rt = rec_t.data() + (size_t(t) * size_t(ng + 2) + size_t(g)) * NBT;
            for (int b = off_block[rt[0]];; b = off_block[rt[b / 16 + 1]]) {  // the chain the step runs
                valu_t += kCs16tValu[b];
                if (b / 16 == NBT - 1) break;
            }
        }
    h.rec_t = std::move(rec_t);
    h.valu_t = valu_t;
    h.D = D;
    h.ngroups = ng;
    h.ntiles = ntiles;
    h.fin_stride = std::max(fin_stride, 1);
    h.groups = std::move(groups);
    h.rec = std::move(rec);
    h.fin = std::move(fin);
    h.fin_off = std::move(fin_off);
    return h;
}

static int upload_cs(DevPlan& p, const CsHost& h, int kind, const std::vector<int32_t>& in_slots, hipStream_t st);

static int build_cs16(DevPlan& p, const std::vector<uint16_t>& pos, const std::vector<int32_t>& in_slots, int D,
                      hipStream_t st) {
    return upload_cs(p, cs16_host(pos, in_slots, D), 0, in_slots, st);
}

static int upload_cs(DevPlan& p, const CsHost& h, int kind, const std::vector<int32_t>& in_slots, hipStream_t st) {
    PlanBlob blob;  // groups, records and finish lists in the plan's one allocation
    const size_t o_g = blob.add(h.groups.data(), h.groups.size() * 4), o_r = blob.add(h.rec.data(), h.rec.size());
    const size_t o_f = blob.add(h.fin.data(), h.fin.size() * 4), o_fo = blob.add(h.fin_off.data(), h.fin_off.size() * 4);
    const bool thr = !h.rec_t.empty();
    const size_t o_t = thr ? blob.add(h.rec_t.data(), h.rec_t.size() * 4) : 0;
    const size_t o_ft = thr ? blob.add(h.fin_t.data(), h.fin_t.size() * 4) : 0;
    const size_t o_fot = thr ? blob.add(h.fin_off_t.data(), h.fin_off_t.size() * 4) : 0;
    if (int rc = blob.upload(p, st)) return rc;
    if (int rc = PlanBlob::finish(p)) return rc;
    auto cs = std::make_unique<DevPlan::Cs>();
    cs->kind = kind;
    cs->D = h.D;
    cs->ngroups = h.ngroups;
    cs->ntiles = h.ntiles;
    cs->fin_stride = h.fin_stride;
    cs->groups = PlanBlob::at<int32_t>(p, o_g);
    cs->h_groups = h.groups;
    cs->rec = PlanBlob::at<uint32_t>(p, o_r);
    if (thr) {
        cs->rec_t = PlanBlob::at<uint32_t>(p, o_t);
        cs->fin_t = PlanBlob::at<int32_t>(p, o_ft);
        cs->fin_off_t = PlanBlob::at<int32_t>(p, o_fot);
        cs->ntiles_t = h.ntiles_t;
        cs->fin_stride_t = h.fin_stride_t;
    }
    cs->valu_t = h.valu_t;
    cs->fin = PlanBlob::at<int32_t>(p, o_f);
    cs->fin_off = PlanBlob::at<int32_t>(p, o_fo);
    for (int32_t v : in_slots) cs->max_slot = std::max<int64_t>(cs->max_slot, v);
    for (int t = 0; t < 16; ++t) cs->nblog[t] = field().log[normal_basis_element(16, t)];
    p.cs = std::move(cs);
    return 0;
}

// The encode second stage on k_bs16: E = the repair positions (whole cosets) makes Lambda binary, so
// the rows of M2 along an output coset are Frobenius conjugates, M2[L 2^b][j] = M2[L][j]^(2^b): output
// coset c accumulates u_t = sum_j bit_t(z_(c, j)) S_j with z = normal repr of M2[L][j], and the finish
// S_(L 2^b) = sum_t nb_((t + b) mod 16) u_t gives all its outputs (as k_cs16's). Returns false when the
// rows do not have that structure (then the plain matrix plan applies M2).
//
// Decode (round 3): when the erased set E is closed under x -> x^(2^d) (d in {2, 4, 8}: e.g. the bench
// pattern, every 4th slot of 16-slot cosets, is closed under x^16), Lambda_E has coefficients in
// GF(2^d) and the rows along an orbit {X, X^(2^d), ...} are conjugates by the same rule with step d:
// runs of rows whose positions multiply by 2^d, finish rotation d * b. d = 1 is the encode case.
static bool bs16_host(const std::vector<uint16_t>& M2, int D, const std::vector<uint16_t>& targets,
                      const std::vector<int>& emit, const std::vector<int32_t>& out_slots, CsHost& h, int d = 1) {
    const Field& F = field();
    const int R = int(emit.size());
    // output orbits: runs of rows whose positions multiply by 2^d (at most 16 / d rows)
    std::vector<std::pair<int, int>> cos;  // (first row, size)
    for (int r = 0; r < R;) {
        int e = r + 1;
        while (e < R && e - r < 16 / d &&
               targets[size_t(emit[size_t(e)])] == uint16_t((uint64_t(targets[size_t(emit[size_t(e - 1)])]) << d) % kN))
            ++e;
        cos.emplace_back(r, e - r);
        r = e;
    }
    for (auto& c : cos)  // M2[r0 + b][j] = M2[r0 + b - 1][j]^(2^d)
        for (int b = 1; b < c.second; ++b)
            for (int j = 0; j < D; ++j) {
                const uint16_t x = M2[size_t(c.first + b - 1) * D + j];
                if (M2[size_t(c.first + b) * D + j] != (x ? F.exp[((uint64_t(1) << d) * F.log[x]) % kN] : 0)) return false;
            }
    if (d > 1 && 2 * cos.size() > size_t(R)) return false;  // runs shorter than 2 rows on average: dense is cheaper
    constexpr int CW = 4;
    const int ngr = (D + 15) / 16, ng = ngr + (ngr & 1), C = int(cos.size()), ntiles = (C + CW - 1) / CW;
    h = CsHost();
    h.D = D;
    h.ngroups = ng;
    h.ntiles = ntiles;
    h.groups.assign(size_t(ng + 3) * 16, -1);
    for (int j = 0; j < D; ++j) h.groups[size_t(j)] = j;  // group g = syndromes 16 g .. 16 g + 15
    const std::vector<uint16_t>& rep = normal_repr_tables()[4];
    std::vector<uint16_t> z(static_cast<size_t>(D));
    h.rec.assign(size_t(ntiles) * size_t(ng + 2) * CW * 64, 0);
    int fin_stride = 1;
    for (int t = 0; t < ntiles; ++t) {
        int cnt = 0;
        for (int c = CW * t; c < std::min(C, CW * t + CW); ++c) cnt += cos[size_t(c)].second;
        fin_stride = std::max(fin_stride, cnt);
    }
    h.fin_stride = fin_stride;
    h.fin.assign(size_t(ntiles) * size_t(fin_stride), 0);
    h.fin_off.assign(size_t(ntiles) * (CW + 1), 0);
    for (int t = 0; t < ntiles; ++t) {
        int e = 0;
        for (int cl = 0; cl < CW; ++cl) {
            const int c = CW * t + cl;
            h.fin_off[size_t(t) * (CW + 1) + size_t(cl)] = e;
            if (c >= C) continue;
            const int r0 = cos[size_t(c)].first;
            for (int b = 0; b < cos[size_t(c)].second; ++b)
                h.fin[size_t(t) * size_t(fin_stride) + size_t(e++)] = cl | ((d * b) << 4) | (out_slots[size_t(r0 + b)] << 8);
            for (int j = 0; j < D; ++j) {
                const uint16_t v = M2[size_t(r0) * D + j];
                z[size_t(j)] = v ? rep[F.log[v]] : 0;
            }
            for (int g = 0; g < ngr; ++g) {
                uint8_t* r = h.rec.data() + ((size_t(t) * size_t(ng + 2) + size_t(g)) * CW + size_t(cl)) * 64;
                for (int q = 0; q < 4; ++q)
                    for (int tb = 0; tb < 16; ++tb) {  // byte 16 q + t: bit d = bit t of z of input 16 g + 4 q + d
                        uint8_t v = 0;
                        for (int d = 0; d < 4; ++d) {
                            const int j = 16 * g + 4 * q + d;
                            if (j < D) v = uint8_t(v | (((z[size_t(j)] >> tb) & 1u) << d));
                        }
                        r[16 * q + tb] = v;
                    }
            }
        }
        h.fin_off[size_t(t) * (CW + 1) + CW] = e;
    }
    return true;
}

// Smallest d in {1, 2, 4, 8} such that the position set is closed under p -> p * 2^d (mod N), i.e. the
// erased elements under x -> x^(2^d); 16 when none is.
static int orbit_step(const std::vector<uint16_t>& pos) {
    std::vector<char> in(kN, 0);
    for (uint16_t p : pos) in[p % kN] = 1;
    for (int d = 1; d < 16; d *= 2) {
        bool closed = true;
        for (uint16_t p : pos)
            if (!in[size_t((uint64_t(p) << d) % kN)]) {
                closed = false;
                break;
            }
        if (closed) return d;
    }
    return 16;
}

// the syndrome route pays when both sides of the matrix are large
static bool cs_route_eligible(const rsg_codec_t* c, int K, int R, int D) {
    // 1: every matrix with K >= 64 inputs (measured at C5: the route wins at every t from 1 to 1024, e.g.
    // t = 32 decode 20.4 -> 4.4 ms, t = 1 13.1 -> 1.1 ms: the dense kernels for R <= 32 walk all K inputs
    // per workgroup); 2 (measurements): every matrix, whatever its shape
    return c->m > 8 && D <= 32768 && R > 0 && ((c->m16_route == 1 && K >= 64) || (c->m16_route == 2 && K > 0));
}

static int make_plan_dense(rsg_codec_t* c, const bool* erased, std::unique_ptr<DevPlan>& out, hipStream_t st);

// GF(2^16) matrix on the syndrome route: the k_cs16 plan over the sources + the D x R second stage
static int make_plan_cs(rsg_codec_t* c, const bool* erased, std::unique_ptr<DevPlan>& out, hipStream_t st) {
    std::vector<uint16_t> targets, sources;
    std::vector<int> emit;
    std::vector<int32_t> in, outs;
    codec_lists(c->positions, c->k, c->r, erased, targets, emit, sources, in, outs);
    const int K = int(in.size()), R = int(outs.size()), D = int(targets.size());
    auto p = std::make_unique<DevPlan>();
    p->device = c->device;
    p->m = 16;
    p->K = K;
    p->R = R;
    p->in_slots = in;
    p->out_slots = outs;
    if (erased) p->erased.assign(erased, erased + size_t(c->k) + c->r);
    if (int rc = build_cs16(*p, c->positions, in, D, st)) return rc;
    std::vector<int32_t> sin(static_cast<size_t>(D));
    for (int j = 0; j < D; ++j) sin[size_t(j)] = j;
    std::vector<uint16_t> M2 = syndrome_solve_matrix(targets, emit);
    std::unique_ptr<DevPlan> second;
    CsHost bh;
    // encode: Frobenius rows, k_bs16; decode: the same when E is closed under a Frobenius power (orbit_step)
    const int dstep = erased ? orbit_step(targets) : 1;
    if (dstep < 16 && bs16_host(M2, D, targets, emit, outs, bh, dstep)) {
        second = std::make_unique<DevPlan>();
        second->device = c->device;
        second->m = 16;
        second->K = D;
        second->R = R;
        second->in_slots = sin;
        second->out_slots = outs;
        if (int rc = upload_cs(*second, bh, 1, sin, st)) return rc;
    } else if (int rc = build_plan(c->device, 16, std::move(M2), D, R, std::move(sin), std::move(outs), second, st)) {
        return rc;
    }
    p->second = std::move(second);
    out = std::move(p);
    return 0;
}

// Re-encode decode eligibility: the codec's encode plan is the route with the k_bs16 second stage, no
// repair slot is erased, and t is close to r (the re-encode pays for all r syndromes of the encode
// route whatever t is; the plain route's syndrome pass shrinks with t: measured cross-over near 0.9 r).
static bool reenc_eligible(const rsg_codec_t* c, const bool* erased) {
    if (!c->m16_reenc || c->m <= 8 || !erased || !c->enc || !c->enc->cs || c->enc->cs->kind != 0 || !c->enc->second ||
        !c->enc->second->cs || c->enc->second->cs->kind != 1 || c->enc->cs->h_groups.empty())
        return false;
    int t = 0;
    for (int i = 0; i < c->k; ++i) t += erased[i] ? 1 : 0;
    for (int i = c->k; i < c->k + c->r; ++i)
        if (erased[i]) return false;
    if (!(t >= 1 && 10 * t >= 9 * c->r && c->k - t >= 64)) return false;
    // an erased set closed under x -> x^16 (or a smaller Frobenius step) gives the plain route a k_bs16
    // second stage with orbits of >= 4 rows (bs16_host): cheaper than re-encoding + the dense t x r stage
    std::vector<uint16_t> pos;
    for (int i = 0; i < c->k; ++i)
        if (erased[i]) pos.push_back(c->positions[size_t(i)]);
    return orbit_step(pos) > 4;
}

static int make_plan_reenc(rsg_codec_t* c, const bool* erased, std::unique_ptr<DevPlan>& out, hipStream_t st) {
    const DevPlan& E = *c->enc;
    const size_t k = c->k, r = c->r;
    std::vector<uint16_t> targets, sources;
    std::vector<int> emit;
    std::vector<int32_t> in_u, outs;
    for (size_t i = 0; i < k; ++i) {
        if (erased[i]) {
            emit.push_back(int(targets.size()));
            targets.push_back(c->positions[i]);
            outs.push_back(int32_t(i));
        } else {
            in_u.push_back(int32_t(i));
        }
    }
    for (size_t p = 0; p < r; ++p) sources.push_back(c->positions[k + p]);
    std::vector<int32_t> groups = E.cs->h_groups;  // the encode route's input groups, erased slots masked
    for (int32_t& g : groups)
        if (g >= 0 && erased[g]) g = -1;
    auto p = std::make_unique<DevPlan>();
    p->device = c->device;
    p->m = 16;
    p->K = int(in_u.size() + r);  // survivors read: U and the r repair symbols
    p->R = int(outs.size());
    p->in_slots = in_u;
    for (size_t q = 0; q < r; ++q) p->in_slots.push_back(int32_t(k + q));
    p->out_slots = outs;
    p->erased.assign(erased, erased + k + r);
    PlanBlob blob;
    const size_t o_g = blob.add(groups.data(), groups.size() * 4);
    if (int rc = blob.upload(*p, st)) return rc;
    if (int rc = PlanBlob::finish(*p)) return rc;
    p->reenc = std::make_unique<DevPlan::Reenc>();
    p->reenc->groups = PlanBlob::at<int32_t>(*p, o_g);
    std::vector<int32_t> rows(r);
    for (size_t q = 0; q < r; ++q) rows[q] = int32_t(q);  // scratch rows y + G_U u
    if (int rc = build_plan_m16_device(c->device, targets, emit, sources, std::move(rows), std::move(outs),
                                       p->reenc->drep, st))
        return rc;
    out = std::move(p);
    return 0;
}

static int make_plan(rsg_codec_t* c, const bool* erased, std::unique_ptr<DevPlan>& out, hipStream_t st) {
    std::vector<uint16_t> targets, sources;
    std::vector<int> emit;
    std::vector<int32_t> in, outs;
    codec_lists(c->positions, c->k, c->r, erased, targets, emit, sources, in, outs);
    const int K = int(in.size()), R = int(outs.size());
    if (cs_route_eligible(c, K, R, int(targets.size()))) {
        // small t: the route's plan (a few syndrome cosets, a t x t second stage) is cheap to build. Larger
        // patterns start dense and move to the route (or the re-encode decode) at the first launch past
        // route_min_bytes (0: the first launch the route covers); the dense plan serves the rest.
        if (!erased || targets.size() <= 64) return make_plan_cs(c, erased, out, st);
        if (int rc = make_plan_dense(c, erased, out, st)) return rc;
        out->route_ok = true;
        out->erased.assign(erased, erased + size_t(c->k) + c->r);
        return 0;
    }
    return make_plan_dense(c, erased, out, st);
}

// the plain matrix plan (host- or device-built)
static int make_plan_dense(rsg_codec_t* c, const bool* erased, std::unique_ptr<DevPlan>& out, hipStream_t st) {
    std::vector<uint16_t> targets, sources;
    std::vector<int> emit;
    std::vector<int32_t> in, outs;
    codec_lists(c->positions, c->k, c->r, erased, targets, emit, sources, in, outs);
    const int K = int(in.size()), R = int(outs.size());
    if (c->m > 8 && R > 0 && (c->m16_plans == 1 || (c->m16_plans == 2 && int64_t(K) * R >= (int64_t(1) << 16))))
        return build_plan_m16_device(c->device, targets, emit, sources, std::move(in), std::move(outs), out, st);
    std::vector<uint16_t> M = solve_matrix(targets, emit, sources);
    return build_plan(c->device, c->m, std::move(M), K, R, std::move(in), std::move(outs), out, st);
}

extern "C" int rsg_codec_create(int device, uint16_t k, uint16_t r, rsg_codec_t** out) {
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

extern "C" void rsg_codec_destroy(rsg_codec_t* c) { delete c; }

extern "C" int rsg_codec_subfield(const rsg_codec_t* c) { return c ? (c->m <= 8 ? 8 : 16) : 0; }

extern "C" int rsg_set_option(rsg_codec_t* c, const char* name, int64_t value) {
    if (!c || !name) return RS_ERR_INVALID;
    if (!std::strcmp(name, "m8_mode")) {
        if (value < 0 || (value > 4 && value < 10) || value > 19) return RS_ERR_INVALID;
#ifndef RS_AMD_DIAG  // 10-13, 15, 16, 19: timing ablations with wrong results; 17: s_memtime stamps
        if ((value >= 10 && value <= 13) || (value >= 15 && value <= 17) || value == 19) return RS_ERR_INVALID;
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
        if (value < 0 || value > 1) return RS_ERR_INVALID;
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
        c->cs_overlap = int(value);
        return 0;
    }
    if (!std::strcmp(name, "m16_ps_chunk")) {  // its stripes per chunk (0 = sized by m16_ps_rec_mib)
        if (value < 0 || value > 65535) return RS_ERR_INVALID;
        c->ps_chunk = value;
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
    if (!std::strcmp(name, "syn_route")) {
        if (value < 0 || value > 1) return RS_ERR_INVALID;
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

extern "C" const char* rsg_last_kernel(const rsg_codec_t* c) { return c ? c->last_kernel.c_str() : "none"; }

static int scratch_acquire(rsg_codec_t* c, hipStream_t st);
static int scratch_release(rsg_codec_t* c, hipStream_t st);

constexpr uint64_t kJitMinBytes = uint64_t(1) << 20;
// SALU per k_cs16t step: the step's own (asm_counts.h) + the block tails (3 each, 1 for the last) + the
// loop's pointer / count updates (7)
constexpr uint64_t kSaluStepCs16t = uint64_t(kSalu_cs16t) + 3 * (4 * kCs16tCw - 1) + 1 + 7;

// Syndrome route launch (p.cs): k_cs16 writes the D syndromes of a chunk of stripes to scratch, then the
// second stage applies the D x R matrix from there into the outputs.
static int run_plan(rsg_codec_t* c, DevPlan& p, const uint8_t* src, int64_t src_stripe, int64_t src_sym, uint8_t* dst,
                    int64_t dst_stripe, int64_t dst_sym, uint64_t n_stripes, uint64_t S, hipStream_t st,
                    const int32_t* d_ids = nullptr, bool dst_local = false);

// The codec's syndrome stream and its events (the per-stripe route and m16_cs_overlap)
static int overlap_objects(rsg_codec_t* c) {
    if (!c->ps_synst) HIP_TRY(hipStreamCreateWithFlags(&c->ps_synst, hipStreamNonBlocking));
    for (hipEvent_t* e : {&c->ps_ev_entry, &c->ps_ev_used[0], &c->ps_ev_used[1], &c->ps_ev_syn[0], &c->ps_ev_syn[1]})
        if (!*e) HIP_TRY(hipEventCreateWithFlags(e, hipEventDisableTiming));
    return 0;
}

constexpr int64_t kCsOverlapChunks = 4, kCsOverlapMinStripes = 16;

static int run_cs(rsg_codec_t* c, DevPlan& p, const uint8_t* src, int64_t src_stripe, int64_t src_sym, uint8_t* dst,
                  int64_t dst_stripe, int64_t dst_sym, uint64_t n_stripes, uint64_t S, hipStream_t st,
                  const int32_t* groups = nullptr) {
    const DevPlan::Cs& cs = *p.cs;
    if ((uintptr_t(src) | uintptr_t(dst) | uint64_t(src_stripe) | uint64_t(src_sym) | uint64_t(dst_stripe) |
         uint64_t(dst_sym)) % 4)
        return RS_ERR_INVALID;
    const uint16_t *logt = nullptr, *expt = nullptr;
    const uint8_t* g8 = nullptr;
    if (int rc = plan_tables(c->device, &logt, &g8, &expt)) return rc;
    // d_goff is codec scratch like d_cs: a launch on another stream may still read it (a route encode on
    // stream A, then a route decode on stream B rewrites it), so wait for that before overwriting it
    if (int rc = scratch_acquire(c, st)) return rc;
    const int ngo = (cs.ngroups + 3) * 16;
    if (int rc = grow(&c->d_goff[cs.kind], c->goff_cap[cs.kind], size_t(ngo) * 4)) return rc;
    HIP_TRY(launch_cs16_goff(groups ? groups : cs.groups, static_cast<uint32_t*>(c->d_goff[cs.kind]), ngo, src_sym, st));
    Cs16Args a{};
    a.src_stripe = src_stripe;
    a.src_sym = src_sym;
    a.goff = static_cast<const uint32_t*>(c->d_goff[cs.kind]);
    a.in_bytes = uint32_t(cs.max_slot * src_sym + int64_t(S));
    a.rec = cs.rec;
    a.fin = cs.fin;
    a.fin_off = cs.fin_off;
    a.fin_stride = cs.fin_stride;
    a.dst_sym = int64_t(S);
    a.logt = logt;
    a.expt = expt;
    for (int t = 0; t < 16; ++t) a.nblog[t] = cs.nblog[t];
    a.ngroups = cs.ngroups;
    a.ntiles = cs.ntiles;
    a.colw = c->m16_cs_col == 1024 ? 1024 : 256;
    a.nchunks = int64_t(S) / a.colw;
    const uint64_t waves_per_unit = uint64_t(a.colw / 256);  // per tile
    if (cs.kind == 1) {  // straight into the outputs
        a.src = src;
        a.dst = dst;
        a.dst_stripe = dst_stripe;
        a.dst_sym = dst_sym;
        a.units = int64_t(n_stripes) * a.nchunks;
        HIP_TRY(launch_bs16(a, st));
        const uint64_t steps = uint64_t(a.units) * waves_per_unit * uint64_t(cs.ntiles) * uint64_t(cs.ngroups);
        c->work_valu += steps * kValu_bs16;
        c->work_salu += steps * kSalu_bs16;
        c->last_kernel = "bs16";
        return scratch_release(c, st);
    }
    const bool thr = c->m16_cs_thread && cs.rec_t;
    if (thr) {  // k_cs16t's own tiling
        a.rec = cs.rec_t;
        a.fin = cs.fin_t;
        a.fin_off = cs.fin_off_t;
        a.fin_stride = cs.fin_stride_t;
        a.ntiles = cs.ntiles_t;
        a.cw = kCs16tCw;
    }
    const int64_t per = int64_t(cs.D) * int64_t(S);
    int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(int64_t(n_stripes), (int64_t(1) << 30) / per));
    // option m16_cs_overlap: at least kCsOverlapChunks chunks, chunk i + 1's syndromes on the codec's
    // syndrome stream (other buffer) beside chunk i's second stage on st
    const bool ovl = c->cs_overlap && int64_t(n_stripes) >= kCsOverlapMinStripes;
    if (ovl) chunk = std::min<int64_t>(chunk, (int64_t(n_stripes) + kCsOverlapChunks - 1) / kCsOverlapChunks);
    if (int rc = grow(&c->d_cs, c->cs_cap, size_t((ovl ? 2 : 1) * chunk * per))) return rc;
    hipStream_t sy = st;
    if (ovl) {
        if (int rc = overlap_objects(c)) return rc;
        sy = c->ps_synst;
        HIP_TRY(hipEventRecord(c->ps_ev_entry, st));  // after the d_goff upload above
        HIP_TRY(hipStreamWaitEvent(sy, c->ps_ev_entry, 0));
    }
    std::string second;
    for (int64_t c0 = 0, ci = 0; c0 < int64_t(n_stripes); c0 += chunk, ++ci) {
        const int64_t cn = std::min<int64_t>(chunk, int64_t(n_stripes) - c0);
        const int set = int(ci & 1);
        uint8_t* csb = static_cast<uint8_t*>(c->d_cs) + (ovl ? set * chunk * per : 0);
        if (ovl && ci >= 2) HIP_TRY(hipStreamWaitEvent(sy, c->ps_ev_used[set], 0));  // buffer read by chunk ci - 2
        a.src = src + c0 * src_stripe;
        a.dst = csb;
        a.dst_stripe = per;
        a.units = cn * a.nchunks;
        if (thr) {
            HIP_TRY(launch_cs16t(a, sy));
            c->work_valu += uint64_t(a.units) * waves_per_unit * cs.valu_t;
            c->work_salu += uint64_t(a.units) * waves_per_unit * uint64_t(cs.ntiles_t) * uint64_t(cs.ngroups) * kSaluStepCs16t;
        } else {
            HIP_TRY(launch_cs16(a, sy));
            const uint64_t steps = uint64_t(a.units) * waves_per_unit * uint64_t(cs.ntiles) * uint64_t(cs.ngroups);
            c->work_valu += steps * kValu_cs16a;  // cs16a and cs16b issue the same counts
            c->work_salu += steps * kSalu_cs16a;
        }
        if (ovl) {
            HIP_TRY(hipEventRecord(c->ps_ev_syn[set], sy));
            HIP_TRY(hipStreamWaitEvent(st, c->ps_ev_syn[set], 0));
        }
        if (int rc = run_plan(c, *p.second, csb, per, int64_t(S), dst + c0 * dst_stripe, dst_stripe, dst_sym,
                              uint64_t(cn), S, st))
            return rc;
        if (ovl) HIP_TRY(hipEventRecord(c->ps_ev_used[set], st));
        second = c->last_kernel;
    }
    c->last_kernel = (thr ? "cs16t+" : "cs16+") + second;
    return scratch_release(c, st);
}

// The re-encode decode (DevPlan::Reenc) over a chunk loop: the encode route over U into scratch rows
// (G_U u), + the received repair rows, then D_Rep from scratch into the erased information slots.
static int run_reenc(rsg_codec_t* c, DevPlan& p, uint8_t* base, int64_t stripe_stride, int64_t sym,
                     uint64_t n_stripes, uint64_t S, hipStream_t st) {
    DevPlan& E = *c->enc;
    if (int rc = E.order_after_build(st)) return rc;  // its records are read directly (run_cs, not run_plan)
    const int64_t k = c->k, r = c->r, per = r * int64_t(S);
    const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>({int64_t(n_stripes), (int64_t(1) << 30) / per, 65535}));
    if (int rc = scratch_acquire(c, st)) return rc;
    if (int rc = grow(&c->d_reenc, c->reenc_cap, size_t(chunk * per))) return rc;
    uint8_t* y = static_cast<uint8_t*>(c->d_reenc);
    std::string k1, k2;
    for (int64_t c0 = 0; c0 < int64_t(n_stripes); c0 += chunk) {
        const int64_t cn = std::min<int64_t>(chunk, int64_t(n_stripes) - c0);
        uint8_t* b = base + c0 * stripe_stride;
        if (int rc = run_cs(c, E, b, stripe_stride, sym, y, per, int64_t(S), uint64_t(cn), S, st, p.reenc->groups))
            return rc;
        k1 = c->last_kernel;  // the encode route over U: "cs16t+bs16" / "cs16+bs16"
        HIP_TRY(launch_xor_rows(y, per, int64_t(S), b + k * sym, stripe_stride, sym, r, int64_t(S), cn, st));
        if (int rc = run_plan(c, *p.reenc->drep, y, per, int64_t(S), b, stripe_stride, sym, uint64_t(cn), S, st))
            return rc;
        k2 = c->last_kernel;
    }
    c->last_kernel = k1 + "+xor+" + k2;
    // the encode plan's records were read by these launches: its guard must cover them (run_plan does
    // this for the plans it launches; E is launched through run_cs directly)
    if (int rc = E.note_use(st)) return rc;
    return scratch_release(c, st);
}

static int run_plan_body(rsg_codec_t* c, DevPlan& p, const uint8_t* src, int64_t src_stripe, int64_t src_sym,
                         uint8_t* dst, int64_t dst_stripe, int64_t dst_sym, uint64_t n_stripes, uint64_t S,
                         hipStream_t st, const int32_t* d_ids, bool dst_local);

static int run_plan(rsg_codec_t* c, DevPlan& p, const uint8_t* src, int64_t src_stripe, int64_t src_sym, uint8_t* dst,
                    int64_t dst_stripe, int64_t dst_sym, uint64_t n_stripes, uint64_t S, hipStream_t st,
                    const int32_t* d_ids, bool dst_local) {
    if (p.R == 0 || n_stripes == 0 || S == 0) return 0;
    const int rc = run_plan_body(c, p, src, src_stripe, src_sym, dst, dst_stripe, dst_sym, n_stripes, S, st, d_ids,
                                 dst_local);
    const int rc2 = p.note_use(st);  // after the launches (also a failed call's partial ones)
    return rc ? rc : rc2;
}

static int run_plan_body(rsg_codec_t* c, DevPlan& p, const uint8_t* src, int64_t src_stripe, int64_t src_sym,
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
                const bool re = reenc_eligible(c, er.get()) && src == dst && src_stripe == dst_stripe &&
                                src_sym == dst_sym && (c->k + c->r) * src_sym < (int64_t(1) << 31) &&
                                int64_t(c->r) * int64_t(S) < (int64_t(1) << 31);
                if (int rc = re ? make_plan_reenc(c, er.get(), p.route, st) : make_plan_cs(c, er.get(), p.route, st))
                    return rc;
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
    const bool m8_generic = p.m == 8 && p.d_idx && a.mode == 18 && !(xj_ok && p.xj) && !(jit_ok && p.jit);
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

extern "C" int rsg_last_work(const rsg_codec_t* c, uint64_t* valu, uint64_t* salu) {
    if (!c) return RS_ERR_INVALID;
    if (valu) *valu = c->work_valu;
    if (salu) *salu = c->work_salu;
    return 0;
}

extern "C" int rsg_encode(rsg_codec_t* c, const void* d_info, uint64_t info_stripe_stride, uint64_t info_symbol_stride,
                          void* d_rep, uint64_t rep_stripe_stride, uint64_t rep_symbol_stride, uint64_t n_stripes,
                          uint64_t symbol_size, void* stream) {
    if (!c) return RS_ERR_INVALID;
    c->work_valu = c->work_salu = 0;
    return run_plan(c, *c->enc, static_cast<const uint8_t*>(d_info), int64_t(info_stripe_stride),
                    int64_t(info_symbol_stride), static_cast<uint8_t*>(d_rep), int64_t(rep_stripe_stride),
                    int64_t(rep_symbol_stride), n_stripes, symbol_size, static_cast<hipStream_t>(stream));
}

static int decode_plan(rsg_codec_t* c, const bool* is_erased, uint16_t t, DevPlan** out, hipStream_t st) {
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

extern "C" int rsg_decode(rsg_codec_t* c, void* d_rcv, uint64_t stripe_stride, uint64_t symbol_stride,
                          uint64_t n_stripes, uint64_t symbol_size, const bool* is_erased, uint16_t t, void* stream) {
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

// rsg_decode_batch scratch: wait until the previous call's launches are done with it / mark this one's
static int scratch_acquire(rsg_codec_t* c, hipStream_t st) {
    // work queued earlier on the same stream runs first anyway; another stream's is waited for
    if (c->scratch_pending && c->scratch_stream != st) HIP_TRY(hipEventSynchronize(c->scratch_ev));
    c->scratch_pending = false;
    return 0;
}
static int scratch_release(rsg_codec_t* c, hipStream_t st) {
    if (!c->scratch_ev) HIP_TRY(hipEventCreateWithFlags(&c->scratch_ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(c->scratch_ev, st));
    c->scratch_pending = true;
    c->scratch_stream = st;
    return 0;
}

// Distinct patterns beyond which rsg_decode_batch builds the decode matrices on the device (the
// host plan cache holds 16; past it every pattern would cost a host build, an upload and a launch).
constexpr size_t kHostPlanGroups = 16;

// Syndrome route eligibility: the r x (k + r) syndrome matrix H[j][i] = X_i^j runs on its bit-plane XOR
// kernel (built once per codec), which covers whole 2 KiB column blocks only.
static bool syn_prepare(rsg_codec_t* c, uint64_t S, int64_t symbol_stride) {
    const int n = int(c->k) + c->r;
    if (!c->syn_route || c->syn_failed || !c->xj || c->jit == 0 || c->m > 8 || S % 2048 || !xj_supported(8, n, c->r) ||
        int64_t(n) * symbol_stride >= (int64_t(1) << 31) || int64_t(c->r) * int64_t(S) >= (int64_t(1) << 31))
        return false;
    if (!c->syn) {
        const Field& F = field();
        std::vector<uint16_t> H(size_t(c->r) * n);
        for (int j = 0; j < c->r; ++j)
            for (int i = 0; i < n; ++i) H[size_t(j) * n + i] = F.exp[(uint64_t(c->positions[i]) * j) % kN];
        std::vector<int32_t> in(n), out(c->r);
        for (int i = 0; i < n; ++i) in[size_t(i)] = i;
        for (int j = 0; j < c->r; ++j) out[size_t(j)] = j;
        std::unique_ptr<DevPlan> p;
        if (build_plan(c->device, 8, std::move(H), n, c->r, std::move(in), std::move(out), p, nullptr) || !p ||
            hipStreamSynchronize(nullptr) != hipSuccess) {
            c->syn_failed = true;
            return false;
        }
        if (xj_build(p->matrix, p->K, p->R, p->in_slots, p->out_slots, p->xj) || !p->xj) {
            std::fprintf(stderr, "librs_amd: syndrome XOR kernel unavailable; per-stripe survivor plans\n");
            c->syn_failed = true;
            return false;
        }
        c->syn = std::move(p);
    }
    return true;
}

// Nonzero bytes of [p, p + len): an erasure pattern's set entries (a bool is erased when nonzero, as in
// reed_solomon.c's `if (is_erased[i])`). Vectorises; the 32-bit partial sums cannot overflow.
static size_t count_nonzero(const uint8_t* p, size_t len) {
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
static uint64_t hash_bytes(const uint8_t* p, size_t len) {
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
static int decode_batch_device_plans(rsg_codec_t* c, uint8_t* base, int64_t stripe_stride, int64_t symbol_stride,
                                     uint64_t n_stripes, uint64_t S, const bool* is_erased, hipStream_t st) {
    const size_t n = size_t(c->k) + c->r;
    if ((S & 1) || (uintptr_t(base) % 8) || (stripe_stride % 8) || (symbol_stride % 8)) return RS_ERR_INVALID;
    std::vector<int32_t> ids;
    std::vector<uint8_t> masks;
    masks.reserve(size_t(n_stripes) * n);
    for (uint64_t s = 0; s < n_stripes; ++s) {
        const uint8_t* e = reinterpret_cast<const uint8_t*>(is_erased + s * n);
        if (!count_nonzero(e, c->k)) continue;
        ids.push_back(int32_t(s));
        const size_t o = masks.size();
        masks.resize(o + n);
        for (size_t i = 0; i < n; ++i) masks[o + i] = e[i] != 0;
    }
    if (ids.empty()) return 0;
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
    // the host lists must outlive the copies: upload on the caller's stream, then wait once
    HIP_TRY(hipMemcpyAsync(c->d_ids, ids.data(), ids.size() * 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(c->d_masks, masks.data(), masks.size(), hipMemcpyHostToDevice, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (syn_prepare(c, S, symbol_stride)) {
        // syndrome route: zero erased information slots + build the t_info x t solves (k_plan_syn_m8),
        // the r syndromes of every selected stripe into scratch (XOR kernel, dst indexed by the chunk-
        // local stripe), then the per-stripe solves from the syndromes into the erased information slots
        const uint16_t* expt = nullptr;
        if ((rc = plan_tables(c->device, &logt, &g8, &expt))) return rc;
        const int64_t per = int64_t(c->r) * int64_t(S);
        const int64_t sch = std::max<int64_t>(1, std::min<int64_t>(chunk, (int64_t(1) << 30) / per));
        if ((rc = grow(&c->d_syn, c->syn_cap, size_t(sch * per)))) return rc;
        for (int64_t c0 = 0; c0 < nsel; c0 += sch) {
            const int64_t cn = std::min(sch, nsel - c0);
            SynPlanArgs pa{};
            pa.masks = static_cast<const uint8_t*>(c->d_masks) + size_t(c0) * n;
            pa.elem = c->d_elem;
            pa.logt = logt;
            pa.expt = expt;
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
            pa.base = base;
            pa.stripe_stride = stripe_stride;
            pa.symbol_stride = symbol_stride;
            pa.S = int64_t(S);
            pa.ids = c->d_ids + c0;
            HIP_TRY(launch_plan_syn_m8(pa, cn, st));
            uint8_t* syn = static_cast<uint8_t*>(c->d_syn);
            if ((rc = run_plan(c, *c->syn, base, stripe_stride, symbol_stride, syn, per, int64_t(S), uint64_t(cn), S,
                               st, c->d_ids + c0, true)))
                return rc;
            V1Args v{};
            v.src = syn;
            v.src_stripe = 0;  // slots are local * r + j
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
            HIP_TRY(launch_apply_m8_ps(v, cn, int64_t(S), tiles, st));
        }
        c->last_kernel = "syn_xj+apply_m8_v1_ps";
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
        HIP_TRY(launch_apply_m8_ps(v, cn, int64_t(S), tiles, st));
    }
    c->last_kernel = "apply_m8_v1_ps";
    return scratch_release(c, st);
}

// ---------------------------------------------------------------- host-memory batches (PCIe)
// Stripes in host memory: batches of stripes alternate over two streams, each H2D -> kernel -> D2H,
// so one batch's kernel overlaps the other's copies and H2D overlaps D2H. Pinned host memory
// (hipHostMalloc / hipHostRegister) runs the copies at PCIe rate; pageable memory works, slower.
static constexpr size_t kHostBatchBytes = size_t(256) << 20;  // device buffer per stream

static int host_pipe_reserve(rsg_codec_t* c, size_t bytes) {
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

extern "C" int rsg_encode_host(rsg_codec_t* c, const void* h_info, uint64_t info_stripe_stride,
                               uint64_t info_symbol_stride, void* h_rep, uint64_t rep_stripe_stride,
                               uint64_t rep_symbol_stride, uint64_t n_stripes, uint64_t symbol_size) {
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

// rsg_decode_batch, GF(2^16) codes past kHostPlanGroups patterns: the codec's one batch plan is rebuilt
// on the stream for every pattern by k_plan16_sums / k_plan16_fill -- the same evaluation and formats as
// build_plan_m16_device, so results are identical -- instead of a cached plan per pattern (allocations,
// synchronous uploads and, past 16 patterns, an eviction that frees device memory). Launches on one
// stream are ordered, so the plan of the next pattern is written after the previous apply has read it;
// only the host staging needs a ring (two pinned buffers, each guarded by the event after its copies).
static size_t al16(size_t v) { return (v + 15) & ~size_t(15); }

static int batch_plan_m16(rsg_codec_t* c, const bool* er, int slot, hipStream_t st, DevPlan** out) {
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
static bool ps16_eligible(const rsg_codec_t* c, uint64_t S, int64_t stripe_stride, int64_t symbol_stride,
                          const void* base) {
    const int64_t n = int64_t(c->k) + c->r;
    return c->m > 8 && c->m16_ps && c->r <= kPs16MaxR && S % 1024 == 0 && int64_t(S) < (int64_t(1) << 31) &&
           (n - 1) * symbol_stride + int64_t(S) < (int64_t(1) << 31) && int64_t(c->r) * int64_t(S) < (int64_t(1) << 31) &&
           (stripe_stride % 16) == 0 && (symbol_stride % 16) == 0 && (uintptr_t(base) % 16) == 0 &&
           symbol_stride >= int64_t(S);
}

static int ps16_syn_plan(rsg_codec_t* c, int D, hipStream_t st, DevPlan** out) {
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

// tr: per stripe, t (erasures) and R (erased information slots), counted by rsg_decode_batch
static int decode_batch_m16_ps(rsg_codec_t* c, uint8_t* base, int64_t stripe_stride, int64_t symbol_stride,
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
    // the host lists must outlive the copies: upload on the caller's stream, then wait once
    HIP_TRY(hipMemcpyAsync(c->d_ids, ids.data(), ids.size() * 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(c->d_masks, mask_src, ids.size() * n, hipMemcpyHostToDevice, st));
    HIP_TRY(launch_cs16_goff(cs.groups, static_cast<uint32_t*>(c->d_goff[0]), ngo, symbol_stride, st));
    HIP_TRY(hipStreamSynchronize(st));
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
        HIP_TRY(hipEventRecord(c->ps_ev_used[set], st));
    }
    if ((rc = syn->note_use(st))) return rc;
    c->last_kernel = thr ? "ps16+cs16t+apply_m16_v1_ps" : "ps16+cs16+apply_m16_v1_ps";
    return scratch_release(c, st);
}

extern "C" int rsg_decode_batch(rsg_codec_t* c, void* d_rcv, uint64_t stripe_stride, uint64_t symbol_stride,
                                uint64_t n_stripes, uint64_t symbol_size, const bool* is_erased, void* stream) {
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
    for (uint64_t s = 0; s < n_stripes; ++s) {
        const uint8_t* e = reinterpret_cast<const uint8_t*>(is_erased + s * n);
        const size_t R = count_nonzero(e, c->k), t = R + count_nonzero(e + c->k, c->r);
        if (t > c->r) return RS_ERR_CANNOT_RESTORE;
        tr[2 * s] = int32_t(t);
        tr[2 * s + 1] = int32_t(R);
        if (!R) continue;  // nothing to restore (erased repair slots are never written)
        if (s > uint64_t(INT32_MAX)) return RS_ERR_INVALID;
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
    if (c->m <= 8 && n <= 256 &&
        (c->batch_plans == 1 || (c->batch_plans == 2 && groups.size() > kHostPlanGroups)))
        return decode_batch_device_plans(c, static_cast<uint8_t*>(d_rcv), int64_t(stripe_stride),
                                         int64_t(symbol_stride), n_stripes, symbol_size, is_erased, st);
    // GF(2^16): more than one pattern -> per-stripe plans on the syndrome route (one shared syndrome pass)
    if (c->m > 8 && (c->batch_plans == 1 || (c->batch_plans == 2 && groups.size() > 1)) &&
        ps16_eligible(c, symbol_size, int64_t(stripe_stride), int64_t(symbol_stride), d_rcv))
        return decode_batch_m16_ps(c, static_cast<uint8_t*>(d_rcv), int64_t(stripe_stride), int64_t(symbol_stride),
                                   n_stripes, symbol_size, is_erased, tr.data(), st);
    std::vector<int32_t> ids;
    std::vector<size_t> first;
    for (auto& g : groups) {
        first.push_back(ids.size());
        ids.insert(ids.end(), g.ids.begin(), g.ids.end());
    }
    if (int rc = scratch_acquire(c, st)) return rc;
    if (ids.size() > c->ids_cap) {
        if (c->d_ids) (void)hipFree(c->d_ids);
        c->d_ids = nullptr;
        c->ids_cap = 0;
        HIP_TRY(hipMalloc(&c->d_ids, ids.size() * 4));
        c->ids_cap = ids.size();
    }
    // the list must stay valid until the launches have read it: upload on the caller's stream
    HIP_TRY(hipMemcpyAsync(c->d_ids, ids.data(), ids.size() * 4, hipMemcpyHostToDevice, st));
    HIP_TRY(hipStreamSynchronize(st));
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
        int rc = stream_plans ? batch_plan_m16(c, er.get(), int(gi & 1), st, &p) : decode_plan(c, er.get(), t, &p, st);
        if (rc) return rc;
        // a pattern shared by every stripe, in order: no stripe-id list (the GF(2^16) route and the re-encode
        // decode cover only that form)
        const bool all = g.ids.size() == n_stripes && g.ids.front() == 0 && g.ids.back() == int32_t(n_stripes - 1);
        rc = run_plan(c, *p, base, int64_t(stripe_stride), int64_t(symbol_stride), base, int64_t(stripe_stride),
                      int64_t(symbol_stride), g.ids.size(), symbol_size, st, all ? nullptr : c->d_ids + first[gi]);
        if (rc) return rc;
        ++gi;
    }
    return scratch_release(c, st);
}

extern "C" int rsg_fill_info(void* d_base, uint64_t stripe_stride, uint64_t symbol_stride, uint64_t symbol_size,
                             uint16_t k, uint64_t stripe0, uint64_t n_stripes, uint64_t seed, void* stream) {
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
    if (matrix) std::memcpy(matrix, M.data(), M.size() * 2);
    if (in_slots) std::memcpy(in_slots, in.data(), in.size() * 4);
    if (out_slots) std::memcpy(out_slots, outs.data(), outs.size() * 4);
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

// ============================================================================ drop-in rs_*
namespace {

constexpr int kMaxChunks = 4;

inline size_t pad16(size_t s) { return (s + 15) & ~size_t(15); }

// Zero-copy eligibility of a per-call launch on arena-resident symbols: the plan's kernel reads each
// input column once and writes each output once -- the bit-plane XOR kernel, or any GF(256) kernel
// with a single 32-row tile (R <= 32; the generic one splits K on small grids) -- so it can stream the
// caller's page-locked symbols across PCIe itself: one launch instead of H2D DMA + launch + D2H DMA and
// their stream hand-offs. Kernels that re-read inputs per output tile (m = 16 tiles, the syndrome
// route) stay on the DMA path.
bool streams_once(const DevPlan& p, size_t S) {
    return p.m == 8 && ((p.xj && !p.xj_failed && S >= 2048) || p.R <= 32);
}
// Stripes up to this many bytes are latency-bound on any path: every kernel runs on them across PCIe
// (one launch, no copies), whatever its re-reads.
constexpr uint64_t kZcSmallBytes = uint64_t(1) << 20;

// Page-locked symbol arenas. seq_create places a sequence's symbols in one page-locked block at stride
// pad16(S) (its own hipHostMalloc block from kArenaMin bytes on, a share of a slab below), so
// rs_generate_repair_symbols / rs_restore_symbols run kernels on the caller's symbols across PCIe or
// DMA straight between them and HBM (no host gather / scatter, no staging copy). The
// registry maps a block's start to its size, device-visible address and live symbol count;
// symbol_destroy returns a block when its last symbol goes. RS_AMD_PINNED_SEQ=0 turns it off (plain
// calloc per symbol, as before).
constexpr size_t kArenaMin = size_t(1) << 20;
// Smaller sequences share page-locked slabs (bump-allocated, 256-byte aligned): pinning memory per
// small sequence would cost more than the call it serves. A slab's space is reused once every
// sequence in it is destroyed; past kMaxSlabs slabs small sequences go to the heap.
constexpr size_t kSlabBytes = size_t(8) << 20;
constexpr size_t kMaxSlabs = 16;  // at most 128 MiB of page-locked slabs
struct Slab {
    uint8_t* base;
    uint8_t* dev;
    size_t used = 0, live = 0;
};
struct Arena {
    size_t bytes;
    uint8_t* dev;  // device-visible address of the block start (nullptr: DMA only)
    size_t live;
    Slab* slab = nullptr;  // the slab the block lives in (nullptr: its own hipHostMalloc block)
};
struct ArenaRegistry {
    std::mutex mu;
    std::map<uintptr_t, Arena> blocks;
    std::vector<Slab*> slabs;
    bool no_pinning = false;  // page-locked allocation failed once (no GPU): heap from then on
    size_t pinned = 0;        // page-locked bytes held by blocks and slabs
};

// Process-wide cap on page-locked symbol memory (arenas, slabs and registered symbols): a quarter of
// physical RAM, or RS_AMD_PINNED_MAX_MB. Sequences past it go to the heap (the gather / scatter path), so
// a caller that creates many large sequences cannot page-lock most of the host without knowing it.
size_t pinned_cap() {
    static const size_t cap = [] {
        if (const char* e = std::getenv("RS_AMD_PINNED_MAX_MB")) return size_t(std::strtoull(e, nullptr, 10)) << 20;
        const long pages = sysconf(_SC_PHYS_PAGES), psz = sysconf(_SC_PAGESIZE);
        return pages > 0 && psz > 0 ? size_t(pages) * size_t(psz) / 4 : size_t(16) << 30;
    }();
    return cap;
}
ArenaRegistry& arenas() {
    static ArenaRegistry* r = new ArenaRegistry;  // never destroyed: symbols may outlive static destructors
    return *r;
}

// a zeroed, mapped page-locked block and its device-visible address (nullptr if none)
static uint8_t* pinned_block(size_t bytes, uint8_t** dev) {
    void* h = nullptr;
    if (hipHostMalloc(&h, bytes, hipHostMallocPortable | hipHostMallocMapped) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    std::memset(h, 0, bytes);
    void* dv = nullptr;
    if (hipHostGetDevicePointer(&dv, h, 0) != hipSuccess) {
        (void)hipGetLastError();
        dv = nullptr;
    }
    *dev = static_cast<uint8_t*>(dv);
    return static_cast<uint8_t*>(h);
}

uint8_t* arena_alloc(size_t length, size_t P) {
    const char* e = std::getenv("RS_AMD_PINNED_SEQ");
    const size_t bytes = length * P;
    if ((e && e[0] == '0') || bytes == 0) return nullptr;
    ArenaRegistry& r = arenas();
    std::lock_guard<std::mutex> lk(r.mu);
    if (r.no_pinning) return nullptr;
    if (bytes >= kArenaMin) {
        if (r.pinned + bytes > pinned_cap()) return nullptr;  // over the cap: heap symbols
        uint8_t* dv = nullptr;
        uint8_t* h = pinned_block(bytes, &dv);
        if (!h) {
            r.no_pinning = true;
            return nullptr;
        }
        r.blocks[uintptr_t(h)] = Arena{bytes, dv, length};
        r.pinned += bytes;
        return h;
    }
    const size_t need = (bytes + 255) & ~size_t(255);
    Slab* sl = nullptr;
    for (Slab* x : r.slabs)
        if (x->used + need <= kSlabBytes) {
            sl = x;
            break;
        }
    if (!sl) {
        if (r.slabs.size() >= kMaxSlabs || r.pinned + kSlabBytes > pinned_cap()) return nullptr;
        uint8_t* dv = nullptr;
        uint8_t* h = pinned_block(kSlabBytes, &dv);
        if (!h) {
            r.no_pinning = true;
            return nullptr;
        }
        sl = new Slab{h, dv};
        r.slabs.push_back(sl);
        r.pinned += kSlabBytes;
    }
    uint8_t* blk = sl->base + sl->used;
    std::memset(blk, 0, need);  // a reused slab holds old data
    r.blocks[uintptr_t(blk)] = Arena{bytes, sl->dev ? sl->dev + sl->used : nullptr, length, sl};
    sl->used += need;
    ++sl->live;
    return blk;
}

// true (and the block released when it was the last) when p lies in an arena
bool arena_release(const uint8_t* p) {
    ArenaRegistry& r = arenas();
    std::lock_guard<std::mutex> lk(r.mu);
    auto it = r.blocks.upper_bound(uintptr_t(p));
    if (it == r.blocks.begin()) return false;
    --it;
    if (uintptr_t(p) >= it->first + it->second.bytes) return false;
    if (--it->second.live == 0) {
        if (Slab* sl = it->second.slab) {
            if (--sl->live == 0) sl->used = 0;  // every sequence of the slab is gone: reuse its space
        } else {
            (void)hipHostFree(reinterpret_cast<void*>(it->first));
            (void)hipGetLastError();
            r.pinned -= it->second.bytes;
        }
        r.blocks.erase(it);
    }
    return true;
}

// The cnt symbols form one strided run inside one arena: symbols[i]->data == base + i * pitch with a
// 16-byte aligned base and pitch >= pad16(S). Returns base (nullptr otherwise); *dev = the run's
// device-visible address (nullptr when the block has none).
const uint8_t* arena_run(symbol_t* const* syms, size_t cnt, size_t S, size_t* pitch, uint8_t** dev) {
    if (!cnt || !syms[0]) return nullptr;
    const uint8_t* b = syms[0]->data;
    size_t p = pad16(S);
    if (cnt > 1) {
        if (!syms[1] || syms[1]->data <= b) return nullptr;
        p = size_t(syms[1]->data - b);
    }
    if (p < pad16(S) || (p & 15) || (uintptr_t(b) & 15)) return nullptr;
    for (size_t i = 2; i < cnt; ++i)
        if (!syms[i] || syms[i]->data != b + i * p) return nullptr;
    ArenaRegistry& r = arenas();
    std::lock_guard<std::mutex> lk(r.mu);
    auto it = r.blocks.upper_bound(uintptr_t(b));
    if (it == r.blocks.begin()) return nullptr;
    --it;
    if (uintptr_t(b) + (cnt - 1) * p + pad16(S) > it->first + it->second.bytes) return nullptr;
    *pitch = p;
    if (dev) *dev = it->second.dev ? it->second.dev + (uintptr_t(b) - it->first) : nullptr;
    return b;
}

// Caller-owned symbols outside the arenas (symbol_create; seq_create with RS_AMD_PINNED_SEQ=0): data of
// kRegMinBytes or more lives in whole pages of its own (sym_va_take), recorded here and page-locked and mapped at
// creation (hipHostRegister, within the pinned cap). A per-call use then moves such symbols with zero-copy
// or gather / scatter kernels across PCIe instead of host copies through staging. Only buffers this
// library allocated are registered: it alone knows when they are freed.
// A registered range is never handed back to the process for reuse: symbol_destroy parks it, still
// registered, in an idle pool (later symbol_create calls of a similar size take it back: no second
// registration), and past the pool's cap unregisters it and leaves its address range reserved with no
// memory behind it (PROT_NONE). Once-registered addresses reused by other allocations -- pageable torch /
// numpy buffers that the runtime copies into -- were followed by GPU faults in those copies.
constexpr size_t kRegMinBytes = size_t(16) << 10;
constexpr size_t kPage = 4096;
struct SymEnt {
    size_t bytes;         // whole pages
    uint8_t* dev;         // device-visible address once registered
};
struct SymRegistry {
    std::mutex mu;
    std::unordered_map<uintptr_t, SymEnt> m;  // live symbols
    size_t idle_bytes = 0;                    // blocks parked in sym_idle()
    uint8_t* va_base = nullptr;               // current address reservation (sym_va_take)
    size_t va_size = 0, va_used = 0;
};
SymRegistry& symreg() {
    static SymRegistry* r = new SymRegistry;  // never destroyed: symbols may outlive static destructors
    return *r;
}
size_t sym_pool_cap() {
    static const size_t cap = [] {
        if (const char* e = std::getenv("RS_AMD_SYM_POOL_MB")) return size_t(std::strtoull(e, nullptr, 10)) << 20;
        return size_t(1) << 30;
    }();
    return cap;
}

bool sym_register(uint8_t* p, SymEnt& e);

// Fresh pages at increasing addresses from a reserved address range (64 GiB per reservation, no memory
// behind it until used), so consecutive symbol_create calls of one size sit at one stride (the zero-copy
// kernels' condition) and no address is ever handed out twice except through the idle pool.
uint8_t* sym_va_take(SymRegistry& R, size_t bytes) {
    if (!R.va_base || R.va_used + bytes > R.va_size) {
        const size_t sz = std::max(size_t(64) << 30, bytes);
        void* r = mmap(nullptr, sz, PROT_NONE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
        if (r == MAP_FAILED) return nullptr;
        R.va_base = static_cast<uint8_t*>(r);
        R.va_size = sz;
        R.va_used = 0;
    }
    uint8_t* p = R.va_base + R.va_used;
    if (mmap(p, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_FIXED, -1, 0) == MAP_FAILED)
        return nullptr;
    R.va_used += bytes;
    return p;
}

// back to a reserved range without memory (the address is never reused)
void sym_va_retire(uint8_t* p, size_t bytes) {
    (void)mmap(p, bytes, PROT_NONE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_FIXED | MAP_NORESERVE, -1, 0);
}

// a parked block (registered, or not when the cap or a missing GPU refused it): host address and entry
struct IdleBlock {
    uint8_t* host;
    SymEnt e;
};
std::multimap<size_t, IdleBlock>& sym_idle() {
    static auto* m = new std::multimap<size_t, IdleBlock>;  // guarded by symreg().mu
    return *m;
}

uint8_t* sym_alloc(size_t S) {
    if (S < kRegMinBytes) return nullptr;
    const size_t bytes = (S + kPage - 1) / kPage * kPage;
    SymRegistry& R = symreg();
    {
        std::lock_guard<std::mutex> lk(R.mu);
        auto& idle = sym_idle();
        auto it = idle.lower_bound(bytes);
        if (it != idle.end() && it->first <= 2 * bytes) {  // a parked registered block of a similar size
            IdleBlock b = it->second;
            idle.erase(it);
            R.idle_bytes -= b.e.bytes;
            std::memset(b.host, 0, b.e.bytes);
            SymEnt& e = R.m[uintptr_t(b.host)] = b.e;
            (void)sym_register(b.host, e);  // parked unregistered (cap, no GPU then): try again
            return b.host;
        }
    }
    std::lock_guard<std::mutex> lk(R.mu);
    uint8_t* p = sym_va_take(R, bytes);
    if (!p) return nullptr;
    SymEnt& e = R.m[uintptr_t(p)] = SymEnt{bytes, nullptr};
    // page-lock it now, as seq_create's arenas are (the per-call path then never pays for it); a failure
    // (no GPU, the pinned cap) leaves it to the first use
    (void)sym_register(static_cast<uint8_t*>(p), e);
    return static_cast<uint8_t*>(p);
}

// page-locks and maps one registry entry (its mutex held); false when the cap or the runtime refuses
bool sym_register(uint8_t* p, SymEnt& e) {
    if (e.dev) return true;
    ArenaRegistry& A = arenas();
    {
        std::lock_guard<std::mutex> la(A.mu);
        if (A.no_pinning || A.pinned + e.bytes > pinned_cap()) return false;
        A.pinned += e.bytes;
    }
    // never touch a range the runtime already knows: a failed registration must not be followed by an
    // unregister, which would remove the owner's mapping
    hipPointerAttribute_t attr{};
    const bool known = hipPointerGetAttributes(&attr, p) == hipSuccess && attr.type != hipMemoryTypeUnregistered;
    (void)hipGetLastError();
    bool ok = !known && hipHostRegister(p, e.bytes, hipHostRegisterMapped | hipHostRegisterPortable) == hipSuccess;
    void* dv = nullptr;
    if (ok && hipHostGetDevicePointer(&dv, p, 0) != hipSuccess) {
        (void)hipHostUnregister(p);  // ours: registered just above
        ok = false;
    }
    (void)hipGetLastError();
    if (!ok) {
        std::lock_guard<std::mutex> la(A.mu);
        A.pinned -= e.bytes;
        return false;
    }
    e.dev = static_cast<uint8_t*>(dv);
    return true;
}

// true (and p parked or released) when p came from sym_alloc
bool sym_release(uint8_t* p) {
    SymRegistry& R = symreg();
    SymEnt e;
    {
        std::lock_guard<std::mutex> lk(R.mu);
        auto it = R.m.find(uintptr_t(p));
        if (it == R.m.end()) return false;
        e = it->second;
        R.m.erase(it);
        if (R.idle_bytes + e.bytes <= sym_pool_cap()) {
            sym_idle().emplace(e.bytes, IdleBlock{p, e});
            R.idle_bytes += e.bytes;
            return true;
        }
        if (!e.dev) {  // never registered
            sym_va_retire(p, e.bytes);
            return true;
        }
    }
    // over the pool's cap: unregister, then keep the address range reserved without memory behind it
    (void)hipHostUnregister(p);
    (void)hipGetLastError();
    sym_va_retire(p, e.bytes);
    ArenaRegistry& A = arenas();
    std::lock_guard<std::mutex> lk(A.mu);
    A.pinned -= e.bytes;
    return true;
}

// device-visible addresses of cnt symbols of at least S bytes, all from sym_alloc, registering the ones
// not yet registered; false (nothing to do for the caller's fast path) when any is not eligible
bool sym_devptrs(symbol_t* const* syms, size_t cnt, size_t S, uint64_t* out) {
    SymRegistry& R = symreg();
    std::lock_guard<std::mutex> lk(R.mu);
    for (size_t i = 0; i < cnt; ++i) {
        if (!syms[i]) return false;
        auto it = R.m.find(uintptr_t(syms[i]->data));
        if (it == R.m.end() || it->second.bytes < S) return false;
        if (!it->second.dev && !sym_register(syms[i]->data, it->second)) return false;
        out[i] = uint64_t(reinterpret_cast<uintptr_t>(it->second.dev));
    }
    return true;
}

// cnt device addresses at one stride >= S (16-byte aligned) with 32-bit kernel offsets; *pitch = it
bool strided_run(const uint64_t* p, size_t cnt, size_t S, size_t* pitch) {
    if (!cnt || (p[0] & 15)) return false;
    const uint64_t d = cnt > 1 ? p[1] - p[0] : pad16(S);
    if (cnt > 1 && (p[1] <= p[0] || d < S || (d & 15))) return false;
    for (size_t i = 2; i < cnt; ++i)
        if (p[i] != p[0] + i * d) return false;
    if ((cnt - 1) * d + S >= (uint64_t(1) << 31)) return false;
    *pitch = size_t(d);
    return true;
}

struct Impl {
    int device = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;
    std::map<std::pair<uint16_t, uint16_t>, std::unique_ptr<rsg_codec>> codecs;
    uint8_t* h_buf = nullptr;
    uint8_t* d_buf = nullptr;
    size_t cap = 0;
    std::unique_ptr<HostPool> pool;  // gather / scatter workers
    hipEvent_t ev[kMaxChunks] = {};
    // arena-resident symbols: chunk c + 1's H2D DMA runs on in_stream while chunk c is encoded /
    // decoded and copied back on stream (ev_in[c] orders the kernel after its columns arrived)
    hipStream_t in_stream = nullptr;
    hipEvent_t ev_in[kMaxChunks] = {};
    // arena-resident stripes: column chunks per call (RS_AMD_DROPIN_CHUNKS, 1..kMaxChunks) and whether
    // repair symbols go back by k_put_rows writes instead of DMA (RS_AMD_DROPIN_PUT)
    int arena_chunks = 2;
    bool arena_put = true;
    bool arena_zc = true;  // RS_AMD_DROPIN_ZC=0: no zero-copy launches (see streams_once)
    int reg_chunks = 1;    // registered caller symbols: column chunks per call (RS_AMD_REG_CHUNKS, 1..kMaxChunks)
    int32_t* h_rows = nullptr;  // pinned / device row list of the decode's packed copy-back
    int32_t* d_rows = nullptr;
    size_t rows_cap = 0;
    // registered caller symbols: [n] device-visible symbol addresses, [n] gathered rows, [n] scattered
    // rows (pinned; uploaded by one copy per call)
    uint8_t* h_ptrs = nullptr;
    uint8_t* d_ptrs = nullptr;
    size_t ptrs_cap = 0;
    int reserve_ptrs(size_t n) {
        if (n <= ptrs_cap) return 0;
        if (h_ptrs) (void)hipHostFree(h_ptrs);
        if (d_ptrs) (void)hipFree(d_ptrs);
        h_ptrs = d_ptrs = nullptr;
        ptrs_cap = 0;
        if (hipHostMalloc(reinterpret_cast<void**>(&h_ptrs), n * 16, hipHostMallocDefault) != hipSuccess) return 1;
        if (hipMalloc(reinterpret_cast<void**>(&d_ptrs), n * 16) != hipSuccess) return 1;
        ptrs_cap = n;
        return 0;
    }
    ~Impl() {
        (void)hipSetDevice(device);
        codecs.clear();
        if (h_rows) (void)hipHostFree(h_rows);
        if (d_rows) (void)hipFree(d_rows);
        if (h_ptrs) (void)hipHostFree(h_ptrs);
        if (d_ptrs) (void)hipFree(d_ptrs);
        for (hipEvent_t e : ev)
            if (e) (void)hipEventDestroy(e);
        for (hipEvent_t e : ev_in)
            if (e) (void)hipEventDestroy(e);
        if (in_stream) (void)hipStreamDestroy(in_stream);
        if (h_buf) (void)hipHostFree(h_buf);
        if (d_buf) (void)hipFree(d_buf);
        if (stream) (void)hipStreamDestroy(stream);
    }
    int reserve(size_t bytes) {
        if (bytes <= cap) return 0;
        if (h_buf) (void)hipHostFree(h_buf);
        if (d_buf) (void)hipFree(d_buf);
        h_buf = nullptr;
        d_buf = nullptr;
        cap = 0;
        if (hipHostMalloc(reinterpret_cast<void**>(&h_buf), bytes, hipHostMallocDefault) != hipSuccess) return 1;
        if (hipMalloc(reinterpret_cast<void**>(&d_buf), bytes) != hipSuccess) return 1;
        cap = bytes;
        return 0;
    }
    int codec(uint16_t k, uint16_t r, rsg_codec** out) {
        auto key = std::make_pair(k, r);
        auto it = codecs.find(key);
        if (it == codecs.end()) {
            rsg_codec* c = nullptr;
            int rc = rsg_codec_create(device, k, r, &c);
            if (rc) return rc;
            // a decode call launches once until its plan is specialised (rs_restore_symbols):
            // specialise a pattern from its third call on
            c->dec_jit_uses = 3;
            it = codecs.emplace(key, std::unique_ptr<rsg_codec>(c)).first;
        }
        *out = it->second.get();
        return 0;
    }
};

// Column chunks of one per-call stripe: large symbols are split into up to kMaxChunks column ranges
// (multiples of the 2 KiB kernel block), so the host gather of chunk c + 1 and the scatter of chunk
// c - 1 overlap the copies and kernel of chunk c.
size_t chunk_width(size_t S, int maxc = kMaxChunks) {
    if (S < 4 * 8192 || maxc <= 1) return S;
    const size_t w = (S + maxc - 1) / maxc;
    return (w + 2047) / 2048 * 2048;
}

}  // namespace

extern "C" RS_t* rs_create(void) {
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev == 0) {
        std::fprintf(stderr, "librs_amd: rs_create: no usable HIP device (%s); there is no CPU fallback\n",
                     hipGetErrorString(e));
        return nullptr;
    }
    RS_t* rs = static_cast<RS_t*>(std::calloc(1, sizeof(RS_t)));
    if (!rs) return nullptr;
    rs->gf = gf_create();
    rs->cc = cc_create();
    auto* impl = new (std::nothrow) Impl();
    if (!rs->gf || !rs->cc || !impl) {
        delete impl;
        if (rs->gf) gf_destroy(rs->gf);
        if (rs->cc) cc_destroy(rs->cc);
        std::free(rs);
        return nullptr;
    }
    (void)hipGetDevice(&impl->device);
    int workers = int(std::min(8u, std::max(1u, std::thread::hardware_concurrency()))) - 1;
    if (const char* e = std::getenv("RS_AMD_HOST_THREADS")) workers = std::max(0, std::atoi(e) - 1);
    impl->pool = std::make_unique<HostPool>(workers);
    if (const char* e = std::getenv("RS_AMD_DROPIN_CHUNKS")) impl->arena_chunks = std::clamp(std::atoi(e), 1, kMaxChunks);
    if (const char* e = std::getenv("RS_AMD_DROPIN_PUT")) impl->arena_put = e[0] == '1';
    if (const char* e = std::getenv("RS_AMD_DROPIN_ZC")) impl->arena_zc = e[0] != '0';
    if (const char* e = std::getenv("RS_AMD_REG_CHUNKS")) impl->reg_chunks = std::clamp(std::atoi(e), 1, kMaxChunks);
    bool ev_ok = true;
    for (hipEvent_t& e : impl->ev) ev_ok = ev_ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
    for (hipEvent_t& e : impl->ev_in) ev_ok = ev_ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
    if (!ev_ok || hipStreamCreateWithFlags(&impl->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&impl->in_stream, hipStreamNonBlocking) != hipSuccess) {
        delete impl;
        gf_destroy(rs->gf);
        cc_destroy(rs->cc);
        std::free(rs);
        return nullptr;
    }
    rs->impl = impl;
    return rs;
}

extern "C" void rs_destroy(RS_t* rs) {
    if (!rs) return;
    delete static_cast<Impl*>(rs->impl);
    gf_destroy(rs->gf);
    cc_destroy(rs->cc);
    std::free(rs);
}

extern "C" int rs_generate_repair_symbols(RS_t* rs, const symbol_seq_t* inf, symbol_seq_t* rep) {
    if (!rs || !rs->impl || !inf || !rep) return RS_ERR_INVALID;
    Impl& im = *static_cast<Impl*>(rs->impl);
    const size_t S = inf->symbol_size;
    if (S != rep->symbol_size || (S & 1) || inf->length + rep->length > kN) return RS_ERR_INVALID;
    const uint16_t k = uint16_t(inf->length), r = uint16_t(rep->length);
    if (r == 0 || S == 0) return 0;
    std::lock_guard<std::mutex> lk(im.mu);
    HIP_TRY(hipSetDevice(im.device));
    rsg_codec* c = nullptr;
    int rc = im.codec(k, r, &c);
    if (rc) return rc;
    // symbols in page-locked arenas (seq_create) are copied in place by DMA; otherwise they are gathered
    // into / scattered from the pinned staging buffer by the host pool
    size_t ip = 0, rp = 0;
    uint8_t* idev = nullptr;
    const uint8_t* ib = arena_run(inf->symbols, k, S, &ip, &idev);
    uint8_t* rdev = nullptr;
    uint8_t* rb = const_cast<uint8_t*>(arena_run(rep->symbols, r, S, &rp, &rdev));
    const size_t P = pad16(S), n = size_t(k) + r, W = chunk_width(S, ib ? im.arena_chunks : kMaxChunks),
                 nch = (S + W - 1) / W;
    if (ib && rb && idev && rdev && im.arena_zc && (streams_once(*c->enc, S) || uint64_t(n) * S <= kZcSmallBytes)) {
        rc = rsg_encode(c, idev, int64_t(n * ip), int64_t(ip), rdev, int64_t(n * rp), int64_t(rp), 1, int64_t(S),
                        im.stream);
        if (rc) return rc;
        HIP_TRY(hipEventRecord(im.ev[0], im.stream));
        HIP_TRY(hipEventSynchronize(im.ev[0]));
        return 0;
    }
    // registered caller symbols (sym_alloc): one gather kernel, the encode, one scatter kernel
    if (!ib && !rb && S % 16 == 0 && S >= kRegMinBytes) {
        if (im.reserve_ptrs(n)) return 1;
        uint64_t* hp = reinterpret_cast<uint64_t*>(im.h_ptrs);
        if (sym_devptrs(inf->symbols, k, S, hp) && sym_devptrs(rep->symbols, r, S, hp + k)) {
            size_t ip2 = 0, rp2 = 0;
            if (im.arena_zc && streams_once(*c->enc, S) && strided_run(hp, k, S, &ip2) && strided_run(hp + k, r, S, &rp2)) {
                // the symbols sit at one stride in the device's view (consecutive symbol_create calls usually
                // do): the encode kernel streams them across PCIe itself, as for arena stripes
                uint8_t* di = reinterpret_cast<uint8_t*>(uintptr_t(hp[0]));
                uint8_t* dr = reinterpret_cast<uint8_t*>(uintptr_t(hp[k]));
                if ((rc = rsg_encode(c, di, int64_t(k * ip2), int64_t(ip2), dr, int64_t(r * rp2), int64_t(rp2), 1,
                                     int64_t(S), im.stream)))
                    return rc;
                HIP_TRY(hipEventRecord(im.ev[0], im.stream));
                HIP_TRY(hipEventSynchronize(im.ev[0]));
                return 0;
            }
            if (im.reserve(n * P)) return 1;
            uint8_t* d = im.d_buf;
            const uint64_t* dp = reinterpret_cast<const uint64_t*>(im.d_ptrs);
            HIP_TRY(hipMemcpyAsync(im.d_ptrs, im.h_ptrs, n * 8, hipMemcpyHostToDevice, im.in_stream));
            // column chunks: the gather of chunk c + 1 (in_stream) reads across PCIe while chunk c is encoded
            // and its repair columns are written back (stream)
            const size_t Wr = chunk_width(S, im.reg_chunks), nr = (S + Wr - 1) / Wr;
            for (size_t ch = 0; ch < nr; ++ch) {
                const size_t off = ch * Wr, w = std::min(Wr, S - off);
                HIP_TRY(launch_gather_ptrs(d, int64_t(P), dp, nullptr, int64_t(k), int64_t(off), int64_t(w), im.in_stream));
                HIP_TRY(hipEventRecord(im.ev_in[ch], im.in_stream));
                HIP_TRY(hipStreamWaitEvent(im.stream, im.ev_in[ch], 0));
                if ((rc = rsg_encode(c, d + off, n * P, P, d + size_t(k) * P + off, n * P, P, 1, w, im.stream))) return rc;
                HIP_TRY(launch_scatter_ptrs(dp + k, d + size_t(k) * P, int64_t(P), nullptr, int64_t(r), int64_t(off),
                                            int64_t(w), im.stream));
            }
            HIP_TRY(hipEventRecord(im.ev[0], im.stream));
            HIP_TRY(hipEventSynchronize(im.ev[0]));
            return 0;
        }
    }
    if (im.reserve(n * P)) return 1;
    uint8_t *h = im.h_buf, *d = im.d_buf;
    // chunk c: gather k columns -> H2D (2D) -> encode -> D2H (2D); scatter of c - 1 overlaps it
    auto scatter = [&](size_t c) {
        if (rb) return;
        const size_t off = c * W, w = std::min(W, S - off);
        im.pool->run(r, [&](int p) { std::memcpy(rep->symbols[p]->data + off, h + (k + size_t(p)) * P + off, w); });
    };
    for (size_t ch = 0; ch < nch; ++ch) {
        const size_t off = ch * W, w = std::min(W, S - off);
        if (ib) {
            HIP_TRY(hipMemcpy2DAsync(d + off, P, ib + off, ip, w, k, hipMemcpyHostToDevice, im.in_stream));
            HIP_TRY(hipEventRecord(im.ev_in[ch], im.in_stream));
            HIP_TRY(hipStreamWaitEvent(im.stream, im.ev_in[ch], 0));
        } else {
            im.pool->run(k, [&](int i) { std::memcpy(h + size_t(i) * P + off, inf->symbols[i]->data + off, w); });
            HIP_TRY(hipMemcpy2DAsync(d + off, P, h + off, P, w, k, hipMemcpyHostToDevice, im.stream));
        }
        rc = rsg_encode(c, d + off, n * P, P, d + size_t(k) * P + off, n * P, P, 1, w, im.stream);
        if (rc) return rc;
        if (rb && rdev && im.arena_put)
            HIP_TRY(launch_put_rows(rdev + off, int64_t(rp), d + size_t(k) * P + off, int64_t(P), nullptr, int64_t(r),
                                    int64_t(ch + 1 == nch ? P - off : w), im.stream));
        else if (rb)
            HIP_TRY(hipMemcpy2DAsync(rb + off, rp, d + size_t(k) * P + off, P, w, r, hipMemcpyDeviceToHost, im.stream));
        else
            HIP_TRY(hipMemcpy2DAsync(h + size_t(k) * P + off, P, d + size_t(k) * P + off, P, w, r,
                                     hipMemcpyDeviceToHost, im.stream));
        HIP_TRY(hipEventRecord(im.ev[ch], im.stream));
        if (ch && !rb) {  // host scatter of chunk c - 1 overlaps chunk c
            HIP_TRY(hipEventSynchronize(im.ev[ch - 1]));
            scatter(ch - 1);
        }
    }
    HIP_TRY(hipEventSynchronize(im.ev[nch - 1]));
    scatter(nch - 1);
    return 0;
}

extern "C" int rs_restore_symbols(RS_t* rs, uint16_t k, uint16_t r, symbol_seq_t* rcv, const bool* is_erased,
                                  uint16_t t) {
    if (r < t) return RS_ERR_CANNOT_RESTORE;  // checked first, as reference reed_solomon.c:467-470
    if (!rs || !rs->impl || !rcv || !is_erased) return RS_ERR_INVALID;
    Impl& im = *static_cast<Impl*>(rs->impl);
    const size_t S = rcv->symbol_size, n = size_t(k) + r;
    if (rcv->length != n || (S & 1) || n > kN) return RS_ERR_INVALID;
    size_t cnt = 0;
    std::vector<int> keep, lost;  // surviving slots (gathered), erased information slots (scattered)
    for (size_t i = 0; i < n; ++i) {
        if (is_erased[i]) {
            ++cnt;
            if (i < k) lost.push_back(int(i));
        } else {
            keep.push_back(int(i));
        }
    }
    if (cnt != t) return RS_ERR_INVALID;
    if (lost.empty() || S == 0) return 0;
    std::lock_guard<std::mutex> lk(im.mu);
    HIP_TRY(hipSetDevice(im.device));
    rsg_codec* c = nullptr;
    int rc = im.codec(k, r, &c);
    if (rc) return rc;
    // A GF(256) plan that will be specialised at a later call runs the generic kernel until then, whose
    // few workgroups per column chunk leave the chip mostly idle (one C3 stripe: 16 per 16 KiB chunk, 87 us
    // a launch): one launch over the whole symbol then beats the copy / kernel pipeline over kMaxChunks
    // column chunks. Plans that are never specialised (GF(2^16) codes, jit = 0, a failed compile) keep
    // the chunked pipeline.
    DevPlan* dplan = nullptr;
    if ((rc = decode_plan(c, is_erased, t, &dplan, im.stream))) return rc;
    const bool pending = c->m <= 8 && c->jit != 0 && !dplan->xj && !dplan->jit && !dplan->xj_failed && !dplan->jit_failed;
    size_t sp = 0;
    uint8_t* sdev = nullptr;
    uint8_t* sb = const_cast<uint8_t*>(arena_run(rcv->symbols, n, S, &sp, &sdev));
    if (sb && sdev && im.arena_zc && (streams_once(*dplan, S) || uint64_t(n) * S <= kZcSmallBytes)) {  // in place, one launch
        rc = rsg_decode(c, sdev, n * sp, sp, 1, S, is_erased, t, im.stream);
        if (rc) return rc;
        HIP_TRY(hipEventRecord(im.ev[0], im.stream));
        HIP_TRY(hipEventSynchronize(im.ev[0]));
        return 0;
    }
    // registered caller symbols (sym_alloc): surviving rows gathered by one kernel, the decode, the restored
    // rows scattered by one kernel
    if (!sb && S % 16 == 0 && S >= kRegMinBytes) {
        if (im.reserve_ptrs(n)) return 1;
        uint64_t* hp = reinterpret_cast<uint64_t*>(im.h_ptrs);
        if (sym_devptrs(rcv->symbols, n, S, hp)) {
            size_t sp2 = 0;
            if (im.arena_zc && streams_once(*dplan, S) && strided_run(hp, n, S, &sp2)) {  // in place, one launch
                uint8_t* ds = reinterpret_cast<uint8_t*>(uintptr_t(hp[0]));
                if ((rc = rsg_decode(c, ds, n * sp2, sp2, 1, S, is_erased, t, im.stream))) return rc;
                HIP_TRY(hipEventRecord(im.ev[0], im.stream));
                HIP_TRY(hipEventSynchronize(im.ev[0]));
                return 0;
            }
            const size_t P = pad16(S);
            if (im.reserve(n * P)) return 1;
            int32_t* hk = reinterpret_cast<int32_t*>(im.h_ptrs + n * 8);
            int32_t* hl = hk + keep.size();
            std::memcpy(hk, keep.data(), keep.size() * 4);
            std::memcpy(hl, lost.data(), lost.size() * 4);
            uint8_t* d = im.d_buf;
            const uint64_t* dp = reinterpret_cast<const uint64_t*>(im.d_ptrs);
            const int32_t* dk = reinterpret_cast<const int32_t*>(im.d_ptrs + n * 8);
            HIP_TRY(hipMemcpyAsync(im.d_ptrs, im.h_ptrs, n * 8 + (keep.size() + lost.size()) * 4, hipMemcpyHostToDevice,
                                   im.in_stream));
            // column chunks as the encode's (a pattern still on its generic kernel decodes in one piece)
            const size_t Wr = pending ? S : chunk_width(S, im.reg_chunks), nr = (S + Wr - 1) / Wr;
            for (size_t ch = 0; ch < nr; ++ch) {
                const size_t off = ch * Wr, w = std::min(Wr, S - off);
                HIP_TRY(launch_gather_ptrs(d, int64_t(P), dp, dk, int64_t(keep.size()), int64_t(off), int64_t(w),
                                           im.in_stream));
                HIP_TRY(hipEventRecord(im.ev_in[ch], im.in_stream));
                HIP_TRY(hipStreamWaitEvent(im.stream, im.ev_in[ch], 0));
                if ((rc = rsg_decode(c, d + off, n * P, P, 1, w, is_erased, t, im.stream))) return rc;
                HIP_TRY(launch_scatter_ptrs(dp, d, int64_t(P), dk + keep.size(), int64_t(lost.size()), int64_t(off),
                                            int64_t(w), im.stream));
            }
            HIP_TRY(hipEventRecord(im.ev[0], im.stream));
            HIP_TRY(hipEventSynchronize(im.ev[0]));
            return 0;
        }
    }
    // a stripe in a page-locked arena (seq_create) is copied in place: all n rows in by one 2D DMA
    // (erased rows ride along unread), restored rows out by DMA of their span or, when scattered,
    // written across PCIe by k_put_rows straight into the arena
    const size_t P = pad16(S), W = pending ? S : chunk_width(S, sb ? im.arena_chunks : kMaxChunks),
                 nch = (S + W - 1) / W,
                 nl = lost.size();
    // erased slots are neither gathered nor read by the decoder. Only restored rows come back: the span
    // lost[0] .. lost.back() when it is (nearly) contiguous, else the rows packed on the device behind
    // the stripe (k_gather_rows) and copied as one block
    const size_t lo = size_t(lost.front()), rows = size_t(lost.back()) - lo + 1;
    const bool packed = rows > nl + nl / 4;
    const bool put = sb && packed && sdev;  // restored rows written in place by the device
    const bool host_scatter = !sb || (packed && !sdev);
    if (im.reserve((n + (packed ? nl : 0)) * P)) return 1;
    uint8_t *h = im.h_buf, *d = im.d_buf;
    if (packed) {
        if (nl > im.rows_cap) {
            if (im.h_rows) (void)hipHostFree(im.h_rows);
            if (im.d_rows) (void)hipFree(im.d_rows);
            im.h_rows = nullptr;
            im.d_rows = nullptr;
            im.rows_cap = 0;
            HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&im.h_rows), nl * 4, hipHostMallocDefault));
            HIP_TRY(hipMalloc(reinterpret_cast<void**>(&im.d_rows), nl * 4));
            im.rows_cap = nl;
        }
        std::memcpy(im.h_rows, lost.data(), nl * 4);  // the previous call has finished with it (synchronous)
        HIP_TRY(hipMemcpyAsync(im.d_rows, im.h_rows, nl * 4, hipMemcpyHostToDevice, im.stream));
    }
    uint8_t *hp = h + n * P, *dp = d + n * P;  // packed restored rows (row j = slot lost[j])
    auto scatter = [&](size_t ch) {
        if (!host_scatter) return;
        const size_t off = ch * W, w = std::min(W, S - off);
        im.pool->run(int(nl), [&](int j) {
            const size_t i = size_t(lost[size_t(j)]);
            std::memcpy(rcv->symbols[i]->data + off, (packed ? hp + size_t(j) * P : h + i * P) + off, w);
        });
    };
    for (size_t ch = 0; ch < nch; ++ch) {
        const size_t off = ch * W, w = std::min(W, S - off);
        if (sb) {
            HIP_TRY(hipMemcpy2DAsync(d + off, P, sb + off, sp, w, n, hipMemcpyHostToDevice, im.in_stream));
            HIP_TRY(hipEventRecord(im.ev_in[ch], im.in_stream));
            HIP_TRY(hipStreamWaitEvent(im.stream, im.ev_in[ch], 0));
        } else {
            im.pool->run(int(keep.size()), [&](int j) {
                const size_t i = size_t(keep[size_t(j)]);
                std::memcpy(h + i * P + off, rcv->symbols[i]->data + off, w);
            });
            HIP_TRY(hipMemcpy2DAsync(d + off, P, h + off, P, w, n, hipMemcpyHostToDevice, im.stream));
        }
        rc = rsg_decode(c, d + off, n * P, P, 1, w, is_erased, t, im.stream);
        if (rc) return rc;
        if (put) {
            // chunk widths are multiples of 2048 but the last; it runs to the padded row end, for which
            // the arena's pitch leaves room
            const size_t wp = ch + 1 == nch ? P - off : w;
            HIP_TRY(launch_put_rows(sdev + off, int64_t(sp), d + off, int64_t(P), im.d_rows, int64_t(nl), int64_t(wp),
                                    im.stream));
        } else if (sb && !packed) {
            HIP_TRY(hipMemcpy2DAsync(sb + lo * sp + off, sp, d + lo * P + off, P, w, rows, hipMemcpyDeviceToHost,
                                     im.stream));
        } else if (packed) {
            HIP_TRY(launch_gather_rows(dp + off, int64_t(P), d + off, int64_t(P), im.d_rows, int64_t(nl), int64_t(w),
                                       im.stream));
            HIP_TRY(hipMemcpy2DAsync(hp + off, P, dp + off, P, w, nl, hipMemcpyDeviceToHost, im.stream));
        } else {
            HIP_TRY(hipMemcpy2DAsync(h + lo * P + off, P, d + lo * P + off, P, w, rows, hipMemcpyDeviceToHost,
                                     im.stream));
        }
        HIP_TRY(hipEventRecord(im.ev[ch], im.stream));
        if (ch && host_scatter) {
            HIP_TRY(hipEventSynchronize(im.ev[ch - 1]));
            scatter(ch - 1);
        }
    }
    HIP_TRY(hipEventSynchronize(im.ev[nch - 1]));
    scatter(nch - 1);
    return 0;
}

// ============================================================================ memory/*.h
extern "C" symbol_t* symbol_create(size_t symbol_size) {
    symbol_t* s = static_cast<symbol_t*>(std::calloc(1, sizeof(symbol_t)));
    if (!s) return nullptr;
    s->data = sym_alloc(symbol_size);  // whole zeroed pages, registrable (>= kRegMinBytes), or:
    if (!s->data) s->data = static_cast<uint8_t*>(std::calloc(symbol_size ? symbol_size : 1, 1));
    if (!s->data) {
        std::free(s);
        return nullptr;
    }
    return s;
}

extern "C" void symbol_destroy(symbol_t* s) {
    if (!s) return;
    if (!arena_release(s->data) && !sym_release(s->data)) std::free(s->data);
    std::free(s);
}

extern "C" bool symbol_eq(const symbol_t* a, const symbol_t* b, size_t symbol_size) {
    if (!a || !b || !a->data || !b->data) return false;
    return std::memcmp(a->data, b->data, symbol_size) == 0;
}

extern "C" void symbol_printf(const symbol_t* s, size_t symbol_size) {
    if (!s || !s->data) {
        std::printf("NULL");
        return;
    }
    std::printf("[");
    for (size_t i = 0; i < symbol_size; ++i) std::printf(i + 1 < symbol_size ? "%u, " : "%u", s->data[i]);
    std::printf("]");
}

extern "C" symbol_seq_t* seq_create(size_t length, size_t symbol_size) {
    symbol_seq_t* q = static_cast<symbol_seq_t*>(std::calloc(1, sizeof(symbol_seq_t)));
    if (!q) return nullptr;
    q->length = length;
    q->symbol_size = symbol_size;
    q->symbols = static_cast<symbol_t**>(std::calloc(length ? length : 1, sizeof(symbol_t*)));
    if (!q->symbols) {
        std::free(q);
        return nullptr;
    }
    // one zeroed page-locked block (or a slab share for small sequences) at stride pad16(S), see arena_alloc
    const size_t P = pad16(symbol_size ? symbol_size : 1);
    if (uint8_t* blk = symbol_size ? arena_alloc(length, P) : nullptr) {
        bool ok = true;
        for (size_t i = 0; i < length && ok; ++i)
            ok = (q->symbols[i] = static_cast<symbol_t*>(std::calloc(1, sizeof(symbol_t)))) != nullptr;
        if (!ok) {
            for (size_t i = 0; i < length; ++i) std::free(q->symbols[i]);
            for (size_t i = 0; i < length; ++i) arena_release(blk);  // drops the block with its last count
            std::free(q->symbols);
            std::free(q);
            return nullptr;
        }
        for (size_t i = 0; i < length; ++i) q->symbols[i]->data = blk + i * P;
        return q;
    }
    for (size_t i = 0; i < length; ++i) {
        if (!(q->symbols[i] = symbol_create(symbol_size))) {
            for (size_t j = 0; j < i; ++j) symbol_destroy(q->symbols[j]);
            std::free(q->symbols);
            std::free(q);
            return nullptr;
        }
    }
    return q;
}

extern "C" void seq_destroy(symbol_seq_t* q) {
    if (!q) return;
    for (size_t i = 0; i < q->length; ++i) symbol_destroy(q->symbols[i]);
    std::free(q->symbols);
    std::free(q);
}

extern "C" bool seq_eq(const symbol_seq_t* a, const symbol_seq_t* b) {
    if (!a || !b || !a->symbols || !b->symbols) return false;
    if (a->length != b->length || a->symbol_size != b->symbol_size) return false;
    for (size_t i = 0; i < a->length; ++i)
        if (!symbol_eq(a->symbols[i], b->symbols[i], a->symbol_size)) return false;
    return true;
}

extern "C" void seq_printf(const symbol_seq_t* q) {
    if (!q || !q->symbols) {
        std::printf("NULL");
        return;
    }
    if (!q->length) {
        std::printf("[]");
        return;
    }
    std::printf("[");
    for (size_t i = 0; i < q->length; ++i) {
        symbol_printf(q->symbols[i], q->symbol_size);
        if (i + 1 < q->length) std::printf(", ");
    }
    std::printf("]");
}

// ============================================================================ rs/gf65536.h, rs/cyclotomic_coset.h
// normal bases of GF(2), GF(4), GF(16), GF(256), GF(2^16): facts restated from reference gf65536.c:21-57
static const uint16_t kNormalBases[GF_NORMAL_BASES_ELEMENTS] = {
    1,                                                           // GF(2)
    44234, 44235,                                                // GF(4)
    10800, 47860, 34555, 5694,                                   // GF(16)
    16402, 53598, 44348, 63986, 22060, 64366, 6088, 32521,       // GF(256)
    2048, 2880, 7129, 30616, 2643, 6897, 29685, 7378, 30100, 2743, 20193, 36223, 24055, 41458, 41014, 61451};

static int m_index(uint8_t m) { return m == 1 ? 0 : m == 2 ? 1 : m == 4 ? 3 : m == 8 ? 7 : 15; }

// normal_repr[li][d]: bits of alpha^d in the normal basis of GF(2^m), m = 1 << li (0 when alpha^d is
// not in GF(2^m)), as reference gf65536.c:90-108 tabulates them
static const std::vector<uint16_t>* normal_repr_tables() {
    static std::once_flag once;
    static std::vector<uint16_t> tab[CC_COSET_SIZES_CNT];
    std::call_once(once, [] {
        const Field& F = field();
        for (int li = 0; li < CC_COSET_SIZES_CNT; ++li) {
            const uint8_t mm = uint8_t(1u << li);
            tab[li].assign(kN, 0);
            for (uint32_t bits = 1; bits < (1u << mm); ++bits) {
                uint16_t e = 0;
                for (int j = 0; j < mm; ++j)
                    if (bits & (1u << j)) e ^= kNormalBases[m_index(mm) + j];
                tab[li][F.log[e]] = uint16_t(bits);
            }
        }
    });
    return tab;
}

static uint16_t normal_basis_element(int m, int i) { return kNormalBases[m_index(uint8_t(m)) + i]; }

extern "C" GF_t* gf_create(void) {
    GF_t* gf = static_cast<GF_t*>(std::calloc(1, sizeof(GF_t)));
    if (!gf) return nullptr;
    const Field& F = field();
    for (uint32_t i = 0; i < (kN << 1) - 1; ++i) gf->pow_table[i] = F.exp[i];
    std::memcpy(gf->log_table, F.log, sizeof(gf->log_table));
    std::memcpy(gf->normal_bases, kNormalBases, sizeof(kNormalBases));
    const std::vector<uint16_t>* tab = normal_repr_tables();
    for (int li = 0; li < CC_COSET_SIZES_CNT; ++li) {
        uint16_t* dst = gf->_normal_repr_by_subfield_memory + size_t(li) * N;
        std::memcpy(dst, tab[li].data(), size_t(N) * sizeof(uint16_t));
        gf->normal_repr_by_subfield[1u << li] = dst;  // other entries stay NULL, as the reference's
    }
    return gf;
}

extern "C" void gf_destroy(GF_t* gf) { std::free(gf); }

extern "C" element_t gf_get_normal_basis_element(GF_t* gf, uint8_t m, uint8_t i) {
    return gf ? gf->normal_bases[m_index(m) + i] : kNormalBases[m_index(m) + i];
}

extern "C" uint16_t gf_get_normal_repr(GF_t* gf, uint8_t m, uint16_t d) {
    if (gf && m <= CC_MAX_COSET_SIZE && gf->normal_repr_by_subfield[m]) return gf->normal_repr_by_subfield[m][d];
    const int li = m == 1 ? 0 : m == 2 ? 1 : m == 4 ? 2 : m == 8 ? 3 : 4;
    return normal_repr_tables()[li][d % kN];
}

extern "C" element_t gf_mul_ee(GF_t* gf, element_t a, element_t b) {
    (void)gf;
    return field().mul(a, b);
}

extern "C" element_t gf_div_ee(GF_t* gf, element_t a, element_t b) {
    (void)gf;
    return field().div(a, b);
}

extern "C" CC_t* cc_create(void) {
    CC_t* cc = static_cast<CC_t*>(std::malloc(sizeof(CC_t)));
    if (!cc) return nullptr;
    const Cosets& cs = cosets();
    uint16_t* w = cc->_leaders_memory;
    for (int i = 0; i < CC_COSET_SIZES_CNT; ++i) {
        cc->leaders[i] = w;
        for (uint16_t l : cs.leaders[i]) *w++ = l;
    }
    return cc;
}

extern "C" void cc_destroy(CC_t* cc) { std::free(cc); }

extern "C" uint8_t cc_get_coset_size(uint16_t leader) {
    uint8_t m = 1;
    while (leader != uint16_t((uint32_t(leader) << m) % kN)) m <<= 1;
    return m;
}

extern "C" void cc_estimate_cosets_cnt(uint16_t k, uint16_t r, uint16_t* inf_max_cnt, uint16_t* rep_max_cnt) {
    if (inf_max_cnt) *inf_max_cnt = coset_upper_bound(k);
    if (rep_max_cnt) *rep_max_cnt = coset_upper_bound(r);
}

extern "C" void cc_select_cosets(CC_t* cc, uint16_t k, uint16_t r, coset_t* inf_cosets, uint16_t inf_max_cnt,
                                 uint16_t* inf_cosets_cnt, coset_t* rep_cosets, uint16_t rep_max_cnt,
                                 uint16_t* rep_cosets_cnt) {
    (void)cc;
    std::vector<CosetRef> inf, rep;
    select_cosets(k, r, inf, rep);
    // the caller's capacities bound the output exactly like the reference loop guards
    const size_t ni = std::min<size_t>(inf.size(), inf_max_cnt), nr = std::min<size_t>(rep.size(), rep_max_cnt);
    for (size_t i = 0; i < ni; ++i) inf_cosets[i] = coset_t{inf[i].leader, inf[i].size};
    for (size_t i = 0; i < nr; ++i) rep_cosets[i] = coset_t{rep[i].leader, rep[i].size};
    *inf_cosets_cnt = uint16_t(ni);
    *rep_cosets_cnt = uint16_t(nr);
}

extern "C" void cc_cosets_to_positions(const coset_t* cs, uint16_t cosets_cnt, uint16_t* positions,
                                       uint16_t positions_cnt) {
    uint16_t w = 0;
    for (uint16_t c = 0; c < cosets_cnt && w < positions_cnt; ++c) {
        uint16_t e = cs[c].leader;
        do {
            positions[w++] = e;
            e = NEXT_COSET_ELEMENT(e);
        } while (e != cs[c].leader && w < positions_cnt);
    }
}

// ============================================================================ context-free host ops
// gf_add / gf_mul / gf_madd and the fft_* transforms take host symbols and no codec. They run on the
// GPU through a pool of engines: a call leases one (a mutex only around the pool's free list, so
// concurrent callers run side by side), and each engine has its own non-blocking stream, page-locked
// mapped staging that only grows (with its device-visible address) and an m = 16 codec shell whose
// matrix kernels, options and split-K scratch the transforms use. An engine serves the device that was
// current when it was created; leases prefer an engine of the caller's current device.
namespace {

struct HostOps {
    int device = -1;
    hipStream_t stream = nullptr;
    uint8_t* h = nullptr;   // page-locked, mapped
    uint8_t* hd = nullptr;  // its device-visible address (zero-copy kernels)
    uint8_t* d = nullptr;   // device staging (transforms)
    size_t cap = 0, dcap = 0;
    std::unique_ptr<rsg_codec> codec;
    int init(int dev) {
        if (device >= 0) return 0;
        HIP_TRY(hipSetDevice(dev));
        HIP_TRY(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        auto c = std::make_unique<rsg_codec>();
        c->device = dev;
        c->m = 16;
        if (int rc = device_tables(dev, &c->d_ltab)) return rc;
        codec = std::move(c);
        device = dev;
        return 0;
    }
    int reserve_host(size_t bytes) {  // mapped staging
        if (bytes <= cap) return 0;
        if (h) (void)hipHostFree(h);
        h = hd = nullptr;
        cap = 0;
        HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&h), bytes, hipHostMallocMapped | hipHostMallocPortable));
        void* dv = nullptr;
        HIP_TRY(hipHostGetDevicePointer(&dv, h, 0));
        hd = static_cast<uint8_t*>(dv);
        cap = bytes;
        return 0;
    }
    int reserve_dev(size_t bytes) {
        if (bytes <= dcap) return 0;
        if (d) (void)hipFree(d);
        d = nullptr;
        dcap = 0;
        HIP_TRY(hipMalloc(reinterpret_cast<void**>(&d), bytes));
        dcap = bytes;
        return 0;
    }
};

struct HostOpsPool {
    std::mutex mu;
    std::map<int, std::vector<HostOps*>> idle;  // per device; engines are never destroyed (they outlive
                                                // the HIP runtime's teardown at exit)
};
HostOpsPool& hostops_pool() {
    static HostOpsPool* p = new HostOpsPool();
    return *p;
}

// an engine for the duration of one call
struct EngineLease {
    HostOps* e = nullptr;
    int rc = 0;
    EngineLease() {
        int ndev = 0, dev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0 || hipGetDevice(&dev) != hipSuccess) {
            (void)hipGetLastError();
            std::fprintf(stderr, "librs_amd: no usable HIP device for the symbol operations (no CPU fallback)\n");
            rc = RS_ERR_DEVICE;
            return;
        }
        HostOpsPool& P = hostops_pool();
        {
            std::lock_guard<std::mutex> lk(P.mu);
            auto& v = P.idle[dev];
            if (!v.empty()) {
                e = v.back();
                v.pop_back();
            }
        }
        if (!e) e = new HostOps();
        rc = e->init(dev);
        if (!rc && hipSetDevice(e->device) != hipSuccess) rc = RS_ERR_DEVICE;
    }
    ~EngineLease() {
        if (!e) return;
        if (e->device < 0) {  // never initialised: nothing to keep
            delete e;
            return;
        }
        HostOpsPool& P = hostops_pool();
        std::lock_guard<std::mutex> lk(P.mu);
        P.idle[e->device].push_back(e);
    }
};

constexpr size_t kSymbolOpDmaBytes = size_t(256) << 10;

// a ^= b (op 0), a = coef * a (1), a ^= coef * b (2) over symbol_size / 2 words, on the GPU: the operands
// are copied into the engine's mapped staging and one kernel reads and writes them there across PCIe
// (zero-copy: no DMA round trips); its completion is the call's only wait
int symbol_op(int op, void* a, element_t coef, const void* b, size_t symbol_size) {
    const size_t nw = symbol_size / 2, bytes = nw * 2, P = pad16(bytes);
    if (!nw) return 0;
    EngineLease L;
    if (L.rc) return L.rc;
    HostOps& o = *L.e;
    if (int rc = o.reserve_host(2 * P)) return rc;
    const uint16_t *logt = nullptr, *expt = nullptr;
    const uint8_t* g8 = nullptr;
    if (int rc = plan_tables(o.device, &logt, &g8, &expt)) return rc;
    std::memcpy(o.h, a, bytes);
    if (P > bytes) std::memset(o.h + bytes, 0, P - bytes);
    if (op != 1) {
        std::memcpy(o.h + P, b, bytes);
        if (P > bytes) std::memset(o.h + P + bytes, 0, P - bytes);
    }
    const uint32_t lc = op == 0 ? 0u : field().log[coef];
    // large operands: DMA in and out (the copy engines beat the kernel's own PCIe reads there: 1 MiB
    // gf_madd 172 us with DMA vs 199 us zero-copy, profiles/r3_hostops.jsonl)
    const bool dma = P >= kSymbolOpDmaBytes;
    uint8_t* dv = o.hd;
    if (dma) {
        if (int rc = o.reserve_dev(2 * P)) return rc;
        dv = o.d;
        HIP_TRY(hipMemcpyAsync(o.d, o.h, op != 1 ? 2 * P : P, hipMemcpyHostToDevice, o.stream));
    }
    HIP_TRY(launch_symbol_op(reinterpret_cast<uint16_t*>(dv), reinterpret_cast<const uint16_t*>(dv + P), op, lc,
                             int64_t(P / 2), logt, expt, o.stream));
    if (dma) HIP_TRY(hipMemcpyAsync(o.h, o.d, bytes, hipMemcpyDeviceToHost, o.stream));
    HIP_TRY(hipStreamSynchronize(o.stream));
    std::memcpy(a, o.h, bytes);
    return 0;
}

[[noreturn]] void symbol_op_failed(const char* what, int rc) {
    // void entry points cannot report an error; a wrong symbol must never be returned silently
    std::fprintf(stderr, "librs_amd: %s failed (code %d); aborting\n", what, rc);
    std::abort();
}

// res[j] = sum_i M[j][i] f[i] for the transforms: f and res gathered / scattered through pinned
// staging, the matrix applied by the engine's GF(2^16) kernels (host-built plan). Odd symbol sizes
// follow the reference under NDEBUG: words cover symbol_size / 2, the outputs' last byte is zero
// (fft.c memsets every output before accumulating into it).
int transform_apply(std::vector<uint16_t> M, const symbol_seq_t* f, symbol_seq_t* res) {
    if (!f || !res || f->symbol_size != res->symbol_size) return RS_ERR_INVALID;
    const size_t S = f->symbol_size, Se = S & ~size_t(1), K = f->length, R = res->length;
    if (R == 0) return 0;
    if (K == 0 || Se == 0) {
        for (size_t j = 0; j < R; ++j) std::memset(res->symbols[j]->data, 0, S);
        return 0;
    }
    if (K > kN || R > kN) return RS_ERR_INVALID;
    EngineLease L;
    if (L.rc) return L.rc;
    HostOps& o = *L.e;
    const size_t P = pad16(Se);
    if (int rc = o.reserve_host((K + R) * P)) return rc;
    if (int rc = o.reserve_dev((K + R) * P)) return rc;
    for (size_t i = 0; i < K; ++i) std::memcpy(o.h + i * P, f->symbols[i]->data, Se);
    HIP_TRY(hipMemcpyAsync(o.d, o.h, K * P, hipMemcpyHostToDevice, o.stream));
    std::vector<int32_t> in(K), out(R);
    for (size_t i = 0; i < K; ++i) in[i] = int32_t(i);
    for (size_t j = 0; j < R; ++j) out[j] = int32_t(j);
    std::unique_ptr<DevPlan> plan;
    if (int rc = build_plan(o.device, 16, std::move(M), int(K), int(R), std::move(in), std::move(out), plan, o.stream))
        return rc;
    uint8_t* dres = o.d + K * P;
    if (int rc = run_plan(o.codec.get(), *plan, o.d, 0, int64_t(P), dres, 0, int64_t(P), 1, Se, o.stream)) return rc;
    HIP_TRY(hipMemcpyAsync(o.h + K * P, dres, R * P, hipMemcpyDeviceToHost, o.stream));
    HIP_TRY(hipStreamSynchronize(o.stream));  // also: the plan's last launch is done before it is freed
    for (size_t j = 0; j < R; ++j) {
        std::memcpy(res->symbols[j]->data, o.h + (K + j) * P, Se);
        if (S != Se) res->symbols[j]->data[Se] = 0;
    }
    return 0;
}

// alpha^e for the reference's int products (a * b) % N, computed exactly (parity where they do not
// overflow an int)
inline element_t pow_mod(uint64_t a, uint64_t b) { return field().exp[(a * b) % kN]; }

}  // namespace

extern "C" void gf_add(void* a, const void* b, size_t symbol_size) {
    if (int rc = symbol_op(0, a, 0, b, symbol_size)) symbol_op_failed("gf_add", rc);
}

extern "C" void gf_mul(GF_t* gf, void* a, element_t coef, size_t symbol_size) {
    (void)gf;
    if (coef == 0) {  // reference gf65536.c:175-181
        std::memset(a, 0, symbol_size);
        return;
    }
    if (coef == 1) return;
    if (int rc = symbol_op(1, a, coef, nullptr, symbol_size)) symbol_op_failed("gf_mul", rc);
}

extern "C" void gf_madd(GF_t* gf, void* a, element_t coef, const void* b, size_t symbol_size) {
    (void)gf;
    if (coef == 0) return;  // reference gf65536.c:199-205
    if (int rc = symbol_op(coef == 1 ? 0 : 2, a, coef, b, symbol_size)) symbol_op_failed("gf_madd", rc);
}

// DFT matrix of fft_transform / fft_transform_cycl: M[j][i] = alpha^(positions[i] * j)
static std::vector<uint16_t> dft_matrix(const symbol_seq_t* f, const uint16_t* positions, const symbol_seq_t* res) {
    const size_t K = f->length, R = res->length;
    std::vector<uint16_t> M(R * K);
    for (size_t j = 0; j < R; ++j)
        for (size_t i = 0; i < K; ++i) M[j * K + i] = pow_mod(positions[i], j);
    return M;
}

extern "C" void fft_transform(GF_t* gf, const symbol_seq_t* f, const uint16_t* positions, symbol_seq_t* res) {
    (void)gf;
    if (!f || !res || (!positions && f->length)) symbol_op_failed("fft_transform (bad arguments)", RS_ERR_INVALID);
    if (int rc = transform_apply(dft_matrix(f, positions, res), f, res)) symbol_op_failed("fft_transform", rc);
}

extern "C" int fft_transform_cycl(GF_t* gf, const symbol_seq_t* f, const uint16_t* positions, symbol_seq_t* res) {
    (void)gf;
    if (!f || !res || (!positions && f->length)) return RS_ERR_INVALID;
    return transform_apply(dft_matrix(f, positions, res), f, res);
}

extern "C" void fft_partial_transform(GF_t* gf, const symbol_seq_t* f, const uint16_t* components,
                                      symbol_seq_t* res) {
    (void)gf;
    if (!f || !res || (!components && res->length))
        symbol_op_failed("fft_partial_transform (bad arguments)", RS_ERR_INVALID);
    const size_t K = f->length, R = res->length;
    std::vector<uint16_t> M(R * K);
    for (size_t r = 0; r < R; ++r) {
        const uint64_t j = (kN - components[r]) % kN;  // reference fft.c:115
        for (size_t i = 0; i < K; ++i) M[r * K + i] = pow_mod(i, j);
    }
    if (int rc = transform_apply(std::move(M), f, res)) symbol_op_failed("fft_partial_transform", rc);
}

extern "C" int fft_partial_transform_cycl(GF_t* gf, const symbol_seq_t* f, const coset_t* cosets, uint16_t cosets_cnt,
                                          symbol_seq_t* res) {
    if (!f || !res || (!cosets && cosets_cnt)) return RS_ERR_INVALID;
    const size_t K = f->length, R = res->length;
    size_t total = 0;
    for (uint16_t c = 0; c < cosets_cnt; ++c) {
        const uint8_t m = cosets[c].size;
        if (m != 1 && m != 2 && m != 4 && m != 8 && m != 16) return RS_ERR_INVALID;
        total += m;
    }
    if (total != R) return RS_ERR_INVALID;  // the reference asserts idx == res->length (fft.c:172)
    // the reference's evaluation entry by entry (fft.c:142-169): res[idx] of coset (L, m), element j,
    // = sum_i f[i] * sum_t bit_t(repr_m((s * i) % N)) * nb^(m)_((j + t) % m), s = N - L
    std::vector<uint16_t> M(R * K);
    size_t idx = 0;
    for (uint16_t c = 0; c < cosets_cnt; ++c) {
        const uint8_t m = cosets[c].size;
        const uint16_t s = uint16_t(N - cosets[c].leader);
        for (uint8_t j = 0; j < m; ++j, ++idx)
            for (size_t i = 0; i < K; ++i) {
                const uint16_t repr = gf_get_normal_repr(gf, m, uint16_t((uint64_t(s) * i) % kN));
                uint16_t v = 0;
                for (uint8_t t = 0; t < m; ++t)
                    if (repr & (1u << t)) v ^= kNormalBases[m_index(m) + (j + t) % m];
                M[idx * K + i] = v;
            }
    }
    return transform_apply(std::move(M), f, res);
}

// Host-only view of the GF(2^16) syndrome route of the encode (is_erased == NULL) or decode matrix: the
// k_cs16 plan (groups, records, finish lists) and the second-stage matrix M2 [R][D]. info = {D, ngroups,
// ntiles, fin_stride, R}; array arguments may be NULL (query the sizes first). No GPU is used.
extern "C" int rsg_symbol_registered(const void* data) {
    SymRegistry& R = symreg();
    std::lock_guard<std::mutex> lk(R.mu);
    auto it = R.m.find(uintptr_t(data));
    return it == R.m.end() ? -1 : (it->second.dev ? 1 : 0);
}

extern "C" int rsg_bs16_dump(uint16_t k, uint16_t r, const bool* is_erased, uint16_t t, int32_t* info, uint8_t* rec,
                             int32_t* fin, int32_t* fin_off) {
    if (uint32_t(k) + r > kN || (is_erased && t > r)) return RS_ERR_INVALID;
    const std::vector<uint16_t> pos = code_positions(k, r);
    std::vector<uint16_t> targets, sources;
    std::vector<int> emit;
    std::vector<int32_t> in, outs;
    codec_lists(pos, k, r, is_erased, targets, emit, sources, in, outs);
    const int D = int(targets.size());
    const std::vector<uint16_t> M2 = syndrome_solve_matrix(targets, emit);
    const int d = is_erased ? orbit_step(targets) : 1;
    CsHost h;
    const bool ok = d < 16 && bs16_host(M2, D, targets, emit, outs, h, d);
    if (info) {
        info[0] = ok ? 1 : 0;
        info[1] = D;
        info[2] = ok ? h.ngroups : 0;
        info[3] = ok ? h.ntiles : 0;
        info[4] = ok ? h.fin_stride : 0;
        info[5] = d;
    }
    if (ok && rec) std::memcpy(rec, h.rec.data(), h.rec.size());
    if (ok && fin) std::memcpy(fin, h.fin.data(), h.fin.size() * 4);
    if (ok && fin_off) std::memcpy(fin_off, h.fin_off.data(), h.fin_off.size() * 4);
    return 0;
}

// k_cs16t's side of the same plan: info = {cw, ntiles_t, fin_stride_t, block count}; records [ntiles_t]
// [ngroups + 2][4 cw] block offsets, finish lists [ntiles_t][fin_stride_t] / [ntiles_t][cw + 1], and the
// block table kCs16tOff ([(4c + n) * 16 + v]). Host only.
extern "C" int rsg_route_dump_t(uint16_t k, uint16_t r, const bool* is_erased, uint16_t t, int32_t* info, uint32_t* rec,
                                int32_t* fin, int32_t* fin_off, uint32_t* blocks) {
    if (uint32_t(k) + r > kN || (is_erased && t > r)) return RS_ERR_INVALID;
    const std::vector<uint16_t> pos = code_positions(k, r);
    std::vector<uint16_t> targets, sources;
    std::vector<int> emit;
    std::vector<int32_t> in, outs;
    codec_lists(pos, k, r, is_erased, targets, emit, sources, in, outs);
    const CsHost h = cs16_host(pos, in, int(targets.size()));
    constexpr int NBLK = int(sizeof(kCs16tOff) / sizeof(kCs16tOff[0]));
    if (info) {
        info[0] = kCs16tCw;
        info[1] = h.ntiles_t;
        info[2] = h.fin_stride_t;
        info[3] = NBLK;
    }
    if (rec) std::memcpy(rec, h.rec_t.data(), h.rec_t.size() * 4);
    if (fin) std::memcpy(fin, h.fin_t.data(), h.fin_t.size() * 4);
    if (fin_off) std::memcpy(fin_off, h.fin_off_t.data(), h.fin_off_t.size() * 4);
    if (blocks) std::memcpy(blocks, kCs16tOff, sizeof(kCs16tOff));
    return 0;
}

extern "C" int rsg_route_dump(uint16_t k, uint16_t r, const bool* is_erased, uint16_t t, int32_t* info, int32_t* groups,
                              uint8_t* rec, int32_t* fin, int32_t* fin_off, uint16_t* m2) {
    if (uint32_t(k) + r > kN || (is_erased && t > r)) return RS_ERR_INVALID;
    const std::vector<uint16_t> pos = code_positions(k, r);
    std::vector<uint16_t> targets, sources;
    std::vector<int> emit;
    std::vector<int32_t> in, outs;
    codec_lists(pos, k, r, is_erased, targets, emit, sources, in, outs);
    const CsHost h = cs16_host(pos, in, int(targets.size()));
    if (info) {
        info[0] = h.D;
        info[1] = h.ngroups;
        info[2] = h.ntiles;
        info[3] = h.fin_stride;
        info[4] = int32_t(outs.size());
    }
    if (groups) std::memcpy(groups, h.groups.data(), size_t(h.ngroups) * 16 * 4);  // even count, without the tail
    if (rec) std::memcpy(rec, h.rec.data(), h.rec.size());
    if (fin) std::memcpy(fin, h.fin.data(), h.fin.size() * 4);
    if (fin_off) std::memcpy(fin_off, h.fin_off.data(), h.fin_off.size() * 4);
    if (m2) {
        const std::vector<uint16_t> M = syndrome_solve_matrix(targets, emit);
        std::memcpy(m2, M.data(), M.size() * 2);
    }
    return 0;
}
