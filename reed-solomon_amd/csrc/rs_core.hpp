// rs_core.hpp -- internal declarations shared by the translation units of librs_amd.so (not installed):
// device plans (rs_plan.cpp), the codec object and its launch dispatcher (rs_api.cpp), the GF(2^16)
// syndrome route (rs_route16.cpp), per-stripe batches (rs_batch.cpp), host memory of the reference API
// (rs_hostmem.cpp), the per-call reference codec API (rs_dropin.cpp) and the secondary surface
// (rs_refops.cpp). Only the C ABI of include/ is the library's interface.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <initializer_list>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "gen/asm_counts.h"
#include "gen/cs16t_off.h"
#include "gf16.hpp"
#include "rs_jit.hpp"
#include "rs_kernels.hpp"
#include "rs_pool.hpp"
#include "rs_xj.hpp"

extern "C" {
#include <memory/seq.h>
#include <rs/cyclotomic_coset.h>
#include <rs/fft.h>
#include <rs/gf65536.h>
#include <rs/reed_solomon.h>
#include <rs_amd/rsg.h>
}

namespace rsamd {

// Every public entry that selects the codec's device (hipSetDevice) holds one of these: the calling thread's
// current HIP device is the same after the call as before it, as with the reference's CPU library, so a
// caller that drives several GPUs (or torch code relying on its current device) is not moved to the codec's.
struct CallerDevice {
    int prev = -1;
    CallerDevice() {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    }
    ~CallerDevice() {
        int now = -1;
        if (prev >= 0 && hipGetDevice(&now) == hipSuccess && now != prev) (void)hipSetDevice(prev);
    }
    CallerDevice(const CallerDevice&) = delete;
    CallerDevice& operator=(const CallerDevice&) = delete;
};

inline int hip_fail(hipError_t e, const char* what) {
    std::fprintf(stderr, "librs_amd: %s failed: %s\n", what, hipGetErrorString(e));
    return RS_ERR_DEVICE;
}

#define HIP_TRY(expr)                                      \
    do {                                                   \
        hipError_t _e = (expr);                            \
        if (_e != hipSuccess) return rsamd::hip_fail(_e, #expr); \
    } while (0)

inline size_t pad16(size_t s) { return (s + 15) & ~size_t(15); }

// the first n elements (all by default) of a host vector into a caller's array; nothing for none (an
// empty vector's data() may be null, which memcpy must not be given)
template <class T>
inline void copy_out(void* dst, const std::vector<T>& v, size_t n = SIZE_MAX) {
    n = std::min(n, v.size());
    if (dst && n) std::memcpy(dst, v.data(), n * sizeof(T));
}

// ------------------------------------------------------------------ rs_plan.cpp
int device_tables(int device, const uint32_t** out);
// log / exp / gamma-byte tables of the device plan builders
int plan_tables(int device, const uint16_t** logt, const uint8_t** g8, const uint16_t** expt = nullptr);
// device scratch that only grows (freed with its owner)
int grow(void** p, size_t& cap, size_t bytes);
int pool_dev_acquire(size_t bytes, int device, void** out, size_t* cap);
void pool_dev_release(void* p, size_t cap, int device, hipEvent_t guard);  // takes ownership of guard
int pool_host_acquire(size_t bytes, void** out, size_t* cap);
void pool_host_release(void* p, size_t cap);  // the copies reading p have completed

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
    bool slots_checked = false;      // check mode: slot lists bounds-checked on the host
    // slots of the layouts the lists index: 0 = the codec's k + r (every codec plan); the context-free
    // transforms (rs_refops.cpp) index their own staging rows
    int32_t slot_bound = 0;
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
    ~DevPlan();
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

int upload(void** dst, const void* src, size_t bytes);  // synchronous hipMalloc + copy
int build_plan(int device, int m, std::vector<uint16_t> M, int K, int R, std::vector<int32_t> in_slots,
               std::vector<int32_t> out_slots, std::unique_ptr<DevPlan>& out, hipStream_t st);
int build_plan_m16_device(int device, const std::vector<uint16_t>& targets, const std::vector<int>& emit,
                          const std::vector<uint16_t>& sources, std::vector<int32_t> in_slots,
                          std::vector<int32_t> out_slots, std::unique_ptr<DevPlan>& out, hipStream_t st);
// Target / source position lists of the encode (erased == NULL) or decode matrix, and their slots.
void codec_lists(const std::vector<uint16_t>& pos, uint16_t k, uint16_t r, const bool* erased,
                 std::vector<uint16_t>& targets, std::vector<int>& emit, std::vector<uint16_t>& sources,
                 std::vector<int32_t>& in_slots, std::vector<int32_t>& out_slots);
int codec_matrix(const std::vector<uint16_t>& pos, uint16_t k, uint16_t r, const bool* erased,
                 std::vector<uint16_t>& M, std::vector<int32_t>& in_slots, std::vector<int32_t>& out_slots);

// ------------------------------------------------------------------ rs_refops.cpp (GF tables)
const std::vector<uint16_t>* normal_repr_tables();  // [li][d]: alpha^d in the normal basis of GF(2^(1 << li))
uint16_t normal_basis_element(int m, int i);          // i-th element of the normal basis of GF(2^m)

}  // namespace rsamd

// ------------------------------------------------------------------ the codec (rs_api.cpp)
struct rsg_codec {
    int device = 0;
    uint16_t k = 0, r = 0;
    int m = 16;
    std::vector<uint16_t> positions;
    const uint32_t* d_ltab = nullptr;
    std::unique_ptr<rsamd::DevPlan> enc;
    std::map<std::vector<uint8_t>, std::unique_ptr<rsamd::DevPlan>> dec;
    std::vector<std::vector<uint8_t>> dec_lru;
    // generic GF(256) kernel: 20 = V = 1 with one nibble table per input (k_apply_m8_v1<2>; 10 % under 18 at
    // K = 128, profiles/r4/v1h_ab.log), 18 = the two-table V = 1 step
    int m8_mode = 20;
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
    // route with a device-built plan per stripe, 2 = its re-encode variant (encode route + t_info x t_info
    // Cauchy solves), 3 = the re-encode variant when the batch's largest pattern needs >= 13/16 r syndromes,
    // else the syndrome route (default), 0 = a plan per distinct pattern
    int m16_ps = 3;
    std::map<int, std::unique_ptr<rsamd::DevPlan>> ps_syn;  // k_cs16 plans over all k + r slots, keyed by D
    std::vector<int> ps_syn_lru;
    void *d_ps_rec = nullptr, *d_ps_small = nullptr;  // per-stripe records / lists of decode_batch_m16_ps
    int32_t* d_ps_in = nullptr;                       // its shared input list 0 .. r + 15
    hipStream_t ps_side = nullptr;                    // plan kernels of the next chunk run here
    hipStream_t ps_synst = nullptr;                   // option m16_ps_overlap: the syndrome passes run here
    hipEvent_t ps_ev_entry = nullptr, ps_ev_zero[2] = {nullptr, nullptr}, ps_ev_plan[2] = {nullptr, nullptr},
               ps_ev_used[2] = {nullptr, nullptr}, ps_ev_syn[2] = {nullptr, nullptr};
    int ps_overlap = 1;  // 1: chunk i + 1's syndrome pass beside chunk i's solve (two syndrome buffers)
    // option m16_cs_overlap: the same for the one-pattern syndrome route (run_cs); off by default: C5 in four
    // overlapped chunks measured 77.5-78.3 GB/s against 80.6-80.7 serial (profiles/r3/r3_cs_overlap_ab.log)
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
    // device-plan decodes of m <= 8 codes: 2 = re-encode route (fixed r x (k + r) matrix [G | I] on the
    // XOR kernel, then a per-stripe t_info x t_info solve; default), 1 = syndrome route (H, then a t_info x t
    // solve), 0 = per-stripe survivor matrices (k_plan_m8)
    int syn_route = 2;
    // option m8_syn_overlap: that route's plans and fixed pass of chunk i + 1 on the codec's syndrome stream
    // beside chunk i's solve (two buffer sets); 0 = one stream (default: two VALU-bound kernels side by side
    // ran no faster than in sequence, profiles/r4/ps8_route2.md)
    int m8_syn_overlap = 0;
    // option m8_ps_kernel: the per-stripe GF(256) solve's kernel: 0 k_apply_m8_v1 (LDS input ring), 1
    // k_apply_m8_ps_w (each wave loads its own inputs; no barriers), 2 k_apply_m8_ps_w2 (the same with
    // two dwords per lane), 3 k_apply_m8_v1<2> (the ring kernel with one nibble table per input), 9 / 10 / 11
    // k_apply_m8_pf<1 / 2 / 3> (no ring, every load issued a step or more ahead; packed records from the plan
    // kernels; two nibble tables / one table and two accumulator sets / one table with the multiples read from
    // LDS). Default 10 (the fastest); symbol sizes with a partial 1 KiB chunk and survivor
    // plans take 0.
    int m8_ps_kernel = 10;
    // option m8_syn_masked: 1 (default) the per-stripe fixed pass reads each stripe's erased slots as zero (masked
    // rs_xj) and the solve stores the erased symbols; 0 the plain pass over the slots as they are and a solve
    // that XORs its result into them (one old-value load per output)
    int m8_syn_masked = 1;
    // option m8_syn_coord (diagnostic build): 1 with the masked pass and solve 10, the fixed pass stores its
    // outputs in GF(256)^2 coordinates and the solve reads them as they are (k_apply_m8_pf<4>); 0 (default) the
    // solve converts. Measured 5-10 % slower: the tiny XOR-kernel workgroups each copy the tables and wait on
    // their reads
    int m8_syn_coord = 0;
    // option m8_syn_scratch_mib: fixed-pass output scratch of the GF(256) per-stripe route per chunk of stripes
    // (r x S bytes per stripe; the chunk count sets the launch count)
    int64_t syn_scratch_mib = 1024;
    // option m8_ps_cpb: 1 KiB column chunks per workgroup of the per-stripe ring kernels (table setup once per
    // block, the next chunk's ring prologue in flight during this chunk's output stage)
    int m8_ps_cpb = 1;
    // diagnostic builds: option m8_ps_ablate, timing ablations of the per-stripe solve (wrong results): 1 no
    // table copy, 2 no output conversion
    int m8_ps_ablate = 0;
    // diagnostic builds: option inject_fail_group, rsg_decode_batch's host-plan grouping path fails with
    // RS_ERR_DEVICE at that group (after the earlier groups' launches; tests of the failure fence)
    int64_t inject_fail_group = -1;
    std::unique_ptr<rsamd::DevPlan> syn;  // syndrome matrix S_j = sum_i X_i^j rcv_i, j < r
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
    std::unique_ptr<rsamd::DevPlan> bp16;
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
    // pinned staging of rsg_decode_batch's host lists (stage_lists, rs_batch.cpp), guarded by stage_ev
    uint8_t* h_stage = nullptr;
    size_t stage_cap = 0;
    hipEvent_t stage_ev = nullptr;
    bool stage_pending = false;
    // rsg_encode_host / rsg_decode_host: two streams, each with its own device batch buffer
    hipStream_t hs[2] = {nullptr, nullptr};
    uint8_t* hbuf[2] = {nullptr, nullptr};
    size_t hbuf_cap = 0;
    ~rsg_codec() {
        (void)hipSetDevice(device);
        if (stage_ev) (void)hipEventSynchronize(stage_ev), (void)hipEventDestroy(stage_ev);
        if (h_stage) (void)hipHostFree(h_stage);
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
                        d_ps_small, static_cast<void*>(d_ps_in), static_cast<void*>(d_slot_err), d_mbits, d_zero})
            if (p) (void)hipFree(p);
    }
    std::string last_kernel = "none";
    int32_t* d_slot_err = nullptr;  // checked launches of diagnostic builds: [4] slot-violation record
    // GF(256) per-stripe route: the selected stripes' patterns as bit words ([nsel][ceil((k + r) / 32)]) for the
    // masked fixed pass, and the zero buffer (one symbol long) its erased slots read
    void* d_mbits = nullptr;
    size_t mbits_cap = 0;
    void* d_zero = nullptr;
    uint64_t zero_cap = 0;
};

namespace rsamd {

// ------------------------------------------------------------------ checked launches (rs_api.cpp)
// RS_AMD_CHECK=1 (read once per process): after every launch group the library waits for the device and
// reads the sticky error, so a fault is reported at the call that queued it, with its kernel, the plan's
// K / R and slot ranges, and the call returns RS_ERR_DEVICE; plans' slot lists are bounds-checked on the
// host before their first launch. Costs a device round trip per launch: diagnosis only.
bool check_mode();
// after a launch group: 0, or RS_ERR_DEVICE with the report on stderr (p may be null)
int check_launch(const rsg_codec_t* c, const DevPlan* p, const char* where, uint64_t n_stripes, uint64_t S);
// host-side bounds of a plan's slot lists against the codec's k + r slots (check mode, first launch)
int check_plan_slots(const rsg_codec_t* c, const DevPlan& p);
#define RS_CHECKPOINT(c, p, where, n, S)                                              \
    do {                                                                              \
        if (rsamd::check_mode())                                                      \
            if (int _rc = rsamd::check_launch((c), (p), (where), (n), (S))) return _rc; \
    } while (0)

// ------------------------------------------------------------------ rs_api.cpp
// Launches below this many bytes do not count toward decode specialisation (a compile costs far more
// than tiny launches can recover).
constexpr uint64_t kJitMinBytes = uint64_t(1) << 20;
// SALU per k_cs16t step: the step's own (asm_counts.h) + the block tails (3 each, 1 for the last) + the
// loop's pointer / count updates (7)
constexpr uint64_t kSaluStepCs16t = uint64_t(kSalu_cs16t) + 3 * (4 * kCs16tCw - 1) + 1 + 7;

// One launch of plan p over n_stripes stripes (the dispatcher: XOR kernel, JIT, generic kernels, the
// GF(2^16) route, the re-encode decode); d_ids = stripe-id list, dst_local = outputs indexed by the
// launch-local stripe (XOR kernel only).
int run_plan(rsg_codec_t* c, DevPlan& p, const uint8_t* src, int64_t src_stripe, int64_t src_sym, uint8_t* dst,
             int64_t dst_stripe, int64_t dst_sym, uint64_t n_stripes, uint64_t S, hipStream_t st,
             const int32_t* d_ids = nullptr, bool dst_local = false);
// the cached decode plan of a pattern (LRU of 16)
int decode_plan(rsg_codec_t* c, const bool* is_erased, uint16_t t, DevPlan** out, hipStream_t st);
// codec scratch shared by launches on different streams: wait for / mark the last user
int scratch_acquire(rsg_codec_t* c, hipStream_t st);
int scratch_release(rsg_codec_t* c, hipStream_t st);
int scratch_fence(rsg_codec_t* c, hipStream_t st, int rc);  // release after a failed route (returns rc)

// ------------------------------------------------------------------ rs_batch.cpp
// the fixed r x (k + r) matrix of the GF(256) per-stripe route (1 syndromes, 2 re-encode differences [G | I])
std::vector<uint16_t> syn_fixed_matrix(const std::vector<uint16_t>& positions, int k, int r, int route);

// ------------------------------------------------------------------ rs_route16.cpp
int make_plan(rsg_codec_t* c, const bool* erased, std::unique_ptr<DevPlan>& out, hipStream_t st);
int make_plan_dense(rsg_codec_t* c, const bool* erased, std::unique_ptr<DevPlan>& out, hipStream_t st);
int make_plan_cs(rsg_codec_t* c, const bool* erased, std::unique_ptr<DevPlan>& out, hipStream_t st);
int make_plan_reenc(rsg_codec_t* c, const bool* erased, std::unique_ptr<DevPlan>& out, hipStream_t st);
bool reenc_eligible(const rsg_codec_t* c, const bool* erased);
// the route plan of a decode pattern: the plain route, or the re-encode decode (reenc_ok: the launch allows it)
int make_plan_route(rsg_codec_t* c, const bool* erased, bool reenc_ok, std::unique_ptr<DevPlan>& out,
                    hipStream_t st);
int build_cs16(DevPlan& p, const std::vector<uint16_t>& pos, const std::vector<int32_t>& in_slots, int D,
               hipStream_t st);
int run_cs(rsg_codec_t* c, DevPlan& p, const uint8_t* src, int64_t src_stripe, int64_t src_sym, uint8_t* dst,
           int64_t dst_stripe, int64_t dst_sym, uint64_t n_stripes, uint64_t S, hipStream_t st,
           const int32_t* groups = nullptr);
int run_reenc(rsg_codec_t* c, DevPlan& p, uint8_t* base, int64_t stripe_stride, int64_t sym, uint64_t n_stripes,
              uint64_t S, hipStream_t st);
// the codec's syndrome stream and its events (per-stripe routes, m16_cs_overlap), created on first use
int overlap_objects(rsg_codec_t* c);

// ------------------------------------------------------------------ rs_hostmem.cpp
// symbols of at least this many bytes are allocated in whole pages of their own and registrable
constexpr size_t kRegMinBytes = size_t(16) << 10;
uint8_t* arena_alloc(size_t length, size_t P);
bool arena_release(const uint8_t* p);
const uint8_t* arena_run(symbol_t* const* syms, size_t cnt, size_t S, size_t* pitch, uint8_t** dev);
uint8_t* sym_alloc(size_t S);
bool sym_release(uint8_t* p);
bool sym_devptrs(symbol_t* const* syms, size_t cnt, size_t S, uint64_t* out);
bool strided_run(const uint64_t* p, size_t cnt, size_t S, size_t* pitch);

}  // namespace rsamd
