// rs_refops.cpp -- the reference's secondary surface: GF_t / CC_t (rs/gf65536.h, rs/cyclotomic_coset.h),
// the context-free symbol operations gf_add / gf_mul / gf_madd and the four fft_* transforms, run on
// the GPU through a pool of engines.
#include "rs_core.hpp"
#include "rs_symops.hpp"

using namespace rsamd;

namespace rsamd {

// normal bases of GF(2), GF(4), GF(16), GF(256), GF(2^16): facts restated from reference gf65536.c:21-57
const uint16_t kNormalBases[GF_NORMAL_BASES_ELEMENTS] = {
    1,                                                           // GF(2)
    44234, 44235,                                                // GF(4)
    10800, 47860, 34555, 5694,                                   // GF(16)
    16402, 53598, 44348, 63986, 22060, 64366, 6088, 32521,       // GF(256)
    2048, 2880, 7129, 30616, 2643, 6897, 29685, 7378, 30100, 2743, 20193, 36223, 24055, 41458, 41014, 61451};

int m_index(uint8_t m) { return m == 1 ? 0 : m == 2 ? 1 : m == 4 ? 3 : m == 8 ? 7 : 15; }

// normal_repr[li][d]: bits of alpha^d in the normal basis of GF(2^m), m = 1 << li (0 when alpha^d is
// not in GF(2^m)), as reference gf65536.c:90-108 tabulates them
const std::vector<uint16_t>* normal_repr_tables() {
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

uint16_t normal_basis_element(int m, int i) { return kNormalBases[m_index(uint8_t(m)) + i]; }

}  // namespace rsamd

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

namespace rsamd {

// ============================================================================ context-free host ops
// gf_add / gf_mul / gf_madd and the fft_* transforms take host symbols and no codec. They run on the
// GPU through a pool of engines: a call leases one (a mutex only around the pool's free list, so
// concurrent callers run side by side), and each engine has its own non-blocking stream, page-locked
// mapped staging that only grows (with its device-visible address) and an m = 16 codec shell whose
// matrix kernels, options and split-K scratch the transforms use. An engine serves the device that was
// current when it was created; leases prefer an engine of the caller's current device.

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
    // gf_madd 172 us with DMA vs 199 us zero-copy, profiles/r3/r3_hostops.jsonl)
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
    plan->slot_bound = int32_t(std::max(K, R));  // staging rows, not codec slots
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

}  // namespace rsamd

extern "C" void gf_add(void* a, const void* b, size_t symbol_size) {
    rsamd::CallerDevice caller_device;
    if (int rc = symbol_op(0, a, 0, b, symbol_size)) symbol_op_failed("gf_add", rc);
}

extern "C" void gf_mul(GF_t* gf, void* a, element_t coef, size_t symbol_size) {
    rsamd::CallerDevice caller_device;
    (void)gf;
    if (coef == 0) {  // reference gf65536.c:175-181
        std::memset(a, 0, symbol_size);
        return;
    }
    if (coef == 1) return;
    if (int rc = symbol_op(1, a, coef, nullptr, symbol_size)) symbol_op_failed("gf_mul", rc);
}

extern "C" void gf_madd(GF_t* gf, void* a, element_t coef, const void* b, size_t symbol_size) {
    rsamd::CallerDevice caller_device;
    (void)gf;
    if (coef == 0) return;  // reference gf65536.c:199-205
    if (int rc = symbol_op(coef == 1 ? 0 : 2, a, coef, b, symbol_size)) symbol_op_failed("gf_madd", rc);
}

// ============================================================================ batched symbol ops
// rsg_symbol_ops (include/rs_amd/rsg.h): many gf_add / gf_mul / gf_madd triples on device-accessible
// symbols in one call, asynchronous on the caller's stream: the ops sorted into per-target chains and folded
// into canonical kinds here, then one op-list copy and two kernels (rs_symops.hip: the multiply constants,
// then the chains). The op list goes to the device through one of kOpSlots page-locked staging slots per
// device (each reused only after the launches that read it are done: its event), so a call returns as soon as
// the copy and the kernels are queued.
namespace rsamd {
namespace {
constexpr int kOpSlots = 4;
struct OpSlot {
    uint8_t* h = nullptr;  // page-locked staging
    uint8_t* d = nullptr;  // device copy read by the kernel
    size_t cap = 0;
    hipEvent_t ev = nullptr;
    bool pending = false;
};
struct OpStage {
    std::mutex mu;
    OpSlot slot[kOpSlots];
    int next = 0;
};
OpStage& op_stage(int device) {
    static std::mutex mu;
    static std::map<int, OpStage*>* m = new std::map<int, OpStage*>();  // never destroyed (outlives HIP teardown)
    std::lock_guard<std::mutex> lk(mu);
    OpStage*& p = (*m)[device];
    if (!p) p = new OpStage();
    return *p;
}

// An rsg_symbol_op_t in the kernel's canonical form (rs_symops.hpp): the reference's special cases folded on
// the host (gf65536.c:175-181 mul by 0 / 1, :199-205 madd by 0 / 1), a source equal to the target read as a
// scale (a ^= a is 0, a ^= c a is (1 + c) a), so the device never branches on them per word.
SymOpRec canonical_op(const rsg_symbol_op_t& o) {
    const uint32_t c = o.coef;
    const bool self = o.b == o.a;
    auto scale = [](uint32_t m) {
        if (m == 0u) return SymOpRec{nullptr, 0u, kSymZero};
        return m == 1u ? SymOpRec{nullptr, 1u, kSymNop} : SymOpRec{nullptr, m, kSymScale};
    };
    switch (o.op) {
        case RSG_OP_ADD:
            return self ? scale(0u) : SymOpRec{static_cast<const uint8_t*>(o.b), 1u, kSymXor};
        case RSG_OP_MUL:
            return scale(c);
        default:  // RSG_OP_MADD
            if (c == 0u) return SymOpRec{nullptr, 0u, kSymNop};
            if (self) return scale(c ^ 1u);
            return c == 1u ? SymOpRec{static_cast<const uint8_t*>(o.b), 1u, kSymXor}
                           : SymOpRec{static_cast<const uint8_t*>(o.b), c, kSymMadd};
    }
}

}  // namespace

}  // namespace rsamd

extern "C" int rsg_symbol_ops(int device, const rsg_symbol_op_t* ops, uint64_t n_ops, uint64_t symbol_size,
                              void* stream) {
    if (n_ops && !ops) return RS_ERR_INVALID;
    if (n_ops > 0xFFFFFFFFull) return RS_ERR_INVALID;
    const uint64_t nwords = symbol_size / 2, span = nwords * 2;  // an odd last byte is not touched
    // chains: the ops of each target in array order = the (target, index) pairs sorted; every pointer 4-byte
    // aligned (dword kernel)
    std::vector<std::pair<uintptr_t, uint32_t>> order(n_ops);
    std::vector<uint8_t> scaling(n_ops);  // the op scales its target (canonical kSymScale / kSymZero)
    for (uint64_t i = 0; i < n_ops; ++i) {
        const rsg_symbol_op_t& o = ops[i];
        if (o.op > RSG_OP_MADD || !o.a || (uintptr_t(o.a) & 3)) return RS_ERR_INVALID;
        if (o.op != RSG_OP_MUL && (!o.b || (uintptr_t(o.b) & 3))) return RS_ERR_INVALID;
        order[i] = {uintptr_t(o.a), uint32_t(i)};
        const bool self = o.op != RSG_OP_MUL && o.b == o.a && !(o.op == RSG_OP_MADD && o.coef == 0);  // (1 + c) a
        scaling[i] = (o.op == RSG_OP_MUL && o.coef != 1) || self;
    }
    std::sort(order.begin(), order.end());
    // distinct targets (ascending), each chain's length and whether it scales its target (known before any
    // record is written: the slice count decides how many combine records those chains need). Targets must not
    // overlap each other, and no op may read another op's target (the chains run side by side): both rejected,
    // nothing is queued
    std::vector<uintptr_t> tg;
    std::vector<uint32_t> cnt;
    std::vector<uint8_t> scales;
    for (size_t j = 0; j < order.size(); ++j) {
        if (!j || order[j].first != order[j - 1].first) {
            tg.push_back(order[j].first);
            cnt.push_back(0);
            scales.push_back(0);
        }
        ++cnt.back();
        scales.back() |= scaling[order[j].second];
    }
    for (size_t i = 1; i < tg.size(); ++i)
        if (tg[i - 1] + span > tg[i]) return RS_ERR_INVALID;
    if (span) {
        for (uint64_t i = 0; i < n_ops; ++i) {
            const rsg_symbol_op_t& o = ops[i];
            if (o.op == RSG_OP_MUL || o.b == o.a) continue;
            const uintptr_t b = uintptr_t(o.b);
            auto hi = std::upper_bound(tg.begin(), tg.end(), b + span - 1);  // first target past the source
            if (hi != tg.begin() && *(hi - 1) + span > b) return RS_ERR_INVALID;
        }
    }
    if (tg.empty() || !nwords) return 0;
    if (device < 0) return RS_ERR_INVALID;
    CallerDevice scope;
    HIP_TRY(hipSetDevice(device));
    hipStream_t st = static_cast<hipStream_t>(stream);
    const size_t nc = tg.size();
    const uint32_t cnt_max = *std::max_element(cnt.begin(), cnt.end());
    const size_t n_scaling = size_t(std::count(scales.begin(), scales.end(), uint8_t(1)));
    // dwords per lane: the largest of 4 / 2 that still gives >= 4096 waves (4 per SIMD), else 1 (more waves
    // for few or short targets: the chains are bound by load latency); RS_AMD_SYMOP_DW = 1 / 2 / 4 overrides
    static const int dw_env = [] {
        const char* e = std::getenv("RS_AMD_SYMOP_DW");
        const int v = e ? std::atoi(e) : 0;
        return v == 1 || v == 2 || v == 4 ? v : 0;
    }();
    const uint64_t nd = nwords / 2 + (nwords & 1);
    auto waves = [&](uint64_t dw) { return uint64_t(nc) * ((nd + 64 * dw - 1) / (64 * dw)); };
    const int dw = dw_env ? dw_env : waves(4) >= 4096 ? 4 : waves(2) >= 4096 ? 2 : 1;
    // waves per chain: while the launch has fewer than 8192 waves, cut the chains into 2, 4, 8 slices (each
    // slice of the longest chain keeping >= 4 ops); RS_AMD_SYMOP_WAVES = 1..8 (a power of 2) overrides
    static const int wv_env = [] {
        const char* e = std::getenv("RS_AMD_SYMOP_WAVES");
        const int v = e ? std::atoi(e) : 0;
        return v == 1 || v == 2 || v == 4 || v == 8 ? v : 0;
    }();
    int wv = 1;
    if (wv_env)
        wv = wv_env;
    else
        while (2 * wv <= kSymMaxWaves && waves(uint64_t(dw)) * wv < 8192 && cnt_max / (2 * wv) >= 4) wv *= 2;
    if (wv > 1 && n_ops + uint64_t(wv) * n_scaling > 0xFFFFFFFFull) wv = 1;  // combine records past 32-bit ids
    const uint64_t n_rec = n_ops + (wv > 1 ? uint64_t(wv) * n_scaling : 0);  // ops + combine records
    const size_t bytes = nc * sizeof(SymChain) + n_rec * sizeof(SymOpRec);  // copied to the device
    const size_t cbase = (bytes + 63) / 64 * 64;                           // multiply constants after them
    const size_t dbytes = cbase + symbol_chains_scratch(n_rec);
    OpStage& S = op_stage(device);
    std::lock_guard<std::mutex> lk(S.mu);
    OpSlot& sl = S.slot[S.next];
    S.next = (S.next + 1) % kOpSlots;
    if (sl.pending) HIP_TRY(hipEventSynchronize(sl.ev));  // the launch that read this slot is done
    sl.pending = false;
    if (!sl.ev) HIP_TRY(hipEventCreateWithFlags(&sl.ev, hipEventDisableTiming));
    if (dbytes > sl.cap) {  // host staging and device copy of one size (the host side never holds constants)
        if (sl.h) (void)hipHostFree(sl.h);
        if (sl.d) (void)hipFree(sl.d);
        sl.h = sl.d = nullptr;
        sl.cap = 0;
        const size_t cap = std::max<size_t>(dbytes + dbytes / 2, 1 << 20);  // grows by half again: few reallocations
        HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&sl.h), cap, hipHostMallocDefault));
        HIP_TRY(hipMalloc(reinterpret_cast<void**>(&sl.d), cap));
        sl.cap = cap;
    }
    // records straight into the page-locked slot: chains, the ops in chain order, the combine records
    SymChain* hc = reinterpret_cast<SymChain*>(sl.h);
    SymOpRec* ho = reinterpret_cast<SymOpRec*>(sl.h + nc * sizeof(SymChain));
    for (size_t j = 0, ci = 0; j < order.size(); ++j) {
        const rsg_symbol_op_t& o = ops[order[j].second];
        if (j && order[j].first != order[j - 1].first) ++ci;
        if (!j || order[j].first != order[j - 1].first)
            hc[ci] = SymChain{static_cast<uint8_t*>(o.a), uint32_t(j), cnt[ci],
                              kChainSplit | (scales[ci] && wv > 1 ? kChainAffine : 0u), 0};
        ho[j] = canonical_op(o);
    }
    if (wv > 1 && n_scaling) {
        // slice w of a chain = ops [w len, (w + 1) len) as the kernel cuts it; its result is multiplied by
        // S_w = M_(w+1) ... M_(W-1), M_l = the product of slice l's scale factors (0 if it zeroes the target)
        const Field& F = field();
        uint64_t comb = n_ops;
        for (size_t c = 0; c < nc; ++c) {
            if (!scales[c]) continue;
            hc[c].comb = uint32_t(comb);
            const uint32_t len = (hc[c].count + uint32_t(wv) - 1) / uint32_t(wv);
            uint16_t M[kSymMaxWaves];
            for (int w = 0; w < wv; ++w) {
                M[w] = 1;
                const uint32_t e0 = std::min(uint32_t(w) * len, hc[c].count);
                const uint32_t e1 = std::min((uint32_t(w) + 1) * len, hc[c].count);
                for (uint32_t i = e0; i < e1; ++i) {
                    const SymOpRec& r = ho[hc[c].start + i];
                    if (r.kind == kSymZero)
                        M[w] = 0;
                    else if (r.kind == kSymScale)
                        M[w] = F.mul(M[w], uint16_t(r.coef));
                }
            }
            uint16_t after = 1;
            for (int w = wv - 1; w >= 0; --w) {
                ho[comb + uint64_t(w)] = after == 0   ? SymOpRec{nullptr, 0u, kSymZero}
                                         : after == 1 ? SymOpRec{nullptr, 1u, kSymNop}
                                                      : SymOpRec{nullptr, after, kSymScale};
                after = F.mul(after, M[w]);
            }
            comb += uint64_t(wv);
        }
    }
    HIP_TRY(hipMemcpyAsync(sl.d, sl.h, bytes, hipMemcpyHostToDevice, st));
    const SymChain* dc = reinterpret_cast<const SymChain*>(sl.d);
    const SymOpRec* dops = reinterpret_cast<const SymOpRec*>(sl.d + nc * sizeof(SymChain));
    uint32_t* dconsts = reinterpret_cast<uint32_t*>(sl.d + cbase);
    hipError_t e = launch_symop_consts(dops, n_rec, dconsts, st);
    for (size_t c0 = 0; c0 < nc && e == hipSuccess; c0 += 65535)
        e = launch_symbol_chains(dc + c0, dops, dconsts, uint32_t(std::min<size_t>(65535, nc - c0)), nwords, st, dw,
                                 wv);
    // the slot is reused after this event, whatever happened to the launches
    HIP_TRY(hipEventRecord(sl.ev, st));
    sl.pending = true;
    if (e != hipSuccess) return hip_fail(e, "k_symbol_chains");
    return 0;
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
    rsamd::CallerDevice caller_device;
    (void)gf;
    if (!f || !res || (!positions && f->length)) symbol_op_failed("fft_transform (bad arguments)", RS_ERR_INVALID);
    if (int rc = transform_apply(dft_matrix(f, positions, res), f, res)) symbol_op_failed("fft_transform", rc);
}

extern "C" int fft_transform_cycl(GF_t* gf, const symbol_seq_t* f, const uint16_t* positions, symbol_seq_t* res) {
    rsamd::CallerDevice caller_device;
    (void)gf;
    if (!f || !res || (!positions && f->length)) return RS_ERR_INVALID;
    return transform_apply(dft_matrix(f, positions, res), f, res);
}

extern "C" void fft_partial_transform(GF_t* gf, const symbol_seq_t* f, const uint16_t* components,
                                      symbol_seq_t* res) {
    rsamd::CallerDevice caller_device;
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
    rsamd::CallerDevice caller_device;
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
