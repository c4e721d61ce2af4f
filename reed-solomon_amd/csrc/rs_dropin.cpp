// rs_dropin.cpp -- the reference codec API (rs/reed_solomon.h:44-74): rs_create / rs_destroy and the
// per-call rs_generate_repair_symbols / rs_restore_symbols over caller-owned host symbols
// (zero-copy launches on page-locked arenas and registered symbols, DMA, host gather / scatter).
#include "rs_core.hpp"

#include <thread>
using namespace rsamd;

namespace rsamd {

constexpr int kMaxChunks = 4;

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

}  // namespace rsamd

extern "C" RS_t* rs_create(void) {
    rsamd::CallerDevice caller_device;
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
    rsamd::CallerDevice caller_device;
    if (!rs) return;
    delete static_cast<Impl*>(rs->impl);
    gf_destroy(rs->gf);
    cc_destroy(rs->cc);
    std::free(rs);
}

namespace {

// The per-call encode on an even symbol size (rs_generate_repair_symbols handles odd ones around it).
int generate_even(RS_t* rs, const symbol_seq_t* inf, symbol_seq_t* rep) {
    Impl& im = *static_cast<Impl*>(rs->impl);
    const size_t S = inf->symbol_size;
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

// The per-call restore on an even symbol size (rs_restore_symbols handles odd ones around it).
int restore_even(RS_t* rs, uint16_t k, uint16_t r, symbol_seq_t* rcv, const bool* is_erased, uint16_t t) {
    Impl& im = *static_cast<Impl*>(rs->impl);
    const size_t S = rcv->symbol_size, n = size_t(k) + r;
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

}  // namespace

// Odd symbol sizes follow the reference's Release build (-DNDEBUG, the baseline's flags), where the
// symbol-wide operations cover symbol_size / 2 words (gf65536.c:158-169): the code runs on the even
// prefix, and every symbol the call writes ends in a zero byte -- fft_partial_transform_cycl memsets each
// repair symbol first (fft.c:163), _rs_restore_erased each restored one (reed_solomon.c:326). Golden cases
// odd_* pin both (tests/golden/make_golden.py).
extern "C" int rs_generate_repair_symbols(RS_t* rs, const symbol_seq_t* inf, symbol_seq_t* rep) {
    rsamd::CallerDevice caller_device;
    if (!rs || !rs->impl || !inf || !rep) return RS_ERR_INVALID;
    const size_t S = inf->symbol_size;
    if (S != rep->symbol_size || inf->length + rep->length > kN) return RS_ERR_INVALID;
    if (!(S & 1)) return generate_even(rs, inf, rep);
    const symbol_seq_t ie = {inf->length, S - 1, inf->symbols};
    symbol_seq_t re = {rep->length, S - 1, rep->symbols};
    const int rc = generate_even(rs, &ie, &re);
    if (rc == 0)
        for (size_t j = 0; j < rep->length; ++j) rep->symbols[j]->data[S - 1] = 0;
    return rc;
}

extern "C" int rs_restore_symbols(RS_t* rs, uint16_t k, uint16_t r, symbol_seq_t* rcv, const bool* is_erased,
                                  uint16_t t) {
    rsamd::CallerDevice caller_device;
    if (r < t) return RS_ERR_CANNOT_RESTORE;  // checked first, as reference reed_solomon.c:467-470
    if (!rs || !rs->impl || !rcv || !is_erased) return RS_ERR_INVALID;
    const size_t S = rcv->symbol_size, n = size_t(k) + r;
    if (rcv->length != n || n > kN) return RS_ERR_INVALID;
    if (!(S & 1)) return restore_even(rs, k, r, rcv, is_erased, t);
    symbol_seq_t e = {rcv->length, S - 1, rcv->symbols};
    const int rc = restore_even(rs, k, r, &e, is_erased, t);
    if (rc == 0)
        for (size_t i = 0; i < k; ++i)
            if (is_erased[i]) rcv->symbols[i]->data[S - 1] = 0;
    return rc;
}
