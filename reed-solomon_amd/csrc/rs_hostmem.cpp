// rs_hostmem.cpp -- host memory of the reference API (memory/symbol.h, memory/seq.h): page-locked
// seq_create arenas and slabs, library-allocated caller symbols (sym_alloc: reserved address
// ranges, lazy registration, the idle pool) and the registry the per-call paths consult.
#include "rs_core.hpp"

#include <sys/mman.h>
#include <unistd.h>
using namespace rsamd;

namespace rsamd {

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
uint8_t* pinned_block(size_t bytes, uint8_t** dev) {
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

// Caller-owned symbols outside the arenas (symbol_create; seq_create with RS_AMD_PINNED_SEQ=0). symbol_create
// stays a host-only allocation, as the reference's calloc (src/memory/symbol.c:25): data of kRegMinBytes or
// more gets whole pages of its own at increasing addresses of a reserved address range (sym_va_take), and
// no HIP call is made. The first rs_* call that moves such symbols page-locks and maps them
// (sym_devptrs -> sym_register, within the pinned cap); from then on calls move them with zero-copy or
// gather / scatter kernels across PCIe instead of host copies through staging. Only buffers this library
// allocated are registered: it alone knows when they are freed.
//
// An address range that was once registered is never handed to another allocator (DESIGN.md section 9,
// "registered caller symbols": the round-3 fault). symbol_destroy parks a block, still registered, in an
// idle pool (later symbol_create calls of a similar size take it back: no second registration); past the
// pool's cap it unregisters the block and retires the range: its memory goes back to the OS (PROT_NONE,
// MAP_NORESERVE) but the addresses stay reserved. Every register / unregister result is checked. A block
// whose registration cannot be undone -- hipHostUnregister fails, or the runtime still reports the range
// afterwards -- is stuck: it stays mapped, out of circulation and counted against the pinned cap, and the
// first such event is logged.
constexpr size_t kPage = 4096;
struct SymEnt {
    size_t bytes;           // whole pages
    uint8_t* dev;           // device-visible address once registered
    bool stuck = false;     // a registration that could not be undone (see above)
};
struct SymRegistry {
    std::mutex mu;
    std::unordered_map<uintptr_t, SymEnt> m;  // live symbols
    size_t idle_bytes = 0;                    // blocks parked in sym_idle()
    uint8_t* va_base = nullptr;               // current address reservation (sym_va_take)
    size_t va_size = 0, va_used = 0;
    size_t pool_cap = 0;                      // idle pool cap (bytes): RS_AMD_SYM_POOL_MB, default 1 GiB
    rsg_symbol_stats_t st{};                  // counters (rsg_symbol_stats)
    std::vector<std::pair<uint8_t*, size_t>> stuck;  // stuck blocks of destroyed symbols
    bool logged = false;                      // the first failure has been reported
    SymRegistry() {
        pool_cap = size_t(1) << 30;
        if (const char* e = std::getenv("RS_AMD_SYM_POOL_MB")) pool_cap = size_t(std::strtoull(e, nullptr, 10)) << 20;
    }
};
SymRegistry& symreg() {
    static SymRegistry* r = new SymRegistry;  // never destroyed: symbols may outlive static destructors
    return *r;
}

// address reservation per mmap: 64 GiB, or RS_AMD_SYM_VA_MB (tests: a small value exercises the step to
// the next reservation)
size_t sym_va_chunk() {
    static const size_t v = [] {
        if (const char* e = std::getenv("RS_AMD_SYM_VA_MB")) return std::max<size_t>(1, std::strtoull(e, nullptr, 10)) << 20;
        return size_t(64) << 30;
    }();
    return v;
}

// Fresh pages at increasing addresses from a reserved address range (no memory behind it until used),
// so consecutive symbol_create calls of one size sit at one stride (the zero-copy kernels' condition)
// and no address is ever handed out twice except through the idle pool. R.mu held.
uint8_t* sym_va_take(SymRegistry& R, size_t bytes) {
    if (!R.va_base || R.va_used + bytes > R.va_size) {
        const size_t sz = std::max(sym_va_chunk(), bytes);
        void* r = mmap(nullptr, sz, PROT_NONE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
        if (r == MAP_FAILED) return nullptr;
        R.va_base = static_cast<uint8_t*>(r);  // the rest of the previous reservation is never used
        R.va_size = sz;
        R.va_used = 0;
    }
    uint8_t* p = R.va_base + R.va_used;
    if (mmap(p, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_FIXED, -1, 0) == MAP_FAILED)
        return nullptr;
    R.va_used += bytes;
    return p;
}

// memory back to the OS, the address range kept reserved (never reused)
void sym_va_retire(uint8_t* p, size_t bytes) {
    if (mmap(p, bytes, PROT_NONE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_FIXED | MAP_NORESERVE, -1, 0) == MAP_FAILED)
        std::fprintf(stderr, "librs_amd: retiring a symbol range failed (its memory stays mapped)\n");
}

// a parked block (registered, or not when it was never registered): host address and entry
struct IdleBlock {
    uint8_t* host;
    SymEnt e;
};
std::multimap<size_t, IdleBlock>& sym_idle() {
    static auto* m = new std::multimap<size_t, IdleBlock>;  // guarded by symreg().mu
    return *m;
}

void sym_log_once(SymRegistry& R, const char* what, uint8_t* p, size_t bytes, hipError_t e) {
    if (R.logged) return;
    R.logged = true;
    std::fprintf(stderr,
                 "librs_amd: %s of symbol pages [%p, +%zu) failed (%s); the block stays mapped, out of circulation "
                 "and counted against the pinned cap (reported once)\n",
                 what, static_cast<void*>(p), bytes, hipGetErrorString(e));
}

// true when the runtime knows an address of [p, p + bytes) (first, middle or last byte)
bool sym_runtime_knows(const uint8_t* p, size_t bytes) {
    for (const uint8_t* q : {p, p + bytes / 2, p + bytes - 1}) {
        hipPointerAttribute_t attr{};
        const bool known = hipPointerGetAttributes(&attr, q) == hipSuccess && attr.type != hipMemoryTypeUnregistered;
        (void)hipGetLastError();
        if (known) return true;
    }
    return false;
}

// undoes one of our registrations (R.mu held): true when the runtime returned success and no longer
// knows the range
bool sym_unregister(SymRegistry& R, uint8_t* p, size_t bytes) {
    const hipError_t e = hipHostUnregister(p);
    (void)hipGetLastError();
    const bool ok = e == hipSuccess && !sym_runtime_knows(p, bytes);
    if (ok) {
        ++R.st.unregistrations;
        return true;
    }
    ++R.st.unregister_failures;
    sym_log_once(R, e == hipSuccess ? "unregistration (range still known to the runtime)" : "unregistration", p,
                 bytes, e);
    return false;
}

uint8_t* sym_alloc(size_t S) {
    if (S < kRegMinBytes) return nullptr;
    const size_t bytes = (S + kPage - 1) / kPage * kPage;
    SymRegistry& R = symreg();
    std::lock_guard<std::mutex> lk(R.mu);
    auto& idle = sym_idle();
    auto it = idle.lower_bound(bytes);
    if (it != idle.end() && it->first <= 2 * bytes) {  // a parked block of a similar size, registration kept
        IdleBlock b = it->second;
        idle.erase(it);
        R.idle_bytes -= b.e.bytes;
        ++R.st.idle_reuses;
        std::memset(b.host, 0, b.e.bytes);
        R.m[uintptr_t(b.host)] = b.e;
        return b.host;
    }
    uint8_t* p = sym_va_take(R, bytes);
    if (!p) return nullptr;
    R.m[uintptr_t(p)] = SymEnt{bytes, nullptr};  // registered by the first call that moves it (sym_devptrs)
    return p;
}

// page-locks and maps one registry entry (R.mu held); false when the cap or the runtime refuses
bool sym_register(SymRegistry& R, uint8_t* p, SymEnt& e) {
    if (e.dev) return true;
    if (e.stuck) return false;
    ArenaRegistry& A = arenas();
    {
        std::lock_guard<std::mutex> la(A.mu);
        if (A.no_pinning || A.pinned + e.bytes > pinned_cap()) return false;
        A.pinned += e.bytes;
    }
    auto unpin = [&] {
        std::lock_guard<std::mutex> la(A.mu);
        A.pinned -= e.bytes;
    };
    // never touch a range the runtime already knows: a failed registration must not be followed by an
    // unregister, which would remove the owner's mapping
    if (sym_runtime_knows(p, e.bytes)) {
        ++R.st.register_failures;
        unpin();
        return false;
    }
    const hipError_t er = hipHostRegister(p, e.bytes, hipHostRegisterMapped | hipHostRegisterPortable);
    (void)hipGetLastError();
    if (er != hipSuccess) {
        ++R.st.register_failures;
        unpin();
        return false;
    }
    ++R.st.registrations;
    void* dv = nullptr;
    const hipError_t ed = hipHostGetDevicePointer(&dv, p, 0);
    (void)hipGetLastError();
    if (ed != hipSuccess || !dv) {
        ++R.st.register_failures;
        if (sym_unregister(R, p, e.bytes)) {
            unpin();
        } else {
            e.stuck = true;  // still registered as far as we know: keep it counted, never register again
        }
        return false;
    }
    e.dev = static_cast<uint8_t*>(dv);
    return true;
}

// a block leaving circulation (R.mu held): unregistered (when registered) and retired, or kept stuck
void sym_retire_block(SymRegistry& R, uint8_t* p, const SymEnt& e) {
    if (e.stuck || (e.dev && !sym_unregister(R, p, e.bytes))) {
        R.stuck.emplace_back(p, e.bytes);  // mapped, out of circulation, still counted as pinned
        ++R.st.stuck_blocks;
        R.st.stuck_bytes += e.bytes;
        return;
    }
    sym_va_retire(p, e.bytes);
    ++R.st.retired_blocks;
    if (e.dev) {
        ArenaRegistry& A = arenas();
        std::lock_guard<std::mutex> la(A.mu);
        A.pinned -= e.bytes;
    }
}

// true (and p parked, retired or kept stuck) when p came from sym_alloc
bool sym_release(uint8_t* p) {
    SymRegistry& R = symreg();
    std::lock_guard<std::mutex> lk(R.mu);
    auto it = R.m.find(uintptr_t(p));
    if (it == R.m.end()) return false;
    const SymEnt e = it->second;
    R.m.erase(it);
    if (!e.stuck && R.idle_bytes + e.bytes <= R.pool_cap) {
        sym_idle().emplace(e.bytes, IdleBlock{p, e});
        R.idle_bytes += e.bytes;
        return true;
    }
    sym_retire_block(R, p, e);
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
        if (!it->second.dev && !sym_register(R, syms[i]->data, it->second)) return false;
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

}  // namespace rsamd

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

extern "C" int rsg_symbol_registered(const void* data) {
    SymRegistry& R = symreg();
    std::lock_guard<std::mutex> lk(R.mu);
    auto it = R.m.find(uintptr_t(data));
    return it == R.m.end() ? -1 : (it->second.dev ? 1 : 0);
}

extern "C" int rsg_symbol_stats(rsg_symbol_stats_t* out) {
    if (!out) return RS_ERR_INVALID;
    SymRegistry& R = symreg();
    std::lock_guard<std::mutex> lk(R.mu);
    *out = R.st;
    out->live = R.m.size();
    out->live_registered = 0;
    for (const auto& kv : R.m) out->live_registered += kv.second.dev ? 1 : 0;
    out->idle_blocks = sym_idle().size();
    out->idle_bytes = R.idle_bytes;
    ArenaRegistry& A = arenas();
    std::lock_guard<std::mutex> la(A.mu);
    out->pinned_bytes = A.pinned;
    return 0;
}

extern "C" int64_t rsg_symbol_pool_cap(int64_t bytes) {
    SymRegistry& R = symreg();
    std::lock_guard<std::mutex> lk(R.mu);
    const int64_t prev = int64_t(R.pool_cap);
    if (bytes < 0) return prev;
    R.pool_cap = size_t(bytes);
    auto& idle = sym_idle();
    while (R.idle_bytes > R.pool_cap && !idle.empty()) {  // a lowered cap: the largest parked blocks leave now
        auto it = std::prev(idle.end());
        const IdleBlock b = it->second;
        idle.erase(it);
        R.idle_bytes -= b.e.bytes;
        sym_retire_block(R, b.host, b.e);
    }
    return prev;
}
