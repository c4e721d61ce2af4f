// rs_xj.cpp -- generator, cache and launcher of the bit-plane XOR kernels (see rs_xj.hpp).
//
// Generated kernel `rs_xj` (one per coding matrix and slot lists):
//   grid (column chunks of 256 B, stripes), block = 64 x roles threads. All waves of a block work on
//   the same 256-byte column of one stripe; wave w ("role") owns outputs 8w .. 8w+7.
//   Register contract of a role (fixed, so the generated code can name registers directly):
//     v[8:71]   accumulators u_{q,t} of output q (0..7), bit-plane t (0..7): v[8 + 8q + t]
//     v[72:95]  input ring, 3 slots x 8 inputs (one group pair = 8 consecutive inputs)
//     v[96:106] / v[107:117]  non-trivial subset XORs of the pair's groups A (inputs 0-3) / B (4-7)
//     v118      this lane's byte offset in the symbol (column)
//     v[72:103] after the XOR network: finish registers H, T1, T2 (spare) of output q at v[72 + 4q]
//     s[32:38]  src base, src symbol stride, dst base, dst symbol stride; s[40:55] address pairs;
//     s[56:59]  call / return address of the shared finish block; s[64:71] output byte offsets
//   The finish block (Horner in alpha^-1 over the 8 bit-plane accumulators of all 8 outputs) is emitted
//   once at the kernel entry and entered by s_swappc_b64 from every role.
#include "rs_xj.hpp"

#include <algorithm>
#include <cstdio>
#include <sstream>

#include "gf16.hpp"
#include "rs_jit.hpp"

namespace rsamd {

// ------------------------------------------------------------------------------- host math
static int parity16(uint32_t v) { return __builtin_popcount(v & 0xFFFFu) & 1; }

XjBasis::XjBasis() {
    const Field& F = field();
    // A: column j = alpha^-j (16-bit); invert over GF(2) by Gauss-Jordan on rows.
    uint32_t row[16];  // row i: bits j = bit i of alpha^-j ; augmented identity in bits 16..31
    for (int i = 0; i < 16; ++i) {
        uint32_t r = 0;
        for (int j = 0; j < 16; ++j)
            if ((F.exp[(kN - j) % kN] >> i) & 1) r |= 1u << j;
        row[i] = r | (1u << (16 + i));
    }
    for (int c = 0; c < 16; ++c) {
        int p = c;
        while (!((row[p] >> c) & 1)) ++p;  // A is invertible (alpha^-j are independent)
        std::swap(row[p], row[c]);
        for (int i = 0; i < 16; ++i)
            if (i != c && ((row[i] >> c) & 1)) row[i] ^= row[c];
    }
    for (int j = 0; j < 16; ++j) inv_row_[j] = uint16_t(row[j] >> 16);
    // RREF basis (pivot = highest set bit) of the GF(256) subspace in alpha^-j coordinates
    uint16_t piv[16] = {0};
    bool has[16] = {false};
    for (int t = 0; t < 8; ++t) {
        uint16_t v = ycoord(F.exp[(257u * t) % kN]);
        for (int b = 15; b >= 0; --b) {
            if (!((v >> b) & 1)) continue;
            if (has[b]) {
                v ^= piv[b];
            } else {
                has[b] = true;
                piv[b] = v;
                break;
            }
        }
    }
    for (int b = 0; b < 16; ++b)  // full reduction
        if (has[b])
            for (int q = 0; q < 16; ++q)
                if (q != b && has[q] && ((piv[q] >> b) & 1)) piv[q] ^= piv[b];
    int t = 0;
    for (int b = 0; b < 16; ++b)
        if (has[b]) {
            pivots[t] = b;
            beta_y[t] = piv[b];
            ++t;
        }
}

uint16_t XjBasis::ycoord(uint16_t x) const {
    uint16_t y = 0;
    for (int j = 0; j < 16; ++j) y |= uint16_t(parity16(inv_row_[j] & x) << j);
    return y;
}

uint8_t XjBasis::bits(uint16_t c) const {
    const uint16_t y = ycoord(c);
    uint8_t b = 0;
    for (int t = 0; t < 8; ++t) b |= uint8_t(((y >> pivots[t]) & 1) << t);
    return b;
}

const XjBasis& xj_basis() {
    static const XjBasis* b = new XjBasis();
    return *b;
}

bool xj_supported(int m, int K, int R) {
    return m <= 8 && K >= 1 && R >= 1 && R <= kXjOutputsPerRole * kXjMaxRoles && K * R <= kXjMaxWork;
}

// --------------------------------------------------------------------------- code generator
namespace {

constexpr int kAcc = 8, kRing = 72, kTabA = 96, kTabB = 107, kCol = 118;

// built-entry register index of subset pattern e (popcount >= 2) within a group's 11 registers
int built_index(int e) {
    static const int idx[16] = {-1, -1, -1, 0, -1, 1, 2, 3, -1, 4, 5, 6, 7, 8, 9, 10};
    return idx[e];
}

struct Emitter {
    std::vector<std::string> L;
    void e(const std::string& s) { L.push_back(s); }
    template <class... A>
    void f(const char* fmt, A... a) {
        char buf[160];
        std::snprintf(buf, sizeof buf, fmt, a...);
        L.emplace_back(buf);
    }
};

std::string as_string_literals(const std::vector<std::string>& L) {
    std::string o;
    for (const std::string& s : L) o += "\"" + s + "\\n\"\n";
    return o;
}

// The finish block: for every output q, H_q = sum_j alpha^-j v_j with v_j = XOR of u_{q,t} over the t
// whose beta_t has coordinate j; Horner from the top coordinate down, the 8 chains interleaved.
std::vector<std::string> finish_block() {
    const XjBasis& B = xj_basis();
    std::vector<std::vector<std::string>> chains(8);
    for (int q = 0; q < 8; ++q) {
        std::vector<std::string>& c = chains[q];
        char buf[160];
        auto add = [&](const char* fmt, auto... a) {
            std::snprintf(buf, sizeof buf, fmt, a...);
            c.emplace_back(buf);
        };
        const int H = 72 + 4 * q, T1 = H + 1, T2 = H + 2;
        auto terms = [&](int j) {
            std::vector<int> r;
            for (int t = 0; t < 8; ++t)
                if ((B.beta_y[t] >> j) & 1) r.push_back(kAcc + 8 * q + t);
            return r;
        };
        // fold `rest` (after `first` went into dst) pairwise into dst
        auto fold = [&](int dst, const std::vector<int>& v, size_t from) {
            size_t i = from;
            for (; i + 1 < v.size(); i += 2) add("v_bitop3_b32 v%d, v%d, v%d, v%d bitop3:0x96", dst, dst, v[i], v[i + 1]);
            if (i < v.size()) add("v_xor_b32 v%d, v%d, v%d", dst, v[i], dst);
        };
        int jtop = 15;
        while (jtop > 0 && terms(jtop).empty()) --jtop;
        std::vector<int> top = terms(jtop);
        int cur;
        if (top.size() == 1) {
            cur = top[0];
        } else if (top.empty()) {
            add("v_mov_b32 v%d, 0", H);
            cur = H;
        } else {
            add("v_xor_b32 v%d, v%d, v%d", H, top[0], top[1]);
            fold(H, top, 2);
            cur = H;
        }
        for (int j = jtop - 1; j >= 0; --j) {
            // cur * alpha^-1 per 16-bit lane: (w >> 1) ^ (w & 1 ? 0x8016 : 0)
            add("v_and_b32 v%d, 0xfffeffff, v%d", T1, cur);
            add("v_lshrrev_b32 v%d, 1, v%d", T1, T1);
            add("v_and_b32 v%d, 0x10001, v%d", T2, cur);
            add("v_mul_u32_u24 v%d, 0x8016, v%d", T2, T2);
            std::vector<int> v = terms(j);
            if (v.empty()) {
                add("v_xor_b32 v%d, v%d, v%d", H, T1, T2);
            } else {
                add("v_bitop3_b32 v%d, v%d, v%d, v%d bitop3:0x96", H, T1, T2, v[0]);
                fold(H, v, 1);
            }
            cur = H;
        }
        if (cur != H) add("v_mov_b32 v%d, v%d", H, cur);
    }
    std::vector<std::string> L;
    L.push_back("s_branch L_xj_fin_end");
    L.push_back("L_xj_fin:");
    const size_t n = chains[0].size();
    for (size_t i = 0; i < n; ++i)
        for (int q = 0; q < 8; ++q) L.push_back(chains[q][i]);
    L.push_back("s_setpc_b64 s[58:59]");
    L.push_back("L_xj_fin_end:");
    return L;
}

// One role: outputs p = 8w + q (q < nq) of the R x K bit-plane matrix `cb` (cb[p*K + i] = b(c_{p,i})).
std::vector<std::string> role_block(int w, const std::vector<uint8_t>& cb, int K, int R,
                                    const std::vector<int32_t>& in_slots, const std::vector<int32_t>& out_slots) {
    Emitter E;
    const int p0 = 8 * w, nq = std::min(8, R - p0);
    E.e("s_nop 4");  // "s" operands may come from v_readfirstlane (VALU SGPR write -> VMEM read)
    E.e("s_mov_b32 s32, %[sl]");
    E.e("s_mov_b32 s33, %[sh]");
    E.e("s_mov_b32 s34, %[ss]");
    E.e("s_mov_b32 s36, %[dl]");
    E.e("s_mov_b32 s37, %[dh]");
    E.e("s_mov_b32 s38, %[ds]");
    E.f("v_mov_b32 v%d, %%[col]", kCol);
    for (int q = 0; q < nq; ++q) E.f("s_mul_i32 s%d, s38, %d", 64 + q, out_slots[size_t(p0 + q)]);
    const int ngp = (K + 7) / 8;
    auto nload = [&](int g) { return g < ngp ? std::min(8, K - 8 * g) : 0; };
    auto loads = [&](int g) {
        const int n = nload(g);
        for (int j = 0; j < n; ++j) {
            E.f("s_mul_i32 s62, s34, %d", in_slots[size_t(8 * g + j)]);
            E.f("s_add_u32 s%d, s32, s62", 40 + 2 * j);
            E.f("s_addc_u32 s%d, s33, 0", 41 + 2 * j);
        }
        for (int j = 0; j < n; ++j)
            E.f("global_load_dword v%d, v%d, s[%d:%d]", kRing + 8 * (g % 3) + j, kCol, 40 + 2 * j, 41 + 2 * j);
    };
    bool init[8][8] = {};
    loads(0);
    loads(1);
    for (int g = 0; g < ngp; ++g) {
        loads(g + 2);
        E.f("s_waitcnt vmcnt(%d)", nload(g + 1) + nload(g + 2));
        // patterns of this role's rows over the pair's two groups
        int pat[8][8][2];
        bool need[2][16] = {};
        for (int q = 0; q < nq; ++q)
            for (int t = 0; t < 8; ++t)
                for (int h = 0; h < 2; ++h) {
                    int e = 0;
                    for (int jj = 0; jj < 4; ++jj) {
                        const int i = 8 * g + 4 * h + jj;
                        if (i < K && ((cb[size_t(p0 + q) * K + i] >> t) & 1)) e |= 1 << jj;
                    }
                    pat[q][t][h] = e;
                    need[h][e] = true;
                }
        auto single = [&](int h, int jj) { return kRing + 8 * (g % 3) + 4 * h + jj; };
        auto reg = [&](int h, int e) {
            if (__builtin_popcount(e) == 1) return single(h, __builtin_ctz(e));
            return (h ? kTabB : kTabA) + built_index(e);
        };
        for (int h = 0; h < 2; ++h) {
            // popcount 2 and 3 straight from the inputs; 15 from a built triple or pair
            bool built[16] = {};
            for (int e = 3; e < 15; ++e) {
                if (!need[h][e] || __builtin_popcount(e) < 2) continue;
                int b[3], nb = 0;
                for (int jj = 0; jj < 4; ++jj)
                    if ((e >> jj) & 1) b[nb++] = single(h, jj);
                if (nb == 2)
                    E.f("v_xor_b32 v%d, v%d, v%d", reg(h, e), b[0], b[1]);
                else
                    E.f("v_bitop3_b32 v%d, v%d, v%d, v%d bitop3:0x96", reg(h, e), b[0], b[1], b[2]);
                built[e] = true;
            }
            if (need[h][15]) {
                int tri = -1, pair = -1;
                for (int e : {7, 11, 13, 14})
                    if (built[e]) tri = e;
                for (int e : {3, 5, 6, 9, 10, 12})
                    if (built[e]) pair = e;
                if (tri >= 0) {
                    E.f("v_xor_b32 v%d, v%d, v%d", reg(h, 15), reg(h, tri), single(h, __builtin_ctz(15 & ~tri)));
                } else {
                    if (pair < 0) {
                        pair = 3;
                        E.f("v_xor_b32 v%d, v%d, v%d", reg(h, 3), single(h, 0), single(h, 1));
                    }
                    const int rest = 15 & ~pair;
                    E.f("v_bitop3_b32 v%d, v%d, v%d, v%d bitop3:0x96", reg(h, 15), reg(h, pair),
                        single(h, __builtin_ctz(rest)), single(h, 31 - __builtin_clz(rest)));
                }
            }
        }
        for (int t = 0; t < 8; ++t)
            for (int q = 0; q < nq; ++q) {
                const int a = pat[q][t][0], b = pat[q][t][1], acc = kAcc + 8 * q + t;
                if (!a && !b) continue;
                if (!init[q][t]) {
                    if (a && b)
                        E.f("v_xor_b32 v%d, v%d, v%d", acc, reg(0, a), reg(1, b));
                    else
                        E.f("v_mov_b32 v%d, v%d", acc, a ? reg(0, a) : reg(1, b));
                    init[q][t] = true;
                } else if (a && b) {
                    E.f("v_bitop3_b32 v%d, v%d, v%d, v%d bitop3:0x96", acc, acc, reg(0, a), reg(1, b));
                } else {
                    E.f("v_xor_b32 v%d, v%d, v%d", acc, a ? reg(0, a) : reg(1, b), acc);
                }
            }
    }
    for (int q = 0; q < nq; ++q)
        for (int t = 0; t < 8; ++t)
            if (!init[q][t]) E.f("v_mov_b32 v%d, 0", kAcc + 8 * q + t);
    // finish (shared block; returns through s[58:59]); L_xj_fin precedes every role block
    E.e("s_getpc_b64 s[56:57]");
    E.e("s_add_u32 s56, s56, L_xj_fin-.");
    E.e("s_addc_u32 s57, s57, -1");
    E.e("s_swappc_b64 s[58:59], s[56:57]");
    for (int q = 0; q < nq; ++q) {
        E.f("s_add_u32 s%d, s36, s%d", 40 + 2 * q, 64 + q);
        E.f("s_addc_u32 s%d, s37, 0", 41 + 2 * q);
    }
    for (int q = 0; q < nq; ++q) E.f("global_store_dword v%d, v%d, s[%d:%d]", kCol, 72 + 4 * q, 40 + 2 * q, 41 + 2 * q);
    E.e("s_waitcnt vmcnt(0)");
    return E.L;
}

}  // namespace

std::string xj_source(const std::vector<uint16_t>& M, int K, int R, const std::vector<int32_t>& in_slots,
                      const std::vector<int32_t>& out_slots) {
    const XjBasis& B = xj_basis();
    std::vector<uint8_t> cb(M.size());
    for (size_t e = 0; e < M.size(); ++e) cb[e] = B.bits(M[e]);
    const int roles = (R + kXjOutputsPerRole - 1) / kXjOutputsPerRole;
    std::ostringstream o;
    o << "typedef unsigned int uint32_t; typedef int int32_t; typedef unsigned char uint8_t;\n"
         "typedef long long int64_t; typedef unsigned long long uint64_t;\n"
         "struct XJArgs { const uint8_t* src; int64_t src_stripe; uint8_t* dst; int64_t dst_stripe;"
         " int32_t src_sym, dst_sym; };\n"
      << "// K=" << K << " R=" << R << " roles=" << roles << "\n"
      << "extern \"C\" __global__ void __launch_bounds__(" << 64 * roles << ") rs_xj(XJArgs a) {\n"
      << "  asm volatile(\n" << as_string_literals(finish_block()) << "  ::: \"memory\");\n"
      << "  const uint64_t stripe = blockIdx.y;\n"
         "  const uint64_t sb = (uint64_t)a.src + stripe * (uint64_t)a.src_stripe;\n"
         "  const uint64_t db = (uint64_t)a.dst + stripe * (uint64_t)a.dst_stripe;\n"
         "  const uint32_t col = blockIdx.x * 256u + (threadIdx.x & 63u) * 4u;\n"
         "  const uint32_t sl = (uint32_t)sb, sh = (uint32_t)(sb >> 32), dl = (uint32_t)db, dh = (uint32_t)(db >> 32);\n"
         "  const int role = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));\n"
         "  switch (role) {\n";
    std::string clob;
    for (int v = 8; v <= 119; ++v) clob += "\"v" + std::to_string(v) + "\", ";
    for (int s = 32; s <= 71; ++s) clob += "\"s" + std::to_string(s) + "\", ";
    clob += "\"scc\", \"memory\"";
    for (int w = 0; w < roles; ++w) {
        o << "  case " << w << ": asm volatile(\n"
          << as_string_literals(role_block(w, cb, K, R, in_slots, out_slots))
          << "  : : [col] \"v\"(col), [sl] \"s\"(sl), [sh] \"s\"(sh), [dl] \"s\"(dl), [dh] \"s\"(dh),"
             " [ss] \"s\"(a.src_sym), [ds] \"s\"(a.dst_sym)\n  : "
          << clob << ");\n    break;\n";
    }
    o << "  }\n}\n";
    return o.str();
}

int xj_precompile(const std::vector<uint16_t>& M, int K, int R, const std::vector<int32_t>& in_slots,
                  const std::vector<int32_t>& out_slots) {
    if (!xj_supported(8, K, R)) return 0;
    const std::string src = xj_source(M, K, R, in_slots, out_slots);
    std::vector<char> code;
    return jit_code(src, "xj", jit_hash(src), code) ? 3 : 0;
}

int xj_build(const std::vector<uint16_t>& M, int K, int R, const std::vector<int32_t>& in_slots,
             const std::vector<int32_t>& out_slots, std::unique_ptr<XjKernel>& out) {
    out.reset();
    if (!xj_supported(8, K, R)) return 0;
    const std::string src = xj_source(M, K, R, in_slots, out_slots);
    uint64_t h = 0;
    std::shared_ptr<JitModule> mod;
    if (jit_module(src, "xj", mod, &h)) return 3;
    auto k = std::make_unique<XjKernel>();
    k->mod = mod;
    (void)hipGetDevice(&k->device);
    k->roles = (R + kXjOutputsPerRole - 1) / kXjOutputsPerRole;
    if (hipModuleGetFunction(&k->fn, jit_module_handle(*mod), "rs_xj") != hipSuccess) return 3;
    char nm[64];
    std::snprintf(nm, sizeof nm, "rs_xj[%dx%d:%08llx]", R, K, static_cast<unsigned long long>(h & 0xffffffff));
    k->name = nm;
    out = std::move(k);
    return 0;
}

int xj_launch(const XjKernel& k, const XJArgs& a0, int64_t n_stripes, int64_t nchunks, hipStream_t st) {
    if (n_stripes <= 0 || nchunks <= 0) return 0;
    for (int64_t s0 = 0; s0 < n_stripes; s0 += 65535) {  // grid.y limit
        XJArgs a = a0;
        a.src += s0 * a.src_stripe;
        a.dst += s0 * a.dst_stripe;
        const unsigned ny = unsigned(std::min<int64_t>(65535, n_stripes - s0));
        void* args[] = {&a};
        hipError_t e = hipModuleLaunchKernel(k.fn, unsigned(nchunks), ny, 1, unsigned(64 * k.roles), 1, 1, 0, st, args,
                                             nullptr);
        if (e != hipSuccess) {
            std::fprintf(stderr, "librs_amd: xj launch: %s\n", hipGetErrorString(e));
            return 3;
        }
    }
    return 0;
}

}  // namespace rsamd
