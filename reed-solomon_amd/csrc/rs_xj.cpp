// rs_xj.cpp -- generator, cache and launcher of the bit-plane XOR kernels (see rs_xj.hpp).
//
// Generated kernel `rs_xj_<source hash>` (one per coding matrix and slot lists):
//   grid (column chunks of 256 B, stripes), block = 64 x roles threads. All waves of a block work on
//   the same 256-byte column of one stripe; wave w ("role") owns outputs opr*w .. opr*w + opr - 1
//   (opr = min(16, R) outputs per role by default, XjConfig).
//   Register contract of a role (XjConfig's map; fixed, so the generated code names registers directly):
//     v[1 : 8 opr]              accumulators u_{q,t} of output q, bit-plane t: v[1 + 8q + t]
//     ring_base = 1 + 8 opr     input ring: `ring` slots x 8 inputs (one group pair = 8 consecutive inputs)
//     tab(h) = ring_base + 8 ring + 11 h    the 11 non-trivial subset XORs of group h (inputs 4h..4h+3)
//     after the XOR network: fin(q) = ring_base + q holds output q; tmp(q, k) Horner temporaries
//     s[32:38]  src base, src symbol stride, dst base, dst symbol stride; s[40:55] address pairs /
//               buffer offsets + V#s; s[56:59] call / return address of the shared finish block;
//               s62 scratch, s63 saved m0; the column offset is the compiler's %[col] VGPR
//   The finish block (Horner in alpha^-1 over the 16 z-coordinates, chains interleaved 8 at a time) is
//   emitted once at the kernel entry and entered by s_swappc_b64 from every role.
//   Loads (early issue, the default): pairs 0 and 1 go out first; inside pair g, the rows that read one of
//   the pair's raw inputs run first, then pair g+2's loads go into the freed ring slot, then the rows that
//   read only built table entries -- so every wait is for loads issued about 1.5 pairs earlier.
//   Experimental forms (knobs in XjConfig, measured in DESIGN.md section 5): LDS-DMA input ring,
//   buffer addressing, spread loads, Horner in alpha, LDS-table finish (persistent grid), LDS table
//   sharing between roles.
#include "rs_xj.hpp"
#include <cstring>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <sstream>

#include "gf16.hpp"
#include "rs_jit.hpp"

namespace rsamd {

// ------------------------------------------------------------------------------- host math
static int parity16(uint32_t v) { return __builtin_popcount(v & 0xFFFFu) & 1; }

// finish instructions per output for basis coordinates `B` (see finish_block)
static int finish_cost(const uint16_t* B, int horner) {
    int w[16] = {0};
    for (int j = 0; j < 16; ++j)
        for (int t = 0; t < 8; ++t) w[j] += (B[t] >> j) & 1;
    int jtop = 15;
    while (jtop > 0 && !w[jtop]) --jtop;
    int c = w[jtop] > 1 ? w[jtop] / 2 : 0;
    for (int j = jtop - 1; j >= 0; --j) c += horner ? 3 + (w[j] + 1) / 2 : 4 + (w[j] ? 1 + w[j] / 2 : 1);
    return c;
}

XjBasis::XjBasis(int horner_) : horner(horner_) {
    const Field& F = field();
    // A: column j = z^j (16-bit); invert over GF(2) by Gauss-Jordan on rows.
    uint32_t row[16];  // row i: bits j = bit i of z^j ; augmented identity in bits 16..31
    for (int i = 0; i < 16; ++i) {
        uint32_t r = 0;
        for (int j = 0; j < 16; ++j) {
            const uint16_t zj = F.exp[horner ? uint32_t(j) : (kN - uint32_t(j)) % kN];
            if ((zj >> i) & 1) r |= 1u << j;
        }
        row[i] = r | (1u << (16 + i));
    }
    for (int c = 0; c < 16; ++c) {
        int p = c;
        while (!((row[p] >> c) & 1)) ++p;  // the z^j are independent
        std::swap(row[p], row[c]);
        for (int i = 0; i < 16; ++i)
            if (i != c && ((row[i] >> c) & 1)) row[i] ^= row[c];
    }
    for (int j = 0; j < 16; ++j) inv_row_[j] = uint16_t(row[j] >> 16);
    // GF(256) = span of gamma^t (gamma = alpha^257) in z-coordinates; for every pivot set whose 8 x 8
    // minor is invertible, the reduced basis is unique -- keep the cheapest finish
    uint16_t G[8];
    for (int t = 0; t < 8; ++t) G[t] = ycoord(F.exp[(257u * t) % kN]);
    int best = 1 << 30;
    for (uint32_t set = 0; set < (1u << 16); ++set) {
        if (__builtin_popcount(set) != 8) continue;
        int pv[8], n = 0;
        for (int j = 0; j < 16; ++j)
            if ((set >> j) & 1) pv[n++] = j;
        // solve: rows of G restricted to pv -> invert the 8 x 8 minor
        uint16_t aug[8];
        for (int t = 0; t < 8; ++t) {
            uint8_t m = 0;
            for (int s2 = 0; s2 < 8; ++s2) m |= uint8_t(((G[t] >> pv[s2]) & 1) << s2);
            aug[t] = uint16_t(m | (1u << (8 + t)));
        }
        bool ok = true;
        for (int c = 0; c < 8 && ok; ++c) {
            int p = c;
            while (p < 8 && !((aug[p] >> c) & 1)) ++p;
            if (p == 8) {
                ok = false;
                break;
            }
            std::swap(aug[p], aug[c]);
            for (int i = 0; i < 8; ++i)
                if (i != c && ((aug[i] >> c) & 1)) aug[i] ^= aug[c];
        }
        if (!ok) continue;
        uint16_t B[8];
        for (int t = 0; t < 8; ++t) {  // basis vector with unit coordinate at pv[t]
            uint16_t v = 0;
            for (int i = 0; i < 8; ++i)
                if ((aug[t] >> (8 + i)) & 1) v ^= G[i];
            B[t] = v;
        }
        const int c = finish_cost(B, horner);
        if (c < best) {
            best = c;
            for (int t = 0; t < 8; ++t) pivots[t] = pv[t], beta_y[t] = B[t];
        }
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

const XjBasis& xj_basis(int horner) {
    static const XjBasis* b[2] = {new XjBasis(0), new XjBasis(1)};
    return *b[horner ? 1 : 0];
}

bool xj_supported(int m, int K, int R) {
    return m <= 8 && K >= 1 && R >= 1 && xj_roles(R) <= xj_max_roles(R) && K * R <= kXjMaxWork;
}

// --------------------------------------------------------------------------- code generator
namespace {

// Generation knobs (defaults = measured best; RS_XJ_* environment variables override them for
// experiments -- they change the source text, hence the cache key).
struct XjConfig {
    int opr = 16;      // outputs per role (wave): 8 -> 64 accumulators (4 waves/SIMD), 16 -> 128 (3 waves/SIMD)
    int ring = 2;      // input ring slots (group pairs in flight = ring - 1)
    int buffer = 0;    // 1: buffer_load/store with a V# and one SALU offset per input; 0: global + SGPR pair
    int spread = 0;    // 1: next pairs' loads interleaved into the row stream; 0: issued as a burst
    int horner = 0;    // finish: 1 = Horner in alpha (packed-16 ops), 0 = in alpha^-1
    int ablate = 0;    // timing ablations (wrong results): 1 no finish, 2 no rows, 4 no tables
    int nt = 0;        // cache policy bits on the global loads / stores: 1 = nt loads, 2 = nt stores, 3 = both
    int lds = 0;       // > 0: per-wave LDS-DMA prefetch ring of `lds` group pairs (2 KiB each); 0: direct loads
    int share = 0;     // 1 (two roles): each role builds one group's subset tables, exchanged via LDS
    int kreg = 1;      // finish step constants: 1 = in VGPRs (4-byte VOP2 forms), 0 = literals
    int lfin = 0;      // finish: 0 = VALU Horner over z (above); 1 = Horner in gamma through a 128 KiB LDS
                       // table T[w] = gamma * w (persistent kernel, one workgroup per CU)
    int xcd = 0;       // 1: workgroup -> column remap so each XCD walks contiguous 1/8 spans of every stripe
                       // (dispatch puts workgroup i on XCD i % 8); 0: consecutive columns round-robin
    int cpb = 1;       // columns per block: > 1 loops each role over cpb consecutive 256-byte columns of a
                       // stripe; the next column's first input pair is loaded during the current column's
                       // last pair and finish (its ring slot stays clear of the finish registers), so only
                       // the block's first column waits for a cold load. Needs an even pair count (set_k).
    int cpb_sync = 1;  // column loop: s_barrier per column
    int endwait = 0;   // 1: wait for the stores between the two store batches and at the end of the role
    int splitwait = 0; // 1: wait for a pair's first group of four inputs, build its tables, then wait for the rest
    int inlinefin = 0; // 1: each role carries its own copy of the finish (no s_swappc / s_setpc per column)
    int prio = 0;      // 1: s_setprio 1 over the XOR network, 0 over the finish; 2: 2 over the finish only;
                       // 3: 1 over each early load burst
    int early = 1;     // 1 (ring 2): pair g+2's loads go out inside pair g, right after its last row that reads
                       // one of the pair's raw inputs (those rows first), so a load has ~1.5 pairs to land
    int masked = 0;    // 1 (set_masked; the per-stripe fixed pass of rsg_decode_batch): every input slot whose
                       // bit is set in the launch-local stripe's mask words reads a zero buffer instead
                       // (s_bitcmp1 + s_cselect_b64 on the load's base pair): erased slots count as zero
    int coord = 0;     // 1 (set_masked(2)): the outputs are stored in GF(256)^2 coordinates (the L byte tables of
                       // XJArgs::tab in LDS, four reads per output), the form the per-stripe solve consumes
    // env: read the RS_XJ_* generation knobs (experiments, the emulator tests through rsg_xj_source, the
    // diagnostic build). The kernels the release library launches are generated with the defaults
    // whatever the environment says, so no deployment's environment changes the shipped kernel.
    explicit XjConfig(int R = 0, bool env_knobs = false) {
#ifdef RS_AMD_DIAG
        env_knobs = true;
#endif
        auto env = [env_knobs](const char* n, int& v) {
            if (!env_knobs) return;
            if (const char* e = std::getenv(n)) v = std::atoi(e);
        };
        env("RS_XJ_OPR", opr);
        env("RS_XJ_RING", ring);
        env("RS_XJ_BUFFER", buffer);
        env("RS_XJ_SPREAD", spread);
        env("RS_XJ_HORNER", horner);
#ifdef RS_AMD_DIAG  // timing ablations produce wrong results: diagnostic build only
        env("RS_XJ_ABLATE", ablate);
#endif
        env("RS_XJ_LDS", lds);
        env("RS_XJ_NT", nt);
        env("RS_XJ_FIN", lfin);
        env("RS_XJ_SHARE", share);
        env("RS_XJ_KREG", kreg);
        env("RS_XJ_XCD", xcd);
        env("RS_XJ_CPB", cpb);
        env("RS_XJ_CPB_SYNC", cpb_sync);
        env("RS_XJ_EARLY", early);
        env("RS_XJ_ENDWAIT", endwait);
        env("RS_XJ_SPLITWAIT", splitwait);
        env("RS_XJ_INLINEFIN", inlinefin);
        env("RS_XJ_PRIO", prio);

        lfin = lfin ? 1 : 0;
        if (lfin) lds = 0;  // the table takes the LDS
        lds = lds ? std::max(2, std::min(8, lds)) : 0;
        if (lds) ring = 2;  // VGPR double buffer behind the LDS ring
        opr = std::max(1, std::min(16, opr));
        if (R > 0) opr = std::min(opr, R);  // small codes: smaller register layout, more waves per SIMD
        share = (share && !lds && !lfin && R > 0 && (R + opr - 1) / opr == 2) ? 1 : 0;
        ring = std::max(2, std::min(6, ring));
        horner = horner ? 1 : 0;
        cpb = std::max(1, std::min(64, cpb));
        if (lfin || lds || share || spread || xcd || buffer || ring != 2) cpb = 1;
        early = (early && !lds && !share && !spread && ring == 2 && cpb == 1) ? std::min(2, std::max(1, early)) : 0;
        splitwait = (splitwait && !lds && !share && cpb == 1) ? 1 : 0;
        inlinefin = (inlinefin && !lfin && cpb == 1) ? 1 : 0;
    }
    // masked loads exist for the default layout only (global loads with an SGPR base pair per input, one
    // column per block, plain block order)
    void set_masked(int mode = 1) {
        masked = 1;
        coord = mode == 2 ? 1 : 0;
        buffer = lds = lfin = share = xcd = spread = 0;
        cpb = 1;
        ring = 2;
    }
    // the column loop needs the last pair in ring slot 1, so the next column's pair 0 has slot 0 to itself
    void set_k(int K) {
        if (((K + 7) / 8) % 2) cpb = 1;
    }
    // register map (the column offset is the compiler's %[col] operand register, outside this range)
    int acc(int q, int t) const { return 1 + 8 * q + t; }
    int ring_base() const { return 1 + 8 * opr; }
    int tab(int h) const { return ring_base() + 8 * ring + 11 * h; }
    int max_vgpr() const { return tab(2) - 1; }
    // after the XOR network: result of output q, and per-chain temporaries (chains run in batches of 8).
    // Column loop (cpb > 1): results and temporaries above ring slot 0 (slot 1 + the tables), one batch of
    // 8 results at a time, each batch stored before the next is computed.
    int fin(int q) const { return cpb > 1 ? ring_base() + 8 + q % 8 : ring_base() + q; }
    int tmp(int q, int k) const { return (cpb > 1 ? ring_base() + 16 : ring_base() + opr) + 2 * (q % 8) + k; }
    int cst() const { return cpb > 1 ? ring_base() + 32 : ring_base() + opr + 16; }  // cst + 2 <= max_vgpr
    std::string tag() const {
        char b[128];
        std::snprintf(b, sizeof b, "opr%d ring%d buf%d spread%d horner%d ablate%d lds%d nt%d fin%d share%d kreg%d",
                      opr, ring, buffer, spread, horner, ablate, lds, nt, lfin, share, kreg);
        std::string s = xcd ? std::string(b) + " xcd" + std::to_string(xcd) : std::string(b);
        if (early) s += early == 2 ? " early2" : " early";
        if (!endwait) s += " noendwait";
        if (splitwait) s += " splitwait";
        if (inlinefin) s += " inlinefin";
        if (prio) s += " prio";
        if (masked) s += coord ? " masked coord" : " masked";
        return cpb > 1 ? s + " cpb" + std::to_string(cpb) + (cpb_sync ? " sync" : "") : s;
    }
};

// built-entry register index of subset pattern e (popcount >= 2) within a group's 11 registers
int built_index(int e) {
    static const int idx[16] = {-1, -1, -1, 0, -1, 1, 2, 3, -1, 4, 5, 6, 7, 8, 9, 10};
    return idx[e];
}

struct Emitter {
    std::vector<std::string> L;
    void e(const std::string& s) { L.push_back(s); }
    template <class... A>
    std::string fmt(const char* f, A... a) {
        char buf[160];
        std::snprintf(buf, sizeof buf, f, a...);
        return buf;
    }
    template <class... A>
    void f(const char* f, A... a) {
        L.push_back(fmt(f, a...));
    }
};

std::string as_string_literals(const std::vector<std::string>& L) {
    std::string o;
    for (const std::string& s : L) o += "\"" + s + "\\n\"\n";
    return o;
}

// The finish block: for every output q, H_q = sum_j z^j v_j with v_j = XOR of u_{q,t} over the t whose
// beta_t has z-coordinate j; Horner from the top coordinate down, up to 8 chains interleaved.
//   z = alpha:    H <- (H + H per 16-bit lane) ^ (sign mask per lane & 0x2D), then ^ v_j
//   z = alpha^-1: H <- ((H & 0xfffeffff) >> 1) ^ ((H & 0x10001) * 0x8016) ^ v_j
std::vector<std::string> finish_block_lds(const XjConfig& C);

std::vector<std::string> finish_block(const XjConfig& C) {
    if (C.lfin) return finish_block_lds(C);
    const XjBasis& B = xj_basis(C.horner);
    std::vector<std::string> L;
    L.push_back("s_branch L_xj_fin_end");
    auto consts = [&]() {
        if (C.horner) {
            L.push_back("v_mov_b32 v" + std::to_string(C.cst()) + ", 0x2d002d");
        } else if (C.kreg) {  // step constants in VGPRs: 4-byte VOP2 forms issue faster than literal ones (bank_bench)
            L.push_back("v_mov_b32 v" + std::to_string(C.cst()) + ", 0xfffeffff");
            L.push_back("v_mov_b32 v" + std::to_string(C.cst() + 1) + ", 0x10001");
            L.push_back("v_mov_b32 v" + std::to_string(C.cst() + 2) + ", 0x8016");
        }
    };
    if (C.cpb == 1) {
        L.push_back("L_xj_fin:");
        consts();
    }
    for (int q0 = 0; q0 < C.opr; q0 += 8) {
        if (C.cpb > 1) {  // column loop: one entry per batch of 8 outputs (L_xj_fin0, L_xj_fin1)
            L.push_back("L_xj_fin" + std::to_string(q0 / 8) + ":");
            consts();
        }
        const int nc = std::min(8, C.opr - q0);
        std::vector<std::vector<std::string>> chains(static_cast<size_t>(nc));
        for (int c = 0; c < nc; ++c) {
            const int q = q0 + c;
            std::vector<std::string>& out = chains[size_t(c)];
            char buf[160];
            auto add = [&](const char* fmt, auto... a) {
                std::snprintf(buf, sizeof buf, fmt, a...);
                out.emplace_back(buf);
            };
            const int H = C.fin(q), T1 = C.tmp(q, 0), T2 = C.tmp(q, 1);
            auto terms = [&](int j) {
                std::vector<int> r;
                for (int t = 0; t < 8; ++t)
                    if ((B.beta_y[t] >> j) & 1) r.push_back(C.acc(q, t));
                return r;
            };
            auto fold = [&](int dst, const std::vector<int>& v, size_t from) {  // v[from..] into dst
                size_t i = from;
                for (; i + 1 < v.size(); i += 2)
                    add("v_bitop3_b32 v%d, v%d, v%d, v%d bitop3:0x96", dst, dst, v[i], v[i + 1]);
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
                std::vector<int> v = terms(j);
                if (C.horner) {
                    add("v_pk_add_u16 v%d, v%d, v%d", T1, cur, cur);
                    add("v_pk_ashrrev_i16 v%d, 15, v%d op_sel_hi:[0,1]", T2, cur);
                    add("v_bitop3_b32 v%d, v%d, v%d, v%d bitop3:0x78", H, T1, T2, C.cst());  // T1 ^ (T2 & C)
                    fold(H, v, 0);
                } else {
                    if (C.kreg) {
                        add("v_and_b32 v%d, v%d, v%d", T1, C.cst(), cur);
                        add("v_lshrrev_b32 v%d, 1, v%d", T1, T1);
                        add("v_and_b32 v%d, v%d, v%d", T2, C.cst() + 1, cur);
                        add("v_mul_u32_u24 v%d, v%d, v%d", T2, C.cst() + 2, T2);
                    } else {
                        add("v_and_b32 v%d, 0xfffeffff, v%d", T1, cur);
                        add("v_lshrrev_b32 v%d, 1, v%d", T1, T1);
                        add("v_and_b32 v%d, 0x10001, v%d", T2, cur);
                        add("v_mul_u32_u24 v%d, 0x8016, v%d", T2, T2);
                    }
                    if (v.empty()) {
                        add("v_xor_b32 v%d, v%d, v%d", H, T1, T2);
                    } else {
                        add("v_bitop3_b32 v%d, v%d, v%d, v%d bitop3:0x96", H, T1, T2, v[0]);
                        fold(H, v, 1);
                    }
                }
                cur = H;
            }
            if (cur != H) add("v_mov_b32 v%d, v%d", H, cur);
        }
        const size_t n = chains[0].size();
        for (size_t i = 0; i < n; ++i)
            for (int c = 0; c < nc; ++c) L.push_back(chains[size_t(c)][i]);
        if (C.cpb > 1) L.push_back("s_setpc_b64 s[58:59]");
    }
    if (C.cpb == 1) L.push_back("s_setpc_b64 s[58:59]");
    L.push_back("L_xj_fin_end:");
    return L;
}

// LDS finish (fin = 1): bit-planes over the gamma power basis (beta_t = gamma^t), so
//   out = u_0 + gamma (u_1 + gamma (u_2 + ... + gamma u_7))
// and gamma * H on both 16-bit lanes of H is two LDS reads from T[w] = gamma * w at LDS address 0, each
// into its own address register: ds_read_u16 (zero-extended low lane) and ds_read_u16_d16_hi (high lane;
// on gfx950, an SRAM-ECC target, d16 loads zero the unused half, so two d16 loads into one register
// would clobber each other). 4 address ops + 2 LDS reads + 1 XOR3 per step, 7 steps per output. Chains run in two
// groups of 4 so that one group's reads (8 in flight) overlap the other group's address arithmetic.
std::vector<std::string> finish_block_lds(const XjConfig& C) {
    std::vector<std::string> L;
    char buf[160];
    auto add = [&](const char* fmt, auto... a) {
        std::snprintf(buf, sizeof buf, fmt, a...);
        L.emplace_back(buf);
    };
    L.push_back("s_branch L_xj_fin_end");
    L.push_back("L_xj_fin:");
    for (int q0 = 0; q0 < C.opr; q0 += 8) {
        const int nc = std::min(8, C.opr - q0);
        std::vector<int> grp[2];
        for (int c = 0; c < nc; ++c) grp[c < 4 ? 0 : 1].push_back(q0 + c);
        auto addr = [&](int g, int t) {  // addresses of gamma * (current H), H = u_7 before the first step
            for (int q : grp[g]) {
                const int cur = t == 6 ? C.acc(q, 7) : C.fin(q);
                add("v_add_u32 v%d, v%d, v%d", C.tmp(q, 0), cur, cur);
                add("v_lshrrev_b32 v%d, 15, v%d", C.tmp(q, 1), cur);
            }
            for (int q : grp[g]) {
                add("v_and_b32 v%d, 0x1fffe, v%d", C.tmp(q, 0), C.tmp(q, 0));
                add("v_and_b32 v%d, 0x1fffe, v%d", C.tmp(q, 1), C.tmp(q, 1));
            }
        };
        auto reads = [&](int g) {
            for (int q : grp[g]) {
                add("ds_read_u16 v%d, v%d", C.tmp(q, 0), C.tmp(q, 0));
                add("ds_read_u16_d16_hi v%d, v%d", C.tmp(q, 1), C.tmp(q, 1));
            }
        };
        auto xors = [&](int g, int t) {
            for (int q : grp[g])
                add("v_bitop3_b32 v%d, v%d, v%d, v%d bitop3:0x96", C.fin(q), C.tmp(q, 0), C.tmp(q, 1), C.acc(q, t));
        };
        const bool two = !grp[1].empty();
        addr(0, 6);
        reads(0);
        if (two) addr(1, 6);
        for (int t = 6; t >= 0; --t) {
            L.push_back("s_waitcnt lgkmcnt(0)");
            xors(0, t);
            if (two) reads(1);
            if (t > 0) addr(0, t - 1);
            if (two) {
                L.push_back("s_waitcnt lgkmcnt(0)");
                xors(1, t);
            }
            if (t > 0) {
                reads(0);
                if (two) addr(1, t - 1);
            }
        }
    }
    L.push_back("s_setpc_b64 s[58:59]");
    L.push_back("L_xj_fin_end:");
    return L;
}

// One role: outputs p = opr*w + q (q < nq) of the R x K bit-plane matrix `cb` (cb[p*K + i] = b(c_{p,i})).
// SGPRs: s[32:33] src base, s34 src stride, s[36:37] dst base, s38 dst stride, s[40:55] address pairs
// (global form) / s[40:47] offsets + s[48:51] src V# + s[52:55] dst V# (buffer form), s[56:59] call,
// s62 scratch.
std::vector<std::string> role_block(const XjConfig& C, int w, const std::vector<uint8_t>& cb, int K, int R,
                                    const std::vector<int32_t>& in_slots, const std::vector<int32_t>& out_slots) {
    Emitter E;
    const int p0 = C.opr * w, nq = std::min(C.opr, R - p0);
    const char* COL = "%[col]";
    E.e("s_nop 4");  // "s" operands may come from v_readfirstlane (VALU SGPR write -> VMEM read)
    E.e("s_mov_b32 s32, %[sl]");
    E.e("s_mov_b32 s33, %[sh]");
    E.e("s_mov_b32 s34, %[ss]");
    E.e("s_mov_b32 s36, %[dl]");
    E.e("s_mov_b32 s37, %[dh]");
    E.e("s_mov_b32 s38, %[ds]");
    if (C.buffer || C.lds) {  // raw buffer descriptors: base, stride 0, num_records 2^32 - 1, 32-bit data format
        E.e("s_mov_b32 s48, s32");
        E.e("s_and_b32 s49, s33, 0xffff");
        E.e("s_mov_b32 s50, -1");
        E.e("s_mov_b32 s51, 0x20000");
        E.e("s_mov_b32 s52, s36");
        E.e("s_and_b32 s53, s37, 0xffff");
        E.e("s_mov_b32 s54, -1");
        E.e("s_mov_b32 s55, 0x20000");
    }
    if (C.prio == 1) E.e("s_setprio 1");  // rows (which issue the loads) ahead of other waves' finishes
    const int ngp = (K + 7) / 8;
    // column loop: s39 = columns left; the block's columns are gridDim.x apart (s63 = that stride in bytes),
    // so the blocks in flight still read neighbouring columns together; s[60:61] = source base + stride
    const bool loop = C.cpb > 1;
    if (loop) {
        E.e("s_mov_b32 s39, %[nc]");
        E.e("s_mov_b32 s63, %[cs]");
        E.e("s_add_u32 s60, s32, s63");
        E.e("s_addc_u32 s61, s33, 0");
    }
    auto nload = [&](int g) { return g < ngp ? std::min(8, K - 8 * g) : 0; };
    // instruction lists of the loads of pair g (address arithmetic first, then the loads); `next_col`:
    // the same pair of the block's next column (base s[60:61])
    auto load_ops = [&](int g, bool next_col = false, int j0 = 0, int j1 = 8) {
        std::vector<std::string> ops;
        const int n = std::min(nload(g), j1);
        for (int j = j0; j < n; ++j) {
            const int dst = C.ring_base() + 8 * (g % C.ring) + j;
            const int slot = in_slots[size_t(8 * g + j)];
            if (C.buffer) {
                ops.push_back(E.fmt("s_mul_i32 s%d, s34, %d", 40 + j, slot));
                ops.push_back(E.fmt("buffer_load_dword v%d, %s, s[48:51], s%d offen", dst, COL, 40 + j));
            } else {
                ops.push_back(E.fmt("s_mul_i32 s62, s34, %d", slot));
                ops.push_back(E.fmt("s_add_u32 s%d, s%d, s62", 40 + 2 * j, next_col ? 60 : 32));
                ops.push_back(E.fmt("s_addc_u32 s%d, s%d, 0", 41 + 2 * j, next_col ? 61 : 33));
                if (C.masked) {  // an erased slot of this stripe reads the zero buffer
                    ops.push_back(E.fmt("s_bitcmp1_b32 %%[mw%d], %d", slot / 32, slot % 32));
                    ops.push_back(E.fmt("s_cselect_b64 s[%d:%d], %%[zb], s[%d:%d]", 40 + 2 * j, 41 + 2 * j, 40 + 2 * j,
                                        41 + 2 * j));
                }
                ops.push_back(E.fmt("global_load_dword v%d, %s, s[%d:%d]%s", dst, COL, 40 + 2 * j, 41 + 2 * j,
                                    (C.nt & 1) ? " nt" : ""));
            }
        }
        return ops;
    };
    bool init[16][8] = {};
    const int ahead = C.ring - 1;  // pairs in flight beyond the current one
    const int D = C.lds;
    // LDS-DMA ring: pair g lives in LDS slot g % D of this wave's region (s39 = region base); each lane's
    // dword of input j at slot * 2048 + j * 256 + 4 * lane (%[la] = region base + 4 * lane)
    auto dma_ops = [&](int g) {
        std::vector<std::string> ops;
        for (int j = 0; j < nload(g); ++j) {
            ops.push_back(E.fmt("s_mul_i32 s%d, s34, %d", 40 + j, in_slots[size_t(8 * g + j)]));
            ops.push_back(E.fmt("s_add_u32 m0, s39, %d", (g % D) * 2048 + j * 256));
            ops.push_back("s_nop 0");
            ops.push_back(E.fmt("buffer_load_dword %s, s[48:51], s%d offen lds", COL, 40 + j));
        }
        return ops;
    };
    auto ds_ops = [&](int g) {
        std::vector<std::string> ops;
        for (int j = 0; j < nload(g); ++j)
            ops.push_back(E.fmt("ds_read_b32 v%d, %%[la] offset:%d", C.ring_base() + 8 * (g % C.ring) + j,
                                (g % D) * 2048 + j * 256));
        return ops;
    };
    if (D) {
        E.e("s_mov_b32 s63, m0");
        E.e("s_mov_b32 s39, %[lb]");
        for (int g = 0; g < std::min(D, ngp); ++g)
            for (auto& op : dma_ops(g)) E.e(op);
        int pend = 0;
        for (int x = 1; x < std::min(D, ngp); ++x) pend += nload(x);
        E.f("s_waitcnt vmcnt(%d)", pend);
        for (auto& op : ds_ops(0)) E.e(op);
    } else {
        for (int g = 0; g < ahead + (C.early ? 1 : 0); ++g)
            for (auto& op : load_ops(g)) E.e(op);
    }
    if (loop) {  // the first column's pair 0 is the block's only cold wait
        E.e("s_waitcnt vmcnt(0)");
        E.f("L_xj_col%d:", w);
        if (C.cpb_sync) E.e("s_barrier");  // the roles of a column stay together (their loads share L1)
    }
    for (int g = 0; g < ngp; ++g) {
        std::vector<std::string> next, mid;
        std::string second_wait;  // splitwait: the wait for the pair's group-1 inputs
        if (D) {
            E.e("s_waitcnt lgkmcnt(0)");
            if (g + 1 < ngp) {  // pair g+1 has landed in LDS once only pairs g+2 .. g+D-1 are pending
                int pend = 0;
                for (int x = g + 2; x <= std::min(g + D - 1, ngp - 1); ++x) pend += nload(x);
                mid.push_back(E.fmt("s_waitcnt vmcnt(%d)", pend));
                for (auto& op : ds_ops(g + 1)) mid.push_back(op);
            }
            if (g + D < ngp)  // into the slot pair g has left (its ds_reads completed above)
                for (auto& op : dma_ops(g + D)) mid.push_back(op);
        } else {
            // loads issued so far beyond pair g: pairs g+1 .. g+ahead-1 (g+ahead is issued below); early:
            // pair g+1 was issued inside pair g-1, pair g+2 goes out inside this pair's rows
            int pending = 0;
            for (int x = g + 1; x < g + ahead + (C.early ? 1 : 0); ++x) pending += nload(x);
            if (!C.early) next = load_ops(g + ahead);
            if (!C.spread && !C.early) {
                for (auto& op : next) E.e(op);
                pending += nload(g + ahead);
            }
            // column loop: the previous column's stores were issued after this pair 0 and before the
            // loads above (vmcnt retires in issue order)
            if (loop && g == 0) pending += nq;
            if (C.splitwait && nload(g) > 4) {  // group 0's four inputs first; group 1's before its tables
                E.f("s_waitcnt vmcnt(%d)", pending + nload(g) - 4);
                second_wait = E.fmt("s_waitcnt vmcnt(%d)", pending);
            } else {
                E.f("s_waitcnt vmcnt(%d)", pending);
            }
            if (loop && g == ngp - 1) {  // the next column's pair 0 into ring slot 0 (free: pair ngp-2 is done)
                E.e("s_cmp_gt_u32 s39, 1");
                E.f("s_cbranch_scc0 L_xj_npf%d", w);
                for (auto& op : load_ops(0, true)) E.e(op);
                E.f("L_xj_npf%d:", w);
            }
        }
        // patterns of this role's rows over the pair's two groups
        int pat[16][8][2];
        bool need[2][16] = {};
        auto pattern = [&](int row, int t, int h) {
            int e = 0;
            for (int jj = 0; jj < 4; ++jj) {
                const int i = 8 * g + 4 * h + jj;
                if (i < K && ((cb[size_t(row) * K + i] >> t) & 1)) e |= 1 << jj;
            }
            return e;
        };
        for (int q = 0; q < nq; ++q)
            for (int t = 0; t < 8; ++t)
                for (int h = 0; h < 2; ++h) {
                    pat[q][t][h] = pattern(p0 + q, t, h);
                    need[h][pat[q][t][h]] = true;
                }
        if (C.share)  // both roles build / receive the entries either of them needs
            for (int row = 0; row < R; ++row)
                for (int t = 0; t < 8; ++t)
                    for (int h = 0; h < 2; ++h) need[h][pattern(row, t, h)] = true;
        auto single = [&](int h, int jj) { return C.ring_base() + 8 * (g % C.ring) + 4 * h + jj; };
        auto reg = [&](int h, int e) {
            if (__builtin_popcount(e) == 1) return single(h, __builtin_ctz(e));
            return C.tab(h) + built_index(e);
        };
        std::vector<std::string> body;
        for (int h = 0; h < 2; ++h) {
            if (h == 1 && !second_wait.empty()) body.push_back(second_wait);
            if (C.share && h != w) continue;  // the partner role builds the other group
            // popcount 2 and 3 straight from the inputs; 15 from a built triple or pair
            bool built[16] = {};
            for (int e = 3; e < 15; ++e) {
                if (!need[h][e] || __builtin_popcount(e) < 2) continue;
                int b[3], nb = 0;
                for (int jj = 0; jj < 4; ++jj)
                    if ((e >> jj) & 1) b[nb++] = single(h, jj);
                if (nb == 2)
                    body.push_back(E.fmt("v_xor_b32 v%d, v%d, v%d", reg(h, e), b[0], b[1]));
                else
                    body.push_back(E.fmt("v_bitop3_b32 v%d, v%d, v%d, v%d bitop3:0x96", reg(h, e), b[0], b[1], b[2]));
                built[e] = true;
            }
            if (need[h][15]) {
                int tri = -1, pair = -1;
                for (int e : {7, 11, 13, 14})
                    if (built[e]) tri = e;
                for (int e : {3, 5, 6, 9, 10, 12})
                    if (built[e]) pair = e;
                if (tri >= 0) {
                    body.push_back(E.fmt("v_xor_b32 v%d, v%d, v%d", reg(h, 15), reg(h, tri),
                                         single(h, __builtin_ctz(15 & ~tri))));
                } else {
                    if (pair < 0) {
                        pair = 3;
                        body.push_back(E.fmt("v_xor_b32 v%d, v%d, v%d", reg(h, 3), single(h, 0), single(h, 1)));
                    }
                    const int rest = 15 & ~pair;
                    body.push_back(E.fmt("v_bitop3_b32 v%d, v%d, v%d, v%d bitop3:0x96", reg(h, 15), reg(h, pair),
                                         single(h, __builtin_ctz(rest)), single(h, 31 - __builtin_clz(rest))));
                }
            }
        }
        if (C.share) {
            // exchange through LDS slot (g % 2, group, entry) x 64 lanes: write own group's entries,
            // barrier (the block is the two roles), read the partner's group
            auto off = [&](int h, int e) { return (((g % 2) * 2 + h) * 16 + e) * 256; };
            for (int e = 3; e < 16; ++e)
                if (need[w][e] && __builtin_popcount(e) >= 2)
                    body.push_back(E.fmt("ds_write_b32 %%[la], v%d offset:%d", reg(w, e), off(w, e)));
            body.push_back("s_waitcnt lgkmcnt(0)");
            body.push_back("s_barrier");
            for (int e = 3; e < 16; ++e)
                if (need[1 - w][e] && __builtin_popcount(e) >= 2)
                    body.push_back(E.fmt("ds_read_b32 v%d, %%[la] offset:%d", reg(1 - w, e), off(1 - w, e)));
            body.push_back("s_waitcnt lgkmcnt(0)");
        }
        if (C.ablate & 4) body.clear();
        for (auto& op : mid) body.push_back(op);  // LDS ring: next pair's reads + refills after the tables
        const size_t nbuild = body.size();
        // early: rows that read only built entries go after the next loads; early 2: the rows reading a
        // raw input of group 1 (and none of group 0) go between group 0's and group 1's loads
        std::vector<std::string> rest, raw1;
        for (int t = 0; t < 8; ++t)
            for (int q = 0; q < nq; ++q) {
                const int a = pat[q][t][0], b = pat[q][t][1], acc = C.acc(q, t);
                if ((!a && !b) || (C.ablate & 2)) continue;
                const bool r0 = __builtin_popcount(a) == 1, r1 = __builtin_popcount(b) == 1;
                std::vector<std::string>& dst =
                    !C.early ? body : r0 ? body : r1 ? (C.early == 2 ? raw1 : body) : rest;
                if (!init[q][t]) {
                    if (a && b)
                        dst.push_back(E.fmt("v_xor_b32 v%d, v%d, v%d", acc, reg(0, a), reg(1, b)));
                    else
                        dst.push_back(E.fmt("v_mov_b32 v%d, v%d", acc, a ? reg(0, a) : reg(1, b)));
                    init[q][t] = true;
                } else if (a && b) {
                    dst.push_back(E.fmt("v_bitop3_b32 v%d, v%d, v%d, v%d bitop3:0x96", acc, acc, reg(0, a), reg(1, b)));
                } else {
                    dst.push_back(E.fmt("v_xor_b32 v%d, v%d, v%d", acc, a ? reg(0, a) : reg(1, b), acc));
                }
            }
        if (C.early) {  // this pair's raw inputs are dead now: pair g+2 into their ring slot, then the rest
            const bool pr = C.prio == 3 && nload(g + 2) > 0;  // prio 3: the load burst ahead of other waves
            if (pr) body.push_back("s_setprio 1");
            for (auto& op : load_ops(g + 2, false, 0, C.early == 2 ? 4 : 8)) body.push_back(op);
            if (pr) body.push_back("s_setprio 0");
            for (auto& op : raw1) body.push_back(op);
            if (C.early == 2)
                for (auto& op : load_ops(g + 2, false, 4, 8)) body.push_back(op);
            for (auto& op : rest) body.push_back(op);
        }
        if (C.spread && !next.empty()) {
            // the next pair's loads go into this pair's row stream (after the table build: their ring
            // slot was last read by the previous pair), one every few rows
            std::vector<std::string> merged(body.begin(), body.begin() + long(nbuild));
            const size_t rows = body.size() - nbuild, nn = next.size();
            size_t k = 0;
            for (size_t i = 0; i < rows; ++i) {
                merged.push_back(body[nbuild + i]);
                while (k < nn && k * rows < (i + 1) * nn) merged.push_back(next[k++]);
            }
            while (k < nn) merged.push_back(next[k++]);
            body.swap(merged);
        }
        for (auto& op : body) E.e(op);
    }
    for (int q = 0; q < nq; ++q)
        for (int t = 0; t < 8; ++t)
            if (!init[q][t]) E.f("v_mov_b32 v%d, 0", C.acc(q, t));
    if (loop) {  // per batch of 8 outputs: its finish entry, then its stores (no wait: operands are read at issue)
        for (int q0 = 0; q0 < nq; q0 += 8) {
            const int nb = std::min(8, nq - q0);
            if (!(C.ablate & 1)) {
                E.e("s_getpc_b64 s[56:57]");
                E.f("s_add_u32 s56, s56, L_xj_fin%d-.", q0 / 8);
                E.e("s_addc_u32 s57, s57, -1");
                E.e("s_swappc_b64 s[58:59], s[56:57]");
            } else {
                for (int j = 0; j < nb; ++j) E.f("v_mov_b32 v%d, v%d", C.fin(q0 + j), C.acc(q0 + j, 0));
            }
            for (int j = 0; j < nb; ++j) {
                E.f("s_mul_i32 s62, s38, %d", out_slots[size_t(p0 + q0 + j)]);
                E.f("s_add_u32 s%d, s36, s62", 40 + 2 * j);
                E.f("s_addc_u32 s%d, s37, 0", 41 + 2 * j);
            }
            for (int j = 0; j < nb; ++j)
                E.f("global_store_dword %s, v%d, s[%d:%d]%s", COL, C.fin(q0 + j), 40 + 2 * j, 41 + 2 * j,
                    (C.nt & 2) ? " nt" : "");
        }
        E.f("v_add_u32 %s, s63, %s", COL, COL);
        E.e("s_sub_u32 s39, s39, 1");
        E.e("s_cmp_lg_u32 s39, 0");
        E.f("s_cbranch_scc1 L_xj_col%d", w);
        E.e("s_waitcnt vmcnt(0)");
        return E.L;
    }
    // prio 1: the finish issues no loads, the other waves' rows go first; prio 2: the finish first
    if (C.prio == 1 || C.prio == 2) E.e(C.prio == 1 ? "s_setprio 0" : "s_setprio 2");
    // finish (shared block; returns through s[58:59]); L_xj_fin precedes every role block
    if (!(C.ablate & 1) && C.inlinefin) {  // the block's body in place: no call / return
        std::vector<std::string> fb = finish_block(C);
        for (size_t i = 2; i + 2 < fb.size(); ++i) E.e(fb[i]);  // minus branch + label, return + end label
    } else if (!(C.ablate & 1)) {
        E.e("s_getpc_b64 s[56:57]");
        E.e("s_add_u32 s56, s56, L_xj_fin-.");
        E.e("s_addc_u32 s57, s57, -1");
        E.e("s_swappc_b64 s[58:59], s[56:57]");
    } else {  // keep the network live: store accumulator 0 of each output
        for (int q = 0; q < nq; ++q) E.f("v_mov_b32 v%d, v%d", C.fin(q), C.acc(q, 0));
    }
    if (C.coord) {
        // outputs into GF(256)^2 coordinates: y = L0[b0] ^ L1[b1] ^ L2[b2] ^ L3[b3] over the bytes of each result
        // (table k at LDS byte 1024 k, entry b at 4 b; the kernel's only LDS array, at 0), two outputs per round
        // of 8 reads; the accumulators are dead after the finish and serve as address / read registers
        for (int q0 = 0; q0 < nq; q0 += 2) {
            const int nb = std::min(2, nq - q0);
            for (int j = 0; j < nb; ++j) {
                const int f = C.fin(q0 + j), t = C.acc(0, 0) + 4 * j;
                E.f("v_lshlrev_b32 v%d, 2, v%d", t, f);
                E.f("v_and_b32 v%d, 0x3fc, v%d", t, t);
                for (int k = 1; k < 4; ++k) {
                    E.f("v_lshrrev_b32 v%d, %d, v%d", t + k, 8 * k - 2, f);
                    E.f("v_and_b32 v%d, 0x3fc, v%d", t + k, t + k);
                }
                E.f("ds_read_b32 v%d, v%d", t, t);
                for (int k = 1; k < 4; ++k) E.f("ds_read_b32 v%d, v%d offset:%d", t + k, t + k, 1024 * k);
            }
            E.e("s_waitcnt lgkmcnt(0)");
            for (int j = 0; j < nb; ++j) {
                const int f = C.fin(q0 + j), t = C.acc(0, 0) + 4 * j;
                E.f("v_xor_b32 v%d, v%d, v%d", f, t, t + 1);
                E.f("v_bitop3_b32 v%d, v%d, v%d, v%d bitop3:0x96", f, f, t + 2, t + 3);
            }
        }
    }
    for (int q0 = 0; q0 < nq; q0 += 8) {  // stores in batches of 8 address registers
        const int nb = std::min(8, nq - q0);
        for (int j = 0; j < nb; ++j) {
            const int slot = out_slots[size_t(p0 + q0 + j)];
            if (C.buffer) {
                E.f("s_mul_i32 s%d, s38, %d", 40 + j, slot);
            } else {
                E.f("s_mul_i32 s62, s38, %d", slot);
                E.f("s_add_u32 s%d, s36, s62", 40 + 2 * j);
                E.f("s_addc_u32 s%d, s37, 0", 41 + 2 * j);
            }
        }
        for (int j = 0; j < nb; ++j) {
            if (C.buffer)
                E.f("buffer_store_dword v%d, %s, s[52:55], s%d offen", C.fin(q0 + j), COL, 40 + j);
            else
                E.f("global_store_dword %s, v%d, s[%d:%d]%s", COL, C.fin(q0 + j), 40 + 2 * j, 41 + 2 * j,
                    (C.nt & 2) ? " nt" : "");
        }
        // endwait 0: no waits -- a store reads its address and data registers at issue, and the wave may
        // end with stores in flight
        if (q0 + 8 < nq && C.endwait) E.e("s_waitcnt vmcnt(0)");
    }
    if (C.endwait || D) E.e("s_waitcnt vmcnt(0)");
    if (D) E.e("s_mov_b32 m0, s63");
    return E.L;
}

}  // namespace

// Static instruction counts of one column (see XjKernel::valu_per_col): VALU = "v_" lines; SALU = "s_"
// lines other than program-flow / wait / message (SOPP) and scalar memory ops.
static void count_insts(const std::vector<std::string>& L, uint64_t mult, uint64_t* valu, uint64_t* salu) {
    static const char* kNotSalu[] = {"s_waitcnt", "s_nop", "s_barrier", "s_branch", "s_cbranch", "s_setprio",
                                     "s_sleep", "s_endpgm", "s_load", "s_buffer_load", "s_store", "s_dcache",
                                     "s_set_gpr_idx_on", "s_set_gpr_idx_off"};
    for (const std::string& ln : L) {
        size_t i = ln.find_first_not_of(" \t");
        if (i == std::string::npos) continue;
        if (ln.compare(i, 2, "v_") == 0) {
            *valu += mult;
        } else if (ln.compare(i, 2, "s_") == 0) {
            bool flow = false;
            for (const char* f : kNotSalu) flow = flow || ln.compare(i, std::strlen(f), f) == 0;
            if (!flow) *salu += mult;
        }
    }
}

static void xj_counts(const std::vector<uint16_t>& M, int K, int R, const std::vector<int32_t>& in_slots,
               const std::vector<int32_t>& out_slots, int masked, uint64_t* valu, uint64_t* salu) {
    XjConfig C(R);
    if (masked) C.set_masked(masked);
    C.set_k(K);
    const XjBasis& B = xj_basis(C.horner);
    std::vector<uint8_t> cb(M.size());
    for (size_t e = 0; e < M.size(); ++e) cb[e] = C.lfin ? gamma8().coord(M[e]) : B.bits(M[e]);
    const int roles = (R + C.opr - 1) / C.opr;
    *valu = *salu = 0;
    std::vector<std::string> fin = finish_block(C);
    if (!fin.empty()) fin.erase(fin.begin(), fin.begin() + 2);  // the branch around the block and its label
    for (int w = 0; w < roles; ++w) {
        count_insts(role_block(C, w, cb, K, R, in_slots, out_slots), 1, valu, salu);
        if (!(C.ablate & 1)) count_insts(fin, 1, valu, salu);
    }
}

std::string xj_source(const std::vector<uint16_t>& M, int K, int R, const std::vector<int32_t>& in_slots,
                      const std::vector<int32_t>& out_slots, bool env_knobs, int masked) {
    XjConfig C(R, env_knobs);
    if (masked) C.set_masked(masked);
    C.set_k(K);
    int nmw = 0;  // mask words the loads test (slot / 32 < nmw)
    for (int32_t v : in_slots) nmw = std::max(nmw, v / 32 + 1);
    const XjBasis& B = xj_basis(C.horner);
    std::vector<uint8_t> cb(M.size());
    for (size_t e = 0; e < M.size(); ++e) cb[e] = C.lfin ? gamma8().coord(M[e]) : B.bits(M[e]);
    const int roles = (R + C.opr - 1) / C.opr;
    const int pairs = C.lfin ? xj_pairs(R) : 1;
    std::ostringstream o;
    o << "typedef unsigned int uint32_t; typedef int int32_t; typedef unsigned char uint8_t;\n"
         "typedef unsigned short uint16_t; typedef long long int64_t; typedef unsigned long long uint64_t;\n"
         "typedef unsigned int xj_u4 __attribute__((ext_vector_type(4)));\n"
         "struct XJArgs { const uint8_t* src; int64_t src_stripe; uint8_t* dst; int64_t dst_stripe;"
         " int32_t src_sym, dst_sym; const int32_t* ids; const uint16_t* tab; uint32_t nchunks, ncols,"
      << (C.masked ? " dst_local, mask_words; const uint32_t* masks; const uint8_t* zero; };\n" : " dst_local; };\n")
      << "// K=" << K << " R=" << R << " roles=" << roles << " pairs=" << pairs << " " << C.tag() << "\n"
      << "extern \"C\" __global__ void __launch_bounds__(" << 64 * roles * pairs << ") rs_xj(XJArgs a) {\n";
    if (C.lfin) {
        // the gamma table is the kernel's only LDS variable, at address 0 (checked: the finish block
        // addresses it absolutely); every workgroup copies it once, then loops over columns
        o << "  __shared__ __attribute__((aligned(16))) uint16_t xj_tab[65536];\n"
          << "  asm volatile(\n" << as_string_literals(finish_block(C)) << "  ::: \"memory\");\n"
          << "  if ((uint32_t)(unsigned long)xj_tab != 0u) __builtin_trap();\n"  // a layout change faults, never wrong data
             "  for (uint32_t i = threadIdx.x; i < 8192u; i += blockDim.x)\n"
             "    ((xj_u4*)xj_tab)[i] = ((const xj_u4*)a.tab)[i];\n"
             "  __syncthreads();\n"
             "  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));\n"
          << "  const int role = wave % " << roles << ", pair = wave / " << roles << ";\n"
          << "  const uint32_t la = 0u, lb = 0u;\n"
             "  for (uint32_t c = blockIdx.x * " << pairs << "u + (uint32_t)pair; c < a.ncols; c += gridDim.x * "
          << pairs << "u) {\n"
             "  const uint32_t local = c / a.nchunks, chunk = c - local * a.nchunks;\n"
             "  const uint64_t stripe = a.ids ? (uint64_t)a.ids[local] : (uint64_t)local;\n"
             "  const uint64_t dstripe = a.dst_local ? (uint64_t)local : stripe;\n"
             "  const uint32_t col = chunk * 256u + (threadIdx.x & 63u) * 4u;\n";
    } else {
        o << "  __shared__ __attribute__((aligned(16))) uint32_t xj_lds["
          << (C.coord ? 1024 : C.share ? 4096 : std::max(1, roles * C.lds * 512)) << "];\n"
          << "  asm volatile(\n" << as_string_literals(finish_block(C)) << "  ::: \"memory\");\n"
          << (C.coord ? "  if ((uint32_t)(unsigned long)xj_lds != 0u) __builtin_trap();\n"  // the reads address it absolutely
                        "  for (uint32_t i = threadIdx.x; i < 1024u; i += blockDim.x) xj_lds[i] = ((const uint32_t*)a.tab)[i];\n"
                        "  __syncthreads();\n"
                      : "")
          << (C.xcd ? "  const uint32_t xl = blockIdx.x + blockIdx.y * gridDim.x, xw = gridDim.x >> 3, xk = xl >> 3;\n"
                      "  const uint32_t by = xk / xw, bx = (xl & 7u) * xw + xk % xw;\n"
                      "  const uint64_t stripe = a.ids ? (uint64_t)a.ids[by] : (uint64_t)by;\n"
                      "  const uint64_t dstripe = a.dst_local ? (uint64_t)by : stripe;\n"
                      "  const uint32_t col = bx * 256u + (threadIdx.x & 63u) * 4u;\n"
                    : "  const uint64_t stripe = a.ids ? (uint64_t)a.ids[blockIdx.y] : (uint64_t)blockIdx.y;\n"
                      "  const uint64_t dstripe = a.dst_local ? (uint64_t)blockIdx.y : stripe;\n")
          << (C.cpb > 1 ? "  const uint32_t nc0 = (a.nchunks - blockIdx.x + gridDim.x - 1) / gridDim.x;\n"
                          "  const uint32_t nc = nc0 < " + std::to_string(C.cpb) + "u ? nc0 : " + std::to_string(C.cpb) + "u;\n"
                          "  const uint32_t cs = gridDim.x * 256u;\n"
                          "  uint32_t col = blockIdx.x * 256u + (threadIdx.x & 63u) * 4u;\n"
                        : std::string(C.xcd ? "" : "  const uint32_t col = blockIdx.x * 256u + (threadIdx.x & 63u) * 4u;\n"))
          << ""
             "  const int role = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));\n"
             "  const uint32_t lb = (uint32_t)(unsigned long)xj_lds + (uint32_t)role * "
          << (C.share ? 0 : C.lds * 2048) << "u;\n"
             "  const uint32_t la = lb + (threadIdx.x & 63u) * 4u;\n"
             "  {\n";
    }
    if (C.masked) {  // the launch-local stripe's mask words; the zero buffer's base for this column
        o << "  const uint32_t* xj_mk = a.masks + (uint64_t)blockIdx.y * a.mask_words;\n";
        for (int w = 0; w < nmw; ++w)  // wave-uniform values for the asm's SGPR operands
            o << "  const uint32_t mw" << w << " = __builtin_amdgcn_readfirstlane(xj_mk[" << w << "]);\n";
        o << "  const uint64_t zb = (uint64_t)a.zero;\n";  // a zero buffer as long as the symbols
    }
    o << "  const uint64_t sb = (uint64_t)a.src + stripe * (uint64_t)a.src_stripe;\n"
         "  const uint64_t db = (uint64_t)a.dst + dstripe * (uint64_t)a.dst_stripe;\n"
         "  const uint32_t sl = (uint32_t)sb, sh = (uint32_t)(sb >> 32), dl = (uint32_t)db, dh = (uint32_t)(db >> 32);\n"
         "  switch (role) {\n";
    std::string clob;
    for (int v = 1; v <= C.max_vgpr(); ++v) clob += "\"v" + std::to_string(v) + "\", ";
    for (int s = 32; s <= 63; ++s) clob += "\"s" + std::to_string(s) + "\", ";
    clob += "\"scc\", \"memory\"";
    for (int w = 0; w < roles; ++w) {
        o << "  case " << w << ": asm volatile(\n"
          << as_string_literals(role_block(C, w, cb, K, R, in_slots, out_slots))
          << (C.cpb > 1 ? "  : [col] \"+v\"(col) : [nc] \"s\"(nc), [cs] \"s\"(cs), "  // no LDS address: one VGPR fewer (3 waves/SIMD)
                        : "  : : [col] \"v\"(col), [la] \"v\"(la), ")
          << "[sl] \"s\"(sl), [sh] \"s\"(sh), [dl] \"s\"(dl), [dh] \"s\"(dh),"
             " [ss] \"s\"(a.src_sym), [ds] \"s\"(a.dst_sym), [lb] \"s\"(lb)";
        if (C.masked) {
            for (int m = 0; m < nmw; ++m) o << ", [mw" << m << "] \"s\"(mw" << m << ")";
            o << ", [zb] \"s\"(zb)";
        }
        o << "\n  : "
          << clob << ");\n    break;\n";
    }
    o << "  }\n  }\n}\n";
    return o.str();
}

int xj_outputs_per_role() { return XjConfig().opr; }
int xj_roles(int R) {
    const int opr = XjConfig(R).opr;
    return (R + opr - 1) / opr;
}
int xj_horner(bool env_knobs) { return XjConfig(0, env_knobs).horner; }
int xj_fin() { return XjConfig().lfin; }
int xj_max_roles(int R) {
    // all role waves of a column are one workgroup, so they must fit one CU at the layout's VGPR
    // footprint (fixed map + the compiler's column register, 8-register granules): 12 at 16 outputs
    const XjConfig C(R);
    const int vgprs = (C.max_vgpr() + 2 + 7) / 8 * 8;
    return std::min(kXjMaxRoles, 4 * std::max(1, std::min(8, 512 / vgprs)));
}
int xj_pairs(int R) {
    if (!XjConfig(R).lfin) return 1;
    // column pairs per persistent workgroup: every wave slot of the CU (the 128 KiB table allows one
    // workgroup per CU); VGPRs per wave = the fixed map + the compiler's column / loop registers
    return std::max(1, xj_max_roles(R) / xj_roles(R));
}

// The kernel's symbol carries the hash of its generated source (rs_xj_<8 hex>), so profiler records
// (rocprofv3 Kernel_Name) tell the encode and decode kernels of one run apart; the same hash names
// the kernel in rsg_last_kernel ("rs_xj[RxK:<hash>]").
static std::string xj_named_source(const std::vector<uint16_t>& M, int K, int R, const std::vector<int32_t>& in_slots,
                                   const std::vector<int32_t>& out_slots, std::string* fname, int masked = 0) {
    std::string src = xj_source(M, K, R, in_slots, out_slots, false, masked);
    char nm[32];
    std::snprintf(nm, sizeof nm, "rs_xj_%08llx", static_cast<unsigned long long>(jit_hash(src) & 0xffffffff));
    const std::string key = ") rs_xj(XJArgs a)";
    const size_t at = src.find(key);
    if (at != std::string::npos) src.replace(at, key.size(), std::string(") ") + nm + "(XJArgs a)");
    *fname = nm;
    return src;
}

int xj_precompile(const std::vector<uint16_t>& M, int K, int R, const std::vector<int32_t>& in_slots,
                  const std::vector<int32_t>& out_slots, int masked) {
    if (!xj_supported(8, K, R)) return 0;
    std::string fname;
    const std::string src = xj_named_source(M, K, R, in_slots, out_slots, &fname, masked);
    std::vector<char> code;
    return jit_code(src, "xj", jit_hash(src), code) ? 3 : 0;
}

int xj_build(const std::vector<uint16_t>& M, int K, int R, const std::vector<int32_t>& in_slots,
             const std::vector<int32_t>& out_slots, std::unique_ptr<XjKernel>& out, int masked) {
    out.reset();
    if (!xj_supported(8, K, R)) return 0;
    std::string fname;
    const std::string src = xj_named_source(M, K, R, in_slots, out_slots, &fname, masked);
    uint64_t h = 0;
    std::shared_ptr<JitModule> mod;
    if (jit_module(src, "xj", mod, &h)) return 3;
    auto k = std::make_unique<XjKernel>();
    k->mod = mod;
    (void)hipGetDevice(&k->device);
    k->roles = xj_roles(R);
    k->masked = masked != 0;
    k->coord = masked == 2;
    {
        XjConfig C(R);
        if (masked) C.set_masked(masked);
        C.set_k(K);
        k->cpb = C.cpb;
        k->pairs = C.lfin ? xj_pairs(R) : 0;
    }
    if (hipModuleGetFunction(&k->fn, jit_module_handle(*mod), fname.c_str()) != hipSuccess) return 3;
    char nm[64];
    std::snprintf(nm, sizeof nm, "rs_xj[%dx%d:%s]", R, K, fname.c_str() + 6);
    k->name = nm;
    xj_counts(M, K, R, in_slots, out_slots, masked, &k->valu_per_col, &k->salu_per_col);
    out = std::move(k);
    return 0;
}

namespace {
// Per-device T[w] = gamma * w (128 KiB) for the LDS finish, and the CU count for persistent grids.
struct XjDevState {
    uint16_t* tab = nullptr;
    int cus = 0;
};
XjDevState* xj_dev_state(int device) {
    static std::mutex mu;
    static std::map<int, XjDevState> st;
    std::lock_guard<std::mutex> lk(mu);
    XjDevState& d = st[device];
    if (!d.tab) {
        const Field& F = field();
        std::vector<uint16_t> t(65536, 0);
        for (uint32_t w = 1; w < 65536; ++w) t[w] = F.exp[(F.log[w] + 257u) % kN];
        void* p = nullptr;
        if (hipMalloc(&p, t.size() * 2) != hipSuccess) return nullptr;
        if (hipMemcpy(p, t.data(), t.size() * 2, hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipFree(p);
            return nullptr;
        }
        d.tab = static_cast<uint16_t*>(p);
        if (hipDeviceGetAttribute(&d.cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || d.cus < 1)
            d.cus = 256;
    }
    return &d;
}
}  // namespace

int xj_launch(const XjKernel& k, const XJArgs& a0, int64_t n_stripes, int64_t nchunks, hipStream_t st) {
    if (n_stripes <= 0 || nchunks <= 0) return 0;
#ifdef RS_AMD_DIAG  // every stripe reads and writes stripe 0 (wrong results): diagnostic build only
    static const bool alias = std::getenv("RS_XJ_ALIAS") && std::atoi(std::getenv("RS_XJ_ALIAS"));
#else
    constexpr bool alias = false;
#endif
    if (k.pairs > 0) {  // persistent form: one workgroup per CU loops over all (stripe, chunk) columns
        XjDevState* d = xj_dev_state(k.device);
        if (!d) return 3;
        const unsigned block = unsigned(64 * k.roles * k.pairs);
        for (int64_t s0 = 0; s0 < n_stripes;) {
            const int64_t ns = std::min<int64_t>(n_stripes - s0, int64_t(0x7fffffff) / nchunks);
            XJArgs a = a0;
            if (a.ids) {
                a.ids += s0;
                if (a.dst_local) a.dst += s0 * a.dst_stripe;
            } else {
                a.src += s0 * a.src_stripe;
                a.dst += s0 * a.dst_stripe;
            }
            if (alias) a.src_stripe = a.dst_stripe = 0;
            a.tab = d->tab;
            a.nchunks = uint32_t(nchunks);
            a.ncols = uint32_t(ns * nchunks);
            const int64_t want = (int64_t(a.ncols) + k.pairs - 1) / k.pairs;
            const unsigned grid = unsigned(std::max<int64_t>(1, std::min<int64_t>(d->cus, want)));
            void* args[] = {&a};
            hipError_t e = hipModuleLaunchKernel(k.fn, grid, 1, 1, block, 1, 1, 0, st, args, nullptr);
            if (e != hipSuccess) {
                std::fprintf(stderr, "librs_amd: xj launch: %s\n", hipGetErrorString(e));
                return 3;
            }
            s0 += ns;
        }
        return 0;
    }
    if (alias) {  // diagnostic (wrong results): every stripe reads and writes stripe 0, inputs cache-resident
        XJArgs a = a0;
        a.src_stripe = 0;
        a.dst_stripe = 0;
        void* args[] = {&a};
        a.nchunks = uint32_t(nchunks);
        const unsigned ny = unsigned(std::min<int64_t>(65535, n_stripes));
        hipError_t e = hipModuleLaunchKernel(k.fn, unsigned((nchunks + k.cpb - 1) / k.cpb), ny, 1,
                                             unsigned(64 * k.roles), 1, 1, 0, st, args, nullptr);
        return e == hipSuccess ? 0 : 3;
    }
    for (int64_t s0 = 0; s0 < n_stripes; s0 += 65535) {  // grid.y limit
        XJArgs a = a0;
        if (a.ids) {
            a.ids += s0;
            if (a.dst_local) a.dst += s0 * a.dst_stripe;
        } else {
            a.src += s0 * a.src_stripe;
            a.dst += s0 * a.dst_stripe;
        }
        if (a.masks) a.masks += s0 * int64_t(a.mask_words);  // indexed by the launch-local stripe
        a.nchunks = uint32_t(nchunks);
        const unsigned ny = unsigned(std::min<int64_t>(65535, n_stripes - s0));
        void* args[] = {&a};
        hipError_t e = hipModuleLaunchKernel(k.fn, unsigned((nchunks + k.cpb - 1) / k.cpb), ny, 1,
                                             unsigned(64 * k.roles), 1, 1, 0, st, args, nullptr);
        if (e != hipSuccess) {
            std::fprintf(stderr, "librs_amd: xj launch: %s\n", hipGetErrorString(e));
            return 3;
        }
    }
    return 0;
}

}  // namespace rsamd
