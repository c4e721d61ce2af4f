// rs_route16.cpp -- the GF(2^16) syndrome route: the reference's own
// factorisation of a coding matrix (cyclotomic-FFT syndromes, then evaluator + Forney, reference
// reed_solomon.c:186-559) as device plans for k_cs16t / k_cs16 and the k_bs16 / dense second stage,
// the re-encode decode, plan selection (make_plan) and the route launches (run_cs, run_reenc).
#include "rs_core.hpp"

using namespace rsamd;

namespace rsamd {

// Second stage of the syndrome route: out_p = sum_{j < D} M2[p][j] S_j for the emitted targets p, with
// E = all D targets. This is the reference's evaluator + Forney restore (reed_solomon.c:186-336, the same
// for encode, E = repair positions, and decode, E = erased positions):
//   Omega = S * Lambda_E mod x^D,  out_p = F_p * sum_{i < D} X_p^-i Omega_i,  F_p = X_p / Lambda_E'(X_p^-1)
// so M2[p][j] = F_p x^j sum_{d = 0}^{D - 1 - j} Lambda_d x^d with x = X_p^-1 (O(D) per row).
std::vector<uint16_t> syndrome_solve_matrix(const std::vector<uint16_t>& targets, const std::vector<int>& emit) {
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

CsHost cs16_host(const std::vector<uint16_t>& pos, const std::vector<int32_t>& in_slots, int D) {
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

int upload_cs(DevPlan& p, const CsHost& h, int kind, const std::vector<int32_t>& in_slots, hipStream_t st);

int build_cs16(DevPlan& p, const std::vector<uint16_t>& pos, const std::vector<int32_t>& in_slots, int D,
               hipStream_t st) {
    return upload_cs(p, cs16_host(pos, in_slots, D), 0, in_slots, st);
}

int upload_cs(DevPlan& p, const CsHost& h, int kind, const std::vector<int32_t>& in_slots, hipStream_t st) {
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
bool bs16_host(const std::vector<uint16_t>& M2, int D, const std::vector<uint16_t>& targets,
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
int orbit_step(const std::vector<uint16_t>& pos) {
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
bool cs_route_eligible(const rsg_codec_t* c, int K, int R, int D) {
    // 1: every matrix with K >= 64 inputs (measured at C5: the route wins at every t from 1 to 1024, e.g.
    // t = 32 decode 20.4 -> 4.4 ms, t = 1 13.1 -> 1.1 ms: the dense kernels for R <= 32 walk all K inputs
    // per workgroup); 2 (measurements): every matrix, whatever its shape
    return c->m > 8 && D <= 32768 && R > 0 && ((c->m16_route == 1 && K >= 64) || (c->m16_route == 2 && K > 0));
}

int make_plan_dense(rsg_codec_t* c, const bool* erased, std::unique_ptr<DevPlan>& out, hipStream_t st);

// GF(2^16) matrix on the syndrome route: the k_cs16 plan over the sources + the D x R second stage
int make_plan_cs(rsg_codec_t* c, const bool* erased, std::unique_ptr<DevPlan>& out, hipStream_t st) {
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
bool reenc_eligible(const rsg_codec_t* c, const bool* erased) {
    if (!c->m16_reenc || c->m <= 8 || !erased || !c->enc || !c->enc->cs || c->enc->cs->kind != 0 || !c->enc->second ||
        !c->enc->second->cs || c->enc->second->cs->kind != 1 || c->enc->cs->h_groups.empty())
        return false;
    int t = 0;
    for (int i = 0; i < c->k; ++i) t += erased[i] ? 1 : 0;
    for (int i = c->k; i < c->k + c->r; ++i)
        if (erased[i]) return false;
    return t >= 1 && 10 * t >= 9 * c->r && c->k - t >= 64;
}

// The route plan of a decode pattern, built when its dense plan has moved route_min_bytes. Among the
// re-encode-eligible patterns, one whose erased set is closed under x -> x^(2^d), d <= 4, may give the plain
// route a k_bs16 second stage over orbits of >= 4 rows -- cheaper than re-encoding plus the dense t x r
// stage -- but only when bs16_host accepts its rows (orbit runs of at least 2 rows on average): so the plain
// route is built, and replaced by the re-encode decode when its second stage came out dense (no speed cliff).
int make_plan_route(rsg_codec_t* c, const bool* erased, bool reenc_ok, std::unique_ptr<DevPlan>& out,
                    hipStream_t st) {
    if (!reenc_ok || !reenc_eligible(c, erased)) return make_plan_cs(c, erased, out, st);
    std::vector<uint16_t> pos;
    for (int i = 0; i < c->k; ++i)
        if (erased[i]) pos.push_back(c->positions[size_t(i)]);
    if (orbit_step(pos) > 4) return make_plan_reenc(c, erased, out, st);
    if (int rc = make_plan_cs(c, erased, out, st)) return rc;
    if (out->second && out->second->cs && out->second->cs->kind == 1) return 0;  // the k_bs16 orbit stage
    out.reset();  // never launched: its memory goes back to the pool behind its upload
    return make_plan_reenc(c, erased, out, st);
}

int make_plan_reenc(rsg_codec_t* c, const bool* erased, std::unique_ptr<DevPlan>& out, hipStream_t st) {
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

int make_plan(rsg_codec_t* c, const bool* erased, std::unique_ptr<DevPlan>& out, hipStream_t st) {
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
int make_plan_dense(rsg_codec_t* c, const bool* erased, std::unique_ptr<DevPlan>& out, hipStream_t st) {
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

// The codec's syndrome stream and its events (the per-stripe route and m16_cs_overlap)
int overlap_objects(rsg_codec_t* c) {
    if (!c->ps_synst) HIP_TRY(hipStreamCreateWithFlags(&c->ps_synst, hipStreamNonBlocking));
    for (hipEvent_t* e : {&c->ps_ev_entry, &c->ps_ev_used[0], &c->ps_ev_used[1], &c->ps_ev_syn[0], &c->ps_ev_syn[1]})
        if (!*e) HIP_TRY(hipEventCreateWithFlags(e, hipEventDisableTiming));
    return 0;
}

constexpr int64_t kCsOverlapChunks = 4, kCsOverlapMinStripes = 16;

int run_cs(rsg_codec_t* c, DevPlan& p, const uint8_t* src, int64_t src_stripe, int64_t src_sym, uint8_t* dst,
           int64_t dst_stripe, int64_t dst_sym, uint64_t n_stripes, uint64_t S, hipStream_t st,
           const int32_t* groups) {
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
    // a failure after the first launch goes through scratch_fence: the scratch stays marked busy on st
    const int rc = [&]() -> int {
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
            RS_CHECKPOINT(c, &p, "GF(2^16) route k_bs16", n_stripes, S);
            const uint64_t steps = uint64_t(a.units) * waves_per_unit * uint64_t(cs.ntiles) * uint64_t(cs.ngroups);
            c->work_valu += steps * kValu_bs16;
            c->work_salu += steps * kSalu_bs16;
            c->last_kernel = "bs16";
            return 0;
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
                RS_CHECKPOINT(c, &p, "GF(2^16) route syndromes k_cs16t", uint64_t(cn), S);
                c->work_valu += uint64_t(a.units) * waves_per_unit * cs.valu_t;
                c->work_salu += uint64_t(a.units) * waves_per_unit * uint64_t(cs.ntiles_t) * uint64_t(cs.ngroups) * kSaluStepCs16t;
            } else {
                HIP_TRY(launch_cs16(a, sy));
                RS_CHECKPOINT(c, &p, "GF(2^16) route syndromes k_cs16", uint64_t(cn), S);
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
        return 0;
    }();
    return rc ? scratch_fence(c, st, rc) : scratch_release(c, st);
}

// The re-encode decode (DevPlan::Reenc) over a chunk loop: the encode route over U into scratch rows
// (G_U u), + the received repair rows, then D_Rep from scratch into the erased information slots.
int run_reenc(rsg_codec_t* c, DevPlan& p, uint8_t* base, int64_t stripe_stride, int64_t sym,
              uint64_t n_stripes, uint64_t S, hipStream_t st) {
    DevPlan& E = *c->enc;
    if (int rc = E.order_after_build(st)) return rc;  // its records are read directly (run_cs, not run_plan)
    const int64_t k = c->k, r = c->r, per = r * int64_t(S);
    const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>({int64_t(n_stripes), (int64_t(1) << 30) / per, 65535}));
    if (int rc = scratch_acquire(c, st)) return rc;
    const int rc = [&]() -> int {
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
        return 0;
    }();
    return rc ? scratch_fence(c, st, rc) : scratch_release(c, st);
}

}  // namespace rsamd

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
    if (ok) copy_out(rec, h.rec);
    if (ok) copy_out(fin, h.fin);
    if (ok) copy_out(fin_off, h.fin_off);
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
    copy_out(rec, h.rec_t);
    copy_out(fin, h.fin_t);
    copy_out(fin_off, h.fin_off_t);
    if (blocks) std::memcpy(blocks, kCs16tOff, sizeof(kCs16tOff));
    return 0;
}

// Host-only view of the GF(2^16) syndrome route of the encode (is_erased == NULL) or decode matrix: the
// k_cs16 plan (groups, records, finish lists) and the second-stage matrix M2 [R][D]. info = {D, ngroups,
// ntiles, fin_stride, R}; array arguments may be NULL (query the sizes first). No GPU is used.
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
    copy_out(groups, h.groups, size_t(h.ngroups) * 16);  // even count, without the tail
    copy_out(rec, h.rec);
    copy_out(fin, h.fin);
    copy_out(fin_off, h.fin_off);
    if (m2) {
        const std::vector<uint16_t> M = syndrome_solve_matrix(targets, emit);
        copy_out(m2, M);
    }
    return 0;
}
