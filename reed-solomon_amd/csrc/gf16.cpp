// gf16.cpp -- see gf16.hpp.
#include "gf16.hpp"

#include <algorithm>
#include <stdexcept>

namespace rsamd {

Field::Field() {
    uint32_t v = 1;
    for (uint32_t i = 0; i < kN; ++i) {
        exp[i] = exp[i + kN] = uint16_t(v);
        log[v] = uint16_t(i);
        v <<= 1;
        if (v & 0x10000u) v ^= kPoly;
    }
    log[0] = 0;
}

const Field& field() {
    static const Field* f = new Field();
    return *f;
}

static inline uint16_t next_elem(uint16_t s) { return uint16_t((uint32_t(s) << 1) % kN); }

Cosets::Cosets() {
    std::vector<uint8_t> seen(kN, 0);
    for (uint32_t s = 0; s < kN; ++s) {
        if (seen[s]) continue;
        uint16_t e = uint16_t(s);
        int size = 0;
        do {
            seen[e] = 1;
            e = next_elem(e);
            ++size;
        } while (e != s);
        int li = 0;
        while ((1 << li) != size) ++li;
        leaders[li].push_back(uint16_t(s));
    }
}

const Cosets& cosets() {
    static const Cosets* c = new Cosets();
    return *c;
}

static const uint16_t kThreshold[5] = {0, 1, 3, 15, 255};  // reference cyclotomic_coset.h:58-78

uint16_t coset_upper_bound(uint16_t n) {
    uint16_t cnt = 0;
    for (int i = 4; i >= 0 && n; --i) {
        if (n > kThreshold[i]) {
            uint16_t take = uint16_t((n - kThreshold[i] + (1u << i) - 1) >> i);
            cnt = uint16_t(cnt + take);
            n = uint16_t(n - (take << i));
        }
    }
    return cnt;
}

// Mirrors the reference selection rule (cyclotomic_coset.c:154-207): repair first, largest coset
// sizes while the remainder exceeds the size's threshold; information next from the unused
// leaders with thresholds lowered by the repair consumption of smaller sizes; last may be partial.
void select_cosets(uint16_t k, uint16_t r, std::vector<CosetRef>& inf, std::vector<CosetRef>& rep) {
    const Cosets& cs = cosets();
    inf.clear();
    rep.clear();
    size_t used[5] = {0, 0, 0, 0, 0};
    const uint16_t rep_cap = coset_upper_bound(r), inf_cap = coset_upper_bound(k);
    for (int i = 4; i >= 0 && r; --i) {
        while (r > kThreshold[i] && rep.size() < rep_cap) {
            rep.push_back({cs.leaders[i].at(used[i]++), uint8_t(1u << i)});
            r = uint16_t(r - (1u << i));
        }
    }
    uint16_t th[5];
    for (int j = 0; j < 5; ++j) {
        th[j] = kThreshold[j];
        for (int i = 0; i < j; ++i) th[j] = uint16_t(th[j] - (used[i] << i));
    }
    for (int i = 4; i >= 0 && k; --i) {
        while (k > th[i] && inf.size() < inf_cap) {
            inf.push_back({cs.leaders[i].at(used[i]++), uint8_t(1u << i)});
            k = uint16_t(k - std::min<uint32_t>(k, 1u << i));
        }
    }
}

static void expand(const std::vector<CosetRef>& cs, uint16_t want, std::vector<uint16_t>& out) {
    uint16_t got = 0;
    for (const CosetRef& c : cs) {
        uint16_t e = c.leader;
        do {
            if (got == want) return;
            out.push_back(e);
            ++got;
            e = next_elem(e);
        } while (e != c.leader);
    }
}

std::vector<uint16_t> code_positions(uint16_t k, uint16_t r) {
    std::vector<CosetRef> inf, rep;
    select_cosets(k, r, inf, rep);
    std::vector<uint16_t> pos;
    pos.reserve(size_t(k) + r);
    expand(inf, k, pos);
    expand(rep, r, pos);
    if (pos.size() != size_t(k) + r) throw std::runtime_error("position selection failed");
    return pos;
}

int subfield_degree(const std::vector<uint16_t>& positions) {
    // alpha^pos lies in GF(2^m) iff pos is a multiple of (2^16 - 1) / (2^m - 1).
    static const int ms[5] = {1, 2, 4, 8, 16};
    for (int m : ms) {
        uint32_t step = kN / ((1u << m) - 1);
        bool ok = true;
        for (uint16_t p : positions)
            if (p % step) {
                ok = false;
                break;
            }
        if (ok) return m;
    }
    return 16;
}

std::vector<uint16_t> solve_matrix(const std::vector<uint16_t>& targets, const std::vector<int>& emit,
                                   const std::vector<uint16_t>& sources) {
    const Field& F = field();
    const size_t d = targets.size(), ns = sources.size();
    std::vector<uint16_t> X(d), Y(ns);
    for (size_t i = 0; i < d; ++i) X[i] = F.exp[targets[i]];
    for (size_t j = 0; j < ns; ++j) Y[j] = F.exp[sources[j]];
    // log P(Y_q) = sum_e log(Y_q + X_e); log P'(X_p) = sum_{e != p} log(X_p + X_e)  (all mod N)
    std::vector<uint32_t> lp(ns), ld(d);
    for (size_t j = 0; j < ns; ++j) {
        uint64_t s = 0;
        for (size_t e = 0; e < d; ++e) s += F.log[Y[j] ^ X[e]];
        lp[j] = uint32_t(s % kN);
    }
    for (size_t i = 0; i < d; ++i) {
        uint64_t s = 0;
        for (size_t e = 0; e < d; ++e)
            if (e != i) s += F.log[X[i] ^ X[e]];
        ld[i] = uint32_t(s % kN);
    }
    std::vector<uint16_t> M(emit.size() * ns);
    for (size_t row = 0; row < emit.size(); ++row) {
        const size_t p = size_t(emit[row]);
        uint16_t* out = M.data() + row * ns;
        for (size_t j = 0; j < ns; ++j) {
            uint32_t e = lp[j] + 2 * kN - ld[p] - F.log[X[p] ^ Y[j]];
            out[j] = F.exp[e % kN];
        }
    }
    return M;
}

Gamma8::Gamma8() {
    const Field& F = field();
    uint16_t g[8];
    for (int j = 0; j < 8; ++j) g[j] = F.exp[(257u * j) % kN];
    for (int b = 0; b < 256; ++b) {
        uint16_t e = 0;
        for (int j = 0; j < 8; ++j)
            if (b & (1 << j)) e ^= g[j];
        to_elem[b] = e;
    }
    for (int b = 0; b < 256; ++b) {
        ibyte[0][b] = to_elem[b];
        ibyte[1][b] = F.mul(to_elem[b], 2);  // * alpha
    }
    std::vector<uint16_t> inv(65536);
    for (uint32_t u = 0; u < 65536; ++u) {
        uint16_t w = uint16_t(ibyte[0][u & 255] ^ ibyte[1][u >> 8]);
        inv[w] = uint16_t(u);
    }
    for (int b = 0; b < 256; ++b) {
        lbyte[0][b] = inv[b];
        lbyte[1][b] = inv[uint32_t(b) << 8];
    }
    for (uint32_t i = 0; i < kN; ++i) from_elem_log[i] = 0;
    for (int b = 1; b < 256; ++b) from_elem_log[F.log[to_elem[b]]] = uint8_t(b);
    red = coord(F.exp[(257u * 8) % kN]);
}

uint8_t Gamma8::coord(uint16_t c) const {
    if (!c) return 0;
    uint16_t u = uint16_t(lbyte[0][c & 255] ^ lbyte[1][c >> 8]);
    if (u >> 8) throw std::runtime_error("coefficient outside GF(256)");
    return uint8_t(u);
}

const Gamma8& gamma8() {
    static const Gamma8* g = new Gamma8();
    return *g;
}

}  // namespace rsamd
