// gf16.hpp -- host-side GF(2^16) arithmetic, code-position selection and coding-matrix
// construction for the MI355X Reed-Solomon engine.
//
// Field: GF(2)[x]/(x^16+x^5+x^3+x^2+1), alpha = x   (reference include/rs/gf65536.h:21-27).
// Positions: 2-cyclotomic cosets mod N = 65535 chosen exactly like the reference
//            (src/rs/cyclotomic_coset.c:154-230), so every matrix below reproduces the
//            reference's linear maps bit for bit.
//
// The reference computes repair symbols and restored symbols through syndromes, a locator,
// an evaluator and Forney's formula (src/rs/reed_solomon.c:338-559). Both are solutions of a
// d x d Vandermonde system  sum_{p in E} X_p^j e_p = S_j (j < d), S_j = sum_q X_q^j f_q,
// so each output is a fixed GF(2^16)-linear combination of the inputs:
//     e_p = sum_q L_p(X_q) f_q,   L_p(z) = prod_{e in E, e != p} (z + X_e) / (X_p + X_e),
// i.e. a scaled Cauchy matrix  P(X_q) / ((X_p + X_q) P'(X_p)) with P(z) = prod_{e in E}(z + X_e).
// The engine applies that matrix on the GPU; construction here is O(d * n) field operations.
#pragma once
#include <cstdint>
#include <cstddef>
#include <vector>

namespace rsamd {

constexpr uint32_t kN = 65535;         // multiplicative group order (reference prelude.h:16)
constexpr uint32_t kPoly = 0x1002Du;   // reference gf65536.h:27

struct Field {
    uint16_t exp[2 * kN];  // alpha^i, i < 2N
    uint16_t log[65536];   // log[0] unused
    Field();
    uint16_t mul(uint16_t a, uint16_t b) const {
        return (a && b) ? exp[uint32_t(log[a]) + log[b]] : 0;
    }
    uint16_t inv(uint16_t a) const { return exp[(kN - log[a]) % kN]; }
    uint16_t div(uint16_t a, uint16_t b) const {
        return a ? exp[(kN + uint32_t(log[a]) - log[b]) % kN] : 0;
    }
    uint16_t pow_alpha(uint64_t e) const { return exp[e % kN]; }
};

const Field& field();

// Coset leaders of size 2^i (i = 0..4) in ascending order (reference cyclotomic_coset.c:52-106).
struct Cosets {
    std::vector<uint16_t> leaders[5];
    Cosets();
};
const Cosets& cosets();

struct CosetRef {
    uint16_t leader;
    uint8_t size;
};

uint16_t coset_upper_bound(uint16_t n);  // reference _cc_get_cosets_cnt (cyclotomic_coset.c:129-147)
void select_cosets(uint16_t k, uint16_t r, std::vector<CosetRef>& inf, std::vector<CosetRef>& rep);
// positions[0..k) information, positions[k..k+r) repair.
std::vector<uint16_t> code_positions(uint16_t k, uint16_t r);

// Smallest m in {1,2,4,8,16} such that every X = alpha^pos lies in GF(2^m).
int subfield_degree(const std::vector<uint16_t>& positions);

// Coding matrix: rows = targets, cols = sources, entry (p, q) = L_p(X_q) as above.
// `targets` holds the d positions of E (the system is solved over all of them), `emit` the
// subset of target indices (into `targets`) whose rows are returned, in order.
std::vector<uint16_t> solve_matrix(const std::vector<uint16_t>& targets, const std::vector<int>& emit,
                                   const std::vector<uint16_t>& sources);

// ---------------------------------------------------------------------------------------------
// GF(256) coordinates used by the m <= 8 kernels. gamma = alpha^257 generates GF(256);
// x in GF(2^16) is written x = x0 + x1 * alpha with x0, x1 in GF(256) and each x_h in the
// gamma-polynomial basis (one byte). Multiplication by c in GF(256) then acts byte-wise.
struct Gamma8 {
    uint16_t to_elem[256];   // byte -> element of GF(256) as a GF(2^16) value
    uint8_t from_elem_log[kN];  // only valid for logs that are multiples of 257
    uint16_t lbyte[2][256];  // L(w) = lbyte[0][w & 255] ^ lbyte[1][w >> 8]   (alpha basis -> coords)
    uint16_t ibyte[2][256];  // L^-1(u) = ibyte[0][u & 255] ^ ibyte[1][u >> 8] (coords -> alpha basis)
    uint8_t red;             // gamma^8 in gamma-basis coordinates (xtime reduction byte)
    Gamma8();
    uint8_t coord(uint16_t c) const;  // c in GF(256) subfield -> byte
};
const Gamma8& gamma8();

}  // namespace rsamd
