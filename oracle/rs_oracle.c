/*
 * rs_oracle.c -- CPU restatement of the reference Reed-Solomon algorithm (TEST INFRASTRUCTURE ONLY).
 * See rs_oracle.h for scope. Every function cites the reference file:line it follows
 * (paths relative to /root/reference).
 */
#define _GNU_SOURCE
#include "rs_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- field tables ---------------
 * Follows src/rs/gf65536.c:59-111: alpha = x, modulus 0x1002D, pow[] wraps at N, log[0] unused. */
#define POLY 0x1002Du

static uint16_t g_exp[2 * ORC_N];
static uint16_t g_log[65536];
static uint16_t g_nrepr[5][ORC_N]; /* [log2 m][d]: normal-basis coordinates of alpha^d in GF(2^m) */

/* Normal bases of the subfields GF(2^m), m = 1,2,4,8,16 (values stated in src/rs/gf65536.c:21-57). */
static const uint16_t NB1[1] = {1};
static const uint16_t NB2[2] = {44234, 44235};
static const uint16_t NB4[4] = {10800, 47860, 34555, 5694};
static const uint16_t NB8[8] = {16402, 53598, 44348, 63986, 22060, 64366, 6088, 32521};
static const uint16_t NB16[16] = {2048, 2880,  7129,  30616, 2643,  6897,  29685, 7378,
                                  30100, 2743, 20193, 36223, 24055, 41458, 41014, 61451};

static const uint16_t* nb_of(uint8_t m) {
    switch (m) {
    case 1: return NB1;
    case 2: return NB2;
    case 4: return NB4;
    case 8: return NB8;
    default: return NB16;
    }
}

static int lg2m(uint8_t m) { return m == 1 ? 0 : m == 2 ? 1 : m == 4 ? 2 : m == 8 ? 3 : 4; }

/* ---------------------------------------------------------------- cosets -------------------
 * Follows include/rs/cyclotomic_coset.h:18-87 and src/rs/cyclotomic_coset.c:52-106. */
static const uint16_t THRESH[5] = {0, 1, 3, 15, 255};
static uint16_t g_leaders[5][4080]; /* leaders by coset size 2^i, ascending */

static inline uint16_t dbl(uint16_t s) { return (uint16_t)(((uint32_t)s << 1) % ORC_N); }

static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void build_tables(void) {
    uint32_t v = 1;
    for (uint32_t i = 0; i < ORC_N; ++i) {
        g_exp[i] = (uint16_t)v;
        g_exp[i + ORC_N] = (uint16_t)v;
        g_log[v] = (uint16_t)i;
        v <<= 1;
        if (v & 0x10000u) v ^= POLY;
    }
    for (int li = 0; li < 5; ++li) {
        uint8_t m = (uint8_t)(1u << li);
        const uint16_t* nb = nb_of(m);
        memset(g_nrepr[li], 0, sizeof(g_nrepr[li]));
        for (uint32_t bits = 1; bits < (1u << m); ++bits) {
            uint16_t e = 0;
            for (int j = 0; j < m; ++j)
                if (bits & (1u << j)) e ^= nb[j];
            g_nrepr[li][g_log[e]] = (uint16_t)bits;
        }
    }
    static uint8_t seen[ORC_N];
    uint16_t fill[5] = {0, 0, 0, 0, 0};
    memset(seen, 0, sizeof(seen));
    for (uint32_t s = 0; s < ORC_N; ++s) {
        if (seen[s]) continue;
        uint16_t e = (uint16_t)s;
        int sz = 0;
        do {
            seen[e] = 1;
            e = dbl(e);
            ++sz;
        } while (e != s);
        int li = lg2m((uint8_t)sz);
        g_leaders[li][fill[li]++] = (uint16_t)s;
    }
}

int orc_init(void) {
    pthread_once(&g_once, build_tables);
    return 0;
}

uint16_t orc_pow(uint32_t e) { return g_exp[e % ORC_N]; }
uint16_t orc_log(uint16_t a) { return g_log[a]; }

/* gf_mul_ee / gf_div_ee semantics: src/rs/gf65536.c:132-153. */
uint16_t orc_mul(uint16_t a, uint16_t b) {
    if (!a || !b) return 0;
    return g_exp[(uint32_t)g_log[a] + g_log[b]];
}

uint16_t orc_div(uint16_t a, uint16_t b) {
    if (!a) return 0;
    return g_exp[(ORC_N + (uint32_t)g_log[a] - g_log[b]) % ORC_N];
}

uint16_t orc_normal_repr(uint8_t m, uint16_t d) { return g_nrepr[lg2m(m)][d % ORC_N]; }

/* cc_get_coset_size: src/rs/cyclotomic_coset.c:114-122 */
uint8_t orc_coset_size(uint16_t leader) {
    uint8_t m = 1;
    while (leader != (uint16_t)(((uint32_t)leader << m) % ORC_N)) m <<= 1;
    return m;
}

/* _cc_get_cosets_cnt: src/rs/cyclotomic_coset.c:129-147 */
uint16_t orc_cosets_upper(uint16_t n) {
    uint16_t cnt = 0;
    for (int i = 4; i >= 0 && n; --i) {
        if (n > THRESH[i]) {
            uint16_t take = (uint16_t)((n - THRESH[i] + (1u << i) - 1) >> i);
            cnt += take;
            n -= (uint16_t)(take << i);
        }
    }
    return cnt;
}

/* cc_select_cosets: src/rs/cyclotomic_coset.c:154-207. Repair cosets are chosen first (largest
 * sizes while the remainder exceeds the size threshold), information cosets continue from the
 * unused leaders with thresholds lowered by what repair consumed; the last one may be partial. */
void orc_select_cosets(uint16_t k, uint16_t r, uint16_t* inf_leader, uint8_t* inf_size, uint16_t* n_inf,
                       uint16_t* rep_leader, uint8_t* rep_size, uint16_t* n_rep) {
    orc_init();
    uint16_t used[5] = {0, 0, 0, 0, 0};
    uint16_t inf_cap = orc_cosets_upper(k), rep_cap = orc_cosets_upper(r);
    uint16_t nr = 0, ni = 0;

    for (int i = 4; i >= 0 && r; --i) {
        while (r > THRESH[i] && nr < rep_cap) {
            rep_leader[nr] = g_leaders[i][used[i]++];
            rep_size[nr++] = (uint8_t)(1u << i);
            r -= (uint16_t)(1u << i);
        }
    }
    *n_rep = nr;

    uint16_t th[5];
    for (int j = 0; j < 5; ++j) {
        th[j] = THRESH[j];
        for (int i = 0; i < j; ++i) th[j] = (uint16_t)(th[j] - (used[i] << i));
    }
    for (int i = 4; i >= 0 && k; --i) {
        while (k > th[i] && ni < inf_cap) {
            inf_leader[ni] = g_leaders[i][used[i]++];
            inf_size[ni++] = (uint8_t)(1u << i);
            k -= (uint16_t)(k < (1u << i) ? k : (1u << i));
        }
    }
    *n_inf = ni;
}

/* cc_cosets_to_positions: src/rs/cyclotomic_coset.c:209-230 (coset order leader, 2L, 4L, ...). */
static void expand(const uint16_t* leader, uint16_t n, uint16_t* out, uint16_t want) {
    uint16_t w = 0;
    for (uint16_t c = 0; c < n && w < want; ++c) {
        uint16_t e = leader[c];
        do {
            out[w++] = e;
            e = dbl(e);
        } while (e != leader[c] && w < want);
    }
}

void orc_positions(uint16_t k, uint16_t r, uint16_t* positions) {
    uint16_t ci = orc_cosets_upper(k), cr = orc_cosets_upper(r);
    uint16_t* il = calloc(ci + 1, sizeof(uint16_t));
    uint16_t* rl = calloc(cr + 1, sizeof(uint16_t));
    uint8_t* is = calloc(ci + 1, 1);
    uint8_t* rs = calloc(cr + 1, 1);
    uint16_t ni = 0, nr = 0;
    orc_select_cosets(k, r, il, is, &ni, rl, rs, &nr);
    expand(il, ni, positions, k);
    expand(rl, nr, positions + k, r);
    free(il);
    free(rl);
    free(is);
    free(rs);
}

/* ---------------------------------------------------------------- symbol-wide ops ----------
 * gf_add / gf_mul / gf_madd: src/rs/gf65536.c:155-219 (little-endian uint16 words), with the
 * reference's cost structure: gf_add is a 64-bit XOR loop with a 16-bit tail (:161-169), gf_mul /
 * gf_madd read and write whole 16-bit words through pow_table shifted by log(c), skipping zero
 * words (:186-193, :211-218). The word types are alias-safe and alignment-free, so any byte offset
 * works (x86-64 and the compilers here do unaligned word access natively). */
typedef uint64_t __attribute__((may_alias, aligned(1))) u64w;
typedef uint16_t __attribute__((may_alias, aligned(1))) u16w;

static void sym_xor(uint8_t* a, const uint8_t* b, size_t S) {
    u64w* x = (u64w*)a;
    const u64w* y = (const u64w*)b;
    size_t n8 = S / 8, i;
    for (i = 0; i < n8; ++i) x[i] ^= y[i];
    u16w* x2 = (u16w*)(a + 8 * n8);
    const u16w* y2 = (const u16w*)(b + 8 * n8);
    for (i = 0; i < (S - 8 * n8) / 2; ++i) x2[i] ^= y2[i];
}

static void sym_madd(uint8_t* a, uint16_t c, const uint8_t* b, size_t S) {
    if (c == 0) return;
    if (c == 1) {
        sym_xor(a, b, S);
        return;
    }
    const uint16_t* shifted = g_exp + g_log[c];
    u16w* x = (u16w*)a;
    const u16w* y = (const u16w*)b;
    for (size_t i = 0, n = S / 2; i < n; ++i) {
        uint16_t w = y[i];
        if (w) x[i] ^= shifted[g_log[w]];
    }
}

static void sym_scale(uint8_t* a, uint16_t c, size_t S) {
    if (c == 1) return;
    if (c == 0) {
        memset(a, 0, S);
        return;
    }
    const uint16_t* shifted = g_exp + g_log[c];
    u16w* x = (u16w*)a;
    for (size_t i = 0, n = S / 2; i < n; ++i) {
        uint16_t w = x[i];
        if (w) x[i] = shifted[g_log[w]];
    }
}

/* ---------------------------------------------------------------- transforms ---------------
 * Syndromes S_j = sum_i f_i * alpha^(pos_i * j), j < L, by the cyclotomic FFT of
 * src/rs/fft.c:39-100: for every coset {s, 2s, 4s, ...} of a syndrome index, accumulate each
 * input into the normal-basis slots u_t selected by the bits of alpha^(s*pos_i), then combine
 * S_(2^j s) = sum_t nb_((j+t) mod m) * u_t; u is a 16-symbol sequence per call (fft.c:53). */
static uint8_t** seq_alloc(size_t n, size_t S);
static void seq_free(uint8_t** v, size_t n);

static int syndromes(const uint8_t* const* f, const uint16_t* pos, size_t nf, size_t S, uint8_t* const* res,
                     size_t L) {
    uint8_t* done = calloc(L ? L : 1, 1);
    uint8_t** u = seq_alloc(16, S);
    if (!done || !u) {
        free(done);
        seq_free(u, 16);
        return 1;
    }
    for (size_t s = 0; s < L; ++s) {
        if (done[s]) continue;
        uint8_t m = orc_coset_size((uint16_t)s);
        const uint16_t* nb = nb_of(m);
        const uint16_t* repr = g_nrepr[lg2m(m)];
        for (int t = 0; t < m; ++t) memset(u[t], 0, S);
        for (size_t i = 0; i < nf; ++i) {
            uint16_t bits = repr[((uint32_t)s * pos[i]) % ORC_N];
            for (int t = 0; t < m; ++t)
                if (bits & (1u << t)) sym_xor(u[t], f[i], S);
        }
        uint32_t idx = (uint32_t)s;
        for (int j = 0; j < m; ++j) {
            if (idx < L) {
                memset(res[idx], 0, S);
                for (int t = 0; t < m; ++t) sym_madd(res[idx], nb[(j + t) % m], u[t], S);
                done[idx] = 1;
            }
            idx = dbl((uint16_t)idx);
        }
    }
    free(done);
    seq_free(u, 16);
    return 0;
}

/* Locator Lambda(x) = prod_e (1 + X_e x): src/rs/reed_solomon.c:83-102 (for the repair set the
 * reference multiplies per-coset factors, :116-175, which is the same polynomial). */
static void locator(const uint16_t* pos, size_t n, uint16_t* lam) {
    lam[0] = 1;
    for (size_t d = 0; d < n; ++d) {
        uint16_t X = g_exp[pos[d]];
        lam[d + 1] = 0;
        for (size_t i = d + 1; i > 0; --i) lam[i] ^= orc_mul(lam[i - 1], X);
    }
}

/* Omega = S * Lambda mod x^L: src/rs/reed_solomon.c:220-246 */
static void evaluator(uint8_t* const* syn, const uint16_t* lam, size_t L, size_t S, uint8_t* const* om) {
    for (size_t i = 0; i < L; ++i) memset(om[i], 0, S);
    for (size_t i = 0; i < L; ++i) {
        if (!lam[i]) continue;
        for (size_t j = 0; i + j < L; ++j) sym_madd(om[i + j], lam[i], syn[j], S);
    }
}

/* Forney coefficient X_p / Lambda'(X_p^-1): src/rs/reed_solomon.c:186-210 */
static uint16_t forney(const uint16_t* lam, size_t d, uint16_t p) {
    uint16_t q = 0;
    for (size_t j = 0; j < d; j += 2) {
        uint16_t c = lam[j + 1];
        if (c) q ^= orc_mul(c, g_exp[((uint64_t)j * (ORC_N - p)) % ORC_N]);
    }
    return orc_div(g_exp[p], q);
}

/* ---------------------------------------------------------------- encode / decode ----------*/
/* Temporaries allocated as the reference allocates them: seq_create callocs every symbol on its own
 * (src/memory/seq.c:17-46, symbol.c:17-32), per call (reed_solomon.c:384-402, fft.c:53,143), so the
 * port pays the same allocation and first-touch cost as the reference. */
static void seq_free(uint8_t** v, size_t n) {
    if (!v) return;
    for (size_t i = 0; i < n; ++i) free(v[i]);
    free(v);
}

static uint8_t** seq_alloc(size_t n, size_t S) {
    uint8_t** v = calloc(n ? n : 1, sizeof(uint8_t*));
    if (!v) return NULL;
    for (size_t i = 0; i < n; ++i)
        if (!(v[i] = calloc(S ? S : 1, 1))) {
            seq_free(v, n);
            return NULL;
        }
    return v;
}

static uint8_t** carve(uint8_t* base, size_t n, size_t S) {
    uint8_t** v = malloc((n ? n : 1) * sizeof(uint8_t*));
    if (!v) return NULL;
    for (size_t i = 0; i < n; ++i) v[i] = base + i * S;
    return v;
}

/* rs_generate_repair_symbols: src/rs/reed_solomon.c:338-441 */
int orc_encode(uint16_t k, uint16_t r, size_t S, const uint8_t* const* info, uint8_t* const* rep) {
    orc_init();
    int rc = 1;
    uint16_t* pos = calloc((size_t)k + r + 1, sizeof(uint16_t));
    uint16_t* lam = calloc((size_t)r + 2, sizeof(uint16_t));
    uint16_t ci = orc_cosets_upper(k), cr = orc_cosets_upper(r);
    uint16_t *il = calloc(ci + 1, 2), *rl = calloc(cr + 1, 2);
    uint8_t *is = calloc(ci + 1, 1), *rsz = calloc(cr + 1, 1);
    uint8_t **syn = seq_alloc(r, S), **om = seq_alloc(r, S), **u = NULL;
    if (!pos || !lam || !il || !rl || !is || !rsz || !syn || !om) goto out;

    uint16_t ni = 0, nr = 0;
    orc_select_cosets(k, r, il, is, &ni, rl, rsz, &nr);
    expand(il, ni, pos, k);
    expand(rl, nr, pos + k, r);

    if (syndromes(info, pos, k, S, syn, r)) goto out;
    locator(pos + k, r, lam);
    evaluator(syn, lam, r, S, om);

    /* _rs_get_repair_symbols (:260-286) via fft_partial_transform_cycl (fft.c:126-177):
     * evaluate Omega at alpha^(-L*2^j) per repair coset with normal-basis slots, then Forney. */
    if (!(u = seq_alloc(16, S))) goto out;
    size_t o = 0;
    for (uint16_t c = 0; c < nr; ++c) {
        uint8_t m = rsz[c];
        const uint16_t* nb = nb_of(m);
        const uint16_t* repr = g_nrepr[lg2m(m)];
        uint32_t s = ORC_N - rl[c];
        for (int t = 0; t < m; ++t) memset(u[t], 0, S);
        for (uint32_t i = 0; i < r; ++i) {
            uint16_t bits = repr[(s * i) % ORC_N];
            for (int t = 0; t < m; ++t)
                if (bits & (1u << t)) sym_xor(u[t], om[i], S);
        }
        for (int j = 0; j < m; ++j, ++o) {
            memset(rep[o], 0, S);
            for (int t = 0; t < m; ++t) sym_madd(rep[o], nb[(j + t) % m], u[t], S);
        }
    }
    for (size_t i = 0; i < r; ++i) sym_scale(rep[i], forney(lam, r, pos[k + i]), S);
    rc = 0;
out:
    seq_free(syn, r);
    seq_free(om, r);
    seq_free(u, 16);
    free(pos);
    free(lam);
    free(il);
    free(rl);
    free(is);
    free(rsz);
    return rc;
}

/* rs_restore_symbols: src/rs/reed_solomon.c:443-559 with _rs_restore_erased (:299-336):
 * t syndromes over all k+r received symbols (erased ones are zero), locator over the erased
 * positions, evaluator, then only erased INFORMATION slots are rewritten. */
int orc_decode(uint16_t k, uint16_t r, size_t S, uint8_t* const* rcv, const bool* erased, uint16_t t) {
    orc_init();
    if (r < t) return ORC_ERR_CANNOT_RESTORE;
    int rc = 1;
    size_t n = (size_t)k + r;
    uint16_t* pos = calloc(n + 1, sizeof(uint16_t));
    uint16_t* epos = calloc((size_t)t + 1, sizeof(uint16_t));
    uint16_t* lam = calloc((size_t)t + 2, sizeof(uint16_t));
    uint8_t **syn = seq_alloc(t, S), **om = seq_alloc(t, S);
    if (!pos || !epos || !lam || !syn || !om) goto out;

    orc_positions(k, r, pos);
    if (syndromes((const uint8_t* const*)rcv, pos, n, S, syn, t)) goto out;
    size_t ne = 0;
    for (size_t i = 0; i < n && ne < t; ++i)
        if (erased[i]) epos[ne++] = pos[i];
    locator(epos, t, lam);
    evaluator(syn, lam, t, S, om);

    for (uint16_t id = 0; id < k; ++id) {
        if (!erased[id]) continue;
        uint16_t p = pos[id];
        uint16_t F = forney(lam, t, p);
        uint32_t step = (ORC_N - p) % ORC_N;
        memset(rcv[id], 0, S);
        for (uint32_t i = 0; i < t; ++i)
            sym_madd(rcv[id], orc_mul(F, g_exp[((uint64_t)i * step) % ORC_N]), om[i], S);
    }
    rc = 0;
out:
    seq_free(syn, t);
    seq_free(om, t);
    free(pos);
    free(epos);
    free(lam);
    return rc;
}

int orc_encode_stripe(uint16_t k, uint16_t r, size_t S, uint8_t* stripe) {
    uint8_t** v = carve(stripe, (size_t)k + r, S);
    if (!v) return 1;
    int rc = orc_encode(k, r, S, (const uint8_t* const*)v, v + k);
    free(v);
    return rc;
}

int orc_decode_stripe(uint16_t k, uint16_t r, size_t S, uint8_t* stripe, const bool* erased, uint16_t t) {
    uint8_t** v = carve(stripe, (size_t)k + r, S);
    if (!v) return 1;
    int rc = orc_decode(k, r, S, v, erased, t);
    free(v);
    return rc;
}

/* ---------------------------------------------------------------- threaded batch (baseline) */
typedef struct {
    int dec;
    uint16_t k, r, t;
    size_t S, lo, hi;
    uint8_t* base;
    const bool* erased;
    int rc;
} job_t;

static void* run_job(void* arg) {
    job_t* j = (job_t*)arg;
    size_t stride = ((size_t)j->k + j->r) * j->S;
    j->rc = 0;
    for (size_t s = j->lo; s < j->hi && !j->rc; ++s) {
        uint8_t* st = j->base + s * stride;
        j->rc = j->dec ? orc_decode_stripe(j->k, j->r, j->S, st, j->erased, j->t)
                       : orc_encode_stripe(j->k, j->r, j->S, st);
    }
    return NULL;
}

static int run_many(int dec, uint16_t k, uint16_t r, size_t S, uint8_t* stripes, size_t n, const bool* erased,
                    uint16_t t, int nt) {
    orc_init();
    if (nt < 1) nt = 1;
    if ((size_t)nt > n) nt = (int)(n ? n : 1);
    pthread_t* th = calloc((size_t)nt, sizeof(pthread_t));
    job_t* jobs = calloc((size_t)nt, sizeof(job_t));
    if (!th || !jobs) {
        free(th);
        free(jobs);
        return 1;
    }
    for (int i = 0; i < nt; ++i) {
        jobs[i] = (job_t){dec, k, r, t, S, n * (size_t)i / nt, n * (size_t)(i + 1) / nt, stripes, erased, 0};
        pthread_create(&th[i], NULL, run_job, &jobs[i]);
    }
    int rc = 0;
    for (int i = 0; i < nt; ++i) {
        pthread_join(th[i], NULL);
        rc |= jobs[i].rc;
    }
    free(th);
    free(jobs);
    return rc;
}

int orc_encode_many(uint16_t k, uint16_t r, size_t S, uint8_t* stripes, size_t n_stripes, int n_threads) {
    return run_many(0, k, r, S, stripes, n_stripes, NULL, 0, n_threads);
}

int orc_decode_many(uint16_t k, uint16_t r, size_t S, uint8_t* stripes, size_t n_stripes, const bool* erased,
                    uint16_t t, int n_threads) {
    return run_many(1, k, r, S, stripes, n_stripes, erased, t, n_threads);
}
