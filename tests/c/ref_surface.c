/*
 * ref_surface.c -- calls every function the reference declares in its include/rs/ and
 * include/memory/ headers, built against THIS repo's headers and linked against librs_amd.so (the
 * drop-in check of the boundary). Writes the outputs of a set of golden cases to <outdir>/<name>.bin;
 * tests/test_gpu.py compares them with tests/golden/. Inputs are regenerated with the fixtures'
 * portable generator (oracle/gen_golden.c:gen_byte / pos_gen).
 *
 * The codec part follows the reference's own callers, so their coverage does not depend on the
 * reference's compiled programs (which never travel to the GPU box): src/example.c (a k + r sequence
 * from seq_create, information / repair views into it, a received copy, erase, restore, seq_eq) on the
 * ex_* fixtures and the C3-shape c3_* fixtures, and test/src/rs/test_random_data.c's 100 rounds of
 * random (k, r, t) round trips over 16-byte symbols (self-checked with seq_eq on the information view).
 *
 * Usage: ref_surface <outdir>
 */
#include <stdbool.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <memory/seq.h>
#include <memory/symbol.h>
#include <rs/cyclotomic_coset.h>
#include <rs/fft.h>
#include <rs/gf65536.h>
#include <rs/prelude.h>
#include <rs/reed_solomon.h>
#include <util/util.h>

#define SEED 0x5EEDull

static uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static uint8_t gen_byte(uint64_t seed, uint64_t s, uint64_t b) {
    uint64_t x = seed ^ (s * 0x9E3779B97F4A7C15ULL) ^ ((b >> 3) * 0xC2B2AE3D27D4EB4FULL);
    return (uint8_t)(mix64(x + 0x9E3779B97F4A7C15ULL) >> (8 * (b & 7)));
}
static uint16_t pos_gen(uint64_t seed, uint64_t i) { return (uint16_t)(mix64(seed ^ ((i + 1) * 0x9E3779B97F4A7C15ULL)) % 65535u); }

static const char* outdir;
static int failures;

static void save(const char* name, const symbol_seq_t* q, size_t first, size_t cnt) {
    char path[1024];
    snprintf(path, sizeof path, "%s/%s.bin", outdir, name);
    FILE* f = fopen(path, "wb");
    for (size_t i = 0; i < cnt; ++i) fwrite(q->symbols[first + i]->data, 1, q->symbol_size, f);
    fclose(f);
}
static void save_raw(const char* name, const void* p, size_t n) {
    char path[1024];
    snprintf(path, sizeof path, "%s/%s.bin", outdir, name);
    FILE* f = fopen(path, "wb");
    fwrite(p, 1, n, f);
    fclose(f);
}
static void check(int ok, const char* what) {
    if (!ok) {
        fprintf(stderr, "FAIL: %s\n", what);
        ++failures;
    }
}
static symbol_seq_t* gen_seq(size_t len, size_t S, uint64_t stripe) {
    symbol_seq_t* q = seq_create(len, S);
    for (size_t i = 0; i < len; ++i)
        for (size_t b = 0; b < S; ++b) q->symbols[i]->data[b] = gen_byte(SEED, stripe, i * S + b);
    return q;
}

/* src/example.c's call pattern on one golden case: per stripe, encode through views into a seq_create
 * sequence, then (decode cases) copy to a received sequence, zero the erased slots, restore, and check
 * the information symbols with seq_eq. Writes the repair rows (encode) or whole stripes (decode). */
static void codec_case(RS_t* rs, const char* name, uint16_t k, uint16_t r, size_t S, int n, const uint16_t* erased,
                       uint16_t t, int decode) {
    const size_t rows = decode ? (size_t)(k + r) : r;
    uint8_t* out = malloc((size_t)n * rows * S);
    bool* is_erased = calloc(k + r, sizeof(bool));
    for (uint16_t e = 0; e < t; ++e) is_erased[erased[e]] = true;
    for (int s = 0; s < n; ++s) {
        symbol_seq_t* src = seq_create(k + r, S);
        for (size_t i = 0; i < k; ++i)
            for (size_t b = 0; b < S; ++b) src->symbols[i]->data[b] = gen_byte(SEED, (uint64_t)s, i * S + b);
        symbol_seq_t inf = {k, S, src->symbols}, rep = {r, S, src->symbols + k};
        check(rs_generate_repair_symbols(rs, &inf, &rep) == 0, name);
        if (!decode) {
            for (size_t j = 0; j < r; ++j) memcpy(out + ((size_t)s * rows + j) * S, rep.symbols[j]->data, S);
        } else {
            symbol_seq_t* rcv = seq_create(k + r, S);
            for (size_t i = 0; i < (size_t)(k + r); ++i) memcpy(rcv->symbols[i]->data, src->symbols[i]->data, S);
            for (size_t i = 0; i < (size_t)(k + r); ++i)
                if (is_erased[i]) memset(rcv->symbols[i]->data, 0, S);
            check(t == 0 || !seq_eq(src, rcv), name);
            check(rs_restore_symbols(rs, k, r, rcv, is_erased, t) == 0, name);
            symbol_seq_t rinf = {k, S, rcv->symbols};
            check((S & 1) || seq_eq(&inf, &rinf), name);  /* odd S: restored symbols end in 0 (reference) */
            for (size_t i = 0; i < rows; ++i) memcpy(out + ((size_t)s * rows + i) * S, rcv->symbols[i]->data, S);
            seq_destroy(rcv);
        }
        seq_destroy(src);
    }
    save_raw(name, out, (size_t)n * rows * S);
    free(is_erased);
    free(out);
}

/* test/src/rs/test_random_data.c's call pattern: 100 rounds, symbol size 16, k in [100, 200), r in
 * [50, 100), t erasures anywhere (half the rounds t in [11, r), half t = r); each round encodes through
 * views into one sequence, erases a random set in a received copy, restores, and compares the
 * information views with seq_eq. The random choices come from splitmix, not libc rand(). */
static void random_data_rounds(RS_t* rs) {
    uint64_t st = 234546127u;
    for (int round = 0; round < 100; ++round) {
        const uint16_t k = (uint16_t)(100 + mix64(++st) % 100), r = (uint16_t)(50 + mix64(++st) % 50);
        const uint16_t t = round < 50 ? (uint16_t)(11 + mix64(++st) % (uint64_t)(r - 10)) : r;
        const size_t S = 16;
        symbol_seq_t* src = seq_create(k + r, S);
        symbol_seq_t* rcv = seq_create(k + r, S);
        bool* is_erased = calloc(k + r, sizeof(bool));
        for (size_t i = 0; i < k; ++i)
            for (size_t b = 0; b < S; ++b) src->symbols[i]->data[b] = (uint8_t)(mix64(++st) >> 24);
        symbol_seq_t inf = {k, S, src->symbols}, rep = {r, S, src->symbols + k}, rinf = {k, S, rcv->symbols};
        check(rs_generate_repair_symbols(rs, &inf, &rep) == 0, "random_data encode");
        for (size_t i = 0; i < (size_t)(k + r); ++i) memcpy(rcv->symbols[i]->data, src->symbols[i]->data, S);
        for (uint16_t e = 0; e < t;) {
            const size_t i = mix64(++st) % (uint64_t)(k + r);
            if (is_erased[i]) continue;
            is_erased[i] = true;
            memset(rcv->symbols[i]->data, 0, S);
            ++e;
        }
        check(!seq_eq(src, rcv), "random_data erase");
        check(rs_restore_symbols(rs, k, r, rcv, is_erased, t) == 0, "random_data restore");
        check(seq_eq(&inf, &rinf), "random_data inf_symbols == rcv_inf_symbols");
        free(is_erased);
        seq_destroy(rcv);
        seq_destroy(src);
    }
}

int main(int argc, char** argv) {
    if (argc != 2) return 2;
    outdir = argv[1];
    GF_t* gf = gf_create();
    CC_t* cc = cc_create();
    check(gf && cc, "gf_create / cc_create");
    /* scalar helpers (reference test/src/rs/gf65536 KATs) */
    check(gf_mul_ee(gf, 31981, 38739) == 42167, "gf_mul_ee");
    check(gf_div_ee(gf, 12320, 29623) == 11439, "gf_div_ee");
    check(gf_get_normal_basis_element(gf, 4, 0) == 10800, "gf_get_normal_basis_element");
    check(gf_get_normal_repr(gf, 16, gf->log_table[gf_get_normal_basis_element(gf, 16, 3)]) == (1u << 3),
          "gf_get_normal_repr");
    check(gf->normal_repr_by_subfield[16] == gf->_normal_repr_by_subfield_memory + 4 * N &&
              gf->normal_repr_by_subfield[3] == NULL && gf->normal_repr_by_subfield[1][0] == 1,
          "GF_t normal_repr_by_subfield");
    check(MIN(3, 5) == 3, "util MIN");
    /* cosets (reference test/src/rs/cyclotomic_coset KATs) */
    check(cc_get_coset_size(0) == 1 && cc_get_coset_size(21845) == 2 && cc_get_coset_size(1) == 16, "cc_get_coset_size");
    uint16_t imax = 0, rmax = 0, icnt = 0, rcnt = 0;
    cc_estimate_cosets_cnt(16, 3, &imax, &rmax);
    coset_t* ic = calloc(imax, sizeof(coset_t));
    coset_t* rc = calloc(rmax, sizeof(coset_t));
    cc_select_cosets(cc, 16, 3, ic, imax, &icnt, rc, rmax, &rcnt);
    uint16_t pos[19];
    cc_cosets_to_positions(rc, rcnt, pos, 3);
    check(rcnt == 2 && pos[0] == 21845 && pos[1] == 43690 && pos[2] == 0, "cc_select_cosets / cc_cosets_to_positions");
    free(ic);
    free(rc);
    /* symbol-wide ops: golden cases gf_add_64, gf_mul_c, gf_madd_c */
    {
        symbol_t* a = symbol_create(256);
        symbol_t* b = symbol_create(256);
        for (int i = 0; i < 256; ++i) a->data[i] = gen_byte(SEED, 0, i), b->data[i] = gen_byte(SEED, 1, i);
        gf_add(a->data, b->data, 64);
        save_raw("gf_add_64", a->data, 64);
        for (int i = 0; i < 256; ++i) a->data[i] = gen_byte(SEED, 0, i);
        gf_mul(gf, a->data, 31981, 256);
        save_raw("gf_mul_c", a->data, 256);
        for (int i = 0; i < 256; ++i) a->data[i] = gen_byte(SEED, 0, i);
        gf_madd(gf, a->data, 12345, b->data, 256);
        save_raw("gf_madd_c", a->data, 256);
        check(!symbol_eq(a, b, 256), "symbol_eq");
        symbol_printf(b, 0);
        symbol_destroy(a);
        symbol_destroy(b);
    }
    /* transforms: fft_t_small, fft_tc_small (k = 20, r = 12), fft_p_small (16, 10), fft_pc_mixed (40) */
    {
        symbol_seq_t* f = gen_seq(20, 64, 0);
        symbol_seq_t* res = seq_create(12, 64);
        uint16_t p[40];
        for (int i = 0; i < 20; ++i) p[i] = pos_gen(SEED, (uint64_t)i);
        fft_transform(gf, f, p, res);
        save("fft_t_small", res, 0, 12);
        check(fft_transform_cycl(gf, f, p, res) == 0, "fft_transform_cycl rc");
        save("fft_tc_small", res, 0, 12);
        seq_destroy(f);
        seq_destroy(res);
        f = gen_seq(16, 64, 0);
        res = seq_create(10, 64);
        for (int j = 0; j < 10; ++j) p[j] = pos_gen(SEED, (uint64_t)j);
        fft_partial_transform(gf, f, p, res);
        save("fft_p_small", res, 0, 10);
        seq_destroy(f);
        seq_destroy(res);
        const coset_t cs[6] = {{0, 1}, {21845, 2}, {4369, 4}, {257, 8}, {1, 16}, {3, 16}};
        f = gen_seq(40, 64, 0);
        res = seq_create(47, 64);
        check(fft_partial_transform_cycl(gf, f, cs, 6, res) == 0, "fft_partial_transform_cycl rc");
        save("fft_pc_mixed", res, 0, 47);
        seq_destroy(f);
        seq_destroy(res);
    }
    /* codec: c1_enc (k = 4, r = 2, 256 B) and c1_dec_info_rep (erase info 1 and repair 0) */
    {
        RS_t* rs = rs_create();
        check(rs != NULL, "rs_create");
        symbol_seq_t* all = seq_create(6, 256);
        for (int i = 0; i < 4; ++i)
            for (int b = 0; b < 256; ++b) all->symbols[i]->data[b] = gen_byte(SEED, 0, (uint64_t)(i * 256 + b));
        symbol_seq_t inf = {4, 256, all->symbols}, rep = {2, 256, all->symbols + 4};
        check(rs_generate_repair_symbols(rs, &inf, &rep) == 0, "rs_generate_repair_symbols");
        save("c1_enc", all, 4, 2);
        symbol_seq_t* kept = seq_create(6, 256);
        for (int i = 0; i < 6; ++i) memcpy(kept->symbols[i]->data, all->symbols[i]->data, 256);
        bool er[6] = {false, true, false, false, true, false};
        memset(all->symbols[1]->data, 0, 256);
        memset(all->symbols[4]->data, 0, 256);
        check(rs_restore_symbols(rs, 4, 2, all, er, 2) == 0, "rs_restore_symbols");
        save("c1_dec_info_rep", all, 0, 6);
        check(symbol_eq(all->symbols[1], kept->symbols[1], 256) && !seq_eq(all, kept), "restore / seq_eq");
        check(rs_restore_symbols(rs, 4, 2, all, er, 3) == RS_ERR_CANNOT_RESTORE, "RS_ERR_CANNOT_RESTORE");
        symbol_seq_t* tiny = seq_create(1, 2);
        seq_printf(tiny);
        printf("\n");
        seq_destroy(tiny);
        seq_destroy(kept);
        seq_destroy(all);
        /* src/example.c on its golden pair, the C3-shape fixtures, then test_random_data.c's rounds */
        const uint16_t ex_er[10] = {2, 8, 11, 13, 19, 30, 38, 50, 61, 92};
        codec_case(rs, "ex_enc", 100, 10, 10, 1, NULL, 0, 0);
        codec_case(rs, "ex_dec", 100, 10, 10, 1, ex_er, 10, 1);
        uint16_t bench[32];
        for (int i = 0; i < 32; ++i) bench[i] = (uint16_t)(4 * i);
        const uint16_t rand17[17] = {0, 7, 16, 24, 30, 34, 53, 65, 97, 99, 110, 115, 120, 124, 126, 145, 155};
        codec_case(rs, "c3_enc", 128, 32, 512, 2, NULL, 0, 0);
        codec_case(rs, "c3_dec_bench", 128, 32, 512, 2, bench, 32, 1);
        codec_case(rs, "c3_dec_rand17", 128, 32, 512, 1, rand17, 17, 1);
        /* odd symbol sizes: the reference's Release semantics (even prefix coded, written symbols end in 0) */
        const uint16_t odd9[2] = {1, 4}, odd4097[4] = {0, 3, 7, 12};
        codec_case(rs, "odd_enc_9", 4, 2, 9, 1, NULL, 0, 0);
        codec_case(rs, "odd_dec_9", 4, 2, 9, 1, odd9, 2, 1);
        codec_case(rs, "odd_enc_4097", 10, 4, 4097, 2, NULL, 0, 0);
        codec_case(rs, "odd_dec_4097", 10, 4, 4097, 2, odd4097, 4, 1);
        random_data_rounds(rs);
        rs_destroy(rs);
    }
    cc_destroy(cc);
    gf_destroy(gf);
    printf("%s (%d failures)\n", failures ? "FAILED" : "ok", failures);
    return failures ? 1 : 0;
}
