/*
 * gen_golden.c -- golden-vector generator (TEST INFRASTRUCTURE, survey container only).
 *
 * Links against oracle/_ref/librs_ref.so, which oracle/Makefile builds from the reference sources
 * where they lie (/root/reference/src/rs and src/memory). It drives the reference's public
 * API exactly like its own callers (src/example.c:131-159, test/src/rs/test_random_data.c:53-89):
 * symbol_seq_t views, rs_generate_repair_symbols, erase, rs_restore_symbols.
 *
 * Usage: gen_golden <case-spec-file> <out-dir>
 * Each spec line:  name op k r S n_stripes seed t erased_csv
 *   op = encode | encode_iota | decode | decode_noncw | gmatrix | dmatrix   (codec, reed_solomon.h)
 *      | gf_add | gf_mul | gf_madd        a = stripe-0 bytes, b = stripe-1 bytes, coef = t; out: a
 *      | fft_t | fft_tc | fft_p | fft_pc  f = k symbols (stripe 0), r outputs; fft_t / fft_tc positions,
 *        fft_p components = pos_gen(seed, i); fft_pc cosets "leader:size,..." in the erased_csv field;
 *        out: the r outputs (fft_tc / fft_pc print their return code)
 * For every case it writes <out-dir>/<name>.bin (raw outputs) and prints "name rc" to stdout.
 * Inputs come from the portable counter-based generator below (mirrored in tests/ and on device).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <memory/seq.h>
#include <rs/fft.h>
#include <rs/gf65536.h>
#include <rs/reed_solomon.h>

static uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

/* byte b of the information region of stripe s (same definition as rs_amd.gen_info_bytes). */
static uint8_t gen_byte(uint64_t seed, uint64_t s, uint64_t b) {
    uint64_t q = b >> 3;
    uint64_t x = seed ^ (s * 0x9E3779B97F4A7C15ULL) ^ (q * 0xC2B2AE3D27D4EB4FULL);
    uint64_t v = mix64(x + 0x9E3779B97F4A7C15ULL);
    return (uint8_t)(v >> (8 * (b & 7)));
}

static void fill(symbol_seq_t* seq, size_t first, size_t cnt, uint64_t seed, uint64_t s) {
    size_t S = seq->symbol_size;
    for (size_t i = 0; i < cnt; ++i)
        for (size_t b = 0; b < S; ++b) seq->symbols[first + i]->data[b] = gen_byte(seed, s, i * S + b);
}

static void dump(FILE* f, const symbol_seq_t* seq, size_t first, size_t cnt) {
    for (size_t i = 0; i < cnt; ++i) fwrite(seq->symbols[first + i]->data, 1, seq->symbol_size, f);
}

/* i-th position / component of the fft cases: mix64(seed ^ (i + 1) * G) % N (tests/_util.py:pos_gen) */
static uint16_t pos_gen(uint64_t seed, uint64_t i) { return (uint16_t)(mix64(seed ^ ((i + 1) * 0x9E3779B97F4A7C15ULL)) % 65535u); }

/* the symbol-wide ops and the transforms (reference include/rs/gf65536.h:146-167, include/rs/fft.h) */
static int run_extra(RS_t* rs, const char* op, unsigned k, unsigned r, unsigned S, unsigned long long seed, unsigned t,
                     const char* ecsv, FILE* out, int* handled) {
    *handled = 1;
    if (!strncmp(op, "gf_", 3)) {
        uint8_t* a = malloc(S + 1);
        uint8_t* b = malloc(S + 1);
        for (unsigned i = 0; i < S; ++i) a[i] = gen_byte(seed, 0, i), b[i] = gen_byte(seed, 1, i);
        if (!strcmp(op, "gf_add")) gf_add(a, b, S);
        else if (!strcmp(op, "gf_mul")) gf_mul(rs->gf, a, (element_t)t, S);
        else gf_madd(rs->gf, a, (element_t)t, b, S);
        fwrite(a, 1, S, out);
        free(a);
        free(b);
        return 0;
    }
    if (strncmp(op, "fft_", 4)) {
        *handled = 0;
        return 0;
    }
    symbol_seq_t* f = seq_create(k, S);
    symbol_seq_t* res = seq_create(r, S);
    fill(f, 0, k, seed, 0);
    for (unsigned j = 0; j < r; ++j) memset(res->symbols[j]->data, 0xA5, S); /* outputs are overwritten */
    uint16_t* pos = calloc(k + r + 1, sizeof(uint16_t));
    int rc = 0;
    if (!strcmp(op, "fft_t") || !strcmp(op, "fft_tc")) {
        for (unsigned i = 0; i < k; ++i) pos[i] = pos_gen(seed, i);
        if (!strcmp(op, "fft_t")) fft_transform(rs->gf, f, pos, res);
        else rc = fft_transform_cycl(rs->gf, f, pos, res);
    } else if (!strcmp(op, "fft_p")) {
        for (unsigned j = 0; j < r; ++j) pos[j] = pos_gen(seed, j);
        fft_partial_transform(rs->gf, f, pos, res);
    } else { /* fft_pc */
        coset_t cs[4200];
        uint16_t cnt = 0;
        const char* p = ecsv;
        while (*p && cnt < 4200) {
            char* q;
            cs[cnt].leader = (uint16_t)strtoul(p, &q, 10);
            cs[cnt].size = (uint8_t)strtoul(q + 1, &q, 10);
            ++cnt;
            p = *q == ',' ? q + 1 : q;
        }
        rc = fft_partial_transform_cycl(rs->gf, f, cs, cnt, res);
    }
    dump(out, res, 0, r);
    free(pos);
    seq_destroy(f);
    seq_destroy(res);
    return rc;
}

int main(int argc, char** argv) {
    if (argc != 3) {
        fprintf(stderr, "usage: %s spec outdir\n", argv[0]);
        return 2;
    }
    FILE* spec = fopen(argv[1], "r");
    if (!spec) return 2;
    RS_t* rs = rs_create();
    char line[65536];
    while (fgets(line, sizeof line, spec)) {
        char name[256], op[32], ecsv[60000];
        unsigned k, r, S, n, t;
        unsigned long long seed;
        ecsv[0] = 0;
        if (line[0] == '#' || line[0] == '\n') continue;
        int got = sscanf(line, "%255s %31s %u %u %u %u %llu %u %59999s", name, op, &k, &r, &S, &n, &seed, &t, ecsv);
        if (got < 8) continue;
        bool* er = calloc(k + r + 1, 1);
        if (got == 9 && strcmp(ecsv, "-") != 0 && strncmp(op, "fft_", 4) != 0) {
            char* p = ecsv;
            while (*p) {
                er[strtoul(p, &p, 10)] = true;
                if (*p == ',') ++p;
            }
        }
        char path[1024];
        snprintf(path, sizeof path, "%s/%s.bin", argv[2], name);
        FILE* out = fopen(path, "wb");
        int rc = 0, handled = 0;
        rc = run_extra(rs, op, k, r, S, seed, t, ecsv, out, &handled);
        if (handled) {
            fclose(out);
            printf("%s %d\n", name, rc);
            free(er);
            continue;
        }
        for (unsigned s = 0; s < n; ++s) {
            symbol_seq_t* all = seq_create(k + r, S);
            symbol_seq_t inf = {k, S, all->symbols}, rep = {r, S, all->symbols + k};
            if (!strcmp(op, "gmatrix")) {
                /* info symbol i = unit word at column i -> rep word i of row p is G[p][i] */
                for (unsigned i = 0; i < k; ++i) all->symbols[i]->data[2 * i] = 1;
            } else if (!strcmp(op, "dmatrix")) {
                for (unsigned q = 0; q < k + r; ++q)
                    if (!er[q]) all->symbols[q]->data[2 * q] = 1;
            } else if (!strcmp(op, "encode_iota")) {
                for (unsigned i = 0; i < k; ++i)
                    for (unsigned b = 0; b < S; ++b) all->symbols[i]->data[b] = (uint8_t)(i * S + b);
            } else if (!strcmp(op, "decode_noncw")) {
                for (unsigned q = 0; q < k + r; ++q)
                    for (unsigned b = 0; b < S; ++b) all->symbols[q]->data[b] = er[q] ? 0 : gen_byte(seed, s, q * S + b);
            } else {
                fill(all, 0, k, seed, s);
            }
            if (!strcmp(op, "encode") || !strcmp(op, "encode_iota") || !strcmp(op, "gmatrix")) {
                rc = rs_generate_repair_symbols(rs, &inf, &rep);
                dump(out, all, k, r);
            } else {
                if (!strcmp(op, "decode")) {
                    rc = rs_generate_repair_symbols(rs, &inf, &rep);
                    for (unsigned q = 0; q < k + r; ++q)
                        if (er[q]) memset(all->symbols[q]->data, 0, S);
                }
                rc = rs_restore_symbols(rs, k, r, all, er, t);
                dump(out, all, 0, k + r);
            }
            seq_destroy(all);
        }
        fclose(out);
        printf("%s %d\n", name, rc);
        free(er);
    }
    rs_destroy(rs);
    fclose(spec);
    return 0;
}
