/*
 * bench_hostops.c -- per-call latency of the secondary surface (MEASUREMENT ONLY): gf_add / gf_madd
 * (reference include/rs/gf65536.h:146-167) and fft_transform_cycl (include/rs/fft.h:29-65), through
 * librs_amd.so (GPU) and, beside it on the same host, the reference compiled from its own sources
 * (oracle/_ref/librs_ref.so, CPU). Both libraries are dlopen'ed RTLD_LOCAL (they export the same names).
 * Also: aggregate gf_madd calls/s of 1 and 4 host threads on librs_amd.so (engine pool, no global lock).
 *
 *   bench_hostops <librs_amd.so> [<librs_ref.so>]      -> one JSON line per measurement
 */
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef struct {
    uint8_t* data;
} sym_t;
typedef struct {
    size_t length;
    size_t symbol_size;
    sym_t** symbols;
} seq_t;

typedef struct {
    const char* name;
    void* (*gf_create)(void);
    void (*gf_add)(void*, const void*, size_t);
    void (*gf_madd)(void*, void*, uint16_t, const void*, size_t);
    seq_t* (*seq_create)(size_t, size_t);
    void (*seq_destroy)(seq_t*);
    int (*fft_tc)(void*, const seq_t*, const uint16_t*, seq_t*);
    void* gf;
} lib_t;

static double now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static int load(lib_t* L, const char* path, const char* name) {
    void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        fprintf(stderr, "dlopen %s: %s\n", path, dlerror());
        return 1;
    }
    L->name = name;
    *(void**)&L->gf_create = dlsym(h, "gf_create");
    *(void**)&L->gf_add = dlsym(h, "gf_add");
    *(void**)&L->gf_madd = dlsym(h, "gf_madd");
    *(void**)&L->seq_create = dlsym(h, "seq_create");
    *(void**)&L->seq_destroy = dlsym(h, "seq_destroy");
    *(void**)&L->fft_tc = dlsym(h, "fft_transform_cycl");
    if (!L->gf_create || !L->gf_add || !L->gf_madd || !L->seq_create || !L->seq_destroy || !L->fft_tc) return 1;
    L->gf = L->gf_create();
    return L->gf ? 0 : 1;
}

static uint64_t sm = 0x5EED;
static uint8_t rnd8(void) {
    sm += 0x9E3779B97F4A7C15ull;
    uint64_t z = sm;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return (uint8_t)(z ^ (z >> 31));
}

/* calls until ~min_s seconds (at least 5, at most max_calls); returns seconds per call */
#define TIME_CALLS(expr, min_s, max_calls, out)                       \
    do {                                                              \
        for (int w_ = 0; w_ < 3; ++w_) { expr; }                      \
        long n_ = 0;                                                  \
        double t0_ = now(), t_ = t0_;                                 \
        while ((n_ < 5 || t_ - t0_ < (min_s)) && n_ < (max_calls)) {  \
            expr;                                                     \
            ++n_;                                                     \
            t_ = now();                                               \
        }                                                             \
        (out) = (t_ - t0_) / n_;                                      \
    } while (0)

static void symbol_ops(lib_t* L) {
    const size_t sizes[] = {16, 1024, 65536, 1 << 20};
    for (int i = 0; i < 4; ++i) {
        const size_t S = sizes[i];
        uint8_t* a = malloc(S);
        uint8_t* b = malloc(S);
        for (size_t j = 0; j < S; ++j) a[j] = rnd8(), b[j] = rnd8();
        double t_add, t_madd;
        TIME_CALLS(L->gf_add(a, b, S), 0.2, 200000, t_add);
        TIME_CALLS(L->gf_madd(L->gf, a, 31981, b, S), 0.2, 200000, t_madd);
        printf("{\"lib\": \"%s\", \"op\": \"gf_add\", \"bytes\": %zu, \"us_per_call\": %.3f, \"GBps\": %.3f}\n", L->name,
               S, t_add * 1e6, 2.0 * S / t_add / 1e9);
        printf("{\"lib\": \"%s\", \"op\": \"gf_madd\", \"bytes\": %zu, \"us_per_call\": %.3f, \"GBps\": %.3f}\n", L->name,
               S, t_madd * 1e6, 2.0 * S / t_madd / 1e9);
        fflush(stdout);
        free(a);
        free(b);
    }
}

/* the golden shapes fft_tc_small (20 inputs, 12 outputs, 64 B) and fft_tc_r1000 (1100, 1000, 32 B) */
static void transforms(lib_t* L) {
    const unsigned shapes[2][3] = {{20, 12, 64}, {1100, 1000, 32}};
    for (int sh = 0; sh < 2; ++sh) {
        const unsigned k = shapes[sh][0], r = shapes[sh][1], S = shapes[sh][2];
        seq_t* f = L->seq_create(k, S);
        seq_t* res = L->seq_create(r, S);
        uint16_t* pos = calloc(k + 1, sizeof(uint16_t));
        for (unsigned i = 0; i < k; ++i) {
            for (unsigned j = 0; j < S; ++j) f->symbols[i]->data[j] = rnd8();
            pos[i] = (uint16_t)(1 + (rnd8() | (rnd8() << 8)) % 65534);
        }
        double t;
        int rc = 0;
        TIME_CALLS(rc |= L->fft_tc(L->gf, f, pos, res), 0.3, 20000, t);
        printf("{\"lib\": \"%s\", \"op\": \"fft_transform_cycl\", \"k\": %u, \"r\": %u, \"bytes\": %u, \"us_per_call\": %.3f, "
               "\"rc\": %d}\n",
               L->name, k, r, S, t * 1e6, rc);
        fflush(stdout);
        free(pos);
        L->seq_destroy(f);
        L->seq_destroy(res);
    }
}

typedef struct {
    lib_t* L;
    size_t S;
    double secs;
    long calls;
} thr_t;

static void* madd_loop(void* p) {
    thr_t* a = p;
    uint8_t* x = malloc(a->S);
    uint8_t* y = malloc(a->S);
    memset(x, 1, a->S);
    memset(y, 2, a->S);
    double t0 = now();
    long n = 0;
    while (now() - t0 < a->secs) {
        a->L->gf_madd(a->L->gf, x, 4660, y, a->S);
        ++n;
    }
    a->calls = n;
    free(x);
    free(y);
    return NULL;
}

static void concurrency(lib_t* L) {
    const size_t S = 65536;
    for (int nt = 1; nt <= 4; nt *= 4) {
        pthread_t th[4];
        thr_t a[4];
        for (int i = 0; i < nt; ++i) {
            a[i] = (thr_t){L, S, 0.5, 0};
            pthread_create(&th[i], NULL, madd_loop, &a[i]);
        }
        long total = 0;
        for (int i = 0; i < nt; ++i) pthread_join(th[i], NULL), total += a[i].calls;
        printf("{\"lib\": \"%s\", \"op\": \"gf_madd_threads\", \"bytes\": %zu, \"threads\": %d, \"calls_per_s\": %.0f}\n",
               L->name, S, nt, total / 0.5);
        fflush(stdout);
    }
}

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s librs_amd.so [librs_ref.so]\n", argv[0]);
        return 2;
    }
    lib_t libs[2];
    int nl = 0;
    if (load(&libs[nl], argv[1], "rs_amd")) return 1;
    ++nl;
    if (argc > 2 && !load(&libs[nl], argv[2], "reference")) ++nl;
    for (int i = 0; i < nl; ++i) {
        symbol_ops(&libs[i]);
        transforms(&libs[i]);
    }
    concurrency(&libs[0]);
    return 0;
}
