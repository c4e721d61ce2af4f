/*
 * cpu_baseline.c -- the CPU baseline leg of bench.py (TEST / MEASUREMENT INFRASTRUCTURE ONLY).
 *
 * Times the reference's CPU path over resident stripes on a pthread pool, the way SURVEY.md 8(d)
 * asks: one codec context per thread, stripes statically partitioned, CLOCK_MONOTONIC around the
 * coding calls only (symbol_t / symbol_seq_t views are built before the clock starts; erased slots
 * are re-zeroed between decode passes outside the timed region, as the reference requires,
 * reference include/rs/reed_solomon.h:64).
 *
 * The library is loaded with dlopen so one driver serves both kinds:
 *   kind 0 "reference": oracle/_ref/librs_ref.so -- the reference src/rs + src/memory compiled from
 *          /root/reference by oracle/Makefile; rs_create / rs_generate_repair_symbols /
 *          rs_restore_symbols (reference include/rs/reed_solomon.h:44,61,74).
 *   kind 1 "port":      oracle/librs_oracle.so -- the clean-room restatement (orc_encode / orc_decode).
 * Nothing here is linked into, or called by, the product library librs_amd.so.
 */

#include <dlfcn.h>
#include <pthread.h>
#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef struct {
    uint8_t* data;
} sym_t; /* reference include/memory/symbol.h:20-25 */

typedef struct {
    size_t length;
    size_t symbol_size;
    sym_t** symbols;
} seq_t; /* reference include/memory/seq.h:21-36 */

typedef void* (*rs_create_f)(void);
typedef void (*rs_destroy_f)(void*);
typedef int (*rs_enc_f)(void*, const seq_t*, seq_t*);
typedef int (*rs_dec_f)(void*, uint16_t, uint16_t, seq_t*, const bool*, uint16_t);
typedef int (*orc_init_f)(void);
typedef int (*orc_enc_f)(uint16_t, uint16_t, size_t, const uint8_t* const*, uint8_t* const*);
typedef int (*orc_dec_f)(uint16_t, uint16_t, size_t, uint8_t* const*, const bool*, uint16_t);

typedef struct {
    int kind;
    rs_create_f rs_create;
    rs_destroy_f rs_destroy;
    rs_enc_f rs_enc;
    rs_dec_f rs_dec;
    orc_enc_f orc_enc;
    orc_dec_f orc_dec;
} api_t;

typedef struct {
    const api_t* api;
    int k, r, t, op, passes, tid, nthreads;
    size_t S, n;
    uint8_t* stripes;
    const bool* erased;
    pthread_barrier_t* bar;
    double* seconds; /* thread 0 writes the summed timed seconds */
    int rc;
} job_t;

static double now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void* worker(void* p) {
    job_t* j = (job_t*)p;
    const size_t n_sym = (size_t)j->k + (size_t)j->r, stride = n_sym * j->S;
    const size_t lo = j->n * (size_t)j->tid / (size_t)j->nthreads, hi = j->n * (size_t)(j->tid + 1) / (size_t)j->nthreads;
    const size_t cnt = hi - lo;
    /* views of this thread's stripes, built before any timing */
    sym_t* syms = calloc(cnt * n_sym + 1, sizeof(sym_t));
    sym_t** sp = calloc(cnt * n_sym + 1, sizeof(sym_t*));
    uint8_t** raw = calloc(cnt * n_sym + 1, sizeof(uint8_t*));
    void* ctx = NULL;
    int rc = (!syms || !sp || !raw) ? 1 : 0;
    if (!rc && j->api->kind == 0 && !(ctx = j->api->rs_create())) rc = 1;
    for (size_t s = 0; !rc && s < cnt; ++s)
        for (size_t i = 0; i < n_sym; ++i) {
            uint8_t* d = j->stripes + (lo + s) * stride + i * j->S;
            syms[s * n_sym + i].data = d;
            sp[s * n_sym + i] = &syms[s * n_sym + i];
            raw[s * n_sym + i] = d;
        }
    double total = 0.0;
    for (int pass = 0; pass < j->passes; ++pass) {
        if (j->op == 1 && !rc) /* the reference requires erased slots to be zero on entry (untimed) */
            for (size_t s = 0; s < cnt; ++s)
                for (size_t i = 0; i < n_sym; ++i)
                    if (j->erased[i]) memset(raw[s * n_sym + i], 0, j->S);
        pthread_barrier_wait(j->bar);
        const double t0 = now();
        for (size_t s = 0; !rc && s < cnt; ++s) {
            sym_t** st = sp + s * n_sym;
            if (j->api->kind == 0) {
                if (j->op == 0) {
                    seq_t inf = {(size_t)j->k, j->S, st}, rep = {(size_t)j->r, j->S, st + j->k};
                    rc = j->api->rs_enc(ctx, &inf, &rep);
                } else {
                    seq_t rcv = {n_sym, j->S, st};
                    rc = j->api->rs_dec(ctx, (uint16_t)j->k, (uint16_t)j->r, &rcv, j->erased, (uint16_t)j->t);
                }
            } else {
                uint8_t** rw = raw + s * n_sym;
                rc = j->op == 0 ? j->api->orc_enc((uint16_t)j->k, (uint16_t)j->r, j->S, (const uint8_t* const*)rw, rw + j->k)
                                : j->api->orc_dec((uint16_t)j->k, (uint16_t)j->r, j->S, rw, j->erased, (uint16_t)j->t);
            }
        }
        pthread_barrier_wait(j->bar);
        total += now() - t0;
    }
    if (j->tid == 0) *j->seconds = total;
    if (ctx) j->api->rs_destroy(ctx);
    free(syms);
    free(sp);
    free(raw);
    j->rc = rc;
    return NULL;
}

/* Runs `passes` encode (op 0) or decode (op 1) passes over n contiguous stripes ([k + r][S] bytes
 * each) on `threads` pthreads with the library at lib_path (kind 0 reference, 1 port).
 * *seconds = summed wall time of the timed regions. Returns 0, or the first nonzero library /
 * setup code (-1: library or symbol not found). */
int cpub_run(const char* lib_path, int kind, int k, int r, size_t S, uint8_t* stripes, size_t n, const bool* erased,
             int t, int op, int passes, int threads, double* seconds) {
    void* h = dlopen(lib_path, RTLD_NOW | RTLD_LOCAL);
    if (!h) return -1;
    api_t api = {0};
    api.kind = kind;
    if (kind == 0) {
        api.rs_create = (rs_create_f)dlsym(h, "rs_create");
        api.rs_destroy = (rs_destroy_f)dlsym(h, "rs_destroy");
        api.rs_enc = (rs_enc_f)dlsym(h, "rs_generate_repair_symbols");
        api.rs_dec = (rs_dec_f)dlsym(h, "rs_restore_symbols");
        if (!api.rs_create || !api.rs_destroy || !api.rs_enc || !api.rs_dec) return -1;
    } else {
        orc_init_f init = (orc_init_f)dlsym(h, "orc_init");
        api.orc_enc = (orc_enc_f)dlsym(h, "orc_encode");
        api.orc_dec = (orc_dec_f)dlsym(h, "orc_decode");
        if (!init || !api.orc_enc || !api.orc_dec) return -1;
        init();
    }
    if (threads < 1) threads = 1;
    if ((size_t)threads > n && n > 0) threads = (int)n;
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, NULL, (unsigned)threads);
    job_t* jobs = calloc((size_t)threads, sizeof(job_t));
    pthread_t* th = calloc((size_t)threads, sizeof(pthread_t));
    if (!jobs || !th) return 1;
    *seconds = 0.0;
    for (int i = 0; i < threads; ++i) {
        jobs[i] = (job_t){&api, k, r, t, op, passes, i, threads, S, n, stripes, erased, &bar, seconds, 0};
        pthread_create(&th[i], NULL, worker, &jobs[i]);
    }
    int rc = 0;
    for (int i = 0; i < threads; ++i) {
        pthread_join(th[i], NULL);
        if (jobs[i].rc && !rc) rc = jobs[i].rc;
    }
    pthread_barrier_destroy(&bar);
    free(jobs);
    free(th);
    return rc;
}
