/*
 * oracle_reduce.c -- CPU restatement of the reduce-to-all schedule and the
 * timed CPU baseline.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Restates udr_<T>_to_all, src/reductions.c:32-120:
 *   :40      me = shmem_my_pe()
 *   :79-81   write_to[j] = source[j]                (everyone initialises)
 *   :82      barrier
 *   :84-111  pe = PE_start; for i < PE_size: if pe != me, pull the peer's
 *            whole source in SHMEM_REDUCE_MIN_WRKDATA_SIZE (= 64, defs.h:91)
 *            element chunks into pWrk (:90-100) plus a remainder (:102-108),
 *            folding write_to[ti] = op(write_to[ti], pWrk[j]); pe += 1<<stride
 *   :113     barrier
 *   :114-119 copy the temporary target back when target/source overlap
 * Element i of PE me's target is therefore
 *   op(...op(op(src_me[i], src_{PE_start}[i]), src_{PE_start+s}[i])..., ...)
 * with `me` skipped in the ascending walk.  Because peers only ever read
 * `source`, and an overlapping target is staged in a temporary until after
 * the second barrier, the team result equals this per-PE fold evaluated
 * sequentially -- which is what oracle_to_all does.
 *
 * oracle_cpu_baseline keeps the reference's loop shape instead (pthreads as
 * PEs, memcpy getmem from the peer's slot of an in-process heap, 64-element
 * chunks, per-element call through a function pointer); with
 * oracle_cpu_baseline_ref that pointer is the reference's own compiled
 * element function (oracle/_ref).
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <pthread.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define WRK 64 /* SHMEM_REDUCE_MIN_WRKDATA_SIZE, include/shmem/defs.h:91 */

int oracle_to_all(int type, int op, int npes, int PE_start, int logPE_stride,
                  int PE_size, const void *const *sources, void *const *targets,
                  int nreduce)
{
    if (!oracle_has_op(type, op) || npes <= 0 || PE_size <= 0 || PE_start < 0 ||
        logPE_stride < 0 || logPE_stride > 30)
        return -1;
    const int step = 1 << logPE_stride;
    if ((long) PE_start + (long) (PE_size - 1) * step >= npes) return -1;
    if (nreduce <= 0) return 0; /* only the two barriers happen */
    const size_t s = oracle_type_size(type);
    const size_t nbytes = s * (size_t) nreduce;
    /* stage every result first: a target may alias another PE's source in
       this single-address-space restatement only if the caller says so; the
       reference's own temp-target rule (:52-69,:114-119) makes in-place safe */
    void **tmp = calloc((size_t) PE_size, sizeof(void *));
    if (!tmp) return -1;
    int rc = 0;
    for (int k = 0; k < PE_size && rc == 0; k++) {
        const int me = PE_start + k * step;
        tmp[k] = malloc(nbytes);
        if (!tmp[k]) { rc = -1; break; }
        memcpy(tmp[k], sources[me], nbytes); /* :79-81 */
        for (int i = 0, pe = PE_start; i < PE_size; i++, pe += step) { /* :84-111 */
            if (pe == me) continue;
            rc = oracle_op(type, op, tmp[k], sources[pe], tmp[k], (size_t) nreduce);
            if (rc) break;
        }
    }
    for (int k = 0; k < PE_size; k++) {
        if (rc == 0) memcpy(targets[PE_start + k * step], tmp[k], nbytes);
        free(tmp[k]);
    }
    free(tmp);
    return rc;
}

/* ------------------------------------------------------------------------ */
/* CPU baseline: reference loop shape, pthreads as PEs                       */
/* ------------------------------------------------------------------------ */

typedef void (*elem_fn)(void *acc, const void *in); /* acc = op(acc, in) */

#define DEF_ELEM(NAME, T, EXPR)                                                \
    static void NAME(void *acc, const void *in)                                \
    {                                                                          \
        T a = *(T *) acc, b = *(const T *) in;                                 \
        *(T *) acc = (EXPR);                                                   \
    }
/* the baseline times the loop, not the NaN model: plain C ops, like the
   reference's one-liners */
DEF_ELEM(e_sum_d, double, a + b)
DEF_ELEM(e_prod_d, double, a * b)
DEF_ELEM(e_max_d, double, a > b ? a : b)
DEF_ELEM(e_min_d, double, a < b ? a : b)
DEF_ELEM(e_sum_f, float, a + b)
DEF_ELEM(e_prod_f, float, a * b)
DEF_ELEM(e_max_f, float, a > b ? a : b)
DEF_ELEM(e_min_f, float, a < b ? a : b)
DEF_ELEM(e_sum_i, int, (int) ((unsigned) a + (unsigned) b))
DEF_ELEM(e_sum_l, long, (long) ((unsigned long) a + (unsigned long) b))
DEF_ELEM(e_and_l, long, a & b)
DEF_ELEM(e_or_l, long, a | b)
DEF_ELEM(e_xor_l, long, a ^ b)

static elem_fn pick_elem(int type, int op)
{
    switch (type) {
    case OR_DOUBLE:
        return op == OR_SUM ? e_sum_d : op == OR_PROD ? e_prod_d : op == OR_MAX ? e_max_d
             : op == OR_MIN ? e_min_d : NULL;
    case OR_FLOAT:
        return op == OR_SUM ? e_sum_f : op == OR_PROD ? e_prod_f : op == OR_MAX ? e_max_f
             : op == OR_MIN ? e_min_f : NULL;
    case OR_INT:
        return op == OR_SUM ? e_sum_i : NULL;
    case OR_LONG: case OR_LONGLONG:
        return op == OR_SUM ? e_sum_l : op == OR_AND ? e_and_l : op == OR_OR ? e_or_l
             : op == OR_XOR ? e_xor_l : NULL;
    }
    return NULL;
}

/* The reference's own element function (src/shmemu/miscops.c:12-105,
   compiled unmodified into oracle/_ref/libref_ops.so), called by value
   through a pointer exactly as src/reductions.c:95-96 does:
   write_to[ti] = (*the_op)(write_to[ti], pWrk[j]).  One loop per C type. */
#define REF_FOLD(T)                                                            \
    do {                                                                       \
        T (*f)(T, T) = (T (*)(T, T)) t->ref_fn;                                \
        T *w = (T *) dst + ti0;                                                \
        const T *p = (const T *) pw;                                           \
        for (size_t j = 0; j < cnt; j++) w[j] = (*f)(w[j], p[j]);              \
    } while (0)

typedef struct {
    int type, npes, nreduce, reps, pin, tpp;  /* tpp: threads per PE */
    void *ref_fn;                             /* reference element fn, or NULL */
    int *cpus;                                /* thread i pinned to cpus[i] */
    size_t s;
    elem_fn fn;
    const void *const *sources;
    void *const *targets;
    pthread_barrier_t bar;
    double *times; /* [reps+1] written by PE 0 */
} bl_team;

typedef struct {
    bl_team *t;
    int me, part;  /* PE, and which of its tpp element ranges */
} bl_arg;

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double) ts.tv_sec + 1e-9 * (double) ts.tv_nsec;
}

/* One thread of PE `me`: with tpp = 1 the whole loop of src/reductions.c
   :79-113; with tpp > 1 PE me's loop is split over tpp threads, each running
   the same shape (copy, barrier, 64-element getmem chunks, indirect op,
   barrier) over a contiguous 1/tpp of the elements -- the reference's
   algorithm on npes * tpp cores. */
/* the k-th CPU this process may run on (its affinity mask, e.g. a
   container's CPU share), so pinned threads land on allowed cores */
static int allowed_cpu(int k)
{
    cpu_set_t cs;
    CPU_ZERO(&cs);
    if (sched_getaffinity(0, sizeof(cs), &cs) != 0 || CPU_COUNT(&cs) == 0) return k % CPU_SETSIZE;
    k %= CPU_COUNT(&cs);
    for (int c = 0; c < CPU_SETSIZE; c++)
        if (CPU_ISSET(c, &cs) && k-- == 0) return c;
    return 0;
}

static void *bl_pe(void *p)
{
    bl_arg *ar = (bl_arg *) p;
    bl_team *t = ar->t;
    const int me = ar->me;
    if (t->pin) {
        cpu_set_t cs;
        CPU_ZERO(&cs);
        CPU_SET(t->cpus[me * t->tpp + ar->part], &cs);
        pthread_setaffinity_np(pthread_self(), sizeof(cs), &cs);
    }
    const size_t s = t->s;
    const size_t lo = (size_t) t->nreduce * (size_t) ar->part / (size_t) t->tpp;
    const size_t hi = (size_t) t->nreduce * (size_t) (ar->part + 1) / (size_t) t->tpp;
    const size_t n = hi - lo, nloops = n / WRK, nrem = n % WRK;
    char *src = (char *) t->sources[me] + lo * s;
    char *dst = (char *) t->targets[me] + lo * s;
    char *pwrk = malloc(WRK * s);
    /* first touch of target by its PE */
    memset(dst, 0, n * s);
    for (int r = 0; r <= t->reps; r++) {
        pthread_barrier_wait(&t->bar);
        double t0 = now_s();
        memcpy(dst, src, n * s);                      /* :79-81 */
        pthread_barrier_wait(&t->bar);                /* :82 */
        for (int pe = 0; pe < t->npes; pe++) {        /* :84-111 */
            if (pe == me) continue;
            const char *peer = (const char *) t->sources[pe] + lo * s; /* same offset */
            size_t ti = 0, si = 0;
            for (size_t k = 0; k <= nloops; k++) {
                const size_t cnt = k < nloops ? WRK : nrem;
                memcpy(pwrk, peer + si * s, cnt * s); /* shmem_getmem :92, :103 */
                if (t->ref_fn) {                      /* :95-96, the reference's op */
                    const size_t ti0 = ti;
                    const char *pw = pwrk;
                    switch (t->type) {
                    case OR_DOUBLE: REF_FOLD(double); break;
                    case OR_FLOAT: REF_FOLD(float); break;
                    case OR_INT: REF_FOLD(int); break;
                    default: REF_FOLD(long); break;    /* long, long long */
                    }
                    ti += cnt;
                } else {
                    for (size_t j = 0; j < cnt; j++, ti++)
                        t->fn(dst + ti * s, pwrk + j * s);
                }
                si += cnt;
            }
        }
        pthread_barrier_wait(&t->bar);                /* :113 */
        if (me == 0 && ar->part == 0) t->times[r] = now_s() - t0;
    }
    free(pwrk);
    return NULL;
}

static int cmp_d(const void *a, const void *b)
{
    double x = *(const double *) a, y = *(const double *) b;
    return x < y ? -1 : x > y;
}

/* the reference loop shape with npes * tpp pthreads (tpp per PE, pinned to
   cores 0 .. npes*tpp-1 when pin_cores); median seconds per call */
double oracle_cpu_baseline_ref(int type, int op, int npes, const void *const *sources,
                               void *const *targets, int nreduce, int reps, int pin_cores,
                               int tpp, void *ref_fn)
{
    elem_fn fn = pick_elem(type, op);
    if (!fn || npes < 1 || reps < 1 || nreduce < 0 || tpp < 1) return -1.0;
    if (ref_fn && type != OR_DOUBLE && type != OR_FLOAT && type != OR_INT &&
        type != OR_LONG && type != OR_LONGLONG)
        return -1.0;
    bl_team t;
    memset(&t, 0, sizeof(t));
    t.ref_fn = ref_fn;
    t.type = type; t.npes = npes; t.nreduce = nreduce; t.reps = reps; t.pin = pin_cores;
    t.tpp = tpp;
    t.s = oracle_type_size(type); t.fn = fn; t.sources = sources; t.targets = targets;
    t.times = calloc((size_t) reps + 1, sizeof(double));
    const int nth = npes * tpp;
    /* chosen before any thread is pinned (a pinned thread's mask is one CPU) */
    t.cpus = calloc((size_t) nth, sizeof(int));
    for (int i = 0; i < nth; i++) t.cpus[i] = allowed_cpu(i);
    pthread_barrier_init(&t.bar, NULL, (unsigned) nth);
    pthread_t *th = calloc((size_t) nth, sizeof(pthread_t));
    bl_arg *args = calloc((size_t) nth, sizeof(bl_arg));
    for (int i = 0; i < nth; i++) {
        args[i].t = &t;
        args[i].me = i / tpp;
        args[i].part = i % tpp;
        pthread_create(&th[i], NULL, bl_pe, &args[i]);
    }
    for (int i = 0; i < nth; i++) pthread_join(th[i], NULL);
    pthread_barrier_destroy(&t.bar);
    qsort(t.times + 1, (size_t) reps, sizeof(double), cmp_d); /* drop warm-up */
    double med = t.times[1 + reps / 2];
    free(t.times);
    free(t.cpus);
    free(th);
    free(args);
    return med;
}

double oracle_cpu_baseline_split(int type, int op, int npes,
                                 const void *const *sources, void *const *targets,
                                 int nreduce, int reps, int pin_cores, int tpp)
{
    return oracle_cpu_baseline_ref(type, op, npes, sources, targets, nreduce, reps, pin_cores,
                                   tpp, NULL);
}

double oracle_cpu_baseline(int type, int op, int npes,
                           const void *const *sources, void *const *targets,
                           int nreduce, int reps, int pin_cores)
{
    return oracle_cpu_baseline_split(type, op, npes, sources, targets, nreduce, reps,
                                     pin_cores, 1);
}
