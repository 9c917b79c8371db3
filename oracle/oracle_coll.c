/*
 * oracle_coll.c -- timed CPU baseline of the data-movement collectives in
 * the reference's loop shape.  TEST INFRASTRUCTURE ONLY (see oracle.h): used
 * by bench.py's cpu_baseline leg and tools/coll_bench.py, never by the
 * product.  The results themselves are checked by oracle_coll.py.
 *
 * pthreads as PEs over an in-process heap; a UCX put/get between PEs of one
 * node is a memcpy into/out of the peer's slot (the shared-memory transport),
 * so each collective is restated as the memcpys its reference code issues:
 *   fcollect  src/shmemc/fcollect.c:32-38  every PE puts its source at block
 *             vpe of every target (PE_size puts), barrier (:39)
 *   collect   src/shmemc/collect.c:32-64   offset wavefront through pSync
 *             (left to right: PE i waits for PE i-1's offset), then PE_size
 *             puts at that offset, barrier (:68)
 *   broadcast src/shmemc/broadcast.c:29-42 linear: barrier, every non-root
 *             gets the root's source
 *   alltoall  src/alltoall.c:59-82          PE_size gets of one block each
 * Kinds: 0 broadcast, 1 collect, 2 fcollect, 3 alltoall (oracle_coll.py).
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <pthread.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef struct {
    int kind, npes, reps, pin, root;
    size_t nb; /* bytes per PE contribution (block) */
    char *const *src;
    char *const *tgt;
    pthread_barrier_t bar;
    volatile long *wave; /* collect: per-PE offset slot, -1 = not yet */
    double *times;
} cb_team;

typedef struct {
    cb_team *t;
    int me;
} cb_arg;

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double) ts.tv_sec + 1e-9 * (double) ts.tv_nsec;
}

static void *cb_pe(void *p)
{
    cb_arg *ar = (cb_arg *) p;
    cb_team *t = ar->t;
    const int me = ar->me, P = t->npes;
    const size_t nb = t->nb;
    if (t->pin) {
        cpu_set_t cs;
        CPU_ZERO(&cs);
        CPU_SET(me % CPU_SETSIZE, &cs);
        pthread_setaffinity_np(pthread_self(), sizeof(cs), &cs);
    }
    memset(t->tgt[me], 0, (t->kind == 0 ? 1 : (size_t) P) * nb); /* first touch */
    for (int r = 0; r <= t->reps; r++) {
        if (me == 0)
            for (int i = 0; i < P; i++) t->wave[i] = -1;
        pthread_barrier_wait(&t->bar);
        double t0 = now_s();
        switch (t->kind) {
        case 0: /* broadcast, linear */
            pthread_barrier_wait(&t->bar);
            if (me != t->root) memcpy(t->tgt[me], t->src[t->root], nb);
            break;
        case 1: { /* collect: wavefront, then puts */
            long off;
            if (me == 0) off = 0;
            else
                while ((off = __atomic_load_n(&t->wave[me], __ATOMIC_ACQUIRE)) < 0) {
                }
            if (me < P - 1) __atomic_store_n(&t->wave[me + 1], off + (long) nb, __ATOMIC_RELEASE);
            for (int pe = 0; pe < P; pe++) memcpy(t->tgt[pe] + off, t->src[me], nb);
            break;
        }
        case 2: /* fcollect */
            for (int pe = 0; pe < P; pe++) memcpy(t->tgt[pe] + (size_t) me * nb, t->src[me], nb);
            break;
        case 3: /* alltoall (gets) */
            for (int pe = 0; pe < P; pe++)
                memcpy(t->tgt[me] + (size_t) pe * nb, t->src[pe] + (size_t) me * nb, nb);
            break;
        }
        pthread_barrier_wait(&t->bar);
        if (me == 0) t->times[r] = now_s() - t0;
    }
    return NULL;
}

static int cmp_d(const void *a, const void *b)
{
    double x = *(const double *) a, y = *(const double *) b;
    return x < y ? -1 : x > y;
}

/* median seconds per call over `reps` (after one warm-up); src[pe] holds
   nb bytes (alltoall: npes * nb), tgt[pe] npes * nb bytes */
double oracle_coll_baseline(int kind, int npes, char *const *src, char *const *tgt, size_t nb,
                            int root, int reps, int pin_cores)
{
    if (kind < 0 || kind > 3 || npes < 1 || reps < 1 || root < 0 || root >= npes) return -1.0;
    cb_team t;
    memset(&t, 0, sizeof(t));
    t.kind = kind; t.npes = npes; t.reps = reps; t.pin = pin_cores; t.root = root;
    t.nb = nb; t.src = src; t.tgt = tgt;
    t.wave = calloc((size_t) npes, sizeof(long));
    t.times = calloc((size_t) reps + 1, sizeof(double));
    pthread_barrier_init(&t.bar, NULL, (unsigned) npes);
    pthread_t *th = calloc((size_t) npes, sizeof(pthread_t));
    cb_arg *args = calloc((size_t) npes, sizeof(cb_arg));
    for (int i = 0; i < npes; i++) {
        args[i].t = &t;
        args[i].me = i;
        pthread_create(&th[i], NULL, cb_pe, &args[i]);
    }
    for (int i = 0; i < npes; i++) pthread_join(th[i], NULL);
    pthread_barrier_destroy(&t.bar);
    qsort(t.times + 1, (size_t) reps, sizeof(double), cmp_d);
    double med = t.times[1 + reps / 2];
    free(t.times);
    free((void *) t.wave);
    free(th);
    free(args);
    return med;
}
