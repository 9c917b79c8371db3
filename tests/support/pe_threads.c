/*
 * pe_threads.c -- TEST INFRASTRUCTURE: an in-process OpenSHMEM PE runtime,
 * one thread per PE ("threads-as-PEs").
 *
 * Supplies the PE services libosgpu_reduce.so takes from the OpenSHMEM
 * runtime (struct osgpu_pe_ops): shmem_my_pe (src/ranks.c:17-23),
 * shmem_n_pes, shmem_barrier over an active set (src/barrier.c:21-27) and
 * shmem_getmem (src/putget.h:539-561) as a memcpy from the peer's host heap
 * at the same offset (the base-offset translation of src/shmemc/comms.c:89-105).
 * Only the transport is replaced; the library under test is the product.
 */
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    int (*my_pe)(void);
    int (*n_pes)(void);
    void (*barrier)(int, int, int, long *);
    void (*getmem)(void *, const void *, size_t, int);
} pe_ops_t;

#define MAXPE 64
#define MAXBAR 64

static int g_npes = 0;
static __thread int t_me = -1;
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;

/* A polling barrier, as the reference's: its PEs spin on their pSync
   (shmemc_wait_eq_until64 / _ne_until64, src/shmemc/barrier.c:32,47) rather
   than sleep, and so does the multi-process runtime (pe_shm.c).  A sleeping
   pthread barrier put a futex wake-up (5-20 us) into every call's timing.
   Sense-reversing: the last arrival resets the count, then bumps gen.
   PET_SLEEP_BARRIER=1: the sleeping form (mutex + condition variable), kept
   for the A/B of tools/call_overhead.py. */
typedef struct {
    int size, count;
    unsigned gen;
    pthread_mutex_t mu;
    pthread_cond_t cv;
} spin_bar_t;

static int sleep_barrier(void)
{
    static int v = -1;
    if (v < 0) {
        const char *e = getenv("PET_SLEEP_BARRIER");
        v = e && e[0] == '1';
    }
    return v;
}

static void spin_bar_init(spin_bar_t *b, int size)
{
    b->size = size;
    b->count = 0;
    b->gen = 0;
    pthread_mutex_init(&b->mu, NULL);
    pthread_cond_init(&b->cv, NULL);
}

static void spin_bar_wait(spin_bar_t *b)
{
    if (sleep_barrier()) {
        pthread_mutex_lock(&b->mu);
        const unsigned g = b->gen;
        if (++b->count == b->size) {
            b->count = 0;
            __atomic_store_n(&b->gen, g + 1, __ATOMIC_RELEASE);
            pthread_cond_broadcast(&b->cv);
        } else {
            while (b->gen == g) pthread_cond_wait(&b->cv, &b->mu);
        }
        pthread_mutex_unlock(&b->mu);
        return;
    }
    const unsigned gen = __atomic_load_n(&b->gen, __ATOMIC_ACQUIRE);
    if (__atomic_add_fetch(&b->count, 1, __ATOMIC_ACQ_REL) == b->size) {
        __atomic_store_n(&b->count, 0, __ATOMIC_RELAXED);
        __atomic_store_n(&b->gen, gen + 1, __ATOMIC_RELEASE);
    } else {
        unsigned spins = 0;
        while (__atomic_load_n(&b->gen, __ATOMIC_ACQUIRE) == gen) {
            __builtin_ia32_pause();
            if (++spins > 4096) sched_yield();  /* more PE threads than cores */
        }
    }
}

typedef struct {
    int used, start, stride, size;
    spin_bar_t b;
} bar_t;
static bar_t g_bars[MAXBAR];
static long g_bar_calls[MAXPE];

static char *g_heap[MAXPE];
static size_t g_heap_bytes[MAXPE];

int pet_my_pe(void) { return t_me; }
int pet_n_pes(void) { return g_npes; }

void pet_set_me(int pe) { t_me = pe; }

int pet_init(int npes)
{
    if (npes < 1 || npes > MAXPE) return -1;
    pthread_mutex_lock(&g_mu);
    for (int i = 0; i < MAXBAR; i++)
        g_bars[i].used = 0;
    memset(g_bar_calls, 0, sizeof(g_bar_calls));
    memset(g_heap, 0, sizeof(g_heap));
    memset(g_heap_bytes, 0, sizeof(g_heap_bytes));
    g_npes = npes;
    pthread_mutex_unlock(&g_mu);
    return 0;
}

static spin_bar_t *find_bar(int start, int stride, int size)
{
    spin_bar_t *r = NULL;
    pthread_mutex_lock(&g_mu);
    for (int i = 0; i < MAXBAR && !r; i++)
        if (g_bars[i].used && g_bars[i].start == start && g_bars[i].stride == stride &&
            g_bars[i].size == size)
            r = &g_bars[i].b;
    for (int i = 0; i < MAXBAR && !r; i++)
        if (!g_bars[i].used) {
            g_bars[i].used = 1;
            g_bars[i].start = start;
            g_bars[i].stride = stride;
            g_bars[i].size = size;
            spin_bar_init(&g_bars[i].b, size);
            r = &g_bars[i].b;
        }
    pthread_mutex_unlock(&g_mu);
    return r;
}

void pet_barrier(int PE_start, int logPE_stride, int PE_size, long *pSync)
{
    (void) pSync; /* left at SHMEM_SYNC_VALUE, as the reference's barrier leaves it */
    if (t_me >= 0 && t_me < MAXPE) __atomic_add_fetch(&g_bar_calls[t_me], 1, __ATOMIC_RELAXED);
    spin_bar_t *b = find_bar(PE_start, logPE_stride, PE_size);
    if (!b) { fprintf(stderr, "pe_threads: barrier table full\n"); abort(); }
    spin_bar_wait(b);
}

long pet_barrier_calls(int pe) { return (pe >= 0 && pe < MAXPE) ? g_bar_calls[pe] : -1; }

int pet_register_host_heap(int pe, void *base, size_t bytes)
{
    if (pe < 0 || pe >= MAXPE) return -1;
    g_heap[pe] = (char *) base;
    g_heap_bytes[pe] = bytes;
    return 0;
}

void pet_getmem(void *dest, const void *src, size_t n, int pe)
{
    const char *s = (const char *) src;
    const int me = t_me;
    if (me < 0 || pe < 0 || pe >= g_npes || !g_heap[me] || !g_heap[pe] || s < g_heap[me] ||
        s + n > g_heap[me] + g_heap_bytes[me]) {
        fprintf(stderr, "pe_threads: getmem of a non-symmetric address\n");
        abort();
    }
    memcpy(dest, g_heap[pe] + (s - g_heap[me]), n);
}

static pe_ops_t g_table = {pet_my_pe, pet_n_pes, pet_barrier, pet_getmem};

/* ---- C-level timing of the API: npes pthreads each call fn (a
   shmem_<T>_<op>_to_all) `reps` times; PE 0 times each collective call from
   a common start (polling barrier) to its own return, after one warm-up. */
typedef void (*to_all_fn)(void *, void *, int, int, int, int, void *, long *);
/* shmem_collect/fcollect/alltoall<bits> and shmem_broadcast<bits> */
typedef void (*coll_fn)(void *, const void *, size_t, int, int, int, long *);
typedef void (*bcast_fn)(void *, const void *, size_t, int, int, int, int, long *);

typedef struct {
    to_all_fn fn;
    int npes, n, reps, me;
    void **tgt, **src, **psync;
    spin_bar_t *bar;
    double *times;
    int kind;        /* 0 to_all, 1 collect-like, 2 broadcast */
    size_t nelems;   /* kinds 1, 2 */
    int root;        /* kind 2 */
} timing_arg;

#include <time.h>
static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double) ts.tv_sec + 1e-9 * (double) ts.tv_nsec;
}

static void *timing_body(void *p)
{
    timing_arg *a = (timing_arg *) p;
    long local_psync[128] = {0};
    long *psync = a->psync ? (long *) a->psync[a->me] : local_psync;
    char wrk[4096];
    t_me = a->me;
    for (int r = 0; r <= a->reps; r++) {
        spin_bar_wait(a->bar);
        double t0 = now_s();
        if (a->kind == 0)
            a->fn(a->tgt[a->me], a->src[a->me], a->n, 0, 0, a->npes, wrk, psync);
        else if (a->kind == 1)
            ((coll_fn) (void *) a->fn)(a->tgt[a->me], a->src[a->me], a->nelems, 0, 0, a->npes,
                                       psync);
        else
            ((bcast_fn) (void *) a->fn)(a->tgt[a->me], a->src[a->me], a->nelems, a->root, 0, 0,
                                        a->npes, psync);
        spin_bar_wait(a->bar);
        if (a->me == 0) a->times[r] = now_s() - t0;
    }
    return NULL;
}

static int cmpd(const void *x, const void *y)
{
    double a = *(const double *) x, b = *(const double *) y;
    return a < b ? -1 : a > b;
}

static double time_calls(void *fn, int kind, int npes, void **tgt, void **src, void **psync,
                         int n, size_t nelems, int root, int reps)
{
    if (npes < 1 || npes > MAXPE || reps < 1) return -1.0;
    spin_bar_t bar;
    spin_bar_init(&bar, npes);
    double *times = calloc((size_t) reps + 1, sizeof(double));
    pthread_t th[MAXPE];
    timing_arg args[MAXPE];
    for (int i = 0; i < npes; i++) {
        args[i] = (timing_arg){(to_all_fn) fn, npes, n, reps, i, tgt, src, psync, &bar, times,
                               kind, nelems, root};
        pthread_create(&th[i], NULL, timing_body, &args[i]);
    }
    for (int i = 0; i < npes; i++) pthread_join(th[i], NULL);
    qsort(times + 1, (size_t) reps, sizeof(double), cmpd);
    double med = times[1 + reps / 2];
    free(times);
    return med;
}

double pet_time_to_all(void *fn, int npes, void **tgt, void **src, void **psync, int n,
                       int reps)
{
    return time_calls(fn, 0, npes, tgt, src, psync, n, 0, 0, reps);
}

/* fn = shmem_{collect,fcollect,alltoall}<bits> (root < 0) or
   shmem_broadcast<bits> (root = PE_root); whole team, median seconds */
double pet_time_coll(void *fn, int npes, void **tgt, void **src, void **psync, size_t nelems,
                     int root, int reps)
{
    return time_calls(fn, root < 0 ? 1 : 2, npes, tgt, src, psync, 0, nelems, root, reps);
}

const void *pet_ops(void) { return &g_table; }
