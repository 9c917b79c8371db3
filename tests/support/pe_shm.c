/*
 * pe_shm.c -- TEST/BENCH INFRASTRUCTURE: an intra-node OpenSHMEM PE runtime
 * for one process per PE (the way an OpenSHMEM job runs), standing in for
 * the reference's UCX/PMIx layer:
 *   shmem_my_pe / shmem_n_pes   rank and size given at pes_init
 *   shmem_barrier(active set)   sense-reversing counter per active set in a
 *                               POSIX shared-memory segment (the reference's
 *                               tree barrier is AMO-based, src/shmemc/barrier.c:64-97;
 *                               this is its intra-node analogue: µs, not a
 *                               TCP round trip)
 *   shmem_getmem                memcpy from the peer's slot of a shared host
 *                               heap at the same offset (XPMEM-style; the
 *                               base-offset translation of src/shmemc/comms.c:89-105)
 * pes_set_thread_pe lets a thread act as another PE (jobs mixing PE threads
 * and PE processes, to test that the library refuses them where it must).
 */
#define _GNU_SOURCE
#include <fcntl.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#define MAXSETS 64

typedef struct {
    volatile int32_t used, start, stride, size;
    volatile int32_t count;
    volatile int32_t gen;
    char pad[40];
} set_t;

typedef struct {
    volatile int32_t lock;
    int32_t npes;
    uint64_t heap_bytes;
    set_t sets[MAXSETS];
} hdr_t;

static hdr_t *g_hdr;
static char *g_heap;     /* npes slots of heap_bytes */
static int g_me = -1, g_npes = 0;
static size_t g_map_bytes;

static size_t hdr_bytes(void) { return (sizeof(hdr_t) + 4095) & ~(size_t) 4095; }

int pes_init(const char *name, int me, int npes, unsigned long long heap_bytes, int create)
{
    heap_bytes = (heap_bytes + 4095) & ~4095ull;
    g_map_bytes = hdr_bytes() + (size_t) npes * heap_bytes;
    int fd = shm_open(name, O_RDWR | (create ? O_CREAT : 0), 0600);
    if (fd < 0) { perror("pe_shm: shm_open"); return -1; }
    if (create && ftruncate(fd, (off_t) g_map_bytes) != 0) { perror("pe_shm: ftruncate"); close(fd); return -1; }
    void *p = mmap(NULL, g_map_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) { perror("pe_shm: mmap"); return -1; }
    g_hdr = (hdr_t *) p;
    g_heap = (char *) p + hdr_bytes();
    if (create) {
        g_hdr->npes = npes;
        g_hdr->heap_bytes = heap_bytes;
    }
    g_me = me;
    g_npes = npes;
    return 0;
}

int pes_unlink(const char *name) { return shm_unlink(name); }

/* several PEs per process (threads): a thread may take another PE's rank */
static __thread int t_me = -1;
void pes_set_thread_pe(int pe) { t_me = pe; }
int pes_my_pe(void) { return t_me >= 0 ? t_me : g_me; }
int pes_n_pes(void) { return g_npes; }

void *pes_heap(int pe) { return g_heap + (size_t) pe * g_hdr->heap_bytes; }
unsigned long long pes_heap_bytes(void) { return g_hdr->heap_bytes; }

static void lock(void)
{
    while (__atomic_exchange_n(&g_hdr->lock, 1, __ATOMIC_ACQUIRE)) sched_yield();
}
static void unlock(void) { __atomic_store_n(&g_hdr->lock, 0, __ATOMIC_RELEASE); }

static set_t *find_set(int start, int stride, int size)
{
    set_t *r = NULL;
    lock();
    for (int i = 0; i < MAXSETS && !r; i++)
        if (g_hdr->sets[i].used && g_hdr->sets[i].start == start &&
            g_hdr->sets[i].stride == stride && g_hdr->sets[i].size == size)
            r = &g_hdr->sets[i];
    for (int i = 0; i < MAXSETS && !r; i++)
        if (!g_hdr->sets[i].used) {
            set_t *s = &g_hdr->sets[i];
            s->start = start; s->stride = stride; s->size = size;
            s->count = 0; s->gen = 0;
            __atomic_store_n(&s->used, 1, __ATOMIC_RELEASE);
            r = s;
        }
    unlock();
    if (!r) { fprintf(stderr, "pe_shm: too many active sets\n"); abort(); }
    return r;
}

void pes_barrier(int PE_start, int logPE_stride, int PE_size, long *pSync)
{
    (void) pSync; /* left at SHMEM_SYNC_VALUE */
    set_t *s = find_set(PE_start, logPE_stride, PE_size);
    const int32_t gen = __atomic_load_n(&s->gen, __ATOMIC_ACQUIRE);
    if (__atomic_add_fetch(&s->count, 1, __ATOMIC_ACQ_REL) == PE_size) {
        __atomic_store_n(&s->count, 0, __ATOMIC_RELAXED);
        __atomic_store_n(&s->gen, gen + 1, __ATOMIC_RELEASE);
    } else {
        unsigned spins = 0;
        while (__atomic_load_n(&s->gen, __ATOMIC_ACQUIRE) == gen)
            if (++spins > 4096) sched_yield();
    }
}

void pes_getmem(void *dest, const void *src, size_t n, int pe)
{
    const char *s = (const char *) src, *mine = (const char *) pes_heap(pes_my_pe());
    if (pe < 0 || pe >= g_npes || s < mine || s + n > mine + g_hdr->heap_bytes) {
        fprintf(stderr, "pe_shm: getmem of a non-symmetric address\n");
        abort();
    }
    memcpy(dest, (const char *) pes_heap(pe) + (s - mine), n);
}

typedef struct {
    int (*my_pe)(void);
    int (*n_pes)(void);
    void (*barrier)(int, int, int, long *);
    void (*getmem)(void *, const void *, size_t, int);
} pe_ops_t;

static pe_ops_t g_table = {pes_my_pe, pes_n_pes, pes_barrier, pes_getmem};

const void *pes_ops(void) { return &g_table; }

/* Per-call time of a reduce-to-all entry point timed in C, as the CPU
 * baseline is (oracle_reduce.c: CLOCK_MONOTONIC from barrier to barrier):
 * `reps` calls after 5 warm-up calls, each between two pes_barrier()s over
 * the whole job; median seconds per call.  fn has the reference's signature
 * (include/shmem/api.h: target, source, nreduce, PE_start, logPE_stride,
 * PE_size, pWrk, pSync). */
typedef void (*to_all_fn)(void *, void *, int, int, int, int, void *, long *);

static int cmp_dbl(const void *a, const void *b)
{
    const double x = *(const double *) a, y = *(const double *) b;
    return x < y ? -1 : x > y;
}

double pes_time_to_all(void *fn, void *target, void *source, int nreduce, int PE_start,
                       int logPE_stride, int PE_size, void *pWrk, long *pSync, int reps)
{
    if (reps < 1) return -1.0;
    double *t = malloc(sizeof(double) * (size_t) reps);
    for (int r = -5; r < reps; r++) {
        struct timespec a, b;
        pes_barrier(0, 0, g_npes, NULL);
        clock_gettime(CLOCK_MONOTONIC, &a);
        ((to_all_fn) fn)(target, source, nreduce, PE_start, logPE_stride, PE_size, pWrk, pSync);
        pes_barrier(0, 0, g_npes, NULL);
        clock_gettime(CLOCK_MONOTONIC, &b);
        if (r >= 0) t[r] = (double) (b.tv_sec - a.tv_sec) + 1e-9 * (double) (b.tv_nsec - a.tv_nsec);
    }
    qsort(t, (size_t) reps, sizeof(double), cmp_dbl);
    const double med = t[reps / 2];
    free(t);
    return med;
}
