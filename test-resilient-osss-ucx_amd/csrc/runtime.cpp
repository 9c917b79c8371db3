// runtime.cpp -- services shared by every collective of libosgpu_reduce.so
// (declared in runtime.hpp) and the control surface of include/osgpu_reduce.h
// (Part 2 below).  The collectives themselves live in shmem_reduce.cpp
// (the 44 reduce-to-all entry points) and shmem_collect.cpp (broadcast,
// collect, fcollect).
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <dlfcn.h>
#include <stdarg.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <mutex>
#include <thread>
#include <tuple>
#include <vector>

#include "../../include/osgpu_reduce.h"
#include "combine.hpp"
#include "runtime.hpp"

namespace osgpu {
namespace rt {

// ------------------------------------------------------------------ errors

thread_local char g_err[512];

void set_err(const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

// The shmem_* entry points are void (src/reductions.c:139-154); the
// reference logs LOG_FATAL and returns on OOM (:55-61) and asserts on
// transport errors (src/shmemc/comms.c:250).  Silent wrong results are
// worse than both, so an unrecoverable error is reported and aborts.
[[noreturn]] void fatal(const char *where, const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    fprintf(stderr, "osgpu_reduce: %s: %s\n", where, buf);
    fflush(stderr);
    abort();
}

// OSGPU_DEBUG=1 enables the DBG lines (runtime.hpp)
int debug_level()
{
    static int lvl = -1;
    if (lvl < 0) {
        const char *e = getenv("OSGPU_DEBUG");
        lvl = e ? atoi(e) : 0;
    }
    return lvl;
}

// Environment knobs are read ONCE each (function-local statics at their
// points of use), never per call; include/osgpu_reduce.h lists them.
static long long env_ll(const char *var, long long def)
{
    const char *e = getenv(var);
    return e && *e ? strtoll(e, nullptr, 0) : def;
}

static int env_word(const char *var, const char *const *words, int n, int def)
{
    const char *e = getenv(var);
    for (int i = 0; e && i < n; i++)
        if (!strcmp(e, words[i])) return i;
    return def;
}

// ----------------------------------------------------------- synchronisation

int env_choice(const char *var, const char *alt, int def_is_alt)
{
    const char *e = getenv(var);
    if (!e) return def_is_alt;
    return strcmp(e, alt) == 0;
}

// Entry: device work this process enqueued earlier may still be producing
// `source`; the collective reads it only after it is done.  OSGPU_ENTRY_SYNC:
//   stream (default)  hipStreamSynchronize of the legacy default stream,
//                     which waits for every blocking stream too (PyTorch's
//                     default stream is that stream); producer work on the
//                     caller's own non-blocking streams is the caller's to
//                     order, as with CUDA-aware MPI;
//   device            hipDeviceSynchronize: every stream of the process,
//                     including this PE's own, whose last fused launch may
//                     still be retiring (~15 us after its completion word);
//   spin              device, after spinning until this PE's stream is idle;
//   none              the caller orders its own producer work.
int entry_mode()
{
    static const int m = [] {
        const char *e = getenv("OSGPU_ENTRY_SYNC");
        if (!e || !strcmp(e, "stream")) return ENTRY_STREAM;
        if (!strcmp(e, "device")) return ENTRY_DEVICE;
        if (!strcmp(e, "spin")) return ENTRY_SPIN;
        if (!strcmp(e, "none")) return ENTRY_NONE;
        return ENTRY_STREAM;
    }();
    return m;
}

static void spin_idle(const char *where, hipStream_t st)
{
    hipError_t e;
    while ((e = hipStreamQuery(st)) == hipErrorNotReady) __builtin_ia32_pause();
    if (e != hipSuccess) fatal(where, "stream: %s", hipGetErrorString(e));
}

// host-side entry wait (paths whose first barrier is a host barrier)
void entry_sync(const char *where, hipStream_t own)
{
    switch (entry_mode()) {
    case ENTRY_SPIN:
        if (own) spin_idle(where, own);
        HIPCHK(where, hipDeviceSynchronize());
        break;
    case ENTRY_DEVICE: HIPCHK(where, hipDeviceSynchronize()); break;
    case ENTRY_STREAM: HIPCHK(where, hipStreamSynchronize(nullptr)); break;
    }
}

// Entry ordering of a launch on `st` whose barriers run on the device (the
// fused path).  The same waits as entry_sync; in `stream` mode they never
// include this PE's own (non-blocking) stream, whose previous launch may
// still be retiring after its host-visible completion word was written
// (measured ~15 us; a GPU-side event wait on the default stream measured
// slower still, ~55 us per call).
void entry_order(const char *where, hipStream_t st)
{
    entry_sync(where, st);
}

// Completion of our own stream.  OSGPU_SYNC:
//   word (default)   hipStreamWriteValue64 of a sequence number into a
//                    host-mapped word behind the stream's work, the host
//                    spinning on that word (an empty kernel's host-visible
//                    word: 6.4 us); hipStreamQuery every 64 K spins turns a
//                    faulted stream into an error instead of a hang.  The
//                    reference's PEs poll too (shmemc_wait_*_until64).  A
//                    2-PE 64 Mi-double team call: 369.6 us against 379-391
//                    with `block` (profiles/r04_bench_merge_word.log,
//                    r04_call_overhead_6.jsonl); 1 Ki ints with host
//                    barriers 11.2 us against 15.4;
//   block            hipStreamSynchronize (11.8 us launch-to-return for an
//                    empty kernel, profiles/r01_overhead_probe.jsonl);
//   spin             poll hipStreamQuery (13.5 us).
// OSGPU_CALL_TRACE=1: host clock at each phase of a host-barrier call
// (run_team), printed on stderr by PE 0 as "[osgpu call] <phase> <us> ..."
void call_trace(int me, int phase, const char *label)
{
    static const bool on = getenv("OSGPU_CALL_TRACE") != nullptr;
    if (!on || me != 0) return;
    thread_local std::chrono::steady_clock::time_point t[8];
    thread_local const char *names[8];
    thread_local int n = 0;
    if (phase == 0) n = 0;
    if (n < 8) {
        t[n] = std::chrono::steady_clock::now();
        names[n++] = label;
    }
    if (!strcmp(label, "end")) {
        std::string out = "[osgpu call]";
        for (int i = 1; i < n; i++) {
            char b[64];
            snprintf(b, sizeof(b), " %s %.2f", names[i],
                     std::chrono::duration<double, std::micro>(t[i] - t[i - 1]).count());
            out += b;
        }
        fprintf(stderr, "%s us\n", out.c_str());
    }
}

int sync_mode()
{
    static const int m = [] {
        const char *e = getenv("OSGPU_SYNC");
        if (e && !strcmp(e, "block")) return 0;
        if (e && !strcmp(e, "spin")) return 1;
        return 2;
    }();
    return m;
}

struct DoneWord {
    volatile unsigned long long *h = nullptr;
    void *d = nullptr;
    unsigned long long seq = 0;  // the last value written (travels with the word)
    int device = -1;
};
// Words of threads that exited, for reuse by new ones (PE threads come and
// go; no HIP call at thread exit)
std::mutex g_words_mu;
std::vector<DoneWord> g_words_free;
struct ThreadWord {
    DoneWord w;
    ~ThreadWord()
    {
        if (!w.h) return;
        std::lock_guard<std::mutex> lk(g_words_mu);
        g_words_free.push_back(w);
    }
};
thread_local ThreadWord t_word;

void stream_wait(const char *where, hipStream_t st)
{
    const int mode = sync_mode();
    if (mode == 0) {
        HIPCHK(where, hipStreamSynchronize(st));
        return;
    }
    hipError_t e;
    if (mode == 1) {
        while ((e = hipStreamQuery(st)) == hipErrorNotReady) __builtin_ia32_pause();
        if (e != hipSuccess) fatal(where, "stream: %s", hipGetErrorString(e));
        return;
    }
    int dev = 0;
    HIPCHK(where, hipGetDevice(&dev));
    DoneWord &t_done = t_word.w;
    if (!t_done.h || t_done.device != dev) {  // one word per thread and device
        bool reused = false;
        {
            std::lock_guard<std::mutex> lk(g_words_mu);
            if (t_done.h) g_words_free.push_back(t_done);
            for (size_t i = 0; i < g_words_free.size(); i++)
                if (g_words_free[i].device == dev) {
                    t_done = g_words_free[i];
                    g_words_free.erase(g_words_free.begin() + (long) i);
                    reused = true;
                    break;
                }
        }
        if (!reused) {
            void *h = nullptr;
            HIPCHK(where, hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent));
            HIPCHK(where, hipHostGetDevicePointer(&t_done.d, h, 0));
            t_done.h = static_cast<volatile unsigned long long *>(h);
            *t_done.h = 0;
            t_done.seq = 0;
            t_done.device = dev;
        }
    }
    const unsigned long long want = ++t_done.seq;
    HIPCHK(where, hipStreamWriteValue64(st, t_done.d, want, 0));
    for (unsigned long spins = 1;; spins++) {
        if (*t_done.h >= want) return;
        __builtin_ia32_pause();
        // past ~4 K spins (tens of us) give the core away now and then, like
        // the PE-thread barrier (tests/support/pe_threads.c): with more PE
        // threads than cores, spinning here must not starve the members this
        // call is waiting for
        if (spins > 4096 && (spins & 15) == 0) sched_yield();
        if ((spins & 0xffff) == 0) {
            e = hipStreamQuery(st);
            if (e == hipSuccess) {  // the write is behind everything: it must show
                for (int k = 0; k < 1000000 && *t_done.h < want; k++) __builtin_ia32_pause();
                if (*t_done.h >= want) return;
                fatal(where, "stream idle but its completion word was not written");
            }
            if (e != hipErrorNotReady) fatal(where, "stream: %s", hipGetErrorString(e));
        }
    }
}

// --------------------------------------------------------------- type info

size_t type_size(int t)
{
    switch (t) {
    case OSGPU_T_SHORT: return sizeof(short);
    case OSGPU_T_INT: return sizeof(int);
    case OSGPU_T_LONG: return sizeof(long);
    case OSGPU_T_LONGLONG: return sizeof(long long);
    case OSGPU_T_FLOAT: return sizeof(float);
    case OSGPU_T_DOUBLE: return sizeof(double);
    case OSGPU_T_LONGDOUBLE: return sizeof(long double);
    case OSGPU_T_COMPLEXF: return 2 * sizeof(float);
    case OSGPU_T_COMPLEXD: return 2 * sizeof(double);
    }
    return 0;
}

bool has_op(int t, int op)
{
    if (t < OSGPU_T_SHORT || t > OSGPU_T_COMPLEXD) return false;
    switch (op) {
    case OSGPU_OP_SUM: case OSGPU_OP_PROD: return true;
    case OSGPU_OP_AND: case OSGPU_OP_OR: case OSGPU_OP_XOR: return t <= OSGPU_T_LONGLONG;
    case OSGPU_OP_MAX: case OSGPU_OP_MIN: return t <= OSGPU_T_LONGDOUBLE;
    }
    return false;
}

// ------------------------------------------------------------- PE services

std::mutex g_mu;
PeOps g_ops;
bool g_ops_set = false;

PeOps pe_ops()
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_ops_set) {
        // bind to the OpenSHMEM runtime the application links (the reference
        // library exports these as strong or weak symbols)
        g_ops.my_pe = (int (*)(void)) dlsym(RTLD_DEFAULT, "shmem_my_pe");
        g_ops.n_pes = (int (*)(void)) dlsym(RTLD_DEFAULT, "shmem_n_pes");
        g_ops.barrier = (void (*)(int, int, int, long *)) dlsym(RTLD_DEFAULT, "shmem_barrier");
        g_ops.getmem = (void (*)(void *, const void *, size_t, int)) dlsym(RTLD_DEFAULT,
                                                                          "shmem_getmem");
        g_ops_set = true;
    }
    return g_ops;
}

// -------------------------------------------------------- device sym. heap

// A PE's device heap is one or more segments (separate allocations: HIP IPC
// cannot export a single allocation of 2 GiB or more on this platform, see
// DESIGN.md 6).  A symmetric object lives in the same segment at the same
// offset on every PE.
std::vector<std::vector<HeapEntry>> g_heap;  // [PE][segment]

bool heap_segment(int pe, int seg, HeapEntry *out)
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (pe < 0 || (size_t) pe >= g_heap.size() || seg < 0 ||
        (size_t) seg >= g_heap[pe].size() || !g_heap[pe][seg].base)
        return false;
    *out = g_heap[pe][seg];
    return true;
}

// segment of PE `pe` holding [addr, addr + nbytes), and the offset in it
bool heap_locate(int pe, const void *addr, size_t nbytes, int *seg, size_t *off)
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (pe < 0 || (size_t) pe >= g_heap.size()) return false;
    const char *p = (const char *) addr;
    for (size_t s = 0; s < g_heap[pe].size(); s++) {
        const HeapEntry &h = g_heap[pe][s];
        if (h.base && p >= h.base && p + nbytes <= h.base + h.bytes) {
            *seg = (int) s;
            *off = (size_t) (p - h.base);
            return true;
        }
    }
    return false;
}

// address of the symmetric object at (seg, off) on PE pe, checked for nbytes
bool heap_peer(int pe, int seg, size_t off, size_t nbytes, char **out, bool *remote)
{
    HeapEntry h;
    if (!heap_segment(pe, seg, &h) || off + nbytes > h.bytes) return false;
    *out = h.base + off;
    if (remote) *remote = h.remote;
    return true;
}

void heap_set_remote(int pe, int seg, bool remote)
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (pe >= 0 && (size_t) pe < g_heap.size() && seg >= 0 && (size_t) seg < g_heap[pe].size())
        g_heap[pe][seg].remote = remote;
}

// lowest segment index free on every PE of `pes` in this process's registry
int heap_free_segment(const std::vector<int> &pes)
{
    std::lock_guard<std::mutex> lk(g_mu);
    for (int seg = 0;; seg++) {
        bool free = true;
        for (int pe : pes)
            if (pe >= 0 && (size_t) pe < g_heap.size() && (size_t) seg < g_heap[pe].size() &&
                g_heap[pe][seg].base)
                free = false;
        if (free) return seg;
    }
}

void heap_clear_segment(int pe, int seg)
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (pe >= 0 && (size_t) pe < g_heap.size() && seg >= 0 && (size_t) seg < g_heap[pe].size())
        g_heap[pe][seg] = HeapEntry();
}

// ---------------------------------------------------------------- RCCL

Rccl g_rccl;

int g_path = -1;  // -1: not yet read from the environment

int path_mode()
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_path < 0) {
        g_path = OSGPU_PATH_AUTO;
        const char *e = getenv("OSGPU_REDUCE_PATH");
        if (e && !strcmp(e, "p2p")) g_path = OSGPU_PATH_P2P;
        if (e && !strcmp(e, "rccl")) g_path = OSGPU_PATH_RCCL;
        if (e && !strcmp(e, "pull")) g_path = OSGPU_PATH_PULL;
    }
    return g_path;
}

// ------------------------------------------------------ per-PE / per-thread

// Resources of one PE on one device (stream, scratch, pinned staging).  Keyed
// by (PE, device), not by thread: a PE is one logical thread of execution
// whatever OS thread happens to make its calls, so nothing leaks when a
// runtime runs PEs on short-lived threads.  Calls of one PE never overlap.
struct PeCtx {
    hipStream_t stream = nullptr;
    void *dscratch = nullptr;
    size_t dscratch_bytes = 0;
    void *hstage = nullptr;  // pinned
    size_t hstage_bytes = 0;
};
std::map<std::pair<int, int>, PeCtx *> g_pectx;

// per-thread: the stream chosen with osgpu_set_stream (overrides the PE's),
// and a default stream for the raw osgpu_combine launcher
struct ThreadStream {
    int device = -1;
    hipStream_t stream = nullptr;
    bool user_stream = false;
};
thread_local ThreadStream t_ctx;

hipStream_t thread_stream(const char *where)
{
    int dev = 0;
    HIPCHK(where, hipGetDevice(&dev));
    if (t_ctx.stream && (t_ctx.user_stream || t_ctx.device == dev)) return t_ctx.stream;
    HIPCHK(where, hipStreamCreateWithFlags(&t_ctx.stream, hipStreamNonBlocking));
    t_ctx.device = dev;
    t_ctx.user_stream = false;
    return t_ctx.stream;
}

PeCtx &pe_ctx(const char *where, int me)
{
    int dev = 0;
    HIPCHK(where, hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(g_mu);
    PeCtx *&p = g_pectx[std::make_pair(me, dev)];
    if (!p) {
        p = new PeCtx();
        HIPCHK(where, hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking));
    }
    return *p;
}

hipStream_t pe_stream(const char *where, int me)
{
    if (t_ctx.user_stream && t_ctx.stream) return t_ctx.stream;
    return pe_ctx(where, me).stream;
}

void *device_scratch(const char *where, int me, size_t bytes)
{
    PeCtx &x = pe_ctx(where, me);
    if (x.dscratch_bytes < bytes) {
        if (x.dscratch) HIPCHK(where, hipFree(x.dscratch));
        x.dscratch = nullptr;
        x.dscratch_bytes = 0;
        HIPCHK(where, hipMalloc(&x.dscratch, bytes));
        x.dscratch_bytes = bytes;
    }
    return x.dscratch;
}

void *host_stage(const char *where, int me, size_t bytes)
{
    PeCtx &x = pe_ctx(where, me);
    if (x.hstage_bytes < bytes) {
        if (x.hstage) HIPCHK(where, hipHostFree(x.hstage));
        x.hstage = nullptr;
        x.hstage_bytes = 0;
        HIPCHK(where, hipHostMalloc(&x.hstage, bytes, hipHostMallocMapped));
        x.hstage_bytes = bytes;
    }
    return x.hstage;
}

MemKind mem_kind(const void *p, int *dev)
{
    // virtual-memory heaps (heap.cpp) are device memory whatever the pointer
    // query says about a hipMemMap'ed range
    int hd = -1;
    if (heap_created_range(p, 1, &hd)) {
        if (dev) {
            if (hd < 0 && hipGetDevice(&hd) != hipSuccess) hd = 0;
            *dev = hd;
        }
        return MEM_DEVICE;
    }
    hipPointerAttribute_t a;
    memset(&a, 0, sizeof(a));
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void) hipGetLastError();  // unregistered pageable host memory
        return MEM_HOST;
    }
    if (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged ||
        a.type == hipMemoryTypeUnified) {
        if (dev) *dev = a.device;
        return MEM_DEVICE;
    }
    return MEM_HOST;
}

bool ranges_overlap(const void *a, const void *b, size_t n)
{
    // byte-exact: the reference's OVERLAP_CHECK (src/reductions.c:27-30)
    // adds a byte count to a typed pointer and over-detects by sizeof(T)
    uintptr_t x = (uintptr_t) a, y = (uintptr_t) b;
    return (x < y + n) && (y < x + n);
}

void fold_order(int me, int PE_start, int step, int PE_size, int *order)
{
    int k = 0;
    order[k++] = me;
    for (int i = 0, pe = PE_start; i < PE_size; i++, pe += step)
        if (pe != me) order[k++] = pe;
}

// ------------------------------------------------------------ active sets

Coll make_coll(const char *name, int PE_start, int logPE_stride, int PE_size, long *pSync)
{
    if (PE_size < 1 || PE_start < 0 || logPE_stride < 0 || logPE_stride > 30)
        fatal(name, "invalid active set (PE_start=%d logPE_stride=%d PE_size=%d)", PE_start,
              logPE_stride, PE_size);
    Coll c;
    c.name = name;
    c.PE_start = PE_start;
    c.logPE_stride = logPE_stride;
    c.PE_size = PE_size;
    c.pSync = pSync;
    c.step = 1 << logPE_stride;
    c.ops = pe_ops();
    if (!c.ops.my_pe || !c.ops.barrier)
        fatal(name, "no OpenSHMEM runtime: shmem_my_pe/shmem_barrier not found "
                    "(link the OpenSHMEM library or call osgpu_set_pe_ops)");
    c.me = c.ops.my_pe();
    return c;
}

void barrier(const Coll &c)
{
    DBG("%s PE %d: barrier enter", c.name, c.me);
    c.ops.barrier(c.PE_start, c.logPE_stride, c.PE_size, c.pSync);
    DBG("%s PE %d: barrier exit", c.name, c.me);
}

// Pageable host arrays: the runtime's own bounce copies move ~27 GB/s each
// way; this path stages them through the PE's pinned bounce slots with a
// multi-threaded memcpy instead (OSGPU_COPY_THREADS, default 4), so the DMA
// always runs from pinned memory.
bool host_pinned(const void *p)
{
    // OSGPU_HOST_BOUNCE=0: leave pageable memory to the runtime's own copies
    static const int no_bounce = env_choice("OSGPU_HOST_BOUNCE", "0", 0);
    if (no_bounce) return true;
    hipPointerAttribute_t a;
    memset(&a, 0, sizeof(a));
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void) hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// Helper threads are capped process-wide (OSGPU_COPY_THREADS_TOTAL, default
// 8): with many PE threads copying at once, more threads than that only
// contend for the same memory channels.
std::atomic<int> g_copy_helpers{0};

void par_memcpy(void *dst, const void *src, size_t n)
{
    static const int nt = [] {
        const char *e = getenv("OSGPU_COPY_THREADS");
        const int v = e ? atoi(e) : 4;
        return v < 1 ? 1 : (v > 32 ? 32 : v);
    }();
    static const int cap = [] {
        const char *e = getenv("OSGPU_COPY_THREADS_TOTAL");
        const int v = e ? atoi(e) : 8;
        return v < 0 ? 0 : (v > 256 ? 256 : v);
    }();
    const size_t min_piece = (size_t) 1 << 20;
    const int want = (int) std::min<size_t>((size_t) nt, (n + min_piece - 1) / min_piece) - 1;
    int got = 0;  // helpers reserved under the cap
    for (int cur = g_copy_helpers.load(); want > 0;) {
        got = std::min(want, cap - cur);
        if (got <= 0) {
            got = 0;
            break;
        }
        if (g_copy_helpers.compare_exchange_weak(cur, cur + got)) break;
    }
    if (got == 0) {
        memcpy(dst, src, n);
        return;
    }
    const int k = got + 1;
    const size_t piece = (n / k + 4095) & ~(size_t) 4095;
    std::vector<std::thread> th;
    for (int i = 1; i < k; i++) {
        const size_t lo = (size_t) i * piece;
        if (lo >= n) break;
        const size_t len = std::min(piece, n - lo);
        th.emplace_back([=] { memcpy((char *) dst + lo, (const char *) src + lo, len); });
    }
    memcpy(dst, src, std::min(piece, n));
    for (auto &t : th) t.join();
    g_copy_helpers.fetch_sub(got);
}

// ---------------------------------------------------------------------
// STAGED host path: H2D of my own source -> exchange ON THE GPUs (team
// kernel over every PE's device staging buffers, IPC-mapped) -> D2H.
// Pipelined over chunks with two slots and three streams:
//   H2D(c+1) || team(c) || D2H(c-1).
// The peers' data never crosses the host: PCIe carries N*s in and N*s out
// per PE, xGMI carries the exchange.  Setup (once per active set) publishes
// each PE's staging allocation through spare words of the symmetric pSync
// (the reference's barrier only uses pSync[0], src/shmemc/barrier.c:64-97)
// and reads the peers' with shmem_getmem; pSync is returned zeroed.
// ---------------------------------------------------------------------

constexpr int kPsyncBase = 16;  // pSync[16..28] used during setup only

std::map<std::tuple<int, int, int, int, int>, StageSet> g_stage;  // (me, set, device)

long long g_stage_bytes = -1;  // osgpu_set_stage_bytes; -1: OSGPU_STAGE_BYTES, 32 MiB

size_t stage_slot_bytes()
{
    static const long long env = [] {
        const long long v = env_ll("OSGPU_STAGE_BYTES", 0);
        return v > 0 ? v : (32LL << 20);
    }();
    long long b;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        b = g_stage_bytes > 0 ? g_stage_bytes : env;
    }
    return ((size_t) b + 255) & ~(size_t) 255;
}

struct StageMsg {  // what a PE publishes in pSync[16..30]
    long handle[OSGPU_IPC_HANDLE_BYTES / sizeof(long)];
    long raw_ptr, pid, slot, status, pci, pad[2];
};
// the smallest pSync a caller hands us: SHMEM_BCAST/COLLECT/ALLTOALL_SYNC_SIZE
static_assert(sizeof(StageMsg) <= (64 - kPsyncBase) * sizeof(long), "pSync room");

long pci_key(int dev)
{
    int dom = 0, bus = 0, d = 0;
    if (hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, dev) != hipSuccess ||
        hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, dev) != hipSuccess ||
        hipDeviceGetAttribute(&d, hipDeviceAttributePciDeviceId, dev) != hipSuccess) {
        (void) hipGetLastError();
        return -1 - dev;
    }
    return ((long) dom << 16 | (long) bus << 8 | d) + 1;
}

// Publish `local` (a device allocation of `bytes`) to every member of the
// active set through spare pSync words and map every member's allocation:
// same process -> raw pointer, other processes -> HIP IPC.  Collective (three
// barriers); every member returns the same verdict.  pSync is returned zeroed.
bool map_members(const Coll &c, char *local, size_t bytes, std::vector<char *> &peer,
                 std::vector<void *> &opened, int *ndev, bool distinct_processes,
                 int *max_share, int *procs_here)
{
    int dev = 0;
    HIPCHK(c.name, hipGetDevice(&dev));
    StageMsg *mine = reinterpret_cast<StageMsg *>(c.pSync + kPsyncBase);
    memset(mine, 0, sizeof(*mine));
    hipIpcMemHandle_t h;
    if (local && hipIpcGetMemHandle(&h, local) == hipSuccess) memcpy(mine->handle, &h, sizeof(h));
    else (void) hipGetLastError();
    mine->raw_ptr = (long) (uintptr_t) local;
    mine->pid = (long) getpid();
    mine->slot = local ? (long) bytes : -1;
    mine->pci = pci_key(dev);
    barrier(c);
    bool ok = local != nullptr;
    peer.assign(c.PE_size, nullptr);
    std::vector<long> pcis(1, mine->pci), all_pci(1, mine->pci);
    std::vector<long> pids_here(1, mine->pid);  // processes on my GPU
    for (int i = 0, pe = c.PE_start; i < c.PE_size; i++, pe += c.step) {
        if (pe == c.me) {
            peer[i] = local;
            continue;
        }
        StageMsg m;
        c.ops.getmem(&m, mine, sizeof(m), pe);
        all_pci.push_back(m.pci);
        if (std::find(pcis.begin(), pcis.end(), m.pci) == pcis.end()) pcis.push_back(m.pci);
        if (m.pci == mine->pci &&
            std::find(pids_here.begin(), pids_here.end(), m.pid) == pids_here.end())
            pids_here.push_back(m.pid);
        if (m.slot != (long) bytes) {
            ok = false;
        } else if (m.pid == (long) getpid()) {
            peer[i] = (char *) (uintptr_t) m.raw_ptr;   // same process (threads as PEs)
            if (distinct_processes) ok = false;
        } else {
            hipIpcMemHandle_t ph;
            memcpy(&ph, m.handle, sizeof(ph));
            void *p = nullptr;
            if (hipIpcOpenMemHandle(&p, ph, hipIpcMemLazyEnablePeerAccess) == hipSuccess) {
                peer[i] = (char *) p;
                opened.push_back(p);
            } else {
                (void) hipGetLastError();
                ok = false;
            }
        }
    }
    mine->status = ok ? 1 : 2;
    barrier(c);
    bool all_ok = ok;
    for (int i = 0, pe = c.PE_start; i < c.PE_size; i++, pe += c.step) {
        if (pe == c.me) continue;
        long st = 0;
        c.ops.getmem(&st, &mine->status, sizeof(long), pe);
        all_ok = all_ok && st == 1;
    }
    barrier(c);
    memset(mine, 0, sizeof(*mine));  // pSync back to SHMEM_SYNC_VALUE
    if (ndev) *ndev = (int) pcis.size();
    if (procs_here) *procs_here = (int) pids_here.size();
    if (max_share) {
        int mx = 0;
        for (long k : pcis) mx = std::max(mx, (int) std::count(all_pci.begin(), all_pci.end(), k));
        *max_share = mx;
    }
    return all_ok;
}

// One H2D and one D2H stream per device for every PE of this process: the
// DMA engines run one copy per direction at full duplex (48.6 GB/s each way
// on this link), but two per direction at once drop to 28.7 GB/s each way
// (tools/pcie_kernel_probe.hip, profiles/r01_pcie_kernel_probe.jsonl), so
// PEs that are threads of one process queue their staging copies on the
// same pair instead of competing.
std::map<int, std::pair<hipStream_t, hipStream_t>> g_copy_streams;

// The H2D and D2H copy streams must never share a hardware queue: HIP
// gives a process GPU_MAX_HW_QUEUES queues per priority level (4 on the
// pool) and deals further streams onto them, so with one more stream in the
// process than the staging set expects (a torch side stream, the thread's
// osgpu_combine stream) the D2H copies queued behind the H2D ones on one
// queue -- the two directions took turns: 27.7 GB/s each way instead of
// 44.5, and pageable 25 instead of 38-41 (tools/host_staged_context.py,
// profiles/r05_host_staged_streams.jsonl; the round-3 regression of
// BENCH_r03/r04).  Streams of different priorities come from different
// queue pools, so H2D takes the lowest priority and D2H the highest: never
// one queue, whatever else the process created.  (OSGPU_COPY_STREAMS=plain
// restores default-priority streams, cumask gives each its own CU-masked
// queue; both measured in that file.)
extern "C" int osgpu_copy_stream_priorities(int least, int greatest, int *in, int *out)
{
    if (!in || !out) return OSGPU_EINVAL;
    *in = least;
    *out = greatest;
    return least != greatest ? OSGPU_OK : OSGPU_EINVAL;  // one level: no separate pools
}

static void create_copy_stream(const char *where, int dev, hipStream_t *s, bool out)
{
    static const int mode = [] {
        static const char *w[] = {"prio", "plain", "cumask"};
        return env_word("OSGPU_COPY_STREAMS", w, 3, 0);
    }();
    const bool plain = mode == 1;
    bool cumask = mode == 2;
    if (!plain && !cumask) {
        int least = 0, greatest = 0, pin = 0, pout = 0;
        HIPCHK(where, hipDeviceGetStreamPriorityRange(&least, &greatest));
        if (osgpu_copy_stream_priorities(least, greatest, &pin, &pout) == OSGPU_OK) {
            HIPCHK(where, hipStreamCreateWithPriority(s, hipStreamNonBlocking, out ? pout : pin));
            return;
        }
        cumask = true;  // a single priority level: a queue of its own instead
    }
    if (cumask) {
        int ncu = 0;
        HIPCHK(where, hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
        std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
        for (int i = 0; i < ncu; i++) mask[i / 32] |= 1u << (i % 32);
        HIPCHK(where, hipExtStreamCreateWithCUMask(s, (uint32_t) mask.size(), mask.data()));
        return;
    }
    HIPCHK(where, hipStreamCreateWithFlags(s, hipStreamNonBlocking));
}

// the priorities of this device's staging copy streams (tests)
extern "C" int osgpu_copy_stream_info(int dev, int *in_prio, int *out_prio)
{
    hipStream_t a = nullptr, b = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto it = g_copy_streams.find(dev);
        if (it == g_copy_streams.end()) return OSGPU_EINVAL;
        a = it->second.first;
        b = it->second.second;
    }
    if (hipStreamGetPriority(a, in_prio) != hipSuccess || hipStreamGetPriority(b, out_prio) != hipSuccess) {
        (void) hipGetLastError();
        return OSGPU_EHIP;
    }
    return OSGPU_OK;
}

void device_copy_streams(const char *where, int dev, hipStream_t *in, hipStream_t *out)
{
    std::lock_guard<std::mutex> lk(g_mu);
    auto &p = g_copy_streams[dev];
    if (!p.first) {
        create_copy_stream(where, dev, &p.first, false);
        create_copy_stream(where, dev, &p.second, true);
    }
    *in = p.first;
    *out = p.second;
}

StageSet *stage_setup(const Coll &c)
{
    int dev = 0;
    HIPCHK(c.name, hipGetDevice(&dev));
    auto key = std::make_tuple(c.me, c.PE_start, c.step, c.PE_size, dev);
    std::unique_lock<std::mutex> lk(g_mu);
    auto it = g_stage.find(key);
    if (it != g_stage.end()) return it->second.ok ? &it->second : nullptr;
    StageSet &S = g_stage[key];  // std::map: the reference stays valid
    lk.unlock();
    S.device = dev;
    S.slot = stage_slot_bytes();
    HIPCHK(c.name, hipMalloc((void **) &S.local, 4 * S.slot));
    for (int s = 0; s < 2; s++) {
        HIPCHK(c.name, hipEventCreateWithFlags(&S.ev_in[s], hipEventDisableTiming));
        HIPCHK(c.name, hipEventCreateWithFlags(&S.ev_out[s], hipEventDisableTiming));
    }
    int procs_here = 1;
    S.ok = map_members(c, S.local, S.slot, S.peer, S.opened, &S.ndev, false, nullptr,
                       &procs_here);
    if (procs_here > 1) {
        // PE processes sharing this GPU also share its hardware queue slots
        // (HIP gives each process up to 4; past 16 on the GPU its scheduler
        // time-slices them in milliseconds, DESIGN_HISTORY.md 10) and its PCIe link:
        // the staging copies and folds go on the PE's own stream, in order,
        // so this process holds no queue beyond it
        S.st_in = S.st_out = S.st_c = pe_ctx(c.name, c.me).stream;
    } else {
        device_copy_streams(c.name, dev, &S.st_in, &S.st_out);
        HIPCHK(c.name, hipStreamCreateWithFlags(&S.st_c, hipStreamNonBlocking));
        S.own_c = true;
    }
    return S.ok ? &S : nullptr;
}

// host ranges pinned through osgpu_host_register, with their device view
struct HostReg {
    char *base;
    size_t bytes;
    char *dev;
};
std::vector<HostReg> g_hostreg;

void *host_device_view(const void *p, size_t nbytes)
{
    std::lock_guard<std::mutex> lk(g_mu);
    const char *c = (const char *) p;
    for (const HostReg &r : g_hostreg)
        if (r.dev && c >= r.base && c + nbytes <= r.base + r.bytes) return r.dev + (c - r.base);
    return nullptr;
}

// Settings with a setter (osgpu_set_*) and an environment default (env_ll /
// env_word, read once into a function-local static the first time a setting
// is needed); a setter's value wins until it is set back to -1.
int g_team_exchange = -1;  // -1: OSGPU_TEAM_EXCHANGE (pull|push), default pull

int team_exchange()
{
    static const int env = [] {
        static const char *w[] = {"pull", "push"};
        return env_word("OSGPU_TEAM_EXCHANGE", w, 2, 0);
    }();
    std::lock_guard<std::mutex> lk(g_mu);
    return g_team_exchange < 0 ? env : g_team_exchange;
}

long long g_fused_max = -1;  // -1: OSGPU_FUSED_MAX_BYTES, default 1 MiB

size_t fused_max_bytes()
{
    static const long long env = [] {
        const long long v = env_ll("OSGPU_FUSED_MAX_BYTES", 1LL << 20);
        return v < 0 ? 0 : v;
    }();
    std::lock_guard<std::mutex> lk(g_mu);
    return (size_t) (g_fused_max < 0 ? env : g_fused_max);
}

// Host symmetric-heap calls (shmem_reduce.cpp to_all, shmem_collect.cpp):
// OSGPU_HOST_PATH = auto | staged | getmem (osgpu_set_host_path).
int g_host_path = -1;

int host_path()
{
    static const int env = [] {
        static const char *w[] = {"auto", "staged", "getmem"};
        return env_word("OSGPU_HOST_PATH", w, 3, OSGPU_HOST_AUTO);
    }();
    std::lock_guard<std::mutex> lk(g_mu);
    return g_host_path < 0 ? env : g_host_path;
}

// Limit of the host fold (host_fold.hip) on the automatic host path, on the
// bytes each PE pulls from its peers, (PE_size - 1) * nreduce * size:
// OSGPU_HOST_FOLD_MAX_BYTES, default 256 KiB (2 PEs: 64 Ki ints, where the
// fold took 10 us against 41 us for the fused staged launch and 15 us for
// the fused launch on device heaps, profiles/r06_bench_run2.log small_call);
// 0 turns it off.
long long g_host_fold_max = -1;

size_t host_fold_max_bytes()
{
    static const long long env = [] {
        const long long v = env_ll("OSGPU_HOST_FOLD_MAX_BYTES", 256LL << 10);
        return v < 0 ? 0 : v;
    }();
    std::lock_guard<std::mutex> lk(g_mu);
    return (size_t) (g_host_fold_max < 0 ? env : g_host_fold_max);
}

// How the STAGED path's legs cross PCIe: OSGPU_STAGE_COPY = dma | kout |
// kernel (osgpu_set_stage_copy; shmem_reduce.cpp stage_leg).
int g_stage_copy = -1;

int stage_copy_mode()
{
    static const int env = [] {
        static const char *w[] = {"dma", "kout", "kernel"};
        return env_word("OSGPU_STAGE_COPY", w, 3, 0);
    }();
    std::lock_guard<std::mutex> lk(g_mu);
    return g_stage_copy < 0 ? env : g_stage_copy;
}

// Chunk of the GETMEM host path: OSGPU_HOST_CHUNK_BYTES, default 64 MiB
// (osgpu_set_host_chunk_bytes).
long long g_host_chunk = -1;

size_t host_chunk_bytes()
{
    static const long long env = [] {
        const long long v = env_ll("OSGPU_HOST_CHUNK_BYTES", 0);
        return v > 0 ? v : (64LL << 20);
    }();
    std::lock_guard<std::mutex> lk(g_mu);
    return (size_t) (g_host_chunk <= 0 ? env : g_host_chunk);
}

// ---------------------------------------------------------------------
// Device-side barriers of the fused small-call path (fused.hip): one flag
// area per member and active set, in uncached device memory (remote writes
// over xGMI are seen by a polling load without cache maintenance), mapped
// into every member like the staging above.
// ---------------------------------------------------------------------

std::map<std::tuple<int, int, int, int, int>, SyncSet> g_sync;  // (me, set, device)

// Completion of a fused launch: spin on the host-mapped word the kernel's
// last workgroup writes once every member is done (no wait for the launch to
// retire); also return when the launch reports a barrier it did not pass in
// its slice (error word), or when the stream ends without either.
static void fused_wait(const char *where, const SyncSet &S, hipStream_t st,
                       unsigned long long epoch)
{
    for (unsigned it = 1;; it++) {
        if (__atomic_load_n(S.done_h, __ATOMIC_ACQUIRE) >= epoch) return;
        if (__atomic_load_n(S.err_h, __ATOMIC_ACQUIRE)) return;
        if ((it & 4095) == 0) {
            const hipError_t q = hipStreamQuery(st);
            if (q == hipSuccess) return;  // ended; the caller tells done from failed
            if (q != hipErrorNotReady) fatal(where, "fused launch: %s", hipGetErrorString(q));
        }
        __builtin_ia32_pause();
    }
}

// Device-barrier policy (osgpu_set_device_barrier): how long a member may
// stay away before the call fails (<= 0: OSGPU_DEVICE_BARRIER_TIMEOUT_S, else
// without bound, the reference's barrier), and whether that failure aborts
// the process (default) or is reported.
double g_dbar_secs = -1;
int g_dbar_fatal = 1;

static double fused_bound_secs()
{
    static const double env = [] {
        const char *e = getenv("OSGPU_DEVICE_BARRIER_TIMEOUT_S");
        return e ? atof(e) : 0.0;
    }();
    double secs;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        secs = g_dbar_secs;
    }
    if (secs <= 0) secs = env;
    return secs > 0 ? secs : 0.0;
}

// One wait slice of a fused launch (OSGPU_DEVICE_BARRIER_SLICE_MS, default
// 100 ms): the longest a launch holds its CUs waiting at a device barrier.
static double fused_slice_secs()
{
    static const double s = [] {
        const char *e = getenv("OSGPU_DEVICE_BARRIER_SLICE_MS");
        const double ms = e ? atof(e) : 100.0;
        return (ms > 0 ? ms : 100.0) * 1e-3;
    }();
    return s;
}

static double now_secs()
{
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double) ts.tv_sec + 1e-9 * (double) ts.tv_nsec;
}

static bool fused_fail(const char *where, SyncSet &S, int err, unsigned long long epoch,
                       double absent)
{
    char msg[256];
    if (err == 3)
        snprintf(msg, sizeof(msg),
                 "collect: a member's contribution exceeds its source object in the heap");
    else if (err)
        snprintf(msg, sizeof(msg),
                 "device barrier (%s): a member of the active set stayed away for %.2f s, "
                 "longer than the device-barrier bound",
                 err == 1 ? "entry" : "exit", absent);
    else
        snprintf(msg, sizeof(msg), "fused launch ended without completing epoch %llu", epoch);
    int fatal_policy;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        fatal_policy = g_dbar_fatal;
    }
    if (fatal_policy) fatal(where, "%s", msg);
    // reported, not fatal: this call's target is not valid, and the set's
    // epochs may disagree from now on -- its fused path is switched off
    set_err("%s: %s", where, msg);
    __atomic_store_n(S.err_h, 0, __ATOMIC_RELEASE);
    S.ok = false;
    return false;
}

thread_local int t_continuations = 0;  // of the calling thread's last fused call

bool fused_complete(const char *where, SyncSet &S, hipStream_t st, osgpu::FusedArgs &a,
                    const std::function<hipError_t(const osgpu::FusedArgs &)> &launch)
{
    t_continuations = 0;
    const double slice = fused_slice_secs();
    a.timeout = (unsigned long long) (slice * 1e3 * S.rate_khz);
    a.resume = 0;
    a.attempt = 0;
    hipError_t e = launch(a);
    if (e != hipSuccess) fatal(where, "fused launch: %s", hipGetErrorString(e));
    const double bound = fused_bound_secs();
    double since = -1;  // when the current wait began (first unpassed barrier)
    for (;;) {
        fused_wait(where, S, st, a.epoch);
        const int err = __atomic_load_n(S.err_h, __ATOMIC_ACQUIRE);
        if (!err && __atomic_load_n(S.done_h, __ATOMIC_ACQUIRE) >= a.epoch) return true;
        if (err != 1 && err != 2) return fused_fail(where, S, err, a.epoch, 0);
        // a member has not reached the barrier yet: continue there
        const double now = now_secs();
        if (since < 0 || a.resume != err) since = now - slice;
        if (bound > 0 && now - since > bound) return fused_fail(where, S, err, a.epoch, now - since);
        __atomic_store_n(S.err_h, 0, __ATOMIC_RELEASE);
        a.resume = err;
        a.attempt++;
        t_continuations++;
        DBG("%s: epoch %llu: %s barrier not passed yet, continuation %u", where, a.epoch,
            err == 1 ? "entry" : "exit", a.attempt);
        e = launch(a);
        if (e != hipSuccess) fatal(where, "fused continuation launch: %s", hipGetErrorString(e));
    }
}

SyncSet *sync_setup(const Coll &c)
{
    int dev = 0;
    HIPCHK(c.name, hipGetDevice(&dev));
    auto key = std::make_tuple(c.me, c.PE_start, c.step, c.PE_size, dev);
    std::unique_lock<std::mutex> lk(g_mu);
    auto it = g_sync.find(key);
    if (it != g_sync.end()) return it->second.ok ? &it->second : nullptr;
    SyncSet &S = g_sync[key];
    lk.unlock();
    S.idx = c.index_of(c.me);
    const size_t bytes = osgpu::kFlagWords * sizeof(unsigned long long);
    void *p = nullptr;
    bool ok = hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached) == hipSuccess;
    if (!ok) (void) hipGetLastError();
    if (ok && hipMemset(p, 0, bytes) != hipSuccess) ok = false;
    if (ok && hipHostMalloc((void **) &S.err_h, sizeof(int) * 64,
                            hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
        ok = false;
    if (ok) {  // int 0: error code; ints 8..9: completion epoch; 16..33: collect counts
        memset(S.err_h, 0, sizeof(int) * 64);
        S.done_h = reinterpret_cast<unsigned long long *>(S.err_h + 8);
        S.cnt_h = reinterpret_cast<unsigned long long *>(S.err_h + 16);
        ok = hipHostGetDevicePointer((void **) &S.err_d, S.err_h, 0) == hipSuccess;
        S.done_d = reinterpret_cast<unsigned long long *>(S.err_d + 8);
        S.cnt_d = reinterpret_cast<unsigned long long *>(S.err_d + 16);
    }
    int rate_khz = 0;
    if (ok) ok = hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, dev) ==
                 hipSuccess && rate_khz > 0;
    if (!ok) (void) hipGetLastError();
    if (ok) HIPCHK(c.name, hipDeviceSynchronize());  // zeroed before anyone can write
    S.local = (unsigned long long *) p;
    std::vector<char *> peer;
    // members must be separate processes: PEs that are threads of one process
    // share its few hardware queues, where one member's spinning kernel can
    // sit in front of another member's (no co-residency, a deadlock)
    int share = c.PE_size;
    ok = map_members(c, ok ? (char *) p : nullptr, bytes, peer, S.opened, nullptr, true, &share);
    // every member's workgroups must fit on a shared GPU at once (see fused.hip)
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 0;
    (void) hipGetLastError();
    cus = std::min(std::max(cus, 1), osgpu::kFusedBlocksPerGpu);
    S.max_blocks = std::max(1, cus / (share > 0 ? share : c.PE_size));
    S.peer.resize(peer.size());
    for (size_t i = 0; i < peer.size(); i++) S.peer[i] = (unsigned long long *) peer[i];
    S.rate_khz = rate_khz;
    S.ok = ok;
    return S.ok ? &S : nullptr;
}

}  // namespace rt
}  // namespace osgpu

// ======================================================================
// Part 2: control surface
// ======================================================================

using namespace osgpu::rt;

extern "C" {

int osgpu_set_pe_ops(const osgpu_pe_ops *ops)
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (!ops) {
        g_ops = PeOps();
        g_ops_set = false;
        return OSGPU_OK;
    }
    if (!ops->my_pe || !ops->barrier) {
        set_err("osgpu_set_pe_ops: my_pe and barrier are required");
        return OSGPU_EINVAL;
    }
    g_ops.my_pe = ops->my_pe;
    g_ops.n_pes = ops->n_pes;
    g_ops.barrier = ops->barrier;
    g_ops.getmem = ops->getmem;
    g_ops_set = true;
    return OSGPU_OK;
}

int osgpu_heap_register_segment(int pe, int seg, void *base, size_t bytes)
{
    if (pe < 0 || seg < 0 || seg > 255 || !base || !bytes) {
        set_err("osgpu_heap_register_segment: bad arguments");
        return OSGPU_EINVAL;
    }
    std::lock_guard<std::mutex> lk(g_mu);
    if ((size_t) pe >= g_heap.size()) g_heap.resize(pe + 1);
    if ((size_t) seg >= g_heap[pe].size()) g_heap[pe].resize(seg + 1);
    g_heap[pe][seg].base = (char *) base;
    g_heap[pe][seg].bytes = bytes;
    g_heap[pe][seg].remote = false;  // caller-made segments: the local shapes
    return OSGPU_OK;
}

int osgpu_heap_register(int pe, void *base, size_t bytes)
{
    return osgpu_heap_register_segment(pe, 0, base, bytes);
}

int osgpu_heap_unregister(int pe)
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (pe < 0 || (size_t) pe >= g_heap.size()) return OSGPU_EINVAL;
    g_heap[pe].clear();
    return OSGPU_OK;
}

void *osgpu_heap_translate(const void *addr, int from_pe, int to_pe)
{
    int seg = -1;
    size_t off = 0;
    char *p = nullptr;
    if (!heap_locate(from_pe, addr, 1, &seg, &off) || !heap_peer(to_pe, seg, off, 1, &p))
        return nullptr;
    return p;
}

int osgpu_ipc_get_handle(void *dev_base, void *handle_out)
{
    static_assert(sizeof(hipIpcMemHandle_t) <= OSGPU_IPC_HANDLE_BYTES, "ipc handle size");
    hipIpcMemHandle_t h;
    hipError_t e = hipIpcGetMemHandle(&h, dev_base);
    if (e != hipSuccess) {
        set_err("hipIpcGetMemHandle: %s", hipGetErrorString(e));
        return OSGPU_EHIP;
    }
    memset(handle_out, 0, OSGPU_IPC_HANDLE_BYTES);
    memcpy(handle_out, &h, sizeof(h));
    return OSGPU_OK;
}

void *osgpu_ipc_open(const void *handle)
{
    hipIpcMemHandle_t h;
    memcpy(&h, handle, sizeof(h));
    void *p = nullptr;
    hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) {
        set_err("hipIpcOpenMemHandle: %s", hipGetErrorString(e));
        return nullptr;
    }
    return p;
}

int osgpu_ipc_close(void *mapped)
{
    hipError_t e = hipIpcCloseMemHandle(mapped);
    if (e != hipSuccess) {
        set_err("hipIpcCloseMemHandle: %s", hipGetErrorString(e));
        return OSGPU_EHIP;
    }
    return OSGPU_OK;
}

int osgpu_rccl_unique_id(void *uid_out)
{
    static_assert(sizeof(ncclUniqueId) == OSGPU_RCCL_UID_BYTES, "uid size");
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) {
        set_err("ncclGetUniqueId: %s", ncclGetErrorString(r));
        return OSGPU_ERCCL;
    }
    memcpy(uid_out, &id, sizeof(id));
    return OSGPU_OK;
}

int osgpu_rccl_init(int npes, int me, const void *uid)
{
    if (g_rccl.world) return OSGPU_OK;
    ncclUniqueId id;
    memcpy(&id, uid, sizeof(id));
    ncclComm_t comm;
    ncclResult_t r = ncclCommInitRank(&comm, npes, id, me);
    if (r != ncclSuccess) {
        set_err("ncclCommInitRank: %s", ncclGetErrorString(r));
        return OSGPU_ERCCL;
    }
    g_rccl.world = comm;
    g_rccl.npes = npes;
    g_rccl.me = me;
    return OSGPU_OK;
}

int osgpu_rccl_comm_info(int *nranks, int *rank, int *device)
{
    if (!g_rccl.world) {
        set_err("osgpu_rccl_comm_info: no communicator (osgpu_rccl_init)");
        return OSGPU_EINVAL;
    }
    int n = -1, r = -1, d = -1;
    ncclResult_t e = ncclCommCount(g_rccl.world, &n);
    if (e == ncclSuccess) e = ncclCommUserRank(g_rccl.world, &r);
    if (e == ncclSuccess) e = ncclCommCuDevice(g_rccl.world, &d);
    if (e != ncclSuccess) {
        set_err("ncclCommCount / UserRank / CuDevice: %s", ncclGetErrorString(e));
        return OSGPU_ERCCL;
    }
    if (nranks) *nranks = n;
    if (rank) *rank = r;
    if (device) *device = d;
    return OSGPU_OK;
}

int osgpu_device_identity(char *out, size_t out_bytes)
{
    int d = -1;
    hipError_t e = hipGetDevice(&d);
    char bus[64] = {0};
    if (e == hipSuccess) e = hipDeviceGetPCIBusId(bus, (int) sizeof(bus) - 1, d);
    hipUUID u;
    if (e == hipSuccess) e = hipDeviceGetUuid(&u, d);
    if (e != hipSuccess) {
        set_err("osgpu_device_identity: %s", hipGetErrorString(e));
        (void) hipGetLastError();
        return OSGPU_EHIP;
    }
    char hex[2 * sizeof(u.bytes) + 1];
    for (size_t i = 0; i < sizeof(u.bytes); i++)
        snprintf(hex + 2 * i, 3, "%02x", (unsigned) (unsigned char) u.bytes[i]);
    const int need = snprintf(out, out_bytes, "{\"device\": %d, \"pci_bus_id\": \"%s\", \"uuid\": \"%s\"}",
                              d, bus, hex);
    if (need < 0 || (size_t) need >= out_bytes) {
        set_err("osgpu_device_identity: the report needs %d bytes", need + 1);
        return OSGPU_EINVAL;
    }
    return OSGPU_OK;
}

int osgpu_rccl_finalize(void)
{
    if (!g_rccl.world) return OSGPU_OK;
    ncclResult_t r = ncclCommDestroy(g_rccl.world);
    g_rccl = Rccl();
    return r == ncclSuccess ? OSGPU_OK : OSGPU_ERCCL;
}

int osgpu_finalize(void)
{
    // fused launches may still be retiring after their calls returned
    (void) hipDeviceSynchronize();
    std::lock_guard<std::mutex> lk(g_mu);
    for (auto &kv : g_stage) {
        StageSet &S = kv.second;
        for (void *p : S.opened) (void) hipIpcCloseMemHandle(p);
        if (S.local) (void) hipFree(S.local);
        for (int s = 0; s < 2; s++) {
            if (S.ev_in[s]) (void) hipEventDestroy(S.ev_in[s]);
            if (S.ev_out[s]) (void) hipEventDestroy(S.ev_out[s]);
        }
        if (S.st_c && S.own_c) (void) hipStreamDestroy(S.st_c);
    }
    g_stage.clear();
    for (auto &kv : g_copy_streams) {  // shared by the staging sets above
        if (kv.second.first) (void) hipStreamDestroy(kv.second.first);
        if (kv.second.second) (void) hipStreamDestroy(kv.second.second);
    }
    g_copy_streams.clear();
    for (auto &kv : g_sync) {
        SyncSet &S = kv.second;
        for (void *p : S.opened) (void) hipIpcCloseMemHandle(p);
        if (S.local) (void) hipFree(S.local);
        if (S.err_h) (void) hipHostFree(S.err_h);
    }
    g_sync.clear();
    for (auto &kv : g_pectx) {
        PeCtx *x = kv.second;
        if (x->dscratch) (void) hipFree(x->dscratch);
        if (x->hstage) (void) hipHostFree(x->hstage);
        if (x->stream) (void) hipStreamDestroy(x->stream);
        delete x;
    }
    g_pectx.clear();
    (void) hipGetLastError();
    return OSGPU_OK;
}

int osgpu_host_register(void *base, size_t bytes)
{
    hipError_t e = hipHostRegister(base, bytes, hipHostRegisterMapped);
    if (e != hipSuccess) {
        set_err("hipHostRegister: %s", hipGetErrorString(e));
        return OSGPU_EHIP;
    }
    void *dev = nullptr;
    if (hipHostGetDevicePointer(&dev, base, 0) != hipSuccess) {
        (void) hipGetLastError();
        dev = nullptr;
    }
    std::lock_guard<std::mutex> lk(g_mu);
    g_hostreg.push_back({(char *) base, bytes, (char *) dev});
    return OSGPU_OK;
}

int osgpu_host_unregister(void *base)
{
    hipError_t e = hipHostUnregister(base);
    {
        std::lock_guard<std::mutex> lk(g_mu);
        for (size_t i = 0; i < g_hostreg.size(); i++)
            if (g_hostreg[i].base == (char *) base) {
                g_hostreg.erase(g_hostreg.begin() + (long) i);
                break;
            }
    }
    if (e != hipSuccess) {
        set_err("hipHostUnregister: %s", hipGetErrorString(e));
        return OSGPU_EHIP;
    }
    return OSGPU_OK;
}

int osgpu_set_path(int path)
{
    if (path < OSGPU_PATH_AUTO || path > OSGPU_PATH_PULL) return OSGPU_EINVAL;
    std::lock_guard<std::mutex> lk(g_mu);
    g_path = path;
    return OSGPU_OK;
}

int osgpu_set_fused_max_bytes(long long bytes)
{
    std::lock_guard<std::mutex> lk(g_mu);
    g_fused_max = bytes < 0 ? -1 : bytes;
    return OSGPU_OK;
}

int osgpu_set_host_path(int mode)
{
    if (mode < -1 || mode > OSGPU_HOST_GETMEM) return OSGPU_EINVAL;
    std::lock_guard<std::mutex> lk(g_mu);
    g_host_path = mode;
    return OSGPU_OK;
}

int osgpu_set_host_fold_max_bytes(long long bytes)
{
    std::lock_guard<std::mutex> lk(g_mu);
    g_host_fold_max = bytes < 0 ? -1 : bytes;
    return OSGPU_OK;
}

int osgpu_set_stage_copy(int mode)
{
    if (mode < -1 || mode > 2) return OSGPU_EINVAL;
    std::lock_guard<std::mutex> lk(g_mu);
    g_stage_copy = mode;
    return OSGPU_OK;
}

int osgpu_set_stage_bytes(long long bytes)
{
    std::lock_guard<std::mutex> lk(g_mu);
    g_stage_bytes = bytes <= 0 ? -1 : bytes;
    return OSGPU_OK;
}

int osgpu_set_host_chunk_bytes(long long bytes)
{
    std::lock_guard<std::mutex> lk(g_mu);
    g_host_chunk = bytes <= 0 ? -1 : bytes;
    return OSGPU_OK;
}

int osgpu_set_team_exchange(int mode)
{
    if (mode < -1 || mode > 1) return OSGPU_EINVAL;
    std::lock_guard<std::mutex> lk(g_mu);
    g_team_exchange = mode;
    return OSGPU_OK;
}

int osgpu_set_device_barrier(double timeout_s, int fatal_on_timeout)
{
    std::lock_guard<std::mutex> lk(g_mu);
    g_dbar_secs = timeout_s;
    g_dbar_fatal = fatal_on_timeout ? 1 : 0;
    return OSGPU_OK;
}

int osgpu_set_stream(void *hip_stream)
{
    t_ctx.stream = (hipStream_t) hip_stream;
    t_ctx.user_stream = hip_stream != nullptr;
    if (!hip_stream) t_ctx.device = -1;
    return OSGPU_OK;
}

void *osgpu_get_stream(void)
{
    return (void *) thread_stream("osgpu_get_stream");
}

int osgpu_combine(int type, int op, void *target, const void *const *srcs, int nsrc,
                  size_t nelems, void *hip_stream)
{
    if (!has_op(type, op) || nsrc < 1 || !target || !srcs) {
        set_err("osgpu_combine: bad arguments");
        return OSGPU_EINVAL;
    }
    hipStream_t st = hip_stream ? (hipStream_t) hip_stream : thread_stream("osgpu_combine");
    hipError_t e = osgpu::launch_combine(type, op, target, srcs, nsrc, nelems, st);
    if (e == hipErrorNotSupported) {
        set_err("osgpu_combine: type %d op %d not supported on the GPU", type, op);
        return OSGPU_ENOTSUP;
    }
    if (e != hipSuccess) {
        set_err("osgpu_combine: %s", hipGetErrorString(e));
        return OSGPU_EHIP;
    }
    return OSGPU_OK;
}

int osgpu_team_combine(int type, int op, int P, void *const *dsts, const void *const *srcs,
                       size_t nelems, void *hip_stream)
{
    return osgpu_team_combine_shape(type, op, P, dsts, srcs, nelems, hip_stream, 0);
}

int osgpu_team_combine_shape(int type, int op, int P, void *const *dsts, const void *const *srcs,
                             size_t nelems, void *hip_stream, int remote)
{
    if (!has_op(type, op) || P < 2 || P > osgpu::kMaxTeam || !dsts || !srcs) {
        set_err("osgpu_team_combine: bad arguments");
        return OSGPU_EINVAL;
    }
    hipStream_t st = hip_stream ? (hipStream_t) hip_stream : thread_stream("osgpu_team_combine");
    hipError_t e = osgpu::launch_team(type, op, P, dsts, srcs, nelems, st, remote != 0);
    if (e != hipSuccess) {
        set_err("osgpu_team_combine: %s", hipGetErrorString(e));
        return OSGPU_EHIP;
    }
    return OSGPU_OK;
}

int osgpu_copy(void *const *dsts, const void *const *srcs, const size_t *bytes, int n,
               void *hip_stream)
{
    if (n < 0 || (n > 0 && (!dsts || !srcs || !bytes))) {
        set_err("osgpu_copy: bad arguments");
        return OSGPU_EINVAL;
    }
    hipStream_t st = hip_stream ? (hipStream_t) hip_stream : thread_stream("osgpu_copy");
    for (int i = 0; i < n; i += osgpu::kMaxCopySegs) {
        osgpu::CopySeg seg[osgpu::kMaxCopySegs];
        const int m = n - i < osgpu::kMaxCopySegs ? n - i : osgpu::kMaxCopySegs;
        for (int j = 0; j < m; j++) seg[j] = {srcs[i + j], dsts[i + j], bytes[i + j]};
        hipError_t e = osgpu::launch_copy(seg, m, st);
        if (e != hipSuccess) {
            set_err("osgpu_copy: %s", hipGetErrorString(e));
            return OSGPU_EHIP;
        }
    }
    return OSGPU_OK;
}

// result words of the verification launchers, per thread and device
struct VerifyBuf {
    int device = -1;
    unsigned long long *d = nullptr, *h = nullptr;
};
thread_local VerifyBuf t_vbuf;

static int verify_begin(const char *where, void *hip_stream, hipStream_t *st)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) {
        set_err("%s: no GPU", where);
        return OSGPU_EHIP;
    }
    if (!t_vbuf.d || t_vbuf.device != dev) {
        if (hipMalloc((void **) &t_vbuf.d, 2 * sizeof(unsigned long long)) != hipSuccess ||
            hipHostMalloc((void **) &t_vbuf.h, 2 * sizeof(unsigned long long),
                          hipHostMallocDefault) != hipSuccess) {
            set_err("%s: out of memory", where);
            return OSGPU_EHIP;
        }
        t_vbuf.device = dev;
    }
    *st = hip_stream ? (hipStream_t) hip_stream : thread_stream(where);
    return OSGPU_OK;
}

static int verify_end(const char *where, hipError_t e, hipStream_t st)
{
    if (e == hipSuccess)
        e = hipMemcpyAsync(t_vbuf.h, t_vbuf.d, 2 * sizeof(unsigned long long),
                           hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        set_err("%s: %s", where, hipGetErrorString(e));
        return OSGPU_EHIP;
    }
    return OSGPU_OK;
}

int osgpu_checksum(int type, int mode, const void *data, size_t nelems, void *hip_stream,
                   unsigned long long *result)
{
    const size_t es = type_size(type);
    if (!es || mode < 0 || mode > 2 || !result || (!data && nelems)) {
        set_err("osgpu_checksum: bad arguments");
        return OSGPU_EINVAL;
    }
    hipStream_t st;
    int rc = verify_begin("osgpu_checksum", hip_stream, &st);
    if (rc) return rc;
    hipError_t e = hipMemsetAsync(t_vbuf.d, 0, 2 * sizeof(unsigned long long), st);
    if (e == hipSuccess && nelems)
        e = osgpu::launch_checksum((int) es, mode, data, nelems, t_vbuf.d, st);
    if ((rc = verify_end("osgpu_checksum", e, st))) return rc;
    *result = t_vbuf.h[0];
    return OSGPU_OK;
}

int osgpu_compare(const void *a, const void *b, size_t nbytes, void *hip_stream,
                  unsigned long long *mismatches, unsigned long long *first_offset)
{
    if (!mismatches || (nbytes && (!a || !b))) {
        set_err("osgpu_compare: bad arguments");
        return OSGPU_EINVAL;
    }
    hipStream_t st;
    int rc = verify_begin("osgpu_compare", hip_stream, &st);
    if (rc) return rc;
    hipError_t e = hipMemsetAsync(t_vbuf.d, 0, sizeof(unsigned long long), st);
    if (e == hipSuccess)
        e = hipMemsetAsync(t_vbuf.d + 1, 0xff, sizeof(unsigned long long), st);
    if (e == hipSuccess && nbytes) e = osgpu::launch_compare(a, b, nbytes, t_vbuf.d, st);
    if ((rc = verify_end("osgpu_compare", e, st))) return rc;
    *mismatches = t_vbuf.h[0];
    if (first_offset) *first_offset = t_vbuf.h[1];
    return OSGPU_OK;
}

int osgpu_has_op(int type, int op) { return has_op(type, op) ? 1 : 0; }

size_t osgpu_type_size(int type) { return type_size(type); }

int osgpu_fold_order(int me, int PE_start, int logPE_stride, int PE_size, int *order_out)
{
    if (PE_size < 1 || logPE_stride < 0 || logPE_stride > 30 || !order_out)
        return OSGPU_EINVAL;
    const int step = 1 << logPE_stride;
    bool member = false;
    for (int i = 0; i < PE_size; i++) member |= (PE_start + i * step == me);
    if (!member) return OSGPU_EINVAL;
    fold_order(me, PE_start, step, PE_size, order_out);
    return OSGPU_OK;
}

int osgpu_shard_range(long long nreduce, int PE_size, int idx, int elem_bytes, long long *lo,
                      long long *hi)
{
    if (nreduce < 0 || PE_size < 1 || idx < 0 || idx >= PE_size || elem_bytes < 1 ||
        elem_bytes > 16 || !lo || !hi)
        return OSGPU_EINVAL;
    // shard boundaries on 16-byte vector granules so every shard stays on
    // the vector path; the last shard takes the ragged remainder
    const long long g = elem_bytes >= 16 ? 1 : 16 / elem_bytes;
    const long long granules = nreduce / g;
    const long long base = granules / PE_size, rem = granules % PE_size;
    const long long start = idx * base + (idx < rem ? idx : rem);
    const long long cnt = base + (idx < rem ? 1 : 0);
    *lo = start * g;
    *hi = (idx == PE_size - 1) ? nreduce : (start + cnt) * g;
    return OSGPU_OK;
}

int osgpu_last_continuations(void) { return t_continuations; }

const char *osgpu_last_error(void) { return g_err; }

const char *osgpu_version(void) { return "osgpu_reduce 0.2 (gfx950)"; }

#ifndef OSGPU_BUILD_ID
#define OSGPU_BUILD_ID "unknown"
#endif
const char *osgpu_build_id(void) { return OSGPU_BUILD_ID; }

}  // extern "C"
