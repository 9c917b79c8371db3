// runtime.hpp -- internal services shared by the collectives of
// libosgpu_reduce.so (runtime.cpp): error reporting, stream completion, the
// OpenSHMEM PE services the library borrows from the application's runtime,
// the device symmetric-heap registry, per-PE streams/scratch, the RCCL
// communicator, and the host-staging sets of the STAGED paths.
// Not installed: the public surface is include/osgpu_reduce.h.
#pragma once
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <stdio.h>
#include <unistd.h>

#include <functional>
#include <vector>

#include "combine.hpp"

namespace osgpu {
namespace rt {

// ------------------------------------------------------------------ errors

void set_err(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
[[noreturn]] void fatal(const char *where, const char *fmt, ...)
    __attribute__((format(printf, 2, 3)));
int debug_level();

// OSGPU_DEBUG=1: one stderr line per protocol step (call entry, path,
// barriers, launches, syncs) -- for diagnosing multi-process runs
#define DBG(...)                                                               \
    do {                                                                       \
        if (::osgpu::rt::debug_level() > 0) {                                  \
            fprintf(stderr, "[osgpu pid %d] ", (int) getpid());                \
            fprintf(stderr, __VA_ARGS__);                                      \
            fputc('\n', stderr);                                               \
            fflush(stderr);                                                    \
        }                                                                      \
    } while (0)

#define HIPCHK(where, call)                                                    \
    do {                                                                       \
        hipError_t e_ = (call);                                                \
        if (e_ != hipSuccess)                                                  \
            ::osgpu::rt::fatal(where, "%s: %s", #call, hipGetErrorString(e_)); \
    } while (0)

// ----------------------------------------------------------- synchronisation

int env_choice(const char *var, const char *alt, int def_is_alt);
enum { ENTRY_DEVICE = 0, ENTRY_SPIN, ENTRY_STREAM, ENTRY_NONE };
int entry_mode();
void entry_sync(const char *where, hipStream_t own = nullptr);
void entry_order(const char *where, hipStream_t st);
void stream_wait(const char *where, hipStream_t st);
void call_trace(int me, int phase, const char *label);

// --------------------------------------------------------------- type info

size_t type_size(int t);
bool has_op(int t, int op);

// ------------------------------------------------------------- PE services

struct PeOps {
    int (*my_pe)(void) = nullptr;
    int (*n_pes)(void) = nullptr;
    void (*barrier)(int, int, int, long *) = nullptr;
    void (*getmem)(void *, const void *, size_t, int) = nullptr;
};
PeOps pe_ops();

// -------------------------------------------------------- device sym. heap

struct HeapEntry {
    char *base = nullptr;
    size_t bytes = 0;
    bool remote = false;  // backed by another GPU's HBM (osgpu_heap_create knows)
};
bool heap_segment(int pe, int seg, HeapEntry *out);
bool heap_locate(int pe, const void *addr, size_t nbytes, int *seg, size_t *off);
bool heap_peer(int pe, int seg, size_t off, size_t nbytes, char **out, bool *remote = nullptr);
void heap_set_remote(int pe, int seg, bool remote);
// PCI location of a device: PEs with equal keys share one GPU and its link
long pci_key(int dev);
// [p, p + n) inside a heap made by osgpu_heap_create (heap.cpp) -- the PE's
// own range (*dev = its device) or a member's mapped here (*dev = -1)
bool heap_created_range(const void *p, size_t n, int *dev);
// lowest segment index unused by every PE of `pes` (this process's registry)
int heap_free_segment(const std::vector<int> &pes);
void heap_clear_segment(int pe, int seg);

// ---------------------------------------------------------------- RCCL

struct Rccl {
    ncclComm_t world = nullptr;
    int npes = 0, me = -1;
};
extern Rccl g_rccl;
int path_mode();

// ------------------------------------------------------ per-PE / per-thread

hipStream_t thread_stream(const char *where);
hipStream_t pe_stream(const char *where, int me);
void *device_scratch(const char *where, int me, size_t bytes);
void *host_stage(const char *where, int me, size_t bytes);

enum MemKind { MEM_HOST = 0, MEM_DEVICE = 1 };
MemKind mem_kind(const void *p, int *dev);
bool ranges_overlap(const void *a, const void *b, size_t n);
void fold_order(int me, int PE_start, int step, int PE_size, int *order);

// ------------------------------------------------------------ active sets

// One collective call on an active set (PE_start, 2^logPE_stride, PE_size).
struct Coll {
    const char *name = nullptr;
    int PE_start = 0, logPE_stride = 0, PE_size = 0;
    long *pSync = nullptr;
    int me = -1, step = 1;
    PeOps ops;
    // index of PE `pe` in the active set, or -1
    int index_of(int pe) const
    {
        if (pe < PE_start || (pe - PE_start) % step) return -1;
        const int i = (pe - PE_start) / step;
        return i < PE_size ? i : -1;
    }
    int pe_at(int i) const { return PE_start + i * step; }
};

// Fills name/active set/pSync/me/ops; aborts on an invalid active set or a
// missing runtime (the shared entry checks of every collective).
Coll make_coll(const char *name, int PE_start, int logPE_stride, int PE_size, long *pSync);

void barrier(const Coll &c);

// ---------------------------------------------------------- host staging

// pinned (registered or hipHostMalloc) host memory?
bool host_pinned(const void *p);
// memcpy split over OSGPU_COPY_THREADS threads (default 4) for large copies
void par_memcpy(void *dst, const void *src, size_t n);

// Device staging of one PE for one active set: four slots of `slot` bytes,
// mapped into every member PE (same process: raw pointer; other processes:
// HIP IPC), exchanged once through spare pSync words (runtime.cpp).
struct StageSet {
    bool ok = false;
    int device = -1;
    int ndev = 0;                    // distinct GPUs (PCI locations) among the members
    size_t slot = 0;                 // bytes per slot (in0, in1, out0, out1)
    char *local = nullptr;
    std::vector<char *> peer;        // by active-set index
    std::vector<void *> opened;      // IPC mappings to close
    hipStream_t st_in = nullptr, st_c = nullptr, st_out = nullptr;
    bool own_c = false;              // st_c created for this set (else the PE's stream)
    hipEvent_t ev_in[2] = {nullptr, nullptr}, ev_out[2] = {nullptr, nullptr};
    char *in(int i, int s) const { return peer[i] + (size_t) s * slot; }
    char *out(int i, int s) const { return peer[i] + (size_t) (2 + s) * slot; }
    char *region(int i) const { return peer[i]; }  // the whole 4-slot area
};
StageSet *stage_setup(const Coll &c);

// Publish a device allocation to every member of the active set and map
// every member's (collective; the same verdict on every member).
// distinct_processes: fail unless every member is its own process.
// max_share: the largest number of members on one GPU.  procs_here: the
// processes among the members on this process's GPU (this one included).
bool map_members(const Coll &c, char *local, size_t bytes, std::vector<char *> &peer,
                 std::vector<void *> &opened, int *ndev, bool distinct_processes,
                 int *max_share, int *procs_here = nullptr);

// ------------------------------------------------- device-side barriers

// Flag areas of one PE for one active set (fused.hip protocol): mine and
// every member's, mapped.  `epoch` counts the fused calls made on the set.
struct SyncSet {
    bool ok = false;
    int idx = -1;                              // my active-set index
    unsigned long long *local = nullptr;       // my flag area (uncached HBM)
    std::vector<unsigned long long *> peer;    // by active-set index
    std::vector<void *> opened;                // IPC mappings to close
    unsigned long long epoch = 0;
    unsigned long long ncollect = 0;           // collect calls on the set (count tags)
    int rate_khz = 0;                          // wall clock of the device
    int max_blocks = 0;                        // workgroups per fused launch
    int *err_h = nullptr, *err_d = nullptr;    // host-mapped error word
    unsigned long long *done_h = nullptr, *done_d = nullptr;  // host-mapped completion epoch
    unsigned long long *cnt_h = nullptr, *cnt_d = nullptr;    // host-mapped collect counts
};
SyncSet *sync_setup(const Coll &c);
// Launch a fused call (`launch(a)` on stream st, a.epoch set) and drive it to
// completion: whenever the launch ended at a device barrier that a member
// had not reached within one wait slice, launch its continuation there
// (a.resume) -- the barrier waits without bound, the GPU is never held for
// more than a slice.  true: complete (the host completion word carries
// a.epoch).  false (not fatal by policy): a member stayed away longer than
// the device-barrier bound, or a collect contribution was out of bounds;
// the call failed and the set's fused path is off.
bool fused_complete(const char *where, SyncSet &S, hipStream_t st, osgpu::FusedArgs &a,
                    const std::function<hipError_t(const osgpu::FusedArgs &)> &launch);

// Team exchange form: 0 pull (remote reads, default), 1 push (remote writes
// through the members' staging inboxes); osgpu_set_team_exchange /
// OSGPU_TEAM_EXCHANGE.
int team_exchange();

// Device view of host memory inside a range pinned with
// osgpu_host_register, or nullptr.
void *host_device_view(const void *p, size_t nbytes);

// Per-PE byte limit of the fused path: osgpu_set_fused_max_bytes, else
// OSGPU_FUSED_MAX_BYTES, else 1 MiB; 0 = fused path off.
size_t fused_max_bytes();
// host symmetric-heap calls: OSGPU_HOST_AUTO / _STAGED / _GETMEM
// (osgpu_set_host_path), the host fold's per-PE limit, the STAGED legs'
// copy mode (0 dma, 1 kout, 2 kernel) and the GETMEM path's chunk
int host_path();
size_t host_fold_max_bytes();
int stage_copy_mode();
size_t host_chunk_bytes();

}  // namespace rt
}  // namespace osgpu
