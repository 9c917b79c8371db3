// combine.hpp -- internal interface between the C-ABI layer and the kernels.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stddef.h>

namespace osgpu {

// 16-byte vectors in flight per lane per input of the register-form combine
// for <= 2, <= 4 and <= 8 inputs (register budget vs bytes in flight;
// tools/tune_combine.hip)
constexpr int kUK2 = 4, kUK4 = 4, kUK8 = 4;

// type codes (same numbering as include/osgpu_reduce.h OSGPU_T_*)
enum TypeCode {
    T_SHORT = 0, T_INT, T_LONG, T_LONGLONG, T_FLOAT, T_DOUBLE, T_LONGDOUBLE,
    T_COMPLEXF, T_COMPLEXD, T_NTYPES
};

// out[i] = fold(op, srcs[0][i], srcs[1][i], ..., srcs[k-1][i]) for i < n,
// enqueued on stream s.  All pointers are device-accessible (local HBM or a
// peer GPU's HBM mapped into this process).  `out` may alias srcs[0].
hipError_t launch_combine(int type, int op, void *out, const void *const *srcs, int k,
                          size_t n, hipStream_t s);

// Owner-computes team combine over an active set of P PEs (2 <= P <= 8):
// for i < n, dsts[q][i] = fold of srcs[*][i] in PE q's order (q first, then
// ascending, skipping q).  srcs/dsts indexed by position in the active set
// and already offset to this PE's shard.
// remote: some member's arrays live in another GPU's HBM (xGMI) -- the team
// kernel then takes the shapes last measured across GPUs (team.hip TeamShape)
constexpr int kMaxTeam = 8;

// Threads per launch of the one-tile-per-workgroup kernels (combine_lds,
// combine_vec, team_lds, team_vec): a grid's thread count must stay below
// 2^32 (HIP refuses larger grids: an 8-member team call of 1 Gi doubles,
// config 4's shape, needs 2^32 threads in the LDS form), so a larger call
// runs as several launches over consecutive runs of tiles.
constexpr size_t kMaxLaunchThreads = (size_t) 1 << 31;
// the limit in force: kMaxLaunchThreads, or a smaller one a test set
// (osgpu_test_max_launch_threads) to run the multi-launch path at small sizes
size_t max_launch_threads();
void set_max_launch_threads(size_t n);
hipError_t launch_team(int type, int op, int P, void *const *dsts, const void *const *srcs,
                       size_t n, hipStream_t s, bool remote = false);
hipError_t launch_team_longdouble(int op, int P, void *const *dsts, const void *const *srcs,
                                  size_t n, hipStream_t s);
// The same over [0, n) split by tiles instead of contiguous shards: of m
// members sharing one GPU, member k folds the tiles k, k + m, k + 2m, ...
// (a tile = one workgroup's vectors), so their concurrent grids stream the
// same address range together (run_team).  m = 1, k = 0: launch_team.
// hipErrorNotSupported for long double (contiguous shards only).
hipError_t launch_team_tiles(int type, int op, int P, void *const *dsts, const void *const *srcs,
                             size_t n, int m, int k, hipStream_t s, bool remote = false);

// Byte copy of up to kMaxCopySegs independent ranges in one launch (copy.hip):
// the data movement of broadcast / collect / fcollect / alltoall.  Sources may
// be peer HBM.  Zero-length segments are skipped; more than kMaxCopySegs
// non-empty segments is an error (callers batch).
constexpr int kMaxCopySegs = 8;
struct CopySeg {
    const void *src;
    void *dst;
    size_t bytes;
};
hipError_t launch_copy(const CopySeg *segs, int nseg, hipStream_t s);
// Host fold of small host-heap calls (host_fold.hip): acc[i] = op(acc[i],
// in[i]) for i < n with the kernels' element ops compiled for the host
bool host_fold_supported(int type, int op);
bool host_fold(int type, int op, void *acc, const void *in, size_t n);
// One range between HBM and pinned host memory mapped into the GPU (either
// side may be the host's device view): a fixed grid (OSGPU_HOST_COPY_GRID,
// default 256 workgroups) sized for one PCIe link, not for HBM (copy.hip)
hipError_t launch_host_copy(void *dst, const void *src, size_t bytes, hipStream_t s);
// <= kProbeLoadBytes of 8-byte words read with plain (L2-cached) loads into dst
constexpr size_t kProbeLoadBytes = 2048;
hipError_t launch_probe_load(const void *src, void *dst, size_t bytes, hipStream_t s);

// One-launch reduce-to-all for small calls (fused.hip): the call's two
// barriers run inside the kernel as epoch flags in every member's flag area
// (uncached device memory, mapped into every member).  Word layout of a
// flag area (unsigned long long):
constexpr int kFlagArrive = 0;    // [0, 8): arrive[member]
constexpr int kFlagDone = 8;      // [8, 16): done[member]
constexpr int kFlagTicket = 16;   // last-workgroup tickets (u32): completion,
constexpr int kFlagTicketIn = 17;  //   staged copy-in,
constexpr int kFlagTicketOut = 18; //   staged copy-out
constexpr int kFlagCount = 20;    // [20, 28): count[member] (collect: tag << 40 | source bytes)
constexpr int kFlagGateIn = 28;   // entry gate: (epoch << 20 | attempt << 1 | go), my grid's
constexpr int kFlagGateOut = 29;  //   verdict on the entry / exit wait (one decider per grid)
constexpr int kCountBits = 40;
constexpr int kFlagWords = 32;
// fused grids: at most one workgroup of 256 lanes per CU of the GPU (256 on
// MI355X), split between the members sharing it (one member per GPU: all)
constexpr int kFusedBlocksPerGpu = 256;
struct FusedArgs {
    const void *src[kMaxTeam];            // every member's source, active-set order
    void *dst[kMaxTeam];                  // outputs: team form every member's target, pull form mine
    int q[kMaxTeam];                      // active-set index whose fold order dst[d] uses
    unsigned long long *flags[kMaxTeam];  // every member's flag area
    unsigned long long *mine;             // my flag area
    int *err;                             // host-mapped: 1 arrive / 2 done not passed in time
    unsigned long long *done_host;        // host-mapped: epoch, written once the call is complete
    unsigned long long epoch, timeout;    // timeout: one wait slice, in wall-clock ticks
    int resume;                           // 0 first launch, 1 continue at the entry barrier,
                                          //   2 continue at the exit barrier
    unsigned attempt;                     // launches of this call so far (gate keys)
    size_t n;                             // elements from src[p] / dst[d]
    size_t nvec, head, tail_start;        // filled by launch_fused
    int nedge, P, D, me;                  // me: my active-set index
    int max_blocks;                       // grid cap (co-residency on a shared GPU)
    unsigned long long *trace;            // optional host-mapped phase clock (8 words)
    // staged form (host memory): null host_in = device form
    const void *host_in;                  // my host source (device-accessible)
    void *host_out;                       // my host target (device-accessible)
    void *stage_mine;                     // my input staging slot (= src[me])
    const void *stage_result;             // my result staging slot (= one of dst[])
    size_t host_bytes;
    // copy form (launch_fused_copy): nseg segments src[d] -> dst[d]
    size_t seg_bytes[kMaxTeam];
    int nseg;
    // collect form (launch_fused_collect): src[i] every member's source,
    // dst[0] my output; contributions differ per member and are exchanged
    // in the flag areas at arrival
    size_t my_count;                      // bytes of my source (< 2^kCountBits)
    unsigned long long count_tag;         // the set's collect sequence number
    size_t src_avail[kMaxTeam];           // bytes mapped from src[i] (bounds)
    size_t copy_limit;                    // copy in the launch iff the total fits
    unsigned long long *counts_host;      // host-mapped: every member's count, then
                                          //   counts_host[kMaxTeam] = 1 if copied
};
bool fused_supported(int type);
hipError_t launch_fused_copy(const FusedArgs &a, hipStream_t s);
hipError_t launch_fused_collect(const FusedArgs &a, hipStream_t s);
hipError_t launch_fused(int type, int op, const FusedArgs &a, hipStream_t s);

// Full-size parity checks on the GPU (verify.hip).  Checksum of n elements
// of elem_bytes (2, 4, 8, 16) into *out (device memory, zeroed by the
// caller): CK_SUM adds the zero-extended elements mod 2^64, CK_XOR xors
// them, CK_HASH adds a position-weighted mix of each element's bits.
// Compare: out[0] += differing 16-B vectors (bytes when unaligned), out[1]
// = min(out[1], byte offset of the first difference); out[1] preset to ~0.
enum { CK_SUM = 0, CK_XOR = 1, CK_HASH = 2 };
hipError_t launch_checksum(int elem_bytes, int mode, const void *p, size_t n,
                           unsigned long long *out, hipStream_t s);
hipError_t launch_compare(const void *a, const void *b, size_t nbytes, unsigned long long *out,
                          hipStream_t s);

// x87 80-bit extended combine (soft-float on the GPU), longdouble.hip
hipError_t launch_longdouble(int op, void *out, const void *const *srcs, int k, size_t n,
                             hipStream_t s);

}  // namespace osgpu
