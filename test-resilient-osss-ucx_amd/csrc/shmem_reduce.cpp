// shmem_reduce.cpp -- C-ABI layer of libosgpu_reduce.so.
//
// Replaces the reduce-to-all entry points of the reference
// (SHMEM_REDUCE_TYPE_OP, src/reductions.c:139-154, instantiated at :248-297)
// with the same 44 signatures.  Where the reference walks its peers with a
// blocking 64-element shmem_getmem per chunk and folds through a function
// pointer per element (udr_<T>_to_all, src/reductions.c:32-120), this layer
// picks one of these MI355X paths:
//
//   TEAM    device-resident, source and target symmetric in registered
//           heaps, 2..8 PEs: owner-computes kernel (team.hip) -- PE g folds
//           shard g of every PE's target, each in that PE's own fold order,
//           reading every source once over HBM/xGMI (bit-exact);
//   PULL    device-resident, source symmetric: the reference's pull
//           schedule as ONE combine kernel streaming all PE_size sources in
//           the PE's fold order (bit-exact);
//   RCCL    device-resident, one process per GPU with an RCCL communicator:
//           ncclAllReduce over xGMI (FP within tolerance);
//   STAGED  host symmetric-heap arguments: H2D own source -> TEAM over
//           IPC-mapped device staging -> D2H, pipelined (bit-exact);
//   GETMEM  host arguments when staging cannot be mapped by every PE: peers'
//           sources pulled with the runtime's shmem_getmem, H2D, combine, D2H.
//
// The two shmem_barrier calls of the reference (:82, :113) keep their roles
// (every source ready / every reader or writer done) on every non-RCCL path.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <thread>
#include <tuple>
#include <vector>

#include "../../include/osgpu_reduce.h"
#include "combine.hpp"
#include "runtime.hpp"

namespace {

using namespace osgpu::rt;

thread_local int t_last_path = OSGPU_RAN_NONE;

// ------------------------------------------------------------- the paths

// one reduce-to-all call: the active set (Coll) plus the arrays
struct Call : Coll {
    int type = 0, op = 0;
    void *target = nullptr, *source = nullptr;
    int nreduce = 0;
    size_t nbytes = 0;
};

bool p2p_sources(const Call &c, std::vector<const void *> &srcs)
{
    int seg = -1;
    size_t off = 0;
    if (!heap_locate(c.me, c.source, c.nbytes, &seg, &off)) return false;
    std::vector<int> order(c.PE_size);
    fold_order(c.me, c.PE_start, c.step, c.PE_size, order.data());
    srcs.resize(c.PE_size);
    for (int k = 0; k < c.PE_size; k++) {
        char *p = nullptr;
        if (!heap_peer(order[k], seg, off, c.nbytes, &p)) return false;
        srcs[k] = p;
    }
    return true;
}

// every member's source in active-set order (the fused pull form)
bool member_sources(const Call &c, std::vector<const void *> &srcs)
{
    int seg = -1;
    size_t off = 0;
    if (!heap_locate(c.me, c.source, c.nbytes, &seg, &off)) return false;
    srcs.resize(c.PE_size);
    for (int i = 0, pe = c.PE_start; i < c.PE_size; i++, pe += c.step) {
        char *p = nullptr;
        if (!heap_peer(pe, seg, off, c.nbytes, &p)) return false;
        srcs[i] = p;
    }
    return true;
}

// Owner-computes team path (team.hip): needs both source and target inside
// every active PE's registered heap at the same offsets (symmetric), no
// overlap between them, and 2 <= PE_size <= 8.  Fills srcs/dsts in active-set
// order and returns this PE's index, or -1.
int team_ptrs(const Call &c, std::vector<const void *> &srcs, std::vector<void *> &dsts,
              bool *remote = nullptr)
{
    if (c.PE_size < 2 || c.PE_size > osgpu::kMaxTeam) return -1;
    if (ranges_overlap(c.target, c.source, c.nbytes)) return -1;
    int ss = -1, st = -1;
    size_t os = 0, ot = 0;
    if (!heap_locate(c.me, c.source, c.nbytes, &ss, &os)) return -1;
    if (!heap_locate(c.me, c.target, c.nbytes, &st, &ot)) return -1;
    srcs.resize(c.PE_size);
    dsts.resize(c.PE_size);
    int idx = -1;
    bool far = false;
    for (int i = 0, pe = c.PE_start; i < c.PE_size; i++, pe += c.step) {
        char *sp = nullptr, *tp = nullptr;
        bool rs = false, rt_ = false;
        if (!heap_peer(pe, ss, os, c.nbytes, &sp, &rs) || !heap_peer(pe, st, ot, c.nbytes, &tp, &rt_))
            return -1;
        srcs[i] = sp;
        dsts[i] = tp;
        far = far || rs || rt_;
        if (pe == c.me) idx = i;
    }
    if (remote) *remote = far;
    return idx;
}

// Members of one active set that are threads of THIS process on the same
// GPU (threads-as-PEs; mixed topologies): each registers its call here
// before the entry barrier, so after it every local member is known, and a
// run of consecutive local members [first, last] folds the union of their
// shards split by TILES (launch_team_tiles: member k of m takes the tiles k,
// k + m, ...) instead of one contiguous shard each.  Their grids share the
// GPU; with contiguous shards the two concurrent half-grids of a 2-PE call
// streamed two distant ranges and ended ~16 us apart, the whole call taking
// ~6 % longer than one full grid (profiles/r04_call_overhead_1..4.jsonl).
// Calls on a set are matched by a sequence number kept per (set, device,
// PE) in this process -- not per OS thread, so a PE whose calls move
// between threads (a thread pool) keeps its count: OpenSHMEM members call
// a set's collectives in the same order.
// OSGPU_TEAM_LOCAL: merge (the default: the run's first member launches one
// grid over the whole run, the others only wait in the barriers) | shards
// (contiguous shards always) | tiles.  A 2-PE 64 Mi-double call: merged
// 379-384 us, 376.5-376.8 with OSGPU_SYNC=word, shards 377-391, tiles
// 401-409 (profiles/r04_call_overhead_6.jsonl); merged + word in the bench
// 0.726 of 8 TB/s (r04_bench_merge_word.log) against 0.68-0.71.
struct LocalCall {
    unsigned mask = 0;  // active-set indices of the local members
    int left = 0;       // registered members not yet done
};
std::mutex g_local_mu;
std::map<std::tuple<int, int, int, int, unsigned long long>, LocalCall> g_local;
std::map<std::tuple<int, int, int, int, int>, unsigned long long> g_local_seq;  // + PE

enum { LOCAL_SHARDS = 0, LOCAL_TILES, LOCAL_MERGE };
int local_mode()
{
    static const int m = [] {
        const char *e = getenv("OSGPU_TEAM_LOCAL");
        if (e && !strcmp(e, "tiles")) return (int) LOCAL_TILES;
        if (e && !strcmp(e, "shards")) return (int) LOCAL_SHARDS;
        return (int) LOCAL_MERGE;
    }();
    return m;
}

void run_team(const Call &c, const std::vector<const void *> &srcs,
              const std::vector<void *> &dsts, int idx, bool remote)
{
    hipStream_t st = pe_stream(c.name, c.me);
    const size_t s = type_size(c.type);
    const int es = (int) (s > 16 ? 16 : s);
    const int mode = local_mode();
    // (long double: contiguous shards or merged runs, no tiles)
    const bool tiles = mode == LOCAL_MERGE || (mode == LOCAL_TILES && c.type != osgpu::T_LONGDOUBLE);
    std::tuple<int, int, int, int, unsigned long long> key;
    if (tiles) {
        int dev = 0;
        HIPCHK(c.name, hipGetDevice(&dev));
        const auto set = std::make_tuple(c.PE_start, c.step, c.PE_size, dev);
        std::lock_guard<std::mutex> lk(g_local_mu);
        const unsigned long long seq = ++g_local_seq[std::tuple_cat(set, std::make_tuple(c.me))];
        key = std::tuple_cat(set, std::make_tuple(seq));
        LocalCall &L = g_local[key];
        L.mask |= 1u << idx;
        L.left++;
    }
    t_last_path = OSGPU_RAN_TEAM;
    call_trace(c.me, 0, "start");
    entry_sync(c.name, st);
    call_trace(c.me, 1, "entry_sync");
    barrier(c);  // src/reductions.c:82 -- sources ready, every target writable
    call_trace(c.me, 2, "barrier1");
    // the run of consecutive local members I belong to (just me without tiles)
    int first = idx, last = idx;
    if (tiles) {
        unsigned mask;
        {
            std::lock_guard<std::mutex> lk(g_local_mu);
            mask = g_local[key].mask;
        }
        while (first > 0 && (mask >> (first - 1) & 1u)) first--;
        while (last + 1 < c.PE_size && (mask >> (last + 1) & 1u)) last++;
    }
    long long lo = 0, hi = 0, t = 0;
    osgpu_shard_range(c.nreduce, c.PE_size, first, es, &lo, &t);
    osgpu_shard_range(c.nreduce, c.PE_size, last, es, &t, &hi);
    std::vector<const void *> sp(c.PE_size);
    std::vector<void *> dp(c.PE_size);
    for (int i = 0; i < c.PE_size; i++) {
        sp[i] = (const char *) srcs[i] + (size_t) lo * s;
        dp[i] = (char *) dsts[i] + (size_t) lo * s;
    }
    DBG("%s PE %d: team path, [%lld, %lld) of %d, tiles %d of %d, P=%d", c.name, c.me, lo, hi,
        c.nreduce, idx - first, last - first + 1, c.PE_size);
    int m = last - first + 1, k = idx - first;
    if (mode == LOCAL_MERGE) {
        if (k > 0) hi = lo;  // the run's first member launches for all of it
        m = 1;
        k = 0;
    }
    if (hi > lo) {
        hipError_t e = osgpu::launch_team_tiles(c.type, c.op, c.PE_size, dp.data(), sp.data(),
                                                (size_t) (hi - lo), m, k, st, remote);
        if (e != hipSuccess) fatal(c.name, "team combine launch: %s", hipGetErrorString(e));
    }
    call_trace(c.me, 3, "launch");
    DBG("%s PE %d: team kernel launched", c.name, c.me);
    stream_wait(c.name, st);
    call_trace(c.me, 4, "wait");
    DBG("%s PE %d: team kernel done", c.name, c.me);
    barrier(c);  // src/reductions.c:113 -- every shard of my target is written
    call_trace(c.me, 5, "barrier2");
    call_trace(c.me, 6, "end");
    if (tiles) {
        std::lock_guard<std::mutex> lk(g_local_mu);
        auto it = g_local.find(key);
        if (it != g_local.end() && --it->second.left == 0) g_local.erase(it);
    }
}

// Push form of the team exchange (osgpu_set_team_exchange(1)): every byte
// crosses the fabric as a remote WRITE.  Per chunk of every shard:
//   scatter  PE q copies its source's part of shard g into slot q of PE g's
//            inbox (the STAGED path's IPC-mapped staging, 4 x slot bytes per
//            PE: P slots of C elements), for every g -- one copy launch;
//   barrier  every inbox holds the chunk (every member has entered, so every
//            target is writable);
//   fold     PE g runs the team kernel over its inbox (local HBM reads) and
//            writes shard g of every member's target (remote writes);
//   barrier  every inbox slot is drained / every target shard written.
// Same fabric bytes as the pull form ((P-1)/P * N * s each way per PE),
// plus N * s of local inbox traffic; which form the links prefer is
// measured by bench.py's N > 1 xgmi_probe.
void run_team_push(const Call &c, const std::vector<const void *> &srcs,
                   const std::vector<void *> &dsts, int idx, StageSet &S)
{
    hipStream_t st = pe_stream(c.name, c.me);
    const size_t s = type_size(c.type);
    const int P = c.PE_size;
    const long long g16 = s >= 16 ? 1 : (long long) (16 / s);
    std::vector<long long> lo(P), hi(P);
    long long most = 0;
    for (int g = 0; g < P; g++) {
        osgpu_shard_range(c.nreduce, P, g, (int) (s > 16 ? 16 : s), &lo[g], &hi[g]);
        most = std::max(most, hi[g] - lo[g]);
    }
    long long C = (long long) ((4 * S.slot) / (size_t) P / s) / g16 * g16;  // elements per slot
    if (C < 1) fatal(c.name, "staging too small for the push exchange of %d PEs", P);
    const long long nchunks = (most + C - 1) / C;
    t_last_path = OSGPU_RAN_TEAM_PUSH;
    DBG("%s PE %d: team push, %lld chunks of %lld", c.name, c.me, nchunks, C);
    entry_sync(c.name, st);
    // The inboxes are the staging areas of this active set, whose out slots
    // a member may still be draining into its host target after a STAGED or
    // fused-staged call it has not yet returned from: no member scatters
    // before every member has entered this call.
    barrier(c);
    std::vector<osgpu::CopySeg> segs;
    std::vector<const void *> sp(P);
    std::vector<void *> dp(P);
    for (long long k = 0; k < nchunks; k++) {
        segs.clear();
        for (int g = 0; g < P; g++) {
            const long long a = lo[g] + k * C, b = std::min(hi[g], a + C);
            if (b > a)
                segs.push_back({(const char *) srcs[idx] + (size_t) a * s,
                                S.region(g) + (size_t) idx * C * s, (size_t) (b - a) * s});
        }
        for (size_t i = 0; i < segs.size(); i += osgpu::kMaxCopySegs) {
            const int m = (int) std::min(segs.size() - i, (size_t) osgpu::kMaxCopySegs);
            hipError_t e = osgpu::launch_copy(segs.data() + i, m, st);
            if (e != hipSuccess) fatal(c.name, "scatter launch: %s", hipGetErrorString(e));
        }
        stream_wait(c.name, st);
        barrier(c);  // every inbox holds chunk k; every member has entered (:82)
        const long long a = lo[idx] + k * C, b = std::min(hi[idx], a + C);
        if (b > a) {
            for (int i = 0; i < P; i++) {
                sp[i] = S.region(idx) + (size_t) i * C * s;
                dp[i] = (char *) dsts[i] + (size_t) a * s;
            }
            hipError_t e = osgpu::launch_team(c.type, c.op, P, dp.data(), sp.data(),
                                              (size_t) (b - a), st, S.ndev > 1);
            if (e != hipSuccess) fatal(c.name, "team fold launch: %s", hipGetErrorString(e));
            stream_wait(c.name, st);
        }
        barrier(c);  // inboxes drained; after the last chunk every target is complete (:113)
    }
}

void run_p2p(const Call &c, const std::vector<const void *> &srcs)
{
    hipStream_t st = pe_stream(c.name, c.me);
    t_last_path = OSGPU_RAN_PULL;
    // prior device work of this process that produced `source` must be done
    entry_sync(c.name, st);
    barrier(c);  // src/reductions.c:82 -- every source is ready
    const bool overlap = c.PE_size > 1 && ranges_overlap(c.target, c.source, c.nbytes);
    void *out = overlap ? device_scratch(c.name, c.me, c.nbytes) : c.target;
    hipError_t e = osgpu::launch_combine(c.type, c.op, out, srcs.data(), c.PE_size,
                                         (size_t) c.nreduce, st);
    if (e != hipSuccess) fatal(c.name, "combine launch: %s", hipGetErrorString(e));
    stream_wait(c.name, st);
    barrier(c);  // src/reductions.c:113 -- peers are done reading my source
    if (overlap) {
        HIPCHK(c.name, hipMemcpyAsync(c.target, out, c.nbytes, hipMemcpyDeviceToDevice, st));
        stream_wait(c.name, st);
    }
}

// ---------------------------------------------------- fused small calls

// A device-resident call of at most fused_max_bytes() per PE runs as ONE
// launch with its barriers on the device (fused.hip); larger calls keep the
// host barriers around the full-chip streaming kernels.
// Only with entry ordering that does not wait for this PE's own stream:
// under hipDeviceSynchronize every call would first wait for the previous
// fused launch to retire (measured 26 us per 1 Ki-int call against 16 us on
// the host-barrier path; 12 us with `stream` ordering).
// The pull form reads P sources per PE (P times the team form's bytes) on
// its share of the CUs: its limit is a quarter of the team form's (measured
// with 4 processes on one GPU at 1 MiB per PE: fused pull 42 us against 29
// us with host barriers; fused team 23 us).
bool fused_eligible(const Call &c, bool team)
{
    const int em = entry_mode();
    const size_t lim = team ? fused_max_bytes() : fused_max_bytes() / 4;
    return (em == ENTRY_STREAM || em == ENTRY_NONE) && osgpu::fused_supported(c.type) &&
           c.PE_size >= 2 && c.PE_size <= osgpu::kMaxTeam && c.nbytes <= lim &&
           c.ops.getmem != nullptr;
}

// team = true: owner-computes over every member's target (srcs/dsts in
// active-set order); false: pull form, my own target from every source.
void run_fused(const Call &c, SyncSet &S, const std::vector<const void *> &srcs,
               const std::vector<void *> &dsts, bool team, const StageSet *G = nullptr,
               const void *host_in = nullptr, void *host_out = nullptr)
{
    hipStream_t st = pe_stream(c.name, c.me);
    const size_t s = type_size(c.type);
    const int P = c.PE_size, idx = S.idx;
    osgpu::FusedArgs a;
    memset(&a, 0, sizeof(a));
    long long lo = 0, hi = c.nreduce;
    if (team) osgpu_shard_range(c.nreduce, P, idx, (int) (s > 16 ? 16 : s), &lo, &hi);
    // (staged form: target and source may overlap -- the source is copied
    // into staging before any member writes, the target after all are done)
    const bool overlap = !G && !team && ranges_overlap(c.target, c.source, c.nbytes);
    void *out = overlap ? device_scratch(c.name, c.me, c.nbytes) : c.target;
    for (int i = 0; i < P; i++) {
        a.src[i] = (const char *) srcs[i] + (size_t) lo * s;
        a.flags[i] = S.peer[i];
    }
    if (team) {
        for (int d = 0; d < P; d++) {
            a.dst[d] = (char *) dsts[d] + (size_t) lo * s;
            a.q[d] = d;
        }
        a.D = P;
    } else {
        a.dst[0] = out;
        a.q[0] = idx;
        a.D = 1;
    }
    a.mine = S.local;
    a.err = S.err_d;
    a.done_host = S.done_d;
    a.epoch = ++S.epoch;
    a.n = (size_t) (hi - lo);
    a.P = P;
    a.me = idx;
    a.max_blocks = S.max_blocks;
    if (G) {
        a.host_in = host_in;
        a.host_out = host_out;
        a.stage_mine = G->in(idx, 0);
        a.stage_result = G->out(idx, 0);
        a.host_bytes = c.nbytes;
    }
    t_last_path = G ? OSGPU_RAN_FUSED_STAGED : team ? OSGPU_RAN_FUSED_TEAM : OSGPU_RAN_FUSED_PULL;
    DBG("%s PE %d: fused %s path, epoch %llu, [%lld, %lld)", c.name, c.me,
        G ? "staged" : team ? "team" : "pull", a.epoch, lo, hi);
    // OSGPU_FUSED_TRACE=1: phase clocks of workgroup 0 / the last workgroup
    static unsigned long long *trace = [] {
        unsigned long long *p = nullptr;
        if (getenv("OSGPU_FUSED_TRACE") &&
            hipHostMalloc((void **) &p, 64, hipHostMallocMapped | hipHostMallocCoherent) !=
                hipSuccess)
            p = nullptr;
        return p;
    }();
    a.trace = trace;
    if (trace) memset(trace, 0, 64);  // slots a continuation launch leaves unwritten stay 0
    entry_order(c.name, st);
    if (!fused_complete(c.name, S, st, a, [&](const osgpu::FusedArgs &x) {
            return osgpu::launch_fused(c.type, c.op, x, st);
        })) {
        t_last_path = OSGPU_RAN_FUSED_FAILED;
        return;
    }
    if (overlap) {  // every reader of my source is done: the call passed its exit barrier
        HIPCHK(c.name, hipMemcpyAsync(c.target, out, c.nbytes, hipMemcpyDeviceToDevice, st));
        stream_wait(c.name, st);
    }
    if (trace && osgpu_last_continuations() > 0) {
        // the phase clocks are taken by the first launch only (fused.hip):
        // a call that needed continuations has no consistent breakdown
        fprintf(stderr, "[osgpu fused PE %d epoch %llu] %d continuation launch(es): no phase "
                        "breakdown\n", c.me, a.epoch, osgpu_last_continuations());
    } else if (trace) {
        const double tk = 1e3 / S.rate_khz;  // us per tick of the device wall clock
        fprintf(stderr, "[osgpu fused PE %d epoch %llu] arrive-wait %.2f body %.2f fence %.2f "
                        "ticket+fence %.2f done-wait %.2f us\n", c.me, a.epoch,
                (trace[1] - trace[0]) * tk, (trace[2] - trace[1]) * tk,
                (trace[3] - trace[2]) * tk, (trace[4] - trace[3]) * tk,
                (trace[6] - trace[5]) * tk);
    }
}

// RCCL's arithmetic for a (type, op), or false.
//  * integer sum/prod/min/max: order-independent (wrapping ring, lattice),
//    so ncclAllReduce is bit-exact -- allowed on the automatic path;
//  * FP / complex sum and prod: RCCL folds in its own order, identical on
//    every PE, where the reference folds in a per-PE order
//    (src/reductions.c:79-111): within tolerance only, so only when the
//    caller forces OSGPU_PATH_RCCL (`fp_ok`);
//  * FP min/max: never.  The reference's `a<b?a:b` / `a>b?a:b`
//    (src/shmemu/miscops.c:80-90) resolves NaN and signed-zero ties by fold
//    position; RCCL's min/max do not follow it.
bool rccl_types(int type, int op, bool fp_ok, ncclDataType_t *dt, ncclRedOp_t *rop,
                size_t *mult)
{
    *mult = 1;
    switch (op) {
    case OSGPU_OP_SUM: *rop = ncclSum; break;
    case OSGPU_OP_PROD: *rop = ncclProd; break;
    case OSGPU_OP_MAX: *rop = ncclMax; break;
    case OSGPU_OP_MIN: *rop = ncclMin; break;
    default: return false;
    }
    const bool arith = op == OSGPU_OP_SUM || op == OSGPU_OP_PROD;
    switch (type) {
    case OSGPU_T_INT: *dt = ncclInt32; return true;
    case OSGPU_T_LONG: case OSGPU_T_LONGLONG: *dt = ncclInt64; return true;
    case OSGPU_T_FLOAT: *dt = ncclFloat32; return fp_ok && arith;
    case OSGPU_T_DOUBLE: *dt = ncclFloat64; return fp_ok && arith;
    case OSGPU_T_COMPLEXF: *dt = ncclFloat32; *mult = 2; return fp_ok && op == OSGPU_OP_SUM;
    case OSGPU_T_COMPLEXD: *dt = ncclFloat64; *mult = 2; return fp_ok && op == OSGPU_OP_SUM;
    }
    return false;
}

bool rccl_usable(const Call &c, bool forced)
{
    ncclDataType_t dt;
    ncclRedOp_t rop;
    size_t mult;
    // the whole job only: a subset communicator would need ncclCommSplit,
    // which every PE of the parent must call -- OpenSHMEM forbids
    // non-members from calling a collective on an active set
    return g_rccl.world && c.PE_start == 0 && c.step == 1 && c.PE_size == g_rccl.npes &&
           c.me == g_rccl.me && rccl_types(c.type, c.op, forced, &dt, &rop, &mult);
}

void run_rccl(const Call &c)
{
    ncclDataType_t dt;
    ncclRedOp_t rop;
    size_t mult;
    rccl_types(c.type, c.op, true, &dt, &rop, &mult);
    t_last_path = OSGPU_RAN_RCCL;
    hipStream_t st = pe_stream(c.name, c.me);
    entry_sync(c.name);
    const bool overlap = ranges_overlap(c.target, c.source, c.nbytes) && c.target != c.source;
    void *out = overlap ? device_scratch(c.name, c.me, c.nbytes) : c.target;
    ncclResult_t r = ncclAllReduce(c.source, out, (size_t) c.nreduce * mult, dt, rop,
                                   g_rccl.world, st);
    if (r != ncclSuccess) fatal(c.name, "ncclAllReduce: %s", ncclGetErrorString(r));
    stream_wait(c.name, st);
    if (overlap) {
        HIPCHK(c.name, hipMemcpyAsync(c.target, out, c.nbytes, hipMemcpyDeviceToDevice, st));
        stream_wait(c.name, st);
    }
}

// How the STAGED path moves its chunks across PCIe (OSGPU_STAGE_COPY):
//   dma (default)   both legs by the DMA engines (hipMemcpyAsync on the two
//                   copy streams, runtime.cpp device_copy_streams): 44.5 GB/s
//                   each way pinned, 38-41 pageable, 2 PEs at 64 Mi doubles;
//   kout            H2D by DMA, D2H by launch_host_copy (a kernel writing
//                   the host's device view); 34.7 pinned;
//   kernel          both legs by kernel; 30.6-31.0 pinned
//   (profiles/r05_staged_copy_modes.jsonl).  The kernel legs exist for the
//   GPU's low power state, in which the DMA engine's D2H rate falls to
//   28-30 GB/s (the first second of an idle box) while a kernel's writes
//   hold 54 (tools/d2h_timeline.hip, profiles/r05_dma_state_timeline.jsonl);
//   the bench reports that state beside the rates (dma_state).
// A leg whose host memory has no device view takes the DMA engine.
// (runtime.cpp stage_copy_mode: osgpu_set_stage_copy, else the environment)
enum { STAGE_DMA = 0, STAGE_KOUT, STAGE_KERNEL };

// one staged leg: a kernel over the host side's device view (dview) when
// the mode asks for one and the view exists, else the DMA engine
void stage_leg(const char *name, int mode, void *dst, const void *src, size_t bytes,
               bool to_host, const void *dview, hipStream_t st)
{
    const bool kern = dview && (mode == STAGE_KERNEL || (mode == STAGE_KOUT && to_host));
    hipError_t e;
    if (kern)
        e = to_host ? osgpu::launch_host_copy(const_cast<void *>(dview), src, bytes, st)
                    : osgpu::launch_host_copy(dst, dview, bytes, st);
    else
        e = hipMemcpyAsync(dst, src, bytes, to_host ? hipMemcpyDeviceToHost : hipMemcpyHostToDevice,
                           st);
    if (e != hipSuccess) fatal(name, "staging copy: %s", hipGetErrorString(e));
}

void run_staged(const Call &c, StageSet &S)
{
    const size_t s = type_size(c.type);
    const size_t C = S.slot / s;                       // elements per chunk
    const size_t N = (size_t) c.nreduce;
    const size_t nchunks = (N + C - 1) / C;
    t_last_path = OSGPU_RAN_STAGED;
    const int P = c.PE_size;
    int idx = 0;
    for (int i = 0, pe = c.PE_start; i < P; i++, pe += c.step)
        if (pe == c.me) idx = i;
    const bool overlap = ranges_overlap(c.target, c.source, c.nbytes) && c.target != c.source;
    char *result = overlap ? (char *) malloc(c.nbytes) : (char *) c.target;
    if (!result) fatal(c.name, "out of memory for the temporary target");
    const char *src = (const char *) c.source;
    std::vector<const void *> sp(P);
    std::vector<void *> dp(P);
    // pinned bounce slots for pageable arrays: in[2], out[2] of S.slot bytes
    const bool bounce_in = !host_pinned(c.source), bounce_out = !host_pinned(result);
    char *bounce = (bounce_in || bounce_out)
                       ? (char *) host_stage(c.name, c.me, 4 * S.slot) : nullptr;
    auto bin = [&](int sl) { return bounce + (size_t) sl * S.slot; };
    auto bout = [&](int sl) { return bounce + (size_t) (2 + sl) * S.slot; };
    // the GPU's view of the host side of each leg (null: DMA engine)
    const int cmode = stage_copy_mode();
    char *bounce_dev = nullptr;
    if (bounce && cmode != STAGE_DMA &&
        hipHostGetDevicePointer((void **) &bounce_dev, bounce, 0) != hipSuccess) {
        (void) hipGetLastError();
        bounce_dev = nullptr;
    }
    auto view = [&](const char *h, bool is_bounce, size_t n) -> const void * {
        if (cmode == STAGE_DMA) return nullptr;
        if (is_bounce) return bounce_dev ? bounce_dev + (h - bounce) : nullptr;
        return host_device_view(h, n);
    };
    auto chunk_n = [&](size_t ch) { return (ch + 1) * C <= N ? C : N - ch * C; };
    // D2H of chunk ch landed in bout: copy it to the caller's array
    auto drain = [&](size_t ch) {
        if (bounce_out) par_memcpy(result + ch * C * s, bout((int) (ch & 1)), chunk_n(ch) * s);
    };

    auto h2d = [&](size_t ch) {
        const size_t n = chunk_n(ch);
        const char *from = src + ch * C * s;
        if (bounce_in) {  // bin[ch & 1] is free: its previous H2D was waited for
            par_memcpy(bin((int) (ch & 1)), from, n * s);
            from = bin((int) (ch & 1));
        }
        stage_leg(c.name, cmode, S.in(idx, ch & 1), from, n * s, false, view(from, bounce_in, n * s),
                  S.st_in);
        HIPCHK(c.name, hipEventRecord(S.ev_in[ch & 1], S.st_in));
    };
    entry_sync(c.name);
    h2d(0);
    for (size_t ch = 0; ch < nchunks; ch++) {
        const int sl = (int) (ch & 1);
        const size_t n = (ch + 1) * C <= N ? C : N - ch * C;
        if (ch + 1 < nchunks) h2d(ch + 1);   // slot reuse is safe: team(ch-1) ended everywhere
        HIPCHK(c.name, hipEventSynchronize(S.ev_in[sl]));
        if (ch >= 2) {  // my out slot (and its bounce) drained
            HIPCHK(c.name, hipEventSynchronize(S.ev_out[sl]));
            drain(ch - 2);
        }
        barrier(c);  // chunk ch staged on every PE, every out[sl] free
        if (P == 1) {
            const void *one = S.in(0, sl);
            hipError_t e = osgpu::launch_combine(c.type, c.op, S.out(0, sl), &one, 1, n, S.st_c);
            if (e != hipSuccess) fatal(c.name, "combine launch: %s", hipGetErrorString(e));
        } else if (P <= osgpu::kMaxTeam) {
            long long lo = 0, hi = 0;
            osgpu_shard_range((long long) n, P, idx, (int) (s > 16 ? 16 : s), &lo, &hi);
            for (int i = 0; i < P; i++) {
                sp[i] = S.in(i, sl) + (size_t) lo * s;
                dp[i] = S.out(i, sl) + (size_t) lo * s;
            }
            if (hi > lo) {
                hipError_t e = osgpu::launch_team(c.type, c.op, P, dp.data(), sp.data(),
                                                  (size_t) (hi - lo), S.st_c, S.ndev > 1);
                if (e != hipSuccess) fatal(c.name, "team launch: %s", hipGetErrorString(e));
            }
        } else {  // large active sets: every PE folds its own chunk (pull form)
            std::vector<int> order(P);
            fold_order(c.me, c.PE_start, c.step, P, order.data());
            for (int k = 0; k < P; k++) sp[k] = S.in((order[k] - c.PE_start) / c.step, sl);
            hipError_t e = osgpu::launch_combine(c.type, c.op, S.out(idx, sl), sp.data(), P, n,
                                                 S.st_c);
            if (e != hipSuccess) fatal(c.name, "combine launch: %s", hipGetErrorString(e));
        }
        stream_wait(c.name, S.st_c);
        barrier(c);  // every shard of my out[sl] written
        char *to = bounce_out ? bout(sl) : result + ch * C * s;
        stage_leg(c.name, cmode, to, S.out(idx, sl), n * s, true, view(to, bounce_out, n * s), S.st_out);
        HIPCHK(c.name, hipEventRecord(S.ev_out[sl], S.st_out));
    }
    stream_wait(c.name, S.st_out);
    for (size_t ch = nchunks >= 2 ? nchunks - 2 : 0; ch < nchunks; ch++) drain(ch);
    if (overlap) {
        memcpy(c.target, result, c.nbytes);
        free(result);
    }
}

// Host symmetric-heap arguments: the data arrives and leaves through host
// memory (the UCX heap).  Peers' sources are pulled with the runtime's
// shmem_getmem (src/putget.h:539-561), like the reference, but in large
// chunks into pinned staging, then combined on the GPU.
void run_host(const Call &c)
{
    if (!c.ops.getmem) fatal(c.name, "host-memory arguments need shmem_getmem");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        fatal(c.name, "no GPU visible: the combine runs only on the GPU");
    hipStream_t st = pe_stream(c.name, c.me);
    const size_t s = type_size(c.type);
    const int P = c.PE_size;
    t_last_path = OSGPU_RAN_GETMEM;
    std::vector<int> order(P);
    fold_order(c.me, c.PE_start, c.step, P, order.data());

    size_t chunk = host_chunk_bytes() / s;
    if (chunk == 0) chunk = 1;
    if (chunk > (size_t) c.nreduce) chunk = (size_t) c.nreduce;
    chunk = (chunk + 1) & ~(size_t) 1;
    const size_t cb = chunk * s;
    // device: P input slots + 1 output slot; pinned: P input slots + output
    char *dbuf = (char *) device_scratch(c.name, c.me, cb * (P + 1));
    char *hbuf = (char *) host_stage(c.name, c.me, cb * (P + 1));
    const bool overlap = P > 1 && ranges_overlap(c.target, c.source, c.nbytes);
    char *result = overlap ? (char *) malloc(c.nbytes) : (char *) c.target;
    if (!result) fatal(c.name, "out of memory for the temporary target");
    std::vector<const void *> srcs(P);
    for (int k = 0; k < P; k++) srcs[k] = dbuf + (size_t) k * cb;

    barrier(c);  // src/reductions.c:82
    for (size_t off = 0; off < (size_t) c.nreduce; off += chunk) {
        const size_t n = ((size_t) c.nreduce - off) < chunk ? ((size_t) c.nreduce - off) : chunk;
        const size_t nb = n * s;
        for (int k = 0; k < P; k++) {
            char *hk = hbuf + (size_t) k * cb;
            const char *src = (const char *) c.source + off * s;
            if (order[k] == c.me) memcpy(hk, src, nb);
            else c.ops.getmem(hk, src, nb, order[k]);
            HIPCHK(c.name, hipMemcpyAsync((void *) srcs[k], hk, nb, hipMemcpyHostToDevice, st));
        }
        char *dout = dbuf + (size_t) P * cb;
        hipError_t e = osgpu::launch_combine(c.type, c.op, dout, srcs.data(), P, n, st);
        if (e != hipSuccess) fatal(c.name, "combine launch: %s", hipGetErrorString(e));
        char *hout = hbuf + (size_t) P * cb;
        HIPCHK(c.name, hipMemcpyAsync(hout, dout, nb, hipMemcpyDeviceToHost, st));
        stream_wait(c.name, st);
        memcpy(result + off * s, hout, nb);
    }
    barrier(c);  // src/reductions.c:113
    if (overlap) {
        memcpy(c.target, result, c.nbytes);  // src/reductions.c:114-119
        free(result);
    }
}

// Small calls on HOST symmetric-heap memory (each PE pulling at most
// host_fold_max_bytes() from its peers, automatic host path): the reference's algorithm on this PE's
// thread with the kernels' element ops compiled for the host (host_fold.hip)
// -- the source copied into the target, barrier (src/reductions.c:82), every
// other PE's whole source pulled with ONE shmem_getmem (the reference pulls
// 64 elements per getmem, :90-103) and folded in this PE's order (:84-111),
// barrier (:113), the temporary target copied back on overlap (:114-119).
// No GPU round trip: below this size the fastest GPU form (one fused launch
// reading and writing the host heap over PCIe) costs more than the whole
// loop.
void run_host_fold(const Call &c)
{
    t_last_path = OSGPU_RAN_HOST_FOLD;
    const int P = c.PE_size;
    std::vector<int> order(P);
    fold_order(c.me, c.PE_start, c.step, P, order.data());
    const bool overlap = ranges_overlap(c.target, c.source, c.nbytes);
    thread_local std::vector<unsigned char> tmp, peer;
    if (overlap) tmp.resize(c.nbytes);
    void *acc = overlap ? (void *) tmp.data() : c.target;
    memcpy(acc, c.source, c.nbytes);  // :79-81
    barrier(c);                       // :82 -- every source is ready
    peer.resize(c.nbytes);
    for (int k = 1; k < P; k++) {     // order[0] is this PE
        c.ops.getmem(peer.data(), c.source, c.nbytes, order[k]);
        if (!osgpu::host_fold(c.type, c.op, acc, peer.data(), (size_t) c.nreduce))
            fatal(c.name, "host fold: type %d op %d", c.type, c.op);
    }
    barrier(c);                       // :113 -- every peer is done reading my source
    if (overlap) memcpy(c.target, acc, c.nbytes);  // :114-119
}

void to_all(const char *name, int type, int op, void *target, void *source, int nreduce,
            int PE_start, int logPE_stride, int PE_size, void *pWrk, long *pSync)
{
    (void) pWrk;  // the combine needs no bounce buffer: peers are read directly
    Call c;
    static_cast<Coll &>(c) = make_coll(name, PE_start, logPE_stride, PE_size, pSync);
    c.type = type;
    c.op = op;
    c.target = target;
    c.source = source;
    c.nreduce = nreduce;
    if (nreduce <= 0) {  // nothing to combine; the collective still syncs
        t_last_path = OSGPU_RAN_BARRIER_ONLY;
        barrier(c);
        barrier(c);
        return;
    }
    c.nbytes = type_size(type) * (size_t) nreduce;  // no int overflow (cf. :44)

    int dt = -1, ds = -1;
    MemKind kt = mem_kind(target, &dt), ks = mem_kind(source, &ds);
    if (kt != ks)
        fatal(name, "target and source must both be device or both be host memory");
    if (kt == MEM_HOST) {
        const int hp = host_path();
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
            fatal(name, "no GPU visible: the combine runs only on the GPU");
        if (!c.ops.getmem) fatal(name, "host-memory arguments need shmem_getmem");
        // a size every member shares: all of them take the same path
        const size_t fold_lim = host_fold_max_bytes();  // 0: off
        if (hp == OSGPU_HOST_AUTO && fold_lim > 0 && (size_t) (c.PE_size - 1) * c.nbytes <= fold_lim &&
            osgpu::host_fold_supported(type, op)) {
            run_host_fold(c);
            return;
        }
        StageSet *S = hp == OSGPU_HOST_GETMEM ? nullptr : stage_setup(c);
        // small calls on host heaps pinned with osgpu_host_register (on every
        // PE, like the heap itself): H2D, exchange and D2H in one launch
        void *hin = nullptr, *hout = nullptr;
        SyncSet *Y = nullptr;
        if (S && fused_eligible(c, true) && c.nbytes <= S->slot &&
            (hin = host_device_view(source, c.nbytes)) &&
            (hout = host_device_view(target, c.nbytes)) && (Y = sync_setup(c))) {
            std::vector<const void *> srcs(c.PE_size);
            std::vector<void *> dsts(c.PE_size);
            for (int i = 0; i < c.PE_size; i++) {
                srcs[i] = S->in(i, 0);
                dsts[i] = S->out(i, 0);
            }
            run_fused(c, *Y, srcs, dsts, true, S, hin, hout);
        } else if (S) {
            run_staged(c, *S);
        } else {
            run_host(c);
        }
        return;
    }
    int cur = 0;
    HIPCHK(name, hipGetDevice(&cur));
    if (cur != dt) HIPCHK(name, hipSetDevice(dt));
    const int mode = path_mode();
    std::vector<const void *> srcs;
    std::vector<void *> dsts;
    int idx = -1;
    bool remote = false;
    SyncSet *S = nullptr;
    // RCCL only where its result is the reference's: integer (type, op)s on
    // the automatic path when no device heap is registered; FP sum/prod only
    // when the caller forces OSGPU_PATH_RCCL (tolerance, not bit-exact); FP
    // min/max never (they take the exact kernels even when RCCL is forced).
    if (mode == OSGPU_PATH_RCCL && rccl_usable(c, true)) {
        run_rccl(c);
    } else if (mode != OSGPU_PATH_PULL && (idx = team_ptrs(c, srcs, dsts, &remote)) >= 0) {
        StageSet *G = nullptr;
        if (fused_eligible(c, true) && (S = sync_setup(c)))
            run_fused(c, *S, srcs, dsts, true);
        else if (team_exchange() == 1 && c.ops.getmem && (G = stage_setup(c)))
            run_team_push(c, srcs, dsts, idx, *G);
        else
            run_team(c, srcs, dsts, idx, remote);
    } else if (member_sources(c, srcs)) {
        if (fused_eligible(c, false) && (S = sync_setup(c))) {
            run_fused(c, *S, srcs, dsts, false);
        } else {
            p2p_sources(c, srcs);
            run_p2p(c, srcs);
        }
    } else if (mode == OSGPU_PATH_AUTO && rccl_usable(c, false)) {
        run_rccl(c);
    } else {
        fatal(name,
              "device-resident arguments need every active PE's device heap registered "
              "(osgpu_heap_create / osgpu_heap_register), or -- integer types only, or FP "
              "sum/prod under OSGPU_PATH_RCCL -- an RCCL communicator over the whole job "
              "(path mode %d)",
              mode);
    }
    if (cur != dt) HIPCHK(name, hipSetDevice(cur));
}

}  // namespace

extern "C" int osgpu_last_path(void) { return t_last_path; }

// ======================================================================
// Part 1: the 44 entry points (pshmem_* strong, shmem_* weak aliases, as in
// the reference's --enable-pshmem build, src/reductions.c:156-245)
// ======================================================================

#define OSGPU_DEFINE(_name, _type, _op, _tcode, _ocode)                        \
    extern "C" void pshmem_##_name##_##_op##_to_all(                           \
        _type *target, _type *source, int nreduce, int PE_start,               \
        int logPE_stride, int PE_size, _type *pWrk, long *pSync)               \
    {                                                                          \
        to_all("shmem_" #_name "_" #_op "_to_all", _tcode, _ocode, target,     \
               source, nreduce, PE_start, logPE_stride, PE_size, pWrk, pSync); \
    }                                                                          \
    extern "C" void shmem_##_name##_##_op##_to_all(                            \
        _type *target, _type *source, int nreduce, int PE_start,               \
        int logPE_stride, int PE_size, _type *pWrk, long *pSync)               \
        __attribute__((weak, alias("pshmem_" #_name "_" #_op "_to_all")));

#define OSGPU_DEFINE_TYPE_OPS(_name, _type, _tcode)                            \
    OSGPU_DEFINE(_name, _type, sum, _tcode, OSGPU_OP_SUM)                      \
    OSGPU_DEFINE(_name, _type, prod, _tcode, OSGPU_OP_PROD)

#define OSGPU_DEFINE_BITS(_name, _type, _tcode)                                \
    OSGPU_DEFINE(_name, _type, and, _tcode, OSGPU_OP_AND)                      \
    OSGPU_DEFINE(_name, _type, or, _tcode, OSGPU_OP_OR)                        \
    OSGPU_DEFINE(_name, _type, xor, _tcode, OSGPU_OP_XOR)

#define OSGPU_DEFINE_MINMAX(_name, _type, _tcode)                              \
    OSGPU_DEFINE(_name, _type, max, _tcode, OSGPU_OP_MAX)                      \
    OSGPU_DEFINE(_name, _type, min, _tcode, OSGPU_OP_MIN)

typedef std::complex<float> osgpu_cf;
typedef std::complex<double> osgpu_cd;

OSGPU_DEFINE_TYPE_OPS(short, short, OSGPU_T_SHORT)
OSGPU_DEFINE_TYPE_OPS(int, int, OSGPU_T_INT)
OSGPU_DEFINE_TYPE_OPS(long, long, OSGPU_T_LONG)
OSGPU_DEFINE_TYPE_OPS(longlong, long long, OSGPU_T_LONGLONG)
OSGPU_DEFINE_TYPE_OPS(float, float, OSGPU_T_FLOAT)
OSGPU_DEFINE_TYPE_OPS(double, double, OSGPU_T_DOUBLE)
OSGPU_DEFINE_TYPE_OPS(longdouble, long double, OSGPU_T_LONGDOUBLE)
OSGPU_DEFINE_TYPE_OPS(complexf, osgpu_cf, OSGPU_T_COMPLEXF)
OSGPU_DEFINE_TYPE_OPS(complexd, osgpu_cd, OSGPU_T_COMPLEXD)
OSGPU_DEFINE_BITS(short, short, OSGPU_T_SHORT)
OSGPU_DEFINE_BITS(int, int, OSGPU_T_INT)
OSGPU_DEFINE_BITS(long, long, OSGPU_T_LONG)
OSGPU_DEFINE_BITS(longlong, long long, OSGPU_T_LONGLONG)
OSGPU_DEFINE_MINMAX(short, short, OSGPU_T_SHORT)
OSGPU_DEFINE_MINMAX(int, int, OSGPU_T_INT)
OSGPU_DEFINE_MINMAX(long, long, OSGPU_T_LONG)
OSGPU_DEFINE_MINMAX(longlong, long long, OSGPU_T_LONGLONG)
OSGPU_DEFINE_MINMAX(float, float, OSGPU_T_FLOAT)
OSGPU_DEFINE_MINMAX(double, double, OSGPU_T_DOUBLE)
OSGPU_DEFINE_MINMAX(longdouble, long double, OSGPU_T_LONGDOUBLE)
