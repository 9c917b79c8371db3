// shmem_collect.cpp -- the data-movement collectives on the reduce path's
// machinery: broadcast32/64, collect32/64,
// fcollect32/64, alltoall32/64, same signatures as the reference
// (include/shmem/api.h:2415-2450).
//
// Reference algorithms (bytes move with UCX puts/gets, one PE at a time):
//   broadcast  src/shmemc/broadcast.c:29-42 (linear: barrier, every non-root
//              gets the root's source; the tree/binomial variants :48-250
//              forward it) -- the root's own target is never written;
//   collect    src/shmemc/collect.c:24-69: an offset wavefront through pSync
//              (each PE learns the sum of its left neighbours' nelems), then
//              every PE puts its source at that offset of every target,
//              barrier;
//   fcollect   src/shmemc/fcollect.c:19-40: every PE puts its source at
//              block vpe = (me - PE_start) >> logPE_stride (:27) of every
//              target (:32-38), barrier (:39);
//   alltoall   src/alltoall.c:59-82: block i of my target <- a block of PE
//              i's source (gets, no synchronisation at all).
//
// Here every PE PULLS all the pieces of its own target in one launch of
// copy.hip's kernel (16-byte streaming loads from local or peer HBM):
//
//   COPY    device-resident, source symmetric in registered heaps (any
//           active-set size): copy kernel over peer pointers, two barriers
//           (sources ready / every reader done);
//   RCCL    device-resident without registered heaps, one process per GPU,
//           whole job: ncclBroadcast / ncclAllGather (broadcast, fcollect);
//   STAGED  host arguments, every member on a GPU of its own: H2D my source
//           -> copy kernel over every PE's IPC-mapped device staging -> D2H
//           of my target, chunked (each PE's PCIe link carries its bytes);
//   GETMEM  host arguments of small calls, or when members share a GPU (and
//           so its PCIe link), or when staging cannot be mapped: the
//           reference's own linear algorithm over the runtime's shmem_getmem
//           -- pure byte movement, which the runtime's memcpy does at memory
//           speed.
//   FUSED   small calls with every member its own process: ONE launch whose
//           barriers are device flags (fused.hip) -- device heaps always,
//           host heaps when staging is forced (OSGPU_HOST_PATH=staged).
//
// collect needs every PE's nelems before any byte moves.  On device heaps
// the counts ride on the device-side arrival of a fused launch (fused.hip
// fused_collect_kernel), which also moves the pieces when the gathered total
// is within the fused limit.  Otherwise each PE publishes its count in a
// spare pSync word (the reference's barrier uses pSync[0] only,
// src/shmemc/barrier.c:64-97), reads its peers' with shmem_getmem after the
// first barrier and clears its word after the last -- pSync is returned at
// SHMEM_SYNC_VALUE, as the reference's wavefront leaves it (collect.c:67).
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/osgpu_reduce.h"
#include "combine.hpp"
#include "runtime.hpp"

namespace {

using namespace osgpu::rt;

thread_local int t_last_coll = OSGPU_RAN_NONE;

enum Kind { K_BCAST, K_COLLECT, K_FCOLLECT, K_ALLTOALL };

constexpr int kCountWord = 8;  // pSync word carrying nelems during collect

// one piece of my target: bytes [src_off, src_off + len) of the source of the
// PE at active-set index `from`, to byte dst_off of my target
struct Piece {
    int from;
    size_t src_off, len, dst_off;
};

struct CCall : Coll {
    Kind kind = K_BCAST;
    void *target = nullptr;
    const void *source = nullptr;
    size_t esz = 0;
    size_t nelems = 0;
    int root = 0;                  // broadcast: active-set index of the root
    int idx = -1;                  // my active-set index
    std::vector<size_t> src_len;   // bytes of every member's source
    std::vector<Piece> pieces;     // what my target receives
    size_t out_bytes = 0;          // extent of my target that is written
};

bool overlap2(const void *a, size_t na, const void *b, size_t nb)
{
    if (!na || !nb) return false;
    const uintptr_t x = (uintptr_t) a, y = (uintptr_t) b;
    return x < y + nb && y < x + na;
}

// Every member's nelems (collect), through pSync[kCountWord] + getmem.
void exchange_counts(CCall &c)
{
    if (!c.ops.getmem) fatal(c.name, "collect needs shmem_getmem to learn every PE's nelems");
    if (mem_kind(c.pSync, nullptr) != MEM_HOST)
        fatal(c.name, "collect needs pSync in host symmetric memory");
    c.pSync[kCountWord] = (long) c.nelems;
    barrier(c);  // every count published (and, for the data, every source ready)
    c.src_len.assign(c.PE_size, 0);
    for (int i = 0; i < c.PE_size; i++) {
        long n = 0;
        if (i == c.idx) n = (long) c.nelems;
        else c.ops.getmem(&n, &c.pSync[kCountWord], sizeof(long), c.pe_at(i));
        if (n < 0) fatal(c.name, "negative nelems published by PE %d", c.pe_at(i));
        c.src_len[i] = (size_t) n * c.esz;
    }
}

// The pieces of my target and every member's source extent.
void plan(CCall &c)
{
    const int P = c.PE_size;
    const size_t nb = c.nelems * c.esz;
    c.pieces.clear();
    switch (c.kind) {
    case K_BCAST:
        c.src_len.assign(P, 0);
        c.src_len[c.root] = nb;
        if (c.idx != c.root) c.pieces.push_back({c.root, 0, nb, 0});
        c.out_bytes = c.idx != c.root ? nb : 0;
        break;
    case K_FCOLLECT:
        c.src_len.assign(P, nb);
        for (int i = 0; i < P; i++) c.pieces.push_back({i, 0, nb, (size_t) i * nb});
        c.out_bytes = (size_t) P * nb;
        break;
    case K_COLLECT: {  // src_len from exchange_counts
        size_t off = 0;
        for (int i = 0; i < P; i++) {
            c.pieces.push_back({i, 0, c.src_len[i], off});
            off += c.src_len[i];
        }
        c.out_bytes = off;
        break;
    }
    case K_ALLTOALL:
        c.src_len.assign(P, (size_t) P * nb);
        for (int i = 0; i < P; i++)
            c.pieces.push_back({i, (size_t) c.idx * nb, nb, (size_t) i * nb});
        c.out_bytes = (size_t) P * nb;
        break;
    }
}

// Does any PE (me included) read my source while my target is written?
bool my_source_read(const CCall &c)
{
    if (c.kind == K_BCAST) return c.idx == c.root;  // the root's target is untouched anyway
    return true;
}

void copy_pieces(const CCall &c, const std::vector<osgpu::CopySeg> &segs, hipStream_t st)
{
    for (size_t i = 0; i < segs.size(); i += osgpu::kMaxCopySegs) {
        const int n = (int) std::min(segs.size() - i, (size_t) osgpu::kMaxCopySegs);
        hipError_t e = osgpu::launch_copy(segs.data() + i, n, st);
        if (e != hipSuccess) fatal(c.name, "copy launch: %s", hipGetErrorString(e));
    }
}

// ------------------------------------------------------------ COPY (device)

// Peer addresses of every member's source (symmetric: same segment and
// offset in every registered heap); false if the heaps do not cover them.
bool device_sources(const CCall &c, std::vector<const char *> &src)
{
    size_t mine = c.src_len[c.idx];
    int seg = -1;
    size_t off = 0;
    // locate the source object in my heap (at least one byte, so that a
    // zero-length contribution still has a segment)
    if (!heap_locate(c.me, c.source, mine ? mine : 1, &seg, &off)) return false;
    src.assign(c.PE_size, nullptr);
    for (int i = 0; i < c.PE_size; i++) {
        bool needed = false;
        for (const Piece &p : c.pieces) needed |= (p.from == i && p.len);
        if (!needed) continue;
        char *p = nullptr;
        if (!heap_peer(c.pe_at(i), seg, off, c.src_len[i], &p)) return false;
        src[i] = p;
    }
    return true;
}

// Bytes a call moves into targets, a figure every member computes alike:
// broadcast nb, fcollect / alltoall P * nb, collect the gathered total.
size_t shared_bytes(const CCall &c)
{
    const size_t nb = c.nelems * c.esz;
    if (c.kind == K_BCAST) return nb;
    if (c.kind != K_COLLECT) return (size_t) c.PE_size * nb;
    size_t t = 0;
    for (size_t l : c.src_len) t += l;
    return t;
}

// Small broadcast / fcollect / alltoall calls run as ONE launch with the
// reduce path's device-side barriers (fused.hip fused_copy_kernel).  The
// decision uses only arguments every member shares (never which member I
// am), so every member takes the same path.
bool fused_copy_eligible(const CCall &c)
{
    const int em = entry_mode();
    return (em == ENTRY_STREAM || em == ENTRY_NONE) && c.kind != K_COLLECT &&
           c.PE_size >= 2 && c.PE_size <= osgpu::kMaxTeam && shared_bytes(c) <= fused_max_bytes() &&
           c.ops.getmem != nullptr;
}

void run_fused_copy(const CCall &c, SyncSet &S, const std::vector<osgpu::CopySeg> &segs,
                    char *out, hipStream_t st)
{
    osgpu::FusedArgs a;
    memset(&a, 0, sizeof(a));
    a.nseg = (int) segs.size();
    for (int d = 0; d < a.nseg; d++) {
        a.src[d] = segs[d].src;
        a.dst[d] = segs[d].dst;
        a.seg_bytes[d] = segs[d].bytes;
    }
    for (int i = 0; i < c.PE_size; i++) a.flags[i] = S.peer[i];
    a.mine = S.local;
    a.err = S.err_d;
    a.done_host = S.done_d;
    a.epoch = ++S.epoch;
    a.P = c.PE_size;
    a.me = S.idx;
    a.max_blocks = S.max_blocks;
    DBG("%s PE %d: fused copy, %d pieces, epoch %llu", c.name, c.me, a.nseg, a.epoch);
    entry_order(c.name, st);
    if (!fused_complete(c.name, S, st, a,
                        [&](const osgpu::FusedArgs &x) { return osgpu::launch_fused_copy(x, st); })) {
        t_last_coll = OSGPU_RAN_FUSED_FAILED;
        return;
    }
    if (out != (char *) c.target) {  // every reader of my source is done: exit barrier passed
        if (c.out_bytes)
            HIPCHK(c.name, hipMemcpyAsync(c.target, out, c.out_bytes, hipMemcpyDeviceToDevice, st));
        stream_wait(c.name, st);
    }
}

// Host heaps pinned on every PE (osgpu_host_register): a small broadcast /
// fcollect / alltoall as ONE launch -- my host source copied into my device
// staging area, the device barriers, every piece pulled from the members'
// staging areas straight into my host target (the STAGED path's H2D,
// exchange and D2H, like the reduce's fused staged form).  My source is in
// staging before I arrive and peers read only staging, so a target that
// overlaps my source needs no temporary.  false: not taken (same verdict on
// every member: shared sizes, and the heap pinned on every PE).
bool run_fused_staged_copy(const CCall &c, StageSet &G)
{
    if (!fused_copy_eligible(c)) return false;
    const size_t mine = c.src_len[c.idx];
    size_t most = 0;  // the largest source, the same figure on every member
    for (size_t l : c.src_len) most = std::max(most, l);
    if (most > 4 * G.slot) return false;
    void *hin = mine ? host_device_view(c.source, mine) : nullptr;
    void *hout = c.out_bytes ? host_device_view(c.target, c.out_bytes) : nullptr;
    if ((mine && !hin) || (c.out_bytes && !hout)) return false;
    SyncSet *S = sync_setup(c);
    if (!S) return false;
    t_last_coll = OSGPU_RAN_FUSED_STAGED;
    osgpu::FusedArgs a;
    memset(&a, 0, sizeof(a));
    for (const Piece &p : c.pieces) {
        if (!p.len) continue;
        a.src[a.nseg] = G.region(p.from) + p.src_off;
        a.dst[a.nseg] = (char *) hout + p.dst_off;
        a.seg_bytes[a.nseg] = p.len;
        a.nseg++;
    }
    a.host_in = hin;
    a.stage_mine = G.region(c.idx);
    a.host_bytes = mine;
    for (int i = 0; i < c.PE_size; i++) a.flags[i] = S->peer[i];
    a.mine = S->local;
    a.err = S->err_d;
    a.done_host = S->done_d;
    a.epoch = ++S->epoch;
    a.P = c.PE_size;
    a.me = S->idx;
    a.max_blocks = S->max_blocks;
    DBG("%s PE %d: fused staged copy, %d pieces, epoch %llu", c.name, c.me, a.nseg, a.epoch);
    hipStream_t st = pe_stream(c.name, c.me);
    entry_order(c.name, st);
    if (!fused_complete(c.name, *S, st, a,
                        [&](const osgpu::FusedArgs &x) { return osgpu::launch_fused_copy(x, st); }))
        t_last_coll = OSGPU_RAN_FUSED_FAILED;
    return true;
}

// collect on device heaps as ONE launch (fused.hip fused_collect_kernel):
// the counts ride on the device arrival instead of pSync + getmem + a host
// barrier.  Every member reaches the same outcome (the choice depends on
// the exchanged counts and the shared fused limit only):
//   2  the whole call ran in the launch (or failed, reported);
//   1  the launch exchanged the counts (c.src_len) and passed the entry
//      barrier; the pieces are left to the COPY path (total over the limit);
//   0  not eligible: the host exchanges the counts.
int fused_collect(CCall &c)
{
    const int em = entry_mode();
    const size_t lim = fused_max_bytes();
    const int P = c.PE_size;
    if (!(em == ENTRY_STREAM || em == ENTRY_NONE) || P < 2 || P > osgpu::kMaxTeam ||
        !c.ops.getmem || lim == 0)
        return 0;
    // every member's source object; its length is not known yet, so the
    // bytes from it to the end of its heap segment bound what may be read
    const size_t mine = c.nelems * c.esz;
    int seg = -1;
    size_t off = 0;
    if (!heap_locate(c.me, c.source, mine ? mine : 1, &seg, &off)) return 0;
    osgpu::FusedArgs a;
    memset(&a, 0, sizeof(a));
    for (int i = 0; i < P; i++) {
        HeapEntry h;
        if (!heap_segment(c.pe_at(i), seg, &h) || off >= h.bytes) return 0;
        a.src[i] = h.base + off;
        a.src_avail[i] = h.bytes - off;
    }
    SyncSet *S = sync_setup(c);
    if (!S) return 0;
    hipStream_t st = pe_stream(c.name, c.me);
    // my output: the target, or scratch when the target (at most `lim` bytes
    // if copied here) may overlap my source, which peers read in the launch
    const bool scratch = overlap2(c.target, lim, c.source, mine);
    char *out = scratch ? (char *) device_scratch(c.name, c.me, lim) : (char *) c.target;
    for (int i = 0; i < P; i++) a.flags[i] = S->peer[i];
    a.dst[0] = out;
    a.mine = S->local;
    a.err = S->err_d;
    a.done_host = S->done_d;
    a.counts_host = S->cnt_d;
    a.epoch = ++S->epoch;
    a.P = P;
    a.me = S->idx;
    a.max_blocks = S->max_blocks;
    if (mine >> osgpu::kCountBits) fatal(c.name, "contribution of %zu bytes too large", mine);
    a.my_count = mine;
    a.count_tag = ++S->ncollect;
    a.copy_limit = lim;
    DBG("%s PE %d: fused collect, %zu bytes mine, epoch %llu", c.name, c.me, mine, a.epoch);
    entry_order(c.name, st);
    if (!fused_complete(c.name, *S, st, a, [&](const osgpu::FusedArgs &x) {
            return osgpu::launch_fused_collect(x, st);
        })) {
        t_last_coll = OSGPU_RAN_FUSED_FAILED;
        return 2;
    }
    c.src_len.assign(P, 0);
    size_t total = 0;
    for (int i = 0; i < P; i++) total += (c.src_len[i] = (size_t) S->cnt_h[i]);
    if (!S->cnt_h[osgpu::kMaxTeam]) return 1;
    t_last_coll = OSGPU_RAN_FUSED_COPY;
    if (scratch && total) {  // every reader of my source is done: the launch passed done
        HIPCHK(c.name, hipMemcpyAsync(c.target, out, total, hipMemcpyDeviceToDevice, st));
        stream_wait(c.name, st);
    }
    return 2;
}

void run_copy(const CCall &c, const std::vector<const char *> &src, bool counts_done)
{
    hipStream_t st = pe_stream(c.name, c.me);
    const bool scratch = my_source_read(c) &&
                         overlap2(c.target, c.out_bytes, c.source, c.src_len[c.idx]);
    char *out = scratch ? (char *) device_scratch(c.name, c.me, c.out_bytes) : (char *) c.target;
    std::vector<osgpu::CopySeg> segs;
    for (const Piece &p : c.pieces)
        if (p.len) segs.push_back({src[p.from] + p.src_off, out + p.dst_off, p.len});
    SyncSet *Y = nullptr;
    if (!counts_done && fused_copy_eligible(c) && (Y = sync_setup(c))) {
        t_last_coll = OSGPU_RAN_FUSED_COPY;
        run_fused_copy(c, *Y, segs, out, st);
        return;
    }
    t_last_coll = OSGPU_RAN_COPY;
    DBG("%s PE %d: copy path, %zu pieces, %zu bytes out%s", c.name, c.me, segs.size(),
        c.out_bytes, scratch ? " (scratch)" : "");
    if (!counts_done) {
        entry_sync(c.name);
        barrier(c);  // every source ready
    }
    copy_pieces(c, segs, st);
    stream_wait(c.name, st);
    barrier(c);  // every reader of my source is done
    if (scratch && c.out_bytes) {
        HIPCHK(c.name, hipMemcpyAsync(c.target, out, c.out_bytes, hipMemcpyDeviceToDevice, st));
        stream_wait(c.name, st);
    }
}

// ------------------------------------------------------------ RCCL (device)

bool rccl_whole_job(const CCall &c)
{
    return g_rccl.world && c.PE_start == 0 && c.step == 1 && c.PE_size == g_rccl.npes &&
           c.me == g_rccl.me && (c.kind == K_BCAST || c.kind == K_FCOLLECT);
}

void run_rccl(const CCall &c)
{
    t_last_coll = OSGPU_RAN_RCCL;
    hipStream_t st = pe_stream(c.name, c.me);
    const size_t nb = c.nelems * c.esz;
    entry_sync(c.name);
    ncclResult_t r;
    if (c.kind == K_BCAST) {
        // the root receives in place (recvbuff == sendbuff: RCCL copies
        // nothing), so its target stays untouched as in the reference
        void *recv = c.idx == c.root ? (void *) c.source : c.target;
        r = ncclBroadcast(c.source, recv, nb, ncclUint8, c.root, g_rccl.world, st);
        if (r != ncclSuccess) fatal(c.name, "ncclBroadcast: %s", ncclGetErrorString(r));
        stream_wait(c.name, st);
        return;
    }
    const bool scratch = overlap2(c.target, c.out_bytes, c.source, nb) &&
                         (char *) c.target + (size_t) c.idx * nb != (const char *) c.source;
    char *out = scratch ? (char *) device_scratch(c.name, c.me, c.out_bytes) : (char *) c.target;
    r = ncclAllGather(c.source, out, nb, ncclUint8, g_rccl.world, st);
    if (r != ncclSuccess) fatal(c.name, "ncclAllGather: %s", ncclGetErrorString(r));
    stream_wait(c.name, st);
    if (scratch) {
        HIPCHK(c.name, hipMemcpyAsync(c.target, out, c.out_bytes, hipMemcpyDeviceToDevice, st));
        stream_wait(c.name, st);
    }
}

// ------------------------------------------------------------ STAGED (host)

// Chunk k covers source bytes [k*C, (k+1)*C) of every member.  Each PE
// stages its chunk in the `in` area of its device staging; each PE's copy
// kernel pulls the parts of its pieces inside chunk k from the members' `in`
// areas (IPC-mapped) into its own `out` area; D2H to the target.  The four
// slots of a StageSet are one region: in = C bytes, out = P*C bytes.
void run_staged(const CCall &c, StageSet &S)
{
    t_last_coll = OSGPU_RAN_STAGED;
    const int P = c.PE_size;
    const size_t region = 4 * S.slot;
    size_t C = region / (size_t) (P + 1);
    C &= ~(size_t) 255;
    if (C == 0) fatal(c.name, "staging too small for %d PEs", P);
    size_t maxlen = 0;
    for (size_t l : c.src_len) maxlen = std::max(maxlen, l);
    const size_t nchunks = (maxlen + C - 1) / C;
    const size_t mine = c.src_len[c.idx];
    const bool tmp = overlap2(c.target, c.out_bytes, c.source, mine);
    char *result = tmp ? (char *) malloc(c.out_bytes) : (char *) c.target;
    if (tmp && !result) fatal(c.name, "out of memory for the temporary target");
    char *in_me = S.region(c.idx);
    char *out_me = S.region(c.idx) + C;
    std::vector<osgpu::CopySeg> segs;
    std::vector<size_t> seg_dst;  // target offset of each staged piece part

    entry_sync(c.name);
    for (size_t k = 0; k < nchunks; k++) {
        const size_t lo = k * C, hi = lo + C;
        if (mine > lo) {
            const size_t n = std::min(mine, hi) - lo;
            HIPCHK(c.name, hipMemcpyAsync(in_me, (const char *) c.source + lo, n,
                                          hipMemcpyHostToDevice, S.st_in));
            stream_wait(c.name, S.st_in);
        }
        barrier(c);  // chunk k staged everywhere; every `in` area of k-1 drained
        segs.clear();
        seg_dst.clear();
        size_t packed = 0;
        for (const Piece &p : c.pieces) {
            const size_t a = std::max(p.src_off, lo), b = std::min(p.src_off + p.len, hi);
            if (a >= b) continue;
            segs.push_back({S.region(p.from) + (a - lo), out_me + packed, b - a});
            seg_dst.push_back(p.dst_off + (a - p.src_off));
            packed += b - a;
        }
        copy_pieces(c, segs, S.st_c);
        stream_wait(c.name, S.st_c);
        barrier(c);  // every reader of chunk k is done
        for (size_t i = 0; i < segs.size(); i++)
            HIPCHK(c.name, hipMemcpyAsync(result + seg_dst[i], segs[i].dst, segs[i].bytes,
                                          hipMemcpyDeviceToHost, S.st_out));
        stream_wait(c.name, S.st_out);
    }
    if (tmp) {
        memcpy(c.target, result, c.out_bytes);
        free(result);
    }
}

// GETMEM: the reference's linear schedule over the runtime's getmem (used
// only when the staging cannot be mapped by every PE).  No arithmetic is
// involved, so nothing is left for the GPU to do on this path.
void run_getmem(const CCall &c)
{
    t_last_coll = OSGPU_RAN_GETMEM;
    if (!c.ops.getmem) fatal(c.name, "host-memory arguments need shmem_getmem");
    const bool tmp = overlap2(c.target, c.out_bytes, c.source, c.src_len[c.idx]) &&
                     my_source_read(c);
    char *result = tmp ? (char *) malloc(c.out_bytes) : (char *) c.target;
    if (tmp && !result) fatal(c.name, "out of memory for the temporary target");
    for (const Piece &p : c.pieces) {
        if (!p.len) continue;
        const char *s = (const char *) c.source + p.src_off;
        if (p.from == c.idx) memmove(result + p.dst_off, s, p.len);
        else c.ops.getmem(result + p.dst_off, s, p.len, c.pe_at(p.from));
    }
    barrier(c);  // every reader of my source is done
    if (tmp) {
        memcpy(c.target, result, c.out_bytes);
        free(result);
    }
}

// ------------------------------------------------------------ dispatcher

void collective(const char *name, Kind kind, size_t esz, void *target, const void *source,
                size_t nelems, int PE_root, int PE_start, int logPE_stride, int PE_size,
                long *pSync)
{
    CCall c;
    static_cast<Coll &>(c) = make_coll(name, PE_start, logPE_stride, PE_size, pSync);
    c.kind = kind;
    c.target = target;
    c.source = source;
    c.esz = esz;
    c.nelems = nelems;
    c.root = PE_root;
    c.idx = c.index_of(c.me);
    if (c.idx < 0) fatal(name, "PE %d is not in the active set", c.me);
    if (kind == K_BCAST && (PE_root < 0 || PE_root >= PE_size))
        fatal(name, "PE_root %d outside the active set of %d PEs", PE_root, PE_size);
    if (kind != K_COLLECT && nelems == 0) {  // nothing moves; the collective still syncs
        t_last_coll = OSGPU_RAN_BARRIER_ONLY;
        barrier(c);
        barrier(c);
        return;
    }
    int dt = -1, ds = -1;
    const MemKind kt = mem_kind(target, &dt), ks = mem_kind(source, &ds);
    if (kt != ks) fatal(name, "target and source must both be device or both be host memory");

    bool counts_done = false, psync_counts = false;
    if (kind == K_COLLECT && kt == MEM_DEVICE) {  // counts on the device arrival
        int cur = 0;
        HIPCHK(name, hipGetDevice(&cur));
        if (cur != dt) HIPCHK(name, hipSetDevice(dt));
        const int f = fused_collect(c);
        if (cur != dt) HIPCHK(name, hipSetDevice(cur));
        if (f == 2) return;
        counts_done = f == 1;
    }
    if (kind == K_COLLECT && !counts_done) {
        if (kt == MEM_DEVICE) entry_sync(name);  // my source is final before I publish
        exchange_counts(c);                      // includes the first barrier
        counts_done = psync_counts = true;
    }
    plan(c);
    size_t moved = 0;
    for (size_t l : c.src_len) moved += l;
    if (moved == 0) {  // a collect of empty contributions only synchronises
        t_last_coll = OSGPU_RAN_BARRIER_ONLY;
        barrier(c);
        if (psync_counts) c.pSync[kCountWord] = 0;
        return;
    }

    if (kt == MEM_HOST) {
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
            fatal(name, "no GPU visible: the collectives run on the GPU");
        if (!c.ops.getmem) fatal(name, "host-memory arguments need shmem_getmem");
        // STAGED moves 1 + P (in + out) bytes per target byte over each
        // PE's PCIe link; that beats the runtime's memcpy only for large
        // calls and only when every member has a GPU (and a link) of its
        // own -- PEs sharing a GPU share its link (tools/coll_bench.py,
        // DESIGN_HISTORY.md 9).  Small calls (the fused limit, a size every member
        // shares) stay on the runtime's getmem: no GPU round trip beats a
        // same-node copy of a few KiB (1 Ki ints: 1.6 us vs 14 us for the
        // one-launch staged form, profiles/r01_mp_latency_host_coll.jsonl).
        // osgpu_set_host_path / OSGPU_HOST_PATH=staged|getmem override;
        // forced staging runs small calls as one launch
        // (run_fused_staged_copy).
        const int hp = host_path();
        const bool force_getmem = hp == OSGPU_HOST_GETMEM;
        const bool force_staged = hp == OSGPU_HOST_STAGED;
        StageSet *S = force_getmem ? nullptr : stage_setup(c);
        if (S && force_staged && !counts_done && run_fused_staged_copy(c, *S)) return;
        if (!counts_done) barrier(c);  // sources ready
        const bool small = shared_bytes(c) <= fused_max_bytes();
        if (S && (force_staged || (!small && (S->ndev == c.PE_size || c.PE_size == 1))))
            run_staged(c, *S);
        else
            run_getmem(c);
        barrier(c);
        if (psync_counts) c.pSync[kCountWord] = 0;
        return;
    }

    int cur = 0;
    HIPCHK(name, hipGetDevice(&cur));
    if (cur != dt) HIPCHK(name, hipSetDevice(dt));
    const int mode = path_mode();
    std::vector<const char *> src;
    if (mode != OSGPU_PATH_RCCL && device_sources(c, src)) {
        run_copy(c, src, counts_done);
    } else if ((mode == OSGPU_PATH_AUTO || mode == OSGPU_PATH_RCCL) && !counts_done &&
               rccl_whole_job(c)) {
        run_rccl(c);
    } else {
        fatal(name,
              "device-resident arguments need every active PE's device heap registered "
              "(osgpu_heap_register)%s",
              kind == K_BCAST || kind == K_FCOLLECT
                  ? " or an RCCL communicator over the whole job"
                  : "");
    }
    if (psync_counts) c.pSync[kCountWord] = 0;
    if (cur != dt) HIPCHK(name, hipSetDevice(cur));
}

}  // namespace

extern "C" int osgpu_last_coll_path(void) { return t_last_coll; }

// pshmem_* strong, shmem_* weak aliases (as src/broadcast.c:14-20,
// src/collect.c:14-20, src/fcollect.c:14-20, src/alltoall.c:11-23 under
// ENABLE_PSHMEM)
#define OSGPU_ALIAS(_n) __attribute__((weak, alias("pshmem_" #_n)))

#define OSGPU_DEFINE_COLL(_bits, _bytes)                                                   \
    extern "C" void pshmem_broadcast##_bits(void *target, const void *source, size_t nelems, \
                                            int PE_root, int PE_start, int logPE_stride,   \
                                            int PE_size, long *pSync)                      \
    {                                                                                      \
        collective("shmem_broadcast" #_bits, K_BCAST, _bytes, target, source, nelems,      \
                   PE_root, PE_start, logPE_stride, PE_size, pSync);                       \
    }                                                                                      \
    extern "C" void shmem_broadcast##_bits(void *, const void *, size_t, int, int, int,    \
                                           int, long *) OSGPU_ALIAS(broadcast##_bits);     \
    extern "C" void pshmem_collect##_bits(void *target, const void *source, size_t nelems, \
                                          int PE_start, int logPE_stride, int PE_size,     \
                                          long *pSync)                                     \
    {                                                                                      \
        collective("shmem_collect" #_bits, K_COLLECT, _bytes, target, source, nelems, 0,   \
                   PE_start, logPE_stride, PE_size, pSync);                                \
    }                                                                                      \
    extern "C" void shmem_collect##_bits(void *, const void *, size_t, int, int, int,      \
                                         long *) OSGPU_ALIAS(collect##_bits);              \
    extern "C" void pshmem_fcollect##_bits(void *target, const void *source, size_t nelems, \
                                           int PE_start, int logPE_stride, int PE_size,    \
                                           long *pSync)                                    \
    {                                                                                      \
        collective("shmem_fcollect" #_bits, K_FCOLLECT, _bytes, target, source, nelems, 0, \
                   PE_start, logPE_stride, PE_size, pSync);                                \
    }                                                                                      \
    extern "C" void shmem_fcollect##_bits(void *, const void *, size_t, int, int, int,     \
                                          long *) OSGPU_ALIAS(fcollect##_bits);            \
    extern "C" void pshmem_alltoall##_bits(void *target, const void *source, size_t nelems, \
                                           int PE_start, int logPE_stride, int PE_size,    \
                                           long *pSync)                                    \
    {                                                                                      \
        collective("shmem_alltoall" #_bits, K_ALLTOALL, _bytes, target, source, nelems, 0, \
                   PE_start, logPE_stride, PE_size, pSync);                                \
    }                                                                                      \
    extern "C" void shmem_alltoall##_bits(void *, const void *, size_t, int, int, int,     \
                                          long *) OSGPU_ALIAS(alltoall##_bits);

OSGPU_DEFINE_COLL(32, 4)
OSGPU_DEFINE_COLL(64, 8)
