// fused.hip -- one launch per small reduce-to-all call: the two barriers of
// the reference (src/reductions.c:82 and :113, the AMO tree barrier of
// src/shmemc/barrier.c:64-97 on pSync[0]) become epoch flags in device
// memory, written over xGMI (or inside one GPU) by the kernel itself.
//
// Why: a small call on the host-barrier path costs a launch, a completion
// wait and two host barriers (~25-30 us for 1 Ki ints, DESIGN_HISTORY.md 5); the
// compute is noise.  Here the host enqueues ONE kernel and waits once.
//
// Per active set every member PE owns a flag area (uncached device memory,
// IPC-mapped into every member, runtime.cpp sync_setup):
//   words [0, 8)   arrive[i]: epoch of the last call member i entered
//   words [8, 16)  done[i]:   epoch of the last call member i finished
//   words 16-18    tickets:   last-workgroup elections inside one launch
//   words [20, 28) count[i]:  collect only, member i's contribution + tag
// Epochs grow by one per fused call on the set, so nothing is ever reset
// (pSync stays at SHMEM_SYNC_VALUE, untouched).
//
// Protocol of one launch (member `me`, epoch E):
//  1. workgroup 0, lanes i < P: arrive[me] := E in member i's area;
//  2. every workgroup: one lane waits until all P arrive[] words of MY area
//     are >= E (every source ready, every target writable);
//  3. the combine body (grid-stride): team form -- shard of every member's
//     target, each in that member's fold order -- or pull form -- my own
//     target over all n;
//  4. every workgroup: system-scope release, then (grids of more than one
//     workgroup) a ticket; the last one
//     writes done[me] := E into every member's area and waits until all P
//     done[] words of my area are >= E (every peer finished writing my
//     target and reading my source), then stores E to a host-mapped word the
//     calling thread spins on -- it returns without waiting for the launch
//     to retire (the launch-to-completion notification is most of the
//     latency of a small call).
// Staged form (host symmetric heaps, the reference's placement): step 1 is
// preceded by the whole grid copying my host source (pinned, mapped) into
// my device staging slot, the body folds the members' staging slots into
// their result slots, and after step 4 every workgroup waits for the done
// flags and copies my result slot to my host target -- H2D, exchange and
// D2H of the STAGED path in the same single launch.
// Waits never hold the GPU for long, yet the barriers wait without bound,
// like the reference's (src/shmemc/barrier.c:78-89 spinning in
// shmemc_wait_eq_until64, src/shmemc/waituntil.c:57-71): ONE lane per grid
// (the decider) waits at most one slice (FusedArgs::timeout) and publishes
// the grid's verdict in a gate word of my flag area; every workgroup follows
// the gate, so the whole grid either passes the barrier or ends before it
// (no workgroup runs the body while another gave up).  On "not yet" the
// decider sets the host-mapped error word (1 entry, 2 exit) and the host
// launches a continuation (FusedArgs::resume) that picks up at that barrier
// -- arrivals and done flags are epochs, so nothing is repeated or undone.
// Only a member absent for longer than the device-barrier bound (none by
// default) fails the call (runtime.cpp fused_complete).
//
// Co-residency: step 2 needs every member's workgroup 0 to run while my
// workgroups wait.  Members on other GPUs always make progress; members
// sharing my GPU (separate processes: threads of one process share its few
// hardware queues and are refused in runtime.cpp) split the GPU's 256 CUs,
// one workgroup of 256 lanes per CU, so every member's grid is resident at
// once (FusedArgs::max_blocks).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include <type_traits>

#include "combine.hpp"
#include "elem_ops.hpp"

#pragma clang fp contract(off)

namespace osgpu {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int kFBlock = 256;

template <typename T>
union FVec {
    u32x4 v;
    T e[16 / sizeof(T)];
};

__device__ __forceinline__ unsigned long long ld_sys(const unsigned long long *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void st_sys(unsigned long long *p, unsigned long long v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Results are stored system-coherent (write-through, sc0 sc1): they leave no
// dirty L2 line for the completion fence to write back.  Measured at 1 MiB
// per PE, 2 processes on one GPU: fence 7.4 us with nontemporal stores and a
// fence per wave, 4.2 us with one fence per workgroup, 2.7 us write-through.
__device__ __forceinline__ void store_out(u32x4 *p, u32x4 v)
{
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}

// one lane: wait until f[0..P) >= epoch; false (and the error word set) on timeout
__device__ bool wait_epoch(const unsigned long long *f, int P, unsigned long long epoch,
                           unsigned long long timeout, int *err, int code)
{
    const unsigned long long t0 = (unsigned long long) wall_clock64();
    for (int j = 0; j < P; j++) {
        while (ld_sys(f + j) < epoch) {
            if ((unsigned long long) wall_clock64() - t0 > timeout) {
                __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                return false;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    return true;
}

// the host-mapped completion word of a device-form call
__device__ __forceinline__ void signal_host(const FusedArgs &a)
{
    __hip_atomic_store(a.done_host, a.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Gate words (my flag area): the key names this call and this launch, so a
// verdict of an earlier launch of the same call is never mistaken for this
// one's; bit 0 = pass.
__device__ __forceinline__ unsigned long long gate_key(const FusedArgs &a)
{
    return (a.epoch << 20) | ((unsigned long long) (a.attempt & 0x7ffffu) << 1);
}

__device__ __forceinline__ void gate_set(const FusedArgs &a, int word, bool pass)
{
    st_sys(a.mine + word, gate_key(a) | (pass ? 1ull : 0ull));
}

// one lane per workgroup: the grid's verdict (the decider always publishes
// within one slice: it belongs to this grid and waits on nothing of it)
__device__ __forceinline__ int gate_wait(const FusedArgs &a, int word)
{
    const unsigned long long key = gate_key(a);
    unsigned long long v;
    while (((v = ld_sys(a.mine + word)) & ~1ull) != key) __builtin_amdgcn_s_sleep(1);
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    return (int) (v & 1);
}

// Step 2: workgroup 0 waits for every member's arrival (one slice at most)
// and decides for the grid.  False: not everyone is there yet (error word 1
// set: the host continues the call with resume = 1).
__device__ __forceinline__ bool entry_gate(const FusedArgs &a, int &s_go)
{
    if (gridDim.x == 1) {  // the decider is the whole grid: no gate word round trip
        if (threadIdx.x == 0)
            s_go = wait_epoch(a.mine + kFlagArrive, a.P, a.epoch, a.timeout, a.err, 1);
        __syncthreads();
        return s_go;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0)
        gate_set(a, kFlagGateIn, wait_epoch(a.mine + kFlagArrive, a.P, a.epoch, a.timeout, a.err, 1));
    if (threadIdx.x == 0) s_go = gate_wait(a, kFlagGateIn);
    __syncthreads();
    return s_go;
}

// D outputs of one element: output d belongs to member q[d] and folds
// x[q[d]] first, then the others ascending (src/reductions.c:79-111).
// Integer ops are order-independent: fold once.
template <typename T, int OP>
__device__ __forceinline__ void fold_outputs(const T (&x)[kMaxTeam], int P, int D,
                                             const int (&q)[kMaxTeam], T (&r)[kMaxTeam])
{
    if (std::is_integral<T>::value) {
        T acc = x[0];
#pragma unroll
        for (int j = 1; j < kMaxTeam; j++)
            if (j < P) acc = Elem<T, OP>::f(acc, x[j]);
#pragma unroll
        for (int d = 0; d < kMaxTeam; d++) r[d] = acc;
        return;
    }
#pragma unroll
    for (int d = 0; d < kMaxTeam; d++) {
        if (d >= D) break;
        const int o = q[d];
        T acc = x[0];
#pragma unroll
        for (int j = 0; j < kMaxTeam; j++)
            if (j == o) acc = x[j];
#pragma unroll
        for (int j = 0; j < kMaxTeam; j++)
            if (j < P && j != o) acc = Elem<T, OP>::f(acc, x[j]);
        r[d] = acc;
    }
}

template <typename T, int OP>
__device__ __forceinline__ void do_elem(const FusedArgs &a, size_t i)
{
    const T *const *src = reinterpret_cast<const T *const *>(a.src);
    T x[kMaxTeam], r[kMaxTeam];
#pragma unroll
    for (int j = 0; j < kMaxTeam; j++)
        x[j] = j < a.P ? src[j][i] : T();
    fold_outputs<T, OP>(x, a.P, a.D, a.q, r);
#pragma unroll
    for (int d = 0; d < kMaxTeam; d++)
        if (d < a.D) static_cast<T *>(a.dst[d])[i] = r[d];
}

// Lane 0 of every workgroup, after the workgroup's stores: release them
// system-wide and take ticket `w`; true for the last workgroup of the grid
// (which resets the ticket for the next launch and acquires).
__device__ __forceinline__ bool last_workgroup(const FusedArgs &a, int w)
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    if (gridDim.x == 1) return true;
    unsigned *ticket = reinterpret_cast<unsigned *>(a.mine + w);
    const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    if (t != gridDim.x - 1) return false;
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    return true;
}

// Grid-stride byte copy between host memory (pinned, mapped) and a device
// staging slot: 16-B vectors when both ends allow it, else dwords, else bytes.
__device__ void stage_copy(void *dst, const void *src, size_t nbytes)
{
    const size_t tid = (size_t) blockIdx.x * kFBlock + threadIdx.x;
    const size_t stride = (size_t) gridDim.x * kFBlock;
    const uintptr_t al = (uintptr_t) dst | (uintptr_t) src;
    if ((al & 15) == 0) {
        const size_t nv = nbytes / 16;
        for (size_t j = tid; j < nv; j += stride)
            static_cast<u32x4 *>(dst)[j] = static_cast<const u32x4 *>(src)[j];
        for (size_t b = nv * 16 + tid; b < nbytes; b += stride)
            static_cast<char *>(dst)[b] = static_cast<const char *>(src)[b];
    } else if ((al & 3) == 0) {
        const size_t nw = nbytes / 4;
        for (size_t j = tid; j < nw; j += stride)
            static_cast<unsigned *>(dst)[j] = static_cast<const unsigned *>(src)[j];
        for (size_t b = nw * 4 + tid; b < nbytes; b += stride)
            static_cast<char *>(dst)[b] = static_cast<const char *>(src)[b];
    } else {
        for (size_t b = tid; b < nbytes; b += stride)
            static_cast<char *>(dst)[b] = static_cast<const char *>(src)[b];
    }
}

// Step 4 (device form): release, ticket; the last workgroup signals done,
// waits for every member's done (one slice) and publishes the host
// completion word.  resume 2: only that wait, by workgroup 0.
__device__ __forceinline__ void fused_done(const FusedArgs &a)
{
    if (a.resume == 2) {
        if (blockIdx.x == 0 && threadIdx.x == 0 &&
            wait_epoch(a.mine + kFlagDone, a.P, a.epoch, a.timeout, a.err, 2))
            signal_host(a);
        return;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    if (threadIdx.x == 0 && last_workgroup(a, kFlagTicket)) {
        for (int i = 0; i < a.P; i++) st_sys(a.flags[i] + kFlagDone + a.me, a.epoch);
        if (wait_epoch(a.mine + kFlagDone, a.P, a.epoch, a.timeout, a.err, 2))
            signal_host(a);
    }
}

// Grid-stride copy of one piece at the widest width both ends allow.
__device__ __forceinline__ void copy_piece(char *dst, const char *src, size_t nb, size_t tid,
                                           size_t stride)
{
    const uintptr_t al = (uintptr_t) src | (uintptr_t) dst;
    size_t done = 0;
    if ((al & 15) == 0) {
        const size_t nv = nb / 16;
        for (size_t j = tid; j < nv; j += stride)
            store_out(reinterpret_cast<u32x4 *>(dst) + j,
                      __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(src) + j));
        done = nv * 16;
    } else if ((al & 7) == 0) {
        const size_t nw = nb / 8;
        for (size_t j = tid; j < nw; j += stride)
            reinterpret_cast<unsigned long long *>(dst)[j] =
                reinterpret_cast<const unsigned long long *>(src)[j];
        done = nw * 8;
    } else if ((al & 3) == 0) {
        const size_t nw = nb / 4;
        for (size_t j = tid; j < nw; j += stride)
            reinterpret_cast<unsigned *>(dst)[j] = reinterpret_cast<const unsigned *>(src)[j];
        done = nw * 4;
    }
    for (size_t b = done + tid; b < nb; b += stride) dst[b] = src[b];
}

// The data-movement collectives' small calls (shmem_collect.cpp): the pieces
// of my target pulled from every member's source, between the same device
// barriers.  Segment d: a.seg_bytes[d] bytes from a.src[d] to a.dst[d].
// Staged form (host heaps): my host source is first copied into my device
// staging slot by the whole grid, the last workgroup arrives; the segments
// then read the members' staging slots and write my host target directly.
__global__ __launch_bounds__(kFBlock) void fused_copy_kernel(FusedArgs a)
{
    __shared__ int s_go;
    if (a.resume < 2) {
        if (a.resume == 0 && a.host_in) {
            stage_copy(a.stage_mine, a.host_in, a.host_bytes);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __syncthreads();
            if (threadIdx.x == 0 && last_workgroup(a, kFlagTicketIn))
                for (int i = 0; i < a.P; i++) st_sys(a.flags[i] + kFlagArrive + a.me, a.epoch);
        } else if (a.resume == 0 && blockIdx.x == 0 && (int) threadIdx.x < a.P) {
            st_sys(a.flags[threadIdx.x] + kFlagArrive + a.me, a.epoch);
        }
        if (!entry_gate(a, s_go)) return;
        const size_t tid = (size_t) blockIdx.x * kFBlock + threadIdx.x;
        const size_t stride = (size_t) gridDim.x * kFBlock;
        for (int d = 0; d < a.nseg; d++)
            copy_piece(static_cast<char *>(a.dst[d]), static_cast<const char *>(a.src[d]),
                       a.seg_bytes[d], tid, stride);
    }
    fused_done(a);
}

// collect (shmem_collect.cpp, src/shmemc/collect.c:24-69): contributions
// differ per member, so the counts ARE the arrival: workgroup 0 writes
// (tag << 40 | count) into slot me of every member's area, tag = the set's
// collect sequence number (the same on every member; consecutive collects
// differ by one, so a slot holds this call's count or the previous one's --
// no member writes the next before every member has passed this call's done
// barrier, which follows its reads).  Lanes i < P of every workgroup wait
// for slot i to carry this call's tag.  All members see the same counts, so
// they all make the same choice: if the gathered total fits copy_limit the
// pieces are copied here (member i's source to my output at the prefix
// offset of i); otherwise the launch is only the count exchange and the
// entry barrier, and the host copies.  The host learns the counts (and the
// choice) from counts_host.  arrive[] is not written: epochs only grow, so
// the next fused call's wait (arrive >= E') is unaffected.
__global__ __launch_bounds__(kFBlock) void fused_collect_kernel(FusedArgs a)
{
    __shared__ int s_go;
    __shared__ unsigned long long s_cnt[kMaxTeam];
    constexpr unsigned long long kCountMask = (1ull << kCountBits) - 1;
    const unsigned long long tag = a.count_tag & ((1ull << (64 - kCountBits)) - 1);
    if (a.resume == 2) {
        fused_done(a);
        return;
    }
    if (a.resume == 0 && blockIdx.x == 0 && (int) threadIdx.x < a.P)
        st_sys(a.flags[threadIdx.x] + kFlagCount + a.me,
               tag << kCountBits | ((unsigned long long) a.my_count & kCountMask));
    // workgroup 0 decides for the grid: lanes i < P wait (one slice at most)
    // for slot i to carry this call's tag
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) s_go = 1;
        __syncthreads();
        if ((int) threadIdx.x < a.P) {
            const unsigned long long *w = a.mine + kFlagCount + threadIdx.x;
            const unsigned long long t0 = (unsigned long long) wall_clock64();
            while ((ld_sys(w) >> kCountBits) != tag) {
                if ((unsigned long long) wall_clock64() - t0 > a.timeout) {
                    s_go = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            if (!s_go) __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            gate_set(a, kFlagGateIn, s_go);
        }
    }
    if (threadIdx.x == 0) s_go = gate_wait(a, kFlagGateIn);
    __syncthreads();
    if (!s_go) return;
    // the slots hold this call's counts until every member has passed its
    // done barrier
    if ((int) threadIdx.x < a.P) s_cnt[threadIdx.x] = ld_sys(a.mine + kFlagCount + threadIdx.x) & kCountMask;
    __syncthreads();
    unsigned long long total = 0;
    bool fits = true;
    for (int i = 0; i < a.P; i++) {
        total += s_cnt[i];
        fits = fits && s_cnt[i] <= a.src_avail[i];
    }
    const bool copy = fits && total <= a.copy_limit;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        for (int i = 0; i < a.P; i++) st_sys(a.counts_host + i, s_cnt[i]);
        st_sys(a.counts_host + kMaxTeam, copy ? 1ull : 0ull);
        if (!fits) __hip_atomic_store(a.err, 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (copy) {
        const size_t tid = (size_t) blockIdx.x * kFBlock + threadIdx.x;
        const size_t stride = (size_t) gridDim.x * kFBlock;
        char *out = static_cast<char *>(a.dst[0]);
        size_t off = 0;
        for (int i = 0; i < a.P; i++) {
            if (s_cnt[i]) copy_piece(out + off, static_cast<const char *>(a.src[i]), s_cnt[i],
                                     tid, stride);
            off += s_cnt[i];
        }
    }
    fused_done(a);
}

template <typename T, int OP, bool VEC>
__global__ __launch_bounds__(kFBlock) void fused_kernel(FusedArgs a)
{
    __shared__ int s_go;
    const bool tr = a.trace && blockIdx.x == 0 && threadIdx.x == 0 && a.resume == 0;
    if (tr) a.trace[0] = (unsigned long long) wall_clock64();
    if (a.resume < 2) {
        // 1. arrive (src/reductions.c:82 -- my source is ready, my target
        // free).  Staged form: my host source is first copied into my staging
        // slot by the whole grid; the last workgroup to finish its part
        // arrives.  A continuation (resume 1) has arrived already.
        if (a.resume == 0 && a.host_in) {
            stage_copy(a.stage_mine, a.host_in, a.host_bytes);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __syncthreads();
            if (threadIdx.x == 0 && last_workgroup(a, kFlagTicketIn))
                for (int i = 0; i < a.P; i++) st_sys(a.flags[i] + kFlagArrive + a.me, a.epoch);
        } else if (a.resume == 0 && blockIdx.x == 0 && (int) threadIdx.x < a.P) {
            st_sys(a.flags[threadIdx.x] + kFlagArrive + a.me, a.epoch);
        }
        // 2. every member's arrival (one decider, the grid follows)
        if (!entry_gate(a, s_go)) return;
        if (tr) a.trace[1] = (unsigned long long) wall_clock64();

        // 3. combine body
        if (VEC) {
            constexpr int W = 16 / sizeof(T);
            if (blockIdx.x == 0 && (int) threadIdx.x < a.nedge) {
                const size_t e =
                    threadIdx.x < a.head ? threadIdx.x : a.tail_start + (threadIdx.x - a.head);
                do_elem<T, OP>(a, e);
            }
            const size_t stride = (size_t) gridDim.x * kFBlock;
            for (size_t j = (size_t) blockIdx.x * kFBlock + threadIdx.x; j < a.nvec; j += stride) {
                FVec<T> in[kMaxTeam];
#pragma unroll
                for (int p = 0; p < kMaxTeam; p++)
                    if (p < a.P)
                        in[p].v = __builtin_nontemporal_load(
                            reinterpret_cast<const u32x4 *>(static_cast<const T *>(a.src[p]) +
                                                            a.head) + j);
                FVec<T> out[kMaxTeam];
#pragma unroll
                for (int w = 0; w < W; w++) {
                    T x[kMaxTeam], r[kMaxTeam];
#pragma unroll
                    for (int p = 0; p < kMaxTeam; p++) x[p] = p < a.P ? in[p].e[w] : T();
                    fold_outputs<T, OP>(x, a.P, a.D, a.q, r);
#pragma unroll
                    for (int d = 0; d < kMaxTeam; d++) out[d].e[w] = r[d];
                }
#pragma unroll
                for (int d = 0; d < kMaxTeam; d++)
                    if (d < a.D)
                        store_out(
                            reinterpret_cast<u32x4 *>(static_cast<T *>(a.dst[d]) + a.head) + j,
                            out[d].v);
            }
        } else {
            const size_t stride = (size_t) gridDim.x * kFBlock;
            for (size_t i = (size_t) blockIdx.x * kFBlock + threadIdx.x; i < a.n; i += stride)
                do_elem<T, OP>(a, i);
        }

        // 4. completion (src/reductions.c:113): my stores and reads are
        // done.  Every wave waits for its own stores, then ONE lane per
        // workgroup makes them visible system-wide (an L2 writeback per fence:
        // one per workgroup, not one per wave) and takes a ticket; the last
        // workgroup signals done and waits for every member's (one slice).
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __syncthreads();
        if (tr) a.trace[2] = (unsigned long long) wall_clock64();
        if (threadIdx.x == 0) {
            const bool last = last_workgroup(a, kFlagTicket);
            if (tr) a.trace[3] = (unsigned long long) wall_clock64();
            if (last) {
                if (a.trace) a.trace[4] = a.trace[5] = (unsigned long long) wall_clock64();
                for (int i = 0; i < a.P; i++) st_sys(a.flags[i] + kFlagDone + a.me, a.epoch);
                const bool all = wait_epoch(a.mine + kFlagDone, a.P, a.epoch, a.timeout, a.err, 2);
                if (!a.host_out) {
                    if (all) {
                        if (a.trace) a.trace[6] = (unsigned long long) wall_clock64();
                        // the host returns on this word, without waiting for
                        // the launch to retire
                        signal_host(a);
                    }
                } else {
                    gate_set(a, kFlagGateOut, all);
                }
            }
        }
        if (!a.host_out) return;
    } else if (!a.host_out) {
        // continuation at the exit barrier, device form: the done wait only
        if (blockIdx.x == 0 && threadIdx.x == 0 &&
            wait_epoch(a.mine + kFlagDone, a.P, a.epoch, a.timeout, a.err, 2))
            signal_host(a);
        return;
    } else if (blockIdx.x == 0 && threadIdx.x == 0) {
        // continuation at the exit barrier, staged form: workgroup 0 decides
        gate_set(a, kFlagGateOut,
                 wait_epoch(a.mine + kFlagDone, a.P, a.epoch, a.timeout, a.err, 2));
    }
    // Staged form: once every member has written its shard of my result
    // slot (the exit gate passed), the whole grid copies it to my host
    // target; the last workgroup to finish publishes the completion word.
    if (threadIdx.x == 0) s_go = gate_wait(a, kFlagGateOut);
    __syncthreads();
    if (!s_go) return;
    stage_copy(a.host_out, a.stage_result, a.host_bytes);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    if (threadIdx.x == 0 && last_workgroup(a, kFlagTicketOut)) {
        if (a.trace) a.trace[6] = (unsigned long long) wall_clock64();
        __hip_atomic_store(a.done_host, a.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

template <typename T, int OP>
hipError_t fused_launch_t(FusedArgs a, hipStream_t s)
{
    constexpr int W = 16 / sizeof(T);
    const uintptr_t phase = (uintptr_t) a.src[0] & 15;
    bool vec = (phase % sizeof(T)) == 0;
    for (int p = 0; p < a.P; p++) vec = vec && (((uintptr_t) a.src[p] & 15) == phase);
    for (int d = 0; d < a.D; d++) vec = vec && (((uintptr_t) a.dst[d] & 15) == phase);
    size_t work;
    if (vec) {
        size_t head = phase ? (16 - phase) / sizeof(T) : 0;
        if (head > a.n) head = a.n;
        a.head = head;
        a.nvec = (a.n - head) / W;
        a.tail_start = head + a.nvec * W;
        a.nedge = (int) (head + (a.n - a.tail_start));
        work = a.nvec;
    } else {
        a.head = a.nvec = a.tail_start = 0;
        a.nedge = 0;
        work = a.n;
    }
    size_t blocks = (work + kFBlock - 1) / kFBlock;
    if (blocks < 1) blocks = 1;
    if (blocks > (size_t) a.max_blocks) blocks = (size_t) a.max_blocks;
    if (vec)
        hipLaunchKernelGGL((fused_kernel<T, OP, true>), dim3((unsigned) blocks), dim3(kFBlock), 0,
                           s, a);
    else
        hipLaunchKernelGGL((fused_kernel<T, OP, false>), dim3((unsigned) blocks), dim3(kFBlock),
                           0, s, a);
    return hipGetLastError();
}

#define FUSED_CASE(OPC)                                                        \
    case OPC: return fused_launch_t<T, OPC>(a, s);

template <typename T>
hipError_t fused_int(int op, const FusedArgs &a, hipStream_t s)
{
    switch (op) {
        FUSED_CASE(OP_SUM) FUSED_CASE(OP_PROD) FUSED_CASE(OP_AND) FUSED_CASE(OP_OR)
        FUSED_CASE(OP_XOR) FUSED_CASE(OP_MAX) FUSED_CASE(OP_MIN)
    }
    return hipErrorInvalidValue;
}

template <typename T>
hipError_t fused_real(int op, const FusedArgs &a, hipStream_t s)
{
    switch (op) {
        FUSED_CASE(OP_SUM) FUSED_CASE(OP_PROD) FUSED_CASE(OP_MAX) FUSED_CASE(OP_MIN)
    }
    return hipErrorInvalidValue;
}

template <typename T>
hipError_t fused_cplx(int op, const FusedArgs &a, hipStream_t s)
{
    switch (op) {
        FUSED_CASE(OP_SUM) FUSED_CASE(OP_PROD)
    }
    return hipErrorInvalidValue;
}

}  // namespace

hipError_t launch_fused_copy(const FusedArgs &a0, hipStream_t s)
{
    FusedArgs a = a0;
    if (a.P < 2 || a.P > kMaxTeam || a.nseg < 0 || a.nseg > kMaxTeam || a.me < 0 ||
        a.me >= a.P || a.max_blocks < 1 || a.max_blocks > kFusedBlocksPerGpu)
        return hipErrorInvalidValue;
    size_t most = a.host_in ? a.host_bytes : 0;
    for (int d = 0; d < a.nseg; d++) most = a.seg_bytes[d] > most ? a.seg_bytes[d] : most;
    size_t blocks = (most / 16 + kFBlock - 1) / kFBlock;
    if (blocks < 1) blocks = 1;
    if (blocks > (size_t) a.max_blocks) blocks = (size_t) a.max_blocks;
    hipLaunchKernelGGL(fused_copy_kernel, dim3((unsigned) blocks), dim3(kFBlock), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_fused_collect(const FusedArgs &a, hipStream_t s)
{
    if (a.P < 2 || a.P > kMaxTeam || a.me < 0 || a.me >= a.P || a.max_blocks < 1 ||
        a.max_blocks > kFusedBlocksPerGpu || !a.counts_host || !a.dst[0])
        return hipErrorInvalidValue;
    // pieces are copied one after another, each grid-stride: sized by my
    // estimate of one piece (contributions like mine), as the fused copy
    const size_t est = a.my_count < a.copy_limit ? a.my_count : a.copy_limit;
    size_t blocks = (est / 16 + kFBlock - 1) / kFBlock;
    if (blocks < 1) blocks = 1;
    if (blocks > (size_t) a.max_blocks) blocks = (size_t) a.max_blocks;
    hipLaunchKernelGGL(fused_collect_kernel, dim3((unsigned) blocks), dim3(kFBlock), 0, s, a);
    return hipGetLastError();
}

bool fused_supported(int type) { return type != T_LONGDOUBLE && type >= 0 && type < T_NTYPES; }

hipError_t launch_fused(int type, int op, const FusedArgs &a, hipStream_t s)
{
    if (a.P < 2 || a.P > kMaxTeam || a.D < 1 || a.D > kMaxTeam || a.me < 0 || a.me >= a.P ||
        a.max_blocks < 1 || a.max_blocks > kFusedBlocksPerGpu)
        return hipErrorInvalidValue;
    switch (type) {
    case T_SHORT: return fused_int<int16_t>(op, a, s);
    case T_INT: return fused_int<int32_t>(op, a, s);
    case T_LONG:
    case T_LONGLONG: return fused_int<int64_t>(op, a, s);
    case T_FLOAT: return fused_real<float>(op, a, s);
    case T_DOUBLE: return fused_real<double>(op, a, s);
    case T_COMPLEXF: return fused_cplx<cfloat>(op, a, s);
    case T_COMPLEXD: return fused_cplx<cdouble>(op, a, s);
    }
    return hipErrorInvalidValue;
}

}  // namespace osgpu
