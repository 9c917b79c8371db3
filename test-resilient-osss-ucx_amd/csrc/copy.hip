// copy.hip -- the data-movement kernel of the broadcast / collect / fcollect /
// alltoall collectives (shmem_collect.cpp): up to kMaxCopySegs independent
// byte ranges (src -> dst), each source in local HBM or in a peer GPU's HBM
// mapped into this process, copied by ONE launch.
//
// The reference moves these bytes with shmemc_put / shmemc_get over UCX
// (src/shmemc/fcollect.c:32-38, src/shmemc/collect.c:52-64,
// src/shmemc/broadcast.c:39-41).  Here the owner of every target pulls all
// its pieces with 16-byte streaming loads: HBM-bound on one GPU, xGMI-bound
// across GPUs; 2 bytes of traffic (read + write) per byte copied.
//
// Layout of a launch: each segment gets ceil(body / (256 * U)) workgroups of
// 256 lanes, each lane U 16-byte vectors (all loads issued before the first
// store, non-temporal both ways -- the shape tools/tune_combine.hip found
// fastest for the combine).  The segments' tiles are dealt round-robin
// (workgroup b -> segment b % m, for as many rounds as the smallest segment
// has tiles; the rest of the larger segments follow, segment by segment):
// dispatch runs workgroups roughly in order, so with segments one after
// another the ~2 K workgroups resident at any moment would all stream ONE
// segment -- over xGMI one peer link at a time while the others idle.
// Round-robin keeps every segment (every peer's link) streaming at once.  Vectors are aligned on the DESTINATION; the
// source may sit at any 4-byte phase (gfx950 serves dword-aligned
// global_load_dwordx4), so a 32-bit collect whose block offsets are not
// 16-byte multiples stays on the vector path.  The first workgroup of a
// segment also copies the unaligned head (< 16 B) and tail (< 16 B) bytes.
// A segment whose source and destination differ in byte phase (impossible for
// 32/64-bit elements at natural alignment) takes the byte kernel.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdlib.h>

#include "combine.hpp"

namespace osgpu {
namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_a4 __attribute__((aligned(4)));  // dword-aligned 16-B load

constexpr int kThreads = 256;
constexpr int kU = 4;  // 16-B vectors per lane
constexpr size_t kBlockBytes = (size_t) kThreads * kU * 16;

struct SegTable {
    const char *src[kMaxCopySegs];
    char *dst[kMaxCopySegs];
    size_t bytes[kMaxCopySegs];
    unsigned first_block[kMaxCopySegs + 1];  // of the blocked part (tiles past `rounds`)
    unsigned rounds;                          // round-robin rounds (vector kernel)
    int n;
};

__device__ __forceinline__ int find_seg(const SegTable &t, unsigned b)
{
    int k = 0;
#pragma unroll
    for (int i = 1; i < kMaxCopySegs; i++)
        if (i < t.n && b >= t.first_block[i]) k = i;
    return k;
}

__global__ __launch_bounds__(kThreads) void copy_vec_kernel(SegTable t)
{
    // round-robin part first: block b -> segment b % n, tile b / n; then
    // every segment's tiles from `rounds` on, segment after segment
    const unsigned inter = t.rounds * (unsigned) t.n;
    int k;
    unsigned lb;
    if (blockIdx.x < inter) {
        k = (int) (blockIdx.x % (unsigned) t.n);
        lb = blockIdx.x / (unsigned) t.n;
    } else {
        const unsigned b = blockIdx.x - inter;
        k = find_seg(t, b);
        lb = t.rounds + (b - t.first_block[k]);
    }
    const char *s = t.src[k];
    char *d = t.dst[k];
    const size_t bytes = t.bytes[k];
    size_t head = (size_t) ((0 - (uintptr_t) d) & 15);
    if (head > bytes) head = bytes;
    const size_t nvec = (bytes - head) / 16;
    const size_t tail0 = head + nvec * 16;
    if (lb == 0) {
        const unsigned x = threadIdx.x;
        if (x < head) d[x] = s[x];
        if (x < bytes - tail0) d[tail0 + x] = s[tail0 + x];
    }
    const u32x4_a4 *sv = reinterpret_cast<const u32x4_a4 *>(s + head);
    u32x4 *dv = reinterpret_cast<u32x4 *>(d + head);
    const size_t base = (size_t) lb * kThreads * kU + threadIdx.x;
    u32x4 v[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) {
        const size_t i = base + (size_t) u * kThreads;
        if (i < nvec) v[u] = __builtin_nontemporal_load(sv + i);
    }
#pragma unroll
    for (int u = 0; u < kU; u++) {
        const size_t i = base + (size_t) u * kThreads;
        if (i < nvec) __builtin_nontemporal_store(v[u], dv + i);
    }
}

__global__ __launch_bounds__(kThreads) void copy_byte_kernel(SegTable t)
{
    const int k = find_seg(t, blockIdx.x);
    const size_t per_block = (size_t) kThreads * 16;
    const size_t lo = (size_t) (blockIdx.x - t.first_block[k]) * per_block;
    for (size_t i = lo + threadIdx.x; i < t.bytes[k] && i < lo + per_block; i += kThreads)
        t.dst[k][i] = t.src[k][i];
}

// plain (cached) 8-byte loads, one word per lane: the preflight's owner-side
// read, which first leaves the lines in this GPU's L2 and later re-reads
// them after peers wrote them remotely (heap.cpp, remote-write leg)
__global__ __launch_bounds__(kThreads) void probe_load_kernel(const unsigned long long *src,
                                                              unsigned long long *dst,
                                                              unsigned words)
{
    if (threadIdx.x < words) dst[threadIdx.x] = src[threadIdx.x];
}

// One range across PCIe, device <-> pinned host memory mapped into the GPU
// (the STAGED path's legs, shmem_reduce.cpp run_staged).  A fixed grid of
// kHostGrid workgroups walks the range in tiles of kThreads * kU vectors,
// every lane's kU loads in flight before its stores.  Why a kernel and not
// the DMA engine: the engine's device-to-host rate follows the GPU's power
// state -- 28.4-29.5 GB/s for the first second of an idle box and again at
// random later, 56.6 once the state is up -- while this kernel's writes
// hold 53.9-54.0 GB/s in both states, and a DMA read beside it 41.8-42.0
// each way (tools/d2h_timeline.hip, profiles/r05_dma_state_timeline.jsonl).
// Vectors are aligned on the destination; block 0 copies the head and the
// tail bytes.
__global__ __launch_bounds__(kThreads) void host_copy_kernel(const char *__restrict__ s,
                                                             char *__restrict__ d, size_t bytes)
{
    size_t head = (size_t) ((0 - (uintptr_t) d) & 15);
    if (head > bytes) head = bytes;
    const size_t nvec = (bytes - head) / 16;
    const size_t tail0 = head + nvec * 16;
    if (blockIdx.x == 0) {
        const unsigned x = threadIdx.x;
        if (x < head) d[x] = s[x];
        if (x < bytes - tail0) d[tail0 + x] = s[tail0 + x];
    }
    const u32x4_a4 *sv = reinterpret_cast<const u32x4_a4 *>(s + head);
    u32x4 *dv = reinterpret_cast<u32x4 *>(d + head);
    const size_t stride = (size_t) gridDim.x * kThreads * kU;
    for (size_t base = (size_t) blockIdx.x * kThreads * kU + threadIdx.x; base < nvec;
         base += stride) {
        u32x4 v[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const size_t i = base + (size_t) u * kThreads;
            if (i < nvec) v[u] = __builtin_nontemporal_load(sv + i);
        }
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const size_t i = base + (size_t) u * kThreads;
            if (i < nvec) dv[i] = v[u];
        }
    }
}

}  // namespace

hipError_t launch_host_copy(void *dst, const void *src, size_t bytes, hipStream_t stream)
{
    static const unsigned grid = [] {
        const char *e = getenv("OSGPU_HOST_COPY_GRID");
        const long v = e ? atol(e) : 256;
        return (unsigned) (v < 1 ? 1 : (v > 4096 ? 4096 : v));
    }();
    if (bytes == 0) return hipSuccess;
    if (((uintptr_t) src ^ (uintptr_t) dst) & 3) {  // byte phases differ: the byte kernel
        CopySeg g = {src, dst, bytes};
        return launch_copy(&g, 1, stream);
    }
    const size_t tiles = (bytes + kBlockBytes - 1) / kBlockBytes;
    hipLaunchKernelGGL(host_copy_kernel, dim3((unsigned) (tiles < grid ? tiles : grid)),
                       dim3(kThreads), 0, stream, static_cast<const char *>(src),
                       static_cast<char *>(dst), bytes);
    return hipGetLastError();
}

hipError_t launch_probe_load(const void *src, void *dst, size_t bytes, hipStream_t stream)
{
    static_assert(kProbeLoadBytes == (size_t) kThreads * 8, "one word per lane");
    if (bytes % 8 || bytes > kProbeLoadBytes || ((uintptr_t) src | (uintptr_t) dst) & 7)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(probe_load_kernel, dim3(1), dim3(kThreads), 0, stream,
                       static_cast<const unsigned long long *>(src),
                       static_cast<unsigned long long *>(dst), (unsigned) (bytes / 8));
    return hipGetLastError();
}

hipError_t launch_copy(const CopySeg *segs, int nseg, hipStream_t stream)
{
    SegTable vt{}, bt{};
    unsigned vblocks = 0, bblocks = 0;
    for (int i = 0; i < nseg; i++) {
        const CopySeg &g = segs[i];
        if (g.bytes == 0) continue;
        const uintptr_t phase = (uintptr_t) g.src ^ (uintptr_t) g.dst;
        SegTable &t = (phase & 3) ? bt : vt;
        unsigned &nb = (phase & 3) ? bblocks : vblocks;
        const size_t per = (phase & 3) ? (size_t) kThreads * 16 : kBlockBytes;
        const size_t blocks = (g.bytes + per - 1) / per;
        if (blocks > 0x7fffffffu - nb) return hipErrorInvalidValue;
        if (t.n == kMaxCopySegs) return hipErrorInvalidValue;  // callers batch
        t.src[t.n] = (const char *) g.src;
        t.dst[t.n] = (char *) g.dst;
        t.bytes[t.n] = g.bytes;
        t.first_block[t.n] = nb;
        t.n++;
        nb += (unsigned) blocks;
    }
    if (vt.n) {
        // round-robin rounds = the smallest segment's tile count; the
        // blocked table then holds only each segment's tiles beyond them
        unsigned rounds = ~0u;
        for (int i = 0; i < vt.n; i++) {
            const unsigned next = i + 1 < vt.n ? vt.first_block[i + 1] : vblocks;
            rounds = next - vt.first_block[i] < rounds ? next - vt.first_block[i] : rounds;
        }
        unsigned nb = 0;
        for (int i = 0; i < vt.n; i++) {
            const unsigned next = i + 1 < vt.n ? vt.first_block[i + 1] : vblocks;
            const unsigned tiles = next - vt.first_block[i];
            vt.first_block[i] = nb;
            nb += tiles - rounds;
        }
        vt.first_block[vt.n] = nb;
        vt.rounds = rounds;
        hipLaunchKernelGGL(copy_vec_kernel, dim3(vblocks), dim3(kThreads), 0, stream, vt);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (bt.n) {
        bt.first_block[bt.n] = bblocks;
        hipLaunchKernelGGL(copy_byte_kernel, dim3(bblocks), dim3(kThreads), 0, stream, bt);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace osgpu
