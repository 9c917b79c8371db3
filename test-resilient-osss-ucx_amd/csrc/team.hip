// team.hip -- owner-computes reduce-to-all for a whole active set.
//
// The reference makes every PE pull every other PE's whole source
// (src/reductions.c:84-111): P*(P-1)*N elements cross the PE boundary and
// every PE reads P*N.  Here PE g (index g of the active set) owns the element
// shard [lo_g, hi_g) of ALL targets (targets are symmetric objects in
// OpenSHMEM 1.4): it reads shard g of the P sources once, computes the P
// per-PE results -- each in that PE's own fold order, op(op(x_q, x_0), x_1)
// ... skipping q (src/reductions.c:79-111) -- and writes shard g of every
// PE's target.  Per call the team moves 2*P*N*s bytes instead of
// P*(P+1)*N*s; across GPUs each PE exchanges (P-1)/P * N * s each way, the
// traffic of a reduce-scatter + all-gather, and the result stays bit-exact.
//
// Order-independent ops (every integer op) fold once and store P copies.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include <type_traits>

#include "combine.hpp"
#include "elem_ops.hpp"

#pragma clang fp contract(off)

namespace osgpu {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <typename T>
union TVec {
    u32x4 v;
    T e[16 / sizeof(T)];
};

template <typename T, int P>
struct TeamPtrs {
    const T *src[P];
    T *dst[P];
};

constexpr int kTeamBlock = 256;

// ---------------------------------------------------------------- shapes
// Tuning constants of the launch shapes.  Each was chosen by an in-process
// A/B on the same allocations (tools/team_inproc_ab.py); the records are
// cited here and in DESIGN_HISTORY.md.  The four left overridable with -D
// (tools/build_ab.sh) are the ones a round-6 A/B still builds.
//
// Above 4 members: U vectors per input per lane, G of them in flight per
// round.  U = 4 in two rounds of G = 2 (16 vectors of 16 B in flight per lane
// at 8 members) beat one round of U = G = 2 at P = 8 for every type: float
// 0.715 -> 0.786, complexf 0.723 -> 0.790 of 8 TB/s
// (profiles/r03_team_variants_interleaved.jsonl); U = G = 4 spills the
// 8-input complexf fold (0.45).
constexpr int kTeamU8 = 4;
constexpr int kTeamG8 = 2;  // complex sum; every type when members are remote
// ... for the real (non-complex) types on one GPU: one round of all U = 4
// vectors, 1.006x over 7 (type, op) pairs at 5-8 members
// (profiles/r05_team_p8_tile_ab.jsonl).  Not measured across GPUs (xGMI):
// calls with remote members keep G = kTeamG8 (TeamShape REMOTE).
#ifndef OSGPU_TEAM_G8R
#define OSGPU_TEAM_G8R 4
#endif
// the register-heavy folds above 4 members (complex products: 4-6 VALU
// temporaries per element per output) take rounds of kTeamGH vectors
constexpr int kTeamGH = 2;
// Above 4 members integer folds issue round r+1's loads before round r's
// folds and stores (two round buffers): +0.5-1 %; for floating-point folds
// the two buffers cost 0.2-0.4 of the rate in round 4 and 2-3 % once inlined
// (profiles/r04_team_type_op_sweep.jsonl, r05_team_p8_tile_ab.jsonl), so
// only integers pipeline.  Ordered folds above 4 members fold, check and
// store one output at a time (only one output vector live).
// Vectors per input per lane for 2 and for 3-4 members in the register form
// (all loaded before the first fold): U = 2 at 2 members ran 0.71-0.75
// against 0.77 with U = 4.
constexpr int kTeamU2 = 4;
constexpr int kTeamU4 = 4;
// The LDS-staged kernel (team_lds_kernel, one wave per member) serves
// OSGPU_TEAM_LDS_MIN_P .. OSGPU_TEAM_LDS_MAX_P members.  2 members: 1.03x
// over the register form for double sum, 1.00-1.07x for every (type, op)
// probed (profiles/r05_team_p2_ab.jsonl); 3-4 members ahead or equal on
// every box; 5-8 members: the register form's best (0.81 of 8 TB/s at 8) is
// above the LDS form's (0.75) (r04_team_place_3/4.jsonl).  Calls with
// remote members keep the round-4 range, 3-4 (TeamShape REMOTE): the 2-member
// A/B ran on one GPU only.
#ifndef OSGPU_TEAM_LDS_MIN_P
#define OSGPU_TEAM_LDS_MIN_P 2
#endif
#ifndef OSGPU_TEAM_LDS_MAX_P
#define OSGPU_TEAM_LDS_MAX_P 4
#endif
// 16-B vectors per lane per LDS tile: U = 1 (1 KiB per member per workgroup,
// round 6).  In one process on the same allocations against U = 2
// (tools/team_inproc_ab.py, profiles/r06_lds_u1_confirm_ab.jsonl: 6 (type,
// op) pairs x 2-4 members x 4 allocations) every pair's median was faster:
// 1.025x / 1.026x / 1.070x at 2 / 3 / 4 members overall (int xor and float
// prod 1.09x at 4, complex double prod 1.05-1.09x), lifting the 4-member
// kernel from 0.963 to 1.021 of the same-mix copy
// (profiles/r06_team_lds_u1_ab.jsonl: 1.04x / 1.00x / 1.09x for double
// sum).  Above 4 members it wins at 5, 6 and 8 for real types other than
// FP max/min (TeamShape kLds below) and loses at 7 and for complex types
// (0.72x for complex double prod at 8): those keep the register form.  (Round 5 had U = 2 over U = 4, 1.02-1.04x,
// r05_team_p34_ab.jsonl; LDS-DMA staging at 4 members 0.967-0.998x,
// r06_team_p4_ab.jsonl.)  The combine keeps U = 2: U = 1 there ran 0.966x.
#ifndef OSGPU_TEAM_LDS_U
#define OSGPU_TEAM_LDS_U 1
#endif

// Launch shape per (T, OP, P): U vectors per input per lane in rounds of G.
// REMOTE: some member's arrays live in another GPU's HBM (xGMI): the shapes
// last measured across GPUs (round 4) -- the register form at 2 members and
// rounds of kTeamG8 above 4.
template <typename T, int OP, int P, bool REMOTE = false>
struct TeamShape {
    static constexpr bool kComplex = std::is_same<T, cfloat>::value || std::is_same<T, cdouble>::value;
    static constexpr bool kHeavy = kComplex && OP == OP_PROD;
    static constexpr int U = P <= 2 ? kTeamU2 : (P <= 4 ? kTeamU4 : kTeamU8);
    static constexpr int G = P <= 4 ? U
                             : (kHeavy ? kTeamGH : ((kComplex || REMOTE) ? kTeamG8 : OSGPU_TEAM_G8R));
    static constexpr bool kPipe = P > 4 && U / G > 1 && std::is_integral<T>::value;
    static constexpr bool kPerOutput = P > 4;
    // the LDS form also at 5, 6 and 8 members for real types other than FP
    // max/min: in one process on the same allocations, 9 (type, op) cases x
    // 5 allocations, at 8 members every case ran faster (double sum 1.012x,
    // float sum 1.043x, int sum 1.085x, long xor 1.068x, short min 1.060x,
    // float prod 1.042x, double prod 1.110x, int max 1.090x, long sum
    // 1.042x; profiles/r06_team_lds8_ab.jsonl), at 5 and 6 members 1.058x
    // overall (cases 0.989-1.110x; r06_team_lds56_ab.jsonl); complex types
    // and FP max/min lost (0.72-0.98x, r06_team_lds_p58_ab.jsonl), and so
    // did every case at 7 members (7-wave workgroups, 0.78-0.99x).
    static constexpr bool kFpMinMax = std::is_floating_point<T>::value && (OP == OP_MAX || OP == OP_MIN);
    static constexpr bool kLds = REMOTE ? (P >= 3 && P <= 4)
                                        : ((P >= OSGPU_TEAM_LDS_MIN_P && P <= OSGPU_TEAM_LDS_MAX_P) ||
                                           ((P == 5 || P == 6 || P == 8) && !kComplex && !kFpMinMax));
    static constexpr int kLdsU = OSGPU_TEAM_LDS_U;
    // the rounds g = 0, G, 2G, ... must tile [0, U) exactly, or the last
    // round reads and writes past the tile (and past nvec)
    static_assert(G >= 1 && G <= U && U % G == 0, "the round size must divide U");
};

// the remote shape differs from the local one (else the local kernel serves)
template <typename T, int OP, int P>
constexpr bool kRemoteDiffers = TeamShape<T, OP, P, true>::kLds != TeamShape<T, OP, P, false>::kLds ||
                                TeamShape<T, OP, P, true>::G != TeamShape<T, OP, P, false>::G;

// f(integral_constant<int, I>) for I = 0 .. N-1, unrolled by construction
// (a #pragma unroll on the round loop is dropped for the largest bodies)
template <int I, int N>
struct Rounds {
    template <typename F>
    __device__ __forceinline__ static void run(F &&f)
    {
        if constexpr (I < N) {
            f(std::integral_constant<int, I>{});
            Rounds<I + 1, N>::run(f);
        }
    }
};

// (An XCD-aware workgroup -> tile map -- XCD x streaming one contiguous run of
// tiles instead of tiles x, x + 8, ... -- ran slower at every member count
// over ten layouts, 0.853-0.954 against 0.886-0.978 of the same-mix copy,
// profiles/r05_team_layouts.jsonl: the identity map ships.)

// E: Elem<T, OP> (exact) or Fast<T, OP> (branch-free, elem_ops.hpp)
template <typename T, int OP, int P, bool ORDERED, typename E = Elem<T, OP>>
__device__ __forceinline__ void team_fold(const T (&x)[P], T (&r)[P])
{
    if (ORDERED) {
#pragma unroll
        for (int q = 0; q < P; q++) {
            T acc = x[q];
#pragma unroll
            for (int j = 0; j < P; j++)
                if (j != q) acc = E::f(acc, x[j]);
            r[q] = acc;
        }
    } else {
        T acc = x[0];
#pragma unroll
        for (int j = 1; j < P; j++) acc = E::f(acc, x[j]);
#pragma unroll
        for (int q = 0; q < P; q++) r[q] = acc;
    }
}

template <typename T, int OP, int P, bool ORDERED, bool REMOTE>
__global__ __launch_bounds__(kTeamBlock) void team_vec_kernel(TeamPtrs<T, P> a, size_t nvec,
                                                              size_t head, size_t tail_start,
                                                              int nedge, unsigned tm, unsigned tk)
{
    constexpr int W = 16 / sizeof(T);
    using S = TeamShape<T, OP, P, REMOTE>;
    constexpr int U = S::U;
    if (blockIdx.x == 0 && (int) threadIdx.x < nedge) {
        const size_t e = threadIdx.x < head ? threadIdx.x : tail_start + (threadIdx.x - head);
        T x[P], r[P];
#pragma unroll
        for (int p = 0; p < P; p++) x[p] = a.src[p][e];
        team_fold<T, OP, P, ORDERED>(x, r);
#pragma unroll
        for (int p = 0; p < P; p++) a.dst[p][e] = r[p];
    }
    // tile blockIdx.x * tm + tk (launch_team_tiles; tm = 1, tk = 0: tile blockIdx.x)
    const size_t t0 = ((size_t) blockIdx.x * tm + tk) * (kTeamBlock * U) + threadIdx.x;
    // fold one vector of every input into one vector of every output: the
    // branch-free fold first, the exact one only for a vector whose results
    // hold a NaN part (rare; elem_ops.hpp Fast) -- no branch per element, so
    // the tile's loads stay in flight ahead of the folds
    using F = Fast<T, OP>;
    auto fold_store = [&](TVec<T> (&in)[P], size_t j) __attribute__((always_inline)) {
        if constexpr (ORDERED && S::kPerOutput) {
            // one output at a time: fold, check, store -- only one output
            // vector live beside the inputs
            Rounds<0, P>::run([&](auto qc) {
                constexpr int q = decltype(qc)::value;
                TVec<T> out;
                bool bad = false;
#pragma unroll
                for (int w = 0; w < W; w++) {
                    T acc = in[q].e[w];
#pragma unroll
                    for (int k = 0; k < P; k++)
                        if (k != q) acc = F::f(acc, in[k].e[w]);
                    out.e[w] = acc;
                    bad = bad || F::bad(acc);
                }
                if (F::kChecked && __builtin_expect(bad, 0)) {
#pragma unroll
                    for (int w = 0; w < W; w++) {
                        T acc = in[q].e[w];
#pragma unroll
                        for (int k = 0; k < P; k++)
                            if (k != q) acc = Elem<T, OP>::f(acc, in[k].e[w]);
                        out.e[w] = acc;
                    }
                }
                __builtin_nontemporal_store(out.v, reinterpret_cast<u32x4 *>(a.dst[q] + head) + j);
            });
            return;
        }
        TVec<T> out[P];
        bool bad = false;
#pragma unroll
        for (int w = 0; w < W; w++) {
            T x[P], r[P];
#pragma unroll
            for (int p = 0; p < P; p++) x[p] = in[p].e[w];
            team_fold<T, OP, P, ORDERED, F>(x, r);
#pragma unroll
            for (int p = 0; p < P; p++) {
                out[p].e[w] = r[p];
                bad = bad || F::bad(r[p]);
            }
        }
        if (F::kChecked && __builtin_expect(bad, 0)) {
#pragma unroll
            for (int w = 0; w < W; w++) {
                T x[P], r[P];
#pragma unroll
                for (int p = 0; p < P; p++) x[p] = in[p].e[w];
                team_fold<T, OP, P, ORDERED>(x, r);
#pragma unroll
                for (int p = 0; p < P; p++) out[p].e[w] = r[p];
            }
        }
#pragma unroll
        for (int p = 0; p < P; p++)
            __builtin_nontemporal_store(out[p].v, reinterpret_cast<u32x4 *>(a.dst[p] + head) + j);
    };
    if (t0 + (size_t) (U - 1) * kTeamBlock < nvec) {
        // whole tile: the loads of G vectors of every input are in flight
        // before the first fold, as in combine_vec_kernel -- P*G*16 B per
        // lane, not P*16 B per round trip.  G = U up to 4 inputs; above,
        // TeamShape's G (all 4*P at once spills the 8-input complex sum)
        constexpr int G = S::G;
        constexpr int R = U / G;
        auto load_round = [&](TVec<T> (&in)[G][P], int g) __attribute__((always_inline)) {
#pragma unroll
            for (int u = 0; u < G; u++)
#pragma unroll
                for (int p = 0; p < P; p++)
                    in[u][p].v = __builtin_nontemporal_load(
                        reinterpret_cast<const u32x4 *>(a.src[p] + head) + t0 +
                        (size_t) (g * G + u) * kTeamBlock);
        };
        if constexpr (S::kPipe) {
            // round r+1's loads go out before round r's stores
            TVec<T> b0[G][P], b1[G][P];
            load_round(b0, 0);
            Rounds<0, R>::run([&](auto rc) {
                constexpr int r = decltype(rc)::value;
                auto &cur = (r % 2 == 0) ? b0 : b1;
                auto &nxt = (r % 2 == 0) ? b1 : b0;
                if constexpr (r + 1 < R) load_round(nxt, r + 1);
#pragma unroll
                for (int u = 0; u < G; u++) fold_store(cur[u], t0 + (size_t) (r * G + u) * kTeamBlock);
            });
        } else {
            Rounds<0, R>::run([&](auto rc) {
                constexpr int r = decltype(rc)::value;
                TVec<T> in[G][P];
                load_round(in, r);
#pragma unroll
                for (int u = 0; u < G; u++) fold_store(in[u], t0 + (size_t) (r * G + u) * kTeamBlock);
            });
        }
        return;
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t j = t0 + (size_t) u * kTeamBlock;
        if (j < nvec) {
            TVec<T> in[P];
#pragma unroll
            for (int p = 0; p < P; p++)
                in[p].v = __builtin_nontemporal_load(
                    reinterpret_cast<const u32x4 *>(a.src[p] + head) + j);
            fold_store(in, j);
        }
    }
}

// x[k] of a compile-time-sized array at a wave-uniform runtime index
template <typename X, int P>
__device__ __forceinline__ X pick(const X (&x)[P], int k)
{
    X r = x[0];
#pragma unroll
    for (int p = 1; p < P; p++)
        if (k == p) r = x[p];
    return r;
}

// LDS-staged form: P waves per workgroup, a tile of 64*U 16-B vectors of
// every member.  Wave p streams member p's source tile into LDS (one read
// stream per wave, as the copy kernel); after the barrier wave q folds the
// tile of all P inputs from LDS in member q's order and streams member q's
// target tile (one write stream per wave).  HBM bytes as the register form
// (2*P*s per element); the LDS carries P reads of every staged byte.  (A
// persistent grid walking the tiles with two LDS buffers, the next tile's
// loads in flight during this one's folds, ran 2-17 % slower at 3-8
// members: profiles/r04_team_sweep_4.jsonl; two or four members per wave,
// fewer waves per workgroup, no faster: r04_team_place_3.jsonl.)
template <typename T, int OP, int P, bool ORDERED, int U>
__global__ __launch_bounds__(64 * P) void team_lds_kernel(TeamPtrs<T, P> a, size_t nvec,
                                                          size_t head, size_t tail_start,
                                                          int nedge, unsigned tm, unsigned tk)
{
    constexpr int W = 16 / sizeof(T);
    constexpr int V = 64 * U;  // vectors per member per tile
    __shared__ u32x4 tile[P][V];
    if (blockIdx.x == 0 && (int) threadIdx.x < nedge) {
        const size_t e = threadIdx.x < head ? threadIdx.x : tail_start + (threadIdx.x - head);
        T x[P], r[P];
#pragma unroll
        for (int p = 0; p < P; p++) x[p] = a.src[p][e];
        team_fold<T, OP, P, ORDERED>(x, r);
#pragma unroll
        for (int p = 0; p < P; p++) a.dst[p][e] = r[p];
    }
    // the member this wave stages and writes
    const int w = __builtin_amdgcn_readfirstlane((int) (threadIdx.x >> 6));
    const int lane = (int) (threadIdx.x & 63);
    const u32x4 *src = reinterpret_cast<const u32x4 *>(pick(a.src, w) + head);
    u32x4 *dst = reinterpret_cast<u32x4 *>(pick(a.dst, w) + head);
    u32x4 v[U];
    auto load = [&](size_t t) {
        const size_t base = t * V;
        const bool whole = base + V <= nvec;
#pragma unroll
        for (int u = 0; u < U; u++)
            if (whole || base + u * 64 + lane < nvec)
                v[u] = __builtin_nontemporal_load(src + base + u * 64 + lane);
    };
    using F = Fast<T, OP>;
    // member q's fold of element e: x[q] first, then the others ascending
    // (order-independent integer ops: ascending for every q)
    // the vectors [u0, u1) of the tile
    auto fold_store = [&](size_t t, int u0, int u1) {
        const size_t base = t * V;
        const bool whole = base + V <= nvec;
        Rounds<0, P>::run([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            if (w != q) return;
#pragma unroll
            for (int u = u0; u < u1; u++) {
                if (!whole && base + u * 64 + lane >= nvec) continue;
                TVec<T> in[P], out;
#pragma unroll
                for (int p = 0; p < P; p++) in[p].v = tile[p][u * 64 + lane];
                bool bad = false;
#pragma unroll
                for (int e = 0; e < W; e++) {
                    T acc = in[ORDERED ? q : 0].e[e];
#pragma unroll
                    for (int k = 0; k < P; k++)
                        if (k != (ORDERED ? q : 0)) acc = F::f(acc, in[k].e[e]);
                    out.e[e] = acc;
                    bad = bad || F::bad(acc);
                }
                if (F::kChecked && __builtin_expect(bad, 0)) {
#pragma unroll
                    for (int e = 0; e < W; e++) {
                        T acc = in[q].e[e];
#pragma unroll
                        for (int k = 0; k < P; k++)
                            if (k != q) acc = Elem<T, OP>::f(acc, in[k].e[e]);
                        out.e[e] = acc;
                    }
                }
                __builtin_nontemporal_store(out.v, dst + base + u * 64 + lane);
            }
        });
    };
    const size_t t = (size_t) blockIdx.x * tm + tk;
    load(t);
#pragma unroll
    for (int u = 0; u < U; u++) tile[w][u * 64 + lane] = v[u];
    __syncthreads();
    fold_store(t, 0, U);
}

template <typename T, int OP, int P, bool ORDERED>
__global__ __launch_bounds__(kTeamBlock) void team_scalar_kernel(TeamPtrs<T, P> a, size_t n,
                                                                 unsigned tm, unsigned tk)
{
    // tiles of kTeamBlock elements: blockIdx.x * tm + tk, then gridDim.x * tm further
    const size_t stride = (size_t) gridDim.x * tm * kTeamBlock;
    for (size_t i = ((size_t) blockIdx.x * tm + tk) * kTeamBlock + threadIdx.x; i < n;
         i += stride) {
        T x[P], r[P];
#pragma unroll
        for (int p = 0; p < P; p++) x[p] = a.src[p][i];
        team_fold<T, OP, P, ORDERED>(x, r);
#pragma unroll
        for (int p = 0; p < P; p++) a.dst[p][i] = r[p];
    }
}

// tiles of m members, this one k-th (launch_team_tiles)
struct Tiles {
    unsigned m, k;
    bool remote;  // some member's arrays are in another GPU's HBM
    // of `total` tiles, the ones this member folds (at least one block)
    size_t blocks(size_t total) const
    {
        const size_t b = total > k ? (total - k + m - 1) / m : 0;
        return b ? b : 1;
    }
};

template <typename T, int OP, int P, bool REMOTE>
static hipError_t team_launch_p(void *const *dsts, const void *const *srcs, size_t n,
                                Tiles tl, hipStream_t s)
{
    using S = TeamShape<T, OP, P, REMOTE>;
    // integer ops are order-independent (wrapping ring / lattice ops); every
    // floating-point op, min/max included (NaN, signed zero), is not
    constexpr bool ORDERED = !std::is_integral<T>::value;
    TeamPtrs<T, P> a;
    const uintptr_t phase = (uintptr_t) srcs[0] & 15;
    bool same = (phase % sizeof(T)) == 0;
    for (int p = 0; p < P; p++) {
        a.src[p] = static_cast<const T *>(srcs[p]);
        a.dst[p] = static_cast<T *>(dsts[p]);
        same = same && (((uintptr_t) srcs[p] & 15) == phase) && (((uintptr_t) dsts[p] & 15) == phase);
    }
    if (!same) {
        size_t blocks = tl.blocks((n + kTeamBlock - 1) / kTeamBlock);
        blocks = blocks > 8192 ? 8192 : blocks;
        hipLaunchKernelGGL((team_scalar_kernel<T, OP, P, ORDERED>), dim3((unsigned) blocks),
                           dim3(kTeamBlock), 0, s, a, n, tl.m, tl.k);
        return hipGetLastError();
    }
    constexpr int W = 16 / sizeof(T);
    size_t head = phase ? (16 - phase) / sizeof(T) : 0;
    if (head > n) head = n;
    const size_t nvec = (n - head) / W;
    const size_t tail_start = head + nvec * W;
    // the unaligned head and the tail: member 0's first workgroup
    const int nedge = tl.k == 0 ? (int) (head + (n - tail_start)) : 0;
    // tiles of V vectors, this member's every tl.m-th one, one per workgroup
    // of `threads`; at most max_launch_threads() per launch (combine.hpp):
    // runs of tiles that are whole multiples of tl.m, so tile t of a run is
    // still this member's when t % tl.m == tl.k; the first launch takes the
    // edges, the others shifted pointers
    auto launch = [&](size_t V, unsigned threads, auto kernel) -> hipError_t {
        size_t tiles = (nvec + V - 1) / V;
        if (tiles == 0) tiles = 1;
        const size_t lim = max_launch_threads() / threads;
        const size_t run = (lim ? lim : 1) * tl.m;
        for (size_t t0 = 0; t0 < tiles; t0 += run) {
            const size_t nt = tiles - t0 < run ? tiles - t0 : run;
            const size_t nv = nvec - t0 * V < nt * V ? nvec - t0 * V : nt * V;
            const size_t blocks = tl.blocks(nt);
            if (t0 == 0) {
                hipLaunchKernelGGL(kernel, dim3((unsigned) blocks), dim3(threads), 0, s, a, nv, head,
                                   tail_start, nedge, tl.m, tl.k);
            } else {
                const size_t off = head + t0 * V * W;
                TeamPtrs<T, P> c;
                for (int p = 0; p < P; p++) {
                    c.src[p] = a.src[p] + off;
                    c.dst[p] = a.dst[p] + off;
                }
                hipLaunchKernelGGL(kernel, dim3((unsigned) blocks), dim3(threads), 0, s, c, nv,
                                   (size_t) 0, (size_t) 0, 0, tl.m, tl.k);
            }
            const hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    };
    if constexpr (S::kLds) {
        constexpr int UL = S::kLdsU;
        return launch((size_t) 64 * UL, 64 * P, team_lds_kernel<T, OP, P, ORDERED, UL>);
    } else {  // (not instantiated where the LDS form is used)
        return launch((size_t) kTeamBlock * S::U, kTeamBlock,
                      team_vec_kernel<T, OP, P, ORDERED, REMOTE>);
    }
}

// the remote shape only where it differs from the local one
template <typename T, int OP, int P>
static hipError_t team_launch_pr(void *const *d, const void *const *sr, size_t n, Tiles tl,
                                 hipStream_t s)
{
    if constexpr (kRemoteDiffers<T, OP, P>)
        if (tl.remote) return team_launch_p<T, OP, P, true>(d, sr, n, tl, s);
    return team_launch_p<T, OP, P, false>(d, sr, n, tl, s);
}

template <typename T, int OP>
static hipError_t team_launch_op(int P, void *const *d, const void *const *sr, size_t n,
                                 Tiles tl, hipStream_t s)
{
    switch (P) {
    case 2: return team_launch_pr<T, OP, 2>(d, sr, n, tl, s);
    case 3: return team_launch_pr<T, OP, 3>(d, sr, n, tl, s);
    case 4: return team_launch_pr<T, OP, 4>(d, sr, n, tl, s);
    case 5: return team_launch_pr<T, OP, 5>(d, sr, n, tl, s);
    case 6: return team_launch_pr<T, OP, 6>(d, sr, n, tl, s);
    case 7: return team_launch_pr<T, OP, 7>(d, sr, n, tl, s);
    case 8: return team_launch_pr<T, OP, 8>(d, sr, n, tl, s);
    }
    return hipErrorInvalidValue;
}

#define TEAM_CASE(OPC)                                                         \
    case OPC: return team_launch_op<T, OPC>(P, d, sr, n, tl, s);

template <typename T>
static hipError_t team_int(int op, int P, void *const *d, const void *const *sr, size_t n,
                           Tiles tl, hipStream_t s)
{
    switch (op) {
        TEAM_CASE(OP_SUM) TEAM_CASE(OP_PROD) TEAM_CASE(OP_AND) TEAM_CASE(OP_OR)
        TEAM_CASE(OP_XOR) TEAM_CASE(OP_MAX) TEAM_CASE(OP_MIN)
    }
    return hipErrorInvalidValue;
}

template <typename T>
static hipError_t team_real(int op, int P, void *const *d, const void *const *sr, size_t n,
                            Tiles tl, hipStream_t s)
{
    switch (op) {
        TEAM_CASE(OP_SUM) TEAM_CASE(OP_PROD) TEAM_CASE(OP_MAX) TEAM_CASE(OP_MIN)
    }
    return hipErrorInvalidValue;
}

template <typename T>
static hipError_t team_cplx(int op, int P, void *const *d, const void *const *sr, size_t n,
                            Tiles tl, hipStream_t s)
{
    switch (op) {
        TEAM_CASE(OP_SUM) TEAM_CASE(OP_PROD)
    }
    return hipErrorInvalidValue;
}

hipError_t launch_team_tiles(int type, int op, int P, void *const *dsts, const void *const *srcs,
                             size_t n, int m, int k, hipStream_t s, bool remote)
{
    if (P < 2 || P > kMaxTeam || m < 1 || k < 0 || k >= m) return hipErrorInvalidValue;
    if (n == 0) return hipSuccess;
    const Tiles tl{(unsigned) m, (unsigned) k, remote};
    switch (type) {
    case T_SHORT: return team_int<int16_t>(op, P, dsts, srcs, n, tl, s);
    case T_INT: return team_int<int32_t>(op, P, dsts, srcs, n, tl, s);
    case T_LONG:
    case T_LONGLONG: return team_int<int64_t>(op, P, dsts, srcs, n, tl, s);
    case T_FLOAT: return team_real<float>(op, P, dsts, srcs, n, tl, s);
    case T_DOUBLE: return team_real<double>(op, P, dsts, srcs, n, tl, s);
    case T_COMPLEXF: return team_cplx<cfloat>(op, P, dsts, srcs, n, tl, s);
    case T_COMPLEXD: return team_cplx<cdouble>(op, P, dsts, srcs, n, tl, s);
    case T_LONGDOUBLE:
        return m == 1 ? launch_team_longdouble(op, P, dsts, srcs, n, s) : hipErrorNotSupported;
    }
    return hipErrorInvalidValue;
}

hipError_t launch_team(int type, int op, int P, void *const *dsts, const void *const *srcs,
                       size_t n, hipStream_t s, bool remote)
{
    return launch_team_tiles(type, op, P, dsts, srcs, n, 1, 0, s, remote);
}

}  // namespace osgpu
