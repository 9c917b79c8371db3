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

// above 4 members: U vectors per input per lane, G of them in flight per
// round.  With the branch-free folds (elem_ops.hpp Fast), U = 4 in two
// rounds of G = 2 (16 vectors of 16 B in flight per lane at 8 members)
// beats one round of U = G = 2 at P = 8 for every type: float 0.715 ->
// 0.786, complexf 0.723 -> 0.790 of 8 TB/s, int / long +2 %, the rest equal
// (every build loaded in one process, interleaved on the same arrays,
// profiles/r03_team_variants_interleaved.jsonl); U = G = 4 spills the
// 8-input complexf fold (0.45).  The pull combine keeps OSGPU_U_K8
#ifndef OSGPU_TEAM_U8
#define OSGPU_TEAM_U8 4
#endif
#ifndef OSGPU_TEAM_G8
#define OSGPU_TEAM_G8 2
#endif
// ... for the real (non-complex) types: one round of all U = 4 vectors
// (their loads all in flight before the first fold; 3-6 waves per SIMD, no
// scratch).  Against G = 2 in one process on the same allocations
// (tools/team_inproc_ab.py, profiles/r05_team_p8_tile_ab.jsonl): 1.006x
// over 7 (type, op) pairs at 5-8 members, floating-point folds 1.00-1.03x,
// integer ones 0.996-1.004x.  The complex sum keeps G = 2 (G = 4 spills it)
#ifndef OSGPU_TEAM_G8R
#define OSGPU_TEAM_G8R 4
#endif
// the register-heavy folds above 4 members (complex products: 4-6 VALU
// temporaries per element per output) take rounds of OSGPU_TEAM_GH vectors
#ifndef OSGPU_TEAM_GH
#define OSGPU_TEAM_GH 2
#endif
// 1: above 4 members, integer folds issue round r+1's loads before round
// r's folds and stores (two round buffers), so a lane's loads stay in
// flight while it stores; 0: round after round.  Integers only: for every
// floating-point fold the two buffers cost 0.2-0.4 of the rate (the
// compiler no longer keeps a round's loads in flight), against +0.5-1 % for
// the integer ones (profiles/r04_team_type_op_sweep.jsonl)
#ifndef OSGPU_TEAM_PIPE
#define OSGPU_TEAM_PIPE 1
#endif
// floating-point folds on the two-buffer pipeline too: round 4 lost 0.2-0.4
// of the rate to it because fold_store was not inlined and the round buffers
// went to scratch; with the lambdas forced inline it compiles clean, and at
// U = 6 / 8 (3 / 4 rounds of 2) ran 0.97-0.98x of the shipped tile (same
// A/B file), so it stays off
#ifndef OSGPU_TEAM_PIPE_FP
#define OSGPU_TEAM_PIPE_FP 0
#endif
#ifndef OSGPU_TEAM_PIPE_FENCE
#define OSGPU_TEAM_PIPE_FENCE 0
#endif
#ifndef OSGPU_TEAM_OCC_LDS
#define OSGPU_TEAM_OCC_LDS 0
#endif
#ifndef OSGPU_TEAM_PEROUT
#define OSGPU_TEAM_PEROUT 1
#endif
// from this many members on: the LDS-staged kernel (team_lds_kernel), one
// wave per member.  2 members too: against the register form on the same
// fresh allocations it ran 1.03x faster for double sum (20 allocations on
// two leases, median 0.794 against 0.769 of 8 TB/s) and 1.00-1.07x for every
// (type, op) probed -- float sum/prod, double max, int sum, long xor, short
// min, complex sum/prod (profiles/r05_team_p2_ab.jsonl).
// OSGPU_TEAM_LDS_U 16-B vectors per lane per tile.  U = 2
// (2 KiB per member per workgroup): timed against U = 4 in one process on
// the same fresh allocations (tools/team_inproc_ab.py, 10 allocations per
// member count on each of two leases, profiles/r05_team_p34_ab.jsonl) it ran
// 1.02-1.04x faster on average at 3 and 4 members and lifted the slowest
// placement most (4 members: 0.749 against 0.683 of 8 TB/s), losing up to
// 4 % only where the copy itself was fastest.  (Round 4 had chosen U = 4
// from a sweep on one box: r04_team_sweep_3.jsonl.)  U = 8, 64 KiB of LDS
// per workgroup at 8 members: 0.44-0.62, r04_team_sweep_2.jsonl
#ifndef OSGPU_TEAM_LDS_MIN_P
#define OSGPU_TEAM_LDS_MIN_P 2
#endif
// ... up to this many members; above, the register form.  On boxes whose
// P-range copy itself is fast (0.81-0.84 of 8 TB/s) the register form led
// at 5-8 members by 5-7 % (0.956 against 0.884 of the copy at 8, five
// allocations, order rotated, r04_team_place_4.jsonl), on slow ones (0.75-
// 0.77) the LDS form by 3-5 % (r04_team_place_3.jsonl): in absolute terms
// the register form's best (0.81 of 8 TB/s at 8 members) is above the LDS
// form's (0.75), so it keeps 5-8; at 3-4 members the LDS form is ahead or
// equal on both kinds of box
#ifndef OSGPU_TEAM_LDS_MAX_P
#define OSGPU_TEAM_LDS_MAX_P 4
#endif
#ifndef OSGPU_TEAM_LDS_U
#define OSGPU_TEAM_LDS_U 2
#endif
#ifndef OSGPU_TEAM_LDS_U8
#define OSGPU_TEAM_LDS_U8 4
#endif
#ifndef OSGPU_TEAM_LDS_ROT
#define OSGPU_TEAM_LDS_ROT 0
#endif


// vectors per input per lane for 2 and for 3-4 members (all loaded before
// the first fold).  U = 2 at 2 members: 0.71-0.75 against 0.77 with U = 4
// (same interleaved A/B)
#ifndef OSGPU_TEAM_U2
#define OSGPU_TEAM_U2 OSGPU_U_K2
#endif
#ifndef OSGPU_TEAM_U4
#define OSGPU_TEAM_U4 OSGPU_U_K4
#endif

// Launch shape per (T, OP, P): U vectors per input per lane in rounds of G
template <typename T, int OP, int P>
struct TeamShape {
    static constexpr bool kHeavy = (std::is_same<T, cfloat>::value || std::is_same<T, cdouble>::value) &&
                                   OP == OP_PROD;
    static constexpr int U = P <= 2 ? OSGPU_TEAM_U2 : (P <= 4 ? OSGPU_TEAM_U4 : OSGPU_TEAM_U8);
    static constexpr bool kComplex = std::is_same<T, cfloat>::value || std::is_same<T, cdouble>::value;
    static constexpr int G = P <= 4 ? U : (kHeavy ? OSGPU_TEAM_GH : (kComplex ? OSGPU_TEAM_G8 : OSGPU_TEAM_G8R));
    static constexpr bool kPipe = P > 4 && OSGPU_TEAM_PIPE && U / G > 1 &&
                                  (std::is_integral<T>::value || OSGPU_TEAM_PIPE_FP);
    // ordered folds above 4 members: fold, check and store one output at a
    // time instead of all P outputs, then all P stores
    static constexpr bool kPerOutput = P > 4 && OSGPU_TEAM_PEROUT;
    static constexpr bool kLds = P >= OSGPU_TEAM_LDS_MIN_P && P <= OSGPU_TEAM_LDS_MAX_P &&
                                 !(std::is_same<T, cdouble>::value && OP == OP_PROD && P >= 8);
    static constexpr int kLdsU = P >= 8 ? OSGPU_TEAM_LDS_U8 : OSGPU_TEAM_LDS_U;
    // the rounds g = 0, G, 2G, ... must tile [0, U) exactly, or the last
    // round reads and writes past the tile (and past nvec)
    static_assert(G >= 1 && G <= U && U % G == 0, "the round size must divide U");
};

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

// XCD-aware workgroup -> tile map (OSGPU_TEAM_XCD, off): the dispatcher
// deals workgroups round-robin over the 8 XCDs (b % 8), so with the identity
// map XCD x streams tiles x, x + 8, x + 16, ...; remapped, XCD x streams one
// contiguous run of tiles.  A bijection on [0, n) for any n.  Measured
// slower at every member count over ten array layouts (of the same-mix
// copy: 2 members 0.954 vs 0.978 median, 4 members 0.934 vs 0.962, 8
// members 0.853 vs 0.886; tools/team_layout_sweep.py,
// profiles/r05_team_layouts.jsonl), so the identity map ships.
#ifndef OSGPU_TEAM_XCD
#define OSGPU_TEAM_XCD 0
#endif
constexpr unsigned kXcds = 8;
__device__ __forceinline__ unsigned xcd_tile(unsigned b, unsigned n)
{
    if (!OSGPU_TEAM_XCD || n < kXcds) return b;
    const unsigned x = b % kXcds, i = b / kXcds, per = n / kXcds, rem = n % kXcds;
    return x < rem ? x * (per + 1) + i : rem * (per + 1) + (x - rem) * per + i;
}

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

template <typename T, int OP, int P, bool ORDERED>
__global__ __launch_bounds__(kTeamBlock) void team_vec_kernel(TeamPtrs<T, P> a, size_t nvec,
                                                              size_t head, size_t tail_start,
                                                              int nedge, unsigned tm, unsigned tk)
{
    constexpr int W = 16 / sizeof(T);
    using S = TeamShape<T, OP, P>;
    constexpr int U = S::U;
#if OSGPU_TEAM_OCC_LDS
    // occupancy cap (experiment): a workgroup holds this much LDS, so at
    // most 160 KiB / OSGPU_TEAM_OCC_LDS workgroups share a CU.  3 or 4
    // workgroups per CU at 6 / 8 members: 0.99-1.00x (same A/B file)
    if constexpr (P > 4) {
        __shared__ unsigned occ_pad[OSGPU_TEAM_OCC_LDS / 4];
        if (nvec == 0) reinterpret_cast<volatile unsigned *>(occ_pad)[threadIdx.x] = 0;
        __syncthreads();
    }
#endif
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
    const size_t t0 = ((size_t) xcd_tile(blockIdx.x, gridDim.x) * tm + tk) * (kTeamBlock * U) +
                      threadIdx.x;
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
                if constexpr (r + 1 < R) {
                    load_round(nxt, r + 1);
                    // keep the scheduler from sinking these loads below the
                    // stores (it does, to save registers, when it may)
                    if constexpr (OSGPU_TEAM_PIPE_FENCE) asm volatile("" ::: "memory");
                }
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
    const int wave = __builtin_amdgcn_readfirstlane((int) (threadIdx.x >> 6));
    // the member this wave stages and writes: wave w, or with
    // OSGPU_TEAM_LDS_ROT member (w + blockIdx.x) % P (the waves of
    // neighbouring workgroups start on different arrays)
#if OSGPU_TEAM_LDS_ROT
    const int w = __builtin_amdgcn_readfirstlane((int) ((wave + blockIdx.x) % P));
#else
    const int w = wave;
#endif
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
    const size_t t = (size_t) xcd_tile(blockIdx.x, gridDim.x) * tm + tk;
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
    // of `total` tiles, the ones this member folds (at least one block)
    size_t blocks(size_t total) const
    {
        const size_t b = total > k ? (total - k + m - 1) / m : 0;
        return b ? b : 1;
    }
};

template <typename T, int OP, int P>
static hipError_t team_launch_p(void *const *dsts, const void *const *srcs, size_t n,
                                Tiles tl, hipStream_t s)
{
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
    if constexpr (TeamShape<T, OP, P>::kLds) {
        constexpr int UL = TeamShape<T, OP, P>::kLdsU;
        const size_t blocks = tl.blocks((nvec + (size_t) 64 * UL - 1) / ((size_t) 64 * UL));
        hipLaunchKernelGGL((team_lds_kernel<T, OP, P, ORDERED, UL>), dim3((unsigned) blocks),
                           dim3(64 * P), 0, s, a, nvec, head, tail_start, nedge, tl.m, tl.k);
    } else {  // (not instantiated where the LDS form is used)
        constexpr int U = TeamShape<T, OP, P>::U;
        const size_t blocks =
            tl.blocks((nvec + (size_t) kTeamBlock * U - 1) / ((size_t) kTeamBlock * U));
        hipLaunchKernelGGL((team_vec_kernel<T, OP, P, ORDERED>), dim3((unsigned) blocks),
                           dim3(kTeamBlock), 0, s, a, nvec, head, tail_start, nedge, tl.m, tl.k);
    }
    return hipGetLastError();
}

template <typename T, int OP>
static hipError_t team_launch_op(int P, void *const *d, const void *const *sr, size_t n,
                                 Tiles tl, hipStream_t s)
{
    switch (P) {
    case 2: return team_launch_p<T, OP, 2>(d, sr, n, tl, s);
    case 3: return team_launch_p<T, OP, 3>(d, sr, n, tl, s);
    case 4: return team_launch_p<T, OP, 4>(d, sr, n, tl, s);
    case 5: return team_launch_p<T, OP, 5>(d, sr, n, tl, s);
    case 6: return team_launch_p<T, OP, 6>(d, sr, n, tl, s);
    case 7: return team_launch_p<T, OP, 7>(d, sr, n, tl, s);
    case 8: return team_launch_p<T, OP, 8>(d, sr, n, tl, s);
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
                             size_t n, int m, int k, hipStream_t s)
{
    if (P < 2 || P > kMaxTeam || m < 1 || k < 0 || k >= m) return hipErrorInvalidValue;
    if (n == 0) return hipSuccess;
    const Tiles tl{(unsigned) m, (unsigned) k};
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
                       size_t n, hipStream_t s)
{
    return launch_team_tiles(type, op, P, dsts, srcs, n, 1, 0, s);
}

}  // namespace osgpu
