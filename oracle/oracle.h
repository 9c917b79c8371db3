/*
 * oracle.h -- CPU restatement of the OpenSHMEM reduce-to-all path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is linked into, loaded by
 * or called from the product library (libosgpu_reduce.so).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it, and
 * only as the checker / the timed CPU baseline.
 *
 * What it restates (reference paths relative to the reference checkout):
 *   - element operations   src/shmemu/miscops.c:12-105
 *       (+ libgcc __mulsc3/__muldc3 reached from miscops.c:38-39, GCC 11.4)
 *   - reduce-to-all schedule src/reductions.c:32-120 (udr_<T>_to_all)
 *   - 44 public entry points src/reductions.c:248-297
 *
 * Pinning:
 *   - element ops: PINNED against the reference's own miscops.c, compiled
 *     unmodified from /root/reference by oracle/Makefile into oracle/_ref/
 *     (tests/golden/ops_*.npz are produced by it; tests/test_oracle.py checks
 *     this restatement bit for bit against them).
 *   - schedule (fold order me-first then PE_start + i*2^logPE_stride skipping
 *     me, 64-element pWrk chunks, overlap temp): src/reductions.c cannot be
 *     built here (it needs UCX's <ucp/api/ucp.h> through src/shmemu/shmemu.h:6
 *     -> src/shmemc/state.h:6 -> src/shmemc/thispe.h:9, absent from this
 *     image) and the reference holds no test or fixture for it, so the fold
 *     ORDER is restated from the source text only: "parity unpinned" for the
 *     schedule itself.  Every per-element result is still produced with the
 *     reference's compiled arithmetic in the golden generator.
 */
#ifndef OSGPU_ORACLE_H
#define OSGPU_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* type and op codes: same numbering as include/osgpu_reduce.h */
enum { OR_SHORT = 0, OR_INT, OR_LONG, OR_LONGLONG, OR_FLOAT, OR_DOUBLE,
       OR_LONGDOUBLE, OR_COMPLEXF, OR_COMPLEXD, OR_NTYPES };
enum { OR_SUM = 0, OR_PROD, OR_AND, OR_OR, OR_XOR, OR_MAX, OR_MIN, OR_NOPS };

/* sizeof the C type for a type code (long double = 16 on x86-64) */
size_t oracle_type_size(int type);

/* 1 if the reference defines shmem_<type>_<op>_to_all (src/reductions.c:248-297) */
int oracle_has_op(int type, int op);

/* out[i] = op(a[i], b[i]) for i < n; a is the accumulator (first operand) */
int oracle_op(int type, int op, const void *a, const void *b, void *out,
              size_t n);

/*
 * Whole-team reduce-to-all, restating src/reductions.c:32-120 for every PE of
 * the active set.  sources[pe] / targets[pe] are the per-PE arrays for
 * pe in [0, npes); only PEs of the active set (PE_start, logPE_stride,
 * PE_size) are read/written.  Returns 0, or -1 on bad arguments.
 */
int oracle_to_all(int type, int op, int npes, int PE_start, int logPE_stride,
                  int PE_size, const void *const *sources, void *const *targets,
                  int nreduce);

/*
 * CPU baseline: the reference loop shape (copy, barrier, per-peer 64-element
 * getmem into pWrk, per-element indirect op call, barrier) run with one
 * pthread per PE over a shared in-process "symmetric heap" (getmem = memcpy
 * from the peer's heap at the same offset).  Runs `reps` timed repetitions
 * after one warm-up and returns the median seconds per call (barrier to
 * barrier, CLOCK_MONOTONIC).  Inputs/outputs as oracle_to_all, all PEs in the
 * active set 0..npes-1.  pin_cores != 0 pins PE i to core i.
 */
double oracle_cpu_baseline(int type, int op, int npes,
                           const void *const *sources, void *const *targets,
                           int nreduce, int reps, int pin_cores);
/* the same with each PE's loop split over tpp threads (contiguous element
 * ranges, same loop shape each): npes * tpp cores, pinned to cores
 * 0 .. npes*tpp-1 when pin_cores != 0 */
double oracle_cpu_baseline_split(int type, int op, int npes,
                                 const void *const *sources, void *const *targets,
                                 int nreduce, int reps, int pin_cores, int tpp);
/* the same with the reference's own element function (a T (*)(T, T) from
   oracle/_ref/libref_ops.so, e.g. shmemu_sum_double_func) in the loop;
   double, float, int and long / long long only */
double oracle_cpu_baseline_ref(int type, int op, int npes, const void *const *sources,
                               void *const *targets, int nreduce, int reps, int pin_cores,
                               int tpp, void *ref_fn);

/*
 * CPU baseline of the data-movement collectives (oracle_coll.c): kind 0
 * broadcast, 1 collect, 2 fcollect, 3 alltoall, in the reference's loop
 * shape; nb bytes per PE contribution; median seconds per call.
 */
double oracle_coll_baseline(int kind, int npes, char *const *src, char *const *tgt, size_t nb,
                            int root, int reps, int pin_cores);

#ifdef __cplusplus
}
#endif
#endif
