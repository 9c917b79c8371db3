/*
 * ref_ops_shim.c -- exposes the REFERENCE's own compiled element operations.
 *
 * TEST INFRASTRUCTURE ONLY.  Linked by oracle/Makefile with
 * /root/reference/src/shmemu/miscops.c compiled unmodified (that file
 * includes only <sys/types.h>, <stdint.h>, <stddef.h>, <complex.h>; no
 * stand-in headers are involved) into oracle/_ref/libref_ops.so.
 *
 * ref_op() calls shmemu_<op>_<name>_func through a function pointer exactly
 * as src/reductions.c:95-96 does, so the golden element vectors under
 * tests/golden/ are the reference's arithmetic on this host.
 */
#include <complex.h>
#include <stddef.h>

/* prototypes of the reference functions, as defined in
   src/shmemu/miscops.c:12-105 (declared in src/shmemu/shmemu.h:160-231) */
#define P_MATH(N, T) T shmemu_sum_##N##_func(T, T); T shmemu_prod_##N##_func(T, T);
#define P_LOGIC(N, T) T shmemu_and_##N##_func(T, T); T shmemu_or_##N##_func(T, T); \
    T shmemu_xor_##N##_func(T, T);
#define P_MINMAX(N, T) T shmemu_min_##N##_func(T, T); T shmemu_max_##N##_func(T, T);
P_MATH(short, short) P_MATH(int, int) P_MATH(long, long) P_MATH(longlong, long long)
P_MATH(float, float) P_MATH(double, double) P_MATH(longdouble, long double)
P_MATH(complexf, float complex) P_MATH(complexd, double complex)
P_LOGIC(short, short) P_LOGIC(int, int) P_LOGIC(long, long) P_LOGIC(longlong, long long)
P_MINMAX(short, short) P_MINMAX(int, int) P_MINMAX(long, long) P_MINMAX(longlong, long long)
P_MINMAX(float, float) P_MINMAX(double, double) P_MINMAX(longdouble, long double)

/* op codes: 0 sum 1 prod 2 and 3 or 4 xor 5 max 6 min
   type codes: 0 short 1 int 2 long 3 longlong 4 float 5 double
               6 longdouble 7 complexf 8 complexd */

#define LOOP(T, FN)                                                            \
    do {                                                                       \
        T (*f)(T, T) = FN;                                                     \
        const T *A = (const T *) a, *B = (const T *) b;                        \
        T *O = (T *) out;                                                      \
        for (size_t i = 0; i < n; i++) O[i] = (*f)(A[i], B[i]);                \
        return 0;                                                              \
    } while (0)

#define ALLOPS(N, T)                                                           \
    switch (op) {                                                              \
    case 0: LOOP(T, shmemu_sum_##N##_func);                                    \
    case 1: LOOP(T, shmemu_prod_##N##_func);                                   \
    case 2: LOOP(T, shmemu_and_##N##_func);                                    \
    case 3: LOOP(T, shmemu_or_##N##_func);                                     \
    case 4: LOOP(T, shmemu_xor_##N##_func);                                    \
    case 5: LOOP(T, shmemu_max_##N##_func);                                    \
    case 6: LOOP(T, shmemu_min_##N##_func);                                    \
    }                                                                          \
    return -1

#define FPOPS(N, T)                                                            \
    switch (op) {                                                              \
    case 0: LOOP(T, shmemu_sum_##N##_func);                                    \
    case 1: LOOP(T, shmemu_prod_##N##_func);                                   \
    case 5: LOOP(T, shmemu_max_##N##_func);                                    \
    case 6: LOOP(T, shmemu_min_##N##_func);                                    \
    }                                                                          \
    return -1

#define CPXOPS(N, T)                                                           \
    switch (op) {                                                              \
    case 0: LOOP(T, shmemu_sum_##N##_func);                                    \
    case 1: LOOP(T, shmemu_prod_##N##_func);                                   \
    }                                                                          \
    return -1

int ref_op(int type, int op, const void *a, const void *b, void *out, size_t n)
{
    switch (type) {
    case 0: { ALLOPS(short, short); }
    case 1: { ALLOPS(int, int); }
    case 2: { ALLOPS(long, long); }
    case 3: { ALLOPS(longlong, long long); }
    case 4: { FPOPS(float, float); }
    case 5: { FPOPS(double, double); }
    case 6: { FPOPS(longdouble, long double); }
    case 7: { CPXOPS(complexf, float complex); }
    case 8: { CPXOPS(complexd, double complex); }
    }
    return -1;
}
