/* osgpu_test_hooks.h -- test-only entry points of libosgpu_reduce.so.
 * Not part of the public header (include/osgpu_reduce.h); every hook is
 * refused (OSGPU_EINVAL) unless the process runs with OSGPU_TEST_HOOKS=1. */
#pragma once
#ifdef __cplusplus
extern "C" {
#endif

/* The next osgpu_preflight calls of this process plant a wrong mapping --
 * PE `pe` reaches PE `peer` through another member's ranges, which both
 * legs must report.  (-1, -1) clears it; it is logged on stderr while set. */
int osgpu_test_preflight_fault(int pe, int peer);

/* At most n threads per launch of the one-tile-per-workgroup kernels
 * (combine.hpp kMaxLaunchThreads, 2^31): a smaller n runs their multi-launch
 * path at small sizes.  n <= 0 restores the default; logged on stderr. */
int osgpu_test_max_launch_threads(long long n);

#ifdef __cplusplus
}
#endif
