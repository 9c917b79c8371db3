// Per-call cost of the HIP operations on the small-nreduce team path
// (latency): each timed in isolation on an idle device, median
// of many repetitions.  Not part of the product.
//   hipcc --offload-arch=gfx950 -O2 tools/overhead_probe.hip -o tools/overhead_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <functional>
#include <vector>

__global__ void empty_kernel(int *p)
{
    if (p && threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1;
}

// writes seq to a host-mapped word (system scope): the host returns when it
// sees it, without waiting for the launch to retire (the fused path's form)
__global__ void word_kernel(unsigned long long *w, unsigned long long seq)
{
    if (threadIdx.x == 0 && blockIdx.x == 0)
        __hip_atomic_store(w, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double median_us(int reps, const std::function<void()> &f)
{
    std::vector<double> t(reps);
    for (int i = 0; i < 20; i++) f();
    for (int i = 0; i < reps; i++) {
        auto a = std::chrono::steady_clock::now();
        f();
        auto b = std::chrono::steady_clock::now();
        t[i] = std::chrono::duration<double, std::micro>(b - a).count();
    }
    std::sort(t.begin(), t.end());
    return t[reps / 2];
}

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e = (x);                                                   \
        if (e != hipSuccess) {                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));            \
            return 1;                                                         \
        }                                                                     \
    } while (0)

int main()
{
    int *d = nullptr;
    CK(hipMalloc(&d, 1 << 20));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const int R = 2000;
    hipPointerAttribute_t a;
    int dev;
    printf("{\"probe\": \"overhead\"");
    printf(", \"hipGetDevice_us\": %.3f", median_us(R, [&] { (void) hipGetDevice(&dev); }));
    printf(", \"hipPointerGetAttributes_us\": %.3f",
           median_us(R, [&] { (void) hipPointerGetAttributes(&a, d); }));
    printf(", \"hipDeviceSynchronize_idle_us\": %.3f",
           median_us(R, [&] { (void) hipDeviceSynchronize(); }));
    printf(", \"hipStreamQuery_idle_us\": %.3f", median_us(R, [&] { (void) hipStreamQuery(st); }));
    printf(", \"launch_only_us\": %.3f", median_us(R, [&] {
               hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st, d);
           }));
    CK(hipStreamSynchronize(st));
    printf(", \"launch_sync_block_us\": %.3f", median_us(R, [&] {
               hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st, d);
               (void) hipStreamSynchronize(st);
           }));
    printf(", \"launch_sync_poll_us\": %.3f", median_us(R, [&] {
               hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st, d);
               while (hipStreamQuery(st) == hipErrorNotReady) {
               }
           }));
    printf(", \"launch3_sync_poll_us\": %.3f", median_us(R, [&] {
               for (int k = 0; k < 3; k++)
                   hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st, d);
               while (hipStreamQuery(st) == hipErrorNotReady) {
               }
           }));
    printf(", \"devsync_launch_sync_poll_us\": %.3f", median_us(R, [&] {
               (void) hipDeviceSynchronize();
               hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st, d);
               while (hipStreamQuery(st) == hipErrorNotReady) {
               }
           }));
    // a 1 Ki-element 2-input int combine's worth of grid (1 block) vs 2048 blocks
    printf(", \"launch_2048blk_sync_poll_us\": %.3f", median_us(R, [&] {
               hipLaunchKernelGGL(empty_kernel, dim3(2048), dim3(256), 0, st, d);
               while (hipStreamQuery(st) == hipErrorNotReady) {
               }
           }));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    printf(", \"launch_event_sync_us\": %.3f", median_us(R, [&] {
               hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st, d);
               (void) hipEventRecord(ev, st);
               (void) hipEventSynchronize(ev);
           }));
    // launch -> the host sees a word the kernel wrote (pinned, mapped host
    // memory), the previous launch possibly still retiring
    unsigned long long *wh = nullptr, *wd = nullptr;
    CK(hipHostMalloc((void **) &wh, 64, hipHostMallocMapped));
    CK(hipHostGetDevicePointer((void **) &wd, wh, 0));
    *wh = 0;
    unsigned long long seq = 0;
    printf(", \"launch_word_us\": %.3f", median_us(R, [&] {
               ++seq;
               hipLaunchKernelGGL(word_kernel, dim3(1), dim3(64), 0, st, wd, seq);
               while (__atomic_load_n(wh, __ATOMIC_ACQUIRE) < seq) {
               }
           }));
    CK(hipStreamSynchronize(st));
    printf(", \"launch_word_retired_us\": %.3f", median_us(R, [&] {
               ++seq;
               hipLaunchKernelGGL(word_kernel, dim3(1), dim3(64), 0, st, wd, seq);
               while (__atomic_load_n(wh, __ATOMIC_ACQUIRE) < seq) {
               }
               (void) hipStreamSynchronize(st);
           }));
    printf("}\n");
    return 0;
}
