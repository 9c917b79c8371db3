// Probe: does a concurrent H2D + D2H pair still run full duplex when the two
// copy streams were created after K other streams (each used once)?  HIP
// gives a process GPU_MAX_HW_QUEUES hardware queues (4 on the pool); later
// streams share one.  One JSON line per (K, order).  Not part of the product.
//   hipcc --offload-arch=gfx950 -O2 tools/stream_queue_probe.hip -o tools/stream_queue_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <sched.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <cstring>
#include <unistd.h>

// NUMA node holding the page at p (get_mempolicy MPOL_F_NODE|MPOL_F_ADDR)
static int page_node(void *p)
{
    int node = -1;
    if (syscall(SYS_get_mempolicy, &node, nullptr, 0, p, 3) != 0) return -1;
    return node;
}

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

__global__ void touch(int *p) { if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1; }

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv)
{
    const size_t nb = (argc > 1 ? strtoull(argv[1], nullptr, 0) : (size_t) 256 << 20);
    const int kmax = argc > 2 ? atoi(argv[2]) : 6;
    const int reps = 8;
    // argv[3] (what ran before, in this process): 0 nothing, 1 a timing
    // event pair around a kernel on another stream (what torch.cuda.Event
    // does), 2 the same around a copy, 3 a non-timing event pair
    const int before = argc > 3 ? atoi(argv[3]) : 0;
    char *h_in, *h_out, *d_in, *d_out;
    int *flag;
    // argv[4]: host pages -1 hipHostMalloc (default), else mmap bound to
    // that NUMA node (mbind MPOL_BIND) then hipHostRegister
    const int node = argc > 4 ? atoi(argv[4]) : -1;
    auto host_alloc = [&](char **p) {
        if (node < 0) {
            CK(hipHostMalloc((void **) p, nb, 0));
            return;
        }
        void *m = mmap(nullptr, nb, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (m == MAP_FAILED) { perror("mmap"); exit(1); }
        unsigned long mask = 1UL << node;
        if (syscall(SYS_mbind, m, nb, 2, &mask, 64, 0) != 0) { perror("mbind"); exit(1); }
        memset(m, 1, nb);
        CK(hipHostRegister(m, nb, hipHostRegisterMapped));
        *p = (char *) m;
    };
    host_alloc(&h_in);
    host_alloc(&h_out);
    int dev = 0, gpu_node = -1;
    char bus[64] = {0};
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetPCIBusId(bus, sizeof bus, dev));
    for (char *q = bus; *q; q++) *q = (char) tolower(*q);
    {
        char path[128];
        snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
        FILE *f = fopen(path, "r");
        if (f) { if (fscanf(f, "%d", &gpu_node) != 1) gpu_node = -1; fclose(f); }
    }
    CK(hipMalloc((void **) &d_in, nb));
    CK(hipMalloc((void **) &d_out, nb));
    CK(hipMalloc((void **) &flag, 64));
    if (before) {
        hipStream_t s;
        hipEvent_t a, b;
        CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        CK(hipEventCreateWithFlags(&a, before == 3 ? hipEventDisableTiming : 0));
        CK(hipEventCreateWithFlags(&b, before == 3 ? hipEventDisableTiming : 0));
        CK(hipEventRecord(a, s));
        if (before == 2) CK(hipMemcpyAsync(d_in, h_in, 1 << 20, hipMemcpyHostToDevice, s));
        else touch<<<1, 64, 0, s>>>(flag);
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms = 0;
        if (before != 3) CK(hipEventElapsedTime(&ms, a, b));
        CK(hipEventDestroy(a));
        CK(hipEventDestroy(b));
        CK(hipStreamDestroy(s));
    }
    for (int k = 0; k <= kmax; k++) {
        for (int used = 0; used < 2; used++) {
            std::vector<hipStream_t> pre(k);
            for (auto &s : pre) {
                CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
                if (used) touch<<<1, 64, 0, s>>>(flag);
            }
            CK(hipDeviceSynchronize());
            hipStream_t si, so;
            // argv[5]: copy streams 0 default priority, 1 in lowest / out
            // highest, 2 in highest / out lowest, 3 both lowest, 4 both
            // highest, 5 both CU-masked (a queue each)
            const int smode = argc > 5 ? atoi(argv[5]) : 0;
            int lo = 0, hi = 0;
            CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
            auto mk = [&](hipStream_t *s, int pr) {
                if (smode == 0) {
                    CK(hipStreamCreateWithFlags(s, hipStreamNonBlocking));
                } else if (smode == 5) {
                    uint32_t m[8];
                    for (auto &w : m) w = 0xffffffffu;
                    CK(hipExtStreamCreateWithCUMask(s, 8, m));
                } else {
                    CK(hipStreamCreateWithPriority(s, hipStreamNonBlocking, pr));
                }
            };
            mk(&si, smode == 1 || smode == 3 ? lo : hi);
            mk(&so, smode == 2 || smode == 3 ? lo : hi);
            double best[3] = {1e9, 1e9, 1e9};  // h2d alone, d2h alone, both
            for (int r = 0; r < reps; r++) {
                double t0 = now();
                CK(hipMemcpyAsync(d_in, h_in, nb, hipMemcpyHostToDevice, si));
                CK(hipStreamSynchronize(si));
                double t1 = now();
                CK(hipMemcpyAsync(h_out, d_out, nb, hipMemcpyDeviceToHost, so));
                CK(hipStreamSynchronize(so));
                double t2 = now();
                CK(hipMemcpyAsync(d_in, h_in, nb, hipMemcpyHostToDevice, si));
                CK(hipMemcpyAsync(h_out, d_out, nb, hipMemcpyDeviceToHost, so));
                CK(hipStreamSynchronize(si));
                CK(hipStreamSynchronize(so));
                double t3 = now();
                if (r == 0) continue;
                best[0] = std::min(best[0], t1 - t0);
                best[1] = std::min(best[1], t2 - t1);
                best[2] = std::min(best[2], t3 - t2);
            }
            printf("{\"smode\": %d, \"gpu_bus\": \"%s\", \"gpu_node\": %d, \"bind\": %d, \"cpu\": %d, \"in_node\": %d, \"out_node\": %d, \"before\": %d, \"pre_streams\": %d, \"pre_used\": %d, \"bytes\": %zu, \"h2d_GBs\": %.2f, "
                   "\"d2h_GBs\": %.2f, \"duplex_GBs_each_way\": %.2f}\n",
                   smode, bus, gpu_node, node, sched_getcpu(), page_node(h_in), page_node(h_out), before, k, used, nb, nb / best[0] / 1e9, nb / best[1] / 1e9, nb / best[2] / 1e9);
            fflush(stdout);
            CK(hipStreamDestroy(si));
            CK(hipStreamDestroy(so));
            for (auto &s : pre) CK(hipStreamDestroy(s));
        }
    }
    return 0;
}
