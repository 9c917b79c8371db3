// heap.cpp -- the device symmetric heap as ONE contiguous virtual range per
// PE, mapped into every member of the job (osgpu_heap_create).
//
// The reference's symmetric heap is one contiguous region per PE
// (register_symmetric_heap, src/shmemc/ucx-init.c:174-213) and a symmetric
// object of any size is found on PE p at heap_base[p] + offset
// (translate_address, src/shmemc/comms.c:89-105).  HIP IPC
// (hipIpcGetMemHandle) cannot give that on this platform: an exported
// allocation of 2 GiB or more hangs the importer, so
// objects >= 2 GiB could not be symmetric across processes.
//
// Here every PE builds its heap with the virtual memory API instead:
//   * reserve one virtual range of the heap's size (hipMemAddressReserve);
//   * back it with physical chunks of at most OSGPU_HEAP_CHUNK_BYTES
//     (default 1 GiB, a multiple of the allocation granularity), each a
//     hipMemCreate allocation exportable as a dmabuf file descriptor;
//   * map the chunks back to back: the PE's own view is contiguous;
//   * hand the chunk descriptors to every member in another process over a
//     Unix-domain socket (SCM_RIGHTS; the socket's name and the chunk layout
//     travel through spare pSync words and the runtime's shmem_getmem, like
//     the staging setup in runtime.cpp);
//   * each member imports the chunks and maps them back to back into ONE
//     virtual range of its own: its view of the peer's heap is contiguous too.
// Members that are threads of one process share the PE's range directly.
// The result is registered as segment 0 of every member's heap, so every
// path (team, pull, fused) sees base + offset for objects of any size.
#include <hip/hip_runtime_api.h>

#include <errno.h>
#include <poll.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/osgpu_reduce.h"
#include "runtime.hpp"

namespace osgpu {
namespace rt {

namespace {

constexpr int kHeapPsync = 16;       // pSync[16..] during setup only (cf. runtime.cpp)
constexpr int kFdBatch = 64;         // descriptors per SCM_RIGHTS message
constexpr int kSetupTimeoutMs = 120000;
constexpr int kMaxHeapSegment = 255; // osgpu_heap_register_segment's limit

struct Mapping {                     // one heap as mapped in this process
    int pe = -1;
    int device = -1;                 // this process's device whose HBM backs it, or -1
    char *base = nullptr;
    size_t bytes = 0;                // reserved bytes
    std::vector<hipMemGenericAllocationHandle_t> h;
    std::vector<size_t> len;         // chunk lengths
    size_t nmapped = 0;              // chunks mapped so far
};

struct Heap {                        // the heap a PE created, with its imports
    int pe = -1;
    int seg = 0;                     // registry segment of every member's heap
    long key = 0;                    // the same on every member: identifies this creation
    std::vector<int> members;
    std::vector<char *> member_base; // every member's range as seen here, by set index
    std::vector<size_t> member_bytes;
    std::vector<char> member_remote; // backed by another GPU's HBM (reached over xGMI)
    Mapping own;
    std::vector<Mapping> peers;      // members in other processes
};

std::mutex g_hmu;
std::vector<Heap *> g_heaps;
// Destroyed heaps that hold chunks imported from other processes: their HBM
// is not returned before the process exits on this ROCm, so
// they are kept, fully mapped, and handed back when the same member set
// creates a heap of at most that size again (a prefix of the kept range is
// registered; every member agrees on which kept heap).
std::vector<Heap *> g_pool;

// what a PE publishes in pSync[16..] during osgpu_heap_create
struct HeapMsg {
    long pid, nonce, bytes, chunk, raw_ptr, status, device, seg, pci;
};
static_assert(sizeof(HeapMsg) <= (64 - kHeapPsync) * sizeof(long), "pSync room");

void sock_name(long pid, long nonce, sockaddr_un *a, socklen_t *len)
{
    memset(a, 0, sizeof(*a));
    a->sun_family = AF_UNIX;
    // abstract namespace: nothing on the file system to clean up
    const int n = snprintf(a->sun_path + 1, sizeof(a->sun_path) - 1, "osgpu-heap-%ld-%ld", pid,
                           nonce);
    *len = (socklen_t) (offsetof(sockaddr_un, sun_path) + 1 + n);
}

bool write_all(int fd, const void *p, size_t n)
{
    const char *c = (const char *) p;
    while (n) {
        const ssize_t w = send(fd, c, n, MSG_NOSIGNAL);
        if (w < 0 && errno == EINTR) continue;
        if (w <= 0) return false;
        c += w;
        n -= (size_t) w;
    }
    return true;
}

// descriptors in batches of kFdBatch, each batch riding on one byte
bool send_fds(int s, const std::vector<int> &fds)
{
    const unsigned long long n = fds.size();
    if (!write_all(s, &n, sizeof(n))) return false;
    for (size_t i = 0; i < fds.size(); i += kFdBatch) {
        const int m = (int) std::min(fds.size() - i, (size_t) kFdBatch);
        char byte = 'F';
        iovec iov = {&byte, 1};
        std::vector<char> ctl(CMSG_SPACE(sizeof(int) * m));
        msghdr msg;
        memset(&msg, 0, sizeof(msg));
        msg.msg_iov = &iov;
        msg.msg_iovlen = 1;
        msg.msg_control = ctl.data();
        msg.msg_controllen = ctl.size();
        cmsghdr *cm = CMSG_FIRSTHDR(&msg);
        cm->cmsg_level = SOL_SOCKET;
        cm->cmsg_type = SCM_RIGHTS;
        cm->cmsg_len = CMSG_LEN(sizeof(int) * m);
        memcpy(CMSG_DATA(cm), fds.data() + i, sizeof(int) * m);
        ssize_t w;
        do w = sendmsg(s, &msg, MSG_NOSIGNAL); while (w < 0 && errno == EINTR);
        if (w != 1) return false;
    }
    return true;
}

bool read_all(int fd, void *p, size_t n)
{
    char *c = (char *) p;
    while (n) {
        const ssize_t r = recv(fd, c, n, 0);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) return false;
        c += r;
        n -= (size_t) r;
    }
    return true;
}

bool recv_fds(int s, std::vector<int> &fds)
{
    unsigned long long n = 0;
    if (!read_all(s, &n, sizeof(n)) || n > (1u << 20)) return false;
    while (fds.size() < n) {
        const int m = (int) std::min<unsigned long long>(n - fds.size(), kFdBatch);
        char byte = 0;
        iovec iov = {&byte, 1};
        std::vector<char> ctl(CMSG_SPACE(sizeof(int) * m));
        msghdr msg;
        memset(&msg, 0, sizeof(msg));
        msg.msg_iov = &iov;
        msg.msg_iovlen = 1;
        msg.msg_control = ctl.data();
        msg.msg_controllen = ctl.size();
        ssize_t r;
        do r = recvmsg(s, &msg, MSG_CMSG_CLOEXEC); while (r < 0 && errno == EINTR);
        if (r != 1) return false;
        cmsghdr *cm = CMSG_FIRSTHDR(&msg);
        if (!cm || cm->cmsg_type != SCM_RIGHTS || (msg.msg_flags & MSG_CTRUNC)) return false;
        const int got = (int) ((cm->cmsg_len - CMSG_LEN(0)) / sizeof(int));
        if (got <= 0 || got > m) {      // a batch carries 1..m descriptors
            if (got > 0) {
                int tmp[kFdBatch];
                memcpy(tmp, CMSG_DATA(cm), sizeof(int) * std::min(got, kFdBatch));
                for (int k = 0; k < std::min(got, kFdBatch); k++) close(tmp[k]);
            }
            return false;
        }
        const size_t at = fds.size();
        fds.resize(at + got);
        memcpy(fds.data() + at, CMSG_DATA(cm), sizeof(int) * got);
    }
    return true;
}

hipMemAllocationProp chunk_prop(int dev)
{
    hipMemAllocationProp p;
    memset(&p, 0, sizeof(p));
    p.type = hipMemAllocationTypePinned;
    p.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
    p.location.type = hipMemLocationTypeDevice;
    p.location.id = dev;
    return p;
}

// read-write access to a mapped range from device `dev`
bool grant_access(char *base, size_t bytes, int dev)
{
    hipMemAccessDesc d;
    memset(&d, 0, sizeof(d));
    d.location.type = hipMemLocationTypeDevice;
    d.location.id = dev;
    d.flags = hipMemAccessFlagsProtReadWrite;
    const bool ok = hipMemSetAccess(base, bytes, &d, 1) == hipSuccess;
    (void) hipGetLastError();
    return ok;
}

// Unmap and release a heap's chunks.  The virtual range of a heap imported
// from another process stays reserved: on this ROCm (7.2) a range that held
// imported chunks and is freed and reserved again -- for a later heap of
// this process or a later import -- keeps reaching the OLD chunks from the
// GPU (every unmap / release / free call succeeds; reductions in the new
// heap read and write the old memory: test_heap_create_destroy_cycles_
// processes), so such a range is never handed back (address space only).
void unmap(Mapping &m)
{
    size_t off = 0;
    int bad = 0;
    for (size_t k = 0; k < m.nmapped; off += m.len[k], k++)
        bad += hipMemUnmap(m.base + off, m.len[k]) != hipSuccess;
    for (auto h : m.h) bad += hipMemRelease(h) != hipSuccess;
    const bool imported = m.pe >= 0 && m.device < 0;
    if (m.base && !imported) bad += hipMemAddressFree(m.base, m.bytes) != hipSuccess;
    DBG("heap unmap: PE %d's range %p (%zu B, %zu chunks): %d failed calls", m.pe,
        (void *) m.base, m.bytes, m.h.size(), bad);
    (void) hipGetLastError();
    m = Mapping();
}

// chunk lengths of a heap of `bytes` (a multiple of the granularity) in
// chunks of `chunk`
std::vector<size_t> chunk_lens(size_t bytes, size_t chunk)
{
    std::vector<size_t> v;
    for (size_t off = 0; off < bytes; off += chunk) v.push_back(std::min(chunk, bytes - off));
    return v;
}

// reserve one range and map `h` (lengths `len`) back to back into it,
// readable and writable from this process's device
bool map_chunks(Mapping &m, size_t align, int dev)
{
    void *va = nullptr;
    if (hipMemAddressReserve(&va, m.bytes, align, nullptr, 0) != hipSuccess) return false;
    m.base = (char *) va;
    size_t off = 0;
    for (size_t k = 0; k < m.h.size(); off += m.len[k], k++) {
        if (hipMemMap(m.base + off, m.len[k], 0, m.h[k], 0) != hipSuccess) return false;
        m.nmapped = k + 1;
    }
    return grant_access(m.base, m.bytes, dev);
}

size_t heap_chunk_bytes(size_t gran)
{
    static const size_t env = [] {  // read once
        const char *e = getenv("OSGPU_HEAP_CHUNK_BYTES");
        const size_t v = e ? strtoull(e, nullptr, 0) : 0;
        return v ? v : (size_t) 1 << 30;
    }();
    return (env + gran - 1) / gran * gran;
}

}  // namespace

// Inside a heap made by osgpu_heap_create (the PE's own range or a member's
// mapped into this process)?  *dev: the local device backing it, -1 for a
// member's heap in another process.
bool heap_created_range(const void *p, size_t n, int *dev)
{
    std::lock_guard<std::mutex> lk(g_hmu);
    const char *c = (const char *) p;
    for (Heap *h : g_heaps) {
        if (c >= h->own.base && c + n <= h->own.base + h->own.bytes) {
            if (dev) *dev = h->own.device;
            return true;
        }
        for (const Mapping &m : h->peers)
            if (c >= m.base && c + n <= m.base + m.bytes) {
                if (dev) *dev = -1;
                return true;
            }
    }
    return false;
}

}  // namespace rt
}  // namespace osgpu

using namespace osgpu::rt;

extern "C" int osgpu_heap_create(size_t bytes, int PE_start, int logPE_stride, int PE_size,
                                 long *pSync, void **base_out)
{
    const char *where = "osgpu_heap_create";
    if (!bytes || !pSync || !base_out || PE_size < 1) {
        set_err("%s: bad arguments", where);
        return OSGPU_EINVAL;
    }
    Coll c = make_coll(where, PE_start, logPE_stride, PE_size, pSync);
    if (PE_size > 1 && !c.ops.getmem) {
        set_err("%s: the PE runtime has no shmem_getmem", where);
        return OSGPU_ENOPE;
    }
    const int idx = c.index_of(c.me);
    if (idx < 0) {
        set_err("%s: PE %d is not in the active set", where, c.me);
        return OSGPU_EINVAL;
    }
    int dev = 0;
    HIPCHK(where, hipGetDevice(&dev));
    Heap *H = new Heap();
    H->pe = c.me;
    bool ok = true;
    size_t gran = 0;
    hipMemAllocationProp prop = chunk_prop(dev);
    if (hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended) !=
            hipSuccess ||
        !gran) {
        (void) hipGetLastError();
        gran = (size_t) 2 << 20;
    }
    const size_t total = (bytes + gran - 1) / gran * gran;
    const size_t chunk = std::min(heap_chunk_bytes(gran), total);
    for (int i = 0; i < PE_size; i++) H->members.push_back(c.pe_at(i));

    // A kept heap of this member set at least this size, if every member has
    // one from the same creation: register its first `total` bytes again
    // instead of making a new one (the smallest that fits).  A kept heap
    // never serves a LARGER request, and its HBM is not returned: a job
    // holds, per member set, the sum of every heap size that exceeded all
    // the set's earlier heaps (4, then 8, then 16 GiB keeps 28 GiB) -- make
    // the largest heap first and later ones fit inside it.  The candidate
    // must be THIS PE's: PE threads of one process share the pool.
    HeapMsg *mine = reinterpret_cast<HeapMsg *>(pSync + kHeapPsync);
    Heap *cand = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_hmu);
        for (Heap *k : g_pool)
            if (k->pe == c.me && k->members == H->members && k->own.device == dev &&
                k->own.bytes >= total && (!cand || k->own.bytes < cand->own.bytes))
                cand = k;
    }
    memset(mine, 0, sizeof(*mine));
    mine->nonce = cand ? cand->key : 0;
    mine->seg = heap_free_segment(H->members);
    barrier(c);
    bool reuse = cand != nullptr;
    int rseg = (int) mine->seg;
    for (int i = 0; i < PE_size; i++) {
        const int pe = c.pe_at(i);
        if (pe == c.me) continue;
        HeapMsg m;
        c.ops.getmem(&m, mine, sizeof(HeapMsg), pe);
        reuse = reuse && m.nonce == mine->nonce;
        rseg = std::max(rseg, (int) m.seg);
    }
    barrier(c);  // every member has read every message of this phase
    memset(mine, 0, sizeof(*mine));
    // every member computes the same rseg: the same verdict everywhere
    if (rseg > kMaxHeapSegment) {
        set_err("%s: the heap registry is full (segment %d > %d): destroy heaps first", where,
                rseg, kMaxHeapSegment);
        delete H;
        return OSGPU_ENOMEM;
    }
    if (reuse) {
        {
            std::lock_guard<std::mutex> lk(g_hmu);
            g_pool.erase(std::find(g_pool.begin(), g_pool.end(), cand));
            cand->seg = rseg;
            g_heaps.push_back(cand);
        }
        for (int i = 0; i < PE_size; i++) {  // cannot fail: arguments checked above
            (void) osgpu_heap_register_segment(c.pe_at(i), rseg, cand->member_base[i],
                                               std::min(total, cand->member_bytes[i]));
            heap_set_remote(c.pe_at(i), rseg, cand->member_remote[i] != 0);
        }
        delete H;
        *base_out = cand->own.base;
        DBG("%s PE %d: kept heap %p of %zu B registered again for %zu B (segment %d)", where,
            c.me, (void *) cand->own.base, cand->own.bytes, total, rseg);
        return OSGPU_OK;
    }
    std::vector<int> fds;
    H->own.pe = c.me;
    H->own.device = dev;
    H->own.bytes = total;
    H->own.len = chunk_lens(total, chunk);
    bool nomem = false;  // this member's failure is a lack of device memory
    {  // more than the device has free cannot succeed: fail at once instead
       // of creating chunks until the HBM runs out
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) == hipSuccess && total > fr) {
            size_t kept = 0;
            {
                std::lock_guard<std::mutex> lk(g_hmu);
                for (Heap *k : g_pool)
                    if (k->own.device == dev) kept += k->own.bytes;
            }
            set_err("%s: out of device memory: %zu B requested, %zu B free on device %d "
                    "(%zu B held by destroyed heaps kept for reuse: a later heap of the same "
                    "member set up to their size reuses them; their HBM returns at exit)",
                    where, total, fr, dev, kept);
            ok = false;
            nomem = true;
        }
        (void) hipGetLastError();
    }
    for (size_t k = 0; ok && k < H->own.len.size(); k++) {
        hipMemGenericAllocationHandle_t h;
        if (hipMemCreate(&h, H->own.len[k], &prop, 0) != hipSuccess) {
            set_err("%s: out of device memory: hipMemCreate(%zu B) failed", where,
                    H->own.len[k]);
            (void) hipGetLastError();
            ok = false;
            nomem = true;
            break;
        }
        H->own.h.push_back(h);
        int fd = -1;
        if (hipMemExportToShareableHandle(&fd, h, hipMemHandleTypePosixFileDescriptor, 0) !=
                hipSuccess ||
            fd < 0) {
            set_err("%s: hipMemExportToShareableHandle failed", where);
            ok = false;
            break;
        }
        fds.push_back(fd);
    }
    DBG("%s PE %d: %zu chunks of %zu B created and exported (ok=%d)", where, c.me,
        H->own.len.size(), chunk, (int) ok);
    if (ok && !map_chunks(H->own, gran, dev)) {
        set_err("%s: mapping the heap failed", where);
        ok = false;
    }
    (void) hipGetLastError();

    // listening socket for the members in other processes
    static std::atomic<long> nonce_ctr{0};
    const long nonce = ((long) time(nullptr) << 20) ^ (nonce_ctr.fetch_add(1) + 1);
    int lfd = ok ? socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0) : -1;
    if (ok) {
        sockaddr_un a;
        socklen_t al;
        sock_name((long) getpid(), nonce, &a, &al);
        if (lfd < 0 || bind(lfd, (sockaddr *) &a, al) != 0 || listen(lfd, 64) != 0) {
            set_err("%s: unix socket: %s", where, strerror(errno));
            ok = false;
        }
    }
    memset(mine, 0, sizeof(*mine));
    mine->pid = (long) getpid();
    mine->nonce = nonce;
    mine->bytes = ok ? (long) total : -1;
    mine->chunk = (long) chunk;
    mine->raw_ptr = (long) (uintptr_t) H->own.base;
    mine->device = dev;
    mine->pci = pci_key(dev);
    // every heap of a member set gets its own registry segment: the lowest
    // one free for every member here, agreed as the maximum over members
    mine->seg = heap_free_segment(H->members);
    DBG("%s PE %d: own heap mapped at %p, listening (ok=%d)", where, c.me, (void *) H->own.base,
        (int) ok);
    barrier(c);

    // everyone's layout; how many members from other processes will connect
    std::vector<HeapMsg> msg(PE_size);
    for (int i = 0; i < PE_size; i++) {
        const int pe = c.pe_at(i);
        if (pe == c.me) msg[i] = *mine;
        else c.ops.getmem(&msg[i], mine, sizeof(HeapMsg), pe);
        if (msg[i].bytes <= 0) ok = false;
    }
    for (int i = 0; i < PE_size; i++) H->seg = std::max(H->seg, (int) msg[i].seg);
    // Every member reads the same messages, so the checks below give the
    // same verdict on every member.
    //  * the registry has room for the segment;
    //  * no mixed topology: a process holding several PE threads AND
    //    members in other processes would import each remote heap once per
    //    thread, into ranges only that thread's device may access, and the
    //    process-global registry would keep whichever thread wrote last
    //    (a GPU fault for the others).  Threads only, or one PE per process.
    bool refused = false;
    if (H->seg > kMaxHeapSegment) {
        set_err("%s: the heap registry is full (segment %d > %d): destroy heaps first", where,
                H->seg, kMaxHeapSegment);
        refused = true;
    }
    {
        std::vector<long> pids;
        bool shared = false;
        for (int i = 0; i < PE_size; i++) {
            if (std::find(pids.begin(), pids.end(), msg[i].pid) != pids.end()) shared = true;
            else pids.push_back(msg[i].pid);
        }
        if (shared && pids.size() > 1) {
            set_err("%s: unsupported topology: %zu processes, some holding several PEs of the "
                    "active set; use one PE per process, or PE threads of one process only",
                    where, pids.size());
            refused = true;
        }
    }
    if (refused) ok = false;
    // members that are threads of this process on another GPU use my range
    // directly: their devices need access to it too (only theirs -- a grant
    // binds this process to that GPU, which one-process-per-GPU jobs never
    // need); done before the status barrier below, after which they use it
    for (int i = 0; ok && i < PE_size; i++) {
        if (c.pe_at(i) == c.me || msg[i].pid != (long) getpid() || msg[i].device == dev) continue;
        if (!grant_access(H->own.base, H->own.bytes, (int) msg[i].device)) {
            set_err("%s: device %ld cannot access PE %d's heap", where, msg[i].device, c.me);
            ok = false;
        }
    }
    int expected = 0;
    for (int i = 0; i < PE_size; i++)
        if (c.pe_at(i) != c.me && msg[i].pid != (long) getpid()) expected++;
    DBG("%s PE %d: layouts read, %d members in other processes", where, c.me, expected);
    // Serve my descriptors to every member in another process until all of
    // them have connected, or until every member has finished importing (the
    // status barrier below: a member that failed may never connect), or a
    // time bound passes.
    std::atomic<int> served{0};
    std::atomic<bool> stop{false};
    std::thread server;
    if (lfd >= 0 && expected > 0 && mine->bytes > 0) {
        server = std::thread([&, lfd, expected] {
            int waited_ms = 0;
            for (int k = 0; k < expected && !stop.load() && waited_ms < kSetupTimeoutMs;) {
                pollfd p = {lfd, POLLIN, 0};
                const int r = poll(&p, 1, 100);
                if (r < 0 && errno != EINTR) return;
                if (r <= 0) {
                    waited_ms += 100;
                    continue;
                }
                const int s = accept4(lfd, nullptr, nullptr, SOCK_CLOEXEC);
                if (s < 0) continue;
                DBG("osgpu_heap_create: serving connection %d", k);
                if (send_fds(s, fds)) {
                    char ack;
                    (void) read_all(s, &ack, 1);  // the importer has its copies
                    served.fetch_add(1);
                }
                close(s);
                k++;
            }
        });
    }
    // import every member's heap (same process: its own range)
    std::vector<char *> base(PE_size, nullptr);
    for (int i = 0; i < PE_size && ok; i++) {
        const int pe = c.pe_at(i);
        if (pe == c.me) {
            base[i] = H->own.base;
            continue;
        }
        if (msg[i].pid == (long) getpid()) {
            base[i] = (char *) (uintptr_t) msg[i].raw_ptr;
            continue;
        }
        const int s = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
        if (s >= 0) {  // a member that stopped serving must not hang this one
            timeval tv = {kSetupTimeoutMs / 1000, 0};
            setsockopt(s, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
            setsockopt(s, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
        }
        sockaddr_un a;
        socklen_t al;
        sock_name(msg[i].pid, msg[i].nonce, &a, &al);
        std::vector<int> pf;
        bool got = s >= 0 && connect(s, (sockaddr *) &a, al) == 0;
        DBG("%s PE %d: connected to PE %d: %d", where, c.me, pe, (int) got);
        got = got && recv_fds(s, pf);
        DBG("%s PE %d: %zu descriptors from PE %d", where, c.me, pf.size(), pe);
        Mapping m;
        m.pe = pe;
        m.bytes = (size_t) msg[i].bytes;
        m.len = chunk_lens(m.bytes, (size_t) msg[i].chunk);
        got = got && pf.size() == m.len.size();
        for (size_t k = 0; got && k < pf.size(); k++) {
            hipMemGenericAllocationHandle_t h;
            // ROCm reads the descriptor through the pointer (CUDA takes the
            // value itself): passing the fd as an address faults
            int fd = pf[k];
            if (hipMemImportFromShareableHandle(&h, &fd, hipMemHandleTypePosixFileDescriptor) !=
                hipSuccess) {
                set_err("%s: importing PE %d's heap chunk %zu failed", where, pe, k);
                got = false;
                break;
            }
            m.h.push_back(h);
            DBG("%s PE %d: imported chunk %zu of PE %d", where, c.me, k, pe);
        }
        for (int fd : pf) close(fd);
        if (s >= 0) {
            const char ack = 'A';
            (void) write_all(s, &ack, 1);
            close(s);
        }
        if (got && !map_chunks(m, gran, dev)) {
            set_err("%s: mapping PE %d's heap failed", where, pe);
            got = false;
        }
        (void) hipGetLastError();
        if (!got) {
            if (pf.size() != m.len.size())
                set_err("%s: %zu of %zu chunk descriptors from PE %d", where, pf.size(),
                        m.len.size(), pe);
            unmap(m);
            ok = false;
            break;
        }
        base[i] = m.base;
        DBG("%s PE %d: PE %d's heap mapped at %p", where, c.me, pe, (void *) m.base);
        H->peers.push_back(m);
    }
    // every member's verdict; after this barrier every member has finished
    // importing, so no one connects any more: the server can stop
    // 1 ok, 2 failed, 3 failed for lack of device memory
    mine->status = ok ? 1 : (nomem ? 3 : 2);
    barrier(c);
    stop.store(true);
    if (server.joinable()) server.join();
    if (lfd >= 0) close(lfd);
    for (int fd : fds) close(fd);
    DBG("%s PE %d: served %d of %d, ok=%d", where, c.me, served.load(), expected, (int) ok);
    bool all_ok = ok;
    int nomem_pe = nomem ? c.me : -1;
    for (int i = 0; i < PE_size; i++) {
        const int pe = c.pe_at(i);
        if (pe == c.me) continue;
        long st = 0;
        c.ops.getmem(&st, &mine->status, sizeof(long), pe);
        all_ok = all_ok && st == 1;
        if (st == 3 && nomem_pe < 0) nomem_pe = pe;
    }
    barrier(c);
    memset(mine, 0, sizeof(*mine));  // pSync back to SHMEM_SYNC_VALUE
    if (!all_ok) {
        for (Mapping &m : H->peers) unmap(m);
        unmap(H->own);
        delete H;
        if (refused) return OSGPU_EINVAL;  // every member refused the same way
        if (nomem_pe >= 0) {
            if (!nomem)
                set_err("%s: PE %d is out of device memory for its heap", where, nomem_pe);
            return OSGPU_ENOMEM;
        }
        if (ok) set_err("%s: another member failed to create or map its heap", where);
        return OSGPU_EPEER;
    }
    int me_idx = 0;
    for (int i = 0; i < PE_size; i++)
        if (c.pe_at(i) == c.me) me_idx = i;
    unsigned long long key = 0x9e3779b97f4a7c15ull;  // the same on every member
    for (int i = 0; i < PE_size; i++) {
        // cannot fail: base and size checked, segment within the registry
        (void) osgpu_heap_register_segment(c.pe_at(i), H->seg, base[i], (size_t) msg[i].bytes);
        const bool remote = msg[i].pci != msg[me_idx].pci;
        heap_set_remote(c.pe_at(i), H->seg, remote);
        H->member_remote.push_back(remote ? 1 : 0);
        H->member_base.push_back(base[i]);
        H->member_bytes.push_back((size_t) msg[i].bytes);
        key = (key ^ (unsigned long long) msg[i].pid) * 0x100000001b3ull;
        key = (key ^ (unsigned long long) msg[i].nonce) * 0x100000001b3ull;
    }
    H->key = (long) (key | 1);  // never 0 (0 = "no kept heap")
    {
        std::lock_guard<std::mutex> lk(g_hmu);
        g_heaps.push_back(H);
    }
    *base_out = H->own.base;
    DBG("%s PE %d: heap %zu B at %p (%zu chunks), %d members", where, c.me, total,
        (void *) H->own.base, H->own.len.size(), PE_size);
    return OSGPU_OK;
}

extern "C" int osgpu_heap_destroy(void *base)
{
    Heap *H = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_hmu);
        for (size_t i = 0; i < g_heaps.size(); i++)
            if (g_heaps[i]->own.base == (char *) base) {
                H = g_heaps[i];
                g_heaps.erase(g_heaps.begin() + (long) i);
                break;
            }
    }
    if (!H) {
        set_err("osgpu_heap_destroy: %p is not a heap made by osgpu_heap_create", base);
        return OSGPU_EINVAL;
    }
    (void) hipDeviceSynchronize();
    // forget the registrations that point into these ranges
    for (int pe : H->members) heap_clear_segment(pe, H->seg);
    if (!H->peers.empty()) {  // holds imported chunks: kept for a later heap
        std::lock_guard<std::mutex> lk(g_hmu);
        g_pool.push_back(H);
        return OSGPU_OK;
    }
    unmap(H->own);
    delete H;
    return OSGPU_OK;
}

// ---------------------------------------------------------------------
// osgpu_preflight: prove every cross-process mapping of a job before its
// first collective touches it.  A mapping that is wrong (an import that
// failed silently, a peer range this GPU may not access, staging opened on
// the wrong allocation) otherwise first shows up as a GPU fault inside a
// team kernel, with no hint of which peer or chunk.  Each member writes a
// pattern that names (PE, region, chunk, end) into 64 B at both ends of
//   * every chunk of its heap made by osgpu_heap_create (if heap_base),
//   * its STAGED staging area of this active set (if the runtime has
//     shmem_getmem; the staging set is made here when it does not exist),
//   * word 31 (unused by the protocol) of its device-barrier flag area
//     (members in distinct processes only),
// then every member reads every peer's patterns through ITS OWN mapping:
// first with a host copy (hipMemcpy), then -- only where that matched --
// with the copy kernel (copy.hip, the code path of the collectives).
//
// Then the other direction, the one the team kernel (its stores of shard g
// into every member's target, team.hip) and the push form (its scatter into
// the members' staging inboxes) use: remote WRITES into 128 B at both ends
// of every heap chunk and of the staging area, 16 B per writer (its
// active-set index).  The owner first reads its blocks with plain cached
// loads, so the lines sit in its L2; every peer then writes its piece
// through its mapping -- by host copy, and in a second round by the copy
// kernel -- and after a barrier the owner re-reads the blocks by kernel and
// checks every writer's piece.  This is the reference's guarantee that a
// PE's remote puts are complete and visible at its target before the
// barrier returns (shmemc_quiet -> ucp_worker_flush ahead of the barrier,
// src/shmemc/comms.c:147-161, src/shmemc/barrier.c:176-181).
//
// Test hook: osgpu_test_preflight_fault(pe, peer) makes PE <pe> reach peer
// <peer>'s heap chunks and staging through ANOTHER member's mappings (a
// planted wrong mapping), which both legs must report.
// ---------------------------------------------------------------------

namespace {

struct Probe {                // one 64-B block to check on a peer
    const char *region;       // "heap" / "staging" / "flags"
    int chunk;                // chunk index (heap), 0 otherwise
    int end;                  // 0 low end, 1 high end
    const char *addr;         // the peer's block as mapped in this process
    size_t bytes;             // 64, or 8 for the flag word
};

void pattern(unsigned long long *w, size_t words, int pe, int region, int chunk, int end)
{
    unsigned long long x = 0x243f6a8885a308d3ull ^ ((unsigned long long) pe << 40) ^
                           ((unsigned long long) region << 32) ^
                           ((unsigned long long) chunk << 8) ^ (unsigned long long) end;
    for (size_t j = 0; j < words; j++) {  // splitmix64
        x += 0x9e3779b97f4a7c15ull;
        unsigned long long z = x;
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        w[j] = z ^ (z >> 31);
    }
}

int region_code(const char *r) { return r[0] == 'h' ? 1 : r[0] == 's' ? 2 : 3; }

// the remote-write leg's 16-B piece of `writer` in owner's block
void wpattern(unsigned long long *w, int writer, int owner, int region, int chunk, int end,
              int leg)
{
    pattern(w, 2, writer, region + 8 * leg, (chunk << 12) ^ owner, end);
}

// planted by osgpu_test_preflight_fault (test hook; never from the
// environment, so a stray variable cannot redirect real remote writes)
std::atomic<int> g_fault_pe{-1}, g_fault_peer{-1};

// the active-set index whose mappings PE `me` uses for member index i
int probe_view(const Coll &c, int me, int i)
{
    const int fpe = g_fault_pe.load(), fpeer = g_fault_peer.load();
    if (fpe < 0 || fpe != c.me || fpeer != c.pe_at(i)) return i;
    for (int j = 0; j < c.PE_size; j++)
        if (j != i && j != me) return j;
    return me;  // two members: my own range stands in for the peer's
}

// chunk layout of the heap whose own range starts at `base` (this process)
bool own_chunks(const char *base, std::vector<size_t> *len)
{
    std::lock_guard<std::mutex> lk(g_hmu);
    for (Heap *h : g_heaps)
        if (h->own.base == base) {
            *len = h->own.len;
            return true;
        }
    return false;
}

}  // namespace

extern "C" int osgpu_preflight(void *heap_base, int PE_start, int logPE_stride, int PE_size,
                               long *pSync, char *report, size_t report_bytes)
{
    const char *where = "osgpu_preflight";
    if (!pSync || PE_size < 1 || (report && !report_bytes)) {
        set_err("%s: bad arguments", where);
        return OSGPU_EINVAL;
    }
    Coll c = make_coll(where, PE_start, logPE_stride, PE_size, pSync);
    const int me = c.index_of(c.me);
    if (me < 0) {
        set_err("%s: PE %d is not in the active set", where, c.me);
        return OSGPU_EINVAL;
    }
    Heap *H = nullptr;
    if (heap_base) {
        std::lock_guard<std::mutex> lk(g_hmu);
        for (Heap *h : g_heaps)
            if (h->own.base == (char *) heap_base) H = h;
    }
    bool same_set = H && H->members.size() == (size_t) PE_size;
    for (int i = 0; same_set && i < PE_size; i++) same_set = H->members[i] == c.pe_at(i);
    if (heap_base && !same_set) {
        set_err("%s: %p is not a heap of this active set made by osgpu_heap_create", where,
                heap_base);
        return OSGPU_EINVAL;  // the same on every member given the same arguments
    }
    // collective setups (same decision on every member)
    StageSet *S = (PE_size > 1 && c.ops.getmem) ? stage_setup(c) : nullptr;
    // flag areas exist only when every member is its own process
    SyncSet *Y = (PE_size > 1 && c.ops.getmem) ? sync_setup(c) : nullptr;

    // 1. my patterns
    constexpr size_t B = 64;
    unsigned long long w[B / 8];
    auto put = [&](char *at, size_t bytes, int region, int chunk, int end) {
        pattern(w, bytes / 8, c.me, region, chunk, end);
        return hipMemcpy(at, w, bytes, hipMemcpyHostToDevice) == hipSuccess;
    };
    bool wrote = true;
    if (H) {
        size_t off = 0;
        for (size_t k = 0; k < H->own.len.size(); off += H->own.len[k], k++) {
            wrote = put(H->own.base + off, B, 1, (int) k, 0) && wrote;
            wrote = put(H->own.base + off + H->own.len[k] - B, B, 1, (int) k, 1) && wrote;
        }
    }
    if (S) {
        wrote = put(S->local, B, 2, 0, 0) && wrote;
        wrote = put(S->local + 4 * S->slot - B, B, 2, 0, 1) && wrote;
    }
    if (Y) wrote = put((char *) (Y->local + 31), 8, 3, 0, 0) && wrote;
    (void) hipDeviceSynchronize();
    (void) hipGetLastError();
    barrier(c);  // every member's patterns are in place

    // 2. the peers' blocks through my mappings
    std::vector<std::vector<Probe>> probes(PE_size);
    std::vector<std::vector<size_t>> peer_len(PE_size);  // chunk layout of member i's heap
    for (int i = 0; i < PE_size; i++) {
        if (i == me) continue;
        const int v = probe_view(c, me, i);  // = i unless a fault is planted
        if (H) {
            std::vector<size_t> &len = peer_len[i];
            bool have = false;
            for (const Mapping &m : H->peers)
                if (m.pe == c.pe_at(i)) {
                    len = m.len;
                    have = true;
                }
            if (!have) have = own_chunks(H->member_base[i], &len);  // a PE thread here
            if (!have) len.clear();
            size_t off = 0;
            for (size_t k = 0; k < len.size(); off += len[k], k++) {
                probes[i].push_back({"heap", (int) k, 0, H->member_base[v] + off, B});
                probes[i].push_back({"heap", (int) k, 1, H->member_base[v] + off + len[k] - B, B});
            }
        }
        if (S) {
            probes[i].push_back({"staging", 0, 0, S->region(v), B});
            probes[i].push_back({"staging", 0, 1, S->region(v) + 4 * S->slot - B, B});
        }
        if (Y) probes[i].push_back({"flags", 0, 0, (const char *) (Y->peer[i] + 31), 8});
    }
    char *dtmp = nullptr;
    const bool have_tmp = hipMalloc((void **) &dtmp, B) == hipSuccess;
    (void) hipGetLastError();
    hipStream_t st = thread_stream(where);
    bool all = wrote;
    int nprobes = 0, nbad = 0;
    std::vector<std::string> read_bad(PE_size);
    for (int i = 0; i < PE_size; i++) {
        if (i == me) continue;
        std::string &bad = read_bad[i];
        for (const Probe &p : probes[i]) {
            nprobes++;
            unsigned long long want[B / 8], got[B / 8];
            pattern(want, p.bytes / 8, c.pe_at(i), region_code(p.region), p.chunk, p.end);
            const char *what = nullptr;
            hipError_t e = hipMemcpy(got, p.addr, p.bytes, hipMemcpyDeviceToHost);
            if (e != hipSuccess) what = "host copy failed";
            else if (memcmp(got, want, p.bytes)) what = "host copy read other data";
            (void) hipGetLastError();
            if (!what) {  // the copy kernel through the same mapping
                osgpu::CopySeg seg = {p.addr, dtmp, p.bytes};
                e = have_tmp ? osgpu::launch_copy(&seg, 1, st) : hipErrorOutOfMemory;
                if (e == hipSuccess) e = hipStreamSynchronize(st);
                if (e == hipSuccess) e = hipMemcpy(got, dtmp, p.bytes, hipMemcpyDeviceToHost);
                if (e != hipSuccess) what = "copy kernel failed";
                else if (memcmp(got, want, p.bytes)) what = "copy kernel read other data";
                (void) hipGetLastError();
            }
            if (what) {
                nbad++;
                char b[160];
                snprintf(b, sizeof(b), "%s%s %s%d %s: %s", bad.empty() ? "" : "; ", p.region,
                         strcmp(p.region, "heap") ? "" : "chunk ",
                         strcmp(p.region, "heap") ? 0 : p.chunk, p.end ? "high" : "low", what);
                bad += b;
            }
        }
        all = all && bad.empty();
    }
    barrier(c);  // nobody reuses the regions before every member has read them

    // 3. remote writes: 16 B per writer in 128-B blocks at both ends of every
    // heap chunk and of the staging area (what team.hip's stores into the
    // members' targets and the push form's inbox scatter do)
    // 16 B per member, whole 128-B lines: sized by the active set, which may
    // exceed the team kernel's kMaxTeam (staging and PE threads allow more)
    const size_t WB = ((size_t) 16 * PE_size + 127) / 128 * 128;
    struct WBlock {
        const char *region;
        int chunk, end;
        char *at;  // the block in member i's memory, as mapped here (mine: my own)
    };
    auto blocks_of = [&](int i) {
        std::vector<WBlock> v;
        const int m = i == me ? me : probe_view(c, me, i);
        if (H) {
            std::vector<size_t> len;
            if (i == me) len = H->own.len;
            else len = peer_len[i];
            char *base = i == me ? H->own.base : H->member_base[m];
            size_t off = 0;
            for (size_t k = 0; k < len.size(); off += len[k], k++) {
                v.push_back({"heap", (int) k, 0, base + off});
                v.push_back({"heap", (int) k, 1, base + off + len[k] - WB});
            }
        }
        if (S) {
            char *r = i == me ? S->local : S->region(m);
            v.push_back({"staging", 0, 0, r});
            v.push_back({"staging", 0, 1, r + 4 * S->slot - WB});
        }
        return v;
    };
    const std::vector<WBlock> mine = blocks_of(me);
    std::vector<std::string> write_bad(PE_size);  // by writer (my view as owner) + my own errors
    char *wtmp = nullptr;
    const bool have_wtmp = hipMalloc((void **) &wtmp, WB * 2) == hipSuccess;
    (void) hipGetLastError();
    auto note = [&](int i, const WBlock &b, const char *what) {
        char m[160];
        snprintf(m, sizeof(m), "%s%s %s%d %s: %s", write_bad[i].empty() ? "" : "; ", b.region,
                 strcmp(b.region, "heap") ? "" : "chunk ", strcmp(b.region, "heap") ? 0 : b.chunk,
                 b.end ? "high" : "low", what);
        write_bad[i] += m;
    };
    // the owner's view of its blocks, read by kernel with cached loads, in
    // pieces of at most kProbeLoadBytes (one probe workgroup: a block of a
    // set of more than 128 members is larger)
    auto owner_read = [&](const WBlock &b, unsigned long long *got) {
        hipError_t e = have_wtmp ? hipSuccess : hipErrorOutOfMemory;
        for (size_t o = 0; e == hipSuccess && o < WB; o += osgpu::kProbeLoadBytes) {
            const size_t len = WB - o < osgpu::kProbeLoadBytes ? WB - o : osgpu::kProbeLoadBytes;
            e = osgpu::launch_probe_load(b.at + o, wtmp + o, len, st);
        }
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e == hipSuccess) e = hipMemcpy(got, wtmp, WB, hipMemcpyDeviceToHost);
        (void) hipGetLastError();
        return e == hipSuccess;
    };
    int nwrite = 0, nwbad = 0;
    if (!mine.empty() || H || S) {
        // 3a. clear my blocks and pull them into my L2
        std::vector<unsigned long long> gotv(WB / 8);
        unsigned long long *got = gotv.data();
        for (const WBlock &b : mine) {
            (void) hipMemset(b.at, 0, WB);
            (void) hipDeviceSynchronize();
            (void) owner_read(b, got);
        }
        (void) hipGetLastError();
        barrier(c);
        for (int leg = 1; leg <= 2; leg++) {
            // 3b. my piece into every peer's blocks through my mappings
            for (int i = 0; i < PE_size; i++) {
                if (i == me) continue;
                for (const WBlock &b : blocks_of(i)) {
                    nwrite++;
                    unsigned long long w[2];
                    wpattern(w, c.me, c.pe_at(i), region_code(b.region), b.chunk, b.end, leg);
                    char *at = b.at + 16 * me;
                    hipError_t e;
                    if (leg == 1) {
                        e = hipMemcpy(at, w, 16, hipMemcpyHostToDevice);
                    } else {  // the copy kernel's 16-B vector store into peer memory
                        e = have_wtmp ? hipMemcpy(wtmp + WB, w, 16, hipMemcpyHostToDevice)
                                      : hipErrorOutOfMemory;
                        osgpu::CopySeg seg = {wtmp + WB, at, 16};
                        if (e == hipSuccess) e = osgpu::launch_copy(&seg, 1, st);
                        if (e == hipSuccess) e = hipStreamSynchronize(st);
                    }
                    (void) hipGetLastError();
                    if (e != hipSuccess) {
                        nwbad++;
                        note(i, b, leg == 1 ? "host-copy write to the peer failed"
                                            : "copy-kernel write to the peer failed");
                    }
                }
            }
            (void) hipDeviceSynchronize();
            (void) hipGetLastError();
            barrier(c);  // every writer's stores are complete
            // 3c. every writer's piece in my blocks, read by kernel
            for (const WBlock &b : mine) {
                const bool ok = owner_read(b, got);
                for (int j = 0; j < PE_size; j++) {
                    if (j == me) continue;
                    unsigned long long want[2];
                    wpattern(want, c.pe_at(j), c.me, region_code(b.region), b.chunk, b.end, leg);
                    if (!ok || memcmp(got + 2 * j, want, 16)) {
                        nwbad++;
                        note(j, b, !ok ? "owner's read kernel failed"
                                       : leg == 1 ? "its host-copy write not seen by the owner"
                                                  : "its copy-kernel write not seen by the owner");
                    }
                }
            }
            barrier(c);  // the owners have read this round before the next one writes
        }
    }
    if (have_wtmp) (void) hipFree(wtmp);
    if (have_tmp) (void) hipFree(dtmp);

    std::string rep = "{";
    for (int i = 0; i < PE_size; i++) {
        if (i == me) continue;
        char b[96];
        int nheap = 0;
        for (const Probe &p : probes[i]) nheap += !strcmp(p.region, "heap") && p.end == 0;
        snprintf(b, sizeof(b), "%s\"%d\": {\"chunks\": %d, \"staging\": %s, \"flags\": %s, ",
                 rep.size() > 1 ? ", " : "", c.pe_at(i), nheap, S ? "true" : "false",
                 Y ? "true" : "false");
        rep += b;
        rep += read_bad[i].empty() ? "\"status\": \"ok\", " : "\"status\": \"" + read_bad[i] + "\", ";
        rep += write_bad[i].empty() ? "\"remote_write\": \"ok\"}"
                                    : "\"remote_write\": \"" + write_bad[i] + "\"}";
        all = all && write_bad[i].empty();
    }
    rep += "}";
    DBG("%s PE %d: %d probes, %d bad; %d remote writes, %d bad", where, c.me, nprobes, nbad,
        nwrite, nwbad);
    if (report) {
        if (rep.size() + 1 > report_bytes) {
            set_err("%s: the report needs %zu bytes", where, rep.size() + 1);
            snprintf(report, report_bytes, "%s", "{}");
            return OSGPU_EINVAL;
        }
        memcpy(report, rep.c_str(), rep.size() + 1);
    }
    if (!wrote) set_err("%s: writing this PE's patterns failed", where);
    else if (!all)
        set_err("%s: %d of %d read probes and %d remote-write checks failed", where, nbad, nprobes,
                nwbad);
    return all ? OSGPU_OK : OSGPU_EPEER;
}

// Test hook (tests/support/mp_worker.py): plant a wrong mapping for the next
// osgpu_preflight calls of this process -- PE `pe` reaches peer `peer`
// through another member's ranges.  (-1, -1) clears it.  Logged, so a
// planted fault never goes unseen.
// Not in the public header (tests/support/osgpu_test_hooks.h) and refused
// unless the process runs with OSGPU_TEST_HOOKS=1: a production caller can
// never redirect preflight writes by accident.
// Launch-size limit for the one-tile-per-workgroup kernels
// (combine.hpp kMaxLaunchThreads): a smaller limit runs their multi-launch
// path at small sizes.  n <= 0 restores the default.  Test hooks only.
extern "C" int osgpu_test_max_launch_threads(long long n)
{
    const char *on = getenv("OSGPU_TEST_HOOKS");
    if (!on || strcmp(on, "1")) {
        set_err("osgpu_test_max_launch_threads: test hooks are off (OSGPU_TEST_HOOKS=1 enables them)");
        return OSGPU_EINVAL;
    }
    const size_t lim = n <= 0 || (size_t) n > osgpu::kMaxLaunchThreads ? osgpu::kMaxLaunchThreads
                                                                       : (size_t) n;
    osgpu::set_max_launch_threads(lim);
    if (lim != osgpu::kMaxLaunchThreads)
        fprintf(stderr, "[osgpu] test hook: at most %zu threads per kernel launch\n", lim);
    return OSGPU_OK;
}

extern "C" int osgpu_test_preflight_fault(int pe, int peer)
{
    const char *on = getenv("OSGPU_TEST_HOOKS");
    if (!on || strcmp(on, "1")) {
        set_err("osgpu_test_preflight_fault: test hooks are off (OSGPU_TEST_HOOKS=1 enables them)");
        return OSGPU_EINVAL;
    }
    if ((pe < 0) != (peer < 0)) return OSGPU_EINVAL;
    g_fault_pe.store(-1);
    g_fault_peer.store(peer);
    g_fault_pe.store(pe);
    if (pe >= 0)
        fprintf(stderr, "[osgpu] test hook: preflight of PE %d reaches PE %d through another "
                        "member's mappings\n", pe, peer);
    return OSGPU_OK;
}
