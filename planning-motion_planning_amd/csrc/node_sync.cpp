// node_sync.cpp -- host-side sum-all-reduce of one integer across the ranks of ONE node through a
// shared-memory segment (the per-round convergence vote of the live domain decomposition,
// eikonal/dd.py).  A round costs a few cache-line transfers instead of a gloo/TCP collective.
//
// Layout: one 64-byte slot per rank: {uint64 round; int64 value[2]}.  A rank publishes
// value[round & 1], then round (release); it reads every slot after seeing its round >= this
// round (acquire).  A rank cannot publish round + 2 before every other rank has published
// round + 1, i.e. finished reading round, so the parity slot being read is never overwritten.
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <chrono>
#include <cstdint>
#include <cstring>

#include "../../include/eikonal.h"

namespace {
struct alignas(64) Slot {
    uint64_t round;
    int64_t value[2];
};
}  // namespace

extern "C" int eik_node_allreduce(void* shm, int rank, int world, uint64_t round, int64_t value, int64_t* sum,
                                  double timeout_s) {
    if (!shm || !sum || world < 1 || rank < 0 || rank >= world || round == 0) return EIK_ERR_ARG;
    Slot* s = static_cast<Slot*>(shm);
    __atomic_store_n(&s[rank].value[round & 1], value, __ATOMIC_RELAXED);
    __atomic_store_n(&s[rank].round, round, __ATOMIC_RELEASE);
    const auto t0 = std::chrono::steady_clock::now();
    int64_t acc = 0;
    for (int r = 0; r < world; ++r) {
        for (unsigned spin = 0; __atomic_load_n(&s[r].round, __ATOMIC_ACQUIRE) < round; ++spin) {
            if ((spin & 4095u) == 4095u &&
                std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
                return EIK_ERR_HIP;
            __builtin_ia32_pause();
        }
        acc += __atomic_load_n(&s[r].value[round & 1], __ATOMIC_RELAXED);
    }
    *sum = acc;
    return EIK_OK;
}

// The segment: POSIX shared memory, created (and zeroed) by one rank, mapped by all.
extern "C" int eik_node_shm_open(const char* name, int64_t bytes, int create, void** addr) {
    if (!name || !addr || bytes <= 0) return EIK_ERR_ARG;
    *addr = nullptr;
    const int fd = shm_open(name, create ? (O_CREAT | O_EXCL | O_RDWR) : O_RDWR, 0600);
    if (fd < 0) return EIK_ERR_ARG;
    if (create && ftruncate(fd, (off_t)bytes) != 0) {
        close(fd);
        shm_unlink(name);
        return EIK_ERR_NOMEM;
    }
    void* p = mmap(nullptr, (size_t)bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) return EIK_ERR_NOMEM;
    if (create) memset(p, 0, (size_t)bytes);
    *addr = p;
    return EIK_OK;
}

extern "C" int eik_node_shm_close(void* addr, int64_t bytes) {
    if (!addr) return EIK_OK;
    return munmap(addr, (size_t)bytes) == 0 ? EIK_OK : EIK_ERR_ARG;
}

extern "C" int eik_node_shm_unlink(const char* name) { return name && shm_unlink(name) == 0 ? EIK_OK : EIK_ERR_ARG; }
