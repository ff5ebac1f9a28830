// Pageable host -> device copy rates on the box (not product code): hipMemcpyAsync on a
// non-blocking stream vs the null stream vs hipMemcpy, and pinned staging with host threads.
//   hipcc -O2 --offload-arch=gfx950 -o tools/h2d_probe tools/h2d_probe.cpp -lpthread
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main() {
    const size_t n = 128ull << 20;
    std::vector<char> host(n, 1), back(n, 0);
    void* d = nullptr;
    hipMalloc(&d, n);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    for (int rep = 0; rep < 3; ++rep) {
        double t0 = now();
        hipMemcpyAsync(d, host.data(), n, hipMemcpyHostToDevice, s);
        hipStreamSynchronize(s);
        double t1 = now();
        hipMemcpyAsync(d, host.data(), n, hipMemcpyHostToDevice, 0);
        hipStreamSynchronize(0);
        double t2 = now();
        hipMemcpy(d, host.data(), n, hipMemcpyHostToDevice);
        double t3 = now();
        hipMemcpyAsync(back.data(), d, n, hipMemcpyDeviceToHost, s);
        hipStreamSynchronize(s);
        double t4 = now();
        printf("128 MiB pageable: H2D nonblocking stream %.2f ms, null stream %.2f ms, hipMemcpy %.2f ms; D2H stream %.2f ms\n",
               (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, (t4 - t3) * 1e3);
    }
    // pinned staging: chunks of 8 MiB, T host threads copy into a pinned ring of 2 chunks, DMA from it
    const size_t C = 8ull << 20;
    char* pin[2];
    hipHostMalloc((void**)&pin[0], C);
    hipHostMalloc((void**)&pin[1], C);
    hipEvent_t ev[2];
    hipEventCreateWithFlags(&ev[0], hipEventDisableTiming);
    hipEventCreateWithFlags(&ev[1], hipEventDisableTiming);
    for (int T : {1, 4, 8}) {
        for (int rep = 0; rep < 2; ++rep) {
            double t0 = now();
            int k = 0;
            for (size_t off = 0; off < n; off += C, ++k) {
                const int b = k & 1;
                const size_t len = std::min(C, n - off);
                hipEventSynchronize(ev[b]);  // the DMA that last used this buffer is done
                std::vector<std::thread> th;
                for (int t = 0; t < T; ++t)
                    th.emplace_back([&, t] {
                        const size_t a = len * t / T, e = len * (t + 1) / T;
                        std::memcpy(pin[b] + a, host.data() + off + a, e - a);
                    });
                for (auto& x : th) x.join();
                hipMemcpyAsync((char*)d + off, pin[b], len, hipMemcpyHostToDevice, s);
                hipEventRecord(ev[b], s);
            }
            hipStreamSynchronize(s);
            printf("pinned staging, %d host threads: %.2f ms\n", T, (now() - t0) * 1e3);
        }
    }
    return 0;
}
