// Latency probe of the memory operations a persistent tile visit waits on (VERDICT r05 item 3:
// the write-back's drain of a fp64 tile, 64 rows x 512 B, measured p50 9 us in the event trace).
// Not product code.  Each workgroup (256 threads, like a tile visit) times, with s_memrealtime
// (100 MHz), on wave 0 lane 0's clock:
//   st_sc1   : the fp64 tile write-back -- 8 sc1 dwordx4 buffer stores per thread (4 row chunks x 2),
//              rows `pitch` bytes apart -- then s_waitcnt vmcnt(0) + barrier (the drain);
//   st_plain : the same stores without sc1;
//   st_edge  : only the tile's first and last rows (2 chunks per thread of 16 threads) + drain;
//   ld_sc1   : one sc1 dword load + wait (a poll / halo load round trip);
//   atom     : one device-scope atomicAnd with return (the in-place pass's state consumption);
//   ld_tile  : the staging loads of a tile (8 sc1 dwordx4 loads per thread) + wait.
// `grid` workgroups run the same sequence on disjoint tiles at once (1: an idle GPU; 512: every
// workgroup slot of the fp64 solver busy).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/lat_probe.hip -o /tmp/lat_probe
//   /tmp/lat_probe grid reps [pitch_bytes]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int kSC1 = 16;
constexpr int kOps = 6;

__device__ __forceinline__ unsigned long long now() { return __builtin_amdgcn_s_memrealtime(); }

__global__ __launch_bounds__(256) void probe(char* buf, long long pitch, unsigned* word, unsigned long long* out,
                                             int reps) {
    const int tid = threadIdx.x;
    const long long tile_bytes = 64 * pitch;
    char* base = buf + (long long)blockIdx.x * tile_bytes;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)tile_bytes, 0x00020000);
    const unsigned col = (tid & 15) * 32;  // 4 doubles per thread per row chunk
    __shared__ unsigned long long t[kOps];
    if (tid < kOps) t[tid] = 0;
    u32x4 v = {(unsigned)tid, 1u, 2u, 3u};
    for (int r = 0; r < reps; ++r) {
        for (int op = 0; op < kOps; ++op) {
            __syncthreads();
            const unsigned long long t0 = now();
            if (op == 0 || op == 1) {
                for (int k = 0; k < 4; ++k) {
                    const unsigned off = (unsigned)(((tid >> 4) + 16 * k) * pitch + col);
                    if (op == 0) {
                        __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, kSC1);
                        __builtin_amdgcn_raw_buffer_store_b128(v, rs, off + 16, 0, kSC1);
                    } else {
                        __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 0);
                        __builtin_amdgcn_raw_buffer_store_b128(v, rs, off + 16, 0, 0);
                    }
                }
            } else if (op == 2) {
                if (tid < 16) {
                    __builtin_amdgcn_raw_buffer_store_b128(v, rs, col, 0, kSC1);
                    __builtin_amdgcn_raw_buffer_store_b128(v, rs, (unsigned)(63 * pitch + col), 0, kSC1);
                }
            } else if (op == 3) {
                if (tid == 0) {
                    const unsigned x = __builtin_amdgcn_raw_buffer_load_b32(rs, 0, 0, kSC1);
                    v[1] += x;
                }
            } else if (op == 4) {
                if (tid == 0) v[2] += atomicAnd(word + blockIdx.x * 32, ~0u);
            } else {
                for (int k = 0; k < 4; ++k) {
                    const unsigned off = (unsigned)(((tid >> 4) + 16 * k) * pitch + col);
                    const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, kSC1);
                    const u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16, 0, kSC1);
                    v += a + b;
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0 && r > 0) t[op] += now() - t0;
        }
    }
    if (tid < kOps) out[(long long)blockIdx.x * kOps + tid] = t[tid] + (v[0] == 12345u ? 1 : 0);
}

int main(int argc, char** argv) {
    const int grid = argc > 1 ? atoi(argv[1]) : 1;
    const int reps = argc > 2 ? atoi(argv[2]) : 200;
    const long long pitch = argc > 3 ? atoll(argv[3]) : 32768;
    char* buf;
    unsigned* word;
    unsigned long long* out;
    if (hipMalloc(&buf, (size_t)grid * 64 * pitch) || hipMalloc(&word, 128ull * grid) ||
        hipMalloc(&out, 8ull * kOps * grid)) {
        printf("alloc failed\n");
        return 2;
    }
    (void)hipMemset(word, 0, 128ull * grid);
    hipLaunchKernelGGL(probe, dim3(grid), dim3(256), 0, 0, buf, pitch, word, out, 3);  // warm
    hipLaunchKernelGGL(probe, dim3(grid), dim3(256), 0, 0, buf, pitch, word, out, reps);
    if (hipDeviceSynchronize()) {
        printf("kernel failed\n");
        return 2;
    }
    std::vector<unsigned long long> h(kOps * grid);
    (void)hipMemcpy(h.data(), out, 8ull * kOps * grid, hipMemcpyDeviceToHost);
    const char* names[kOps] = {"st_sc1", "st_plain", "st_edge", "ld_sc1", "atom", "ld_tile"};
    printf("grid %d reps %d pitch %lld:", grid, reps, pitch);
    for (int op = 0; op < kOps; ++op) {
        std::vector<double> us(grid);
        for (int b = 0; b < grid; ++b) us[b] = h[(size_t)b * kOps + op] / 100.0 / (reps - 1);
        std::sort(us.begin(), us.end());
        printf("  %s p50 %.2f us max %.2f", names[op], us[grid / 2], us[grid - 1]);
    }
    printf("\n");
    return 0;
}
