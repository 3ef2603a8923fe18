// launch_probe -- what a timed launch costs on the host's critical path, and
// what its HIP events measure, for the three ways to bracket one kernel:
//   ext    hipExtLaunchKernel with start / stop events (the library's way)
//   rec    hipEventRecord, hipLaunchKernel, hipEventRecord
//   plain  hipLaunchKernel alone (no timing)
// Per variant, 200 rounds of: a 100-us spin kernel (the hot kernel's stand-in,
// its duration taken by clock64 inside), the variant's launch of it, a tiny
// follower kernel, hipStreamSynchronize; reported: the host time of the
// launch call(s), the round's wall time, the event time against the kernel's
// own s_memrealtime span.
//   hipcc --offload-arch=gfx950 -O3 -o tools/launch_probe tools/launch_probe.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            printf("%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));           \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

// every workgroup spins ~us microseconds of s_memrealtime (100 MHz); the
// first and last stamps of the grid are kept (atomic min / max on vector memory)
__global__ void k_spin(unsigned us, unsigned long long* span) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)us * 100) {
    }
    if (threadIdx.x == 0) {
        atomicMin(&span[0], t0);
        atomicMax(&span[1], __builtin_amdgcn_s_memrealtime());
    }
}
__global__ void k_tiny(int* sink) {
    if (threadIdx.x == 0 && blockIdx.x == 0) sink[0] += 1;
}

int main() {
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    unsigned long long* span;
    int* sink;
    CHECK(hipMalloc(&span, 16));
    CHECK(hipMalloc(&sink, 4));
    hipEvent_t e0, e1;
    CHECK(hipEventCreateWithFlags(&e0, hipEventDisableSystemFence));
    CHECK(hipEventCreateWithFlags(&e1, hipEventDisableSystemFence));
    const unsigned us = 100, grid = 256, block = 1024;
    const char* names[3] = {"ext", "rec", "plain"};
    printf("# launch_probe: %u-us spin kernel, %u x %u; medians of 200 rounds (us)\n", us, grid, block);
    printf("%-6s %12s %12s %12s %12s\n", "way", "launch_host", "round_wall", "event_ms*1e3", "kernel_span");
    for (int v = 0; v < 3; v++) {
        std::vector<double> lh, rw, ev, ks;
        for (int r = 0; r < 220; r++) {
            const unsigned long long init[2] = {~0ull, 0ull};
            CHECK(hipMemcpyAsync(span, init, 16, hipMemcpyHostToDevice, s));
            CHECK(hipStreamSynchronize(s));
            const auto t0 = std::chrono::steady_clock::now();
            void* args[] = {(void*)&us, (void*)&span};
            if (v == 0) {
                CHECK(hipExtLaunchKernel((const void*)k_spin, dim3(grid), dim3(block), args, 0, s, e0, e1, 0));
            } else if (v == 1) {
                CHECK(hipEventRecord(e0, s));
                CHECK(hipLaunchKernel((const void*)k_spin, dim3(grid), dim3(block), args, 0, s));
                CHECK(hipEventRecord(e1, s));
            } else {
                CHECK(hipLaunchKernel((const void*)k_spin, dim3(grid), dim3(block), args, 0, s));
            }
            const auto t1 = std::chrono::steady_clock::now();
            k_tiny<<<1, 64, 0, s>>>(sink);
            CHECK(hipStreamSynchronize(s));
            const auto t2 = std::chrono::steady_clock::now();
            unsigned long long h[2];
            CHECK(hipMemcpy(h, span, 16, hipMemcpyDeviceToHost));
            float ms = 0;
            if (v < 2) CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (r < 20) continue;  // (warm-up)
            lh.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
            rw.push_back(std::chrono::duration<double, std::micro>(t2 - t0).count());
            ev.push_back(ms * 1e3);
            ks.push_back((h[1] - h[0]) / 100.0);
        }
        auto med = [](std::vector<double> x) { std::sort(x.begin(), x.end()); return x[x.size() / 2]; };
        printf("%-6s %12.2f %12.2f %12.2f %12.2f\n", names[v], med(lh), med(rw), med(ev), med(ks));
    }
    return 0;
}
