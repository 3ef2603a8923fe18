// graph_probe -- does hipEventRecord captured into a hipGraph give usable
// timestamps on this ROCm (event record nodes), and what does a replay of a
// five-kernel chain cost against direct launches?
//   hipcc --offload-arch=gfx950 -O3 -o tools/graph_probe tools/graph_probe.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            printf("%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));           \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

__global__ void k_spin(unsigned long long cycles, int* sink) {
    unsigned long long t0 = clock64();
    while (clock64() - t0 < cycles) {
    }
    if (threadIdx.x == 0 && blockIdx.x == 0) sink[0] += 1;
}

int main() {
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int* sink;
    CHECK(hipMalloc(&sink, 64));
    int* host;
    CHECK(hipHostMalloc((void**)&host, 64, 0));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto chain = [&](bool ev) {
        k_spin<<<256, 256, 0, s>>>(10000, sink);
        if (ev) CHECK(hipEventRecord(e0, s));
        k_spin<<<256, 1024, 0, s>>>(200000, sink);
        if (ev) CHECK(hipEventRecord(e1, s));
        k_spin<<<256, 1024, 0, s>>>(20000, sink);
        k_spin<<<256, 256, 0, s>>>(10000, sink);
        CHECK(hipMemcpyAsync(host, sink, 16, hipMemcpyDeviceToHost, s));
    };
    for (int ev = 0; ev < 2; ev++) {
        for (int w = 0; w < 3; w++) chain(ev);
        CHECK(hipStreamSynchronize(s));
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < 50; i++) {
            chain(ev);
            CHECK(hipStreamSynchronize(s));
        }
        double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / 50;
        float ms = -1;
        if (ev) CHECK(hipEventElapsedTime(&ms, e0, e1));
        printf("direct  events=%d: %.1f us per chain (+sync), middle kernel %.4f ms\n", ev, us, ms);
    }
    hipGraph_t g;
    hipGraphExec_t ge;
    // fresh events, recorded only inside the graph
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
    chain(true);
    hipError_t ec = hipStreamEndCapture(s, &g);
    printf("capture: %s\n", hipGetErrorString(ec));
    if (ec != hipSuccess) return 0;
    CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int w = 0; w < 3; w++) CHECK(hipGraphLaunch(ge, s));
    CHECK(hipStreamSynchronize(s));
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 50; i++) {
        CHECK(hipGraphLaunch(ge, s));
        CHECK(hipStreamSynchronize(s));
    }
    double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / 50;
    float ms = -1;
    hipError_t et = hipEventElapsedTime(&ms, e0, e1);
    printf("graph: %.1f us per chain (+sync), middle kernel %.4f ms (%s)\n", us, ms, hipGetErrorString(et));
    // explicit event record nodes: kernel -> rec(e2) -> kernel -> rec(e3)
    hipEvent_t e2, e3;
    CHECK(hipEventCreate(&e2));
    CHECK(hipEventCreate(&e3));
    hipGraph_t g2;
    CHECK(hipGraphCreate(&g2, 0));
    hipGraphNode_t n0, n1, n2;
    CHECK(hipGraphAddEventRecordNode(&n0, g2, nullptr, 0, e2));
    hipKernelNodeParams kp{};
    unsigned long long cyc = 200000;
    void* args[] = {&cyc, &sink};
    kp.func = (void*)k_spin;
    kp.gridDim = dim3(256);
    kp.blockDim = dim3(1024);
    kp.kernelParams = args;
    CHECK(hipGraphAddKernelNode(&n1, g2, &n0, 1, &kp));
    CHECK(hipGraphAddEventRecordNode(&n2, g2, &n1, 1, e3));
    hipGraphExec_t ge2;
    CHECK(hipGraphInstantiate(&ge2, g2, nullptr, nullptr, 0));
    CHECK(hipGraphLaunch(ge2, s));
    CHECK(hipStreamSynchronize(s));
    et = hipEventElapsedTime(&ms, e2, e3);
    printf("explicit event nodes: middle kernel %.4f ms (%s)\n", ms, hipGetErrorString(et));
    return 0;
}
