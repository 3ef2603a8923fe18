// calib_fetch -- FETCH_SIZE calibration for k_parse_agg's access pattern
// (MI355X_MICROARCH.md, HBM section: "other access widths are uncalibrated:
// calibrate on a known byte count in your own access pattern").
//
// Reads the same 800,000,000 bytes (C2: 10M records of 80 B after a 24-B pcap
// file header) twice per launch pair:
//   k_window  lane per record, five unaligned 16-byte loads (k_parse_agg's
//             load_win pattern, 80-byte stride, 8-byte aligned)
//   k_stream  aligned 16 B/lane streaming read (the guide's calibrated case)
// Run under `rocprofv3 --pmc FETCH_SIZE` (and separately TCC_EA0_RDREQ_sum);
// bytes/FETCH_SIZE of each kernel gives that pattern's correction factor.
//   hipcc --offload-arch=gfx950 -O3 -o tools/calib_fetch tools/calib_fetch.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#define CHECK(x)                                                               \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            return 1;                                                          \
        }                                                                      \
    } while (0)

constexpr uint64_t N_REC = 10000000, REC = 80, HDR = 24;

__global__ void __launch_bounds__(1024) k_window(const uint8_t* buf, uint32_t* sink) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N_REC; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint8_t* p = buf + HDR + i * REC;
#pragma unroll
        for (int c = 0; c < 5; c++) {
            uint4 v;
            __builtin_memcpy(&v, p + 16 * c, 16);
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;  // keeps the loads; never true for the fill below
}

__global__ void __launch_bounds__(1024) k_stream(const uint4* buf, uint64_t n16, uint32_t* sink) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 v = buf[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

__global__ void k_fill(uint32_t* w, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        w[i] = (uint32_t)(i * 2654435761u) | 1u;
}

int main() {
    const uint64_t bytes = HDR + N_REC * REC + 256;
    uint8_t* buf = nullptr;
    uint32_t* sink = nullptr;
    CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMalloc(&sink, 64));
    k_fill<<<4096, 256>>>((uint32_t*)buf, bytes / 4);
    CHECK(hipDeviceSynchronize());
    int n_cu = 256;
    hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int rep = 0; rep < 5; rep++) {
        float ms_w = 0, ms_s = 0;
        CHECK(hipEventRecord(e0));
        k_window<<<n_cu, 1024>>>(buf, sink);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms_w, e0, e1));
        CHECK(hipEventRecord(e0));
        k_stream<<<n_cu * 4, 1024>>>((const uint4*)(buf + 32), N_REC * REC / 16, sink);  // 16-B aligned, same size
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms_s, e0, e1));
        printf("rep %d window %.4f ms (%.1f GB/s)  stream %.4f ms (%.1f GB/s)\n", rep, ms_w, N_REC * REC / (ms_w * 1e6),
               ms_s, N_REC * REC / (ms_s * 1e6));
    }
    printf("bytes read per launch: %llu\n", (unsigned long long)(N_REC * REC));
    CHECK(hipFree(buf));
    CHECK(hipFree(sink));
    return 0;
}
