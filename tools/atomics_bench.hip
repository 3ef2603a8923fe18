// atomics_bench -- VERDICT r5 #3: the cost of aggregating the IMIX capture's
// packets straight into a per-flow accumulator table with device-scope
// atomics (instead of k_parse_spill's 32-B owner records + k_merge_spill),
// measured, not estimated.
//
// Workload (C3 / C4 shapes): 10M packets, flow of packet i uniform over F flows
// (F = 100k: C3, 1M: C4), a packet's update_flow fields as in flows.rs:11-42:
//   A  add64 (bytes << 32 | 1) per direction        -- every packet
//   L  max64 last index                             -- every packet (capture order)
//   F  min64 first index, min/max pkt / ttl          -- guarded (read, atomic only
//                                                      when the packet moves it)
// Variants (one 1024-thread workgroup per CU, grid-stride; HIP events):
//   stream   the capture read alone (80 B a packet, 16-B nt loads): the floor
//   atom     the atomics alone (no capture read)
//   both     capture read + atomics in one kernel (what direct accumulation is)
//   spill    capture read + one 32-B record per packet written to its owner's
//            region (k_parse_spill's store traffic, without its LDS binning)
//   hipcc --offload-arch=gfx950 -O3 -o tools/atomics_bench tools/atomics_bench.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

#define CHECK(x)                                                                                     \
    do {                                                                                             \
        hipError_t e_ = (x);                                                                         \
        if (e_ != hipSuccess) {                                                                      \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));        \
            exit(1);                                                                                 \
        }                                                                                            \
    } while (0)

constexpr uint64_t N = 10000000, REC = 80;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t mix32(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return (uint32_t)x;
}

struct Tab {
    unsigned long long* pb[2];  // (bytes << 32) | packets per direction
    unsigned long long *first, *last;
    uint32_t *mn, *mx;          // (pkt << 8 | ttl) min / max
    uint32_t F;
};

template <int MODE>  // 0 stream, 1 atom, 2 both, 3 spill
__global__ void __launch_bounds__(1024) k_bench(const uint8_t* cap, Tab T, uint4* spill, uint32_t* sink) {
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N; i += stride) {
        uint32_t w0 = 0, w1 = 0;
        if (MODE != 1) {  // the packet's 80-B window (five 16-B nontemporal loads)
            const u32x4* p = reinterpret_cast<const u32x4*>(cap + i * REC);
#pragma unroll
            for (int k = 0; k < 5; k++) {
                const u32x4 v = __builtin_nontemporal_load(p + k);
                acc ^= v.x ^ v.y ^ v.z ^ v.w;
                if (k == 2) { w0 = v.x; w1 = v.y; }
            }
        }
        const uint32_t h = mix32(i * 0x9E3779B97F4A7C15ull + 7);
        const uint32_t f = (uint32_t)(((uint64_t)h * T.F) >> 32);
        const uint32_t dir = (h >> 7) & 1u, pkt = 64u + ((h >> 9) & 1023u) + (w0 & 1u), ttl = 32u + ((h >> 20) & 31u) + (w1 & 1u);
        if (MODE == 1 || MODE == 2) {
            atomicAdd(&T.pb[dir][f], ((unsigned long long)pkt << 32) | 1ull);
            atomicMax(&T.last[f], (unsigned long long)i + 1);
            const uint32_t mm = (pkt << 8) | ttl;
            if (i < T.first[f]) atomicMin(&T.first[f], (unsigned long long)i);
            if (mm < T.mn[f]) atomicMin(&T.mn[f], mm);
            if (mm > T.mx[f]) atomicMax(&T.mx[f], mm);
        }
        if (MODE == 3) {  // one 32-B record into the flow owner's region (256 owners)
            const uint32_t o = h >> 24;
            const uint64_t slot = ((uint64_t)o * (N / 256 + 4096)) + (i % (N / 256 + 4096));
            spill[2 * slot] = make_uint4(f, i, pkt, ttl);
            spill[2 * slot + 1] = make_uint4(dir, acc, 0, 0);
        }
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

int main() {
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const unsigned grid = prop.multiProcessorCount;
    uint8_t* cap;
    CHECK(hipMalloc(&cap, N * REC + 256));
    CHECK(hipMemset(cap, 0x5A, N * REC + 256));
    uint4* spill;
    const uint64_t spill_slots = 256ull * (N / 256 + 4096);
    CHECK(hipMalloc(&spill, spill_slots * 32));
    uint32_t* sink;
    CHECK(hipMalloc(&sink, 64));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    printf("# atomics_bench: %llu packets, %u workgroups x 1024, 80 B/packet read; ms per launch (median of 7)\n",
           (unsigned long long)N, grid);
    printf("%-8s %-8s %10s %12s\n", "flows", "variant", "ms", "Gpackets/s");
    const uint32_t flows[2] = {100000, 1000000};
    for (uint32_t F : flows) {
        Tab T{};
        T.F = F;
        CHECK(hipMalloc(&T.pb[0], F * 8ull));
        CHECK(hipMalloc(&T.pb[1], F * 8ull));
        CHECK(hipMalloc(&T.first, F * 8ull));
        CHECK(hipMalloc(&T.last, F * 8ull));
        CHECK(hipMalloc(&T.mn, F * 4ull));
        CHECK(hipMalloc(&T.mx, F * 4ull));
        const char* names[4] = {"stream", "atom", "both", "spill"};
        for (int m = 0; m < 4; m++) {
            std::vector<float> ts;
            for (int rep = 0; rep < 8; rep++) {
                CHECK(hipMemset(T.pb[0], 0, F * 8ull));
                CHECK(hipMemset(T.pb[1], 0, F * 8ull));
                CHECK(hipMemset(T.first, 0xFF, F * 8ull));
                CHECK(hipMemset(T.last, 0, F * 8ull));
                CHECK(hipMemset(T.mn, 0xFF, F * 4ull));
                CHECK(hipMemset(T.mx, 0, F * 4ull));
                CHECK(hipDeviceSynchronize());
                CHECK(hipEventRecord(e0, 0));
                switch (m) {
                case 0: k_bench<0><<<grid, 1024>>>(cap, T, spill, sink); break;
                case 1: k_bench<1><<<grid, 1024>>>(cap, T, spill, sink); break;
                case 2: k_bench<2><<<grid, 1024>>>(cap, T, spill, sink); break;
                default: k_bench<3><<<grid, 1024>>>(cap, T, spill, sink); break;
                }
                CHECK(hipEventRecord(e1, 0));
                CHECK(hipEventSynchronize(e1));
                float ms = 0;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                if (rep) ts.push_back(ms);  // (the first launch warms up)
            }
            std::sort(ts.begin(), ts.end());
            const float med = ts[ts.size() / 2];
            printf("%-8u %-8s %10.4f %12.2f\n", F, names[m], med, N / (med * 1e-3) / 1e9);
            if (m == 2) {  // check: the last 'both' launch counted every packet once
                std::vector<unsigned long long> a(F), b(F);
                CHECK(hipMemcpy(a.data(), T.pb[0], F * 8ull, hipMemcpyDeviceToHost));
                CHECK(hipMemcpy(b.data(), T.pb[1], F * 8ull, hipMemcpyDeviceToHost));
                unsigned long long tot = 0;
                for (uint32_t f = 0; f < F; f++) tot += (a[f] & 0xFFFFFFFFull) + (b[f] & 0xFFFFFFFFull);
                printf("# F=%u: packets counted by 'both': %llu (expect %llu)\n", F, tot, (unsigned long long)N);
            }
        }
        (void)hipFree(T.pb[0]); (void)hipFree(T.pb[1]); (void)hipFree(T.first);
        (void)hipFree(T.last); (void)hipFree(T.mn); (void)hipFree(T.mx);
    }
    return 0;
}
