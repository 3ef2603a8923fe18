// pattern_bench -- HBM read ceilings of the access patterns the hot kernel can
// use on C2 (10M pcap records of 80 B after a 24-B file header, u32 offsets).
//   V0 stream   aligned 16 B/lane streaming read of the record bytes (ceiling)
//   V1 window   lane per record: five unaligned 16-B loads (k_parse_agg today)
//   V2 win+offs V1 plus the u32 offset load per record
//   V3 stage    wave per 64 records: offsets, coalesced 16-B loads of the
//               wave's byte span into a wave-private LDS slab (register staged,
//               one chunk in flight), then lane windows read back from LDS
//   V4 glds     V3 with global_load_lds_dwordx4 (LDS-DMA), two slabs per wave
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/pattern_bench tools/pattern_bench.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                       \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

constexpr uint64_t N_REC = 10000000, REC = 80, HDR = 24;
constexpr int SLAB = 6144;  // bytes per wave slab: 64 records of 80 B + alignment slack

__global__ void __launch_bounds__(1024) k_stream(const uint4* buf, uint64_t n16, uint32_t* sink) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 v = buf[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

template <bool OFFS>
__global__ void __launch_bounds__(1024) k_window(const uint8_t* buf, const uint32_t* offs, uint32_t* sink) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N_REC; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint8_t* p = buf + (OFFS ? offs[i] : HDR + i * REC);
#pragma unroll
        for (int c = 0; c < 5; c++) {
            uint4 v;
            __builtin_memcpy(&v, p + 16 * c, 16);
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

// wave-per-64-records, register-staged into a wave-private LDS slab
__global__ void __launch_bounds__(1024) k_stage(const uint8_t* buf, const uint32_t* offs, uint32_t* sink) {
    __shared__ uint4 slab[16][SLAB / 16];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nchunk = (N_REC + 63) / 64;
    const uint64_t wstride = (uint64_t)gridDim.x * 16;
    uint32_t acc = 0;
    uint64_t ch = (uint64_t)blockIdx.x * 16 + wv;
    uint4* my = slab[wv];
    for (; ch < nchunk; ch += wstride) {
        const uint64_t i = ch * 64 + lane;
        const uint32_t o = offs[min(i, N_REC - 1)];
        const uint32_t o0 = __builtin_amdgcn_readfirstlane(o);
        const uint32_t base = o0 & ~15u;
        const uint4* g = reinterpret_cast<const uint4*>(buf + base);
        uint4 v[6];
#pragma unroll
        for (int c = 0; c < 6; c++) v[c] = g[c * 64 + lane];
#pragma unroll
        for (int c = 0; c < 6; c++) my[c * 64 + lane] = v[c];
        __builtin_amdgcn_wave_barrier();
        const uint32_t rel = o - base;  // 8-aligned for C2
        const uint2* s = reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(my) + rel);
#pragma unroll
        for (int c = 0; c < 10; c++) {
            const uint2 x = s[c];
            acc ^= x.x ^ x.y;
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

// same with LDS-DMA (global_load_lds_dwordx4), two slabs per wave: the slab of
// chunk i+1 is in flight while chunk i is read
__global__ void __launch_bounds__(512) k_glds(const uint8_t* buf, const uint32_t* offs, uint32_t* sink) {
    __shared__ uint4 slab[8][2][SLAB / 16];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nchunk = (N_REC + 63) / 64;
    const uint64_t wstride = (uint64_t)gridDim.x * 8;
    uint32_t acc = 0;
    uint64_t ch = (uint64_t)blockIdx.x * 8 + wv;
    auto issue = [&](uint64_t c, int b, uint32_t& o) {
        const uint64_t i = c * 64 + lane;
        o = offs[min(i, N_REC - 1)];
        const uint32_t base = __builtin_amdgcn_readfirstlane(o) & ~15u;
        const uint8_t* g = buf + base;
#pragma unroll
        for (int k = 0; k < 6; k++)
            __builtin_amdgcn_global_load_lds(g + (k * 64 + lane) * 16, &slab[wv][b][k * 64], 16, 0, 0);
        o -= base;
    };
    uint32_t oc = 0, on = 0;
    int b = 0;
    if (ch < nchunk) issue(ch, 0, oc);
    for (; ch < nchunk; ch += wstride) {
        const bool more = ch + wstride < nchunk;
        if (more) {
            issue(ch + wstride, b ^ 1, on);
            asm volatile("s_waitcnt vmcnt(7)" ::: "memory");  // chunk ch landed (6 glds + 1 offset load of the next in flight)
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        const uint2* s = reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(&slab[wv][b][0]) + oc);
#pragma unroll
        for (int c = 0; c < 10; c++) {
            const uint2 x = s[c];
            acc ^= x.x ^ x.y;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        oc = on;
        b ^= 1;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}


// per-packet stand-in for the parse / key / table work: WORK dependent VALU pairs
template <int WORK>
__device__ __forceinline__ uint32_t work(uint32_t x) {
    uint32_t a = x;
#pragma unroll 4
    for (int k = 0; k < WORK; k++) a = a * 0x9E3779B1u + (x ^ (uint32_t)k);
    return a;
}

// V1 + offsets + WORK, grid-stride, compiler-scheduled loads (no explicit prefetch)
template <int WORK>
__global__ void __launch_bounds__(1024) k_window_work(const uint8_t* buf, const uint32_t* offs, uint32_t* sink) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N_REC; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint8_t* p = buf + offs[i];
        uint32_t x = 0;
#pragma unroll
        for (int c = 0; c < 5; c++) {
            uint4 v;
            __builtin_memcpy(&v, p + 16 * c, 16);
            x ^= v.x ^ v.y ^ v.z ^ v.w;
        }
        acc += work<WORK>(x);
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

// V5: wave per 64 records; offsets and the four 16-B pieces of each record
// window ([0,16) [28,44) [44,60) [60,76)) arrive by LDS-DMA (inline asm,
// invisible to the compiler's waitcnt bookkeeping); one chunk in flight per
// wave while the previous one is processed from VGPRs.
__device__ __forceinline__ void glds16(const void* g, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"((uint64_t)g), "s"(lds) : "memory");
}
__device__ __forceinline__ void glds4(const void* g, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"((uint64_t)g), "s"(lds) : "memory");
}
template <int NW, int WORK>
__global__ void __launch_bounds__(NW * 64) k_gather(const uint8_t* buf, const uint32_t* offs, uint32_t* sink) {
    __shared__ uint4 slab[NW][4][64];
    __shared__ uint32_t soff[NW][2][64];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nchunk = (N_REC + 63) / 64;
    const uint64_t wstride = (uint64_t)gridDim.x * NW;
    uint64_t ch = (uint64_t)blockIdx.x * NW + wv;
    const uint32_t slab_lds = (uint32_t)(uintptr_t)&slab[wv][0][0];
    const uint32_t off_lds0 = (uint32_t)(uintptr_t)&soff[wv][0][0];
    auto off_issue = [&](uint64_t c, int r) {
        glds4(offs + min(c * 64 + lane, N_REC - 1), off_lds0 + r * 256);
    };
    auto win_issue = [&](uint32_t o) {
        const uint8_t* p = buf + o;
        glds16(p, slab_lds);
        glds16(p + 28, slab_lds + 1024);
        glds16(p + 44, slab_lds + 2048);
        glds16(p + 60, slab_lds + 3072);
    };
    uint32_t acc = 0;
    if (ch < nchunk) {
        off_issue(ch, 0);
        off_issue(ch + wstride, 1);
        asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
        win_issue(soff[wv][0][lane]);
    }
    int r = 0;  // ring slot holding the offsets of chunk ch + wstride
    r = 1;
    for (; ch < nchunk; ch += wstride) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        uint4 w0 = slab[wv][0][lane], w1 = slab[wv][1][lane], w2 = slab[wv][2][lane], w3 = slab[wv][3][lane];
        const uint32_t onext = soff[wv][r][lane];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (ch + wstride < nchunk) {
            off_issue(ch + 2 * wstride, r ^ 1);
            win_issue(onext);
        }
        r ^= 1;
        uint32_t x = w0.x ^ w0.y ^ w0.z ^ w0.w ^ w1.x ^ w1.y ^ w1.z ^ w1.w ^ w2.x ^ w2.y ^ w2.z ^ w2.w ^ w3.x ^ w3.y ^
                     w3.z ^ w3.w;
        acc += work<WORK>(x);
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

// V6: the hot kernel's packet order: each workgroup owns a contiguous range of
// records and walks it in steps of blockDim.x (offset of the next step prefetched)
template <int WORK>
__global__ void __launch_bounds__(1024) k_contig(const uint8_t* buf, const uint32_t* offs, uint32_t* sink) {
    const uint64_t per = (N_REC + gridDim.x - 1) / gridDim.x;
    const uint64_t beg = per * blockIdx.x, end = min(N_REC, beg + per);
    uint32_t acc = 0;
    uint64_t li = beg + threadIdx.x;
    uint32_t o = offs[min(li, N_REC - 1)];
    for (; li < end + 1023; li += 1024) {
        const uint32_t on = offs[min(li + 1024, N_REC - 1)];
        const uint8_t* p = buf + o;
        uint32_t x = 0;
#pragma unroll
        for (int c = 0; c < 5; c++) {
            uint4 v;
            __builtin_memcpy(&v, p + 16 * c, 16);
            x ^= v.x ^ v.y ^ v.z ^ v.w;
        }
        if (li < end) acc += work<WORK>(x);
        o = on;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}
// V7: grid-stride in steps: step s of workgroup b covers records
// [(s * gridDim.x + b) * 1024, +1024)  (all workgroups stream one region together)
template <int WORK>
__global__ void __launch_bounds__(1024) k_interleave(const uint8_t* buf, const uint32_t* offs, uint32_t* sink) {
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 1024;
    uint64_t li = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
    uint32_t o = offs[min(li, N_REC - 1)];
    for (; li < N_REC + 1023; li += stride) {
        const uint32_t on = offs[min(li + stride, N_REC - 1)];
        const uint8_t* p = buf + o;
        uint32_t x = 0;
#pragma unroll
        for (int c = 0; c < 5; c++) {
            uint4 v;
            __builtin_memcpy(&v, p + 16 * c, 16);
            x ^= v.x ^ v.y ^ v.z ^ v.w;
        }
        if (li < N_REC) acc += work<WORK>(x);
        o = on;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}


// nontemporal variants (global_load ... nt): V0nt streaming ceiling, V1nt lane windows
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(1024) k_stream_nt(const u32x4_t* buf, uint64_t n16, uint32_t* sink) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        const u32x4_t v = __builtin_nontemporal_load(buf + i);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}
// V8: wave per 64 dense records (C2: stride 80, no offsets): five coalesced
// 1-KiB nt loads, staged through a wave-private LDS slab, lane windows read back
template <bool NT, int INFL>
__global__ void __launch_bounds__(1024) k_dense(const uint8_t* buf, uint32_t* sink) {
    __shared__ uint4 slab[16][320];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nchunk = (N_REC + 63) / 64;
    const uint64_t wstride = (uint64_t)gridDim.x * 16;
    uint32_t acc = 0;
    for (uint64_t ch = (uint64_t)blockIdx.x * 16 + wv; ch < nchunk; ch += wstride * INFL) {
        u32x4_t v[INFL][5];
#pragma unroll
        for (int j = 0; j < INFL; j++) {
            const uint64_t cj = min(ch + j * wstride, nchunk - 1);
            const u32x4_t* g = reinterpret_cast<const u32x4_t*>(buf + HDR + cj * 64 * REC);
#pragma unroll
            for (int c = 0; c < 5; c++) v[j][c] = NT ? __builtin_nontemporal_load(g + c * 64 + lane) : g[c * 64 + lane];
        }
#pragma unroll
        for (int j = 0; j < INFL; j++) {
#pragma unroll
            for (int c = 0; c < 5; c++) slab[wv][c * 64 + lane] = make_uint4(v[j][c].x, v[j][c].y, v[j][c].z, v[j][c].w);
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int c = 0; c < 5; c++) {
                const uint4 x = slab[wv][lane * 5 + c];
                acc ^= x.x ^ x.y ^ x.z ^ x.w;
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

// V9: lane windows (V1/V2) with nontemporal loads; OFFS: offsets read per record
template <bool OFFS>
__global__ void __launch_bounds__(1024) k_window_nt(const uint8_t* buf, const uint32_t* offs, uint32_t* sink) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N_REC; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint8_t* p = buf + (OFFS ? __builtin_nontemporal_load(offs + i) : HDR + i * REC);
#pragma unroll
        for (int c = 0; c < 5; c++) {
            u32x4_t v;
            // 8-byte aligned record starts: two 8-B nt loads per 16 B
            typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
            const u32x2_t a0 = __builtin_nontemporal_load(reinterpret_cast<const u32x2_t*>(p + 16 * c));
            const u32x2_t a1 = __builtin_nontemporal_load(reinterpret_cast<const u32x2_t*>(p + 16 * c + 8));
            v.x = a0.x; v.y = a0.y; v.z = a1.x; v.w = a1.y;
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}
// V10: lane windows, nt 16-B loads via inline asm (unaligned dwordx4 is legal on gfx950)
__device__ __forceinline__ uint4 ld_nt16(const void* p) {
    uint4 v;
    asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(v) : "v"(p) : "memory");
    return v;
}
template <bool OFFS>
__global__ void __launch_bounds__(1024) k_window_nta(const uint8_t* buf, const uint32_t* offs, uint32_t* sink) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N_REC; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint8_t* p = buf + (OFFS ? offs[i] : HDR + i * REC);
        uint4 v[5];
#pragma unroll
        for (int c = 0; c < 5; c++) v[c] = ld_nt16(p + 16 * c);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int c = 0; c < 5; c++) acc ^= v[c].x ^ v[c].y ^ v[c].z ^ v[c].w;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

// V11: the hot kernel's intended front end: NW waves per CU, wave per 64 dense
// records, six coalesced 16-B nt loads per lane (5136-B span incl. the 8-B
// misalignment of pcap records), the next chunk's loads in flight while the
// current chunk is transposed through a wave-private LDS slab and processed
template <int NW, int WORK>
__global__ void __launch_bounds__(NW * 64) k_dense2(const uint8_t* buf, uint32_t* sink) {
    __shared__ uint4 slab[NW][321];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nchunk = N_REC / 64;
    const uint64_t wstride = (uint64_t)gridDim.x * NW;
    uint32_t acc = 0;
    uint64_t ch = (uint64_t)blockIdx.x * NW + wv;
    u32x4_t v[6];
    auto issue = [&](uint64_t c) {
        const uint64_t off = HDR + min(c, nchunk - 1) * 64 * REC;
        const u32x4_t* g = reinterpret_cast<const u32x4_t*>(buf + (off & ~15ull));
#pragma unroll
        for (int k = 0; k < 5; k++) v[k] = __builtin_nontemporal_load(g + k * 64 + lane);
        if (lane == 0) v[5] = __builtin_nontemporal_load(g + 320);
    };
    issue(ch);
    for (; ch < nchunk; ch += wstride) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int k = 0; k < 5; k++) slab[wv][k * 64 + lane] = make_uint4(v[k].x, v[k].y, v[k].z, v[k].w);
        if (lane == 0) slab[wv][320] = make_uint4(v[5].x, v[5].y, v[5].z, v[5].w);
        __builtin_amdgcn_wave_barrier();
        const uint32_t rel = (uint32_t)((HDR + ch * 64 * REC) & 15) + lane * REC;
        const uint2* sp = reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(&slab[wv][0]) + rel);
        uint32_t w[20];
#pragma unroll
        for (int c = 0; c < 10; c++) { const uint2 x = sp[c]; w[2 * c] = x.x; w[2 * c + 1] = x.y; }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        issue(ch + wstride);
        uint32_t x = 0;
#pragma unroll
        for (int c = 0; c < 20; c++) x ^= w[c];
        acc += work<WORK>(x);
        __builtin_amdgcn_wave_barrier();
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

__global__ void k_fill(uint32_t* w, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        w[i] = (uint32_t)(i * 2654435761u) | 1u;
}
__global__ void k_offs(uint32_t* o, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        o[i] = (uint32_t)(HDR + i * REC);
}

int main() {
    const uint64_t bytes = HDR + N_REC * REC + 8192;
    uint8_t* buf = nullptr;
    uint32_t *sink = nullptr, *offs = nullptr;
    CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMalloc(&offs, N_REC * 4));
    CHECK(hipMalloc(&sink, 64));
    k_fill<<<4096, 256>>>((uint32_t*)buf, bytes / 4);
    k_offs<<<4096, 256>>>(offs, N_REC);
    CHECK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const double alg = (double)N_REC * REC;
    auto run = [&](const char* name, auto launch) {
        float best = 1e9;
        for (int rep = 0; rep < 8; rep++) {
            float ms = 0;
            CHECK(hipEventRecord(e0));
            launch();
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            CHECK(hipGetLastError());
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (rep >= 2 && ms < best) best = ms;
        }
        printf("%-28s %.4f ms  %7.1f GB/s of the 800 MB record bytes\n", name, best, alg / (best * 1e6));
    };
    for (int g : {256, 512, 1024, 2048}) {
        char nm[64];
        snprintf(nm, sizeof nm, "V0 stream g=%d", g);
        run(nm, [&] { k_stream<<<g, 1024>>>((const uint4*)(buf + 32), N_REC * REC / 16, sink); });
    }
    for (int g : {256, 512}) {
        char nm[64];
        snprintf(nm, sizeof nm, "V1 window g=%d", g);
        run(nm, [&] { k_window<false><<<g, 1024>>>(buf, offs, sink); });
        snprintf(nm, sizeof nm, "V2 window+offs g=%d", g);
        run(nm, [&] { k_window<true><<<g, 1024>>>(buf, offs, sink); });
        snprintf(nm, sizeof nm, "V3 stage g=%d", g);
        run(nm, [&] { k_stage<<<g, 1024>>>(buf, offs, sink); });
    }
    for (int g : {256, 512, 1024}) {
        char nm[64];
        snprintf(nm, sizeof nm, "V4 glds g=%d", g);
        run(nm, [&] { k_glds<<<g, 512>>>(buf, offs, sink); });
    }
    for (int g : {256}) {
        char nm[64];
        snprintf(nm, sizeof nm, "V6 contig w0 g=%d", g);
        run(nm, [&] { k_contig<0><<<g, 1024>>>(buf, offs, sink); });
        snprintf(nm, sizeof nm, "V6 contig w64 g=%d", g);
        run(nm, [&] { k_contig<64><<<g, 1024>>>(buf, offs, sink); });
        snprintf(nm, sizeof nm, "V7 interleave w0 g=%d", g);
        run(nm, [&] { k_interleave<0><<<g, 1024>>>(buf, offs, sink); });
        snprintf(nm, sizeof nm, "V7 interleave w64 g=%d", g);
        run(nm, [&] { k_interleave<64><<<g, 1024>>>(buf, offs, sink); });
        snprintf(nm, sizeof nm, "V2w0 g=%d", g);
        run(nm, [&] { k_window_work<0><<<g, 1024>>>(buf, offs, sink); });
        snprintf(nm, sizeof nm, "V2w64 g=%d", g);
        run(nm, [&] { k_window_work<64><<<g, 1024>>>(buf, offs, sink); });
    }
    for (int g : {256, 512, 1024, 2048}) {
        char nm[64];
        snprintf(nm, sizeof nm, "V0nt stream g=%d", g);
        run(nm, [&] { k_stream_nt<<<g, 1024>>>((const u32x4_t*)(buf + 32), N_REC * REC / 16, sink); });
    }
    for (int g : {256}) {
        char nm[64];
        snprintf(nm, sizeof nm, "V8 dense g=%d", g);
        run(nm, [&] { k_dense<false, 1><<<g, 1024>>>(buf, sink); });
        snprintf(nm, sizeof nm, "V8 dense nt g=%d", g);
        run(nm, [&] { k_dense<true, 1><<<g, 1024>>>(buf, sink); });
        snprintf(nm, sizeof nm, "V8 dense nt x2 g=%d", g);
        run(nm, [&] { k_dense<true, 2><<<g, 1024>>>(buf, sink); });
    }
    for (int g : {256, 512}) {
        char nm[64];
        snprintf(nm, sizeof nm, "V9 window nt8 g=%d", g);
        run(nm, [&] { k_window_nt<false><<<g, 1024>>>(buf, offs, sink); });
        snprintf(nm, sizeof nm, "V9 window+offs nt8 g=%d", g);
        run(nm, [&] { k_window_nt<true><<<g, 1024>>>(buf, offs, sink); });
        snprintf(nm, sizeof nm, "V10 window nt16 g=%d", g);
        run(nm, [&] { k_window_nta<false><<<g, 1024>>>(buf, offs, sink); });
        snprintf(nm, sizeof nm, "V10 window+offs nt16 g=%d", g);
        run(nm, [&] { k_window_nta<true><<<g, 1024>>>(buf, offs, sink); });
    }
    for (int g : {256}) {
        char nm[64];
        snprintf(nm, sizeof nm, "V11 dense2 nw8 w0 g=%d", g);
        run(nm, [&] { k_dense2<8, 0><<<g, 512>>>(buf, sink); });
        snprintf(nm, sizeof nm, "V11 dense2 nw8 w64 g=%d", g);
        run(nm, [&] { k_dense2<8, 64><<<g, 512>>>(buf, sink); });
        snprintf(nm, sizeof nm, "V11 dense2 nw8 w128 g=%d", g);
        run(nm, [&] { k_dense2<8, 128><<<g, 512>>>(buf, sink); });
        snprintf(nm, sizeof nm, "V11 dense2 nw16 w0 g=%d", g);
        run(nm, [&] { k_dense2<16, 0><<<g, 1024>>>(buf, sink); });
        snprintf(nm, sizeof nm, "V11 dense2 nw16 w64 g=%d", g);
        run(nm, [&] { k_dense2<16, 64><<<g, 1024>>>(buf, sink); });
        snprintf(nm, sizeof nm, "V11 dense2 nw16 w128 g=%d", g);
        run(nm, [&] { k_dense2<16, 128><<<g, 1024>>>(buf, sink); });
        snprintf(nm, sizeof nm, "V11 dense2 nw4 w0 g=%d", g);
        run(nm, [&] { k_dense2<4, 0><<<g, 256>>>(buf, sink); });
    }
    return 0;
}
