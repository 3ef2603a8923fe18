// Host -> HBM copy rate from staging chunks, by allocation kind (diagnostics
// for the file ingest):
//   tools/h2d_probe [MiB total] [MiB chunk]
// prints, per kind, the host time of the enqueue loop and the rate to completion.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char** argv) {
    const size_t total = (argc > 1 ? atol(argv[1]) : 2048) << 20;
    const size_t chunk = (argc > 2 ? atol(argv[2]) : 32) << 20;
    void* d = nullptr;
    if (hipMalloc(&d, total) != hipSuccess) return 1;
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    struct Kind { const char* name; unsigned flags; int reg; };
    const Kind kinds[] = {{"hipHostMalloc default", hipHostMallocDefault, 0},
                          {"hipHostMalloc non-coherent", hipHostMallocNonCoherent, 0},
                          {"hipHostMalloc coherent", hipHostMallocCoherent, 0},
                          {"malloc + hipHostRegister", 0, 1}};
    const int nslot = 4;
    for (const Kind& k : kinds) {
        std::vector<void*> pin(nslot);
        for (int i = 0; i < nslot; i++) {
            if (k.reg) {
                pin[i] = aligned_alloc(4096, chunk);
                if (hipHostRegister(pin[i], chunk, hipHostRegisterDefault) != hipSuccess) { printf("register failed\n"); return 1; }
            } else if (hipHostMalloc(&pin[i], chunk, k.flags) != hipSuccess) {
                printf("%s: alloc failed\n", k.name);
                return 1;
            }
            memset(pin[i], i + 1, chunk);
        }
        for (int rep = 0; rep < 2; rep++) {
            hipStreamSynchronize(s);
            const double t0 = now();
            for (size_t off = 0, c = 0; off < total; off += chunk, c++)
                hipMemcpyAsync((char*)d + off, pin[c % nslot], chunk, hipMemcpyHostToDevice, s);
            const double t1 = now();
            hipStreamSynchronize(s);
            const double t2 = now();
            if (rep) printf("%-28s enqueue %.1f ms, done %.1f ms: %.2f GB/s\n", k.name, 1e3 * (t1 - t0), 1e3 * (t2 - t0),
                            total / (t2 - t0) / 1e9);
        }
        for (int i = 0; i < nslot; i++) {
            if (k.reg) { hipHostUnregister(pin[i]); free(pin[i]); }
            else hipHostFree(pin[i]);
        }
    }
    // one large registered region (an mmap'd file would be registered this way)
    {
        void* big = aligned_alloc(4096, total);
        memset(big, 7, total);
        const double r0 = now();
        if (hipHostRegister(big, total, hipHostRegisterDefault) != hipSuccess) { printf("big register failed\n"); return 1; }
        const double r1 = now();
        hipStreamSynchronize(s);
        const double t0 = now();
        for (size_t off = 0; off < total; off += chunk)
            hipMemcpyAsync((char*)d + off, (char*)big + off, chunk, hipMemcpyHostToDevice, s);
        hipStreamSynchronize(s);
        const double t2 = now();
        printf("%-28s register %.1f ms, copy %.1f ms: %.2f GB/s\n", "one registered region", 1e3 * (r1 - r0),
               1e3 * (t2 - t0), total / (t2 - t0) / 1e9);
        hipHostUnregister(big);
        free(big);
    }
    return 0;
}
