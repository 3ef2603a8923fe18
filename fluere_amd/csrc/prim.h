// prim.h -- the device-wide primitives the library takes from rocPRIM, called
// directly (no hipCUB layer): exclusive / inclusive sums, inclusive min / max
// scans, and the radix sort of key-value pairs.  Each follows the library's
// two-call protocol (tmp == nullptr: the temp size in tb, nothing launched).
// The hot path's own scans are hand-written (exact.hip flag counts and tile
// scans, order.hip's k_so_*); these serve the rarer and the sort-bound phases.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstring>

#include <rocprim/rocprim.hpp>

namespace fl {

template <class T>
inline hipError_t prim_exclusive_sum(void* tmp, size_t& tb, const T* in, T* out, size_t n, hipStream_t s) {
    return rocprim::exclusive_scan(tmp, tb, in, out, T(0), n, rocprim::plus<T>(), s);
}
template <class T>
inline hipError_t prim_inclusive_sum(void* tmp, size_t& tb, const T* in, T* out, size_t n, hipStream_t s) {
    return rocprim::inclusive_scan(tmp, tb, in, out, n, rocprim::plus<T>(), s);
}
template <class T>
inline hipError_t prim_inclusive_min(void* tmp, size_t& tb, const T* in, T* out, size_t n, hipStream_t s) {
    return rocprim::inclusive_scan(tmp, tb, in, out, n, rocprim::minimum<T>(), s);
}
template <class T>
inline hipError_t prim_inclusive_max(void* tmp, size_t& tb, const T* in, T* out, size_t n, hipStream_t s) {
    return rocprim::inclusive_scan(tmp, tb, in, out, n, rocprim::maximum<T>(), s);
}
// stable LSD radix sort of (key, value) pairs over key bits [b0, b1)
template <class K, class V>
inline hipError_t prim_sort_pairs(void* tmp, size_t& tb, const K* kin, K* kout, const V* vin, V* vout, size_t n,
                                  unsigned b0, unsigned b1, hipStream_t s) {
    return rocprim::radix_sort_pairs(tmp, tb, kin, kout, vin, vout, n, b0, b1, s);
}

}  // namespace fl
