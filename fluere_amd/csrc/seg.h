// seg.h -- the packed forms of a spilled packet in an owner segment (written
// by the hot pass and k_slow, read by the owner merges).  Host-compilable so
// the CPU tests can check the round trip (tests/native/seg_roundtrip.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace fl {

// In an owner segment (dspill, runs without MACs) a spilled packet is packed
// into 24 bytes, three 8-byte words (a 4 KiB page holds 170 of them):
//   {k0, k1}, {k2, tag bits 24..31 and 0 | ttl << 16 | doct bits 16..20 << 11
//   | elig << 10 | dir << 9 | tcp flags << 1}, {pkt | doct bits 0..15 << 16, loc}
// -- the hot pass writes and the owner merge reads 25 % fewer bytes than the
// 32-byte record.  The overflow list and the raw buffers keep the 32-byte form.
constexpr uint32_t SEG_Q = 3;           // 8-byte words per packed record
constexpr uint32_t SEG_DOCT_MAX = 1u << 21;  // doct must stay below (16-bit IP lengths + 40: always)
__host__ __device__ __forceinline__ void seg_pack(const uint4& key, const uint4& pay, uint2 (&q)[SEG_Q]) {
    const uint32_t pkt = pay.y & 0xFFFFu, ttl = (pay.y >> 16) & 0xFFu, elig = (pay.y >> 24) & 1u;
    const uint32_t tf = pay.w & 0xFFu, dir = (pay.w >> 8) & 1u;
    q[0] = make_uint2(key.x, key.y);
    q[1] = make_uint2(key.z, (key.w & 0xFF000001u) | (ttl << 16) | (((pay.x >> 16) & 0x1Fu) << 11) | (elig << 10) |
                                 (dir << 9) | (tf << 1));
    q[2] = make_uint2(pkt | (pay.x << 16), pay.z);
}
__host__ __device__ __forceinline__ void seg_unpack(const uint2 (&q)[SEG_Q], uint4& key, uint4& pay) {
    const uint32_t w = q[1].y;
    key = make_uint4(q[0].x, q[0].y, q[1].x, w & 0xFF000001u);
    pay = make_uint4((q[2].x >> 16) | (((w >> 11) & 0x1Fu) << 16),
                     (q[2].x & 0xFFFFu) | (((w >> 16) & 0xFFu) << 16) | (((w >> 10) & 1u) << 24), q[2].y,
                     ((w >> 1) & 0xFFu) | (((w >> 9) & 1u) << 8));
}
__device__ __forceinline__ void seg_store(uint2* seg, size_t rec, const uint4& key, const uint4& pay) {
    uint2 q[SEG_Q];
    seg_pack(key, pay, q);
#pragma unroll
    for (uint32_t i = 0; i < SEG_Q; i++) seg[rec * SEG_Q + i] = q[i];
}
// two consecutive records from rec on: three 16-byte stores when rec is even
__device__ __forceinline__ void seg_store2(uint2* seg, size_t rec, const uint4& ka, const uint4& pa, const uint4& kb,
                                           const uint4& pb) {
    uint2 qa[SEG_Q], qb[SEG_Q];
    seg_pack(ka, pa, qa);
    seg_pack(kb, pb, qb);
    if ((rec & 1) == 0) {
        uint4* d = reinterpret_cast<uint4*>(seg + rec * SEG_Q);
        d[0] = make_uint4(qa[0].x, qa[0].y, qa[1].x, qa[1].y);
        d[1] = make_uint4(qa[2].x, qa[2].y, qb[0].x, qb[0].y);
        d[2] = make_uint4(qb[1].x, qb[1].y, qb[2].x, qb[2].y);
    } else {
#pragma unroll
        for (uint32_t i = 0; i < SEG_Q; i++) {
            seg[rec * SEG_Q + i] = qa[i];
            seg[(rec + 1) * SEG_Q + i] = qb[i];
        }
    }
}
__device__ __forceinline__ void seg_load(const uint2* seg, size_t rec, uint4& key, uint4& pay) {
    uint2 q[SEG_Q];
#pragma unroll
    for (uint32_t i = 0; i < SEG_Q; i++) q[i] = seg[rec * SEG_Q + i];
    seg_unpack(q, key, pay);
}
// MAC runs: in an owner segment a spilled packet is 48 bytes, three 16-byte
// words -- the packed form's 24 bytes, then {m0, m1}, {m2, key hash}, 8 zero
// bytes (a bin of 8 records: 384 B, three 128-B lines); the raw buffers and
// the overflow list keep 64 bytes: {k0, k1, k2, tag},
// {m0, m1, m2, key hash}, {doct, pt, loc, fl}, padding.
constexpr uint32_t SEGM_U = 3;  // 16-byte words per packed MAC record
__host__ __device__ __forceinline__ void segm_pack(const uint4& key, const uint4& mac, const uint4& pay, uint4 (&u)[SEGM_U]) {
    uint2 q[SEG_Q];
    seg_pack(key, pay, q);
    u[0] = make_uint4(q[0].x, q[0].y, q[1].x, q[1].y);
    u[1] = make_uint4(q[2].x, q[2].y, mac.x, mac.y);
    u[2] = make_uint4(mac.z, mac.w, 0u, 0u);
}
__host__ __device__ __forceinline__ void segm_unpack(const uint4 (&u)[SEGM_U], uint4& key, uint4& mac, uint4& pay) {
    const uint2 q[SEG_Q] = {make_uint2(u[0].x, u[0].y), make_uint2(u[0].z, u[0].w), make_uint2(u[1].x, u[1].y)};
    seg_unpack(q, key, pay);
    mac = make_uint4(u[1].z, u[1].w, u[2].x, u[2].y);
}

}  // namespace fl
