// Round trip of the packed owner-segment records (fluere_amd/csrc/seg.h):
// every field a spilled packet carries (kern.h Spill: key words, tag =
// proto << 24 | V6_TAG or 0xFF << 24, doct < SEG_DOCT_MAX, pkt, ttl, elig,
// the batch-relative position, TCP flags, dir) comes back unchanged, for the
// 24-byte form and the 48-byte MAC form.  Built and run by tests/test_seg_pack.py.
#include "../../fluere_amd/csrc/seg.h"

#include <cstdio>
#include <random>

using namespace fl;

static bool eq(const uint4& a, const uint4& b) { return a.x == b.x && a.y == b.y && a.z == b.z && a.w == b.w; }

int main() {
    std::mt19937 rng(20261019);
    long n = 0, bad = 0;
    auto check = [&](uint4 key, uint4 pay, uint4 mac) {
        uint2 q[SEG_Q];
        seg_pack(key, pay, q);
        uint4 k2, p2;
        seg_unpack(q, k2, p2);
        uint4 u[SEGM_U];
        segm_pack(key, mac, pay, u);
        uint4 k3, m3, p3;
        segm_unpack(u, k3, m3, p3);
        n++;
        if (!eq(k2, key) || !eq(p2, pay) || !eq(k3, key) || !eq(m3, mac) || !eq(p3, pay) || u[2].z || u[2].w) {
            if (bad++ < 5)
                printf("mismatch: key %08x %08x %08x %08x pay %08x %08x %08x %08x\n", key.x, key.y, key.z, key.w, pay.x,
                       pay.y, pay.z, pay.w);
        }
    };
    const uint32_t tags[] = {6u << 24, 17u << 24, (6u << 24) | 1u, (17u << 24) | 1u, 0xFF000000u, 1u << 24, 0u};
    for (int i = 0; i < 2000000; i++) {
        const uint32_t tag = tags[rng() % 7];
        const uint32_t doct = i % 3 == 0 ? SEG_DOCT_MAX - 1 - (rng() & 0xFF) : rng() % SEG_DOCT_MAX;
        const uint32_t pkt = i % 5 == 0 ? 0xFFFFu : rng() & 0xFFFFu, ttl = rng() & 0xFFu, elig = rng() & 1u;
        const uint32_t tf = rng() & 0xFFu, dir = rng() & 1u;
        check(make_uint4(rng(), rng(), rng(), tag), make_uint4(doct, pkt | (ttl << 16) | (elig << 24), rng(), tf | (dir << 8)),
              make_uint4(rng(), rng(), rng(), rng()));
    }
    check(make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0));
    check(make_uint4(~0u, ~0u, ~0u, 0xFF000001u), make_uint4(SEG_DOCT_MAX - 1, 0x1FFFFFFu, ~0u, 0x1FFu), make_uint4(~0u, ~0u, ~0u, ~0u));
    printf("seg round trip: %ld records, %ld mismatches\n", n, bad);
    return bad ? 1 : 0;
}
