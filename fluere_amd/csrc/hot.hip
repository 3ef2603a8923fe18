// hot.hip -- the hot pass: k_parse_agg (LDS flow tables, few flows per window)
// and k_parse_spill (per-owner bins, many flows per window).
#include "ctx.h"

namespace fl {

// ABL (diagnostics only): 5 every LDS-table miss written to its lane's own
// contiguous run (4 consecutive misses of a lane fill one 128-B line; wrong
// results: the merge never sees them) -- the store pattern of per-owner bins;
// 4 every LDS-table miss appended to the workgroup's
// raw buffer (coalesced, wave-aggregated) instead of its owner segment (still
// correct: the overflow list); 0 full kernel; 1 parse + canonical key only; 2 + LDS key
// table, no aggregation; 3 aggregation into hashed slots without the key table
template <int ABL, bool MACS>
__global__ void __launch_bounds__(BLOCK) k_parse_agg(AggArgs a) {
    // LDS flow table.  Per slot: packets (low 32) and bytes (high 32) per
    // canonical direction in one u64 (one ds_add_u64 per packet; a window
    // holds <= 61440 packets of <= 65535 bytes, so neither half wraps);
    // {min pkt, min ttl, max pkt, max ttl}; window-relative positions
    // {first, first create-eligible, first FIN/RST, last + 1}; flag pairs.
    __shared__ uint4 s_key[LK];
    __shared__ unsigned long long s_pb[2][NS];
    __shared__ uint4 s_mm[NS], s_pos[NS];
    __shared__ uint32_t s_fl[4][NS];
    __shared__ uint32_t s_sk[NS];  // key entry of each slot
    __shared__ uint4 s_slab[BLOCK / 64][160];  // per wave: half a dense chunk's span (32 x 80 B)
    __shared__ uint32_t s_nslot, s_chunk, s_nspill;
    __shared__ uint32_t s_own[OWN_WORDS];   // flush: per-owner slot counts -> segment starts (packed, own_get)
    __shared__ uint32_t s_scnt[OWN_WORDS];  // spilled packets per owner (this window) -> segment starts (packed)
    __shared__ unsigned long long s_sbase;
    __shared__ unsigned long long s_cnt[5], s_tmin, s_tmax;
    __shared__ uint32_t s_slow;  // this workgroup's slow-list entries
    const int tid = threadIdx.x;
    // MAC kernels: LK / 2 key entries, each with its MAC sidecar at + LK / 2
    constexpr int LKL = MACS ? LK / 2 : LK, LKL_BITS = MACS ? LK_BITS - 1 : LK_BITS;
    constexpr uint32_t NSL = MACS ? NS_MAC : NS;
    constexpr int SPU = spill_units(MACS);
    for (int e = tid; e < LK; e += BLOCK) s_key[e] = make_uint4(0, 0, 0, 0);
    for (int e = tid; e < NS; e += BLOCK) {
        s_pb[0][e] = s_pb[1][e] = 0;
        s_mm[e] = make_uint4(NONE32, NONE32, 0, 0);
        s_pos[e] = make_uint4(NONE32, NONE32, NONE32, 0);
        s_fl[0][e] = s_fl[1][e] = s_fl[2][e] = s_fl[3][e] = 0;
    }
    if (tid < 5) s_cnt[tid] = 0;
    if (tid == 0) s_slow = 0;
    if (tid == 0) { s_tmin = NONE64; s_tmax = 0; s_nslot = 0; s_chunk = 0; s_nspill = 0; }
    for (int o = tid; o < OWN_WORDS; o += BLOCK) s_scnt[o] = 0;
    __syncthreads();

    const Batch& B = a.B;
    const uint64_t n = B.n;
#ifndef FLUERE_HOT_ORDER
#define FLUERE_HOT_ORDER 1
#endif
    // Packet order.  Step st of workgroup b covers BLOCK consecutive packets:
    //   ORDER 1 (interleaved): packets (st * G + b) * BLOCK + [0, BLOCK) -- all
    //     workgroups stream one moving region of the capture together;
    //   ORDER 0 (contiguous): workgroup b owns the range [b * per, (b+1) * per).
    // Positions inside a window are relative to the window's first packet
    // (at most WIN_ITERS * G * BLOCK apart: they fit u32).
    const uint64_t G = gridDim.x;
    const uint64_t per = (n + G - 1) / G;
    const uint64_t stride = FLUERE_HOT_ORDER ? G * BLOCK : BLOCK;
    const uint64_t beg = FLUERE_HOT_ORDER ? (uint64_t)blockIdx.x * BLOCK : per * blockIdx.x;
    const uint64_t end = FLUERE_HOT_ORDER ? n : min(n, beg + per);
    unsigned long long c_valid = 0, c_drop = 0, c_miss = 0, tmin = NONE64, tmax = 0;
    uint32_t d_loops = 0, d_iters = 0;  // diagnostics (per wave, uniform)
    uint32_t d_abl5 = 0;                // diagnostics (ABL 5): this lane's misses
    const uint64_t nsteps = end > beg ? (end - beg + stride - 1) / stride : 0;
    uint64_t wbase = beg;
    uint32_t win = 0;  // this workgroup's window (set blockIdx.x * W + win)

    // PK packets per lane per iteration (steps st .. st+PK-1), processed
    // phase by phase so that the LDS round trips of the PK packets overlap
    // (every phase issues its reads for all PK packets before using any).
    // Packets the hot parser declines, and packets of keys that find no LDS
    // slot, are appended to the slow list: slow_packets runs the general
    // parser and the global path for them (nothing rare is inlined here).
    struct PS {
        Hot h;
        uint32_t dir, lo_ip, hi_ip, kports, k0, k1, k2, tag, e, e2, slot;
        uint32_t m0, m1, m2;  // MAC kernels: the canonical MAC pair (mac_ckey)
        int state, steps;
        bool valid, slow;
    };
    auto process = [&](const Win (&W)[PK], const uint32_t (&off)[PK], const uint64_t (&li)[PK], const bool (&live)[PK]) {
        PS q[PK];
#pragma unroll
        for (int u = 0; u < PK; u++) {
            Hot& h = q[u].h;
            const uint32_t cls = live[u] ? hot_parse(B, off[u], W[u], h) : HOT_DROP;
            c_drop += (live[u] & (cls == HOT_DROP)) ? 1 : 0;
            q[u].valid = live[u] & (cls == HOT_OK);
            q[u].slow = live[u] & (cls == HOT_SLOW);
            // canonical key: lower endpoint (ip, port[, mac]) first (flow_table.h)
            const uint32_t sp = h.ports >> 16, dp = h.ports & 0xFFFFu;
            bool gt = (h.sip > h.dip) | ((h.sip == h.dip) & (sp > dp));
            uint64_t smac = 0, dmac = 0;
            if (MACS) {
                const uint32_t d_hi = __builtin_amdgcn_perm(W[u].w[5], W[u].w[4], 0x00010203u);  // frame bytes 0..3
                const uint32_t d_lo = __builtin_amdgcn_perm(W[u].w[5], W[u].w[4], 0x0C0C0405u);  // frame bytes 4..5
                const uint32_t s_hi = __builtin_amdgcn_perm(W[u].w[6], W[u].w[5], 0x02030405u);  // frame bytes 6..9
                const uint32_t s_lo = __builtin_amdgcn_perm(W[u].w[6], W[u].w[5], 0x0C0C0607u);  // frame bytes 10..11
                dmac = ((uint64_t)d_hi << 16) | d_lo;
                smac = ((uint64_t)s_hi << 16) | s_lo;
                if ((h.sip == h.dip) & (sp == dp)) gt = smac > dmac;
            }
            q[u].dir = gt ? 1u : 0u;
            q[u].lo_ip = gt ? h.dip : h.sip;
            q[u].hi_ip = gt ? h.sip : h.dip;
            q[u].kports = gt ? __builtin_amdgcn_alignbit(h.ports, h.ports, 16) : h.ports;
            q[u].k0 = q[u].lo_ip;
            q[u].k1 = q[u].hi_ip;
            q[u].k2 = q[u].kports;
            q[u].tag = h.proto << 24;
            if (!MACS && a.phash && live[u])
                a.phash[li[u]] = q[u].valid ? ckey_bucket_v4(q[u].k0, q[u].k1, q[u].k2, h.proto) : PH_PARSE;
            q[u].m0 = q[u].m1 = q[u].m2 = 0;
            if (MACS) {  // the MAC pair joins the key (the dictionary is walked once per slot, at the flush)
                const uint64_t lom = gt ? dmac : smac, him = gt ? smac : dmac;
                q[u].m0 = (uint32_t)(lom >> 16);
                q[u].m1 = ((uint32_t)(lom & 0xFFFF) << 16) | (uint32_t)(him & 0xFFFF);
                q[u].m2 = (uint32_t)(him >> 16);
            }
        }
        if (ABL == 1) {
#pragma unroll
            for (int u = 0; u < PK; u++)
                if (q[u].valid)
                    asm volatile("" ::"v"(q[u].lo_ip ^ q[u].hi_ip ^ q[u].kports ^ q[u].h.proto ^ q[u].h.doct ^
                                          q[u].h.pkt ^ q[u].h.ttl ^ q[u].dir));
            return;
        }
        // find or claim the key entries.  First probe of every packet inline
        // (the common case: a published entry at the home position); the
        // wave-uniform retry loop runs only while some lane still searches (a
        // lane that lost a claim, or saw an entry being written, reads the
        // pair again next step).
        // Probe sequence of a key: pair e1, pair e2, then linear from e2 + 2
        // (write-once table, so lookups and inserts follow one sequence).
        // Two-choice placement keeps nearly every key in one of its first two
        // pairs; both are read inline, so the retry loop below runs only for
        // inserts and for the rare key placed further on.
        uint32_t hk[PK];
        uint4 kp[PK][4];
#pragma unroll
        for (int u = 0; u < PK; u++) {
            hk[u] = lt_hash(q[u].k0, q[u].k1, q[u].k2, q[u].tag);
            if (MACS) hk[u] = mac_hash(hk[u], q[u].m0, q[u].m1, q[u].m2);
            const uint32_t e1 = hk[u] & (LKL - 2);  // even: entries e, e+1 per step
            uint32_t e2 = (hk[u] >> 12) * 0x9E3779B1u >> (32 - LKL_BITS + 1) << 1;
            e2 = FLUERE_PROBE2 ? (e2 == e1 ? e1 ^ 2u : e2) : (e1 + 2) & (LKL - 1);
            q[u].e = e1;
            q[u].e2 = e2;
            kp[u][0] = s_key[e1];
            kp[u][1] = s_key[e1 + 1];
            kp[u][2] = FLUERE_PROBE2 ? s_key[e2] : make_uint4(0, 0, 0, 0);
            kp[u][3] = FLUERE_PROBE2 ? s_key[e2 + 1] : make_uint4(0, 0, 0, 0);
        }
        bool searching = false;
#pragma unroll
        for (int u = 0; u < PK; u++) {
            bool m[4];
#pragma unroll
            for (int k = 0; k < 4; k++)
                m[k] = ((kp[u][k].w & (0xFF000000u | LT_READY)) == (q[u].tag | LT_READY)) & (kp[u][k].x == q[u].k0) &
                       (kp[u][k].y == q[u].k1) & (kp[u][k].z == q[u].k2);
            if (MACS) {
                // the sidecar of an entry whose 5-tuple words match (read after the
                // entry, so a published entry's sidecar is seen written)
                bool hit = false;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    if (m[k] & !hit) {
                        const uint32_t ek = (k < 2 ? q[u].e : q[u].e2) + (k & 1);
                        const uint4 xs = s_key[LKL + ek];
                        m[k] = (xs.w == 1u) & (xs.x == q[u].m0) & (xs.y == q[u].m1) & (xs.z == q[u].m2);
                        hit = m[k];
                    } else {
                        m[k] = false;
                    }
                }
            }
            const uint32_t sw = m[0] ? kp[u][0].w : m[1] ? kp[u][1].w : m[2] ? kp[u][2].w : kp[u][3].w;
            q[u].slot = sw & LT_SLOT;
            const bool found = m[0] | m[1] | m[2] | m[3];
            q[u].state = q[u].valid ? (found ? 1 : 0) : 2;  // 0 searching, 1 found (slot < NS, or NS: no slot), 2 none
            const bool full1 = (kp[u][0].w & kp[u][1].w & LT_READY) != 0;
            const bool full2 = (kp[u][2].w & kp[u][3].w & LT_READY) != 0;
            // where the search goes on: the first pair of the sequence not yet
            // known to be full of other keys
            q[u].steps = full1 ? (full2 ? 2 : 1) : 0;
            q[u].e = full1 ? (full2 ? (q[u].e2 + 2) & (LKL - 1) : q[u].e2) : q[u].e;
            if (ABL == 3) {  // diagnostics: aggregation without the key table (wrong slots)
                q[u].slot = lt_hash(q[u].k0, q[u].k1, q[u].k2, q[u].tag) % 1000u;
                q[u].state = q[u].valid ? 1 : 2;
            }
            searching |= q[u].state == 0;
        }
        // every aggregate slot taken (more flows in this window than NS): a
        // key not in its two inline pairs spills at once -- inserting it
        // would gain nothing, and the search through a full table costs a
        // dozen LDS round trips per chunk
        if (searching && s_nslot >= NSL) {
#pragma unroll
            for (int u = 0; u < PK; u++)
                if (q[u].state == 0) q[u].state = 2;
            searching = false;
        }
        if (ABL != 3 && __ballot(searching)) {
            d_loops++;
            for (int it = 0; it < 2 * LK_STEPS; it++) {
                d_iters++;
                bool more = false;
#pragma unroll
                for (int u = 0; u < PK; u++) {
                    PS& r = q[u];
                    if (r.state == 0) {
                        const uint4 ka = s_key[r.e], kb = s_key[r.e + 1];
                        bool ma = (ka.w & (0xFF000000u | LT_READY)) == (r.tag | LT_READY) && ka.x == r.k0 &&
                                  ka.y == r.k1 && ka.z == r.k2;
                        bool mb = (kb.w & (0xFF000000u | LT_READY)) == (r.tag | LT_READY) && kb.x == r.k0 &&
                                  kb.y == r.k1 && kb.z == r.k2;
                        if (MACS) {
                            const uint4 xa = s_key[LKL + r.e], xb = s_key[LKL + r.e + 1];
                            ma = ma && xa.w == 1u && xa.x == r.m0 && xa.y == r.m1 && xa.z == r.m2;
                            mb = mb && xb.w == 1u && xb.x == r.m0 && xb.y == r.m1 && xb.z == r.m2;
                        }
                        if (ma || mb) {
                            r.slot = (ma ? ka.w : kb.w) & LT_SLOT;
                            r.state = 1;
                        } else if ((ka.w & LT_READY) && (kb.w & LT_READY)) {
                            if (++r.steps == LK_STEPS) r.state = 2;
                            else r.e = r.steps == 1 ? r.e2 : (r.e + 2) & (LKL - 1);
                        } else {
                            // first free entry of the pair; an entry being written (CLAIM) is re-read next step
                            const uint32_t f = (ka.w == 0) ? r.e : ((ka.w & LT_READY) && kb.w == 0 ? r.e + 1 : LKL);
                            if (f < LKL && atomicCAS(&s_key[f].w, 0u, LT_CLAIM) == 0u) {
                                uint32_t sl = atomicAdd(&s_nslot, 1u);
                                if (sl >= NSL) sl = NSL;  // no slot left: the key is kept, its packets spill
                                s_key[f].x = r.k0;
                                s_key[f].y = r.k1;
                                s_key[f].z = r.k2;
                                if (MACS) s_key[LKL + f] = make_uint4(r.m0, r.m1, r.m2, 1u);
                                if (sl < NSL) s_sk[sl] = f;
                                __threadfence_block();
                                atomicExch(&s_key[f].w, r.tag | LT_READY | (sl < NSL ? sl : LT_SLOT));
                                r.slot = sl;
                                r.state = 1;
                            }
                        }
                    }
                    more |= r.state == 0;
                }
                if (__ballot(more) == 0) break;
            }
        }
        bool agg[PK];
#pragma unroll
        for (int u = 0; u < PK; u++) {
            agg[u] = q[u].valid & (q[u].state == 1) & (q[u].slot < NSL);
            // a valid packet whose key has no LDS slot spills: a packed 24-byte
            // record (48 with MACs; seg.h) straight into its merge owner's segment of this
            // set; past the segment's capacity, to this workgroup's raw
            // overflow buffer (wave-aggregated append; listed at the flush)
            const bool miss = q[u].valid & !agg[u];
            c_miss += miss ? 1 : 0;
            bool ovf = false;
            if (miss) {
                const Hot& h = q[u].h;
                const uint32_t loc = (uint32_t)(li[u] - wbase);
                const bool elig = (h.proto != 6u) | ((h.tf & 2u) != 0);
                const uint4 w_key = make_uint4(q[u].k0, q[u].k1, q[u].k2, q[u].tag);
                const uint4 w_pay = make_uint4(h.doct, h.pkt | (h.ttl << 16) | ((elig ? 1u : 0u) << 24), loc,
                                               h.tf | (q[u].dir << 8));
                const uint32_t ow = owner_of(hk[u], a.S.O);
                const uint32_t pos = ABL == 4 ? 0xFFFFFFFFu : ABL == 5 ? 0u : own_add(s_scnt, ow);
                if (ABL == 5) {
                    uint4* dst = reinterpret_cast<uint4*>(a.S.spill_raw) + (size_t)blockIdx.x * SPILL_WG * 2 +
                                 ((size_t)threadIdx.x * WIN_ITERS + (d_abl5++ % WIN_ITERS)) * 2;
                    dst[0] = w_key;
                    dst[1] = w_pay;
                } else if (pos < a.S.cap_o) {
                    const size_t rec = ((size_t)(blockIdx.x * a.S.W + win) * a.S.O + ow) * a.S.cap_o + pos;
                    if (MACS) {
                        uint4 pk[SEGM_U];
                        segm_pack(w_key, make_uint4(q[u].m0, q[u].m1, q[u].m2, hk[u]), w_pay, pk);
                        uint4* dst = reinterpret_cast<uint4*>(a.S.dspill) + rec * SEGM_U;
#pragma unroll
                        for (uint32_t i = 0; i < SEGM_U; i++) dst[i] = pk[i];
                    } else {
                        seg_store(reinterpret_cast<uint2*>(a.S.dspill), rec, w_key, w_pay);
                    }
                } else {
                    ovf = true;
                }
                c_valid++;
                tmin = min(tmin, (unsigned long long)h.t);
                tmax = max(tmax, (unsigned long long)h.t);
            }
            const uint64_t mm_ = __ballot(ovf);
            if (mm_) {
                const uint32_t lead = __builtin_ctzll(mm_);
                uint32_t b0 = 0;
                if ((uint32_t)(threadIdx.x & 63) == lead) b0 = atomicAdd(&s_nspill, (uint32_t)__popcll(mm_));
                b0 = __shfl(b0, lead, 64);
                if (ovf) {
                    const Hot& h = q[u].h;
                    const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(mm_ >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)mm_, 0u));
                    const uint32_t loc = (uint32_t)(li[u] - wbase);
                    const bool elig = (h.proto != 6u) | ((h.tf & 2u) != 0);
                    uint4* dst = reinterpret_cast<uint4*>(a.S.spill_raw) + (size_t)blockIdx.x * SPILL_WG * 2 * SPU + b0 + r;
                    dst[0] = make_uint4(q[u].k0, q[u].k1, q[u].k2, q[u].tag);
                    if (MACS) dst[SPILL_WG] = make_uint4(q[u].m0, q[u].m1, q[u].m2, hk[u]);
                    dst[(MACS ? 2 : 1) * SPILL_WG] = make_uint4(h.doct, h.pkt | (h.ttl << 16) | ((elig ? 1u : 0u) << 24),
                                                                loc, h.tf | (q[u].dir << 8));
                }
            }
            const bool slow = q[u].slow;
            // slow list: wave-aggregated append into this workgroup's region
            // (an LDS cursor; one global atomic per wave on a single counter
            // serialised an all-slow capture: 1.9 ms for 10M packets)
            const uint64_t sm = __ballot(slow);
            if (sm) {
                const uint32_t lead = __builtin_ctzll(sm);
                uint32_t b0 = 0;
                if ((uint32_t)(threadIdx.x & 63) == lead) b0 = atomicAdd(&s_slow, (uint32_t)__popcll(sm));
                b0 = __shfl(b0, lead, 64);
                if (slow) {
                    const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(sm >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)sm, 0u));
                    a.slow[(size_t)blockIdx.x * a.slow_region + b0 + r] = (uint32_t)li[u];
                }
            }
        }
        if (ABL == 2) {  // diagnostics: key table only
#pragma unroll
            for (int u = 0; u < PK; u++) asm volatile("" ::"v"(q[u].slot));
            return;
        }
        // update_flow (flows.rs:11-42), order-free part.  Guard reads of every
        // packet first (a slot index of 0 for lanes without an update keeps
        // them unconditional), then the atomics: min / max and first
        // positions change rarely, so they are written only where the packet
        // moves the value (a stale guard can only cost a redundant atomic,
        // never skip a needed one: the values move monotonically).
        uint4 mm[PK];
        uint2 ps[PK];
#pragma unroll
        for (int u = 0; u < PK; u++) {
            const uint32_t sl = agg[u] ? q[u].slot : 0u;
            if (!(FLUERE_AGG_UNCOND & 1)) mm[u] = s_mm[sl];
            if (!(FLUERE_AGG_UNCOND & 2)) ps[u] = *reinterpret_cast<const uint2*>(&s_pos[sl]);
        }
#pragma unroll
        for (int u = 0; u < PK; u++) {
            if (!agg[u]) continue;
            const Hot& h = q[u].h;
            const uint32_t slot = q[u].slot;
            c_valid++;
            tmin = min(tmin, (unsigned long long)h.t);
            tmax = max(tmax, (unsigned long long)h.t);
            const uint32_t tf = h.tf;
            const uint32_t loc = (uint32_t)(li[u] - wbase);
            atomicAdd(&s_pb[q[u].dir][slot], ((unsigned long long)h.doct << 32) | 1ull);
            atomicMax(&s_pos[slot].w, loc + 1);
            if (FLUERE_AGG_UNCOND & 1) {
                atomicMin(&s_mm[slot].x, h.pkt);
                atomicMin(&s_mm[slot].y, h.ttl);
                atomicMax(&s_mm[slot].z, h.pkt);
                atomicMax(&s_mm[slot].w, h.ttl);
            } else {
                if (h.pkt < mm[u].x) atomicMin(&s_mm[slot].x, h.pkt);
                if (h.ttl < mm[u].y) atomicMin(&s_mm[slot].y, h.ttl);
                if (h.pkt > mm[u].z) atomicMax(&s_mm[slot].z, h.pkt);
                if (h.ttl > mm[u].w) atomicMax(&s_mm[slot].w, h.ttl);
            }
            // a flow is created by any non-TCP packet or a SYN (offline_fluereflows.rs:101-113)
            const bool elig = (h.proto != 6u) | ((tf & 2u) != 0);
            if (FLUERE_AGG_UNCOND & 2) {
                atomicMin(&s_pos[slot].x, loc);
                atomicMin(&s_pos[slot].y, elig ? loc : NONE32);
            } else {
                if (loc < ps[u].x) atomicMin(&s_pos[slot].x, loc);
                if (elig & (loc < ps[u].y)) atomicMin(&s_pos[slot].y, loc);
            }
            if (tf) {
#pragma unroll
                for (int qq = 0; qq < 4; qq++) {
                    const uint32_t w = ((tf >> (2 * qq)) & 1) | (((tf >> (2 * qq + 1)) & 1) << 16);
                    if (w) atomicAdd(&s_fl[qq][slot], w);
                }
                if (tf & 5) atomicMin(&s_pos[slot].z, loc);  // FIN or RST
            }
        }
    };
    unsigned long long cyc_flush = 0, cyc_wait = 0, cyc_start = clock64(), rt_start = wall_clock64();
    uint32_t ovf_total = 0;  // (thread 0) overflow records of every window
    auto flush = [&]() {
        // the window's partial aggregates -> this workgroup's staging set
        // (plain coalesced stores, lane per slot); k_merge_partials merges them
        const unsigned long long fw = clock64();
        if (a.dbg && tid == 0 && win == 0) a.dbg[blockIdx.x * 8 + 1] = wall_clock64();
        // every wave's spill stores have completed (vmcnt) before the barrier
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        const unsigned long long f0 = clock64();  // flush proper (fw..f0: waiting for the slowest wave)
        cyc_wait += f0 - fw;
        const Stage& S = a.S;
        const uint32_t set = blockIdx.x * S.W + win;
        const uint32_t ns = min(s_nslot, NSL), O = S.O;
        if (tid == 0) s_chunk = 0;  // every wave has drawn its last chunk of the window
        // counting sort of this window's flows by merge owner; a thread keeps
        // its slots' (at most two) owners and hashes in registers
        constexpr int SPT = (NS + BLOCK - 1) / BLOCK;  // slots per thread
        for (uint32_t o = tid; o < OWN_WORDS; o += BLOCK) s_own[o] = 0;
        lds_barrier();
        uint32_t own[SPT], hh[SPT];
        uint4 kks[SPT];
#pragma unroll
        for (int k = 0; k < SPT; k++) {
            own[k] = NONE32;
            hh[k] = 0;
        }
#pragma unroll
        for (int k = 0; k < SPT; k++) {
            const uint32_t e = tid + k * BLOCK;
            if (e >= ns || (s_pb[0][e] | s_pb[1][e]) == 0) continue;
            kks[k] = s_key[s_sk[e]];
            hh[k] = lt_hash(kks[k].x, kks[k].y, kks[k].z, kks[k].w & 0xFF000000u);
            if (MACS) {  // the MAC words travel beside the partial (S.partx); same hash as the hot loop's
                const uint4 xs = s_key[LKL + s_sk[e]];
                hh[k] = mac_hash(hh[k], xs.x, xs.y, xs.z);
            }
            own[k] = owner_of(hh[k], O);
            own_add(s_own, own[k]);
        }
        lds_barrier();
        if (a.dbg && tid == 0 && win == 0) a.dbg[blockIdx.x * 8 + 4] = wall_clock64();
        // exclusive scan of the slot counts over the owners (one wave, an
        // even run of owners per lane, so no two lanes write one packed word)
        static_assert(MAX_OWNERS % 2 == 0, "owner runs cover whole words");
        if (tid < 64) {
            uint32_t* arr = s_own;
            const uint32_t l = tid & 63;
            const uint32_t per = 2 * ((O + 127) / 128);
            uint32_t sum = 0;
            for (uint32_t q = 0; q < per; q++) {
                const uint32_t o = l * per + q;
                if (o < O) sum += own_get(arr, o);
            }
            uint32_t incl = sum;
#pragma unroll
            for (int dlt = 1; dlt < 64; dlt <<= 1) {
                const uint32_t y = __shfl_up(incl, dlt, 64);
                if (l >= dlt) incl += y;
            }
            uint32_t run = incl - sum;
            for (uint32_t q = 0; q < per; q++) {
                const uint32_t o = l * per + q;
                if (o < O) {
                    const uint32_t v = own_get(arr, o);
                    own_set(arr, o, run);
                    run += v;
                }
            }
            if (l == 63) own_set(arr, O, incl);
        }
        const uint32_t nsp = s_nspill;  // overflow records of this window
        if (tid == 128) s_sbase = nsp ? atomicAdd(&a.bc[1], (unsigned long long)nsp) : 0ull;
        if (tid == 0) ovf_total += nsp;
        lds_barrier();
        for (uint32_t o = tid; o <= O; o += BLOCK) {
            S.off[(size_t)o * S.n_sets + set] = own_get(s_own, o);
            if (o < O) S.soff[(size_t)o * S.n_sets + set] = min(own_get(s_scnt, o), S.cap_o);
        }
        if (tid == 0) S.base[set] = B.first + wbase;
        lds_barrier();
        if (a.dbg && tid == 0 && win == 0) a.dbg[blockIdx.x * 8 + 5] = wall_clock64();
        // overflow records -> the overflow list (the raw records were written
        // by other waves of this workgroup: nontemporal loads, which bypass
        // the CU's L1); the set goes into fl's high bits
        if (nsp) {
            const uint4* raw = reinterpret_cast<const uint4*>(S.spill_raw) + (size_t)blockIdx.x * SPILL_WG * 2 * SPU;
            const unsigned long long sb = s_sbase;
            // SU records per thread per round, all loads issued first (one
            // round trip per round instead of one per record)
            constexpr int SU = 4;
            typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
            const uint32_t last = nsp ? nsp - 1 : 0;  // (loads stay inside the buffer even if hoisted)
            constexpr int SW = MACS ? 3 : 2;  // 16-byte words per spilled packet
            for (uint32_t i0 = 0; i0 < nsp; i0 += SU * BLOCK) {
                u32x4 av[SU][SW];
#pragma unroll
                for (int u = 0; u < SU; u++) {
                    const uint32_t i = i0 + u * BLOCK + tid;
                    const u32x4* src = reinterpret_cast<const u32x4*>(raw + min(i, last));
#pragma unroll
                    for (int w = 0; w < SW; w++) av[u][w] = __builtin_nontemporal_load(src + (size_t)w * SPILL_WG);
                }
                // every load of the round issued before the first use (the
                // compiler would sink a guarded record's loads into its branch)
#pragma unroll
                for (int u = 0; u < SU; u++)
#pragma unroll
                    for (int w = 0; w < SW; w++) asm volatile("" ::"v"(av[u][w]));
#pragma unroll
                for (int u = 0; u < SU; u++) {
                    const uint32_t i = i0 + u * BLOCK + tid;
                    if (i >= nsp) continue;
                    av[u][SW - 1].w |= set << 9;
                    uint4* dst = reinterpret_cast<uint4*>(S.spill) + (sb + i) * (size_t)(2 * SPU);
#pragma unroll
                    for (int w = 0; w < SW; w++) dst[w] = make_uint4(av[u][w].x, av[u][w].y, av[u][w].z, av[u][w].w);
                }
            }
        }
#pragma unroll
        for (int k = 0; k < SPT; k++) {
            const uint32_t e = tid + k * BLOCK;
            if (own[k] == NONE32) continue;
            const unsigned long long p0 = s_pb[0][e], p1 = s_pb[1][e];
            const uint4 kk = kks[k];
            const uint32_t tag = kk.w & 0xFF000000u;
            const uint32_t h = hh[k];
            const size_t o = (size_t)set * NS + (FLUERE_FLUSH_LINEAR ? e : own_add(s_own, own[k]));
            uint4* dst = reinterpret_cast<uint4*>(S.part + o);
            if (FLUERE_FLUSH_LINEAR == 2 && kk.x != 0x12345678u) continue;  // diagnostics: no stores
            const uint4 mm = s_mm[e], ps = s_pos[e];
            const uint4 fw = make_uint4(s_fl[0][e], s_fl[1][e], s_fl[2][e], s_fl[3][e]);
            // lean (kern.h PART_LEAN): no flag, no FIN/RST, first packet creates
            const bool lean = !MACS && (fw.x | fw.y | fw.z | fw.w) == 0 && ps.z == NONE32 && ps.y == ps.x;
            dst[0] = make_uint4(kk.x, kk.y, kk.z, tag | (lean ? PART_LEAN : 0u));
            dst[1] = make_uint4(h, (uint32_t)(p0 & 0xFFFF) | ((uint32_t)(p1 & 0xFFFF) << 16), (uint32_t)(p0 >> 32),
                                (uint32_t)(p1 >> 32));
            // (plain stores: nontemporal ones, measured, made the kernel ~20 us
            // longer -- 20 MB written through at once at the end of the pass)
            if (lean) {
                dst[2] = make_uint4(mm.x | (mm.z << 16), mm.y | (mm.w << 8), ps.x, ps.w);
            } else {
                dst[2] = make_uint4(mm.x, mm.y, mm.z, mm.w);
                dst[3] = fw;
                dst[4] = ps;
            }
            if (MACS) {  // (re-read from LDS: registers are scarce across the spill scatter)
                const uint4 xs = s_key[LKL + s_sk[e]];
                S.partx[o] = make_uint4(xs.x, xs.y, xs.z, h);
            }
            s_pb[0][e] = s_pb[1][e] = 0;
            s_mm[e] = make_uint4(NONE32, NONE32, 0, 0);
            s_pos[e] = make_uint4(NONE32, NONE32, NONE32, 0);
            s_fl[0][e] = s_fl[1][e] = s_fl[2][e] = s_fl[3][e] = 0;
        }
        lds_barrier();
        if (a.dbg && tid == 0 && win == 0) a.dbg[blockIdx.x * 8 + 6] = wall_clock64();
        for (uint32_t o = tid; o < OWN_WORDS; o += BLOCK) s_scnt[o] = 0;
        if (tid == 0) s_nspill = 0;
        lds_barrier();
        const unsigned long long f1 = clock64() - f0;
        if (a.dbg && tid == 0 && win == 0) a.dbg[blockIdx.x * 8 + 2] = wall_clock64();
        cyc_flush += f1;
        wbase += stride * WIN_ITERS;
        win++;
    };
    const uint64_t lastp = n - 1;  // loads past the end re-read the last packet (in bounds)
    // Window by window.  A window is WIN_ITERS steps of this workgroup, i.e.
    // WIN_ITERS * WAVES wave-chunks of 64 packets; the chunks are dealt to the
    // waves dynamically (an LDS counter) so the waves of a workgroup finish a
    // window together (static assignment left waves idle for ~10% of the
    // kernel while the slowest one finished).  Per chunk the offset of the
    // wave's next chunk is prefetched (one register of carry), the window is
    // loaded and consumed in the same iteration and pinned (pin_win) so its
    // loads form one round trip; only offsets cross the back edge.
    static_assert(PK == 1, "dynamic chunks: one packet per lane per iteration");
    constexpr uint32_t WAVES = BLOCK / 64;
    const uint32_t lane = tid & 63;
    uint4* slab = s_slab[__builtin_amdgcn_readfirstlane(tid >> 6)];
    auto grab = [&]() {
        uint32_t v = 0;
        if (lane == 0) v = atomicAdd(&s_chunk, 1u);
        return __builtin_amdgcn_readfirstlane(v);
    };
    // a per-lane zero the compiler cannot see through: keeps the (uniform)
    // descriptor loads on the vector memory path (vmcnt), so they never hold
    // up the LDS waits (lgkmcnt) of the processing as a scalar load would
    uint32_t vzero;
    asm volatile("v_mov_b32 %0, 0" : "=v"(vzero));
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    for (uint64_t ws = 0; ws < nsteps; ws += WIN_ITERS) {
        const uint32_t nch = (uint32_t)min<uint64_t>(WIN_ITERS, nsteps - ws) * WAVES;
        auto li_of = [&](uint32_t c) -> uint64_t {
            return beg + (ws + c / WAVES) * stride + (uint64_t)(c % WAVES) * 64 + lane;
        };
        // descriptor of chunk c (Batch::desc): a vector load, every lane the same word
        auto desc_of = [&](uint32_t c) -> uint2 {
            const uint64_t ch = (li_of(c) - lane) >> 6;
            if (c >= nch || ch >= B.n_desc) return make_uint2(0, 0);
            return B.desc[ch + vzero];
        };
        // Software pipeline, one chunk deep: while chunk c is processed the
        // loads of the wave's next chunk cn are in flight.  Dense chunks: six
        // coalesced nontemporal 16-byte loads per lane cover the chunk's span
        // (64 windows at stride <= 80 B); they are transposed to per-lane
        // windows through the wave's LDS slab.  Sparse chunks: the record
        // offsets are loaded one chunk ahead, the windows when processed.
        // The loads are issued unconditionally (inline asm; a chunk that does
        // not need them points them at one cached line), so no branch merges
        // registers that are still being loaded: such a merge makes the
        // compiler copy them, which waits for them and drains the pipeline.
        // Their completion is waited for explicitly (vmcnt(0) at the top).
        u32x4 v[5];
        uint32_t osp;
        auto issue = [&](uint32_t c, uint2 d) {
            const bool dense = d.y != 0;
            const uint64_t li = min(li_of(c), lastp);
            const uint8_t* g = dense ? B.bytes + d.x : reinterpret_cast<const uint8_t*>(B.offs + (li & ~63ull));
            const uint32_t np = dense ? (63u * d.y + 80u + 15u) / 16u : 1u;
#pragma unroll
            for (int k = 0; k < 5; k++) {
                const uint8_t* p = g + 16u * min(k * 64u + lane, np - 1u);
                asm volatile("global_load_dwordx4 %0, %1, off " FLUERE_DENSE_POLICY : "=v"(v[k]) : "v"(p) : "memory");
            }
            const uint32_t* po = dense ? B.offs : B.offs + li;
            asm volatile("global_load_dword %0, %1, off" : "=v"(osp) : "v"(po) : "memory");
        };
        uint32_t c = grab();
        uint2 dc = desc_of(c);
        dc.x = __builtin_amdgcn_readfirstlane(dc.x);
        dc.y = __builtin_amdgcn_readfirstlane(dc.y);
        issue(c, dc);
        uint32_t cn = grab();
        uint2 dn_v = desc_of(cn);
        while (c < nch) {
            const uint32_t c2 = grab();
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // chunk c's loads (issue) and dn_v
            const uint2 dn = make_uint2(__builtin_amdgcn_readfirstlane(dn_v.x), __builtin_amdgcn_readfirstlane(dn_v.y));
            Win W[1];
            uint32_t o1[1];
            const uint64_t lis[1] = {li_of(c)};
            bool live[1];
            if (dc.y) {
                // two halves of 32 records through a 160-piece slab: half h
                // needs pieces [2hS, 2hS + 160) of the span, record i its
                // five pieces at slab byte (i & 31) * S (16-byte aligned)
                uint4 r[2][5];
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const uint32_t p0 = 2u * h * dc.y;
#pragma unroll
                    for (int k = 0; k < 5; k++) {
                        const uint32_t sl = k * 64u + lane - p0;
                        if (sl < 160u) slab[sl] = make_uint4(v[k].x, v[k].y, v[k].z, v[k].w);
                    }
                    __builtin_amdgcn_wave_barrier();
                    asm volatile("" ::: "memory");
                    const uint4* sp = reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(slab) + (lane & 31u) * dc.y);
#pragma unroll
                    for (int k = 0; k < 5; k++) r[h][k] = sp[k];
                    __builtin_amdgcn_wave_barrier();
                    asm volatile("" ::: "memory");
                }
                const bool hi = lane >= 32u;
#pragma unroll
                for (int k = 0; k < 5; k++) {
                    W[0].w[4 * k + 0] = hi ? r[1][k].x : r[0][k].x;
                    W[0].w[4 * k + 1] = hi ? r[1][k].y : r[0][k].y;
                    W[0].w[4 * k + 2] = hi ? r[1][k].z : r[0][k].z;
                    W[0].w[4 * k + 3] = hi ? r[1][k].w : r[0][k].w;
                }
                o1[0] = dc.x + lane * dc.y;
                live[0] = true;  // dense chunks are whole
                pin_win(W[0]);
            } else {
                // the record's first 64 bytes (four 16-byte loads): all the
                // hot parser reads; an 80-byte window straddles one more
                // 64-byte memory segment for 3 in 16 alignments
                o1[0] = osp;
                const uint8_t* p = B.bytes + osp;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    uint4 q;
                    __builtin_memcpy(&q, p + 16 * k, 16);
                    W[0].w[4 * k + 0] = q.x; W[0].w[4 * k + 1] = q.y; W[0].w[4 * k + 2] = q.z; W[0].w[4 * k + 3] = q.w;
                }
                W[0].w[16] = W[0].w[17] = W[0].w[18] = W[0].w[19] = 0u;
                live[0] = lis[0] < end;
                pin_win(W[0]);
            }
            // pinned in each branch: after the merge no wait covers the window
            issue(cn < nch ? cn : c, cn < nch ? dn : make_uint2(0, 0));
            dn_v = desc_of(c2);
            process(W, o1, lis, live);
            c = cn;
            dc = dn;
            cn = c2;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last (unused) issue
        flush();
    }
    // sets of windows this workgroup did not have: empty segments
    for (uint32_t w = win; w < a.S.W; w++) {
        const uint32_t set = blockIdx.x * a.S.W + w;
        for (uint32_t oo = tid; oo <= a.S.O; oo += BLOCK) {
            a.S.off[(size_t)oo * a.S.n_sets + set] = 0;
            if (oo < a.S.O) a.S.soff[(size_t)oo * a.S.n_sets + set] = 0;
        }
    }
    // statistics: one record per workgroup (plain stores), summed by k_merge_partials
    if ((tid & 63) == 0 && d_loops && a.dbg) {
        atomicAdd(&s_cnt[3], (unsigned long long)d_loops);
        atomicAdd(&s_cnt[4], (unsigned long long)d_iters);
    }
    // wave reductions (shuffles), then one LDS atomic per wave and counter (a
    // 64-bit LDS atomic from every lane compiles to a 64-step lane loop)
    {
        uint32_t cv = (uint32_t)c_valid, cd = (uint32_t)c_drop, cm = (uint32_t)c_miss;
        unsigned long long tn = tmin, tx = tmax;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            cv += __shfl_xor(cv, o, 64);
            cd += __shfl_xor(cd, o, 64);
            cm += __shfl_xor(cm, o, 64);
            tn = min(tn, (unsigned long long)__shfl_xor(tn, o, 64));
            tx = max(tx, (unsigned long long)__shfl_xor(tx, o, 64));
        }
        if ((tid & 63) == 0) {
            if (cv) atomicAdd(&s_cnt[0], (unsigned long long)cv);
            if (cd) atomicAdd(&s_cnt[1], (unsigned long long)cd);
            if (cm) atomicAdd(&s_cnt[2], (unsigned long long)cm);
            if (cv) { atomicMin(&s_tmin, tn); atomicMax(&s_tmax, tx); }
        }
    }
    lds_barrier();  // LDS only: the flush's stores need not have completed here
    if (tid == 0) {
        unsigned long long* st = a.S.wgs + (size_t)blockIdx.x * WGS_N;
        st[0] = s_cnt[0];
        st[1] = s_cnt[1];
        st[2] = s_cnt[2];
        st[3] = s_cnt[0] ? s_tmin : NONE64;
        st[4] = s_cnt[0] ? s_tmax : 0;
        st[5] = clock64() - cyc_start;
        st[6] = cyc_flush;
        st[7] = cyc_wait;
        a.slow_cnt[blockIdx.x] = s_slow;
        if (s_slow) atomicAdd(a.slow_n, (unsigned long long)s_slow);
        // spills in owner segments: every LDS-table miss but the overflow
        if (s_cnt[2] > ovf_total) atomicAdd(&a.bc[2], s_cnt[2] - ovf_total);
        if (a.dbg) {
            const unsigned long long rt_end = wall_clock64();
            a.dbg[blockIdx.x * 8 + 0] = rt_start;
            a.dbg[blockIdx.x * 8 + 3] = rt_end;
            a.dbg[blockIdx.x * 8 + 7] = s_cnt[3] | (s_cnt[4] << 32);  // probe loops | iterations
        }
    }
}

// ---------------------------------------------------------------------------
// k_parse_spill: the hot pass for captures with many flows per window (the
// last run sent more than half of its packets past k_parse_agg's LDS table:
// C3/C4-like IMIX with 100k-1M flows).  No key table: every valid packet
// becomes a 24-byte record for its merge owner (seg_pack, kern.h), staged in
// an LDS bin per owner (O x BIN records, 128 KiB); a full bin leaves as one
// contiguous run of its owner's segment, written cooperatively by the wave
// that completed it (3*BIN lanes per bin: 8-byte pieces).
// k_parse_agg's scattered per-packet 32-byte stores into the owner segments
// were ~90 us of C3's 0.44-ms kernel (ablation: the same stores coalesced).
// The merge, the segments and the sets are k_parse_agg's (no partials).
// ---------------------------------------------------------------------------
constexpr int SPB_WORDS = 8192;  // LDS bins: 16-byte words (128 KiB); a record is 24 B (MACS: 64 B)

// MACS (-M): the canonical MAC pair joins the key; a segment record is the
// packed MAC form (segm_pack, kern.h: three 16-byte words), the raw overflow
// buffer's four words -- key, MAC words + hash, payload, zero
template <bool MACS>
__global__ void __launch_bounds__(BLOCK) k_parse_spill(AggArgs a) {
    constexpr uint32_t RU = MACS ? 4u : 2u;  // 16-byte words per record (the raw overflow buffer's form)
    // a bin record as it leaves for its owner segment: MACS the packed 48-byte
    // form (three 16-byte pieces), otherwise the packed 24-byte form (three 8-byte pieces)
    constexpr uint32_t PQ = MACS ? SEGM_U : SEG_Q;
    typedef typename std::conditional<MACS, uint4, uint2>::type Piece;
    __shared__ uint4 s_bin[SPB_WORDS];
    Piece* const s_bp = reinterpret_cast<Piece*>(s_bin);
    __shared__ uint32_t s_cl[MAX_OWNERS], s_wr[MAX_OWNERS];  // per bin: slots claimed / records written
    __shared__ uint32_t s_scnt[OWN_WORDS];                   // per owner: records in its segment (packed)
    __shared__ uint32_t s_chunk, s_nspill, s_slow;
    __shared__ unsigned long long s_sbase, s_cnt[3], s_tmin, s_tmax;
    const int tid = threadIdx.x;
    const Stage& S = a.S;
    const Batch& B = a.B;
    const uint32_t O = S.O;
    // Records per bin: a power of two, 16 (256 owners) .. 2 (2048); MACS 8 .. 1.
    // A completed bin leaves as 16-byte pieces, at most one wave's lanes of
    // them (MACS: three per record; otherwise the bin's BIN * 24 contiguous
    // bytes): 16 records (8 with MACS) = 384 B = three whole 128-B lines at
    // line-aligned segment positions
    uint32_t BIN;
    if constexpr (MACS) {
        const uint32_t fit = min((uint32_t)(SPB_WORDS / SEGM_U) / O, 64u / SEGM_U);
        BIN = fit >= 1 ? 1u << (31 - __builtin_clz(fit)) : 1u;  // (O <= 2048: fit >= 1)
    } else {
        const uint32_t fit = min((uint32_t)(SPB_WORDS * 2 / SEG_Q) / O, 64u * 2 / 3);
        BIN = fit >= 2 ? 1u << (31 - __builtin_clz(fit)) : 2u;  // (O <= 2048: fit >= 2)
    }
    const uint32_t PPB = MACS ? SEGM_U * BIN : BIN * 3 / 2;  // 16-byte pieces per bin
    for (uint32_t o = tid; o < MAX_OWNERS; o += BLOCK) s_cl[o] = s_wr[o] = 0;
    for (uint32_t o = tid; o < OWN_WORDS; o += BLOCK) s_scnt[o] = 0;
    if (tid < 3) s_cnt[tid] = 0;
    if (tid == 0) { s_tmin = NONE64; s_tmax = 0; s_chunk = 0; s_nspill = 0; s_slow = 0; }
    __syncthreads();
    const uint64_t n = B.n, G = gridDim.x, stride = G * BLOCK, beg = (uint64_t)blockIdx.x * BLOCK;
    const uint64_t nsteps = n > beg ? (n - beg + stride - 1) / stride : 0;
    const uint64_t lastp = n - 1;
    const uint32_t lane = tid & 63;
    constexpr uint32_t WAVES = BLOCK / 64;
    unsigned long long c_valid = 0, c_drop = 0, tmin = NONE64, tmax = 0;
    uint64_t wbase = beg;
    uint32_t win = 0, ovf_total = 0;
    const unsigned long long rt_start = wall_clock64();
    // a lane's overflow record (its owner segment is full): the workgroup's
    // raw buffer, listed at the window flush (k_parse_agg's overflow list)
    auto overflow = [&](uint32_t q, uint32_t h, uint4 v) {
        uint4* dst = reinterpret_cast<uint4*>(S.spill_raw) + (size_t)blockIdx.x * SPILL_WG * RU + (size_t)h * SPILL_WG + q;
        *dst = v;
    };
    for (uint64_t ws = 0; ws < nsteps; ws += WIN_ITERS) {
        const uint32_t set = blockIdx.x * S.W + win;
        const uint32_t nch = (uint32_t)min<uint64_t>(WIN_ITERS, nsteps - ws) * WAVES;
        Piece* seg0 = reinterpret_cast<Piece*>(S.dspill) + (size_t)set * O * S.cap_o * PQ;
        // record r of bin o, from LDS, in the raw overflow buffer's form (its word h)
        auto bin_rec = [&](uint32_t o, uint32_t r, uint32_t h) -> uint4 {
            if constexpr (MACS) {
                uint4 uu[SEGM_U];
#pragma unroll
                for (uint32_t i = 0; i < SEGM_U; i++) uu[i] = s_bin[(o * BIN + r) * SEGM_U + i];
                uint4 key, mac, pay;
                segm_unpack(uu, key, mac, pay);
                return h == 0 ? key : h == 1 ? mac : h == 2 ? pay : make_uint4(0, 0, 0, 0);
            } else {
                uint2 qq[SEG_Q];
#pragma unroll
                for (uint32_t i = 0; i < SEG_Q; i++) qq[i] = s_bp[(o * BIN + r) * SEG_Q + i];
                uint4 key, pay;
                seg_unpack(qq, key, pay);
                return h ? pay : key;
            }
        };
        auto li_of = [&](uint32_t c) -> uint64_t {
            return beg + (ws + c / WAVES) * stride + (uint64_t)(c % WAVES) * 64 + lane;
        };
        // the record offset of this lane's packet of chunk c (dense chunks: computed)
        auto off_of = [&](uint32_t c) -> uint32_t {
            const uint64_t li = min(li_of(c), lastp);
            const uint64_t ch = (li_of(c) - lane) >> 6;
            uint2 d = make_uint2(0, 0);
            if (ch < B.n_desc) d = B.desc[ch];
            return d.y ? d.x + lane * d.y : B.offs[li];
        };
        uint32_t c = 0;
        if (lane == 0) c = atomicAdd(&s_chunk, 1u);
        c = __builtin_amdgcn_readfirstlane(c);
        uint32_t off = c < nch ? off_of(c) : 0u;
        while (c < nch) {
            uint32_t cn = 0;
            if (lane == 0) cn = atomicAdd(&s_chunk, 1u);
            cn = __builtin_amdgcn_readfirstlane(cn);
            const uint64_t li = li_of(c);
            const bool live = li < n;
            Win W;
            {
                const uint8_t* p = B.bytes + off;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    uint4 q;
                    __builtin_memcpy(&q, p + 16 * k, 16);
                    W.w[4 * k + 0] = q.x; W.w[4 * k + 1] = q.y; W.w[4 * k + 2] = q.z; W.w[4 * k + 3] = q.w;
                }
                W.w[16] = W.w[17] = W.w[18] = W.w[19] = 0u;
            }
            const uint32_t off_n = cn < nch ? off_of(cn) : 0u;  // the next chunk's offset, in flight
            pin_win(W);
            Hot h;
            const uint32_t cls = live ? hot_parse(B, off, W, h) : HOT_DROP;
            c_drop += (live & (cls == HOT_DROP)) ? 1 : 0;
            const bool valid = live & (cls == HOT_OK);
            const bool slow = live & (cls == HOT_SLOW);
            // canonical key (lower endpoint first, flow_table.h; MACS: the MAC breaks a tie)
            const uint32_t sp = h.ports >> 16, dp = h.ports & 0xFFFFu;
            bool gt = (h.sip > h.dip) | ((h.sip == h.dip) & (sp > dp));
            uint32_t m0 = 0, m1 = 0, m2 = 0;
            if (MACS) {
                const uint64_t dmac = ((uint64_t)__builtin_amdgcn_perm(W.w[5], W.w[4], 0x00010203u) << 16) |
                                      __builtin_amdgcn_perm(W.w[5], W.w[4], 0x0C0C0405u);  // frame bytes 0..5
                const uint64_t smac = ((uint64_t)__builtin_amdgcn_perm(W.w[6], W.w[5], 0x02030405u) << 16) |
                                      __builtin_amdgcn_perm(W.w[6], W.w[5], 0x0C0C0607u);  // frame bytes 6..11
                if ((h.sip == h.dip) & (sp == dp)) gt = smac > dmac;
                const uint64_t lom = gt ? dmac : smac, him = gt ? smac : dmac;
                m0 = (uint32_t)(lom >> 16);
                m1 = ((uint32_t)(lom & 0xFFFF) << 16) | (uint32_t)(him & 0xFFFF);
                m2 = (uint32_t)(him >> 16);
            }
            const uint4 w_key = make_uint4(gt ? h.dip : h.sip, gt ? h.sip : h.dip,
                                           gt ? __builtin_amdgcn_alignbit(h.ports, h.ports, 16) : h.ports, h.proto << 24);
            const bool elig = (h.proto != 6u) | ((h.tf & 2u) != 0);
            const uint4 w_pay = make_uint4(h.doct, h.pkt | (h.ttl << 16) | ((elig ? 1u : 0u) << 24), (uint32_t)(li - wbase),
                                           h.tf | ((gt ? 1u : 0u) << 8));
            uint32_t hk = lt_hash(w_key.x, w_key.y, w_key.z, w_key.w);
            if (MACS) hk = mac_hash(hk, m0, m1, m2);
            const uint4 w_mac = make_uint4(m0, m1, m2, hk);
            const uint32_t o = owner_of(hk, O);
            if (!MACS && a.phash && live) a.phash[li] = valid ? ckey_bucket_v4(w_key.x, w_key.y, w_key.z, h.proto) : PH_PARSE;
            if (!MACS && a.exm && live) {  // the exact engine's ExMeta of this packet (k_ex_meta's fields)
                ExMeta m;
                m.t = h.t;
                m.gidx = B.first + li;
                m.d = valid ? 0u : FAIL;  // (the merge's flow word gives it; FAIL: not this parser's packet)
                m.pkt = h.pkt;
                m.doct = h.doct;
                m.dir = gt ? 1 : 0;
                m.tflags = (uint8_t)h.tf;
                m.ttl = (uint8_t)h.ttl;
                m.bits = (elig ? 1 : 0) | ((h.tf & 5u) ? 2 : 0);
                a.exm[li] = m;
                if (a.exm_t) a.exm_t[li] = h.t;
            }
            if (valid) {
                c_valid++;
                tmin = min(tmin, (unsigned long long)h.t);
                tmax = max(tmax, (unsigned long long)h.t);
            }
            // claim a bin slot, write the record, count it written; a lane whose
            // bin is full retries once the bin's completer has flushed it
            bool pend = valid;
            for (int it = 0; it < (1 << 16); it++) {
                if (__ballot(pend) == 0) break;
                uint32_t done = NONE32;
                if (pend) {
                    const uint32_t slot = atomicAdd(&s_cl[o], 1u);
                    if (slot < BIN) {
                        if constexpr (MACS) {
                            uint4 uu[SEGM_U];
                            segm_pack(w_key, w_mac, w_pay, uu);
#pragma unroll
                            for (uint32_t i = 0; i < SEGM_U; i++) s_bin[(o * BIN + slot) * SEGM_U + i] = uu[i];
                        } else {
                            uint2 qq[SEG_Q];
                            seg_pack(w_key, w_pay, qq);
#pragma unroll
                            for (uint32_t i = 0; i < SEG_Q; i++) s_bp[(o * BIN + slot) * SEG_Q + i] = qq[i];
                        }
                        __threadfence_block();
                        if (atomicAdd(&s_wr[o], 1u) + 1 == BIN) done = o;
                        pend = false;
                    }
                }
                // the bins completed this round: their segment positions, then
                // the wave writes them out, PPB lanes per bin
                uint32_t pos = 0;
                if (done != NONE32) pos = own_add_n(s_scnt, done, BIN);
                uint64_t fm = __ballot(done != NONE32);
                while (fm) {
                    const uint32_t j = lane / PPB, pc = lane % PPB;  // this lane: piece pc of the j-th bin of the group
                    uint64_t m = fm;
                    for (uint32_t k = 0; k < j && m; k++) m &= m - 1;
                    const bool act = m != 0 && j < 64 / PPB;  // (64 % PPB != 0: the spare lanes idle)
                    const uint32_t src = act ? (uint32_t)__builtin_ctzll(m) : 0u;
                    const uint32_t bo = __shfl(done, src, 64), bp = __shfl(pos, src, 64);
                    if constexpr (MACS) {
                        const uint32_t r = pc / SEGM_U, hh = pc % SEGM_U;
                        const bool ovf = act && bp + r >= S.cap_o;
                        uint32_t q = 0;  // (the overflow slot: from the record's first lane, every lane shuffling)
                        if (ovf && hh == 0) q = atomicAdd(&s_nspill, 1u);
                        q = __shfl(q, lane - hh, 64);
                        if (act) {
                            if (!ovf) {
                                seg0[((size_t)bo * S.cap_o + bp + r) * SEGM_U + hh] = s_bin[(bo * BIN + r) * SEGM_U + hh];
                            } else {  // past the segment's capacity: the raw buffer's four words
                                overflow(q, hh, bin_rec(bo, r, hh));
                                if (hh == 0) overflow(q, 3, make_uint4(0, 0, 0, 0));
                            }
                        }
                    } else {
                        // the whole bin inside the segment (an even capacity keeps
                        // the 16-byte pieces aligned): its bytes as they are in LDS
                        const bool whole = (S.cap_o & 1u) == 0 && bp + BIN <= S.cap_o;
                        if (act && whole) {
                            reinterpret_cast<uint4*>(S.dspill)[((size_t)set * O * S.cap_o + (size_t)bo * S.cap_o + bp) * 3 / 2 + pc] =
                                s_bin[bo * BIN * 3 / 2 + pc];
                        } else if (act && pc < BIN) {  // (rare) record by record; past the capacity: the overflow list
                            if (bp + pc < S.cap_o) {
#pragma unroll
                                for (uint32_t i = 0; i < SEG_Q; i++)
                                    seg0[((size_t)bo * S.cap_o + bp + pc) * SEG_Q + i] = s_bp[(bo * BIN + pc) * SEG_Q + i];
                            } else {
                                const uint32_t q = atomicAdd(&s_nspill, 1u);
                                overflow(q, 0, bin_rec(bo, pc, 0));
                                overflow(q, 1, bin_rec(bo, pc, 1));
                            }
                        }
                    }
                    // drop the group's bins (the first 64 / PPB set bits)
                    for (uint32_t k = 0; k < 64 / PPB && fm; k++) fm &= fm - 1;
                }
                if (done != NONE32) {  // (the wave's reads of the bin come first: LDS order)
                    atomicExch(&s_wr[done], 0u);
                    atomicExch(&s_cl[done], 0u);
                }
                if (__ballot(pend)) __builtin_amdgcn_s_sleep(1);
            }
            if (pend) atomicOr(a.T.err, ERR_SPIN);  // (cannot happen: a full bin's completer flushes it)
            // slow list: wave-aggregated append into this workgroup's region
            const uint64_t sm = __ballot(slow);
            if (sm) {
                const uint32_t lead = __builtin_ctzll(sm);
                uint32_t b0 = 0;
                if (lane == lead) b0 = atomicAdd(&s_slow, (uint32_t)__popcll(sm));
                b0 = __shfl(b0, lead, 64);
                if (slow)
                    a.slow[(size_t)blockIdx.x * a.slow_region + b0 +
                           __builtin_amdgcn_mbcnt_hi((uint32_t)(sm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)sm, 0u))] = (uint32_t)li;
            }
            c = cn;
            off = off_n;
        }
        // ---- window flush: the partly filled bins, then the set's segment counts
        __syncthreads();
        for (uint32_t o = tid; o < O; o += BLOCK) {
            const uint32_t k = s_wr[o];
            if (!k) continue;
            const uint32_t p0 = own_add_n(s_scnt, o, k);
            for (uint32_t r = 0; r < k; r++) {
                if (p0 + r < S.cap_o) {
                    Piece* d = seg0 + ((size_t)o * S.cap_o + p0 + r) * PQ;
#pragma unroll
                    for (uint32_t u = 0; u < PQ; u++) d[u] = s_bp[(o * BIN + r) * PQ + u];
                } else {
                    const uint32_t q = atomicAdd(&s_nspill, 1u);
#pragma unroll
                    for (uint32_t u = 0; u < RU; u++) overflow(q, u, bin_rec(o, r, u));
                }
            }
            s_cl[o] = s_wr[o] = 0;
        }
        __syncthreads();  // (every overflow record written before the list copy below)
        const uint32_t nsp = s_nspill;
        if (tid == 128) s_sbase = nsp ? atomicAdd(&a.bc[1], (unsigned long long)nsp) : 0ull;
        if (tid == 0) { ovf_total += nsp; S.base[set] = B.first + wbase; s_chunk = 0; }
        for (uint32_t o = tid; o <= O; o += BLOCK) {
            S.off[(size_t)o * S.n_sets + set] = 0;  // no partials
            if (o < O) S.soff[(size_t)o * S.n_sets + set] = min(own_get(s_scnt, o), S.cap_o);
        }
        __syncthreads();
        if (nsp) {  // overflow records -> the overflow list (the set in fl's high bits)
            const uint4* raw = reinterpret_cast<const uint4*>(S.spill_raw) + (size_t)blockIdx.x * SPILL_WG * RU;
            const unsigned long long sb = s_sbase;
            constexpr uint32_t PAY = RU == 4 ? 2u : 1u;  // the payload word (its fl field carries the set)
            for (uint32_t i = tid; i < nsp; i += BLOCK) {
                // (written by other waves of this workgroup: nontemporal loads bypass the CU's L1)
                typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
                uint4* dst = reinterpret_cast<uint4*>(S.spill) + (sb + i) * RU;
#pragma unroll
                for (uint32_t u = 0; u < RU; u++) {
                    const u32x4 kk = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(raw + u * SPILL_WG + i));
                    dst[u] = make_uint4(kk.x, kk.y, kk.z, kk.w | (u == PAY ? (set << 9) : 0u));
                }
            }
        }
        for (uint32_t o = tid; o < OWN_WORDS; o += BLOCK) s_scnt[o] = 0;
        if (tid == 0) s_nspill = 0;
        __syncthreads();
        wbase += stride * WIN_ITERS;
        win++;
    }
    // sets of windows this workgroup did not have: empty segments
    for (uint32_t w = win; w < S.W; w++) {
        const uint32_t set = blockIdx.x * S.W + w;
        for (uint32_t oo = tid; oo <= O; oo += BLOCK) {
            S.off[(size_t)oo * S.n_sets + set] = 0;
            if (oo < O) S.soff[(size_t)oo * S.n_sets + set] = 0;
        }
    }
    // statistics (k_parse_agg's per-workgroup record; every valid packet is a "miss")
    {
        uint32_t cv = (uint32_t)c_valid, cd = (uint32_t)c_drop;
        unsigned long long tn = tmin, tx = tmax;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            cv += __shfl_xor(cv, o, 64);
            cd += __shfl_xor(cd, o, 64);
            tn = min(tn, (unsigned long long)__shfl_xor(tn, o, 64));
            tx = max(tx, (unsigned long long)__shfl_xor(tx, o, 64));
        }
        if (lane == 0) {
            if (cv) atomicAdd(&s_cnt[0], (unsigned long long)cv);
            if (cd) atomicAdd(&s_cnt[1], (unsigned long long)cd);
            if (cv) { atomicMin(&s_tmin, tn); atomicMax(&s_tmax, tx); }
        }
    }
    __syncthreads();
    if (tid == 0) {
        unsigned long long* st = S.wgs + (size_t)blockIdx.x * WGS_N;
        st[0] = s_cnt[0];
        st[1] = s_cnt[1];
        st[2] = s_cnt[0];
        st[3] = s_cnt[0] ? s_tmin : NONE64;
        st[4] = s_cnt[0] ? s_tmax : 0;
        st[5] = st[6] = st[7] = 0;
        a.slow_cnt[blockIdx.x] = s_slow;
        if (s_slow) atomicAdd(a.slow_n, (unsigned long long)s_slow);
        if (s_cnt[0] > ovf_total) atomicAdd(&a.bc[2], s_cnt[0] - ovf_total);
        if (a.dbg) {
            a.dbg[blockIdx.x * 8 + 0] = rt_start;
            a.dbg[blockIdx.x * 8 + 1] = a.dbg[blockIdx.x * 8 + 2] = a.dbg[blockIdx.x * 8 + 3] = wall_clock64();
            a.dbg[blockIdx.x * 8 + 7] = 0;
        }
    }
}

const void* hot_kernel(int spill, int macs, int abl) {
    if (spill) return macs ? (const void*)k_parse_spill<true> : (const void*)k_parse_spill<false>;
    if (macs) return (const void*)k_parse_agg<0, true>;
    switch (abl) {
    case 1: return (const void*)k_parse_agg<1, false>;
    case 2: return (const void*)k_parse_agg<2, false>;
    case 3: return (const void*)k_parse_agg<3, false>;
    case 4: return (const void*)k_parse_agg<4, false>;
    case 5: return (const void*)k_parse_agg<5, false>;
    default: return (const void*)k_parse_agg<0, false>;
    }
}

}  // namespace fl
