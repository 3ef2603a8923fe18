// merge.hip -- after the hot pass on one GPU: the owner merge of the staged
// partials and spilled packets (k_merge_partials), the general-parser packets
// (k_slow), the certificate and the records (k_finalize), the sequential Mode B
// fallback (k_seq_*), and the per-run cleanup (k_cleanup).
#include "ctx.h"

namespace fl {


__device__ __forceinline__ void load_acc(const Acc& A, uint32_t d, AccVals& v) {
    v.fa = A.fa[d]; v.fc = A.fc[d]; v.fr = A.fr[d]; v.la = A.la[d];
#pragma unroll
    for (int q = 0; q < 2; q++) {
        v.pk[q] = A.pk[q][d];
        v.by[q] = A.by[q][d];
        v.mn[q] = A.mn[q][d];
        v.mx[q] = A.mx[q][d];
    }
#pragma unroll
    for (int q = 0; q < 8; q++) v.fl[q] = A.fl[q][d];
}

// Certified flow d -> its record; false when d has no record here (TCP flow
// without a SYN: dropped; complex: marked for the per-flow state machine;
// GEN false: a first packet the register parser declines is listed for
// k_finalize_gen, whose general parser would cost k_finalize its occupancy).
template <bool GEN>
__device__ __forceinline__ bool finalize_vals(const FinArgs& a, uint32_t d, const AccVals& v, fluere_record& r,
                                              bool& cplx, unsigned long long& cplx_pkts, bool one = false, Batch bone = Batch{}) {
    const unsigned long long fa = v.fa, fc = v.fc, fr = v.fr, la = v.la;
    if (fc == NONE64) return false;  // TCP flow without any SYN: every packet is dropped (:101-113)
    bool certified = fc == fa && (fr == NONE64 || fr == la);
    if (!certified) {
        a.complex[d] = 1;
        if (a.cbits) {
            const uint32_t b = ckey_bucket(reinterpret_cast<const uint32_t*>(a.T.flow_key + (size_t)d * 56));
            a.cbits[b] = 1;
        }
        cplx = true;
        cplx_pkts = v.pk[0] + v.pk[1];
        return false;
    }
    const bool macs = a.macs != 0;
    // the first and the last packet: both offsets, then both windows, in flight together
    // (one: a single batch, its descriptor `bone` loaded by the caller ahead of
    // the chain; passed by value -- a pointer to it would live in scratch)
    Batch BP = bone, BQ = bone;
    if (!one) {
        BP = a.bs[find_batch(a.bs, a.nb, fc)];
        BQ = a.bs[find_batch(a.bs, a.nb, la)];
    }
    const uint32_t op = BP.offs[fc - BP.first], oq = BQ.offs[la - BQ.first];
    Win WP;
    load_win(BP, op, WP);
    const uint64_t t_last = record_time(BQ, oq);  // the last packet: its time only
    pin_win(WP);
    Parsed P;
    if constexpr (GEN) {
        parse_loaded(BP, op, WP, macs, 0, P);
    } else {
        parse_loaded_fast(BP, op, WP, macs, P);
        if (P.cls == 2) {  // IPv6, VXLAN, IPv4 options: parse_mid over the 128-byte window
            Win32 W32;
            load_win32(BP, op, W32);
            parse_loaded32<0>(BP, op, W32, macs, P);
        }
        if (P.cls == 2) {  // the general parser's classes (ARP, VLAN, raw fallback ...)
            a.defer[atomicAdd(&a.g->n_fdefer, 1ull)] = d;
            return false;
        }
    }
    const uint8_t cd = canon_dir(P, macs);
    fill_seed(r, P);
    const uint32_t p0 = v.pk[0], p1 = v.pk[1];
    const unsigned long long b0 = v.by[0], b1 = v.by[1];
    r.d_pkts = p0 + p1;
    r.d_octets = b0 + b1;
    r.out_pkts = cd ? p1 : p0; r.in_pkts = cd ? p0 : p1;
    r.out_bytes = cd ? b1 : b0; r.in_bytes = cd ? b0 : b1;
    r.min_pkt = v.mn[0]; r.max_pkt = v.mx[0];
    r.min_ttl = (uint8_t)v.mn[1]; r.max_ttl = (uint8_t)v.mx[1];
    for (int q = 0; q < 8; q++) r.cnt[q] = v.fl[q];
    r.cnt[8] = 0;
    r.last = t_last;
    r.order_key = (fr == la) ? la : NONE64;
    return true;
}

template <bool GEN>
__device__ __forceinline__ bool finalize_one(const FinArgs& a, uint32_t d, fluere_record& r, bool& cplx,
                                             unsigned long long& cplx_pkts) {
    AccVals v;
    load_acc(a.A, d, v);
    return finalize_vals<GEN>(a, d, v, r, cplx, cplx_pkts);
}

// emit + complex-flow counters of one wave's flows (every lane of the wave)
__device__ __forceinline__ void finalize_emit(EmitLds& S, const FinArgs& a, const fluere_record& r, bool want, bool cplx,
                                              unsigned long long cplx_pkts) {
    emit_record_block(S, a.g, a.out, a.out_cap, r, want);
    const uint64_t cm = __ballot(cplx);
    if (cm) {
        const unsigned long long pk = wave_sum(cplx_pkts);
        if ((uint32_t)(threadIdx.x & 63) == (uint32_t)__builtin_ctzll(cm)) {
            atomicAdd(&a.g->n_complex, (unsigned long long)__popcll(cm));
            atomicAdd(&a.g->n_complex_pkts, pk);
        }
    }
}


// (MACS: a run with MAC keys -- the entries' MAC sidecars; a kernel of its own
// so the 5-tuple runs keep 16 KiB of LDS and none of the MAC paths' code)
template <bool MACS>
__global__ void __launch_bounds__(MB) k_merge_partials(AggArgs a) {
    __shared__ uint4 m_key[MT];
    __shared__ uint4 m_kx[MACS ? MT : 1];  // MAC runs: the MAC sidecar of each entry (w = 1 once written)
    __shared__ uint32_t m_pk[2][MT], m_mn[2][MT], m_mx[2][MT], m_fl[8][MT];
    __shared__ unsigned long long m_by[2][MT], m_fa[MT], m_fc[MT], m_fr[MT], m_la[MT];
    __shared__ uint32_t m_nclaim, m_base;
    // per set of the current chunk: this owner's first record (index into the
    // partials or the spill planes), its start in the flattened index space,
    // and the window's first packet (relative to the batch): a record's
    // loads then depend on LDS reads only
    __shared__ uint32_t m_lo[MCH], m_start[MCH], m_wb[MCH], m_scan[MB / 64 + 1];
    // per group of 64 flattened indices: the set holding its first index (the
    // spill records' wave-uniform search, one LDS read instead of a binary search)
    constexpr uint32_t MGRP = 2048;
    __shared__ uint16_t m_grp[MGRP];
    const int tid = threadIdx.x;
    const unsigned long long c0 = clock64();
    if (a.dbg && tid == 0) a.dbg[4096 * 8 - 2048 + blockIdx.x * 8 + 0] = wall_clock64();
    // loads issued before the LDS initialisation (their latency overlaps it):
    // this owner's segment bounds of the first set chunk, and the run counters
    const unsigned long long n_spill_all = __hip_atomic_load(&a.bc[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long n_dspill_all = __hip_atomic_load(&a.bc[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long n_slow_all = __hip_atomic_load(a.slow_n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    constexpr bool macs = MACS;
    const Stage& S = a.S;
    auto reduce_stats = [&]() {
        // the hot kernel's per-workgroup statistics -> the run counters (one wave)
        unsigned long long v[WGS_N] = {0, 0, 0, NONE64, 0, 0, 0, 0};
        for (uint32_t w = tid; w < S.n_wg; w += 64) {
            const unsigned long long* st = S.wgs + (size_t)w * WGS_N;
#pragma unroll
            for (int k = 0; k < WGS_N; k++) v[k] = k == 3 ? min(v[k], st[k]) : k == 4 ? max(v[k], st[k]) : v[k] + st[k];
        }
#pragma unroll
        for (int k = 0; k < WGS_N; k++)
            for (int d = 32; d >= 1; d >>= 1) {
                const unsigned long long o = __shfl_xor(v[k], d, 64);
                v[k] = k == 3 ? min(v[k], o) : k == 4 ? max(v[k], o) : v[k] + o;
            }
        if (tid == 0) {
            Glob* g = a.g;
            if (a.bc != &g->n_slow && a.bc[0]) atomicAdd(&g->n_slow, a.bc[0]);  // (the run's slow-list total)
            if (v[0]) atomicAdd(&g->valid, v[0]);
            if (v[1]) atomicAdd(&g->dropped, v[1]);
            if (v[2]) atomicAdd(&g->n_kc_miss, v[2]);
            if (v[0]) { atomicMin(&g->tmin, v[3]); atomicMax(&g->tmax, v[4]); }
            atomicAdd(&g->cyc_total, v[5]);
            atomicAdd(&g->cyc_flush, v[6]);
            atomicAdd(&g->cyc_flush0, v[7]);
        }
    };
    // Owners o = blockIdx.x, + gridDim.x, ...: the grid is at most one workgroup
    // per CU (one merge table fills a CU's LDS), so a workgroup merges several
    // owners in turn rather than being dispatched again for each.
    // Owner blockIdx.x first; with more owners than workgroups the rest are
    // claimed from a counter (Glob::n_owner), so a workgroup that finishes
    // early takes the next one (owners' record phases spread, e.g. C3 99-199
    // us).  No counter when every workgroup has one owner.
    __shared__ uint32_t s_me;
    if (tid == 0) s_me = a.tail_only ? S.O : blockIdx.x;  // (tail_only: k_merge_spill took the owners)
    __syncthreads();
    const int pass0 = S.no_parts ? 1 : 0;  // (no partials: the segments' pass alone)
    for (uint32_t me = s_me; me < S.O; me = s_me) {
        // the first chunk's bounds, loaded before the LDS initialisation
        // (partials: their offsets; no partials: the segments' counts)
        uint32_t pre_lo[MCH / MB], pre_hi[MCH / MB];
        unsigned long long pre_wb[MCH / MB];
    #pragma unroll
        for (int q = 0; q < MCH / MB; q++) {
            const uint32_t set = tid * (MCH / MB) + q;
            const bool in = set < a.S.n_sets;
            pre_lo[q] = in && !pass0 ? a.S.off[(size_t)me * a.S.n_sets + set] : 0;
            pre_hi[q] = !in ? 0 : pass0 ? a.S.soff[(size_t)me * a.S.n_sets + set] : a.S.off[(size_t)(me + 1) * a.S.n_sets + set];
            pre_wb[q] = in ? a.S.base[set] : 0;
        }
        for (int e = tid; e < MT; e += MB) {
            m_key[e] = make_uint4(0, 0, 0, 0);
            if (MACS) m_kx[e] = make_uint4(0, 0, 0, 0);
            m_pk[0][e] = m_pk[1][e] = 0;
            m_by[0][e] = m_by[1][e] = 0;
            m_mn[0][e] = m_mn[1][e] = NONE32;
            m_mx[0][e] = m_mx[1][e] = 0;
    #pragma unroll
            for (int q = 0; q < 8; q++) m_fl[q][e] = 0;
            m_fa[e] = m_fc[e] = m_fr[e] = NONE64;
            m_la[e] = 0;
        }
        __syncthreads();
        if (a.dbg && tid == 0) a.dbg[4096 * 8 - 2048 + blockIdx.x * 8 + 1] = wall_clock64();
        // This owner's segment of every set, flattened: per chunk of MCH sets, an
        // exclusive scan of the segment lengths; threads then take partials from
        // the flattened index space (binary search for the set), so every thread
        // has about (partials / MB) of them with all their loads in flight.
        // Pass 0 takes the staged partials, pass 1 the spilled packets in this
        // owner's segments (each a one-packet partial), through the same
        // machinery; the overflow list is the tail's.
        const int passes = n_dspill_all ? 2 : 1;  // no spills: one pass
        for (int pass = FLUERE_MERGE_NOPART ? 1 : pass0; pass < passes; pass++)
        for (uint32_t c0s = 0; c0s < S.n_sets; c0s += MCH) {
            const uint32_t nset = min((uint32_t)MCH, S.n_sets - c0s);
            const uint32_t* offs = pass ? S.soff : S.off;
            uint32_t len[MCH / MB], tot = 0;
    #pragma unroll
            for (int q = 0; q < MCH / MB; q++) {
                const uint32_t set = c0s + tid * (MCH / MB) + q;
                uint32_t lo = 0, hi = 0;
                unsigned long long wb = 0, rb = 0;
                if (pass == pass0 && c0s == 0) {  // prefetched
                    lo = pre_lo[q];
                    hi = pre_hi[q];
                    wb = pre_wb[q];
                } else if (set < c0s + nset) {
                    lo = pass ? 0u : offs[(size_t)me * S.n_sets + set];
                    hi = offs[(size_t)(pass ? me : me + 1) * S.n_sets + set];  // pass 1: the segment's count
                    wb = S.base[set];
                }
                rb = !pass ? (unsigned long long)set * NS
                     : set < S.n_hot ? ((unsigned long long)set * S.O + me) * S.cap_o
                                     : S.slow_rec0 + ((unsigned long long)(set - S.n_hot) * S.O + me) * S.cap_s;
                m_lo[tid * (MCH / MB) + q] = (uint32_t)(rb + lo);
                m_wb[tid * (MCH / MB) + q] = (uint32_t)(wb - a.B.first);
                len[q] = hi - lo;
                tot += len[q];
            }
            uint32_t run = block_exclusive_scan(tot, m_scan) ;
            const uint32_t total = m_scan[MB / 64];  // (block_exclusive_scan ends with a barrier)
            const bool grp = pass == 1 && total <= 64u * MGRP;
    #pragma unroll
            for (int q = 0; q < MCH / MB; q++) {
                m_start[tid * (MCH / MB) + q] = run;
                if (grp && len[q])
                    for (uint32_t g = (run + 63) >> 6; g <= (run + len[q] - 1) >> 6; g++)
                        m_grp[g] = (uint16_t)(tid * (MCH / MB) + q);
                run += len[q];
            }
            __syncthreads();
            if (a.dbg && tid == 0 && c0s == 0 && pass == 0) a.dbg[4096 * 8 - 2048 + blockIdx.x * 8 + 2] = wall_clock64();
            // one record (a staged partial or a spilled packet): find or claim
            // its merge entry, then the update (or the global path)
            auto merge_rec = [&](uint32_t h, uint32_t k0, uint32_t k1, uint32_t k2, uint32_t tag, uint32_t x0,
                                 uint32_t x1, uint32_t x2, const FlowPart& f) {
                    // find or claim the merge entry (same protocol as the hot kernel)
                    uint32_t e = (h * 0x85EBCA77u) >> 22;  // 10 bits: MT == 1024
                    int state = 0, probes = 0;
                    for (int it = 0; it < 128; it++) {
                        if (state == 0) {
                            const uint4 kk = m_key[e];
                            bool xm = true;
                            if (macs) {  // MAC words
                                const uint4 xx = m_kx[MACS ? e : 0];
                                xm = xx.w == 1u && xx.x == x0 && xx.y == x1 && xx.z == x2;
                            }
                            if (kk.w & LT_READY) {
                                if (kk.w == (tag | LT_READY) && kk.x == k0 && kk.y == k1 && kk.z == k2 && xm) state = 1;
                                else if (++probes == 64) state = 2;
                                else e = (e + 1) & (MT - 1);
                            } else if (kk.w == 0 && atomicCAS(&m_key[e].w, 0u, LT_CLAIM) == 0u) {
                                m_key[e].x = k0;
                                m_key[e].y = k1;
                                m_key[e].z = k2;
                                if (MACS) m_kx[e] = make_uint4(x0, x1, x2, 1u);
                                __threadfence_block();
                                atomicExch(&m_key[e].w, tag | LT_READY);
                                state = 1;
                            }
                        }
                        if (__ballot(state == 0) == 0) break;
                    }
                    if (state == 1) {
                        // Many records land on one entry (a flow's partials from every
                        // set, its spilled packets), and LDS atomics on one address
                        // serialise: min / max and first / last positions are read
                        // first and written only where the record moves them (values
                        // move monotonically, so a stale read costs at most a
                        // redundant atomic).
    #if FLUERE_MERGE_GUARD
                        const uint32_t gmn0 = m_mn[0][e], gmn1 = m_mn[1][e], gmx0 = m_mx[0][e], gmx1 = m_mx[1][e];
                        const unsigned long long gfa = m_fa[e], gfc = m_fc[e], gla = m_la[e];
    #else
                        const uint32_t gmn0 = NONE32, gmn1 = NONE32, gmx0 = 0, gmx1 = 0;
                        const unsigned long long gfa = NONE64, gfc = NONE64, gla = 0;
    #endif
    #pragma unroll
                        for (int q = 0; q < 2; q++) {
                            if (f.pk[q]) {
                                atomicAdd(&m_pk[q][e], f.pk[q]);
                                atomicAdd(&m_by[q][e], f.by[q]);
                            }
                            if (f.mn[q] < (q ? gmn1 : gmn0) || !FLUERE_MERGE_GUARD) atomicMin(&m_mn[q][e], f.mn[q]);
                            if (f.mx[q] > (q ? gmx1 : gmx0) || !FLUERE_MERGE_GUARD) atomicMax(&m_mx[q][e], f.mx[q]);
                        }
    #pragma unroll
                        for (int q = 0; q < 8; q++)
                            if (f.fl[q]) atomicAdd(&m_fl[q][e], f.fl[q]);
                        if (f.fa != NONE64 && f.fa < gfa) atomicMin(&m_fa[e], f.fa);
                        if (f.fc != NONE64 && f.fc < gfc) atomicMin(&m_fc[e], f.fc);
                        if (f.fr != NONE64) atomicMin(&m_fr[e], f.fr);
                        if (f.la && (f.la > gla || !FLUERE_MERGE_GUARD)) atomicMax(&m_la[e], f.la);
                    } else {
                        uint32_t d;
                        if (macs && tag != 0xFF000000u) {
                            CKey ck;
                            mac_ckey(k0, k1, k2, tag, x0, x1, x2, ck);
                            d = dense_of_key(a.T, ck, true, a.A.slots, nullptr);
                        } else {
                            d = staged_id(a.T, a.v6, k0, k1, k2, tag, a.A.slots);
                        }
                        if (d != FAIL && d < a.T.fmax) part_to_global(a.A, d, f);
                    }
            };
            if (pass == 1) {
                // Spilled packets, the lean path (MAC runs: 48-byte records,
                // the MAC words and the hash beside the key): the merge is
                // instruction-bound (PMC on C3: 28 % of wave time issuing at
                // 4 waves per SIMD, 14k VALU + 7k SALU instructions per wave),
                // so no binary search per record (the wave's first index is
                // searched once, each lane steps forward over the few sets
                // its index is past) and update_flow of one packet written
                // out directly instead of through a FlowPart.
                // the set of flattened index id (the wave's smallest index
                // searched once, each lane stepping forward past the few sets
                // its index is beyond)
                auto set_of = [&](uint32_t id) -> uint32_t {
                    const uint32_t iw = __builtin_amdgcn_readfirstlane(id);
                    uint32_t lo_i = 0, hi_i = nset - 1;
                    if (grp) {
                        lo_i = m_grp[iw >> 6];  // (the set of the group's first index: a lower bound)
                    } else {
                        while (lo_i < hi_i) {
                            const uint32_t mid = (lo_i + hi_i + 1) >> 1;
                            if (m_start[mid] <= iw) lo_i = mid;
                            else hi_i = mid - 1;
                        }
                    }
                    while (lo_i + 1 < nset && m_start[lo_i + 1] <= id) lo_i++;
                    return lo_i;
                };
                // one record ahead: the next iteration's record is loaded
                // while this one is probed and aggregated in LDS
                // (MACS: the packed 48-byte form; otherwise the packed 24-byte form)
                auto load_rec = [&](size_t rix, uint4& k, uint4& p, uint4& x) {
                    if constexpr (MACS) {
                        const uint4* src = reinterpret_cast<const uint4*>(S.dspill) + rix * SEGM_U;
                        uint4 uu[SEGM_U];
#pragma unroll
                        for (uint32_t i = 0; i < SEGM_U; i++) uu[i] = src[i];
                        segm_unpack(uu, k, x, p);
                    } else {
                        seg_load(reinterpret_cast<const uint2*>(S.dspill), rix, k, p);
                    }
                };
                uint32_t lo_n = 0;
                uint4 n0 = make_uint4(0, 0, 0, 0), n1 = n0, nx = n0;
                if ((uint32_t)tid < total) {
                    lo_n = set_of(tid);
                    load_rec((size_t)m_lo[lo_n] + ((uint32_t)tid - m_start[lo_n]), n0, n1, nx);
                }
                for (uint32_t idx = tid; idx < total; idx += MB) {
                    const uint32_t lo_i = lo_n;
                    const uint4 v0 = n0, v1 = n1, vx = nx;  // key, payload, (MACS) MAC words + hash
                    if (idx + MB < total) {
                        lo_n = set_of(idx + MB);
                        load_rec((size_t)m_lo[lo_n] + (idx + MB - m_start[lo_n]), n0, n1, nx);
                    }
                    const unsigned long long gi = a.B.first + m_wb[lo_i] + v1.z;
                    const uint32_t k0 = v0.x, k1 = v0.y, k2 = v0.z, tag = v0.w;
                    if (FLUERE_MERGE_ABL == 1) {  // diagnostics: the loads alone
                        if ((k0 ^ k1 ^ k2 ^ v1.x ^ v1.y) == 0x12345678u) atomicAdd(&m_pk[0][0], 1u);
                        continue;
                    }
                    const uint32_t h = MACS ? vx.w : lt_hash(k0, k1, k2, tag);
                    uint32_t e = (h * 0x85EBCA77u) >> 22;  // 10 bits: MT == 1024
                    int state = 0, probes = 0;
                    for (int it = 0; it < 128; it++) {  // find or claim (the hot kernel's protocol)
                        if (state == 0) {
                            const uint4 kk = m_key[e];
                            bool xm = true;
                            if (MACS) {  // the MAC words (the sidecar is written before the entry is published)
                                const uint4 xx = m_kx[MACS ? e : 0];
                                xm = xx.w == 1u && xx.x == vx.x && xx.y == vx.y && xx.z == vx.z;
                            }
                            if (kk.w & LT_READY) {
                                if (kk.w == (tag | LT_READY) && kk.x == k0 && kk.y == k1 && kk.z == k2 && xm) state = 1;
                                else if (++probes == 64) state = 2;
                                else e = (e + 1) & (MT - 1);
                            } else if (kk.w == 0 && atomicCAS(&m_key[e].w, 0u, LT_CLAIM) == 0u) {
                                m_key[e].x = k0;
                                m_key[e].y = k1;
                                m_key[e].z = k2;
                                if (MACS) m_kx[MACS ? e : 0] = make_uint4(vx.x, vx.y, vx.z, 1u);
                                __threadfence_block();
                                atomicExch(&m_key[e].w, tag | LT_READY);
                                state = 1;
                            }
                        }
                        if (__ballot(state == 0) == 0) break;
                    }
                    const uint32_t dir = (v1.w >> 8) & 1u, tf = v1.w & 0xFFu;
                    const uint32_t pkt = v1.y & 0xFFFFu, ttl = (v1.y >> 16) & 0xFFu;
                    if (FLUERE_MERGE_ABL == 2) {  // diagnostics: the probe, no updates
                        if (state == 1 && pkt == 0x1234u) atomicAdd(&m_pk[0][e], 1u);
                        continue;
                    }
                    if (a.pid && state == 1) a.pid[gi - a.pid_base] = PH_EREF | (a.pid_batch << 21) | (me << 10) | e;
                    if (state == 1) {  // update_flow of one packet (flows.rs:11-42), order-free part
                        atomicAdd(&m_pk[dir][e], 1u);
                        atomicAdd(&m_by[dir][e], (unsigned long long)v1.x);
                        const uint32_t gmn0 = m_mn[0][e], gmn1 = m_mn[1][e], gmx0 = m_mx[0][e], gmx1 = m_mx[1][e];
                        const unsigned long long gfa = m_fa[e], gfc = m_fc[e], gla = m_la[e];
                        if (pkt < gmn0) atomicMin(&m_mn[0][e], pkt);
                        if (ttl < gmn1) atomicMin(&m_mn[1][e], ttl);
                        if (pkt > gmx0) atomicMax(&m_mx[0][e], pkt);
                        if (ttl > gmx1) atomicMax(&m_mx[1][e], ttl);
                        for (uint32_t t = tf; t; t &= t - 1) atomicAdd(&m_fl[__builtin_ctz(t)][e], 1u);
                        if (gi < gfa) atomicMin(&m_fa[e], gi);
                        if (((v1.y >> 24) & 1u) && gi < gfc) atomicMin(&m_fc[e], gi);
                        if (tf & 5u) atomicMin(&m_fr[e], gi);
                        if (gi + 1 > gla) atomicMax(&m_la[e], gi + 1);
                    } else {  // no entry within 64 probes: the global path
                        FlowPart f;
                        spill_to_part(v1.x, v1.y, v1.z, v1.w, a.B.first + m_wb[lo_i], f);
                        uint32_t d;
                        if (MACS && tag != 0xFF000000u) {
                            CKey ck;
                            mac_ckey(k0, k1, k2, tag, vx.x, vx.y, vx.z, ck);
                            d = dense_of_key(a.T, ck, true, a.A.slots, nullptr);
                        } else {
                            d = staged_id(a.T, a.v6, k0, k1, k2, tag, a.A.slots);
                        }
                        if (d != FAIL && d < a.T.fmax) part_to_global(a.A, d, f);
                        if (a.pid && d != FAIL && d < a.T.fmax) a.pid[gi - a.pid_base] = PH_ID | d;
                    }
                }
                __syncthreads();
                continue;
            }
            if (FLUERE_MERGE_NOPART) continue;
            for (uint32_t idx = tid; idx < total; idx += MB) {
                uint32_t lo_i = 0, hi_i = nset - 1;  // last set with start <= idx
                while (lo_i < hi_i) {
                    const uint32_t mid = (lo_i + hi_i + 1) >> 1;
                    if (m_start[mid] <= idx) lo_i = mid;
                    else hi_i = mid - 1;
                }
                const unsigned long long base = a.B.first + m_wb[lo_i];
                uint32_t h, k0, k1, k2, tag, x0 = 0, x1 = 0, x2 = 0;
                FlowPart f;
                if (pass == 0) {
                    const size_t o = (size_t)m_lo[lo_i] + (idx - m_start[lo_i]);
                    Part p;
                    const uint4* src = reinterpret_cast<const uint4*>(S.part + o);
                    uint4 v[5];
    #pragma unroll
                    for (int q = 0; q < 5; q++) v[q] = src[q];
                    __builtin_memcpy(&p, v, sizeof p);  // (a lean partial's last two words are stale: unused)
                    h = p.h; k0 = p.k0; k1 = p.k1; k2 = p.k2; tag = p.tag & ~PART_LEAN;
                    if (macs) {
                        const uint4 xx = S.partx[o];
                        x0 = xx.x; x1 = xx.y; x2 = xx.z;
                    }
                    part_of_stage(p, base, f);
                } else {
                    const size_t o = (size_t)m_lo[lo_i] + (idx - m_start[lo_i]);
                    if (macs) {  // the packed MAC form (segm_pack)
                        const uint4* src = reinterpret_cast<const uint4*>(S.dspill) + o * (size_t)SEGM_U;
                        uint4 uu[SEGM_U], v0, v1, v2;
#pragma unroll
                        for (uint32_t i = 0; i < SEGM_U; i++) uu[i] = src[i];
                        segm_unpack(uu, v0, v1, v2);
                        k0 = v0.x; k1 = v0.y; k2 = v0.z; tag = v0.w;
                        x0 = v1.x; x1 = v1.y; x2 = v1.z;
                        h = v1.w;
                        spill_to_part(v2.x, v2.y, v2.z, v2.w, base, f);
                    } else {  // the packed 24-byte form (kern.h seg_pack)
                        uint4 v0, v1;
                        seg_load(reinterpret_cast<const uint2*>(S.dspill), o, v0, v1);
                        k0 = v0.x; k1 = v0.y; k2 = v0.z; tag = v0.w;
                        h = lt_hash(k0, k1, k2, tag);
                        spill_to_part(v1.x, v1.y, v1.z, v1.w, base, f);
                    }
                }
                merge_rec(h, k0, k1, k2, tag, x0, x1, x2, f);
            }
            __syncthreads();
        }
        // Dense ids: thread per entry (MT == MB).  The owner is the only inserter
        // of its keys, so a claim (EMPTY -> PENDING) normally succeeds at once;
        // the new ids of the whole workgroup come from ONE atomicAdd on the flow
        // counter (a single hot address: per-flow increments would serialise).
        if (a.dbg && tid == 0) a.dbg[4096 * 8 - 2048 + blockIdx.x * 8 + 3] = wall_clock64();
        static_assert(MT == MB, "one merge entry per thread");
        if (tid == 0) m_nclaim = 0;
        __syncthreads();
        const unsigned long long c1 = clock64();
        const int e = tid;
        const uint4 kk = m_key[e];
        const bool have = (kk.w & LT_READY) != 0;
        const uint32_t tag = kk.w & 0xFF000000u;
        uint32_t d = FAIL, s0 = FAIL, s1 = FAIL, rank = 0;
        bool claimed = false, wait = false;
        unsigned long long* val = nullptr;
        if (have) {
            if (kk.w & V6_TAG) {  // an IPv6 5-tuple from k_slow: the full key from the address ids
                CKey ck;
                v6_ckey(a.v6, kk.x, kk.y, kk.z, tag, ck);
                d = dense_of_key(a.T, ck, true, a.A.slots, &a.g->generic_used);
            } else if (tag == 0xFF000000u) {
                d = kk.x;  // MAC kernels' partials carry dense ids
            } else if (macs) {  // a spilled MAC-kernel key: one dictionary walk per flow and owner
                const uint4 xx = m_kx[MACS ? e : 0];
                CKey ck;
                mac_ckey(kk.x, kk.y, kk.z, tag, xx.x, xx.y, xx.z, ck);
                d = dense_of_key(a.T, ck, true, a.A.slots, nullptr);
            } else if (!v4_fast(a.T, tag >> 24)) {  // wide tables: protocols other than TCP / UDP
                d = staged_id(a.T, a.v6, kk.x, kk.y, kk.z, tag, a.A.slots);
            } else {       // IPv4 5-tuple: flow_table.h chain T0 (ip pair) -> T1 (slot, ports, proto)
                unsigned long long v = EMPTY;
                v4_slots(a.T, kk.x, kk.y, kk.z, tag >> 24, true, s0, s1, &v);
                if (s1 != FAIL) {
                    val = &a.T.tab[1][2 * s1 + 1];
                    if (v >= PENDING) v = atomicCAS(val, EMPTY, PENDING);
                    if (v == EMPTY) {
                        claimed = true;
                        rank = atomicAdd(&m_nclaim, 1u);
                    } else if (v == PENDING) {
                        wait = true;
                    } else {
                        d = (uint32_t)v;
                    }
                }
            }
        }
        __syncthreads();
        if (a.dbg && tid == 0) a.dbg[4096 * 8 - 2048 + blockIdx.x * 8 + 7] = wall_clock64();
        if (tid == 0) m_base = m_nclaim ? atomicAdd(a.T.n_flows, m_nclaim) : 0;
        __syncthreads();
        if (a.dbg && tid == 0) a.dbg[4096 * 8 - 2048 + blockIdx.x * 8 + 6] = wall_clock64();
        if (claimed) {
            d = m_base + rank;
            if (d >= a.T.fmax) {
                atomicOr(a.T.err, ERR_FLOWS_FULL);
                d = FAIL;
            } else {
                uint32_t* dst = (uint32_t*)(a.T.flow_key + (size_t)d * 56);
    #pragma unroll
                for (int k = 0; k < 14; k++) dst[k] = k == 0 ? kk.x : k == 4 ? kk.y : k == 8 ? kk.z : k == 9 ? tag >> 24 : 0;
    #pragma unroll
                for (int j = 0; j < N_TABLES; j++) a.A.slots[(size_t)d * N_TABLES + j] = j == 0 ? s0 : j == 1 ? s1 : NONE32;
            }
            atomicExch(val, (unsigned long long)d);
        }
        for (int sp = 0; sp < (1 << 20); sp++) {  // a claim held elsewhere: poll (wave-uniform)
            if (__ballot(wait) == 0) break;
            if (wait) {
                const unsigned long long v = __hip_atomic_load(val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (v != PENDING && v != EMPTY) {
                    d = (uint32_t)v;
                    wait = false;
                }
            }
            if (__ballot(wait) != 0) __builtin_amdgcn_s_sleep(16);
        }
        if (wait) atomicOr(a.T.err, ERR_SPIN);
        if (a.dbg && tid == 0) a.dbg[4096 * 8 - 2048 + blockIdx.x * 8 + 4] = wall_clock64();
        if (a.emap) a.emap[((size_t)a.pid_batch << 21) | ((size_t)me << 10) | (uint32_t)e] = (have && d < a.T.fmax) ? d : FAIL;
        if (have && d != FAIL && d < a.T.fmax) {
            FlowPart f;
    #pragma unroll
            for (int q = 0; q < 2; q++) {
                f.pk[q] = m_pk[q][e];
                f.by[q] = m_by[q][e];
                f.mn[q] = m_mn[q][e];
                f.mx[q] = m_mx[q][e];
            }
    #pragma unroll
            for (int q = 0; q < 8; q++) f.fl[q] = m_fl[q][e];
            f.fa = m_fa[e];
            f.fc = m_fc[e];
            f.fr = m_fr[e];
            f.la = m_la[e];
            part_to_global(a.A, d, f);
        }
        if (a.dbg && tid == 0) a.dbg[4096 * 8 - 2048 + blockIdx.x * 8 + 5] = wall_clock64();
        if (tid == 0 && a.dbg) {  // diagnostics: contended atomics, debug runs only
            atomicAdd(&a.g->cyc_m_scan, c1 - c0);
            atomicAdd(&a.g->cyc_m_ids, clock64() - c1);
        }
        __syncthreads();  // (the next owner re-initialises the table)
        if (tid == 0) s_me = S.O > gridDim.x ? gridDim.x + (uint32_t)atomicAdd(&a.bc[4], 1ull) : S.O;
        __syncthreads();
    }
    // the hot kernel's per-workgroup statistics -> the run counters (one wave
    // of the last workgroup, off the other owners' critical path)
    if (blockIdx.x == gridDim.x - 1 && tid < 64) reduce_stats();
    // k_slow ran: its general-parser list (flat); else the whole slow list
    const unsigned long long n_gen_all =
        a.slow_kernel ? __hip_atomic_load(&a.bc[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
    const bool tail_slow = a.slow_kernel ? n_gen_all != 0 : n_slow_all != 0;
    if (FLUERE_MERGE_TAIL && (tail_slow || n_spill_all)) {
        // The tail: the overflow list (spills past their owner segment's
        // capacity: full keys, no parse) and the packets for the general
        // parser: the whole slow list (packets the hot kernel left over: IPv6,
        // IPv4 options, ARP, VXLAN, VLAN, other IP protocols, short frames),
        // or, when k_slow ran, the ones parse_fast / parse_mid left to it.
        // Each record: dense id from the dictionary, then update_flow's
        // order-free part pre-aggregated per dense id in this workgroup's LDS
        // entries (reused: the owner's flows are in the global accumulators);
        // an id with no entry within 32 probes takes the global atomics.
        // Grid-stride over device-side counts (no host round trip).
        __syncthreads();
        for (int e = tid; e < MT; e += MB) {
            m_key[e].x = NONE32;
            m_pk[0][e] = m_pk[1][e] = 0;
            m_by[0][e] = m_by[1][e] = 0;
            m_mn[0][e] = m_mn[1][e] = NONE32;
            m_mx[0][e] = m_mx[1][e] = 0;
#pragma unroll
            for (int q = 0; q < 8; q++) m_fl[q][e] = 0;
            m_fa[e] = m_fc[e] = m_fr[e] = NONE64;
            m_la[e] = 0;
        }
        // single-word keys (the dense id): a CAS claims or finds an entry,
        // nothing to publish, so the bounded probe needs no other lane
        auto put = [&](uint32_t d, const FlowPart& f) {
            uint32_t e = (d * 0x9E3779B1u) >> 22;  // 10 bits: MT == 1024
            for (int pr = 0; pr < 32; pr++) {
                const uint32_t k = atomicCAS(&m_key[e].x, NONE32, d);
                if (k == NONE32 || k == d) {
#pragma unroll
                    for (int q = 0; q < 2; q++) {
                        if (f.pk[q]) {
                            atomicAdd(&m_pk[q][e], f.pk[q]);
                            atomicAdd(&m_by[q][e], f.by[q]);
                        }
                        atomicMin(&m_mn[q][e], f.mn[q]);
                        atomicMax(&m_mx[q][e], f.mx[q]);
                    }
#pragma unroll
                    for (int q = 0; q < 8; q++)
                        if (f.fl[q]) atomicAdd(&m_fl[q][e], f.fl[q]);
                    if (f.fa != NONE64) atomicMin(&m_fa[e], f.fa);
                    if (f.fc != NONE64) atomicMin(&m_fc[e], f.fc);
                    if (f.fr != NONE64) atomicMin(&m_fr[e], f.fr);
                    if (f.la) atomicMax(&m_la[e], f.la);
                    return;
                }
                e = (e + 1) & (MT - 1);
            }
            part_to_global(a.A, d, f);
        };
        const unsigned long long gstride = (unsigned long long)gridDim.x * MB;
        for (unsigned long long i = (unsigned long long)blockIdx.x * MB + tid; i < n_spill_all; i += gstride) {
            const uint4* src = reinterpret_cast<const uint4*>(S.spill) + i * (macs ? 4 : 2);
            const uint4 v0 = src[0], v1 = src[1];
            uint32_t x0 = 0, x1 = 0, x2 = 0;
            uint4 pay = v1;
            if (macs) {
                pay = src[2];
                x0 = v1.x; x1 = v1.y; x2 = v1.z;
            }
            FlowPart f;
            const unsigned long long wbase = (pay.w >> 9) == SPILL_BATCH_REL ? a.B.first : S.base[pay.w >> 9];
            spill_to_part(pay.x, pay.y, pay.z, pay.w, wbase, f);
            uint32_t d;
            if (macs && v0.w != 0xFF000000u) {
                CKey ck;
                mac_ckey(v0.x, v0.y, v0.z, v0.w, x0, x1, x2, ck);
                d = dense_of_key(a.T, ck, true, a.A.slots, nullptr);
            } else {
                d = staged_id(a.T, a.v6, v0.x, v0.y, v0.z, v0.w, a.A.slots);
            }
            if (d != FAIL && d < a.T.fmax) put(d, f);
            if (a.pid && d != FAIL && d < a.T.fmax) a.pid[wbase + pay.z - a.pid_base] = PH_ID | d;
        }
        if (tail_slow) {
            // the hot workgroups' regions, flattened: exclusive scan of their counts
            const uint32_t nwg = S.n_wg;  // <= MB
            const uint32_t cnt = tid < (int)nwg ? a.slow_cnt[tid] : 0u;
            const uint32_t st0 = block_exclusive_scan(cnt, m_scan);
            if (tid < (int)nwg) m_start[tid] = st0;
            __syncthreads();
            const unsigned long long n = a.slow_kernel ? n_gen_all : (unsigned long long)m_scan[MB / 64];
            unsigned long long c_valid = 0, c_drop = 0, tmin = NONE64, tmax = 0;
            for (unsigned long long i = (unsigned long long)blockIdx.x * MB + tid; i < n; i += gstride) {
                uint64_t li;
                if (a.slow_kernel) {
                    li = a.gen[i];
                } else {
                    uint32_t lo_w = 0, hi_w = nwg - 1;  // last region with start <= i
                    while (lo_w < hi_w) {
                        const uint32_t mid = (lo_w + hi_w + 1) >> 1;
                        if (m_start[mid] <= i) lo_w = mid;
                        else hi_w = mid - 1;
                    }
                    li = a.slow[(size_t)lo_w * a.slow_region + (i - m_start[lo_w])];
                }
                if (a.slow_abl == 2) { c_drop += li == NONE32; continue; }
                Parsed P;
                parse_record(a.B, li, macs, 1, P);
                if (P.cls) { c_drop++; continue; }
                c_valid++;
                tmin = min(tmin, (unsigned long long)P.t);
                tmax = max(tmax, (unsigned long long)P.t);
                uint8_t dir = 0;
                const uint32_t d = a.slow_abl == 1 ? (P.pi.sip[3] ^ P.pi.dip[3] ^ P.pi.ksp) % 8192u
                                                   : flow_of(a.T, P, macs, true, dir, a.A.slots, &a.g->generic_used);
                if (d == FAIL || d >= a.T.fmax) continue;
                FlowPart f;
                pkt_to_part(P.pi, dir, a.B.first + li, f);
                put(d, f);
                if (a.pid) a.pid[a.B.first + li - a.pid_base] = PH_ID | d;
            }
            // run counters: one set of atomics per wave
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                c_valid += __shfl_xor(c_valid, o, 64);
                c_drop += __shfl_xor(c_drop, o, 64);
                tmin = min(tmin, (unsigned long long)__shfl_xor(tmin, o, 64));
                tmax = max(tmax, (unsigned long long)__shfl_xor(tmax, o, 64));
            }
            if ((tid & 63) == 0) {
                if (c_valid) { atomicAdd(&a.g->valid, c_valid); atomicMin(&a.g->tmin, tmin); atomicMax(&a.g->tmax, tmax); }
                if (c_drop) atomicAdd(&a.g->dropped, c_drop);
            }
        }
        __syncthreads();
        for (int e = tid; e < MT; e += MB) {
            const uint32_t d = m_key[e].x;
            if (d == NONE32) continue;
            FlowPart f;
#pragma unroll
            for (int q = 0; q < 2; q++) {
                f.pk[q] = m_pk[q][e];
                f.by[q] = m_by[q][e];
                f.mn[q] = m_mn[q][e];
                f.mx[q] = m_mx[q][e];
            }
#pragma unroll
            for (int q = 0; q < 8; q++) f.fl[q] = m_fl[q][e];
            f.fa = m_fa[e];
            f.fc = m_fc[e];
            f.fr = m_fr[e];
            f.la = m_la[e];
            part_to_global(a.A, d, f);
        }
    }
}


// ---------------------------------------------------------------------------
// k_slow: the slow list (packets the hot parser left over) when the last run
// had one (the host predicts it; otherwise k_merge_partials' tail takes it).
// Runs between the hot kernel and the merge.  Workgroup b takes slow-list
// entries [b * SLOW_SET, (b + 1) * SLOW_SET) of the hot workgroups' regions
// flattened, as staging set n_hot + b.  Per packet: the 128-byte window,
// parse_fast / parse_mid in registers (the rest -- ARP, VLAN, short frames,
// drops -- go to a list for the general parser in the merge tail: inlined
// here, its registers would cost every packet occupancy); then a spill
// record into its merge owner's segment of the set, like the hot kernel's
// LDS-table misses: an IPv4 key as its words (no dictionary walk here: the
// owner resolves each key once), any other key (IPv6, -M, the raw fallback's
// protocol 255) as its dense id from the dictionary.  k_merge_partials then
// aggregates them with the hot kernel's partials.
// ---------------------------------------------------------------------------
// Records of a set's owners are staged in per-owner LDS bins (non-MAC runs;
// SLB_WORDS 16-byte words, 2 per record): a full bin leaves as one contiguous
// run of its owner's segment.  A record written straight to its owner
// segment (one 32-byte store pair per packet, scattered over O segments) cost
// ~230 us of the slow-all step (FLUERE_SLOW_ABL=3: 1.076 -> 0.691 ms).
#ifndef FLUERE_SLB_WORDS
#define FLUERE_SLB_WORDS 2048
#endif
constexpr uint32_t SLB_WORDS = FLUERE_SLB_WORDS;

__global__ void __launch_bounds__(SB) k_slow(AggArgs a) {
    __shared__ uint32_t s_start[MB + 1];
    __shared__ uint32_t s_scnt[OWN_WORDS];  // records per owner (packed 16-bit: a set has <= SLOW_SET)
    __shared__ uint4 s_bin[SLB_WORDS];       // per-owner bins (BINS records of 2 words each)
    __shared__ uint32_t s_cl[SLB_WORDS / 2], s_wr[SLB_WORDS / 2];  // per bin: slots claimed / records written
    const int tid = threadIdx.x;
    const bool macs = a.macs != 0;
    const Stage& S = a.S;
    const uint32_t O = S.O;
    const uint32_t set = S.n_hot + blockIdx.x;
    const int spu = spill_units(macs);
    for (int o = tid; o < OWN_WORDS; o += SB) s_scnt[o] = 0;
    const uint32_t BINS = macs ? 0u : SLB_WORDS / 2 / O;  // records per bin (< 2: no bins)
    const bool bins = BINS >= 2;
    for (uint32_t o = tid; o < SLB_WORDS / 2; o += SB) s_cl[o] = s_wr[o] = 0;
    // the hot workgroups' regions, flattened (wave 0: an exclusive scan, an
    // even run of regions per lane)
    const uint32_t nwg = S.n_wg;  // <= MB
    if (tid < 64 && !a.slow_all) {
        const uint32_t per = (nwg + 63) / 64;
        uint32_t sum = 0;
        for (uint32_t q = 0; q < per; q++) {
            const uint32_t w = tid * per + q;
            if (w < nwg) sum += a.slow_cnt[w];
        }
        uint32_t incl = sum;
#pragma unroll
        for (int dlt = 1; dlt < 64; dlt <<= 1) {
            const uint32_t y = __shfl_up(incl, dlt, 64);
            if (tid >= dlt) incl += y;
        }
        uint32_t run = incl - sum;
        for (uint32_t q = 0; q < per; q++) {
            const uint32_t w = tid * per + q;
            if (w < nwg) {
                s_start[w] = run;
                run += a.slow_cnt[w];
            }
        }
        if (tid == 63) s_start[MB] = incl;
    }
    __syncthreads();
    const unsigned long long n = a.slow_all ? a.B.n : s_start[MB];
    const unsigned long long i0 = (unsigned long long)blockIdx.x * SLOW_SET;
    const unsigned long long i1 = min(n, i0 + SLOW_SET);
    unsigned long long c_valid = 0, c_drop = 0, c_seg = 0, tmin = NONE64, tmax = 0;
    for (unsigned long long ib = i0; ib < i1; ib += SB) {  // (uniform)
        const unsigned long long i = ib + tid;
        bool rec = false, gen = false;
        uint32_t ow = 0, gli = 0;
        Parsed P;
        uint4 wk = make_uint4(0, 0, 0, 0), wx = make_uint4(0, 0, 0, 0), wp = make_uint4(0, 0, 0, 0);
        if (i < i1) {
            uint32_t li = (uint32_t)i;
            if (!a.slow_all) {
                uint32_t lo_w = 0, hi_w = nwg - 1;  // last region with start <= i
                while (lo_w < hi_w) {
                    const uint32_t mid = (lo_w + hi_w + 1) >> 1;
                    if (s_start[mid] <= i) lo_w = mid;
                    else hi_w = mid - 1;
                }
                li = a.slow[(size_t)lo_w * a.slow_region + (i - s_start[lo_w])];
            }
            const uint32_t off = a.B.offs[li];
            Win32 W;
            load_win32(a.B, off, W);
            pin_win32(W);
            if (a.slow_abl == 2) {  // diagnostics: no parse (wrong results)
                P.cls = 0;
                P.t = W.w[0];
                P.pi.v6 = 0; P.pi.kproto = 17; P.pi.sip[0] = W.w[9] & 0xF; P.pi.dip[0] = W.w[10] & 0xF;
                P.pi.sip[1] = P.pi.sip[2] = P.pi.sip[3] = P.pi.dip[1] = P.pi.dip[2] = P.pi.dip[3] = 0;
                P.pi.ksp = (uint16_t)(W.w[11] & 7); P.pi.kdp = (uint16_t)(W.w[12] & 7);
                P.pi.tflags = 0; P.pi.rprot = 17; P.pi.doctets = W.w[13] & 0xFFFF; P.pi.rpkt = W.w[14] & 0xFFFF; P.pi.rttl = 1;
                P.smac = P.dmac = 0;
            } else {
                parse_loaded32<0>(a.B, off, W, macs, P);
            }
            gen = P.cls == 2;
            if (gen) {
                gli = li;
            } else if (P.cls) {
                c_drop++;
            } else {
                c_valid++;
                tmin = min(tmin, (unsigned long long)P.t);
                tmax = max(tmax, (unsigned long long)P.t);
                const PktInfo& pi = P.pi;
                uint8_t dir = 0;
                CKey k;
                canon_key(P, macs, k, dir);
                uint32_t h;
                uint32_t ia = FAIL, ib = FAIL;
                if (!macs && pi.v6 && a.v6.C) v6_ids(a.v6, &k.w[0], &k.w[4], ia, ib);
                if (!macs && !pi.v6 && pi.kproto != 0xFF) {
                    // an IPv4 key: its words, as the hot kernel's spills carry them
                    wk = make_uint4(k.w[0], k.w[4], k.w[8], (uint32_t)pi.kproto << 24);
                    h = lt_hash(wk.x, wk.y, wk.z, wk.w);
                    rec = true;
                } else if (ia != FAIL && ib != FAIL) {
                    // an IPv6 key: the ids of its two addresses (no dictionary walk here)
                    wk = make_uint4(ia, ib, k.w[8], ((uint32_t)pi.kproto << 24) | V6_TAG);
                    h = lt_hash(wk.x, wk.y, wk.z, wk.w);
                    rec = true;
                } else {
                    const uint32_t d = a.slow_abl == 1 ? (k.w[3] ^ k.w[7] ^ k.w[8]) % 8192u  // diagnostics: no dictionary
                                                       : dense_of_key(a.T, k, true, a.A.slots, &a.g->generic_used);
                    wk = make_uint4(d, 0, 0, 0xFF000000u);
                    h = lt_hash(d, 0, 0, 0xFF000000u);
                    rec = d != FAIL && d < a.T.fmax;
                }
                const uint32_t tf = pi.tflags;
                const bool elig = (pi.rprot != 6) | ((tf & 2u) != 0);
                wp = make_uint4(pi.doctets, pi.rpkt | ((uint32_t)pi.rttl << 16) | ((elig ? 1u : 0u) << 24), li,
                                tf | ((uint32_t)dir << 8));
                wx = make_uint4(0, 0, 0, h);
                ow = owner_of(h, O);
            }
        }
        // the general parser's packets: the merge tail's list (wave-aggregated append)
        const uint64_t gm = __ballot(gen);
        if (gm) {
            const uint32_t lead = __builtin_ctzll(gm);
            unsigned long long b0 = 0;
            if ((uint32_t)(tid & 63) == lead) b0 = atomicAdd(&a.bc[3], (unsigned long long)__popcll(gm));
            b0 = __shfl(b0, lead, 64);
            if (gen) a.gen[b0 + __builtin_amdgcn_mbcnt_hi((uint32_t)(gm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)gm, 0u))] = gli;
        }
        if (a.slow_abl == 3) rec = false;  // diagnostics: no spill records
        // the segment position of a record past a full segment: the overflow list below
        // (bins: runs without MACs; the segment holds the packed 24-byte form)
        auto seg_put = [&](uint32_t o, uint32_t p, const uint4& k0, const uint4& k1) -> bool {
            if (p >= S.cap_s) return false;
            seg_store(reinterpret_cast<uint2*>(S.dspill), S.slow_rec0 + ((size_t)blockIdx.x * O + o) * S.cap_s + p, k0, k1);
            return true;
        };
        auto ovf_put = [&](const uint4& k0, uint4 k1) {  // (rare: a key that fills its owner's whole segment)
            const unsigned long long b0 = atomicAdd(&a.bc[1], 1ull);
            uint4* dst = reinterpret_cast<uint4*>(S.spill) + b0 * 2;
            k1.w |= set << 9;
            dst[0] = k0;
            dst[1] = k1;
        };
        // a length the packed segment forms cannot hold (none from 16-bit IP
        // length fields): the overflow list, before any segment count is taken
        const bool big = rec && wp.x >= SEG_DOCT_MAX;
        if (big && bins) {
            ovf_put(wk, wp);
            rec = false;
        }
        if (bins) {
            // claim a bin slot, write the record, count it written; the lane that
            // completes a bin writes it out; a lane whose bin is full retries
            // once the completer has emptied it
            bool pend = rec;
            for (int it = 0; it < (1 << 16); it++) {
                if (__ballot(pend) == 0) break;
                uint32_t done = NONE32;
                if (pend) {
                    const uint32_t slot = atomicAdd(&s_cl[ow], 1u);
                    if (slot < BINS) {
                        uint4* b = &s_bin[(ow * BINS + slot) * 2];
                        b[0] = wk;
                        b[1] = wp;
                        __threadfence_block();
                        if (atomicAdd(&s_wr[ow], 1u) + 1 == BINS) done = ow;
                        pend = false;
                    }
                }
                if (done != NONE32) {
                    const uint32_t p0 = own_add_n(s_scnt, done, BINS);
                    // two records at a time (three 16-byte stores at an even position)
                    for (uint32_t r = 0; r < BINS; r += 2) {
                        const uint4 k0 = s_bin[(done * BINS + r) * 2], k1 = s_bin[(done * BINS + r) * 2 + 1];
                        if (r + 1 < BINS && p0 + r + 1 < S.cap_s) {
                            const uint4 j0 = s_bin[(done * BINS + r + 1) * 2], j1 = s_bin[(done * BINS + r + 1) * 2 + 1];
                            seg_store2(reinterpret_cast<uint2*>(S.dspill),
                                       S.slow_rec0 + ((size_t)blockIdx.x * O + done) * S.cap_s + p0 + r, k0, k1, j0, j1);
                            c_seg += 2;
                            continue;
                        }
                        for (uint32_t u = r; u < min(r + 2, BINS); u++) {
                            const uint4 x0 = s_bin[(done * BINS + u) * 2], x1 = s_bin[(done * BINS + u) * 2 + 1];
                            if (seg_put(done, p0 + u, x0, x1)) c_seg++;
                            else ovf_put(x0, x1);
                        }
                    }
                    atomicExch(&s_wr[done], 0u);  // (this lane's reads of the bin come first: LDS order)
                    atomicExch(&s_cl[done], 0u);
                }
                if (__ballot(pend)) __builtin_amdgcn_s_sleep(1);
            }
            if (pend) atomicOr(a.T.err, ERR_SPIN);  // (cannot happen: a full bin's completer empties it)
            continue;
        }
        const uint32_t pos = rec && !big ? own_add(s_scnt, ow) : 0u;
        const bool ovf = rec && (big || pos >= S.cap_s);
        if (rec && !ovf) {
            const size_t rix = S.slow_rec0 + ((size_t)blockIdx.x * O + ow) * S.cap_s + pos;
            if (macs) {  // the packed MAC form (segm_pack)
                uint4 uu[SEGM_U];
                segm_pack(wk, wx, wp, uu);
                uint4* dst = reinterpret_cast<uint4*>(S.dspill) + rix * SEGM_U;
#pragma unroll
                for (uint32_t i = 0; i < SEGM_U; i++) dst[i] = uu[i];
            } else {
                seg_store(reinterpret_cast<uint2*>(S.dspill), rix, wk, wp);
            }
            c_seg++;
        }
        // past the segment's capacity: the overflow list (wave-aggregated append; rare)
        const uint64_t om = __ballot(ovf);
        if (om) {
            const uint32_t lead = __builtin_ctzll(om);
            unsigned long long b0 = 0;
            if ((uint32_t)(tid & 63) == lead) b0 = atomicAdd(&a.bc[1], (unsigned long long)__popcll(om));
            b0 = __shfl(b0, lead, 64);
            if (ovf) {
                const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(om >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)om, 0u));
                uint4* dst = reinterpret_cast<uint4*>(S.spill) + (b0 + r) * (size_t)(2 * spu);
                wp.w |= set << 9;
                dst[0] = wk;
                if (macs) {
                    dst[1] = wx;
                    dst[2] = wp;
                } else {
                    dst[1] = wp;
                }
            }
        }
    }
    __syncthreads();
    if (bins) {  // the partly filled bins
        for (uint32_t o = tid; o < O; o += SB) {
            const uint32_t k = s_wr[o];
            if (!k) continue;
            const uint32_t p0 = own_add_n(s_scnt, o, k);
            for (uint32_t r = 0; r < k; r++) {
                const uint4 k0 = s_bin[(o * BINS + r) * 2];
                uint4 k1 = s_bin[(o * BINS + r) * 2 + 1];
                if (p0 + r < S.cap_s) {
                    seg_store(reinterpret_cast<uint2*>(S.dspill), S.slow_rec0 + ((size_t)blockIdx.x * O + o) * S.cap_s + p0 + r,
                              k0, k1);
                    c_seg++;
                } else {
                    const unsigned long long b0 = atomicAdd(&a.bc[1], 1ull);
                    uint4* dst = reinterpret_cast<uint4*>(S.spill) + b0 * 2;
                    k1.w |= set << 9;
                    dst[0] = k0;
                    dst[1] = k1;
                }
            }
        }
        __syncthreads();
    }
    // this set's segments: record counts, no partials, positions relative to the batch
    for (uint32_t o = tid; o <= O; o += SB) {
        S.off[(size_t)o * S.n_sets + set] = 0;
        if (o < O) S.soff[(size_t)o * S.n_sets + set] = min(own_get(s_scnt, o), S.cap_s);
    }
    if (tid == 0) S.base[set] = a.B.first;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        c_valid += __shfl_xor(c_valid, o, 64);
        c_drop += __shfl_xor(c_drop, o, 64);
        c_seg += __shfl_xor(c_seg, o, 64);
        tmin = min(tmin, (unsigned long long)__shfl_xor(tmin, o, 64));
        tmax = max(tmax, (unsigned long long)__shfl_xor(tmax, o, 64));
    }
    if ((tid & 63) == 0) {
        if (c_valid) { atomicAdd(&a.g->valid, c_valid); atomicMin(&a.g->tmin, tmin); atomicMax(&a.g->tmax, tmax); }
        if (c_drop) atomicAdd(&a.g->dropped, c_drop);
        if (c_seg) atomicAdd(&a.bc[2], c_seg);
    }
}


// k_finalize: one thread per flow (grid-stride); records appended per
// workgroup (emit_record_block).
// The record is built in place in the block's LDS staging (S.rec[thread]):
// held in registers it took the kernel to 250 VGPRs (2 waves per SIMD).
__global__ void __launch_bounds__(EMIT_BLOCK) k_finalize(FinArgs a) {
    // loaded together, ahead of the flow count they would otherwise wait for:
    // the first flow's accumulators (every dense id below fmax is allocated)
    // and, with one batch, its descriptor -- one dependent round trip less
    const uint32_t d_pre = blockIdx.x * blockDim.x + threadIdx.x;
    AccVals v_pre;
    if (d_pre < a.T.fmax) load_acc(a.A, d_pre, v_pre);
    const Batch b_pre = a.bs[0];
    const Glob& gg = *a.g;
    const bool mode_b = a.timeout_us && gg.valid && gg.tmax - gg.tmin >= a.timeout_us;
    const uint32_t nf = mode_b ? 0u : min(*a.T.n_flows, a.T.fmax);
    __shared__ EmitLds S;
    __shared__ unsigned long long s_tot[4];  // updates, ended, complex flows, their packets (this workgroup)
    if (threadIdx.x < 4) s_tot[threadIdx.x] = 0;
    unsigned long long tot[2] = {0, 0}, n_cplx = 0, cplx_all = 0;  // (thread 0's totals: updates, ended)
    for (uint32_t d0 = blockIdx.x * blockDim.x; d0 < nf; d0 += gridDim.x * blockDim.x) {
        const uint32_t d = d0 + threadIdx.x;
        fluere_record& r = S.rec[threadIdx.x];
        bool cplx = false;
        unsigned long long cplx_pkts = 0;
        bool want = false;
        if (d < nf) {
            AccVals v = v_pre;
            if (d != d_pre) load_acc(a.A, d, v);
            want = finalize_vals<false>(a, d, v, r, cplx, cplx_pkts, a.nb == 1, b_pre);
        }
        const unsigned long long ok = want ? r.order_key : NONE64;
        emit_inplace_block(S, a.g, a.out, a.out_cap, want, want ? r.d_pkts : 0u, ok != NONE64, nullptr, 0, 0, tot,
                           a.rbits);
        if (a.kbits && ok != NONE64) {  // (the ordering behind the pass: k_so_*)
            const unsigned long long q = ok - a.kbase;
            atomicOr(&a.kbits[q >> 5], 1u << (q & 31));
        }
        n_cplx += cplx ? 1 : 0;
        cplx_all += cplx_pkts;
    }
    // the workgroup's counters: one set of global atomics (per-block or
    // per-wave atomics on these few words serialised a million-flow run)
    n_cplx = wave_sum(n_cplx);
    cplx_all = wave_sum(cplx_all);
    if ((threadIdx.x & 63) == 0 && n_cplx) {
        atomicAdd(&s_tot[2], n_cplx);
        atomicAdd(&s_tot[3], cplx_all);
    }
    if (threadIdx.x == 0) {
        s_tot[0] = tot[0];
        s_tot[1] = tot[1];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (s_tot[0]) atomicAdd(&a.g->n_updates, s_tot[0]);
        if (s_tot[1]) atomicAdd(&a.g->n_ended, s_tot[1]);
        if (s_tot[2]) {
            atomicAdd(&a.g->n_complex, s_tot[2]);
            atomicAdd(&a.g->n_complex_pkts, s_tot[3]);
        }
    }
    if (a.host_ctl) publish_ctl(a.g, &a.g->fin_done, a.host_ctl, a.seq);
}

// k_finalize_gen: the flows k_finalize listed (first packet outside the
// register parser's classes), with the general parser.
__global__ void __launch_bounds__(EMIT_BLOCK) k_finalize_gen(FinArgs a) {
    const uint32_t n = (uint32_t)min(a.g->n_fdefer, (unsigned long long)a.T.fmax);
    __shared__ EmitLds S;
    for (uint32_t i0 = blockIdx.x * blockDim.x; i0 < n; i0 += gridDim.x * blockDim.x) {
        const uint32_t i = i0 + threadIdx.x;
        fluere_record r;
        bool cplx = false;
        unsigned long long cplx_pkts = 0;
        const bool want = i < n && finalize_one<true>(a, a.defer[i], r, cplx, cplx_pkts);
        finalize_emit(S, a, r, want, cplx, cplx_pkts);
    }
}

__global__ void __launch_bounds__(256) k_seq_meta(SeqMetaArgs a) {
    uint64_t li = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (li >= a.B.n) return;
    const bool macs = a.macs != 0;
    Parsed P;
    parse_record(a.B, li, macs, 0, P);
    SeqMeta m;
    m.d = NONE32;
    m.dir = 0; m.tflags = 0; m.rprot_tcp = 0; m.ttl = 0; m.pkt = 0; m.doctets = 0; m.t = P.t;
    if (P.cls == 0) {
        uint8_t dir;
        uint32_t d = flow_of(a.T, P, macs, false, dir, nullptr, nullptr);
        m.d = d == FAIL ? NONE32 : d;
        m.dir = dir; m.tflags = P.pi.tflags; m.rprot_tcp = P.pi.rprot == 6; m.ttl = P.pi.rttl;
        m.pkt = P.pi.rpkt; m.doctets = P.pi.doctets;
    }
    a.meta[a.B.first + li - a.base] = m;
}

__device__ __forceinline__ bool h_less(const HeapEnt& x, const HeapEnt& y) {
    return x.exp < y.exp || (x.exp == y.exp && x.seq < y.seq);
}

__global__ void __launch_bounds__(64) k_seq_run(SeqArgs a) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    unsigned long long hn = 0, seq = 0, nout = 0;
    auto emit = [&](const fluere_record& r) {
        if (nout < a.out_cap) { a.out[nout] = r; a.out[nout].order_key = nout; }
        nout++;
    };
    for (unsigned long long gi = 0; gi < a.n; gi++) {  // offline_fluereflows.rs:68-176
        SeqMeta m = a.meta[gi];
        if (m.d == NONE32) continue;
        uint32_t d = m.d;
        bool rev;
        if (a.active[d]) {
            rev = m.dir != a.cdir[d];
        } else {
            if (m.rprot_tcp && !(m.tflags & 2)) continue;  // :101-113 (no sweep either)
            Parsed P;
            parse_global(a.bs, a.nb, gi + a.base, a.macs != 0, P);
            fill_seed(a.cur[d], P);
            a.active[d] = 1;
            a.cdir[d] = m.dir;
            HeapEnt e{m.t + a.timeout_us, seq++, d, m.dir};
            unsigned long long i = hn++;
            a.heap[i] = e;
            while (i) {
                unsigned long long p = (i - 1) / 2;
                if (!h_less(a.heap[i], a.heap[p])) break;
                HeapEnt t = a.heap[i]; a.heap[i] = a.heap[p]; a.heap[p] = t; i = p;
            }
            rev = false;
        }
        fluere_record& r = a.cur[d];
        PktInfo pi;
        pi.doctets = m.doctets; pi.rpkt = m.pkt; pi.rttl = m.ttl; pi.tflags = m.tflags;
        update_flow(r, rev, pi, m.t);
        if (m.tflags & 5) { emit(r); a.active[d] = 0; }
        while (hn && a.heap[0].exp <= m.t) {  // :161-175
            HeapEnt top = a.heap[0];
            // the entry holds the creator Key: it removes whatever flow is now
            // stored under that exact (oriented) key
            if (a.active[top.d] && a.cdir[top.d] == top.dir) { emit(a.cur[top.d]); a.active[top.d] = 0; }
            a.heap[0] = a.heap[--hn];
            unsigned long long i = 0;
            for (;;) {
                unsigned long long l = 2 * i + 1, rr = l + 1, mm = i;
                if (l < hn && h_less(a.heap[l], a.heap[mm])) mm = l;
                if (rr < hn && h_less(a.heap[rr], a.heap[mm])) mm = rr;
                if (mm == i) break;
                HeapEnt t = a.heap[i]; a.heap[i] = a.heap[mm]; a.heap[mm] = t; i = mm;
            }
        }
    }
    unsigned long long ended = nout;
    for (uint32_t d = 0; d < a.n_flows; d++)
        if (a.active[d]) {
            if (nout < a.out_cap) { a.out[nout] = a.cur[d]; a.out[nout].order_key = NONE64; }
            nout++;
        }
    a.g->n_rec = nout;
    a.g->n_heads = ended;  // reused: number of ended records
}


__device__ __forceinline__ void cleanup_one(const CleanArgs& a, uint32_t d, bool tables) {
    // the flow's chain slots (an IPv4 flow uses 2 of the N_TABLES): read as
    // 8-byte pairs, cleared only where set
    uint2* row = reinterpret_cast<uint2*>(a.A.slots + (size_t)d * N_TABLES);
    static_assert(N_TABLES % 2 == 0, "slot rows are whole 8-byte pairs");
    uint2 sv[N_TABLES / 2];
#pragma unroll
    for (int t = 0; t < N_TABLES / 2; t++) sv[t] = (a.bulk && t == 0) ? make_uint2(NONE32, NONE32) : row[t];
#pragma unroll
    for (int t = 0; t < N_TABLES / 2; t++) {
        const uint32_t s0 = sv[t].x, s1 = sv[t].y;
        // one 16-byte store per entry {key, value} (two 8-byte stores were two
        // partial writes of the same random line)
        if (tables && !(a.abl & 1) && s0 != NONE32)
            *reinterpret_cast<ulonglong2*>(&a.T.tab[2 * t][2 * s0]) = make_ulonglong2(EMPTY, EMPTY);
        if (tables && !(a.abl & 1) && s1 != NONE32)
            *reinterpret_cast<ulonglong2*>(&a.T.tab[2 * t + 1][2 * s1]) = make_ulonglong2(EMPTY, EMPTY);
        if (!a.bulk && (s0 & s1) != NONE32) row[t] = make_uint2(NONE32, NONE32);  // (bulk: every claim rewrites its row)
    }
    if (a.abl & 2) return;
    a.A.pk[0][d] = a.A.pk[1][d] = 0;
    a.A.by[0][d] = a.A.by[1][d] = 0;
    a.A.mn[0][d] = a.A.mn[1][d] = NONE32;
    a.A.mx[0][d] = a.A.mx[1][d] = 0;
    for (int q = 0; q < 8; q++) a.A.fl[q][d] = 0;
    a.A.fa[d] = a.A.fc[d] = a.A.fr[d] = NONE64;
    a.A.la[d] = 0;
    a.complex[d] = 0;
    if (a.active) a.active[d] = 0;
}

// Reset the flows of the last run, grid-stride over the device-side count.
// After a failed run (error word set) some table slots may have no dense id,
// so every table word is cleared instead of the recorded chains.
// The workgroup that finishes last re-initialises the run counters (Glob,
// n_flows, err): every other workgroup has read n_flows / err before it
// counted itself done, so nobody can see the reset early.
__global__ void __launch_bounds__(256) k_cleanup(CleanArgs a, size_t tab_words) {
    if (a.spec && !run_complete(*a.g, *a.T.err, a.timeout_us, a.recs_cap)) return;  // every workgroup decides alike
    const bool failed = (*a.T.err & (ERR_TABLE_FULL | ERR_SPIN)) != 0;
    const uint32_t nf = failed ? a.T.fmax : min(*a.T.n_flows, a.T.fmax);
    const size_t stride = (size_t)gridDim.x * blockDim.x, t0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (size_t d = t0; d < nf; d += stride) cleanup_one(a, (uint32_t)d, !failed);
    if (failed)
        for (size_t w = t0; w < tab_words; w += stride) a.T.tab[0][w] = EMPTY;  // tables are contiguous
    else if (a.bulk)  // tables 0 and 1: 2 (C + 1) entries of 16 bytes
        for (size_t w = t0; w < 2 * ((size_t)a.T.C + 1); w += stride)
            reinterpret_cast<ulonglong2*>(a.T.tab[0])[w] = make_ulonglong2(EMPTY, EMPTY);
    __shared__ unsigned long long s_rank;
    __syncthreads();
    // (no fence: what the last workgroup resets, every workgroup read before
    // its work, and its count comes after that work; the stores reach the
    // next kernel at the launch boundary.  A per-workgroup agent-scope fence
    // writes back the XCD's L2 and serialised thousands of workgroups.)
    if (threadIdx.x == 0) s_rank = atomicAdd(&a.g->clean_done, 1ull);
    __syncthreads();
    if (s_rank != gridDim.x - 1) return;
    __threadfence();
    unsigned long long* w = reinterpret_cast<unsigned long long*>(a.g);
    const size_t nw = sizeof(Ctl) / 8;  // Glob + counters (+ padding)
    for (size_t i = threadIdx.x; i < nw; i += blockDim.x)
        w[i] = i == offsetof(Glob, tmin) / 8 ? NONE64 : 0ull;
}

__global__ void k_fill_u64(unsigned long long* p, size_t n, unsigned long long v) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}
__global__ void k_fill_u32(uint32_t* p, size_t n, uint32_t v) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

// ---------------------------------------------------------------------------
// k_merge_spill: the owner merge of runs whose hot pass staged no partials
// (k_parse_spill, k_slow): every record is one packet (packed 24 B, seg.h) in
// its owner's segment of a set.  Lean per record, and loads kept in flight:
//  * an owner's segments of a chunk of sets are flattened (exclusive scan of
//    their counts); a wave takes strips of 64 consecutive flattened records,
//    one per lane, and the next strip's loads are issued before this one is
//    probed and aggregated;
//  * a record's set comes from a 64-record group map (every lane of a
//    64-aligned group starts from the same set) and a forward step;
//  * one LDS read per record gives the segment's record base and the window's
//    first packet (relative to the batch): positions are u32 batch-relative in
//    LDS, the update is update_flow's order-free part (flows.rs:11-42) as
//    unguarded LDS atomics.
// The overflow list and the general-parser packets are not read here:
// k_merge_partials (tail_only) takes them, and the run statistics, after it.
// ---------------------------------------------------------------------------
// The merge's rare paths, out of line: inlined, the dictionary's generic
// chain (dense_of_key, up to 12 levels) puts tens of KiB of code between the
// instructions of the record loop.
#ifndef FLUERE_MS_STRIP
#define FLUERE_MS_STRIP 1  // records per lane per strip (r06: 1 -- no spills, 121 VGPRs -- beat 2 by 5 us on C3, 20 on C4)
#endif
#ifndef FLUERE_MS_BATCH
#define FLUERE_MS_BATCH 1  // the strip's first probes issued together (0: each record's probe loop alone; A/B)
#endif
#ifndef FLUERE_MS_ABL
#define FLUERE_MS_ABL 0  // diagnostics only (wrong results): 1 the record loads alone, 2 + the probe, no updates
#endif
#ifndef FLUERE_MS_COLD
#define FLUERE_MS_COLD 1  // the global path out of line (0: inlined; A/B)
#endif
#if FLUERE_MS_COLD
#define MS_COLD __noinline__
#else
#define MS_COLD __forceinline__
#endif
__device__ MS_COLD uint32_t staged_id_cold(const AggArgs* ap, uint4 kk, uint32_t tag) {
    const AggArgs& a = *ap;
    if (kk.w & V6_TAG) {
        CKey ck;
        v6_ckey(a.v6, kk.x, kk.y, kk.z, tag, ck);
        return dense_of_key(a.T, ck, true, a.A.slots, &a.g->generic_used);
    }
    return staged_id(a.T, a.v6, kk.x, kk.y, kk.z, tag, a.A.slots);
}

// The IPv4 chain for a key its merge owner resolves (k_merge_spill): each
// level's word by a CAS first -- a new word costs one atomic round trip (a
// read, then a CAS, cost two), a present one returns itself.  fresh: this
// call inserted the T1 word (the flow has no dense id yet).
__device__ __forceinline__ uint32_t tab_claim(const TableSet& T, int t, uint64_t w, uint32_t h0, bool& fresh) {
    unsigned long long* tab = T.tab[t];
    fresh = false;
    if (w == EMPTY) return T.C;
    uint32_t h = h0 & (T.C - 1);
    for (int p = 0; p < MAX_PROBE; p++) {
        const unsigned long long old = atomicCAS(&tab[2 * h], EMPTY, (unsigned long long)w);
        if (old == EMPTY) { fresh = true; return h; }
        if (old == w) return h;
        h = (h + 1) & (T.C - 1);
    }
    atomicOr(T.err, ERR_TABLE_FULL);
    return FAIL;
}
__device__ __forceinline__ void v4_claim(const TableSet& T, uint32_t lo, uint32_t hi, uint32_t ports, uint32_t proto,
                                         uint32_t& s0, uint32_t& s1, bool& fresh1) {
    bool f0;
    s1 = FAIL;
    fresh1 = false;
    const uint64_t w0 = ((uint64_t)lo << 32) | hi;
    s0 = tab_claim(T, 0, w0, (uint32_t)mix64(w0), f0);
    if (s0 == FAIL) return;
    s1 = tab_claim(T, 1, v4_t1_word(T, s0, ports, proto), v4_t1_start(lo, hi, ports, proto), fresh1);
}

constexpr int MS_STRIP = FLUERE_MS_STRIP;
// k_merge_spill's key table: MK entries probed in pairs (two-choice: the
// key's home pair e1 and a second pair e2), each holding its aggregate slot
// (< MT) in bits 8..21 of its last word (the tag's protocol, bits 24..31, and
// flags, bits 0..7, stay readable)
constexpr int MK = 2048;
constexpr uint32_t MS_SLOT_MASK = 0x3FFFu << 8, MS_NOSLOT = 0x3FFFu;
static_assert(MT <= 0x3FFF, "slots fit the entry's slot field");
static_assert((LT_READY | LT_CLAIM) & MS_SLOT_MASK ? false : true, "the slot field clears the state bits");
__device__ __forceinline__ void ms_pairs(uint32_t k0, uint32_t k1, uint32_t k2, uint32_t tag, uint32_t& e1, uint32_t& e2) {
    uint32_t x = k0 ^ __builtin_amdgcn_alignbit(k1, k1, 11) ^ __builtin_amdgcn_alignbit(k2, k2, 22) ^ (tag >> 24) ^ (tag << 7);
    x ^= x >> 16;
    x = __umul24(x, 0x9E3779u) ^ (x >> 24);
    x = __umul24(x ^ (x >> 13), 0x5BD1E9u) ^ (x >> 9);
    e1 = (x & (MK - 1)) & ~1u;
    e2 = ((x >> 11) & (MK - 1)) & ~1u;
    if (e2 == e1) e2 ^= 2u;
}
// merge-table home slot of a staged key (10 bits: MT == 1024): the key words
// folded, then mixed with full-rate 24-bit multiplies (lt_hash's 32-bit
// multiplies are quarter rate: a fifth of the record loop's VALU time)
__device__ __forceinline__ uint32_t ms_slot(uint32_t k0, uint32_t k1, uint32_t k2, uint32_t tag) {
    uint32_t x = k0 ^ __builtin_amdgcn_alignbit(k1, k1, 11) ^ __builtin_amdgcn_alignbit(k2, k2, 22) ^ (tag >> 24) ^ (tag << 7);
    x ^= x >> 16;
    x = __umul24(x, 0x9E3779u) ^ (x >> 24);
    x = __umul24(x ^ (x >> 13), 0x5BD1E9u);
    return (x >> 6) & (MT - 1);
}  // records per lane per strip (a strip: 64 * MS_STRIP records of one wave)
constexpr uint32_t MS_GRP = 1024;  // 64-record groups mapped in LDS (owners of more records: a binary search)
__global__ void __launch_bounds__(MB) k_merge_spill(AggArgs a, MergeSrc ms) {
    // the arguments in the kernarg segment, for the out-of-line paths (a
    // reference to `a` would copy the whole struct to every lane's stack)
    const AggArgs* kargs = (const AggArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    // key table: MK entries {k0, k1, k2, tag | READY / CLAIM | slot << 8}, probed as
    // two-choice pairs; the aggregates below are per slot (MT), in claim order
    __shared__ uint4 m_key[MK];
    __shared__ uint16_t m_sk[MT];  // key entry of each slot
    __shared__ uint32_t m_pk[2][MT], m_mn[2][MT], m_mx[2][MT], m_fl[8][MT];
    __shared__ unsigned long long m_by[2][MT];
    __shared__ uint32_t m_pos[4][MT];  // first, first create-eligible, first FIN/RST (min), last + 1 (max):
                                       // relative to the pass's first packet (batch 0's)
    // per non-empty segment of the chunk (k: its rank): {record index - flattened start (mod 2^32),
    // window base}, flattened start; per group of 64 flattened records {segment of its first
    // record, 0, 64-bit mask of the records that start a segment}
    __shared__ uint2 m_sd[MCH];
    __shared__ uint32_t m_st[MCH];
    __shared__ uint4 m_ginfo[MS_GRP];
    __shared__ uint32_t m_scan[MB / 64 + 1], m_nclaim, m_base, s_me, m_nslot, s_sole;
    const int tid = threadIdx.x;
    const uint32_t lane = tid & 63, wv = tid >> 6;
    const uint32_t O = a.S.O;
    const uint64_t bfirst = ms.b[0].first;  // positions in LDS: relative to the pass's first packet
    if (tid == 0) {
        s_me = blockIdx.x;
        // No tail adds to the owners' flows (no overflow list from the hot pass, no
        // general-parser packets): each owner is the only writer of its flows'
        // accumulators, and writes them with plain stores.  (Records this merge
        // sends to the overflow list belong to keys without a slot: other flows.
        // A count raised by them here only makes the choice conservative.)
        uint32_t sole = 1;
        for (int bi = 0; bi < ms.nb; bi++) {
            const unsigned long long* bc = ms.b[bi].bc;
            const unsigned long long ovf = __hip_atomic_load(&bc[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long gen = __hip_atomic_load(&bc[ms.b[bi].slow_kernel ? 3 : 0], __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT);
            // (k_slow's keys: a flow whose IPv6 addresses found no id in the address
            // map travels as its dense id, others of it as address ids: two owners)
            if (ovf || gen || ms.b[bi].slow_kernel) sole = 0;
        }
        s_sole = sole;
    }
    __syncthreads();
    const bool sole = s_sole != 0;
    unsigned long long* dbg = a.dbg ? a.dbg + 4096 * 8 - 2048 + blockIdx.x * 8 : nullptr;  // (FLUERE_DEBUG: phase clocks)
    for (uint32_t me = s_me; me < O; me = s_me) {
        if (dbg && tid == 0) dbg[0] = wall_clock64();
        for (int e = tid; e < MK; e += MB) m_key[e] = make_uint4(0, 0, 0, 0);
        if (tid == 0) m_nslot = 0;
        for (int e = tid; e < MT; e += MB) {
            m_pk[0][e] = m_pk[1][e] = 0;
            m_by[0][e] = m_by[1][e] = 0;
            m_mn[0][e] = m_mn[1][e] = NONE32;
            m_mx[0][e] = m_mx[1][e] = 0;
#pragma unroll
            for (int q = 0; q < 8; q++) m_fl[q][e] = 0;
            m_pos[0][e] = m_pos[1][e] = m_pos[2][e] = NONE32;
            m_pos[3][e] = 0;
        }
        for (int bi = 0; bi < ms.nb; bi++)
        for (uint32_t c0s = 0; c0s < ms.b[bi].n_sets; c0s += MCH) {
            const SegSrc& S = ms.b[bi];
            const uint2* recs = reinterpret_cast<const uint2*>(S.dspill);  // the packed 24-byte form (seg_pack)
            const uint32_t bshift = (uint32_t)(S.first - bfirst);  // the batch's first packet in the pass
            const uint32_t nset = min((uint32_t)MCH, S.n_sets - c0s);
            // this owner's segment of each set of the chunk: count, record base, window base
            static_assert(MCH == MB, "one set per thread");
            const uint32_t s = c0s + tid;
            uint32_t cnt = 0, rb = 0, wb = 0;
            if ((uint32_t)tid < nset) {
                cnt = S.soff[(size_t)me * S.n_sets + s];
                rb = s < S.n_hot ? (uint32_t)(((unsigned long long)s * O + me) * S.cap_o)
                                 : (uint32_t)(S.slow_rec0 + ((unsigned long long)(s - S.n_hot) * O + me) * S.cap_s);
                wb = (uint32_t)(S.base[s] - bfirst);
            }
            // the non-empty segments, compacted (k: rank among them), with their
            // flattened starts (exclusive scan of the counts)
            if (dbg && tid == 0 && c0s == 0 && bi == 0) dbg[1] = wall_clock64();
            const uint32_t st0 = block_exclusive_scan(cnt, m_scan);  // (ends with a barrier)
            const uint32_t total = m_scan[MB / 64];
            const uint32_t k = block_exclusive_scan(cnt ? 1u : 0u, m_scan);
            const uint32_t nk = m_scan[MB / 64];
            const uint32_t ngrp = (total + 63) / 64;
            const bool grp = ngrp <= MS_GRP;
            if (grp)
                for (uint32_t g = tid; g < ngrp; g += MB) m_ginfo[g] = make_uint4(0, 0, 0, 0);
            if (cnt) {
                m_sd[k] = make_uint2(rb - st0, wb);
                m_st[k] = st0;
            }
            __syncthreads();
            // per group of 64 flattened records: the segment holding its first
            // record, and a bit per later record that starts a segment
            if (grp && cnt) {
                if (st0 & 63) atomicOr(&m_ginfo[st0 >> 6].z + ((st0 & 63) >> 5), 1u << (st0 & 31));
                for (uint32_t g = (st0 + 63) >> 6; g <= (st0 + cnt - 1) >> 6; g++) m_ginfo[g].x = k;
            }
            __syncthreads();
            // record f's segment (rank k) -> {record index - flattened start, window base}
            auto seg_of = [&](uint32_t f) -> uint2 {
                uint32_t kk;
                if (grp) {
                    const uint4 gi = m_ginfo[f >> 6];  // (the same for every lane of a 64-aligned group)
                    const uint32_t p = f & 63;
                    const unsigned long long msk = ((unsigned long long)gi.w << 32) | gi.z;
                    kk = gi.x + (uint32_t)__popcll(msk & ((2ull << p) - 2ull));
                } else {
                    uint32_t lo = 0, hi = nk - 1;  // last segment starting at or before f
                    while (lo < hi) {
                        const uint32_t mid = (lo + hi + 1) >> 1;
                        if (m_st[mid] <= f) lo = mid;
                        else hi = mid - 1;
                    }
                    kk = lo;
                }
                return m_sd[kk];
            };
            // strips of 64 * MS_STRIP records; record u * 64 + lane of a strip is
            // this lane's u-th.  Two strips in flight per wave: the next one's
            // loads are issued before this one is probed and aggregated.
            const uint32_t nstrip = (total + 64 * MS_STRIP - 1) / (64 * MS_STRIP);
            auto fetch = [&](uint32_t sp, uint4 (&v0)[MS_STRIP], uint4 (&v1)[MS_STRIP], uint32_t (&wbr)[MS_STRIP]) {
                uint2 sd[MS_STRIP];
                uint32_t fc[MS_STRIP];
#pragma unroll
                for (int u = 0; u < MS_STRIP; u++) {
                    fc[u] = min(sp * (64 * MS_STRIP) + u * 64 + lane, total - 1);  // (past the end: the last record, unused)
                    sd[u] = seg_of(fc[u]);
                }
#pragma unroll
                for (int u = 0; u < MS_STRIP; u++) {
                    const uint32_t idx = sd[u].x + fc[u];
                    seg_load(recs, idx, v0[u], v1[u]);
                    wbr[u] = sd[u].y;
                }
            };
            auto process = [&](uint32_t sp, const uint4 (&v0)[MS_STRIP], const uint4 (&v1)[MS_STRIP],
                               const uint32_t (&wbr)[MS_STRIP]) {
                if (FLUERE_MS_ABL == 1) {  // diagnostics (wrong results): the records' loads alone
#pragma unroll
                    for (int u = 0; u < MS_STRIP; u++)
                        if ((v0[u].x ^ v0[u].y ^ v0[u].z ^ v1[u].x ^ v1[u].y ^ wbr[u]) == 0x12345678u) atomicAdd(&m_pk[0][0], 1u);
                    return;
                }
                // first probes of the strip's records together: both candidate
                // pairs of each key (four 16-byte reads, one LDS round trip); the
                // claim loop runs only for new keys and keys placed further on
                uint32_t e1[MS_STRIP], e2[MS_STRIP];
                uint4 kp[MS_STRIP][4];
#pragma unroll
                for (int u = 0; u < MS_STRIP; u++) {
                    ms_pairs(v0[u].x, v0[u].y, v0[u].z, v0[u].w, e1[u], e2[u]);
                    kp[u][0] = m_key[e1[u]];
                    kp[u][1] = m_key[e1[u] + 1];
                    kp[u][2] = m_key[e2[u]];
                    kp[u][3] = m_key[e2[u] + 1];
                }
#pragma unroll
                for (int u = 0; u < MS_STRIP; u++) {
                    const uint32_t f = sp * (64 * MS_STRIP) + u * 64 + lane;
                    const bool live = f < total;
                    const uint32_t k0 = v0[u].x, k1 = v0[u].y, k2 = v0[u].z, tag = v0[u].w;
                    const uint32_t rel = wbr[u] + v1[u].z;  // the packet's index in the pass
                    const uint32_t want = tag | LT_READY;
                    uint32_t e = MS_NOSLOT;
#pragma unroll
                    for (int j = 3; j >= 0; j--)
                        if ((((kp[u][j].w & ~MS_SLOT_MASK) ^ want) | (kp[u][j].x ^ k0) | (kp[u][j].y ^ k1) | (kp[u][j].z ^ k2)) == 0u)
                            e = (kp[u][j].w >> 8) & 0x3FFFu;
                    int state = !live ? 3 : e != MS_NOSLOT ? 1 : 0;
                    if (__ballot(state == 0)) {
                        // the key's probe sequence: pair e1, pair e2, then pairs from e2 + 2
                        uint32_t pe = e1[u];
                        int steps = 0;
                        for (int it = 0; it < 4 * MK; it++) {  // (bounded: every pass reads or claims)
                            if (state == 0) {
                                const uint4 ka = m_key[pe], kb = m_key[pe + 1];
                                const bool ma = (((ka.w & ~MS_SLOT_MASK) ^ want) | (ka.x ^ k0) | (ka.y ^ k1) | (ka.z ^ k2)) == 0u;
                                const bool mb = (((kb.w & ~MS_SLOT_MASK) ^ want) | (kb.x ^ k0) | (kb.y ^ k1) | (kb.z ^ k2)) == 0u;
                                if (ma | mb) {
                                    e = ((ma ? ka.w : kb.w) >> 8) & 0x3FFFu;
                                    state = e < MT ? 1 : 2;
                                } else if ((ka.w & LT_READY) && (kb.w & LT_READY)) {
                                    if (++steps == MK / 2) state = 2;
                                    else pe = steps == 1 ? e2[u] : (pe + 2) & (MK - 1);
                                } else {
                                    // the pair's first free entry (an entry being written is read again next pass)
                                    const uint32_t fe = ka.w == 0 ? pe : ((ka.w & LT_READY) && kb.w == 0 ? pe + 1 : MK);
                                    if (fe < MK && atomicCAS(&m_key[fe].w, 0u, LT_CLAIM) == 0u) {
                                        uint32_t sl = atomicAdd(&m_nslot, 1u);
                                        if (sl >= MT) sl = MS_NOSLOT;  // no aggregate slot left: the key's records take the global path
                                        else m_sk[sl] = (uint16_t)fe;
                                        m_key[fe].x = k0;
                                        m_key[fe].y = k1;
                                        m_key[fe].z = k2;
                                        __threadfence_block();
                                        atomicExch(&m_key[fe].w, want | (sl << 8));
                                        e = sl;
                                        state = sl < MT ? 1 : 2;
                                    }
                                }
                            }
                            if (__ballot(state == 0) == 0) break;
                        }
                    }
                    const uint32_t dir = (v1[u].w >> 8) & 1u, tf = v1[u].w & 0xFFu;
                    const uint32_t pkt = v1[u].y & 0xFFFFu, ttl = (v1[u].y >> 16) & 0xFFu;
                    if (FLUERE_MS_ABL == 2) {  // diagnostics (wrong results): the probe, no updates
                        if (state == 1 && pkt == 0x1234u) atomicAdd(&m_pk[0][e & (MT - 1)], 1u);
                        continue;
                    }
                    if (state == 1) {  // update_flow of one packet (flows.rs:11-42), order-free part
                        if (a.pid) a.pid[bfirst + rel - a.pid_base] = PH_EREF | (me << 10) | e;  // (batch field 0: one merge per pass)
                        atomicAdd(&m_pk[dir][e], 1u);
                        atomicAdd(&m_by[dir][e], (unsigned long long)v1[u].x);
                        atomicMin(&m_mn[0][e], pkt);
                        atomicMin(&m_mn[1][e], ttl);
                        atomicMax(&m_mx[0][e], pkt);
                        atomicMax(&m_mx[1][e], ttl);
                        atomicMin(&m_pos[0][e], rel);
                        atomicMin(&m_pos[1][e], ((v1[u].y >> 24) & 1u) ? rel : NONE32);
                        atomicMax(&m_pos[3][e], rel + 1);
                        if (tf) {
                            for (uint32_t t = tf; t; t &= t - 1) atomicAdd(&m_fl[__builtin_ctz(t)][e], 1u);
                            if (tf & 5u) atomicMin(&m_pos[2][e], rel);
                        }
                    } else if (state == 2) {  // no aggregate slot: the overflow list (the tail takes it)
                        // (the batch's list, positions relative to the batch: its tail takes it)
                        const unsigned long long q = atomicAdd(&S.bc[1], 1ull);
                        uint4* dst = reinterpret_cast<uint4*>(S.spill) + q * 2;
                        dst[0] = v0[u];
                        dst[1] = make_uint4(v1[u].x, v1[u].y, rel - bshift, (v1[u].w & 0x1FFu) | (SPILL_BATCH_REL << 9));
                    }
                }
            };
            if (dbg && tid == 0 && c0s == 0 && bi == 0) dbg[2] = wall_clock64();
            if (total) {
                uint4 a0[MS_STRIP], a1[MS_STRIP], b0[MS_STRIP], b1[MS_STRIP];
                uint32_t aw[MS_STRIP], bw[MS_STRIP];
                uint32_t sp = wv;
                fetch(sp, a0, a1, aw);
                while (sp < nstrip) {  // (uniform)
                    const uint32_t sq = sp + MB / 64;
                    fetch(sq < nstrip ? sq : sp, b0, b1, bw);  // (always issued: no branch merges loading registers)
                    process(sp, a0, a1, aw);
                    if (sq >= nstrip) break;
                    const uint32_t sr = sq + MB / 64;
                    fetch(sr < nstrip ? sr : sq, a0, a1, aw);
                    process(sq, b0, b1, bw);
                    sp = sr;
                }
            }
            __syncthreads();
        }
        // Dense ids: thread per entry (MT == MB), as k_merge_partials: the owner
        // is the only inserter of its keys; one atomicAdd on the flow counter
        // gives the workgroup's new ids.
        static_assert(MT == MB, "one merge entry per thread");
        if (dbg && tid == 0) dbg[3] = wall_clock64();
        if (tid == 0) m_nclaim = 0;
        __syncthreads();
        const int e = tid;  // aggregate slot
        const bool have = (uint32_t)e < min(m_nslot, (uint32_t)MT);
        uint4 kk = have ? m_key[m_sk[e]] : make_uint4(0, 0, 0, 0);
        kk.w &= ~MS_SLOT_MASK;
        const uint32_t tag = kk.w & 0xFF000000u;
        uint32_t d = FAIL, s0 = FAIL, s1 = FAIL, rank = 0;
        bool claimed = false, wait = false;
        unsigned long long* val = nullptr;
        if (have) {
            if (!(kk.w & V6_TAG) && tag == 0xFF000000u) {
                d = kk.x;  // k_slow's keys of the dictionary's other chains carry dense ids
            } else if ((kk.w & V6_TAG) || !v4_fast(a.T, tag >> 24)) {
                // an IPv6 5-tuple from k_slow (address ids, any protocol), or (wide tables) a
                // protocol other than TCP / UDP
                d = staged_id_cold(kargs, kk, tag);
            } else {  // IPv4 5-tuple: flow_table.h chain T0 (ip pair) -> T1 (slot, ports, proto)
                unsigned long long v = EMPTY;
                bool fresh = false;
                v4_claim(a.T, kk.x, kk.y, kk.z, tag >> 24, s0, s1, fresh);
                if (s1 != FAIL) {
                    val = &a.T.tab[1][2 * s1 + 1];
                    // a key this owner inserted has no id yet and no other claimer
                    // (its owner is the only one that resolves it in this kernel)
                    v = fresh ? EMPTY : atomicCAS(val, EMPTY, PENDING);
                    if (v == EMPTY) {
                        claimed = true;
                        rank = atomicAdd(&m_nclaim, 1u);
                    } else if (v == PENDING) {
                        wait = true;
                    } else {
                        d = (uint32_t)v;
                    }
                }
            }
        }
        __syncthreads();
        if (dbg && tid == 0) dbg[7] = wall_clock64();
        if (tid == 0) m_base = m_nclaim ? atomicAdd(a.T.n_flows, m_nclaim) : 0;
        __syncthreads();
        if (dbg && tid == 0) dbg[6] = wall_clock64();
        if (claimed) {
            d = m_base + rank;
            if (d >= a.T.fmax) {
                atomicOr(a.T.err, ERR_FLOWS_FULL);
                d = FAIL;
            } else {
                uint32_t* dst = (uint32_t*)(a.T.flow_key + (size_t)d * 56);
#pragma unroll
                for (int k = 0; k < 14; k++) dst[k] = k == 0 ? kk.x : k == 4 ? kk.y : k == 8 ? kk.z : k == 9 ? tag >> 24 : 0;
#pragma unroll
                for (int j = 0; j < N_TABLES; j++) a.A.slots[(size_t)d * N_TABLES + j] = j == 0 ? s0 : j == 1 ? s1 : NONE32;
            }
            atomicExch(val, (unsigned long long)d);
        }
        for (int sp = 0; sp < (1 << 20); sp++) {  // a claim held elsewhere: poll (wave-uniform)
            if (__ballot(wait) == 0) break;
            if (wait) {
                const unsigned long long v = __hip_atomic_load(val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (v != PENDING && v != EMPTY) {
                    d = (uint32_t)v;
                    wait = false;
                }
            }
            if (__ballot(wait) != 0) __builtin_amdgcn_s_sleep(16);
        }
        if (wait) atomicOr(a.T.err, ERR_SPIN);
        if (dbg && tid == 0) dbg[4] = wall_clock64();
        if (a.emap) a.emap[((size_t)me << 10) | (uint32_t)e] = (have && d < a.T.fmax) ? d : FAIL;
        if (have && d != FAIL && d < a.T.fmax) {
            FlowPart f;
#pragma unroll
            for (int q = 0; q < 2; q++) {
                f.pk[q] = m_pk[q][e];
                f.by[q] = m_by[q][e];
                f.mn[q] = m_mn[q][e];
                f.mx[q] = m_mx[q][e];
            }
#pragma unroll
            for (int q = 0; q < 8; q++) f.fl[q] = m_fl[q][e];
            const uint32_t p0 = m_pos[0][e], p1 = m_pos[1][e], p2 = m_pos[2][e], p3 = m_pos[3][e];
            f.fa = p0 == NONE32 ? NONE64 : bfirst + p0;
            f.fc = p1 == NONE32 ? NONE64 : bfirst + p1;
            f.fr = p2 == NONE32 ? NONE64 : bfirst + p2;
            f.la = p3 ? bfirst + p3 : 0;
            if (sole) part_store_global(a.A, d, f);
            else part_to_global(a.A, d, f);
        }
        if (dbg && tid == 0) dbg[5] = wall_clock64();
        __syncthreads();  // (the next owner re-initialises the table)
        if (tid == 0) s_me = O > gridDim.x ? gridDim.x + (uint32_t)atomicAdd(&ms.b[0].bc[4], 1ull) : O;
        __syncthreads();
    }
}

const void* merge_kernel(int macs) {
    return macs ? (const void*)k_merge_partials<true> : (const void*)k_merge_partials<false>;
}

}  // namespace fl
