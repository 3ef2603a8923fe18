// shard.hip -- the multi-GPU exchange: per-owner export blocks, the owner
// merge and the composition of order-dependent flows, the compact wire
// encoding, and the hard-timeout sweep composed across shards.
#include "ctx.h"

namespace fl {

// ---------------------------------------------------------------------------
// multi-GPU exchange (include/fluere_gpu.h): every shard exports summaries and
// annexes bucketed by owner; each owner merges its flows and composes, in
// shard order, the flows whose record depends on packet order
// ---------------------------------------------------------------------------


// A flow's local order dependence (shard side): trivial when its first FIN/RST
// (if any) is its last packet and its first packet can create it (or none
// can) -- then the summary alone determines its part of the state machine.
__global__ void __launch_bounds__(256) k_local_cert(FinArgs a, uint32_t* annex_of) {
    const uint32_t nf = min(*a.T.n_flows, a.T.fmax);
    for (uint32_t d0 = blockIdx.x * blockDim.x; d0 < nf; d0 += gridDim.x * blockDim.x) {
        const uint32_t d = d0 + threadIdx.x;
        bool cplx = false;
        if (d < nf) {
            const unsigned long long fa = a.A.fa[d], fc = a.A.fc[d], fr = a.A.fr[d], la = a.A.la[d];
            cplx = !((fr == NONE64 || fr == la) && (fc == fa || fc == NONE64));
            a.complex[d] = cplx ? 1 : 0;
            annex_of[d] = NONE32;
        }
        const uint64_t cm = __ballot(cplx);
        if (cm && (uint32_t)(threadIdx.x & 63) == (uint32_t)__builtin_ctzll(cm))
            atomicAdd(&a.g->n_complex, (unsigned long long)__popcll(cm));
    }
}


__global__ void k_export_hdr(ExportArgs a) {
    const uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= a.n_owners) return;
    fluere_shard_header h{};
    const Glob* g = a.fa.g;
    h.tmin = g->tmin; h.tmax = g->tmax; h.valid = g->valid; h.dropped = g->dropped;
    h.err = *a.fa.T.err;
    h.shard = a.shard;
    // (k_local_cert counted them: exported without annexes, the owner cannot compose them)
    h.n_bare_complex = a.annex ? 0ull : g->n_complex;
    *blk_hdr(a.blocks, a.block_bytes, o) = h;
}

__global__ void __launch_bounds__(256) k_export_owners(ExportArgs a) {
    const uint32_t nf = min(*a.fa.T.n_flows, a.fa.T.fmax);
    for (uint32_t d = blockIdx.x * blockDim.x + threadIdx.x; d < nf; d += gridDim.x * blockDim.x) {
        fluere_flow_summary s;
        export_one(a.fa, s, d);
        s.shard = a.shard;
        const uint32_t o = key_owner(s.key, a.n_owners);
        fluere_shard_header* h = blk_hdr(a.blocks, a.block_bytes, o);
        const unsigned long long pos = atomicAdd(reinterpret_cast<unsigned long long*>(&h->n_flows), 1ull);
        const uint32_t ax = a.annex ? a.annex_of[d] : NONE32;  // (no annexes yet: a speculative export)
        if (ax != NONE32) {
            const unsigned long long apos = atomicAdd(reinterpret_cast<unsigned long long*>(&h->n_annex), 1ull);
            if (apos < a.cap_annex) {
                blk_annex(a.blocks, a.block_bytes, a.cap, o)[apos] = a.annex[ax];
                s.annex = (uint32_t)apos;
            }
        }
        if (pos < a.cap) blk_sum(a.blocks, a.block_bytes, o)[pos] = s;
        a.sumpos[d] = (uint32_t)pos;
    }
}

// need[0..1]: the largest per-owner summary / annex counts; info (may be
// null): the same, then the shard's order-dependent flows and its flow count
// (fluere_export_async: reduced over the ranks on the device, read once).
__global__ void k_export_need(ExportArgs a, unsigned long long* need, unsigned long long* info) {
    if (threadIdx.x || blockIdx.x) return;
    unsigned long long m0 = 0, m1 = 0;
    for (uint32_t o = 0; o < a.n_owners; o++) {
        const fluere_shard_header* h = blk_hdr(a.blocks, a.block_bytes, o);
        m0 = max(m0, (unsigned long long)h->n_flows);
        m1 = max(m1, (unsigned long long)h->n_annex);
    }
    need[0] = m0;
    need[1] = m1;
    if (info) {
        const Glob* g = a.fa.g;
        info[0] = m0;
        info[1] = m1;
        info[2] = g->n_complex;
        info[3] = min(*a.fa.T.n_flows, a.fa.T.fmax);
        // the capture span, reducible with MAX: 2^62 - tmin and tmax (0: no valid packet)
        info[4] = g->valid ? (1ull << 62) - g->tmin : 0ull;
        info[5] = g->valid ? g->tmax : 0ull;
    }
}

struct FirstPay {
    unsigned long long t_first, t_last;
    uint16_t sp, dp;
    uint8_t dir, prot, tos, v6;
    uint8_t src[16], dst[16];
};

struct MergeArgs {
    TableSet T;
    Acc A;
    unsigned long long n;  // n_shards * cap summary slots
    uint32_t* sd;
    FirstPay* pay;
    Glob* g;
    fluere_record* out;
    uint8_t* complex;
    uint64_t out_cap;
    // the gathered blocks: summary i is entry i % cap of block i / cap (the
    // block of rank i / cap); entries past the block's n_flows are absent
    const uint8_t* blocks;
    unsigned long long cap, cap_annex, block_bytes;
    Ctl* host_ctl;   // non-null: k_merge_finalize publishes the counters (publish_ctl)
    uint32_t seq;
    unsigned long long timeout_us;
};
// a merge enqueued by fluere_merge_gathered_async, completed by _finish
struct MergePending {
    MergeArgs ma;
    uint32_t seq = 0, shards = 0;
    uint64_t cap = 0;
    bool pending = false;
};

// summary i of a merge; null when absent
__device__ __forceinline__ const fluere_flow_summary* merge_input(const MergeArgs& a, unsigned long long i) {
    if (i >= a.n) return nullptr;
    uint8_t* blocks = const_cast<uint8_t*>(a.blocks);
    const uint32_t b = (uint32_t)(i / a.cap);
    const unsigned long long j = i % a.cap;
    if (j >= min((unsigned long long)blk_hdr(blocks, a.block_bytes, b)->n_flows, a.cap)) return nullptr;
    return blk_sum(blocks, a.block_bytes, b) + j;
}
__device__ __forceinline__ const fluere_flow_annex* merge_annex(const MergeArgs& a, unsigned long long i, uint32_t k) {
    return blk_annex(const_cast<uint8_t*>(a.blocks), a.block_bytes, a.cap, (uint32_t)(i / a.cap)) + k;
}

__global__ void __launch_bounds__(256) k_merge_insert(MergeArgs a) {
    unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < a.n && i % a.cap == 0) {  // the block's run counters
        const fluere_shard_header* h = blk_hdr(const_cast<uint8_t*>(a.blocks), a.block_bytes, (uint32_t)(i / a.cap));
        if (h->valid) {
            atomicAdd(&a.g->valid, (unsigned long long)h->valid);
            atomicMin(&a.g->tmin, (unsigned long long)h->tmin);
            atomicMax(&a.g->tmax, (unsigned long long)h->tmax);
        }
        if (h->dropped) atomicAdd(&a.g->dropped, (unsigned long long)h->dropped);
        if (h->err) atomicOr(a.T.err, h->err);
        if (h->n_flows > a.cap || h->n_annex > a.cap_annex) atomicOr(a.T.err, ERR_CAPACITY);  // cut short
        if (h->n_bare_complex) atomicAdd(&a.g->n_bare, (unsigned long long)h->n_bare_complex);
    }
    const fluere_flow_summary* sp = merge_input(a, i);
    if (!sp) {
        if (i < a.n) a.sd[i] = FAIL;
        return;
    }
    const fluere_flow_summary& s = *sp;
    CKey k;
    for (int j = 0; j < 14; j++) k.w[j] = s.key[j];
    uint32_t d = dense_of_key(a.T, k, true, a.A.slots, &a.g->generic_used);
    a.sd[i] = d;
    if (d == FAIL || d >= a.T.fmax) return;
    const Acc& A = a.A;
    for (int q = 0; q < 2; q++) {
        if (s.pkts[q]) { atomicAdd(&A.pk[q][d], s.pkts[q]); atomicAdd(&A.by[q][d], (unsigned long long)s.bytes[q]); }
    }
    atomicMin(&A.mn[0][d], s.min_pkt); atomicMax(&A.mx[0][d], s.max_pkt);
    atomicMin(&A.mn[1][d], s.min_ttl); atomicMax(&A.mx[1][d], s.max_ttl);
    for (int q = 0; q < 8; q++) if (s.flag_cnt[q]) atomicAdd(&A.fl[q][d], s.flag_cnt[q]);
    atomicMin(&A.fa[d], (unsigned long long)s.first_all);
    atomicMin(&A.fc[d], (unsigned long long)s.first_create);
    atomicMin(&A.fr[d], (unsigned long long)s.finrst_min);
    atomicMax(&A.la[d], (unsigned long long)s.last);
}

__global__ void __launch_bounds__(256) k_merge_payload(MergeArgs a) {
    unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    uint32_t d = a.sd[i];
    if (d == FAIL || d >= a.T.fmax) return;
    const fluere_flow_summary& s = *merge_input(a, i);
    // packet indices are global and unique: exactly one shard holds each
    if (s.first_create != NONE64 && s.first_create == a.A.fc[d]) {
        FirstPay& p = a.pay[d];
        p.t_first = s.first_time;
        p.sp = s.first_sport; p.dp = s.first_dport;
        p.dir = s.first_dir; p.prot = s.first_prot; p.tos = s.first_tos; p.v6 = s.first_v6;
        for (int k = 0; k < 16; k++) { p.src[k] = s.first_src[k]; p.dst[k] = s.first_dst[k]; }
    }
    if (s.last == a.A.la[d]) a.pay[d].t_last = s.last_time;
}

__device__ __forceinline__ void merge_finalize_one(const MergeArgs& a, uint32_t d, fluere_record& r, bool& want,
                                                   bool& cplx) {
    const Acc& A = a.A;
    unsigned long long fa = A.fa[d], fc = A.fc[d], fr = A.fr[d], la = A.la[d];
    if (fc == NONE64) return;
    if (!(fc == fa && (fr == NONE64 || fr == la))) {
        a.complex[d] = 1;
        cplx = true;
        return;
    }
    const FirstPay p = a.pay[d];
    memset(&r, 0, sizeof r);
    r.src_v6 = r.dst_v6 = p.v6;
    for (int k = 0; k < 16; k++) { r.source[k] = p.src[k]; r.destination[k] = p.dst[k]; }
    r.prot = p.prot; r.tos = p.tos; r.src_port = p.sp; r.dst_port = p.dp;
    uint32_t p0 = A.pk[0][d], p1 = A.pk[1][d];
    unsigned long long b0 = A.by[0][d], b1 = A.by[1][d];
    r.d_pkts = p0 + p1;
    r.d_octets = b0 + b1;
    r.out_pkts = p.dir ? p1 : p0; r.in_pkts = p.dir ? p0 : p1;
    r.out_bytes = p.dir ? b1 : b0; r.in_bytes = p.dir ? b0 : b1;
    r.min_pkt = A.mn[0][d]; r.max_pkt = A.mx[0][d];
    r.min_ttl = (uint8_t)A.mn[1][d]; r.max_ttl = (uint8_t)A.mx[1][d];
    for (int q = 0; q < 8; q++) r.cnt[q] = A.fl[q][d];
    r.first = p.t_first;
    r.last = p.t_last;
    r.order_key = (fr == la) ? la : NONE64;
    want = true;
}

// grid-stride over the flows counted on the device (no host round trip)
__global__ void __launch_bounds__(EMIT_BLOCK) k_merge_finalize(MergeArgs a) {
    // a capture whose span reaches the timeout: no record here, the sweep
    // composition (fluere_sweep_*) builds them all
    const Glob* g = a.g;
    const bool expiry = g->valid && g->tmax >= g->tmin && g->tmax - g->tmin >= a.timeout_us;
    const uint32_t nf = expiry ? 0u : min(*a.T.n_flows, a.T.fmax);
    __shared__ EmitLds S;
    for (uint32_t d0 = blockIdx.x * blockDim.x; d0 < nf; d0 += gridDim.x * blockDim.x) {
        const uint32_t d = d0 + threadIdx.x;
        fluere_record r;
        bool want = false, cplx = false;
        if (d < nf) merge_finalize_one(a, d, r, want, cplx);
        emit_record_block(S, a.g, a.out, a.out_cap, r, want);
        const uint64_t cm = __ballot(cplx);
        if (cm && (uint32_t)(threadIdx.x & 63) == (uint32_t)__builtin_ctzll(cm))
            atomicAdd(&a.g->n_complex, (unsigned long long)__popcll(cm));
    }
    if (a.host_ctl) publish_ctl(a.g, &a.g->fin_done, a.host_ctl, a.seq);
}

// ---- composition of the order-dependent flows at their owner ----------------
// the owner's summaries of complex flows, as (flow << 8 | shard, summary index)
__global__ void __launch_bounds__(256) k_comp_collect(MergeArgs a, unsigned long long* keys, uint32_t* vals) {
    const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const uint32_t d = a.sd[i];
    if (d == FAIL || d >= a.T.fmax || !a.complex[d]) return;
    const unsigned long long pos = atomicAdd(&a.g->n_keys, 1ull);
    keys[pos] = ((unsigned long long)d << 8) | (i / a.cap);
    vals[pos] = (uint32_t)i;
}

// One thread per complex flow: offline_fluereflows.rs:97-157 over the shards
// in order, each shard as (A = its packets up to its first FIN/RST, f0, H =
// the instance it creates from "no flow" up to f0, T = the instance open at
// its end after f0).  Entering with a flow F open: F += A, closed at f0 (then
// T, if any, is open).  Entering with none: H is emitted at f0 (or stays open
// without f0), then T.
__global__ void __launch_bounds__(64) k_compose(MergeArgs a, const unsigned long long* keys, const uint32_t* vals,
                                                unsigned long long n) {
    const unsigned long long p = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n || (p > 0 && (keys[p - 1] >> 8) == (keys[p] >> 8))) return;
    const unsigned long long d = keys[p] >> 8;
    fluere_flow_piece F;
    bool open = false;
    for (unsigned long long q = p; q < n && (keys[q] >> 8) == d; q++) {
        const unsigned long long i = vals[q];
        const fluere_flow_summary& s = *merge_input(a, i);
        fluere_flow_piece A, H, T;
        bool has_f0, has_H, has_T;
        unsigned long long f0;
        if (s.annex == NONE32) {
            piece_of_summary(s, A);
            has_f0 = s.finrst_min != NONE64;
            f0 = s.finrst_min;
            has_H = s.first_create != NONE64;  // == first_all (the local certificate held)
            H = A;
            has_T = false;
        } else if (s.annex >= a.cap_annex) {  // a corrupt block: never read past its annexes
            atomicOr(a.T.err, ERR_CAPACITY);
            return;
        } else {
            const fluere_flow_annex& x = *merge_annex(a, i, s.annex);
            has_f0 = x.flags & 1;
            f0 = x.f0;
            has_H = x.flags & 4;
            has_T = x.flags & 8;
            piece_clear(A);
            if (x.flags & 2) piece_add(A, x.lead);
            if (has_H) piece_add(A, x.head);
            H = x.head;
            T = x.tail;
        }
        fluere_record r;
        if (open) {
            piece_add(F, A);
            if (has_f0) {
                record_of_piece(F, f0, r);
                emit_record(a.g, a.out, a.out_cap, r);
                open = false;
            }
        } else if (has_f0) {
            if (has_H) {
                record_of_piece(H, f0, r);
                emit_record(a.g, a.out, a.out_cap, r);
            }
        } else if (has_H) {
            F = H;
            open = true;
        }
        if (has_f0 && has_T) {
            F = T;
            open = true;
        }
    }
    if (open) {
        fluere_record r;
        record_of_piece(F, NONE64, r);
        emit_record(a.g, a.out, a.out_cap, r);
    }
}

// ---- the compact wire encoding of export blocks ------------------------------
// A wide block (fluere_flow_summary, 256 B each) carries every field at full
// width.  On the wire each summary is a variable-length record: a descriptor
// word says which fields are present and how wide; absent fields (zero
// counters, flag counts, a first FIN/RST, a first packet that differs from the
// creating one, the seed of a flow with no creating packet) take no bytes, and
// an IPv4 5-tuple key takes 12 bytes instead of 56.  Wire block of one owner:
// the block header, a u32 offset table (one per summary, relative to the
// records), the records (4-byte aligned), the annexes verbatim (16-byte
// aligned).  The owner expands every received block back to the wide layout,
// at the same positions, before fluere_merge_gathered.
enum : uint32_t {
    WB_PK0 = 1u << 18, WB_PK1 = 1u << 19, WB_WBY = 1u << 20, WB_WMM = 1u << 21, WB_FC = 1u << 22,
    WB_FA = 1u << 23,  WB_FR = 1u << 24,  WB_AX = 1u << 25,  WB_DIR = 1u << 26, WB_V6 = 1u << 27,
    WB_LADDR = 1u << 28, WB_FULLKEY = 1u << 29,
};
constexpr uint32_t WIRE_REC_MAX = 4 + 56 + 8 + 16 + 20 + 32 + 16 + 16 + 16 + 4 + 32 + 4;  // 224
constexpr uint32_t WIRE_MAX_BLOCKS = 64;  // shards of one unpack (kernel-argument offsets)

__device__ __forceinline__ bool wire_short_key(const fluere_flow_summary& s) {
    uint32_t o = s.key[9] >> 10;
#pragma unroll
    for (int j = 0; j < 14; j++)
        if (j != 0 && j != 4 && j != 8 && j != 9) o |= s.key[j];
    return o == 0;
}
__device__ __forceinline__ bool wire_long_addr(const fluere_flow_summary& s) {
    uint32_t o = s.first_v6;
#pragma unroll
    for (int k = 4; k < 16; k++) o |= s.first_src[k] | s.first_dst[k];
    return o != 0;
}
__device__ __forceinline__ uint32_t wire_desc(const fluere_flow_summary& s) {
    uint32_t fm = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) fm |= (s.flag_cnt[q] ? 1u : 0u) << q;
    uint32_t d = (s.key[9] & 0x3FFu) | (fm << 10);
    d |= s.pkts[0] ? WB_PK0 : 0u;
    d |= s.pkts[1] ? WB_PK1 : 0u;
    d |= (s.bytes[0] > 0xFFFFFFFFull || s.bytes[1] > 0xFFFFFFFFull) ? WB_WBY : 0u;
    d |= (s.min_pkt > 0xFFFFu || s.max_pkt > 0xFFFFu || s.min_ttl > 0xFFu || s.max_ttl > 0xFFu) ? WB_WMM : 0u;
    d |= s.first_create != NONE64 ? WB_FC : 0u;
    d |= s.first_all != s.first_create ? WB_FA : 0u;
    d |= s.finrst_min != NONE64 ? WB_FR : 0u;
    d |= s.annex != NONE32 ? WB_AX : 0u;
    d |= s.first_dir ? WB_DIR : 0u;
    d |= s.first_v6 ? WB_V6 : 0u;
    d |= wire_long_addr(s) ? WB_LADDR : 0u;
    d |= wire_short_key(s) ? 0u : WB_FULLKEY;
    return d;
}
__device__ __forceinline__ uint32_t wire_bytes(uint32_t d) {
    const uint32_t by = (d & WB_WBY) ? 8u : 4u;
    uint32_t n = 4 + ((d & WB_FULLKEY) ? 56u : 12u);
    n += (d & WB_PK0) ? 4u + by : 0u;
    n += (d & WB_PK1) ? 4u + by : 0u;
    n += (d & WB_WMM) ? 20u : 8u;  // min / max pkt, ttl (+ prot, tos)
    n += 4u * __popc((d >> 10) & 0xFFu);
    n += 8u + 8u;  // last, last_time
    n += (d & WB_FA) ? 8u : 0u;
    n += (d & WB_FR) ? 8u : 0u;
    n += (d & WB_FC) ? 8u + 8u + 4u + ((d & WB_LADDR) ? 32u : 8u) : 0u;  // first_create, first_time, ports, addresses
    n += (d & WB_AX) ? 4u : 0u;
    return n;
}
struct WirePut {
    uint32_t* p;
    __device__ __forceinline__ void u32(uint32_t v) { *p++ = v; }
    __device__ __forceinline__ void u64(unsigned long long v) { p[0] = (uint32_t)v; p[1] = (uint32_t)(v >> 32); p += 2; }
    __device__ __forceinline__ void bytes(const uint8_t* b, int n) {
        for (int k = 0; k < n; k += 4) u32(b[k] | (b[k + 1] << 8) | (b[k + 2] << 16) | ((uint32_t)b[k + 3] << 24));
    }
};
struct WireGet {
    const uint32_t* p;
    __device__ __forceinline__ uint32_t u32() { return *p++; }
    __device__ __forceinline__ unsigned long long u64() {
        const unsigned long long v = p[0] | ((unsigned long long)p[1] << 32);
        p += 2;
        return v;
    }
    __device__ __forceinline__ void bytes(uint8_t* b, int n) {
        for (int k = 0; k < n; k += 4) {
            const uint32_t v = u32();
            b[k] = (uint8_t)v; b[k + 1] = (uint8_t)(v >> 8); b[k + 2] = (uint8_t)(v >> 16); b[k + 3] = (uint8_t)(v >> 24);
        }
    }
};
__device__ __forceinline__ void wire_put(const fluere_flow_summary& s, uint32_t d, uint32_t* dst) {
    WirePut w{dst};
    w.u32(d);
    if (d & WB_FULLKEY) {
#pragma unroll
        for (int j = 0; j < 14; j++) w.u32(s.key[j]);
    } else {
        w.u32(s.key[0]); w.u32(s.key[4]); w.u32(s.key[8]);
    }
#pragma unroll
    for (int q = 0; q < 2; q++)
        if (d & (q ? WB_PK1 : WB_PK0)) {
            w.u32(s.pkts[q]);
            if (d & WB_WBY) w.u64(s.bytes[q]);
            else w.u32((uint32_t)s.bytes[q]);
        }
    if (d & WB_WMM) {
        w.u32(s.min_pkt); w.u32(s.max_pkt); w.u32(s.min_ttl); w.u32(s.max_ttl);
        w.u32((uint32_t)s.first_prot | ((uint32_t)s.first_tos << 8));
    } else {
        w.u32(s.min_pkt | (s.max_pkt << 16));
        w.u32(s.min_ttl | (s.max_ttl << 8) | ((uint32_t)s.first_prot << 16) | ((uint32_t)s.first_tos << 24));
    }
#pragma unroll
    for (int q = 0; q < 8; q++)
        if ((d >> (10 + q)) & 1) w.u32(s.flag_cnt[q]);
    w.u64(s.last);
    w.u64(s.last_time);
    if (d & WB_FA) w.u64(s.first_all);
    if (d & WB_FR) w.u64(s.finrst_min);
    if (d & WB_FC) {
        w.u64(s.first_create);
        w.u64(s.first_time);
        w.u32(s.first_sport | ((uint32_t)s.first_dport << 16));
        const int na = (d & WB_LADDR) ? 16 : 4;
        w.bytes(s.first_src, na);
        w.bytes(s.first_dst, na);
    }
    if (d & WB_AX) w.u32(s.annex);
}
__device__ __forceinline__ void wire_get(const uint32_t* src, uint32_t shard, fluere_flow_summary& s) {
    memset(&s, 0, sizeof s);
    WireGet w{src};
    const uint32_t d = w.u32();
    if (d & WB_FULLKEY) {
#pragma unroll
        for (int j = 0; j < 14; j++) s.key[j] = w.u32();
    } else {
        s.key[0] = w.u32(); s.key[4] = w.u32(); s.key[8] = w.u32();
        s.key[9] = d & 0x3FFu;
    }
#pragma unroll
    for (int q = 0; q < 2; q++)
        if (d & (q ? WB_PK1 : WB_PK0)) {
            s.pkts[q] = w.u32();
            s.bytes[q] = (d & WB_WBY) ? w.u64() : (unsigned long long)w.u32();
        }
    if (d & WB_WMM) {
        s.min_pkt = w.u32(); s.max_pkt = w.u32(); s.min_ttl = w.u32(); s.max_ttl = w.u32();
        const uint32_t x = w.u32();
        s.first_prot = (uint8_t)x; s.first_tos = (uint8_t)(x >> 8);
    } else {
        const uint32_t a = w.u32(), b = w.u32();
        s.min_pkt = a & 0xFFFFu; s.max_pkt = a >> 16;
        s.min_ttl = b & 0xFFu; s.max_ttl = (b >> 8) & 0xFFu; s.first_prot = (uint8_t)(b >> 16); s.first_tos = (uint8_t)(b >> 24);
    }
#pragma unroll
    for (int q = 0; q < 8; q++) s.flag_cnt[q] = ((d >> (10 + q)) & 1) ? w.u32() : 0u;
    s.last = w.u64();
    s.last_time = w.u64();
    s.first_create = NONE64;
    s.finrst_min = NONE64;
    const unsigned long long fa = (d & WB_FA) ? w.u64() : 0ull;
    if (d & WB_FR) s.finrst_min = w.u64();
    if (d & WB_FC) {
        s.first_create = w.u64();
        s.first_time = w.u64();
        const uint32_t pp = w.u32();
        s.first_sport = (uint16_t)pp; s.first_dport = (uint16_t)(pp >> 16);
        const int na = (d & WB_LADDR) ? 16 : 4;
        w.bytes(s.first_src, na);
        w.bytes(s.first_dst, na);
    }
    s.first_all = (d & WB_FA) ? fa : s.first_create;
    s.first_dir = (d & WB_DIR) ? 1 : 0;
    s.first_v6 = (d & WB_V6) ? 1 : 0;
    s.annex = (d & WB_AX) ? w.u32() : NONE32;
    s.shard = shard;
}

struct WireArgs {
    const uint8_t* blocks;       // wide blocks (pack: the export's; unpack: the merge's)
    uint8_t* wblocks;
    const uint8_t* wire;
    uint8_t* wwire;
    uint64_t cap, cap_annex, block_bytes;
    uint32_t n_blocks;
    unsigned long long* sz;      // pack: [n_blocks * cap + 1] record bytes (0: absent)
    unsigned long long* scan;    // pack: exclusive sum of sz
    unsigned long long* woff;    // [n_blocks + 1]: offset of each wire block (device)
    unsigned long long* sizes;   // pack: [n_blocks] bytes of each wire block (the caller's device buffer)
    unsigned long long off_h[WIRE_MAX_BLOCKS + 1];  // unpack: offset of each received wire block, then the end
    // slotted form (the device-agreed step, no host-known sizes): block b in
    // the fixed slot [b * slot, (b + 1) * slot), a 16-byte prefix {bytes,
    // 0} before it; a block that does not fit sends only the prefix with
    // bytes = WIRE_OVER, which the owner unpacks as a block cut short
    uint64_t slot;               // 0: the contiguous form
};
constexpr unsigned long long WIRE_OVER = ~0ull;
constexpr uint64_t WIRE_SLOT_PREFIX = 16;
__device__ __forceinline__ uint64_t wire_table_bytes(uint64_t n) { return (4 * n + 15) & ~15ull; }
__device__ __forceinline__ uint64_t blk_count(const uint8_t* blocks, uint64_t block_bytes, uint32_t b, uint64_t cap) {
    return min((unsigned long long)reinterpret_cast<const fluere_shard_header*>(blocks + (size_t)b * block_bytes)->n_flows,
               (unsigned long long)cap);
}
__device__ __forceinline__ uint64_t blk_acount(const uint8_t* blocks, uint64_t block_bytes, uint32_t b, uint64_t cap_annex) {
    return min((unsigned long long)reinterpret_cast<const fluere_shard_header*>(blocks + (size_t)b * block_bytes)->n_annex,
               (unsigned long long)cap_annex);
}

// pack 1: each summary's record bytes (0 for the absent slots past n_flows)
__global__ void __launch_bounds__(256) k_wire_size(WireArgs a) {
    const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned long long n = (unsigned long long)a.n_blocks * a.cap;
    if (i > n) return;
    unsigned long long v = 0;
    if (i < n) {
        const uint32_t b = (uint32_t)(i / a.cap);
        const uint64_t j = i % a.cap;
        if (j < blk_count(a.blocks, a.block_bytes, b, a.cap)) {
            const fluere_flow_summary* s = reinterpret_cast<const fluere_flow_summary*>(
                a.blocks + (size_t)b * a.block_bytes + sizeof(fluere_shard_header)) + j;
            v = wire_bytes(wire_desc(*s));
        }
    }
    a.sz[i] = v;
}
// pack 2 (one thread): each wire block's size and offset
__global__ void k_wire_offsets(WireArgs a) {
    if (threadIdx.x || blockIdx.x) return;
    unsigned long long off = 0;
    for (uint32_t b = 0; b < a.n_blocks; b++) {
        const uint64_t n = blk_count(a.blocks, a.block_bytes, b, a.cap);
        const uint64_t na = blk_acount(a.blocks, a.block_bytes, b, a.cap_annex);
        const uint64_t rec = a.scan[(size_t)(b + 1) * a.cap] - a.scan[(size_t)b * a.cap];
        const uint64_t bytes = sizeof(fluere_shard_header) + wire_table_bytes(n) + ((rec + 15) & ~15ull) +
                               na * sizeof(fluere_flow_annex);
        if (a.slot) {  // fixed slots: the prefix, then the block when it fits
            const bool fits = bytes <= a.slot - WIRE_SLOT_PREFIX;
            reinterpret_cast<unsigned long long*>(a.wwire + (size_t)b * a.slot)[0] = fits ? bytes : WIRE_OVER;
            reinterpret_cast<unsigned long long*>(a.wwire + (size_t)b * a.slot)[1] = 0ull;
            a.woff[b] = (unsigned long long)b * a.slot + WIRE_SLOT_PREFIX;
            a.sizes[b] = fits ? bytes : WIRE_OVER;
            continue;
        }
        a.woff[b] = off;
        a.sizes[b] = bytes;
        off += bytes;
    }
    a.woff[a.n_blocks] = a.slot ? (unsigned long long)a.n_blocks * a.slot : off;
}
// pack 3: header, offset table and record of each summary (thread per summary slot)
__global__ void __launch_bounds__(256) k_wire_pack(WireArgs a) {
    const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (unsigned long long)a.n_blocks * a.cap) return;
    const uint32_t b = (uint32_t)(i / a.cap);
    const uint64_t j = i % a.cap;
    const uint8_t* wb = a.blocks + (size_t)b * a.block_bytes;
    if (a.slot && a.sizes[b] == WIRE_OVER) return;  // (does not fit its slot: the prefix says so)
    uint8_t* out = a.wwire + a.woff[b];
    const uint64_t n = blk_count(a.blocks, a.block_bytes, b, a.cap);
    if (j == 0) *reinterpret_cast<fluere_shard_header*>(out) = *reinterpret_cast<const fluere_shard_header*>(wb);
    if (j >= n) return;
    const uint32_t rel = (uint32_t)(a.scan[i] - a.scan[(size_t)b * a.cap]);
    reinterpret_cast<uint32_t*>(out + sizeof(fluere_shard_header))[j] = rel;
    const fluere_flow_summary& s = *(reinterpret_cast<const fluere_flow_summary*>(wb + sizeof(fluere_shard_header)) + j);
    wire_put(s, wire_desc(s), reinterpret_cast<uint32_t*>(out + sizeof(fluere_shard_header) + wire_table_bytes(n) + rel));
}
// pack 4 / unpack 2: the annexes, verbatim (thread per 16-byte word)
__global__ void __launch_bounds__(256) k_wire_annex(WireArgs a, int unpack) {
    const uint32_t b = blockIdx.y;
    // slotted form: the block's bytes from its prefix (WIRE_OVER: nothing sent)
    const unsigned long long sbytes =
        !a.slot ? 0ull : unpack ? reinterpret_cast<const unsigned long long*>(a.wire + (size_t)b * a.slot)[0] : a.sizes[b];
    if (a.slot && sbytes == WIRE_OVER) return;
    const uint8_t* hdrp = unpack ? a.wire + a.off_h[b] : a.blocks + (size_t)b * a.block_bytes;
    const fluere_shard_header& h = *reinterpret_cast<const fluere_shard_header*>(hdrp);
    const uint64_t n = min((unsigned long long)h.n_flows, (unsigned long long)a.cap);
    const uint64_t na = min((unsigned long long)h.n_annex, (unsigned long long)a.cap_annex);
    const uint64_t words = na * sizeof(fluere_flow_annex) / 16;
    const uint8_t* wide_ax = (unpack ? a.wblocks : a.blocks) + (size_t)b * a.block_bytes + sizeof(fluere_shard_header) +
                             a.cap * sizeof(fluere_flow_summary);
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < words; k += (uint64_t)gridDim.x * blockDim.x) {
        if (!unpack) {
            const uint64_t rec = a.scan[(size_t)(b + 1) * a.cap] - a.scan[(size_t)b * a.cap];
            uint8_t* wax = a.wwire + a.woff[b] + sizeof(fluere_shard_header) + wire_table_bytes(n) + ((rec + 15) & ~15ull);
            reinterpret_cast<uint4*>(wax)[k] = reinterpret_cast<const uint4*>(wide_ax)[k];
        } else {
            // the received block's records end at the start of its annexes: total - annex bytes
            const uint8_t* wend = a.slot ? a.wire + a.off_h[b] + sbytes : a.wire + a.off_h[b + 1];
            const uint8_t* wax = wend - na * sizeof(fluere_flow_annex);
            reinterpret_cast<uint4*>(const_cast<uint8_t*>(wide_ax))[k] = reinterpret_cast<const uint4*>(wax)[k];
        }
    }
}
// unpack 1: the wide block header and summaries (thread per summary slot)
__global__ void __launch_bounds__(256) k_wire_unpack(WireArgs a) {
    const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (unsigned long long)a.n_blocks * a.cap) return;
    const uint32_t b = (uint32_t)(i / a.cap);
    const uint64_t j = i % a.cap;
    const uint8_t* in = a.wire + a.off_h[b];
    uint8_t* wb = a.wblocks + (size_t)b * a.block_bytes;
    if (a.slot && reinterpret_cast<const unsigned long long*>(a.wire + (size_t)b * a.slot)[0] == WIRE_OVER) {
        // the sender's block did not fit its slot: a block cut short (the merge asks for the redo)
        if (j == 0) {
            fluere_shard_header h{};
            h.n_annex = a.cap_annex + 1;  // (no summary is read; k_merge_insert flags ERR_CAPACITY)
            h.shard = b;
            *reinterpret_cast<fluere_shard_header*>(wb) = h;
        }
        return;
    }
    const fluere_shard_header& h = *reinterpret_cast<const fluere_shard_header*>(in);
    if (j == 0) *reinterpret_cast<fluere_shard_header*>(wb) = h;
    const uint64_t n = min((unsigned long long)h.n_flows, (unsigned long long)a.cap);
    if (j >= n) return;
    const uint32_t rel = reinterpret_cast<const uint32_t*>(in + sizeof(fluere_shard_header))[j];
    fluere_flow_summary s;
    wire_get(reinterpret_cast<const uint32_t*>(in + sizeof(fluere_shard_header) + wire_table_bytes(n) + rel), h.shard, s);
    *(reinterpret_cast<fluere_flow_summary*>(wb + sizeof(fluere_shard_header)) + j) = s;
}

}  // namespace fl

// ---------------------------------------------------------------------------
// multi-GPU merge
// ---------------------------------------------------------------------------
extern "C" uint64_t fluere_capacity(fluere_ctx* c) { return c ? c->fmax : 0; }
extern "C" uint64_t fluere_total_packets(fluere_ctx* c) { return c ? c->n_total : 0; }

extern "C" int fluere_set_index_base(fluere_ctx* c, uint64_t base) {
    if (!c) return FLUERE_E_ARG;
    if (!c->batches.empty()) return FLUERE_E_STATE;
    c->index_base = base;
    return FLUERE_OK;
}

extern "C" uint64_t fluere_shard_block_bytes(uint64_t cap, uint64_t cap_annex) {
    return sizeof(fluere_shard_header) + cap * sizeof(fluere_flow_summary) + cap_annex * sizeof(fluere_flow_annex);
}

// Record buffer of at least `need` records, keeping the first `keep`.
int grow_recs_keep(fluere_ctx* c, uint64_t need, uint64_t keep) {
    if (need <= c->d_recs_cap) return FLUERE_OK;
    fluere_record* nr = nullptr;
    const uint64_t cap = std::max<uint64_t>(need, 1024);
    if (hipMalloc(&nr, cap * sizeof(fluere_record)) != hipSuccess) return FLUERE_E_NOMEM;
    if (keep) HIPCHECK(hipMemcpyAsync(nr, c->d_recs, keep * sizeof(fluere_record), hipMemcpyDeviceToDevice, c->stream));
    HIPCHECK(ctx_sync(c));
    hipFree(c->d_recs);
    c->d_recs = nr;
    c->d_recs_cap = cap;
    return FLUERE_OK;
}

extern "C" int fluere_export_device(fluere_ctx* c, void* d_blocks, uint32_t n_owners, uint32_t shard, uint64_t cap,
                                    uint64_t cap_annex, uint64_t* need, uint64_t* need_annex) {
    if (!c || !d_blocks || !n_owners || !cap) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    int rc;
    if ((rc = upload_batches(c))) return rc;
    const TableSet T = tables_of(c);
    const int nb = (int)c->batches.size();
    if (!c->d_annex_of && hipMalloc(&c->d_annex_of, (size_t)c->fmax * 4) != hipSuccess) return FLUERE_E_NOMEM;
    if (!c->d_sumpos && hipMalloc(&c->d_sumpos, (size_t)c->fmax * 4) != hipSuccess) return FLUERE_E_NOMEM;
    if (!c->d_need && hipMalloc(&c->d_need, 16) != hipSuccess) return FLUERE_E_NOMEM;
    FinArgs fa{c->d_batches, nb, T, c->acc, c->d_glob, nullptr, c->d_complex, c->use_mac};
    // 1. flows whose part of the state machine depends on packet order here
    reset_record_counters(c);
    k_local_cert<<<flow_grid(c), 256, 0, s>>>(fa, c->d_annex_of);
    // 3. summaries (+ annexes) into the owners' blocks, enqueued behind it
    //    speculatively: with no order-dependent flow (the common case) the
    //    export needs ONE host round trip
    ExportArgs ea{fa, (uint8_t*)d_blocks, n_owners, shard, cap, cap_annex, fluere_shard_block_bytes(cap, cap_annex),
                  c->d_annex_of, (const fluere_flow_annex*)c->d_annex, c->d_sumpos};
    auto enqueue_export = [&](bool annexes) -> int {
        ea.annex = annexes ? (const fluere_flow_annex*)c->d_annex : nullptr;
        k_export_hdr<<<grid_for(n_owners, 64), 64, 0, s>>>(ea);
        k_export_owners<<<flow_grid(c), 256, 0, s>>>(ea);
        k_export_need<<<1, 64, 0, s>>>(ea, (unsigned long long*)c->d_need, nullptr);
        HIPCHECK(hipGetLastError());
        return FLUERE_OK;
    };
    if ((rc = enqueue_export(false))) return rc;
    struct {
        Ctl ctl;
        unsigned long long nd[2];
    } back;
    HIPCHECK(hipMemcpyAsync(&back.ctl, c->d_glob, sizeof back.ctl, hipMemcpyDeviceToHost, s));
    HIPCHECK(hipMemcpyAsync(back.nd, c->d_need, 16, hipMemcpyDeviceToHost, s));
    HIPCHECK(ctx_sync(c));
    Glob g = back.ctl.g;
    if (!(back.ctl.err & (ERR_TABLE_FULL | ERR_SPIN))) c->last_nf = back.ctl.n_flows;  // (merge owner estimate)
    // 2. order-dependent flows: their annexes (and the records that open and
    //    close in this shard) from the exact state machine, then the export again
    if (g.n_complex) {
        std::vector<Batch> hb(nb);
        for (int i = 0; i < nb; i++) hb[i] = c->batches[i].b;
        ExactJob J{c->d_batches, hb.data(), nb, T, c->use_mac, 0, c->timeout_ms * 1000ull, c->d_complex, c->d_glob,
                   &c->d_recs, &c->d_recs_cap, &c->d_exact, &c->d_exact_bytes,
                   1, &c->d_annex, &c->d_annex_cap, c->d_annex_of};
        J.mail = c->h_mail;
        ExactResult er{};
        if ((rc = exact_run(J, s, &er))) return rc < 0 ? rc : FLUERE_E_HIP;
        if ((rc = enqueue_export(true))) return rc;
        HIPCHECK(hipMemcpyAsync(&g, c->d_glob, sizeof g, hipMemcpyDeviceToHost, s));
        HIPCHECK(hipMemcpyAsync(back.nd, c->d_need, 16, hipMemcpyDeviceToHost, s));
        HIPCHECK(ctx_sync(c));
    }
    if (need) *need = back.nd[0];
    if (need_annex) *need_annex = back.nd[1];
    // the final records this shard produced (kept through the merge)
    c->local_n_rec = g.n_rec;
    c->local_updates = g.n_updates;
    c->local_ended = g.n_ended;
    return FLUERE_OK;
}

// The common-case export without a host round trip: the certificate and the
// summaries (no annexes) are enqueued, and d_info (device, 4 x u64) receives
// {largest per-owner summary count, annex count, order-dependent flows, flow
// count}.  The caller reduces d_info over the ranks (MAX) on the context's
// stream and reads it once; if any rank has order-dependent flows, every rank
// runs fluere_export_device instead (annexes), and blocks that were too small
// are exported again with larger capacities.
extern "C" int fluere_export_async(fluere_ctx* c, void* d_blocks, uint32_t n_owners, uint32_t shard, uint64_t cap,
                                   uint64_t cap_annex, unsigned long long* d_info) {
    if (!c || !d_blocks || !n_owners || !cap || !d_info) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    int rc;
    if ((rc = upload_batches(c))) return rc;
    const int nb = (int)c->batches.size();
    if (!c->d_annex_of && hipMalloc(&c->d_annex_of, (size_t)c->fmax * 4) != hipSuccess) return FLUERE_E_NOMEM;
    if (!c->d_sumpos && hipMalloc(&c->d_sumpos, (size_t)c->fmax * 4) != hipSuccess) return FLUERE_E_NOMEM;
    if (!c->d_need && hipMalloc(&c->d_need, 16) != hipSuccess) return FLUERE_E_NOMEM;
    FinArgs fa{c->d_batches, nb, tables_of(c), c->acc, c->d_glob, nullptr, c->d_complex, c->use_mac};
    reset_record_counters(c);
    k_local_cert<<<flow_grid(c), 256, 0, s>>>(fa, c->d_annex_of);
    ExportArgs ea{fa, (uint8_t*)d_blocks, n_owners, shard, cap, cap_annex, fluere_shard_block_bytes(cap, cap_annex),
                  c->d_annex_of, nullptr, c->d_sumpos};
    k_export_hdr<<<grid_for(n_owners, 64), 64, 0, s>>>(ea);
    k_export_owners<<<flow_grid(c), 256, 0, s>>>(ea);
    k_export_need<<<1, 64, 0, s>>>(ea, (unsigned long long*)c->d_need, d_info);
    HIPCHECK(hipGetLastError());
    c->local_n_rec = c->local_updates = c->local_ended = 0;  // (no order-dependent flow: no local record)
    // the shard's flow count, for the next pass's owner count: read after the
    // merge's wait (a spare word of the pinned control copy)
    HIPCHECK(hipMemcpyAsync(&c->h_ctl->pad[0], c->d_nflows, 4, hipMemcpyDeviceToHost, s));
    c->async_nf = true;
    return FLUERE_OK;
}

// ---- the compact wire encoding (include/fluere_gpu.h) -------------------------
extern "C" uint64_t fluere_wire_bound(uint64_t cap, uint64_t cap_annex) {
    return sizeof(fluere_shard_header) + ((4 * cap + 15) & ~15ull) + ((cap * WIRE_REC_MAX + 15) & ~15ull) +
           cap_annex * sizeof(fluere_flow_annex);
}

static int wire_pack(fluere_ctx* c, const void* d_blocks, uint32_t n_owners, uint64_t cap, uint64_t cap_annex,
                     void* d_wire, unsigned long long* d_sizes, uint64_t slot) {
    if (cap * WIRE_REC_MAX >= (1ull << 32)) return FLUERE_E_ARG;  // u32 record offsets within a block
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const uint64_t n = (uint64_t)n_owners * cap;
    size_t tb = 0;
    (void)prim_exclusive_sum(nullptr, tb, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                           (int)(n + 1), s);
    // (+ n_owners words: the slotted form's block sizes when the caller has no buffer for them)
    const size_t need = 2 * (n + 1) * 8 + (size_t)(n_owners + 1) * 8 + (size_t)n_owners * 8 + ((tb + 255) & ~(size_t)255);
    if (need > c->d_wire_tmp_bytes) {
        hipFree(c->d_wire_tmp);
        c->d_wire_tmp = nullptr;
        c->d_wire_tmp_bytes = 0;
        if (hipMalloc(&c->d_wire_tmp, need) != hipSuccess) return FLUERE_E_NOMEM;
        c->d_wire_tmp_bytes = need;
    }
    WireArgs a{};
    a.blocks = (const uint8_t*)d_blocks;
    a.wwire = (uint8_t*)d_wire;
    a.cap = cap;
    a.cap_annex = cap_annex;
    a.block_bytes = fluere_shard_block_bytes(cap, cap_annex);
    a.n_blocks = n_owners;
    a.slot = slot;
    char* t = (char*)c->d_wire_tmp;
    void* tmp = t;
    a.sz = (unsigned long long*)(t + ((tb + 255) & ~(size_t)255));
    a.scan = a.sz + (n + 1);
    a.woff = a.scan + (n + 1);
    a.sizes = d_sizes ? d_sizes : a.woff + (n_owners + 1);
    k_wire_size<<<grid_for(n + 1, 256), 256, 0, s>>>(a);
    HIPCHECK(prim_exclusive_sum(tmp, tb, a.sz, a.scan, (int)(n + 1), s));
    k_wire_offsets<<<1, 64, 0, s>>>(a);
    k_wire_pack<<<grid_for(n, 256), 256, 0, s>>>(a);
    const unsigned ax = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(64, cap_annex * 32 / 256));
    k_wire_annex<<<dim3(ax, n_owners), 256, 0, s>>>(a, 0);
    HIPCHECK(hipGetLastError());
    return FLUERE_OK;
}

extern "C" int fluere_wire_pack(fluere_ctx* c, const void* d_blocks, uint32_t n_owners, uint64_t cap, uint64_t cap_annex,
                                void* d_wire, unsigned long long* d_sizes) {
    if (!c || !d_blocks || !d_wire || !d_sizes || !n_owners || !cap) return FLUERE_E_ARG;
    return wire_pack(c, d_blocks, n_owners, cap, cap_annex, d_wire, d_sizes, 0);
}

extern "C" int fluere_wire_pack_slots(fluere_ctx* c, const void* d_blocks, uint32_t n_owners, uint64_t cap,
                                      uint64_t cap_annex, uint64_t slot_bytes, void* d_slots) {
    if (!c || !d_blocks || !d_slots || !n_owners || !cap || slot_bytes < WIRE_SLOT_PREFIX + sizeof(fluere_shard_header) ||
        slot_bytes % 16)
        return FLUERE_E_ARG;
    return wire_pack(c, d_blocks, n_owners, cap, cap_annex, d_slots, nullptr, slot_bytes);
}

static int wire_unpack(fluere_ctx* c, const void* d_wire, uint32_t n_shards, const uint64_t* sizes, uint64_t slot,
                       uint64_t cap, uint64_t cap_annex, void* d_blocks) {
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    WireArgs a{};
    a.wire = (const uint8_t*)d_wire;
    a.wblocks = (uint8_t*)d_blocks;
    a.cap = cap;
    a.cap_annex = cap_annex;
    a.block_bytes = fluere_shard_block_bytes(cap, cap_annex);
    a.n_blocks = n_shards;
    a.slot = slot;
    unsigned long long off = 0;
    for (uint32_t b = 0; b < n_shards; b++) {
        if (slot) {
            a.off_h[b] = (unsigned long long)b * slot + WIRE_SLOT_PREFIX;
            continue;
        }
        if (sizes[b] < sizeof(fluere_shard_header)) return FLUERE_E_ARG;
        a.off_h[b] = off;
        off += sizes[b];
    }
    a.off_h[n_shards] = slot ? (unsigned long long)n_shards * slot : off;
    const uint64_t n = (uint64_t)n_shards * cap;
    k_wire_unpack<<<grid_for(n, 256), 256, 0, s>>>(a);
    const unsigned ax = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(64, cap_annex * 32 / 256));
    k_wire_annex<<<dim3(ax, n_shards), 256, 0, s>>>(a, 1);
    HIPCHECK(hipGetLastError());
    return FLUERE_OK;
}

extern "C" int fluere_wire_unpack(fluere_ctx* c, const void* d_wire, uint32_t n_shards, const uint64_t* sizes,
                                  uint64_t cap, uint64_t cap_annex, void* d_blocks) {
    if (!c || !d_wire || !d_blocks || !sizes || !n_shards || n_shards > WIRE_MAX_BLOCKS || !cap) return FLUERE_E_ARG;
    return wire_unpack(c, d_wire, n_shards, sizes, 0, cap, cap_annex, d_blocks);
}

extern "C" int fluere_wire_unpack_slots(fluere_ctx* c, const void* d_slots, uint32_t n_shards, uint64_t slot_bytes,
                                        uint64_t cap, uint64_t cap_annex, void* d_blocks) {
    if (!c || !d_slots || !d_blocks || !n_shards || n_shards > WIRE_MAX_BLOCKS || !cap ||
        slot_bytes < WIRE_SLOT_PREFIX + sizeof(fluere_shard_header) || slot_bytes % 16)
        return FLUERE_E_ARG;
    return wire_unpack(c, d_slots, n_shards, nullptr, slot_bytes, cap, cap_annex, d_blocks);
}

// the run counters the owner merge starts from (the records this rank's
// export produced stay first in d_recs) -- a kernel, not a host copy
__global__ void k_merge_counters(Glob* g, unsigned long long n_rec, unsigned long long updates,
                                 unsigned long long ended) {
    if (threadIdx.x) return;
    g->n_rec = n_rec;
    g->n_updates = updates;
    g->n_ended = ended;
}
// 1 when the merge just enqueued cannot stand as the step's result: a block
// was cut short (a shard had more flows for this owner than cap), a shard's
// flow depends on packet order inside the shard (its annex is needed:
// ERR_BARE), the span reaches the timeout (the sweep composition), or the
// table filled.  Flows that are order-free on every shard but order-dependent
// once merged (a FIN ending shard 0's part, trailing ACKs in shard 1) need no
// redo: merge_complete composes them from the summaries (k_compose), as after
// the host-driven step.
__device__ __host__ __forceinline__ bool merge_redo(const Glob& g, uint32_t err, unsigned long long timeout_us) {
    const bool expiry = g.valid && g.tmax >= g.tmin && g.tmax - g.tmin >= timeout_us;
    return err != 0 || g.n_bare != 0 || expiry;
}
__global__ void k_merge_retry(const Glob* g, const uint32_t* err, unsigned long long timeout_us,
                              unsigned long long* out) {
    if (threadIdx.x) return;
    out[0] = merge_redo(*g, *err, timeout_us) ? 1ull : 0ull;
}

// Enqueues the owner merge (no host wait unless a buffer grows); seq: the
// number k_merge_finalize publishes.
static int merge_enqueue(fluere_ctx* c, const void* d_blocks, uint32_t n_shards, uint64_t cap, uint64_t cap_annex,
                         MergeArgs& ma, uint32_t& seq) {
    hipStream_t s = c->stream;
    int rc;
    const uint64_t n = (uint64_t)n_shards * cap;
    const uint64_t keep = c->local_n_rec;
    if ((rc = clear_flows(c))) return rc;
    c->precleaned = false;
    k_merge_counters<<<1, 64, 0, s>>>(c->d_glob, keep, c->local_updates, c->local_ended);
    if (!c->d_pay && hipMalloc(&c->d_pay, (size_t)c->fmax * sizeof(FirstPay)) != hipSuccess) return FLUERE_E_NOMEM;
    if (std::max<uint64_t>(n, 1) > c->d_sd_cap) {
        hipFree(c->d_sd);
        c->d_sd = nullptr;
        c->d_sd_cap = 0;
        if (hipMalloc(&c->d_sd, std::max<uint64_t>(n, 1) * 4) != hipSuccess) return FLUERE_E_NOMEM;
        c->d_sd_cap = std::max<uint64_t>(n, 1);
    }
    if ((rc = grow_recs_keep(c, keep + std::min<uint64_t>(std::max<uint64_t>(n, 1), c->fmax), keep))) return rc;
    c->merge_t0 = std::chrono::steady_clock::now();
    seq = ++c->run_seq ? c->run_seq : ++c->run_seq;  // never 0 (the initial value)
    ma = MergeArgs{tables_of(c), c->acc, n, c->d_sd, (FirstPay*)c->d_pay, c->d_glob, c->d_recs, c->d_complex,
                   c->d_recs_cap, (const uint8_t*)d_blocks, cap, cap_annex, fluere_shard_block_bytes(cap, cap_annex),
                   c->h_ctl, seq, c->timeout_ms * 1000ull};
    if (n) {
        k_merge_insert<<<grid_for(n, 256), 256, 0, s>>>(ma);
        k_merge_payload<<<grid_for(n, 256), 256, 0, s>>>(ma);
    }
    k_merge_finalize<<<flow_grid(c), 256, 0, s>>>(ma);
    HIPCHECK(hipGetLastError());
    return FLUERE_OK;
}

// The merge's results once k_merge_finalize published: the composition of
// order-dependent flows (unless `redo`: then FLUERE_RETRY), the stats.
static int merge_complete(fluere_ctx* c, MergeArgs& ma, uint32_t seq, uint32_t n_shards, uint64_t cap, bool redo,
                          fluere_stats* st) {
    hipStream_t s = c->stream;
    int rc;
    const uint64_t n = (uint64_t)n_shards * cap;
    Glob g;
    uint32_t nf_err[2];
    if ((rc = wait_published(c, seq, g, nf_err))) return rc;
    if (c->async_nf) {
        c->last_nf = c->h_ctl->pad[0];
        c->async_nf = false;
    }
    const uint64_t timeout_us = c->timeout_ms * 1000ull;
    if (redo && merge_redo(g, nf_err[1], timeout_us)) {
        c->have_results = false;
        return FLUERE_RETRY;
    }
    if (nf_err[1] & ERR_CAPACITY) return FLUERE_E_ARG;  // a shard had more flows than its block holds
    if (nf_err[1]) return FLUERE_E_TABLE_FULL;
    const bool expiry = g.valid && g.tmax >= g.tmin && g.tmax - g.tmin >= timeout_us;
    // order-dependent shard flows without annexes cannot be composed (the sweep
    // composition, with expiry, rebuilds every record from the packets instead)
    if (g.n_bare && !expiry) return FLUERE_E_ARG;
    if (g.n_complex && !expiry) {
        // the order-dependent flows: compose the shards' pieces in shard order
        unsigned long long *keys = nullptr, *keys2 = nullptr;
        uint32_t *vals = nullptr, *vals2 = nullptr;
        void* tmp = nullptr;
        size_t tb = 0;
        const uint64_t m = n;
        if (hipMalloc(&keys, m * 8) != hipSuccess || hipMalloc(&keys2, m * 8) != hipSuccess ||
            hipMalloc(&vals, m * 4) != hipSuccess || hipMalloc(&vals2, m * 4) != hipSuccess) {
            hipFree(keys); hipFree(keys2); hipFree(vals); hipFree(vals2);
            return FLUERE_E_NOMEM;
        }
        HIPCHECK(hipMemsetAsync(&c->d_glob->n_keys, 0, 8, s));
        k_comp_collect<<<grid_for(n, 256), 256, 0, s>>>(ma, keys, vals);
        unsigned long long nk = 0;
        HIPCHECK(hipMemcpyAsync(&nk, &c->d_glob->n_keys, 8, hipMemcpyDeviceToHost, s));
        HIPCHECK(ctx_sync(c));
        // records: the certified ones + at most one per shard piece
        if ((rc = grow_recs_keep(c, g.n_rec + 2 * nk, g.n_rec))) return rc;
        ma.out = c->d_recs;
        ma.out_cap = c->d_recs_cap;
        int end_bit = 8;
        while (end_bit < 64 && (1ull << (end_bit - 8)) <= c->fmax) end_bit++;
        (void)prim_sort_pairs(nullptr, tb, keys, keys2, vals, vals2, (int)nk, 0, end_bit, s);
        if (hipMalloc(&tmp, std::max<size_t>(tb, 16)) != hipSuccess) {
            hipFree(keys); hipFree(keys2); hipFree(vals); hipFree(vals2);
            return FLUERE_E_NOMEM;
        }
        HIPCHECK(prim_sort_pairs(tmp, tb, keys, keys2, vals, vals2, (int)nk, 0, end_bit, s));
        if (nk) k_compose<<<grid_for(nk, 64), 64, 0, s>>>(ma, keys2, vals2, nk);
        HIPCHECK(hipGetLastError());
        HIPCHECK(hipMemcpyAsync(&g, c->d_glob, sizeof g, hipMemcpyDeviceToHost, s));
        HIPCHECK(ctx_sync(c));
        hipFree(tmp); hipFree(keys); hipFree(keys2); hipFree(vals); hipFree(vals2);
    }
    const uint32_t nf = std::min(nf_err[0], c->fmax);
    c->dev_n_rec = g.n_rec;
    c->host_recs = false;
    c->dev_ordered = false;
    c->have_results = true;
    c->local_n_rec = c->local_updates = c->local_ended = 0;
    fluere_stats out{};
    out.valid = g.valid;
    out.dropped_parse = g.dropped;
    out.flows = nf;
    out.records = g.n_rec;
    out.ended = g.n_ended;
    out.complex_flows = g.n_complex;
    out.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - c->merge_t0).count();
    out.updates = g.n_updates;
    if (st) *st = out;
    // the hard-timeout sweep (offline_fluereflows.rs:161-175): the records
    // come from the sweep composition (fluere_sweep_*), which reads the
    // summary -> flow mapping of this merge
    c->merge_cap = cap;
    c->merge_shards = n_shards;
    c->has_aux = false;
    if (expiry) return FLUERE_NEED_SWEEP;
    return FLUERE_OK;
}

extern "C" int fluere_merge_gathered(fluere_ctx* c, const void* d_blocks, uint32_t n_shards, uint64_t cap,
                                     uint64_t cap_annex, fluere_stats* st) {
    if (!c || (!d_blocks && n_shards) || (n_shards && !cap)) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    MergeArgs ma{};
    uint32_t seq = 0;
    int rc;
    if (c->merge_p) c->merge_p->pending = false;
    if ((rc = merge_enqueue(c, d_blocks, n_shards, cap, cap_annex, ma, seq))) return rc;
    return merge_complete(c, ma, seq, n_shards, cap, false, st);
}

// The device-agreed step (dist.py): the merge enqueued without a host wait,
// and d_retry (device, one uint64) set to 1 when its result cannot stand (a
// block cut short, order-dependent flows, the span reaching the timeout) --
// the ranks reduce it (MAX) on the stream and read it once, the step's one
// host round trip; fluere_merge_gathered_finish then returns the stats, or
// FLUERE_RETRY when the step must be redone by the host-driven sequence.
extern "C" int fluere_merge_gathered_async(fluere_ctx* c, const void* d_blocks, uint32_t n_shards, uint64_t cap,
                                           uint64_t cap_annex, unsigned long long* d_retry) {
    if (!c || !d_retry || (!d_blocks && n_shards) || (n_shards && !cap)) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    int rc;
    if (!c->merge_p) c->merge_p = new MergePending{};
    MergePending& M = *c->merge_p;
    M.pending = false;
    if ((rc = merge_enqueue(c, d_blocks, n_shards, cap, cap_annex, M.ma, M.seq))) return rc;
    k_merge_retry<<<1, 64, 0, c->stream>>>(c->d_glob, tables_of(c).err, c->timeout_ms * 1000ull, d_retry);
    HIPCHECK(hipGetLastError());
    M.pending = true;
    M.shards = n_shards;
    M.cap = cap;
    return FLUERE_OK;
}

extern "C" int fluere_merge_gathered_finish(fluere_ctx* c, fluere_stats* st) {
    if (!c) return FLUERE_E_ARG;
    if (!c->merge_p || !c->merge_p->pending) return FLUERE_E_STATE;
    HIPCHECK(hipSetDevice(c->device));
    MergePending& M = *c->merge_p;
    M.pending = false;
    return merge_complete(c, M.ma, M.seq, M.shards, M.cap, true, st);
}

void merge_pending_free(fluere_ctx* c) {
    delete c->merge_p;
    c->merge_p = nullptr;
}

extern "C" uint64_t fluere_host_waits(fluere_ctx* c) { return c ? c->host_waits : 0; }

// ---------------------------------------------------------------------------
// sharded Mode B: the hard-timeout sweep composed across shards
// ---------------------------------------------------------------------------
// When the capture's span reaches the timeout, an expiry entry pushed at a
// creation fires at the first *processed* packet of the whole capture with
// t >= exp (offline_fluereflows.rs:103-119,161-175): shards are coupled.  The
// composition (driven by fluere_amd/dist.py):
//   1. every shard (holder) ships the metadata of its valid packets to the
//      keys' owners (32 B each, capture order within an owner): each owner
//      then holds every packet of its keys, in capture order;
//   2. per pass, every holder computes the sweep point of each of its
//      create-eligible packets over the packets processed so far -- first in
//      its own shard (max segment tree over the processed times), else by a
//      query to the first later shard whose latest processed time reaches
//      exp -- and ships the points to the owners, who run the exact chase
//      (exact.hip) and send back which packets were processed; repeated until
//      no owner's processed set changes (the single-GPU fixed point);
//   3. the owners ask the holders for the FluereRecord seeds of the creating
//      packets and build the records; their order stays global (order_key =
//      the ending packet's index plus two order words, fluere_get_record_order).
struct SweepState {
    // holder (this shard's packets)
    ExMeta* hcm = nullptr;              // valid packets, capture order (d = local flow)
    uint64_t hn = 0;
    uint32_t* hperm = nullptr;          // pack position -> local index
    uint8_t* hpr = nullptr;             // processed (local index)
    unsigned long long* hF = nullptr;   // sweep point (local index)
    unsigned long long* tree = nullptr;
    uint64_t P = 0;
    uint32_t* qk = nullptr;             // the local index of each query (grouped by target shard)
    uint64_t nq = 0;
    uint32_t n_owners = 0;
    std::vector<uint64_t> counts;       // packets per owner
    // owner (its keys' packets from every shard)
    ExMeta* ocm = nullptr;
    uint64_t on = 0;
    ExactSession* es = nullptr;
    unsigned long long* req = nullptr;  // creating packets of the instances (ascending)
    uint32_t* reqq = nullptr;           // their instance ordinals
    uint32_t n_inst = 0;
    Seed* seeds = nullptr;              // by instance ordinal
    int passes = 0;
    // scratch
    uint32_t *k1 = nullptr, *k2 = nullptr, *v1 = nullptr;
    unsigned long long* misc = nullptr; // small device scratch (counts)
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    uint32_t* err = nullptr;
};

void sweep_free(fluere_ctx* c) {
    SweepState* w = c->sw;
    if (!w) return;
    hipFree(w->hcm); hipFree(w->hperm); hipFree(w->hpr); hipFree(w->hF); hipFree(w->tree); hipFree(w->qk);
    hipFree(w->ocm); hipFree(w->req); hipFree(w->reqq); hipFree(w->seeds);
    hipFree(w->k1); hipFree(w->k2); hipFree(w->v1); hipFree(w->misc); hipFree(w->tmp); hipFree(w->err);
    if (w->es) exact_free(w->es);
    delete w;
    c->sw = nullptr;
}

static int sw_tmp(SweepState* w, size_t need) {
    if (need <= w->tmp_bytes) return FLUERE_OK;
    hipFree(w->tmp);
    w->tmp = nullptr;
    w->tmp_bytes = 0;
    if (hipMalloc(&w->tmp, need) != hipSuccess) return FLUERE_E_NOMEM;
    w->tmp_bytes = need;
    return FLUERE_OK;
}

static int bits_for(uint64_t v) {  // radix sort width for keys in [0, v]
    int b = 1;
    while (b < 64 && (v >> b)) b++;
    return b;
}

__global__ void __launch_bounds__(256) k_sw_owner(const ExMeta* cm, uint64_t n, const uint8_t* flow_key,
                                                  uint32_t n_owners, uint32_t* okey, uint32_t* val) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    okey[k] = key_owner(reinterpret_cast<const uint32_t*>(flow_key + (size_t)cm[k].d * 56), n_owners);
    val[k] = (uint32_t)k;
}

// counts[r] = entries equal to r among n sorted keys, r < m
__global__ void k_sw_kcount(const uint32_t* keys, uint64_t n, uint32_t m, unsigned long long* counts) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= m) return;
    auto lb = [&](uint32_t v) {
        uint64_t lo = 0, hi = n;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (keys[mid] < v) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    };
    counts[r] = lb(r + 1) - lb(r);
}

// the packet records for the owners: d = the flow's summary position in its block
__global__ void __launch_bounds__(256) k_sw_pack(const ExMeta* cm, const uint32_t* perm, uint64_t n,
                                                 const uint32_t* sumpos, ExMeta* out) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    ExMeta m = cm[perm[p]];
    m.d = sumpos[m.d];
    out[p] = m;
}

// owner: (shard s, summary position j) -> this context's flow id (the merge's sd)
__global__ void __launch_bounds__(256) k_sw_load(const ExMeta* in, uint64_t n, const unsigned long long* seg,
                                                 uint32_t n_shards, const uint32_t* sd, uint64_t cap, uint32_t fmax,
                                                 ExMeta* out, uint32_t* err) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t sh = 0;
    while (sh + 1 < n_shards && seg[sh + 1] <= i) sh++;
    ExMeta m = in[i];
    const uint32_t d = m.d < cap ? sd[sh * cap + m.d] : FAIL;
    if (d == FAIL || d >= fmax) {
        atomicOr(err, 1u);
        m.d = 0;
    } else {
        m.d = d;
    }
    out[i] = m;
}

__global__ void __launch_bounds__(256) k_sw_feedback(const uint8_t* back, const uint32_t* perm, uint64_t n, uint8_t* pr) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n) pr[perm[p]] = back[p];
}

// sweep point of every create-eligible packet, in this shard or a query
__global__ void __launch_bounds__(256) k_sw_points(const ExMeta* cm, uint64_t n, const unsigned long long* tree,
                                                   uint64_t P, unsigned long long timeout_us, uint32_t rank,
                                                   uint32_t n_ranks, const unsigned long long* maxt,
                                                   unsigned long long* F, uint32_t* tkey, uint32_t* val) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const ExMeta m = cm[k];
    unsigned long long f = NONE64;
    uint32_t target = n_ranks;  // none
    const unsigned long long exp = m.t + timeout_us < m.t ? NONE64 : m.t + timeout_us;
    if ((m.bits & 1) && exp != NONE64) {
        const uint64_t j = tree_first(tree, P, k, exp + 1);
        if (j < n) f = cm[j].gidx;
        else
            for (uint32_t r = rank + 1; r < n_ranks; r++)
                if (maxt[r] >= exp + 1) { target = r; break; }
    }
    F[k] = f;
    tkey[k] = target;
    val[k] = (uint32_t)k;
}

__global__ void __launch_bounds__(256) k_sw_qpack(const ExMeta* cm, const uint32_t* qk, uint64_t nq,
                                                  unsigned long long timeout_us, unsigned long long* q) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nq) q[i] = cm[qk[i]].t + timeout_us;  // (queried only when it does not saturate)
}

__global__ void __launch_bounds__(256) k_sw_answer(const unsigned long long* q, uint64_t nq, const unsigned long long* tree,
                                                   uint64_t P, const ExMeta* cm, uint64_t n, unsigned long long* ans) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq) return;
    const uint64_t j = tree_first(tree, P, 0, q[i] + 1);
    ans[i] = j < n ? cm[j].gidx : NONE64;
}

__global__ void __launch_bounds__(256) k_sw_fill(const unsigned long long* ans, const uint32_t* qk, uint64_t nq,
                                                 unsigned long long* F) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nq) F[qk[i]] = ans[i];
}

__global__ void __launch_bounds__(256) k_sw_fpack(const unsigned long long* F, const uint32_t* perm, uint64_t n,
                                                  unsigned long long* out) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n) out[p] = F[perm[p]];
}

// requests (ascending packet indices) per holder shard: first[r] .. first[r + 1]
__global__ void k_sw_rcount(const unsigned long long* req, uint64_t n, const unsigned long long* first, uint32_t n_ranks,
                            unsigned long long* counts) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_ranks) return;
    auto lb = [&](unsigned long long v) {
        uint64_t lo = 0, hi = n;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (req[mid] < v) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    };
    counts[r] = lb(first[r + 1]) - lb(first[r]);
}

__global__ void __launch_bounds__(256) k_sw_seed(const Batch* bs, int nb, const unsigned long long* req, uint64_t n,
                                                 int macs, Seed* out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Parsed P;
    parse_global(bs, nb, req[i], macs != 0, P);
    fluere_record r;
    fill_seed(r, P);
    Seed sd;
    for (int k = 0; k < 16; k++) { sd.src[k] = r.source[k]; sd.dst[k] = r.destination[k]; }
    sd.sp = r.src_port; sd.dp = r.dst_port;
    sd.v6 = r.src_v6; sd.prot = r.prot; sd.tos = r.tos; sd.pad = 0;
    out[i] = sd;
}

__global__ void __launch_bounds__(256) k_sw_seed_scatter(const Seed* in, const uint32_t* q, uint64_t n, Seed* out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[q[i]] = in[i];
}

static int sw_state(fluere_ctx* c) {
    if (!c->sw) {
        c->sw = new (std::nothrow) SweepState();
        if (!c->sw) return FLUERE_E_NOMEM;
        if (hipMalloc(&c->sw->misc, 4096 * 8) != hipSuccess || hipMalloc(&c->sw->err, 4) != hipSuccess)
            return FLUERE_E_NOMEM;
    }
    return FLUERE_OK;
}

extern "C" int fluere_sweep_pack(fluere_ctx* c, uint32_t n_owners, uint64_t* counts, void* d_send) {
    if (!c || !n_owners || n_owners > 4096 || !counts) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    int rc;
    if ((rc = sw_state(c))) return rc;
    SweepState* w = c->sw;
    if (!d_send || w->n_owners != n_owners || !w->hcm) {
        // (re)index: this shard's valid packets and their owners
        sweep_free(c);
        if ((rc = sw_state(c))) return rc;
        w = c->sw;
        if ((rc = upload_batches(c))) return rc;
        const uint64_t N = c->n_total;
        const uint64_t M = std::max<uint64_t>(N, 1);
        w->P = tree_leaves(M);
        if (hipMalloc(&w->hcm, M * sizeof(ExMeta)) != hipSuccess || hipMalloc(&w->hperm, M * 4) != hipSuccess ||
            hipMalloc(&w->hpr, M) != hipSuccess || hipMalloc(&w->hF, M * 8) != hipSuccess ||
            hipMalloc(&w->tree, 2 * w->P * 8) != hipSuccess || hipMalloc(&w->qk, M * 4) != hipSuccess ||
            hipMalloc(&w->k1, M * 4) != hipSuccess || hipMalloc(&w->k2, M * 4) != hipSuccess ||
            hipMalloc(&w->v1, M * 4) != hipSuccess)
            return FLUERE_E_NOMEM;
        std::vector<Batch> hb(c->batches.size());
        for (size_t i = 0; i < hb.size(); i++) hb[i] = c->batches[i].b;
        ExactJob J{c->d_batches, hb.data(), (int)hb.size(), tables_of(c), c->use_mac, 1, c->timeout_ms * 1000ull,
                   nullptr, c->d_glob, nullptr, nullptr, nullptr, nullptr};
        if ((rc = exact_collect(J, s, w->hcm, &w->hn))) return rc;
        const uint64_t n = w->hn;
        HIPCHECK(hipMemsetAsync(w->misc, 0, n_owners * 8, s));
        if (n) {
            k_sw_owner<<<grid_for(n, 256), 256, 0, s>>>(w->hcm, n, c->d_flow_key, n_owners, w->k1, w->v1);
            size_t tb = 0;
            (void)prim_sort_pairs(nullptr, tb, w->k1, w->k2, w->v1, w->hperm, (int)n, 0,
                                                     bits_for(n_owners), s);
            if ((rc = sw_tmp(w, tb))) return rc;
            HIPCHECK(prim_sort_pairs(w->tmp, tb, w->k1, w->k2, w->v1, w->hperm, (int)n, 0,
                                                        bits_for(n_owners), s));
            k_sw_kcount<<<grid_for(n_owners, 256), 256, 0, s>>>(w->k2, n, n_owners, w->misc);
            HIPCHECK(hipMemsetAsync(w->hpr, 1, n, s));  // first guess: every valid packet is processed
        }
        w->counts.assign(n_owners, 0);
        HIPCHECK(hipMemcpyAsync(w->counts.data(), w->misc, n_owners * 8, hipMemcpyDeviceToHost, s));
        HIPCHECK(hipGetLastError());
        HIPCHECK(ctx_sync(c));
        w->n_owners = n_owners;
    }
    for (uint32_t o = 0; o < n_owners; o++) counts[o] = w->counts[o];
    if (d_send && w->hn) {
        k_sw_pack<<<grid_for(w->hn, 256), 256, 0, s>>>(w->hcm, w->hperm, w->hn, c->d_sumpos, (ExMeta*)d_send);
        HIPCHECK(hipGetLastError());
        HIPCHECK(ctx_sync(c));
    }
    return FLUERE_OK;
}

extern "C" int fluere_sweep_load(fluere_ctx* c, const void* d_recv, uint32_t n_shards, const uint64_t* counts) {
    if (!c || !c->sw || !n_shards || n_shards > 4095 || !counts) return FLUERE_E_ARG;
    if (n_shards != c->merge_shards || !c->d_sd) return FLUERE_E_STATE;
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    SweepState* w = c->sw;
    std::vector<unsigned long long> seg(n_shards + 1, 0);
    for (uint32_t r = 0; r < n_shards; r++) seg[r + 1] = seg[r] + counts[r];
    const uint64_t n = seg[n_shards];
    if (n && !d_recv) return FLUERE_E_ARG;
    hipFree(w->ocm);
    w->ocm = nullptr;
    if (hipMalloc(&w->ocm, std::max<uint64_t>(n, 1) * sizeof(ExMeta)) != hipSuccess) return FLUERE_E_NOMEM;
    w->on = n;
    HIPCHECK(hipMemcpyAsync(w->misc, seg.data(), (n_shards + 1) * 8, hipMemcpyHostToDevice, s));
    HIPCHECK(hipMemsetAsync(w->err, 0, 4, s));
    if (n)
        k_sw_load<<<grid_for(n, 256), 256, 0, s>>>((const ExMeta*)d_recv, n, w->misc, n_shards, c->d_sd,
                                                   c->merge_cap, c->fmax, w->ocm, w->err);
    uint32_t err = 0;
    HIPCHECK(hipMemcpyAsync(&err, w->err, 4, hipMemcpyDeviceToHost, s));
    HIPCHECK(ctx_sync(c));
    if (err) return FLUERE_E_ARG;  // a packet of a flow the merge does not hold
    if (w->es) exact_free(w->es);
    w->es = nullptr;
    w->passes = 0;
    std::vector<Batch> hb(c->batches.size());
    for (size_t i = 0; i < hb.size(); i++) hb[i] = c->batches[i].b;
    ExactJob J{c->d_batches, hb.data(), (int)hb.size(), tables_of(c), c->use_mac, 1, c->timeout_ms * 1000ull,
               nullptr, c->d_glob, &c->d_recs, &c->d_recs_cap, &c->d_exact, &c->d_exact_bytes};
    J.ext_cm = w->ocm;
    J.ext_n = n;
    J.mail = c->h_mail;
    ExactSession* es = nullptr;
    int rc = exact_begin(J, s, &es);
    w->es = es;
    return rc;
}

extern "C" int fluere_sweep_index(fluere_ctx* c, const uint8_t* d_pr, uint64_t* max_time) {
    if (!c || !c->sw || !max_time) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    SweepState* w = c->sw;
    const uint64_t n = w->hn;
    if (d_pr && n) k_sw_feedback<<<grid_for(n, 256), 256, 0, s>>>(d_pr, w->hperm, n, w->hpr);
    int rc = tree_build(n, w->hcm, w->hpr, w->tree, w->P, s);
    if (rc) return rc;
    unsigned long long root = 0;
    HIPCHECK(hipMemcpyAsync(&root, w->tree + 1, 8, hipMemcpyDeviceToHost, s));
    HIPCHECK(ctx_sync(c));
    *max_time = n ? root : 0;  // 1 + the latest processed packet's time (0: none)
    return FLUERE_OK;
}

extern "C" int fluere_sweep_queries(fluere_ctx* c, uint32_t n_ranks, uint32_t rank, const uint64_t* max_times,
                                    uint64_t* qcounts, void* d_q) {
    if (!c || !c->sw || !n_ranks || n_ranks > 4095 || rank >= n_ranks || !max_times || !qcounts) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    SweepState* w = c->sw;
    const uint64_t n = w->hn;
    const unsigned long long T = c->timeout_ms * 1000ull;
    if (!d_q) {
        HIPCHECK(hipMemcpyAsync(w->misc, max_times, n_ranks * 8, hipMemcpyHostToDevice, s));
        HIPCHECK(hipMemsetAsync(w->misc + 2048, 0, (n_ranks + 1) * 8, s));
        std::vector<uint64_t> cnt(n_ranks + 1, 0);
        w->nq = 0;
        if (n) {
            k_sw_points<<<grid_for(n, 256), 256, 0, s>>>(w->hcm, n, w->tree, w->P, T, rank, n_ranks, w->misc, w->hF,
                                                         w->k1, w->v1);
            // queries grouped by target shard (n_ranks: none), capture order within one
            size_t tb = 0;
            (void)prim_sort_pairs(nullptr, tb, w->k1, w->k2, w->v1, w->qk, (int)n, 0,
                                                     bits_for(n_ranks), s);
            int rc = sw_tmp(w, tb);
            if (rc) return rc;
            HIPCHECK(prim_sort_pairs(w->tmp, tb, w->k1, w->k2, w->v1, w->qk, (int)n, 0,
                                                        bits_for(n_ranks), s));
            k_sw_kcount<<<grid_for(n_ranks + 1, 256), 256, 0, s>>>(w->k2, n, n_ranks + 1, w->misc + 2048);
            HIPCHECK(hipGetLastError());
            HIPCHECK(hipMemcpyAsync(cnt.data(), w->misc + 2048, (n_ranks + 1) * 8, hipMemcpyDeviceToHost, s));
            HIPCHECK(ctx_sync(c));
        }
        for (uint32_t r = 0; r < n_ranks; r++) { qcounts[r] = cnt[r]; w->nq += cnt[r]; }
        return FLUERE_OK;
    }
    for (uint32_t r = 0; r < n_ranks; r++) qcounts[r] = 0;
    uint64_t nq = w->nq;
    if (nq) k_sw_qpack<<<grid_for(nq, 256), 256, 0, s>>>(w->hcm, w->qk, nq, T, (unsigned long long*)d_q);
    HIPCHECK(hipGetLastError());
    HIPCHECK(ctx_sync(c));
    return FLUERE_OK;
}

extern "C" int fluere_sweep_answer(fluere_ctx* c, const void* d_q, uint64_t n, void* d_ans) {
    if (!c || !c->sw || (n && (!d_q || !d_ans))) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    SweepState* w = c->sw;
    if (n)
        k_sw_answer<<<grid_for(n, 256), 256, 0, s>>>((const unsigned long long*)d_q, n, w->tree, w->P, w->hcm, w->hn,
                                                     (unsigned long long*)d_ans);
    HIPCHECK(hipGetLastError());
    HIPCHECK(ctx_sync(c));
    return FLUERE_OK;
}

extern "C" int fluere_sweep_points(fluere_ctx* c, const void* d_ans, void* d_f) {
    if (!c || !c->sw || (c->sw->nq && !d_ans) || (c->sw->hn && !d_f)) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    SweepState* w = c->sw;
    if (w->nq) k_sw_fill<<<grid_for(w->nq, 256), 256, 0, s>>>((const unsigned long long*)d_ans, w->qk, w->nq, w->hF);
    if (w->hn) k_sw_fpack<<<grid_for(w->hn, 256), 256, 0, s>>>(w->hF, w->hperm, w->hn, (unsigned long long*)d_f);
    HIPCHECK(hipGetLastError());
    HIPCHECK(ctx_sync(c));
    return FLUERE_OK;
}

extern "C" int fluere_sweep_chase(fluere_ctx* c, const void* d_f, void* d_pr, int* changed) {
    if (!c || !c->sw || !c->sw->es || !changed) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    SweepState* w = c->sw;
    if (w->on && (!d_f || !d_pr)) return FLUERE_E_ARG;
    if (++w->passes > 64) return FLUERE_E_UNSUPPORTED;  // no fixed point (cannot happen: the system is causal)
    bool ch = false;
    int rc = exact_pass(w->es, (const unsigned long long*)d_f, (uint8_t*)d_pr, &ch);
    *changed = ch ? 1 : 0;
    return rc;
}

extern "C" int fluere_sweep_seed_requests(fluere_ctx* c, uint32_t n_ranks, const uint64_t* rank_first,
                                          uint64_t* counts, void* d_req) {
    if (!c || !c->sw || !c->sw->es || !n_ranks || n_ranks > 4095 || !rank_first || !counts) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    SweepState* w = c->sw;
    if (!d_req) {
        hipFree(w->req); hipFree(w->reqq);
        w->req = nullptr; w->reqq = nullptr;
        const uint64_t M = std::max<uint64_t>(w->on, 1);
        if (hipMalloc(&w->req, M * 8) != hipSuccess || hipMalloc(&w->reqq, M * 4) != hipSuccess) return FLUERE_E_NOMEM;
        int rc = exact_seed_requests(w->es, w->req, w->reqq, &w->n_inst);
        if (rc) return rc;
        HIPCHECK(hipMemcpyAsync(w->misc, rank_first, (n_ranks + 1) * 8, hipMemcpyHostToDevice, s));
        k_sw_rcount<<<grid_for(n_ranks, 256), 256, 0, s>>>(w->req, w->n_inst, w->misc, n_ranks, w->misc + 2048);
        HIPCHECK(hipGetLastError());
        std::vector<unsigned long long> cnt(n_ranks);
        HIPCHECK(hipMemcpyAsync(cnt.data(), w->misc + 2048, n_ranks * 8, hipMemcpyDeviceToHost, s));
        HIPCHECK(ctx_sync(c));
        uint64_t tot = 0;
        for (uint32_t r = 0; r < n_ranks; r++) { counts[r] = cnt[r]; tot += cnt[r]; }
        if (tot != w->n_inst) return FLUERE_E_ARG;  // a creating packet outside every shard's range
        return FLUERE_OK;
    }
    if (w->n_inst) HIPCHECK(hipMemcpyAsync(d_req, w->req, (size_t)w->n_inst * 8, hipMemcpyDeviceToDevice, s));
    HIPCHECK(ctx_sync(c));
    return FLUERE_OK;
}

extern "C" int fluere_sweep_seeds(fluere_ctx* c, const void* d_req, uint64_t n, void* d_seeds) {
    if (!c || (n && (!d_req || !d_seeds))) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    int rc;
    if ((rc = upload_batches(c))) return rc;
    if (n)
        k_sw_seed<<<grid_for(n, 256), 256, 0, s>>>(c->d_batches, (int)c->batches.size(), (const unsigned long long*)d_req,
                                                   n, c->use_mac, (Seed*)d_seeds);
    HIPCHECK(hipGetLastError());
    HIPCHECK(ctx_sync(c));
    return FLUERE_OK;
}

extern "C" int fluere_sweep_finish(fluere_ctx* c, const void* d_seeds, fluere_stats* st) {
    if (!c || !c->sw || !c->sw->es) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    SweepState* w = c->sw;
    const uint32_t ni = w->n_inst;
    if (ni && !d_seeds) return FLUERE_E_ARG;
    hipFree(w->seeds);
    w->seeds = nullptr;
    if (hipMalloc(&w->seeds, std::max<uint32_t>(ni, 1) * sizeof(Seed)) != hipSuccess) return FLUERE_E_NOMEM;
    if (ni) k_sw_seed_scatter<<<grid_for(ni, 256), 256, 0, s>>>((const Seed*)d_seeds, w->reqq, ni, w->seeds);
    // the records of this rank: only the sweep's (the merge emitted none)
    Glob g;
    HIPCHECK(hipMemcpyAsync(&g, c->d_glob, sizeof g, hipMemcpyDeviceToHost, s));
    HIPCHECK(ctx_sync(c));
    const uint64_t want = g.n_rec + ni;
    if (want > c->d_recaux_cap) {
        hipFree(c->d_recaux);
        c->d_recaux = nullptr;
        c->d_recaux_cap = 0;
        if (hipMalloc(&c->d_recaux, std::max<uint64_t>(want, 1) * 16) != hipSuccess) return FLUERE_E_NOMEM;
        c->d_recaux_cap = std::max<uint64_t>(want, 1);
    }
    if (g.n_rec) HIPCHECK(hipMemsetAsync(c->d_recaux, 0, g.n_rec * 16, s));
    int rc = exact_finish(w->es, w->seeds, c->d_recaux + 2 * g.n_rec);
    if (rc) return rc;
    HIPCHECK(hipMemcpyAsync(&g, c->d_glob, sizeof g, hipMemcpyDeviceToHost, s));
    HIPCHECK(ctx_sync(c));
    c->dev_n_rec = g.n_rec;
    c->host_recs = false;
    c->dev_ordered = false;
    c->has_aux = true;
    c->have_results = true;
    if (st) {
        fluere_stats out{};
        out.valid = g.valid;
        out.dropped_parse = g.dropped;
        out.records = g.n_rec;
        out.ended = g.n_ended;
        out.updates = g.n_updates;
        out.complex_flows = exact_result(w->es).keys;
        out.sequential_mode = 1;
        *st = out;
    }
    exact_free(w->es);
    w->es = nullptr;
    return FLUERE_OK;
}
