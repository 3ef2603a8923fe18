// exact.hip -- the exact offline state machine, in parallel (exact.h).
//
// The reference runs one loop over the packets (offline_fluereflows.rs:68-184).
// Restated per canonical key, its effect is a sequence of flow *instances*:
// the key's packets in capture order, cut into maximal runs [c, e] where
//   c = the first create-eligible packet (non-TCP, or TCP with SYN;
//       :101-113) at or after the previous instance's end,
//   e = the instance's closing packet: the first FIN/RST at or after c
//       (:152-157), or the last packet of the key at or before the sweep that
//       evicts it (:161-175), or the key's last packet (active at the end).
// Every packet of [c, e] updates the instance (flows.rs:11-42); packets between
// instances are TCP packets without SYN: skipped, no sweep.  Per key this is a
// pointer chase over instances, not packets, so an elephant flow costs one
// step; the per-instance sums / min / max are one segmented reduction over the
// packets sorted by (key, index).
//
// The sweep (Mode B, capture span >= timeout).  An expiry entry is pushed at
// every creation c with exp = t_c + timeout and never removed.  It fires at
// j = the first *processed* packet (valid, not SYN-gated) at or after c with
// t_j >= exp, where it evicts whatever flow is stored under its oriented key
// then -- the instance it created, or a later one of the same orientation (a
// stale entry).  Within one key the entries of an orientation fire in
// creation order when timestamps are non-decreasing, so the chase keeps one
// FIFO per orientation.  Records leave in the reference's order: by the
// packet that ended them, FIN/RST before the sweep, sweeps by (exp, push
// order) -- with non-decreasing timestamps the push order.
//
// Which packets are processed depends on every key's instances (a TCP packet
// without SYN of a key with no flow is skipped and sweeps nothing), and the
// instances depend on the sweeps: the chase is iterated from "every valid
// packet is processed" until the processed set is stable.  The system is
// causal in packet order, so a stable assignment is the sequential one.
// Captures whose timestamps go backwards (or with no fixed point within the
// pass limit) return EXACT_FALLBACK to the caller's sequential kernel.
#include "exact.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <vector>

namespace fl {
namespace {

constexpr uint64_t M40 = (1ull << 40) - 1;
constexpr uint32_t NOPOS = 0xFFFFFFFFu;
constexpr int MAX_PASSES = 32;
enum : uint8_t { K_FIN = 0, K_SWEEP = 1, K_ACTIVE = 2, K_LEAD = 3 };
// shard mode: role of a run in the flow's annex
enum : uint8_t { R_RECORD = 0, R_HEAD = 1, R_TAIL = 2, R_HEAD_TAIL = 3, R_LEAD = 4 };

// One replayed packet (32 bytes).
struct ExMeta {
    uint64_t t, gidx;
    uint32_t d, pkt, doct;
    uint8_t dir, tflags, ttl, bits;  // bits: 1 create-eligible, 2 FIN or RST
};
static_assert(sizeof(ExMeta) == 32, "ExMeta layout");

// Per-instance aggregate of update_flow's order-free fields.
struct Agg {
    uint32_t pk[2];
    unsigned long long by[2];
    uint32_t mnp, mxp, mnt, mxt;
    uint32_t fl[8];
    unsigned long long lastg, lastt;  // the last packet (largest index) and its time
};
struct AggOp {
    __host__ __device__ Agg operator()(const Agg& a, const Agg& b) const {
        Agg r;
        r.pk[0] = a.pk[0] + b.pk[0];
        r.pk[1] = a.pk[1] + b.pk[1];
        r.by[0] = a.by[0] + b.by[0];
        r.by[1] = a.by[1] + b.by[1];
        r.mnp = a.mnp < b.mnp ? a.mnp : b.mnp;
        r.mxp = a.mxp > b.mxp ? a.mxp : b.mxp;
        r.mnt = a.mnt < b.mnt ? a.mnt : b.mnt;
        r.mxt = a.mxt > b.mxt ? a.mxt : b.mxt;
        for (int q = 0; q < 8; q++) r.fl[q] = a.fl[q] + b.fl[q];
        const bool bl = b.lastg > a.lastg;
        r.lastg = bl ? b.lastg : a.lastg;
        r.lastt = bl ? b.lastt : a.lastt;
        return r;
    }
};
struct ToAgg {
    const ExMeta* sm;
    __host__ __device__ Agg operator()(uint32_t p) const {
        const ExMeta m = sm[p];
        Agg a;
        a.pk[0] = m.dir ? 0 : 1;
        a.pk[1] = m.dir ? 1 : 0;
        a.by[0] = m.dir ? 0 : m.doct;
        a.by[1] = m.dir ? m.doct : 0;
        a.mnp = a.mxp = m.pkt;
        a.mnt = a.mxt = m.ttl;
        for (int q = 0; q < 8; q++) a.fl[q] = (m.tflags >> q) & 1;
        a.lastg = m.gidx;
        a.lastt = m.t;
        return a;
    }
};

// ---- 1. per-packet metadata of the packets to replay (one parse pass) -----
__global__ void __launch_bounds__(256) k_ex_meta(Batch B, TableSet T, int macs, int all, const uint8_t* cplx,
                                                 ExMeta* meta, uint32_t* flag, uint64_t off) {
    const uint64_t li = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (li >= B.n) return;
    Parsed P;
    parse_record(B, li, macs != 0, 0, P);
    uint32_t take = 0;
    ExMeta m;
    memset(&m, 0, sizeof m);
    if (P.cls == 0) {
        uint8_t dir;
        const uint32_t d = flow_of(T, P, macs != 0, false, dir, nullptr, nullptr);
        if (d != FAIL && d < T.fmax && (all || cplx[d])) {
            take = 1;
            m.t = P.t;
            m.gidx = B.first + li;
            m.d = d;
            m.pkt = P.pi.rpkt;
            m.doct = P.pi.doctets;
            m.dir = dir;
            m.tflags = P.pi.tflags;
            m.ttl = P.pi.rttl;
            m.bits = ((P.pi.rprot != 6 || (P.pi.tflags & 2)) ? 1 : 0) | ((P.pi.tflags & 5) ? 2 : 0);
        }
    }
    flag[off + li] = take;
    meta[off + li] = m;
}

// compaction in capture order: cm[k] = the k-th replayed packet; sort keys (key, index)
__global__ void __launch_bounds__(256) k_ex_compact(const ExMeta* meta, const uint32_t* flag, const uint32_t* pos,
                                                    uint64_t n, ExMeta* cm, unsigned long long* key, uint32_t* val) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !flag[i]) return;
    const uint32_t k = pos[i];
    const ExMeta m = meta[i];
    cm[k] = m;
    key[k] = ((unsigned long long)m.d << 40) | (m.gidx & M40);
    val[k] = k;
}

// ---- 2. sorted view, key heads, next-eligible / next-FIN inputs -------------
__global__ void __launch_bounds__(256) k_ex_gather(uint64_t n, const unsigned long long* skey, const uint32_t* sval,
                                                   const ExMeta* cm, ExMeta* sm, uint32_t* hf,
                                                   unsigned long long* re, unsigned long long* rf) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const ExMeta m = cm[sval[p]];
    sm[p] = m;
    const unsigned long long d = skey[p] >> 40;
    hf[p] = (p == 0 || (skey[p - 1] >> 40) != d) ? 1u : 0u;
    // reversed, so an inclusive min-scan gives the first eligible / FIN-RST
    // position at or after p within the key (low 40 bits M40: none)
    re[n - 1 - p] = (d << 40) | ((m.bits & 1) ? p : M40);
    rf[n - 1 - p] = (d << 40) | ((m.bits & 2) ? p : M40);
}

__global__ void __launch_bounds__(256) k_ex_heads(uint64_t n, const uint32_t* hf, const uint32_t* hpos, uint32_t* heads) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n && hf[p]) heads[hpos[p]] = (uint32_t)p;
}

// ---- 3. Mode B: timestamps non-decreasing over the valid packets? ---------
__global__ void __launch_bounds__(256) k_ex_mono(uint64_t n, const ExMeta* cm, uint32_t* bad) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k > 0 && k < n && cm[k].t < cm[k - 1].t) atomicOr(bad, 1u);
}

// reversed "k if processed" for the next-processed min-scan
__global__ void __launch_bounds__(256) k_ex_proc_in(uint64_t n, const uint8_t* pr, unsigned long long* npr) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) npr[n - 1 - k] = pr[k] ? k : M40;
}

// ---- 4. the chase: one thread per key ----------------------------------------
struct ChaseArgs {
    uint64_t n;
    uint32_t n_keys;
    const uint32_t* heads;
    const ExMeta* sm;   // sorted by (key, index)
    const uint32_t* sval;  // sorted position -> capture-order index k (Mode B: into cm)
    const unsigned long long* ne_rev;  // scans (reversed)
    const unsigned long long* nf_rev;
    int mode_b;
    uint64_t timeout_us;
    const ExMeta* cm;   // capture order (Mode B sweep points)
    const unsigned long long* np_rev;  // next processed (reversed min-scan)
    // out, indexed by the instance's first position
    uint32_t* sflag;
    uint32_t* iend;
    uint8_t* ikind;
    unsigned long long* ij;   // FIN: its index; sweep: the sweeping packet's index
    unsigned long long* iie;  // sweep: the index of the creation that pushed the firing entry
    unsigned long long* ej;   // Mode B: sweep point of the entry pushed at this creation
    uint32_t* link;           // Mode B: next pending entry of the same orientation
    // shard mode
    int shard_mode;
    uint8_t* irole;
    uint32_t* ikey;           // key ordinal of the run (annex index)
    fluere_flow_annex* annex;
    uint32_t* annex_of;
    const uint8_t* flow_key;  // TableSet::flow_key (56-byte canonical keys by dense id)
};

// first processed packet (capture-order index) k >= i_k with t_k >= exp -> its packet index
__device__ __forceinline__ unsigned long long sweep_point(const ChaseArgs& a, uint32_t k0, unsigned long long exp) {
    // lower_bound over the non-decreasing times of the valid packets
    uint64_t lo = 0, hi = a.n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (a.cm[mid].t < exp) lo = mid + 1;
        else hi = mid;
    }
    const uint64_t k = max((uint64_t)k0, lo);
    if (k >= a.n) return NONE64;
    const unsigned long long kp = a.np_rev[a.n - 1 - k];
    return kp == M40 ? NONE64 : a.cm[kp].gidx;
}

__global__ void __launch_bounds__(64) k_ex_chase(ChaseArgs a) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= a.n_keys) return;
    const uint32_t p0 = a.heads[q];
    const uint32_t pend = q + 1 < a.n_keys ? a.heads[q + 1] : (uint32_t)a.n;
    uint32_t qh[2] = {NOPOS, NOPOS}, qt[2] = {NOPOS, NOPOS};  // pending entries per orientation (FIFO)
    auto drop_upto = [&](unsigned long long lim, bool inclusive) {
        for (int x = 0; x < 2; x++) {
            while (qh[x] != NOPOS && (inclusive ? a.ej[qh[x]] <= lim : a.ej[qh[x]] < lim)) qh[x] = a.link[qh[x]];
            if (qh[x] == NOPOS) qt[x] = NOPOS;
        }
    };
    uint32_t pos = p0;
    // shard mode: from "no flow", the lead piece [p0, min(e0, f0 + 1)) and the
    // roles of the instances (the first one, if created at or before f0, is
    // the head; the one still open at the end, after f0, the tail)
    const unsigned long long f0 = a.nf_rev[a.n - 1 - p0] & M40;
    int n_inst = 0;
    if (a.shard_mode) {
        const unsigned long long e0 = a.ne_rev[a.n - 1 - p0] & M40;
        const uint32_t lead_end = (uint32_t)min(e0 == M40 ? (unsigned long long)pend : e0,
                                                f0 == M40 ? (unsigned long long)pend : f0 + 1);  // exclusive
        const uint32_t d = a.sm[p0].d;
        fluere_flow_annex& ax = a.annex[q];
        const uint32_t* kw = reinterpret_cast<const uint32_t*>(a.flow_key + (size_t)d * 56);
        for (int k = 0; k < 14; k++) ax.key[k] = kw[k];
        ax.flags = (f0 != M40 ? 1u : 0u) | (lead_end > p0 ? 2u : 0u);
        ax.mid_last = 0;
        ax.f0 = f0 != M40 ? a.sm[f0].gidx : NONE64;
        a.annex_of[d] = q;
        if (lead_end > p0) {
            a.sflag[p0] = 1;
            a.iend[p0] = lead_end - 1;
            a.ikind[p0] = K_LEAD;
            a.irole[p0] = R_LEAD;
            a.ikey[p0] = q;
        }
    }
    while (pos < pend) {
        const unsigned long long ce = a.ne_rev[a.n - 1 - pos] & M40;
        if (ce == M40) break;
        const uint32_t c = (uint32_t)ce;
        const ExMeta mc = a.sm[c];
        const uint32_t o = mc.dir;
        unsigned long long jf = NONE64;
        uint32_t front = NOPOS;
        if (a.mode_b) {
            drop_upto(mc.gidx, false);  // entries that fired while the key had no flow
            const unsigned long long exp =
                mc.t + a.timeout_us < mc.t ? NONE64 : mc.t + a.timeout_us;  // (saturating)
            a.ej[c] = sweep_point(a, a.sval[c], exp);
            a.link[c] = NOPOS;
            if (qh[o] == NOPOS) qh[o] = qt[o] = c;
            else { a.link[qt[o]] = c; qt[o] = c; }
            front = qh[o];
            jf = a.ej[front];
        }
        const unsigned long long fe = a.nf_rev[a.n - 1 - c] & M40;
        uint32_t end;
        uint8_t kind;
        unsigned long long cj = NONE64, cie = 0;
        if (fe != M40 && (jf == NONE64 || a.sm[fe].gidx <= jf)) {  // FIN/RST first (the sweep runs after it)
            end = (uint32_t)fe;
            kind = K_FIN;
            cj = a.sm[fe].gidx;
        } else if (jf != NONE64) {  // swept: the key's last packet at or before the sweeping packet
            uint32_t lo = c, hi = pend - 1;
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1) >> 1;
                if (a.sm[mid].gidx <= jf) lo = mid;
                else hi = mid - 1;
            }
            end = lo;
            kind = K_SWEEP;
            cj = jf;
            cie = a.sm[front].gidx;
        } else {
            end = pend - 1;
            kind = K_ACTIVE;
        }
        a.sflag[c] = 1;
        a.iend[c] = end;
        a.ikind[c] = kind;
        a.ij[c] = cj;
        a.iie[c] = cie;
        if (a.shard_mode) {
            const bool head = n_inst == 0 && (f0 == M40 || c <= f0);
            const bool tail = kind == K_ACTIVE;
            a.irole[c] = head ? (tail ? R_HEAD_TAIL : R_HEAD) : (tail ? R_TAIL : R_RECORD);
            a.ikey[c] = q;
            a.annex[q].flags |= (head ? 4u : 0u) | (tail && !head ? 8u : 0u);
        }
        n_inst++;
        if (a.mode_b && kind != K_ACTIVE) drop_upto(cj, true);
        pos = end + 1;
    }
}

// ---- 5. members, processed set, reduction keys ------------------------------
__global__ void __launch_bounds__(256) k_ex_starts(uint64_t n, const uint32_t* sflag, const uint32_t* incl, uint32_t* ist) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n && sflag[p]) ist[incl[p] - 1] = (uint32_t)p;
}

// rk[p] = instance of p (member), or a key no member has; Mode B: the
// processed flag of each replayed packet (members are processed)
__global__ void __launch_bounds__(256) k_ex_members(uint64_t n, const uint32_t* incl, const uint32_t* ist,
                                                    const uint32_t* iend, uint32_t* rk, const uint32_t* sval,
                                                    uint8_t* pr, uint32_t* changed) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint32_t q1 = incl[p];  // instances starting at or before p
    const bool member = q1 > 0 && p <= iend[ist[q1 - 1]];
    rk[p] = member ? q1 - 1 : (0x80000000u | q1);
    if (pr) {
        const uint8_t v = member ? 1 : 0;
        const uint32_t k = sval[p];
        if (pr[k] != v) {
            pr[k] = v;
            atomicOr(changed, 1u);
        }
    }
}

// ---- 6. records ----------------------------------------------------------------
struct RecArgs {
    const Batch* bs;
    int nb;
    int macs, mode_b;
    const uint32_t* ukeys;
    const Agg* aggs;
    const uint32_t* nruns;
    const uint32_t* ist;
    const ExMeta* sm;
    const uint32_t* iend;
    const uint8_t* ikind;
    const unsigned long long* ij;
    const unsigned long long* iie;
    Glob* g;
    fluere_record* out;      // Mode A: the run's records (appended)
    uint64_t out_cap;
    fluere_record* tmp;      // Mode B: by instance, ordered afterwards
    unsigned long long* hi;  // Mode B order: (sweeping / closing index, phase)
    unsigned long long* lo;  //               (the firing entry's creation index)
    uint32_t* idx;
    int shard_mode;
    const uint8_t* irole;
    const uint32_t* ikey;
    fluere_flow_annex* annex;
};

__device__ __forceinline__ void piece_of(const Agg& g, fluere_flow_piece& pc) {
    pc.pkts[0] = g.pk[0]; pc.pkts[1] = g.pk[1];
    pc.bytes[0] = g.by[0]; pc.bytes[1] = g.by[1];
    pc.min_pkt = g.mnp; pc.max_pkt = g.mxp; pc.min_ttl = g.mnt; pc.max_ttl = g.mxt;
    for (int k = 0; k < 8; k++) pc.flag_cnt[k] = g.fl[k];
    pc.last = g.lastg;
    pc.last_time = g.lastt;
}

__global__ void __launch_bounds__(EMIT_BLOCK) k_ex_records(RecArgs a) {
    __shared__ EmitLds S;
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t nr = *a.nruns;
    const bool lane_live = r < nr && !(a.ukeys[r] & 0x80000000u);
    fluere_record rec;
    memset(&rec, 0, sizeof rec);
    uint32_t q = 0;
    uint8_t kind = K_ACTIVE;
    unsigned long long cj = NONE64, cie = 0;
    if (lane_live && a.shard_mode && a.irole[a.ist[a.ukeys[r]]] != R_RECORD) {
        // a piece of the flow's annex (lead / head / tail), not a record
        const uint32_t c = a.ist[a.ukeys[r]];
        const ExMeta mc = a.sm[c];
        const uint8_t role = a.irole[c];
        fluere_flow_annex& ax = a.annex[a.ikey[c]];
        fluere_flow_piece pc;
        memset(&pc, 0, sizeof pc);
        piece_of(a.aggs[r], pc);
        pc.first = mc.gidx;
        pc.first_time = mc.t;
        if (role != R_LEAD) {
            Parsed P;
            parse_global(a.bs, a.nb, mc.gidx, a.macs != 0, P);
            fluere_record sd;
            fill_seed(sd, P);
            for (int k = 0; k < 16; k++) { pc.src[k] = sd.source[k]; pc.dst[k] = sd.destination[k]; }
            pc.v6 = sd.src_v6; pc.prot = sd.prot; pc.tos = sd.tos; pc.dir = mc.dir;
            pc.src_port = sd.src_port; pc.dst_port = sd.dst_port;
        }
        if (role == R_LEAD) ax.lead = pc;
        if (role == R_HEAD || role == R_HEAD_TAIL) ax.head = pc;
        if (role == R_TAIL) ax.tail = pc;
    }
    const bool rec_live = lane_live && !(a.shard_mode && a.irole[a.ist[a.ukeys[r]]] != R_RECORD);
    if (rec_live && a.shard_mode)  // the flow's last processed packet among its in-shard records (live mode)
        atomicMax(reinterpret_cast<unsigned long long*>(&a.annex[a.ikey[a.ist[a.ukeys[r]]]].mid_last),
                  (unsigned long long)a.aggs[r].lastg + 1);
    if (rec_live) {
        q = a.ukeys[r];
        const uint32_t c = a.ist[q];
        const ExMeta mc = a.sm[c];
        Parsed P;
        parse_global(a.bs, a.nb, mc.gidx, a.macs != 0, P);
        fill_seed(rec, P);
        const Agg g = a.aggs[r];
        const uint32_t o = mc.dir;  // orientation of the creating packet
        rec.d_pkts = g.pk[0] + g.pk[1];
        rec.d_octets = g.by[0] + g.by[1];
        rec.out_pkts = g.pk[o];
        rec.in_pkts = g.pk[1 - o];
        rec.out_bytes = g.by[o];
        rec.in_bytes = g.by[1 - o];
        rec.min_pkt = g.mnp;
        rec.max_pkt = g.mxp;
        rec.min_ttl = (uint8_t)g.mnt;
        rec.max_ttl = (uint8_t)g.mxt;
        for (int k = 0; k < 8; k++) rec.cnt[k] = g.fl[k];
        rec.cnt[8] = 0;
        rec.last = g.lastt;
        kind = a.ikind[c];
        cj = a.ij[c];
        cie = a.iie[c];
        rec.order_key = kind == K_ACTIVE ? NONE64 : cj;
    }
    if (!a.mode_b) {  // (uniform: every thread of the block emits)
        emit_record_block(S, a.g, a.out, a.out_cap, rec, rec_live);
        return;
    }
    if (rec_live) {
        a.tmp[q] = rec;
        a.hi[q] = kind == K_ACTIVE ? NONE64 : (cj << 1) | (kind == K_SWEEP ? 1ull : 0ull);
        a.lo[q] = kind == K_SWEEP ? cie : 0ull;
        a.idx[q] = q;
    }
}

// Mode B: records in the reference's emission order; order_key = rank
__global__ void __launch_bounds__(EMIT_BLOCK) k_ex_emit_sorted(uint32_t n_inst, const uint32_t* perm, const fluere_record* tmp,
                                                               Glob* g, fluere_record* out, uint64_t cap) {
    __shared__ EmitLds S;
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    fluere_record rec;
    const bool live = r < n_inst;
    if (live) {
        rec = tmp[perm[r]];
        if (rec.order_key != NONE64) rec.order_key = r;
    } else {
        memset(&rec, 0, sizeof rec);
    }
    emit_record_block(S, g, out, cap, rec, live);
}

__global__ void __launch_bounds__(256) k_ex_gather_u64(uint32_t m, const uint32_t* id, const unsigned long long* h,
                                                       unsigned long long* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) out[i] = h[id[i]];
}

unsigned gridn(uint64_t n, unsigned b) { return (unsigned)std::max<uint64_t>(1, (n + b - 1) / b); }

// bump allocator over the scratch arena (256-byte aligned pieces)
struct Arena {
    char* base = nullptr;
    size_t off = 0, cap = 0;
    template <class T>
    T* take(size_t count) {
        off = (off + 255) & ~(size_t)255;
        T* p = reinterpret_cast<T*>(base + off);
        off += std::max<size_t>(count, 1) * sizeof(T);
        return p;
    }
};

}  // namespace

int exact_run(const ExactJob& J, hipStream_t s, ExactResult* res) {
    ExactResult R{};
    uint64_t N = 0;
    for (int b = 0; b < J.nb; b++) N += J.h_batches[b].n;
    if (!N) {
        if (res) *res = R;
        return FLUERE_OK;
    }
    // ---- arena sizing: phase 1 (all packets) + phase 2 (replayed packets, at most N)
    auto bytes_for = [&](uint64_t n_all, uint64_t n, size_t tmp) {
        size_t b = 0;
        auto add = [&](size_t x) { b += ((x + 255) & ~(size_t)255) + 256; };
        add(n_all * sizeof(ExMeta)); add(n_all * 4); add(n_all * 4);  // meta, flag, pos
        add(n * sizeof(ExMeta)); add(n * 8); add(n * 4);              // cm, key, val
        add(n * 8); add(n * 4); add(n * sizeof(ExMeta));              // skey, sval, sm
        add(n * 4); add(n * 4); add(n * 4);                           // hf, hpos, heads
        add(n * 8); add(n * 8); add(n * 8); add(n * 8);               // re, rf, ne_rev, nf_rev
        add(n); add(n * 8); add(n * 8); add(n * 8); add(n * 4);       // pr, npr, np_rev, ej, link
        add(n * 4); add(n * 4); add(n); add(n * 8); add(n * 8);       // sflag, iend, ikind, ij, iie
        add(n * 4); add(n * 4); add(n * 4); add(n * 4);               // incl, ist, rk, ukeys
        add(n * sizeof(Agg)); add(16);                                // aggs, nruns/counters
        add(n * sizeof(fluere_record)); add(n * 8); add(n * 8);       // tmp, hi, lo
        add(n * 4); add(n * 4); add(n * 8); add(n * 4);               // idx, idx2, hi2, perm
        add(n); add(n * 4);                                           // irole, ikey
        add(tmp);
        return b;
    };
    // hipcub temp storage: the largest of the primitives at size N
    size_t tmp = 0, t = 0;
    {
        const int n = (int)N;
        (void)hipcub::DeviceScan::ExclusiveSum(nullptr, t, (uint32_t*)nullptr, (uint32_t*)nullptr, n, s); tmp = std::max(tmp, t);
        (void)hipcub::DeviceScan::InclusiveSum(nullptr, t, (uint32_t*)nullptr, (uint32_t*)nullptr, n, s); tmp = std::max(tmp, t);
        (void)hipcub::DeviceRadixSort::SortPairs(nullptr, t, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                           (uint32_t*)nullptr, (uint32_t*)nullptr, n, 0, 64, s);
        tmp = std::max(tmp, t);
        (void)hipcub::DeviceScan::InclusiveScan(nullptr, t, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                          hipcub::Min(), n, s);
        tmp = std::max(tmp, t);
        hipcub::CountingInputIterator<uint32_t> cnt(0);
        hipcub::TransformInputIterator<Agg, ToAgg, hipcub::CountingInputIterator<uint32_t>> vit(cnt, ToAgg{nullptr});
        (void)hipcub::DeviceReduce::ReduceByKey(nullptr, t, (uint32_t*)nullptr, (uint32_t*)nullptr, vit, (Agg*)nullptr,
                                          (uint32_t*)nullptr, AggOp(), n, s);
        tmp = std::max(tmp, t);
    }
    const size_t need = bytes_for(N, N, tmp);
    if (need > *J.scratch_bytes) {
        hipFree(*J.scratch);
        *J.scratch = nullptr;
        *J.scratch_bytes = 0;
        if (hipMalloc(J.scratch, need) != hipSuccess) return FLUERE_E_NOMEM;
        *J.scratch_bytes = need;
    }
    Arena A;
    A.base = (char*)*J.scratch;
    A.cap = need;
    ExMeta* meta = A.take<ExMeta>(N);
    uint32_t* flag = A.take<uint32_t>(N);
    uint32_t* pos = A.take<uint32_t>(N);
    // ---- 1. metadata of every packet to replay, compacted in capture order
    uint64_t off = 0;
    for (int b = 0; b < J.nb; b++) {
        const Batch& B = J.h_batches[b];
        if (!B.n) continue;
        k_ex_meta<<<gridn(B.n, 256), 256, 0, s>>>(B, J.T, J.macs, J.mode_b, J.complex, meta, flag, off);
        off += B.n;
    }
    void* tp = nullptr;
    size_t tb = tmp;
    ExMeta* cm = A.take<ExMeta>(N);
    unsigned long long* key = A.take<unsigned long long>(N);
    uint32_t* val = A.take<uint32_t>(N);
    unsigned long long* skey = A.take<unsigned long long>(N);
    uint32_t* sval = A.take<uint32_t>(N);
    ExMeta* sm = A.take<ExMeta>(N);
    uint32_t* hf = A.take<uint32_t>(N);
    uint32_t* hpos = A.take<uint32_t>(N);
    uint32_t* heads = A.take<uint32_t>(N);
    unsigned long long* re = A.take<unsigned long long>(N);
    unsigned long long* rf = A.take<unsigned long long>(N);
    unsigned long long* ne_rev = A.take<unsigned long long>(N);
    unsigned long long* nf_rev = A.take<unsigned long long>(N);
    uint8_t* pr = A.take<uint8_t>(N);
    unsigned long long* npr = A.take<unsigned long long>(N);
    unsigned long long* np_rev = A.take<unsigned long long>(N);
    unsigned long long* ej = A.take<unsigned long long>(N);
    uint32_t* link = A.take<uint32_t>(N);
    uint32_t* sflag = A.take<uint32_t>(N);
    uint32_t* iend = A.take<uint32_t>(N);
    uint8_t* ikind = A.take<uint8_t>(N);
    unsigned long long* ij = A.take<unsigned long long>(N);
    unsigned long long* iie = A.take<unsigned long long>(N);
    uint32_t* incl = A.take<uint32_t>(N);
    uint32_t* ist = A.take<uint32_t>(N);
    uint32_t* rk = A.take<uint32_t>(N);
    uint32_t* ukeys = A.take<uint32_t>(N);
    Agg* aggs = A.take<Agg>(N);
    uint32_t* ctr = A.take<uint32_t>(4);  // [0] nruns, [1] non-monotonic, [2] changed
    fluere_record* tmpr = A.take<fluere_record>(N);
    unsigned long long* hi = A.take<unsigned long long>(N);
    unsigned long long* lo = A.take<unsigned long long>(N);
    uint32_t* idx = A.take<uint32_t>(N);
    uint32_t* idx2 = A.take<uint32_t>(N);
    unsigned long long* hi2 = A.take<unsigned long long>(N);
    uint32_t* perm = A.take<uint32_t>(N);
    uint8_t* irole = A.take<uint8_t>(N);
    uint32_t* ikey = A.take<uint32_t>(N);
    tp = A.take<char>(tmp);
    const int iN = (int)N;
    HIPCHECK(hipcub::DeviceScan::ExclusiveSum(tp, tb, flag, pos, iN, s));
    uint32_t last[2] = {0, 0};
    HIPCHECK(hipMemcpyAsync(&last[0], pos + N - 1, 4, hipMemcpyDeviceToHost, s));
    HIPCHECK(hipMemcpyAsync(&last[1], flag + N - 1, 4, hipMemcpyDeviceToHost, s));
    HIPCHECK(hipStreamSynchronize(s));
    const uint64_t n = (uint64_t)last[0] + last[1];
    R.replayed = n;
    if (!n) {
        if (res) *res = R;
        return FLUERE_OK;
    }
    const int in = (int)n;
    k_ex_compact<<<gridn(N, 256), 256, 0, s>>>(meta, flag, pos, N, cm, key, val);
    // ---- 2. sort by (key, index); key heads; next eligible / FIN-RST
    int end_bit = 40;
    while (end_bit < 64 && (1ull << (end_bit - 40)) <= J.T.fmax) end_bit++;
    tb = tmp;
    HIPCHECK(hipcub::DeviceRadixSort::SortPairs(tp, tb, key, skey, val, sval, in, 0, end_bit, s));
    k_ex_gather<<<gridn(n, 256), 256, 0, s>>>(n, skey, sval, cm, sm, hf, re, rf);
    tb = tmp;
    HIPCHECK(hipcub::DeviceScan::InclusiveScan(tp, tb, re, ne_rev, hipcub::Min(), in, s));
    tb = tmp;
    HIPCHECK(hipcub::DeviceScan::InclusiveScan(tp, tb, rf, nf_rev, hipcub::Min(), in, s));
    tb = tmp;
    HIPCHECK(hipcub::DeviceScan::ExclusiveSum(tp, tb, hf, hpos, in, s));
    k_ex_heads<<<gridn(n, 256), 256, 0, s>>>(n, hf, hpos, heads);
    HIPCHECK(hipMemcpyAsync(&last[0], hpos + n - 1, 4, hipMemcpyDeviceToHost, s));
    HIPCHECK(hipMemcpyAsync(&last[1], hf + n - 1, 4, hipMemcpyDeviceToHost, s));
    HIPCHECK(hipMemsetAsync(ctr, 0, 16, s));
    if (J.mode_b) {
        k_ex_mono<<<gridn(n, 256), 256, 0, s>>>(n, cm, ctr + 1);
        HIPCHECK(hipMemsetAsync(pr, 1, n, s));  // first guess: every valid packet is processed
    }
    uint32_t mono_bad = 0;
    HIPCHECK(hipMemcpyAsync(&mono_bad, ctr + 1, 4, hipMemcpyDeviceToHost, s));
    HIPCHECK(hipStreamSynchronize(s));
    const uint32_t n_keys = last[0] + last[1];
    R.keys = n_keys;
    if (J.mode_b && mono_bad) return EXACT_FALLBACK;
    fluere_flow_annex* annex = nullptr;
    if (J.shard_mode) {
        if (n_keys > *J.annex_cap) {
            hipFree(*J.annex);
            *J.annex = nullptr;
            *J.annex_cap = 0;
            if (hipMalloc(J.annex, (size_t)n_keys * sizeof(fluere_flow_annex)) != hipSuccess) return FLUERE_E_NOMEM;
            *J.annex_cap = n_keys;
        }
        annex = *J.annex;
        R.annexes = n_keys;
    }
    ChaseArgs ca{n, n_keys, heads, sm, sval, ne_rev, nf_rev, J.mode_b, J.timeout_us, cm, np_rev,
                 sflag, iend, ikind, ij, iie, ej, link,
                 J.shard_mode, irole, ikey, annex, J.annex_of, J.T.flow_key};
    // ---- 3..5. chase (Mode B: until the processed set is stable)
    for (int pass = 0;; pass++) {
        if (pass == MAX_PASSES) return EXACT_FALLBACK;
        R.iterations = pass + 1;
        if (J.mode_b) {
            k_ex_proc_in<<<gridn(n, 256), 256, 0, s>>>(n, pr, npr);
            tb = tmp;
            HIPCHECK(hipcub::DeviceScan::InclusiveScan(tp, tb, npr, np_rev, hipcub::Min(), in, s));
        }
        HIPCHECK(hipMemsetAsync(sflag, 0, n * 4, s));
        k_ex_chase<<<gridn(n_keys, 64), 64, 0, s>>>(ca);
        tb = tmp;
        HIPCHECK(hipcub::DeviceScan::InclusiveSum(tp, tb, sflag, incl, in, s));
        k_ex_starts<<<gridn(n, 256), 256, 0, s>>>(n, sflag, incl, ist);
        HIPCHECK(hipMemsetAsync(ctr + 2, 0, 4, s));
        k_ex_members<<<gridn(n, 256), 256, 0, s>>>(n, incl, ist, iend, rk, sval, J.mode_b ? pr : nullptr, ctr + 2);
        HIPCHECK(hipGetLastError());
        if (!J.mode_b) break;
        uint32_t changed = 0;
        HIPCHECK(hipMemcpyAsync(&changed, ctr + 2, 4, hipMemcpyDeviceToHost, s));
        HIPCHECK(hipStreamSynchronize(s));
        if (!changed) break;
    }
    uint32_t n_inst = 0;
    HIPCHECK(hipMemcpyAsync(&n_inst, incl + n - 1, 4, hipMemcpyDeviceToHost, s));
    // ---- 6. per-instance aggregates (segmented over the sorted packets)
    hipcub::CountingInputIterator<uint32_t> cnt(0);
    hipcub::TransformInputIterator<Agg, ToAgg, hipcub::CountingInputIterator<uint32_t>> vit(cnt, ToAgg{sm});
    tb = tmp;
    HIPCHECK(hipcub::DeviceReduce::ReduceByKey(tp, tb, rk, ukeys, vit, aggs, ctr, AggOp(), in, s));
    HIPCHECK(hipStreamSynchronize(s));
    R.instances = n_inst;
    // ---- 7. records
    Glob gh;
    HIPCHECK(hipMemcpyAsync(&gh, J.g, sizeof gh, hipMemcpyDeviceToHost, s));
    HIPCHECK(hipStreamSynchronize(s));
    const uint64_t want = gh.n_rec + n_inst;
    if (want > *J.d_recs_cap) {  // grow, keeping the records already there
        fluere_record* nr = nullptr;
        if (hipMalloc(&nr, want * sizeof(fluere_record)) != hipSuccess) return FLUERE_E_NOMEM;
        if (gh.n_rec)
            HIPCHECK(hipMemcpyAsync(nr, *J.d_recs, gh.n_rec * sizeof(fluere_record), hipMemcpyDeviceToDevice, s));
        HIPCHECK(hipStreamSynchronize(s));
        hipFree(*J.d_recs);
        *J.d_recs = nr;
        *J.d_recs_cap = want;
    }
    RecArgs ra{J.d_batches, J.nb, J.macs, J.mode_b, ukeys, aggs, ctr, ist, sm, iend, ikind, ij, iie, J.g,
               *J.d_recs, *J.d_recs_cap, tmpr, hi, lo, idx, J.shard_mode, irole, ikey, annex};
    // runs <= n (every run holds a packet)
    k_ex_records<<<gridn(n, 256), 256, 0, s>>>(ra);
    if (J.mode_b && n_inst) {
        // order by (closing / sweeping index, phase), then the firing entry's creation
        const int ni = (int)n_inst;
        tb = tmp;
        HIPCHECK(hipcub::DeviceRadixSort::SortPairs(tp, tb, lo, hi2 /* lo sorted (unused) */, idx, idx2, ni, 0, 64, s));
        // hi in lo-sorted order
        k_ex_gather_u64<<<gridn(n_inst, 256), 256, 0, s>>>(n_inst, idx2, hi, lo);
        tb = tmp;
        HIPCHECK(hipcub::DeviceRadixSort::SortPairs(tp, tb, lo, hi2, idx2, perm, ni, 0, 64, s));
        k_ex_emit_sorted<<<gridn(n_inst, 256), 256, 0, s>>>(n_inst, perm, tmpr, J.g, *J.d_recs, *J.d_recs_cap);
    }
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(s));
    if (res) *res = R;
    return FLUERE_OK;
}

}  // namespace fl
