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
// stale entry).  The BTreeMap pops entries by (exp, push order) (:161-175),
// so per key and orientation the chase keeps its pending entries in a list
// sorted by (sweep point, exp, creation): an instance ends at the head's
// sweep point (or its FIN/RST first).  With non-decreasing timestamps every
// insert lands at the tail (the list is a FIFO); when timestamps go backwards
// the sweep point is found in a max segment tree over the processed packets'
// times (first processed packet at or after c with t >= exp), not by a binary
// search over the times.  Records leave in the reference's order: by the
// packet that ended them, FIN/RST before the sweep, sweeps by (exp, push order).
//
// Which packets are processed depends on every key's instances (a TCP packet
// without SYN of a key with no flow is skipped and sweeps nothing), and the
// instances depend on the sweeps: the chase is iterated from "every valid
// packet is processed" until the processed set is stable.  The system is
// causal in packet order, so a stable assignment is the sequential one.
// Without a fixed point within the pass limit the run returns EXACT_FALLBACK
// to the caller's sequential kernel.
//
// Sharded (multi-GPU) Mode B: the owner of a key holds all of its packets'
// metadata (shipped by the shards) and runs this same chase; the sweep points
// come from the shards that hold the packets (ChaseArgs::fext), which compute
// them over their own processed packets and ask later shards for the rest
// (fluere_gpu.hip, fluere_sweep_*).
#include "exact.h"

#include "prim.h"

#include <algorithm>
#include <vector>

namespace fl {
namespace {

// Per-key positions packed below the dense id: (d << PBITS) | p, p < 2^38
// packets, d < 2^26 flows (MAX_FLOWS); MP (all ones): none.
constexpr int PBITS = 38;
constexpr uint64_t MP = (1ull << PBITS) - 1;
constexpr uint32_t NOPOS = 0xFFFFFFFFu;
// (a chain of sweep dependencies settles one link per pass; incremental passes
// re-chase only the keys that changed, so a long chain stays far cheaper than
// the sequential kernel: test_mode_b_sweep_chain_passes)
constexpr int MAX_PASSES = 250;
enum : uint8_t { K_FIN = 0, K_SWEEP = 1, K_ACTIVE = 2, K_LEAD = 3 };
// shard mode: role of a run in the flow's annex
enum : uint8_t { R_RECORD = 0, R_HEAD = 1, R_TAIL = 2, R_HEAD_TAIL = 3, R_LEAD = 4 };

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

// ---- 1. per-packet metadata of the packets to replay (one parse pass) -----
// A block takes EXM_PKTS consecutive packets in two phases:
//  1. candidates: every live packet, or (the hot pass's filter words) those
//     whose bucket may hold a complex flow, listed in LDS in capture order
//     (coalesced 4-byte reads; the skipped packets are not parsed);
//  2. the candidates, 256 at a time (full waves however sparse they are):
//     parse, dictionary walk, the taken ones to the block's region of meta_blk
//     in capture order (one ballot per wave), the block's count to
//     bcount[blk0 + block].
// k_ex_compact concatenates the regions after a scan over the block counts.
constexpr uint32_t EXM_PKTS = 1024;
constexpr int EXM_R = EXM_PKTS / 256;
__global__ void __launch_bounds__(256) k_ex_meta(Batch B, TableSet T, int macs, int all, const uint8_t* cplx,
                                                 const uint8_t* cbits, ExMeta* meta_blk, uint32_t* bcount,
                                                 uint64_t blk0, const uint32_t* phash, const uint32_t* emap,
                                                 const ExMeta* hmeta) {
    __shared__ uint32_t s_c[EXM_PKTS];
    __shared__ uint32_t s_w[2][4];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint64_t base = (uint64_t)blockIdx.x * EXM_PKTS;
    // the words: filter buckets (Mode A, cbits), or the merge's flows (emap)
    const bool words = phash && ((!all && cbits) || emap);
    // phase 1 (the words' loads, then their buckets' bytes / flows' complex
    // flags, all in flight)
    bool cand[EXM_R];
    uint32_t hw[EXM_R];
#pragma unroll
    for (int r = 0; r < EXM_R; r++) {
        const uint64_t li = base + r * 256 + tid;
        cand[r] = li < B.n;
        hw[r] = (words && cand[r]) ? phash[li] : PH_PARSE;
    }
#pragma unroll
    for (int r = 0; r < EXM_R; r++) {
        if (hw[r] == PH_PARSE) continue;
        if (emap && (hw[r] & (PH_ID | PH_EREF))) {
            const uint32_t d = ph_flow(hw[r], emap);
            cand[r] = d < T.fmax && (all || cplx[d]);
        } else if (!all && cbits) {
            cand[r] = cbits[hw[r] & ((1u << CBITS_LOG2) - 1)] != 0;
        }
    }
    uint32_t nc = 0;
#pragma unroll
    for (int r = 0; r < EXM_R; r++) {
        const uint64_t bal = __ballot(cand[r]);
        if (lane == 0) s_w[r & 1][w] = (uint32_t)__popcll(bal);
        __syncthreads();
        uint32_t before = nc;
        for (uint32_t k = 0; k < w; k++) before += s_w[r & 1][k];
        if (cand[r])
            s_c[before + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u))] =
                (uint32_t)(r * 256 + tid);
        nc += s_w[r & 1][0] + s_w[r & 1][1] + s_w[r & 1][2] + s_w[r & 1][3];
    }
    __syncthreads();  // (every candidate listed)
    // phase 2
    uint32_t nt = 0;
    ExMeta* region = meta_blk + (blk0 + blockIdx.x) * EXM_PKTS;
    for (uint32_t j = 0, r = 0; j < nc; j += 256, r++) {
        const uint32_t i = j + tid;
        uint32_t take = 0;
        ExMeta m;
        memset(&m, 0, sizeof m);
        if (i < nc) {
            const uint64_t li = base + s_c[i];
            const uint32_t wd = words ? phash[li] : PH_PARSE;
            const bool known = emap && wd != PH_PARSE && (wd & (PH_ID | PH_EREF));
            // a packet the hot parser took: its metadata from the hot pass
            // (32 bytes instead of a window and a parse)
            bool copied = false;
            if (known && hmeta) {
                const ExMeta h = hmeta[li];
                if (h.d == 0) {
                    copied = true;
                    const uint32_t d = ph_flow(wd, emap);
                    if (d < T.fmax && (all || cplx[d])) {
                        take = 1;
                        m = h;
                        m.d = d;
                    }
                }
            }
            // the register parser first (an 80-byte window), the general one
            // only for the classes it declines
            Parsed P;
            P.cls = 1;
            if (!copied) {
                const uint32_t off = B.offs[li];
                Win W;
                load_win(B, off, W);
                parse_loaded_fast(B, off, W, macs != 0, P);
            }
            if (!copied && P.cls == 2) parse_record(B, li, macs != 0, 0, P);
            if (!copied && P.cls == 0) {
                uint8_t dir;
                uint32_t d;
                if (known) {  // the merge resolved this packet's flow
                    dir = canon_dir(P, macs != 0);
                    d = ph_flow(wd, emap);
                } else {
                    CKey k;
                    canon_key(P, macs != 0, k, dir);
                    bool maybe = true;
                    if (!all && cbits) {  // no complex flow has this key's bucket: no dictionary walk
                        const uint32_t b = ckey_bucket(k.w);
                        maybe = cbits[b] != 0;
                    }
                    d = maybe ? dense_of_key(T, k, false, nullptr, nullptr) : FAIL;
                }
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
        }
        const uint64_t bal = __ballot(take != 0);
        if (lane == 0) s_w[r & 1][w] = (uint32_t)__popcll(bal);
        __syncthreads();
        uint32_t before = nt;
        for (uint32_t k = 0; k < w; k++) before += s_w[r & 1][k];
        if (take)
            region[before + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u))] = m;
        nt += s_w[r & 1][0] + s_w[r & 1][1] + s_w[r & 1][2] + s_w[r & 1][3];
    }
    if (tid == 0) bcount[blk0 + blockIdx.x] = nt;
}

// compaction in capture order: cm[k] = the k-th replayed packet; sort keys
// (key, index).  Block b of k_ex_meta's regions -> positions bpos[b] ...
__global__ void __launch_bounds__(256) k_ex_compact(const ExMeta* meta_blk, const uint32_t* bcount, const uint32_t* bpos,
                                                    ExMeta* cm, uint32_t* key, uint32_t* val) {
    const uint32_t b = blockIdx.x, c = bcount[b];
    for (uint32_t i = threadIdx.x; i < c; i += blockDim.x) {
        const uint32_t k = bpos[b] + i;
        const ExMeta m = meta_blk[(uint64_t)b * EXM_PKTS + i];
        cm[k] = m;
        key[k] = m.d;  // (a stable sort by flow keeps capture order within a flow)
        val[k] = k;
    }
}

// Several small fills in one launch (each hipMemsetAsync is a kernel of its
// own, ~5 us on the stream): up to FILL_MAX (pointer, bytes, byte value),
// 16-byte stores where a range allows them.
constexpr int FILL_MAX = 4;
struct Fills {
    uint8_t* p[FILL_MAX];
    uint64_t n[FILL_MAX];
    uint32_t v[FILL_MAX];  // the byte value, replicated to a word
    int k = 0;
    void add(void* ptr, uint64_t bytes, uint8_t value) {
        if (!bytes) return;
        p[k] = (uint8_t*)ptr;
        n[k] = bytes;
        v[k] = value * 0x01010101u;
        k++;
    }
};
__global__ void __launch_bounds__(256) k_fill_many(Fills f) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (uint64_t)gridDim.x * blockDim.x;
    for (int j = 0; j < f.k; j++) {
        uint8_t* p = f.p[j];
        const uint64_t n = f.n[j];
        const uint32_t v = f.v[j];
        // byte head up to 16-byte alignment, 16-byte body, byte tail
        const uint64_t head = min(n, (uint64_t)((16 - ((uintptr_t)p & 15)) & 15));
        const uint64_t body = (n - head) / 16;
        if (tid < head) p[tid] = (uint8_t)v;
        uint4* q = reinterpret_cast<uint4*>(p + head);
        for (uint64_t i = tid; i < body; i += nt) q[i] = make_uint4(v, v, v, v);
        const uint64_t t0 = head + body * 16;
        if (tid < n - t0) p[t0 + tid] = (uint8_t)v;
    }
}
static hipError_t fill_many(const Fills& f, hipStream_t s) {
    if (!f.k) return hipSuccess;
    uint64_t big = 0;
    for (int j = 0; j < f.k; j++) big = std::max<uint64_t>(big, f.n[j] / 16 + 16);
    k_fill_many<<<(unsigned)std::min<uint64_t>(1024, (big + 255) / 256), 256, 0, s>>>(f);
    return hipGetLastError();
}

// one GPU, Mode B over the hot pass's dense metadata: packet k's flow from
// the merge's word; a packet without one is counted in *bad (then the caller
// takes the k_ex_meta path)
__global__ void __launch_bounds__(256) k_ex_pidkeys(uint64_t n, const uint32_t* pid, const uint32_t* emap, uint32_t fmax,
                                                    uint32_t* key, uint32_t* val, uint32_t* bad) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t d = k < n ? ph_flow(pid[k], emap) : 0u;
    const bool miss = k < n && (d == FAIL || d >= fmax);
    if (bad && __ballot(miss) && (threadIdx.x & 63) == 0) atomicAdd(bad, 1u);
    if (k >= n) return;
    key[k] = miss ? 0xFFFFFFFFu : d;  // (bad null: k_ex_tscan / k_ex_mono count the misses)
    val[k] = (uint32_t)k;
}

// sharded Mode B owner: sort keys of the shards' packets (capture order)
__global__ void __launch_bounds__(256) k_ex_keys(uint64_t n, const ExMeta* cm, uint32_t* key, uint32_t* val) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    key[k] = cm[k].d;
    val[k] = (uint32_t)k;
}

// ---- 2. sorted view, key heads, next-eligible / next-FIN inputs -------------
// GATHER_ITEMS positions per thread (256 apart: coalesced), every random
// 32-byte load issued before the first store
#ifndef FLUERE_GATHER_ITEMS
#define FLUERE_GATHER_ITEMS 1  // (4: 369 vs 327 us on tcp_t1 -- more loads in flight per lane did not pay)
#endif
constexpr uint32_t GATHER_ITEMS = FLUERE_GATHER_ITEMS;
__global__ void __launch_bounds__(256) k_ex_gather(uint64_t n, const uint32_t* skey, const uint32_t* sval,
                                                   const ExMeta* cm, ExMeta* sm, uint32_t* hf, uint8_t* gbits,
                                                   uint8_t* prp) {
    const uint64_t p0 = (uint64_t)blockIdx.x * (256 * GATHER_ITEMS) + threadIdx.x;
    uint32_t v[GATHER_ITEMS];
#pragma unroll
    for (uint32_t j = 0; j < GATHER_ITEMS; j++) {
        const uint64_t p = p0 + j * 256;
        v[j] = p < n ? sval[p] : 0u;
    }
    ExMeta m[GATHER_ITEMS];
#pragma unroll
    for (uint32_t j = 0; j < GATHER_ITEMS; j++)
        if (p0 + j * 256 < n) m[j] = cm[v[j]];
#pragma unroll
    for (uint32_t j = 0; j < GATHER_ITEMS; j++) {
        const uint64_t p = p0 + j * 256;
        if (p >= n) break;
        const uint32_t d = skey[p];
        m[j].d = d;  // (the sort key is the flow: dense capture-order metadata carries none)
        sm[p] = m[j];
        hf[p] = (p == 0 || skey[p - 1] != d) ? 1u : 0u;
        // the next eligible / FIN-RST scans read these flags (k_next_scan)
        gbits[p] = m[j].bits;
        if (prp) prp[p] = 1;  // (Mode B: the first guess, every packet processed)
    }
}

__global__ void k_ex_nkeys(const uint32_t* hpos_last, const uint32_t* hf_last, uint32_t* out) {
    if (threadIdx.x == 0) *out = *hpos_last + *hf_last;
}

// ---- 3. Mode B: timestamps non-decreasing over the valid packets? ---------
__global__ void __launch_bounds__(256) k_ex_mono(uint64_t n, const ExMeta* cm, uint32_t* bad, const uint32_t* mkey,
                                                 uint32_t* miss) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool back = k > 0 && k < n && cm[k].t < cm[k - 1].t;
    if (__ballot(back) && (threadIdx.x & 63) == 0) *bad = 1u;  // (one store per wave, not an atomic per packet)
    if (mkey && __ballot(k < n && mkey[k] == 0xFFFFFFFFu) && (threadIdx.x & 63) == 0) *miss = 1u;  // (k_ex_tscan's)
}

// lower_bound of t0 + b * bw over the non-decreasing times, b = 0..nb
__global__ void __launch_bounds__(256) k_ex_tindex(uint64_t n, const ExMeta* cm, uint64_t t0, uint64_t bw, uint64_t nb,
                                                   uint32_t* tbl) {
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b > nb) return;
    const unsigned long long v = t0 + b * bw;
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (cm[mid].t < v) lo = mid + 1;
        else hi = mid;
    }
    tbl[b] = (uint32_t)lo;
}

// Mode B, one pass over the capture-order times: monotonicity (*bad), and
// the time-bucket index of k_ex_tindex as range starts (starts[b] = the first
// packet of bucket b's range, written by that packet; zero elsewhere) for an
// inclusive max-scan.  The buckets are k_ex_tindex's: t0 = t_0, nb given,
// bw = (t_last - t0) / nb + 1 (the host computes the same from the same
// times); with times that go backwards the index is not used.
__global__ void __launch_bounds__(256) k_ex_tscan(uint64_t n, const ExMeta* cm, const unsigned long long* ct,
                                                  uint64_t nb, uint32_t* starts, uint32_t* bad, const uint32_t* mkey,
                                                  uint32_t* miss) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // (ct: the times alone, 8 of every 32 bytes of cm)
    auto tm = [&](uint64_t q) -> unsigned long long { return ct ? ct[q] : cm[q].t; };
    const unsigned long long t0 = tm(0), tl = tm(n - 1);
    const uint64_t bw = max((uint64_t)1, (tl > t0 ? tl - t0 : 0) / nb + 1);
    auto bucket = [&](unsigned long long v) -> uint64_t { return v <= t0 ? 0 : min(nb, (uint64_t)((v - t0) / bw)); };
    bool back = false;
    if (k < n) {
        const unsigned long long t = tm(k);
        const uint64_t bk = bucket(t);
        if (k > 0) {
            const unsigned long long tp = tm(k - 1);
            back = t < tp;
            const uint64_t bp = bucket(tp);
            if (bk > bp) starts[bp + 1] = (uint32_t)k;  // buckets (bp, bk] start at k
        }
        if (k == n - 1 && bk + 1 <= nb) starts[bk + 1] = (uint32_t)n;  // the buckets past the last time
    }
    if (__ballot(back) && (threadIdx.x & 63) == 0) *bad = 1u;
    // (mkey: k_ex_pidkeys' keys, capture order -- a packet without a flow word)
    if (mkey && __ballot(k < n && mkey[k] == 0xFFFFFFFFu) && (threadIdx.x & 63) == 0) *miss = 1u;
}

// ---- next-position scans --------------------------------------------------------
// out_o[p] = min over p' >= p of v_o(p'), v_o(p) = key(p) << PBITS | (flags[p] & mask_o ?
// p : MP): for sorted position p, the first position at or after p within its
// key whose flags have mask_o (the key in the high bits; MP: none) -- the next
// create-eligible and next FIN/RST packets of a key (two outputs), or with no
// key the next processed packet.  Replaces a reversed input array and a
// library min-scan per output: the keys (4 B) and flags (1 B) read twice, one
// write per output, 16 contiguous items a thread (vector loads and stores).
// k_next_reduce: each tile's minima; k_next_scan: a tile's suffix is the
// minimum of the later tiles' (every workgroup reduces them itself: no chained
// look-back, whose serial cross-XCD waits cost ~0.5 us a tile), then the
// suffix scan within the tile.
struct NextScan {
    uint64_t n;
    const uint32_t* key;        // sorted keys, or null (0)
    const uint8_t* flags;
    uint32_t mask[2];
    int nout;
    unsigned long long* out[2];
    unsigned long long* tagg;   // per tile: its 2 minima
    uint32_t T;                 // tiles
};
constexpr int NSC_ITEMS = 16;
constexpr uint32_t NSC_TILE = 256 * NSC_ITEMS;

// this thread's 16 items starting at p0 (a multiple of 16): values v[o][k]
__device__ __forceinline__ void nsc_load(const NextScan& a, uint64_t p0, unsigned long long (&v)[2][NSC_ITEMS]) {
    uint32_t kk[NSC_ITEMS];
    uint8_t ff[NSC_ITEMS];
    if (p0 + NSC_ITEMS <= a.n) {
        const uint4* kp = reinterpret_cast<const uint4*>(a.key ? a.key + p0 : nullptr);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint4 x = a.key ? kp[q] : make_uint4(0, 0, 0, 0);
            kk[4 * q] = x.x; kk[4 * q + 1] = x.y; kk[4 * q + 2] = x.z; kk[4 * q + 3] = x.w;
        }
        const uint4 f = *reinterpret_cast<const uint4*>(a.flags + p0);
        const uint32_t fw[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
        for (int k = 0; k < NSC_ITEMS; k++) ff[k] = (uint8_t)(fw[k >> 2] >> (8 * (k & 3)));
    } else {
#pragma unroll
        for (int k = 0; k < NSC_ITEMS; k++) {
            const bool in = p0 + k < a.n;
            kk[k] = (in && a.key) ? a.key[p0 + k] : 0u;
            ff[k] = in ? a.flags[p0 + k] : (uint8_t)0;
        }
    }
#pragma unroll
    for (int k = 0; k < NSC_ITEMS; k++) {
        const uint64_t p = p0 + k;
        const unsigned long long hi = (unsigned long long)kk[k] << PBITS;
        const bool in = p < a.n;
        v[0][k] = in ? (hi | ((ff[k] & a.mask[0]) ? p : MP)) : ~0ull;
        v[1][k] = in ? (hi | ((ff[k] & a.mask[1]) ? p : MP)) : ~0ull;
    }
}
// the block's minimum of (x0, x1) into s[0..1] (256 threads; ends with a barrier)
__device__ __forceinline__ void nsc_block_min(unsigned long long x0, unsigned long long x1, unsigned long long (*s_w)[4],
                                              unsigned long long* s) {
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        x0 = min(x0, (unsigned long long)__shfl_xor(x0, d, 64));
        x1 = min(x1, (unsigned long long)__shfl_xor(x1, d, 64));
    }
    if (lane == 0) {
        s_w[0][wv] = x0;
        s_w[1][wv] = x1;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        s[0] = min(min(s_w[0][0], s_w[0][1]), min(s_w[0][2], s_w[0][3]));
        s[1] = min(min(s_w[1][0], s_w[1][1]), min(s_w[1][2], s_w[1][3]));
    }
    __syncthreads();
}
__global__ void __launch_bounds__(256) k_next_reduce(NextScan a) {
    __shared__ unsigned long long s_w[2][4], s_m[2];
    unsigned long long v[2][NSC_ITEMS];
    nsc_load(a, (uint64_t)blockIdx.x * NSC_TILE + (uint64_t)threadIdx.x * NSC_ITEMS, v);
    unsigned long long m0 = ~0ull, m1 = ~0ull;
#pragma unroll
    for (int k = 0; k < NSC_ITEMS; k++) {
        m0 = min(m0, v[0][k]);
        m1 = min(m1, v[1][k]);
    }
    nsc_block_min(m0, m1, s_w, s_m);
    if (threadIdx.x == 0) {
        a.tagg[2 * blockIdx.x] = s_m[0];
        a.tagg[2 * blockIdx.x + 1] = s_m[1];
    }
}
// The tiles' totals scanned once, by one workgroup (each tile used
// to combine every earlier / later tile's total itself, O(T^2) loads -- ~300M
// at 100M items): each thread folds a contiguous run of tiles, the runs'
// results are scanned across the block, then written back in place.
constexpr int TSC_B = 1024;
// tsum[t] <- the sum of tsum[0 .. t) (exclusive prefix, in place)
__global__ void __launch_bounds__(TSC_B) k_tile_prefix(uint32_t* tsum, uint32_t T) {
    __shared__ uint32_t s_w[TSC_B / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t per = (T + TSC_B - 1) / TSC_B, t0 = tid * per, t1 = min(T, t0 + per);
    uint32_t run = 0;
    for (uint32_t t = t0; t < t1; t++) run += tsum[t];
    uint32_t incl = run;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d, 64);
        if (lane >= (uint32_t)d) incl += y;
    }
    if (lane == 63) s_w[wv] = incl;
    __syncthreads();
    uint32_t ex = incl - run;
    for (uint32_t q = 0; q < wv; q++) ex += s_w[q];
    for (uint32_t t = t0; t < t1; t++) {
        const uint32_t v = tsum[t];
        tsum[t] = ex;
        ex += v;
    }
}
// tagg[2t + o] <- the minimum of tagg[2u + o] over u > t (exclusive suffix, in place)
__global__ void __launch_bounds__(TSC_B) k_tile_suffix_min(unsigned long long* tagg, uint32_t T) {
    __shared__ unsigned long long s_w[2][TSC_B / 64];
    constexpr unsigned long long ID = ~0ull;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t per = (T + TSC_B - 1) / TSC_B, t0 = tid * per, t1 = min(T, t0 + per);
    unsigned long long run[2] = {ID, ID}, incl[2], after[2];
    for (uint32_t t = t0; t < t1; t++) {
        run[0] = min(run[0], tagg[2 * t]);
        run[1] = min(run[1], tagg[2 * t + 1]);
    }
#pragma unroll
    for (int o = 0; o < 2; o++) {
        incl[o] = run[o];  // inclusive suffix over the lanes, then the later waves
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const unsigned long long y = __shfl_down(incl[o], d, 64);
            if (lane + d < 64) incl[o] = min(incl[o], y);
        }
        const unsigned long long dn = __shfl_down(incl[o], 1, 64);
        after[o] = lane < 63 ? dn : ID;
        if (lane == 0) s_w[o][wv] = incl[o];
    }
    __syncthreads();
#pragma unroll
    for (int o = 0; o < 2; o++)
        for (uint32_t q = wv + 1; q < TSC_B / 64; q++) after[o] = min(after[o], s_w[o][q]);
    for (uint32_t t = t1; t-- > t0;) {
        const unsigned long long v0 = tagg[2 * t], v1 = tagg[2 * t + 1];
        tagg[2 * t] = after[0];
        tagg[2 * t + 1] = after[1];
        after[0] = min(after[0], v0);
        after[1] = min(after[1], v1);
    }
}

__global__ void __launch_bounds__(256) k_next_scan(NextScan a) {
    __shared__ unsigned long long s_suf[2];
    __shared__ unsigned long long s_w[2][4];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t tile = blockIdx.x;
    constexpr unsigned long long ID = ~0ull;
    // the later tiles' minima (k_tile_suffix_min)
    if (tid == 0) {
        s_suf[0] = a.tagg[2 * tile];
        s_suf[1] = a.tagg[2 * tile + 1];
    }
    __syncthreads();
    const uint64_t p0 = (uint64_t)tile * NSC_TILE + (uint64_t)tid * NSC_ITEMS;
    unsigned long long v[2][NSC_ITEMS];
    nsc_load(a, p0, v);
    unsigned long long after[2];
#pragma unroll
    for (int o = 0; o < 2; o++) {
        // suffix within the thread
        unsigned long long run = ID;
#pragma unroll
        for (int k = NSC_ITEMS - 1; k >= 0; k--) {
            run = min(run, v[o][k]);
            v[o][k] = run;
        }
        // the later lanes of the wave (inclusive suffix scan, then shift by one)
        unsigned long long incl = run;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const unsigned long long y = __shfl_down(incl, d, 64);
            if (lane + d < 64) incl = min(incl, y);
        }
        const unsigned long long dn = __shfl_down(incl, 1, 64);
        after[o] = lane < 63 ? dn : ID;
        if (lane == 0) s_w[o][wv] = incl;  // (nsc_block_min's barriers are behind us)
    }
    __syncthreads();
#pragma unroll
    for (int o = 0; o < 2; o++) {
        for (uint32_t q = wv + 1; q < 4; q++) after[o] = min(after[o], s_w[o][q]);
        after[o] = min(after[o], s_suf[o]);
    }
#pragma unroll
    for (int o = 0; o < 2; o++) {
        if (o >= a.nout) break;
        unsigned long long* dst = a.out[o] + p0;
        if (p0 + NSC_ITEMS <= a.n) {
#pragma unroll
            for (int k = 0; k < NSC_ITEMS; k += 2) {
                ulonglong2 w;
                w.x = min(after[o], v[o][k]);
                w.y = min(after[o], v[o][k + 1]);
                *reinterpret_cast<ulonglong2*>(dst + k) = w;
            }
        } else {
#pragma unroll
            for (int k = 0; k < NSC_ITEMS; k++)
                if (p0 + k < a.n) dst[k] = min(after[o], v[o][k]);
        }
    }
}

// ---- flag counts ---------------------------------------------------------------
// out[p] = the flags before p (exclusive) or up to p (inclusive), flags 0/1
// words; with a list, list[c] = p for the c-th flagged position (the key
// heads, the instance starts: the scatter the separate k_ex_heads /
// k_ex_starts passes did).  k_next_*'s structure: a reduce, then each tile
// adds the earlier tiles' totals itself (no look-back chain) and scans its
// 4096 items, 16 contiguous a thread (vector loads and stores).  Replaces a
// library scan (~50 us for 10M words) and the scatter pass (~20 us).
__global__ void __launch_bounds__(256) k_fc_reduce(uint64_t n, const uint32_t* flags, uint32_t* tsum) {
    __shared__ uint32_t s_w[4];
    const uint64_t p0 = (uint64_t)blockIdx.x * NSC_TILE + (uint64_t)threadIdx.x * NSC_ITEMS;
    uint32_t t = 0;
    if (p0 + NSC_ITEMS <= n) {
        const uint4* fp = reinterpret_cast<const uint4*>(flags + p0);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint4 x = fp[q];
            t += x.x + x.y + x.z + x.w;
        }
    } else {
        for (uint64_t p = p0; p < n && p < p0 + NSC_ITEMS; p++) t += flags[p];
    }
    t = wave_sum(t);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = t;
    __syncthreads();
    if (threadIdx.x == 0) tsum[blockIdx.x] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
}
__global__ void __launch_bounds__(256) k_fc_scan(uint64_t n, const uint32_t* flags, uint32_t* out, int inclusive,
                                                 uint32_t* list, const uint32_t* tsum) {
    __shared__ uint32_t s_w[4];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, tile = blockIdx.x;
    // the earlier tiles' totals (k_tile_prefix)
    const uint32_t s_base = tsum[tile];
    const uint64_t p0 = (uint64_t)tile * NSC_TILE + (uint64_t)tid * NSC_ITEMS;
    uint32_t f[NSC_ITEMS];
    const bool full = p0 + NSC_ITEMS <= n;
    if (full) {
        const uint4* fp = reinterpret_cast<const uint4*>(flags + p0);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint4 x = fp[q];
            f[4 * q] = x.x; f[4 * q + 1] = x.y; f[4 * q + 2] = x.z; f[4 * q + 3] = x.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < NSC_ITEMS; k++) f[k] = p0 + k < n ? flags[p0 + k] : 0u;
    }
    uint32_t run = 0;
#pragma unroll
    for (int k = 0; k < NSC_ITEMS; k++) run += f[k];
    // exclusive prefix of the thread totals: within the wave, then the waves before
    uint32_t incl = run;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d, 64);
        if (lane >= (uint32_t)d) incl += y;
    }
    __syncthreads();  // (s_w's totals above are read)
    if (lane == 63) s_w[wv] = incl;
    __syncthreads();
    uint32_t ex = s_base + incl - run;
    for (uint32_t q = 0; q < wv; q++) ex += s_w[q];
    uint32_t o[NSC_ITEMS];
#pragma unroll
    for (int k = 0; k < NSC_ITEMS; k++) {
        if (list && f[k] && p0 + k < n) list[ex] = (uint32_t)(p0 + k);
        ex += f[k];
        o[k] = inclusive ? ex : ex - f[k];
    }
    if (full) {
        uint4* dp = reinterpret_cast<uint4*>(out + p0);
#pragma unroll
        for (int q = 0; q < 4; q++) dp[q] = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
    } else {
#pragma unroll
        for (int k = 0; k < NSC_ITEMS; k++)
            if (p0 + k < n) out[p0 + k] = o[k];
    }
}
// tmp: a word per tile of 4096 items (exact.h's flag_count)
static int fc_run(hipStream_t s, uint64_t n, const uint32_t* flags, uint32_t* out, bool inclusive, uint32_t* list,
                      void* tmp) {
    if (!n) return FLUERE_OK;
    const uint64_t T = (n + NSC_TILE - 1) / NSC_TILE;
    if (T >= (1u << 31)) return FLUERE_E_ARG;
    k_fc_reduce<<<(unsigned)T, 256, 0, s>>>(n, flags, (uint32_t*)tmp);
    k_tile_prefix<<<1, TSC_B, 0, s>>>((uint32_t*)tmp, (uint32_t)T);
    k_fc_scan<<<(unsigned)T, 256, 0, s>>>(n, flags, out, inclusive ? 1 : 0, list, (const uint32_t*)tmp);
    HIPCHECK(hipGetLastError());
    return FLUERE_OK;
}

// n items; `tmp` holds the tiles' minima (16 bytes a tile of 4096 items: the
// callers pass an n x 8-byte array)
static int next_scan(hipStream_t s, uint64_t n, const uint32_t* key, const uint8_t* flags, uint32_t m0, uint32_t m1,
                     int nout, unsigned long long* o0, unsigned long long* o1, void* tmp) {
    if (!n) return FLUERE_OK;
    const uint64_t T = (n + NSC_TILE - 1) / NSC_TILE;
    if (T >= (1u << 31)) return FLUERE_E_ARG;
    NextScan a{};
    a.n = n;
    a.key = key;
    a.flags = flags;
    a.mask[0] = m0;
    a.mask[1] = m1;
    a.nout = nout;
    a.out[0] = o0;
    a.out[1] = o1;
    a.tagg = (unsigned long long*)tmp;
    a.T = (uint32_t)T;
    k_next_reduce<<<(unsigned)T, 256, 0, s>>>(a);
    k_tile_suffix_min<<<1, TSC_B, 0, s>>>(a.tagg, a.T);
    k_next_scan<<<(unsigned)T, 256, 0, s>>>(a);
    HIPCHECK(hipGetLastError());
    return FLUERE_OK;
}


}  // namespace

// ---- max segment tree over the processed packets' times ---------------------
// tree[P + k] = t_k + 1 if packet k (capture order) is processed, else 0;
// tree[i] = max(tree[2i], tree[2i + 1]).  tree_first (exact.h) walks right
// from leaf k0 to the first leaf >= x: O(log n), any timestamp order.
__global__ void __launch_bounds__(256) k_tree_leaves(uint64_t n, uint64_t P, const ExMeta* cm, const uint8_t* pr,
                                                     unsigned long long* tree) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < P) tree[P + k] = (k < n && pr[k]) ? cm[k].t + 1 : 0ull;
}
__global__ void __launch_bounds__(256) k_tree_level(uint64_t h, unsigned long long* tree) {
    const uint64_t i = h + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < 2 * h) tree[i] = max(tree[2 * i], tree[2 * i + 1]);
}
int tree_build(uint64_t n, const ExMeta* cm, const uint8_t* pr, unsigned long long* tree, uint64_t P, hipStream_t s) {
    k_tree_leaves<<<(unsigned)((P + 255) / 256), 256, 0, s>>>(n, P, cm, pr, tree);
    for (uint64_t h = P / 2; h >= 1; h /= 2)
        k_tree_level<<<(unsigned)((h + 255) / 256), 256, 0, s>>>(h, tree);
    HIPCHECK(hipGetLastError());
    return FLUERE_OK;
}
uint64_t tree_leaves(uint64_t n) {
    uint64_t P = 1;
    while (P < n) P *= 2;
    return P;
}

namespace {

// ---- 4. the chase: one thread per key ----------------------------------------
struct ChaseArgs {
    uint64_t n;
    uint32_t n_keys;         // (d_nkeys non-null: the count is on the device, the grid covers n)
    const uint32_t* heads;
    const ExMeta* sm;   // sorted by (key, index)
    const uint32_t* sval;  // sorted position -> capture-order index k (Mode B: into cm)
    const unsigned long long* ne_rev;  // next eligible / FIN-RST position within the key, at each position (k_next_scan)
    const unsigned long long* nf_rev;
    int mode_b;
    uint64_t timeout_us;
    const ExMeta* cm;   // capture order (Mode B sweep points)
    const unsigned long long* np_rev;  // next processed packet at or after each capture position (non-decreasing times)
    const unsigned long long* tree;    // max segment tree (times that go backwards), or null
    uint64_t tree_P;
    const uint32_t* tbl;               // non-decreasing times: lower_bound of t0 + b * bw for every bucket b
    uint64_t t0, bw, nb;
    const unsigned long long* fext;    // sharded Mode B: sweep point of every packet (capture order), or null
    // out, indexed by the instance's first position
    uint32_t* sflag;
    uint32_t* iend;
    uint8_t* ikind;
    unsigned long long* ij;   // FIN: its index; sweep: the sweeping packet's index
    unsigned long long* iie;  // sweep: the index of the creation that pushed the firing entry
    unsigned long long* iex;  // sweep: that entry's exp
    unsigned long long* ej;   // Mode B: sweep point of the entry pushed at this creation
    uint32_t* link;           // Mode B: pending entries of an orientation, sorted: next
    uint32_t* plink;          //                                               previous
    // shard mode
    int shard_mode;
    uint8_t* irole;
    uint32_t* ikey;           // key ordinal of the run (annex index)
    fluere_flow_annex* annex;
    uint32_t* annex_of;
    const uint8_t* flow_key;  // TableSet::flow_key (56-byte canonical keys by dense id)
    const uint32_t* d_nkeys = nullptr;  // Mode A: the key count, written on the device (no host read)
    // Incremental Mode B passes (non-decreasing times, one GPU; null: off).  A
    // key's chase depends on the processed set only through its sweep
    // lookups, so a pass re-chases only the keys one of whose lookups now
    // answers differently (k_ex_check) and keeps the other keys' instances.
    uint8_t* stamp = nullptr;         // per position: the pass that made it an instance start
    uint8_t* kpass = nullptr;         // per key: the pass that last chased it
    const uint8_t* kdirty = nullptr;  // the keys this pass chases (null: every key)
    uint32_t* elook = nullptr;        // per creation: its sweep lookup's start position (NOPOS: none)
    uint32_t* ekp = nullptr;          //               the answer (capture index; NOPOS: none)
    uint32_t pass_id = 0;
    int np_all = 0;  // every replayed packet processed (the first pass's guess): next processed = itself
    const unsigned long long* ct = nullptr;  // or null: cm's times alone (the sweep points' searches)
};

__device__ __forceinline__ unsigned long long exp_of(uint64_t t, uint64_t timeout_us) {
    return t + timeout_us < t ? NONE64 : t + timeout_us;  // (saturating)
}

// sweep point of the entry pushed at sorted position c: the first processed
// packet k >= c (capture order) with t_k >= exp -> its packet index
// (k0 = sval[c] and the time bucket's range [lo, hi) are loaded by the caller,
// before the stores of the queue insert, so that they are in flight early)
__device__ __forceinline__ void sweep_bucket(const ChaseArgs& a, unsigned long long exp, uint64_t& lo, uint64_t& hi) {
    lo = 0;
    hi = a.n;
    if (a.fext || a.tree || exp == NONE64) return;
    if (exp <= a.t0) {
        hi = 0;
    } else {
        const uint64_t b = (exp - a.t0) / a.bw;
        if (b >= a.nb) lo = a.n;
        else { lo = a.tbl[b]; hi = a.tbl[b + 1]; }
    }
}
__device__ __forceinline__ unsigned long long sweep_point(const ChaseArgs& a, uint32_t c, uint32_t k0,
                                                          unsigned long long exp, uint64_t lo, uint64_t hi) {
    if (a.elook) a.elook[c] = NOPOS;  // (a lookup that no processed set changes)
    if (a.fext) return a.fext[k0];
    if (exp == NONE64) return NONE64;
    if (a.tree) {
        const uint64_t k = tree_first(a.tree, a.tree_P, k0, exp + 1);
        if (a.elook) {  // (times that go backwards: the lookup starts at k0 with this exp)
            a.elook[c] = k0;
            a.ekp[c] = k >= a.n ? NOPOS : (uint32_t)k;
        }
        return k >= a.n ? NONE64 : a.cm[k].gidx;
    }
    // non-decreasing times: lower_bound (within the exp's time bucket), then
    // the next processed packet
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if ((a.ct ? a.ct[mid] : a.cm[mid].t) < exp) lo = mid + 1;
        else hi = mid;
    }
    const uint64_t k = max((uint64_t)k0, lo);
    if (k >= a.n) return NONE64;
    const unsigned long long kp = a.np_all ? k : a.np_rev[k];
    if (a.elook) {
        a.elook[c] = (uint32_t)k;
        a.ekp[c] = kp == MP ? NOPOS : (uint32_t)kp;
    }
    return kp == MP ? NONE64 : a.cm[kp].gidx;
}

__global__ void __launch_bounds__(64) k_ex_chase(ChaseArgs a) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t n_keys = a.d_nkeys ? *a.d_nkeys : a.n_keys;
    if (q >= n_keys) return;
    if (a.kdirty && !a.kdirty[q]) return;  // incremental pass: this key's instances stand
    if (a.kpass) a.kpass[q] = (uint8_t)a.pass_id;
    const uint32_t p0 = a.heads[q];
    const uint32_t pend = q + 1 < n_keys ? a.heads[q + 1] : (uint32_t)a.n;
    // pending expiry entries per orientation, sorted by (sweep point, exp,
    // creation): the BTreeMap's pop order among the entries that can evict
    // this orientation's flow (offline_fluereflows.rs:161-175)
    uint32_t qh[2] = {NOPOS, NOPOS}, qt[2] = {NOPOS, NOPOS};
    auto drop_upto = [&](unsigned long long lim, bool inclusive) {
        for (int x = 0; x < 2; x++) {
            while (qh[x] != NOPOS && (inclusive ? a.ej[qh[x]] <= lim : a.ej[qh[x]] < lim)) qh[x] = a.link[qh[x]];
            if (qh[x] == NOPOS) qt[x] = NOPOS;
            else a.plink[qh[x]] = NOPOS;
        }
    };
    // x before y in the pop order (y is the newer creation on ties)
    auto before = [&](uint32_t x, uint32_t y) {
        if (a.ej[x] != a.ej[y]) return a.ej[x] < a.ej[y];
        return exp_of(a.sm[x].t, a.timeout_us) < exp_of(a.sm[y].t, a.timeout_us);
    };
    uint32_t pos = p0;
    // shard mode: from "no flow", the lead piece [p0, min(e0, f0 + 1)) and the
    // roles of the instances (the first one, if created at or before f0, is
    // the head; the one still open at the end, after f0, the tail)
    const unsigned long long f0 = a.nf_rev[p0] & MP;
    int n_inst = 0;
    if (a.shard_mode) {
        const unsigned long long e0 = a.ne_rev[p0] & MP;
        const uint32_t lead_end = (uint32_t)min(e0 == MP ? (unsigned long long)pend : e0,
                                                f0 == MP ? (unsigned long long)pend : f0 + 1);  // exclusive
        const uint32_t d = a.sm[p0].d;
        fluere_flow_annex& ax = a.annex[q];
        const uint32_t* kw = reinterpret_cast<const uint32_t*>(a.flow_key + (size_t)d * 56);
        for (int k = 0; k < 14; k++) ax.key[k] = kw[k];
        ax.flags = (f0 != MP ? 1u : 0u) | (lead_end > p0 ? 2u : 0u);
        ax.mid_last = 0;
        ax.f0 = f0 != MP ? a.sm[f0].gidx : NONE64;
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
        const unsigned long long ce = a.ne_rev[pos] & MP;
        if (ce == MP) break;
        const uint32_t c = (uint32_t)ce;
        const ExMeta mc = a.sm[c];
        const uint32_t o = mc.dir;
        // the loads that depend on c alone, issued before the queue's stores
        const unsigned long long fe = a.nf_rev[c] & MP;
        const unsigned long long fg = fe != MP ? a.sm[fe].gidx : 0;
        unsigned long long jf = NONE64;
        uint32_t front = NOPOS;
        if (a.mode_b) {
            const uint32_t k0 = a.sval[c];
            const unsigned long long ex = exp_of(mc.t, a.timeout_us);
            uint64_t blo, bhi;
            sweep_bucket(a, ex, blo, bhi);
            drop_upto(mc.gidx, false);  // entries that fired while the key had no flow
            a.ej[c] = sweep_point(a, c, k0, ex, blo, bhi);
            // sorted insert, from the tail (non-decreasing times: at the tail)
            uint32_t p = qt[o];
            while (p != NOPOS && before(c, p)) p = a.plink[p];
            a.plink[c] = p;
            if (p == NOPOS) {
                a.link[c] = qh[o];
                qh[o] = c;
            } else {
                a.link[c] = a.link[p];
                a.link[p] = c;
            }
            if (a.link[c] == NOPOS) qt[o] = c;
            else a.plink[a.link[c]] = c;
            front = qh[o];
            jf = a.ej[front];
        }
        uint32_t end;
        uint8_t kind;
        unsigned long long cj = NONE64, cie = 0, cex = 0;
        if (fe != MP && (jf == NONE64 || fg <= jf)) {  // FIN/RST first (the sweep runs after it)
            end = (uint32_t)fe;
            kind = K_FIN;
            cj = fg;
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
            cex = exp_of(a.sm[front].t, a.timeout_us);
        } else {
            end = pend - 1;
            kind = K_ACTIVE;
        }
        if (a.stamp) a.stamp[c] = (uint8_t)a.pass_id;
        else a.sflag[c] = 1;
        a.iend[c] = end;
        a.ikind[c] = kind;
        a.ij[c] = cj;
        a.iie[c] = cie;
        a.iex[c] = cex;
        if (a.shard_mode) {
            const bool head = n_inst == 0 && (f0 == MP || c <= f0);
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

// incremental pass: key q is dirty when one of the lookups of its last chase
// (at its instance starts, the previous pass's sflag) answers differently over
// this pass's processed set
__global__ void __launch_bounds__(256) k_ex_check(uint64_t n, const uint32_t* sflag, const uint32_t* elook,
                                                  const uint32_t* ekp, const unsigned long long* np_rev,
                                                  const uint32_t* hf, const uint32_t* hpos, uint8_t* kdirty,
                                                  const unsigned long long* tree, uint64_t tree_P, const ExMeta* sm,
                                                  uint64_t timeout_us) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n || !sflag[p]) return;
    const uint32_t L = elook[p];
    if (L == NOPOS) return;
    uint32_t r;
    if (tree) {  // backward times: the first processed packet at or after L with t > exp
        const uint64_t k = tree_first(tree, tree_P, L, exp_of(sm[p].t, timeout_us) + 1);
        r = k >= n ? NOPOS : (uint32_t)k;
    } else {
        const unsigned long long kp = np_rev[L];
        r = kp == MP ? NOPOS : (uint32_t)kp;
    }
    if (r != ekp[p]) kdirty[hpos[p] + hf[p] - 1] = 1;
}
// the instance starts of every key's last chase
__global__ void __launch_bounds__(256) k_ex_flags(uint64_t n, const uint8_t* stamp, const uint8_t* kpass,
                                                  const uint32_t* hf, const uint32_t* hpos, uint32_t* sflag) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n) sflag[p] = stamp[p] == kpass[hpos[p] + hf[p] - 1] ? 1u : 0u;
}

// ---- 5. members, processed set, reduction keys ------------------------------
// Mode B: the processed flag of each replayed packet (the members of an
// instance are processed); *changed when the set moved (one store per wave:
// an atomic per changed packet serialised on the one word).  The flags are
// compared in sorted order (prp, coalesced) and only a changed one is
// scattered to its capture position (pr[sval[p]]): reading pr at capture
// positions cost a random line per packet.
__global__ void __launch_bounds__(256) k_ex_members(uint64_t n, const uint32_t* incl, const uint32_t* ist,
                                                    const uint32_t* iend, const uint32_t* sval, uint8_t* pr,
                                                    uint8_t* prp, uint32_t* changed) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool ch = false;
    if (p < n) {
        const uint32_t q1 = incl[p];  // instances starting at or before p
        const bool member = q1 > 0 && p <= iend[ist[q1 - 1]];
        const uint8_t v = member ? 1 : 0;
        if (prp[p] != v) {
            prp[p] = v;
            pr[sval[p]] = v;
            ch = true;
        }
    }
    if (__ballot(ch) && (threadIdx.x & 63) == 0) *changed = 1u;
}

// ---- per-instance aggregates: update_flow's order-free fields over each
// instance's packets, the contiguous sorted run [ist[q], iend[ist[q]]] ----------
__device__ __forceinline__ void agg_clear(Agg& a) {
    a.pk[0] = a.pk[1] = 0;
    a.by[0] = a.by[1] = 0;
    a.mnp = a.mnt = NONE32;
    a.mxp = a.mxt = 0;
    for (int q = 0; q < 8; q++) a.fl[q] = 0;
    a.lastg = 0;
    a.lastt = 0;
}
__device__ __forceinline__ void agg_add(Agg& a, const ExMeta& m) {
    const bool r = m.dir != 0;  // (selects: a dynamic index would put the arrays in scratch)
    a.pk[0] += r ? 0u : 1u;
    a.pk[1] += r ? 1u : 0u;
    a.by[0] += r ? 0ull : (unsigned long long)m.doct;
    a.by[1] += r ? (unsigned long long)m.doct : 0ull;
    a.mnp = min(a.mnp, m.pkt);
    a.mxp = max(a.mxp, m.pkt);
    a.mnt = min(a.mnt, (uint32_t)m.ttl);
    a.mxt = max(a.mxt, (uint32_t)m.ttl);
    for (int q = 0; q < 8; q++) a.fl[q] += (m.tflags >> q) & 1;
    if (m.gidx >= a.lastg) {  // (the run is in index order: the last packet wins)
        a.lastg = m.gidx;
        a.lastt = m.t;
    }
}
__device__ __forceinline__ Agg agg_shfl_xor(const Agg& a, int o) {
    Agg b;
    b.pk[0] = __shfl_xor(a.pk[0], o, 64);
    b.pk[1] = __shfl_xor(a.pk[1], o, 64);
    b.by[0] = __shfl_xor(a.by[0], o, 64);
    b.by[1] = __shfl_xor(a.by[1], o, 64);
    b.mnp = __shfl_xor(a.mnp, o, 64);
    b.mxp = __shfl_xor(a.mxp, o, 64);
    b.mnt = __shfl_xor(a.mnt, o, 64);
    b.mxt = __shfl_xor(a.mxt, o, 64);
    for (int q = 0; q < 8; q++) b.fl[q] = __shfl_xor(a.fl[q], o, 64);
    b.lastg = __shfl_xor(a.lastg, o, 64);
    b.lastt = __shfl_xor(a.lastt, o, 64);
    return b;
}
__device__ __forceinline__ Agg agg_wave(Agg a) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) a = AggOp()(a, agg_shfl_xor(a, o));
    return a;
}

#ifndef FLUERE_AGG_UNROLL
#define FLUERE_AGG_UNROLL 8  // records loaded together per lane in k_ex_agg (tcp_t1: 4 -> 136 us, 8 -> 105 us, 16 -> 107 us)
#endif
constexpr uint32_t AGG_THREAD = 48;    // runs up to this long: one thread
constexpr uint32_t AGG_WAVE = 16384;   // up to this: one wave; longer: one 1024-thread block

// thread per instance; longer runs are listed for the wave / block kernels
// p_ninst (these three kernels and k_ex_records_t): the instance count on
// the device (Mode A: no host read; the grid covers an upper bound)
__global__ void __launch_bounds__(256) k_ex_agg(uint32_t n_inst, const uint32_t* ist, const uint32_t* iend,
                                                const ExMeta* sm, Agg* aggs, uint32_t* lists, uint32_t* cnt,
                                                const uint32_t* p_ninst) {
    if (p_ninst) n_inst = *p_ninst;
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    bool wide = false, huge = false;
    if (q < n_inst) {
        const uint32_t c = ist[q], e = iend[c];
        const uint32_t len = e - c + 1;
        if (len <= AGG_THREAD) {
            Agg a;
            agg_clear(a);
            // four records' loads in flight before the first is added (one at a
            // time, each lane waited out a load per packet of its run)
            uint32_t p = c;
#if FLUERE_AGG_UNROLL >= 8
            for (; p + 7 <= e; p += 8) {
                ExMeta m[8];
#pragma unroll
                for (int j = 0; j < 8; j++) m[j] = sm[p + j];
#pragma unroll
                for (int j = 0; j < 8; j++) agg_add(a, m[j]);
            }
#endif
            for (; p + 3 <= e; p += 4) {
                const ExMeta m0 = sm[p], m1 = sm[p + 1], m2 = sm[p + 2], m3 = sm[p + 3];
                agg_add(a, m0);
                agg_add(a, m1);
                agg_add(a, m2);
                agg_add(a, m3);
            }
            for (; p <= e; p++) agg_add(a, sm[p]);
            aggs[q] = a;
        } else {
            wide = len <= AGG_WAVE;
            huge = !wide;
        }
    }
    // wave-aggregated appends: lists[0..] wide runs, lists[n_inst - 1 ..] (downwards) huge runs
    const uint64_t mw = __ballot(wide), mh = __ballot(huge);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t rw = __builtin_amdgcn_mbcnt_hi((uint32_t)(mw >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mw, 0u));
    const uint32_t rh = __builtin_amdgcn_mbcnt_hi((uint32_t)(mh >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mh, 0u));
    uint32_t bw = 0, bh = 0;
    if (lane == 0) {
        if (mw) bw = atomicAdd(&cnt[0], (uint32_t)__popcll(mw));
        if (mh) bh = atomicAdd(&cnt[1], (uint32_t)__popcll(mh));
    }
    bw = __shfl(bw, 0, 64);
    bh = __shfl(bh, 0, 64);
    if (wide) lists[bw + rw] = q;
    if (huge) lists[n_inst - 1 - (bh + rh)] = q;
}

// one wave per listed run (grid-stride over the device-side count)
__global__ void __launch_bounds__(256) k_ex_agg_wave(uint32_t n_inst, const uint32_t* ist, const uint32_t* iend,
                                                     const ExMeta* sm, Agg* aggs, const uint32_t* lists,
                                                     const uint32_t* cnt, const uint32_t* p_ninst) {
    if (p_ninst) n_inst = *p_ninst;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w0 = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * blockDim.x) >> 6;
    const uint32_t nwide = cnt[0];
    for (uint32_t i = w0; i < nwide; i += nw) {
        const uint32_t q = lists[i];
        const uint32_t c = ist[q], e = iend[c];
        Agg a;
        agg_clear(a);
        for (uint32_t p = c + lane; p <= e; p += 64) agg_add(a, sm[p]);
        a = agg_wave(a);
        if (lane == 0) aggs[q] = a;
    }
}

// one block per listed huge run (an elephant instance)
__global__ void __launch_bounds__(1024) k_ex_agg_block(uint32_t n_inst, const uint32_t* ist, const uint32_t* iend,
                                                       const ExMeta* sm, Agg* aggs, const uint32_t* lists,
                                                       const uint32_t* cnt, const uint32_t* p_ninst) {
    __shared__ Agg part[16];
    if (p_ninst) n_inst = *p_ninst;
    const uint32_t nhuge = cnt[1];
    for (uint32_t i = blockIdx.x; i < nhuge; i += gridDim.x) {
        const uint32_t q = lists[n_inst - 1 - i];
        const uint32_t c = ist[q], e = iend[c];
        Agg a;
        agg_clear(a);
        for (uint32_t p = c + threadIdx.x; p <= e; p += 1024) agg_add(a, sm[p]);
        a = agg_wave(a);
        if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = a;
        __syncthreads();
        if (threadIdx.x < 64) {
            Agg b;
            if (threadIdx.x < 16) b = part[threadIdx.x];
            else agg_clear(b);
            b = agg_wave(b);
            if (threadIdx.x == 0) aggs[q] = b;
        }
        __syncthreads();
    }
}

// ---- 6. records ----------------------------------------------------------------
struct RecArgs {
    const Batch* bs;
    int nb;
    int macs, mode_b;
    uint32_t n_inst;
    const Agg* aggs;            // by instance
    const uint32_t* ist;
    const ExMeta* sm;
    const uint32_t* iend;
    const uint8_t* ikind;
    const unsigned long long* ij;
    const unsigned long long* iie;
    const unsigned long long* iex;
    Glob* g;
    fluere_record* out;      // the run's records (appended)
    uint64_t out_cap;
    // Mode B: two order words beside each record (indexed like out): {0 for a
    // FIN/RST close, else the firing entry's exp + 1; its creation index}.
    // With order_key = the ending packet's index they give the reference's
    // emission order (by ending packet, FIN/RST before the sweep, sweeps by
    // (exp, push order); offline_fluereflows.rs:152-175); fetch_records sorts by them.
    unsigned long long* aux;
    const uint32_t* p_ninst; // the instance count on the device, or null (n_inst)
    uint32_t* defer;         // k_ex_records_t<false> -> <true>: instances for the general parser
    uint32_t* n_defer;       //   (their count, device)
    int shard_mode;
    const uint8_t* irole;
    const uint32_t* ikey;
    fluere_flow_annex* annex;
    const Seed* seeds;       // sharded Mode B: FluereRecord seed of each instance's creating packet
    // every instance one record (no annex pieces): instance q's record at
    // base0 + q (base0: the records before, known to the host), so no
    // workgroup takes a position with an atomic on the one record counter;
    // k_ex_records_t<true> adds the instances to it
    int fixed;
    uint64_t base0;
};

// fixed positions: the block's records [pos0, pos0 + EMIT_BLOCK), thread t's
// built in S.rec[t] (S.slot[t] = 1 when it is one: the slots of instances
// left to the general parser are skipped, the second kernel fills them),
// written out as coalesced 8-byte words
__device__ __forceinline__ void emit_fixed_block(EmitLds& S, fluere_record* out, uint64_t cap, bool live,
                                                 unsigned long long pos0) {
    S.slot[threadIdx.x] = live ? 1 : 0;
    __syncthreads();
    constexpr uint32_t RW = sizeof(fluere_record) / 8;
    const unsigned long long n = pos0 < cap ? min((unsigned long long)EMIT_BLOCK, cap - pos0) : 0ull;
    uint2* dst = reinterpret_cast<uint2*>(out + pos0);
    const uint2* src = reinterpret_cast<const uint2*>(S.rec);
    for (uint32_t i = threadIdx.x; i < n * RW; i += EMIT_BLOCK)
        if (S.slot[i / RW]) dst[i] = src[i];
    __syncthreads();
}

__device__ __forceinline__ void piece_of(const Agg& g, fluere_flow_piece& pc) {
    pc.pkts[0] = g.pk[0]; pc.pkts[1] = g.pk[1];
    pc.bytes[0] = g.by[0]; pc.bytes[1] = g.by[1];
    pc.min_pkt = g.mnp; pc.max_pkt = g.mxp; pc.min_ttl = g.mnt; pc.max_ttl = g.mxt;
    for (int k = 0; k < 8; k++) pc.flag_cnt[k] = g.fl[k];
    pc.last = g.lastg;
    pc.last_time = g.lastt;
}

// The creating packet's parse: the register parser alone in the fast
// kernel (P.cls = 2: the instance is listed for the general one).
template <bool GEN>
__device__ __forceinline__ void ex_parse(const RecArgs& a, uint64_t gi, Parsed& P) {
    if constexpr (GEN) parse_global(a.bs, a.nb, gi, a.macs != 0, P);
    else parse_global_fast(a.bs, a.nb, gi, a.macs != 0, P);
}

// Records (and, in shard mode, annex pieces) of the instances.  GEN false:
// instance q = the thread's index, the register parser only, instances whose
// creating packet it declines listed in a.defer; GEN true: the listed ones,
// with the general parser.  Each thread builds its record in place in the
// block's LDS staging (S.rec[thread]): held in registers, the record and the
// general parser took the kernel to 178 VGPRs (2 waves per SIMD).
template <bool GEN>
__global__ void __launch_bounds__(EMIT_BLOCK) k_ex_records_t(RecArgs a) {
    __shared__ EmitLds S;
    unsigned long long tot[2] = {0, 0};  // thread 0: the workgroup's updates / ended (one atomic pair at the end)
    unsigned long long upd = 0, ended = 0;  // fixed positions: this thread's
    const uint32_t n_inst = a.p_ninst ? *a.p_ninst : a.n_inst;
    const uint32_t n_items = GEN ? min(*a.n_defer, n_inst) : n_inst;
    if (GEN && a.fixed && blockIdx.x == 0 && threadIdx.x == 0) {  // every instance's record counted
        const unsigned long long nok = okey_count(okey_ref(a.g), a.out_cap, a.base0, n_inst);
        if (nok) atomicAdd(&a.g->n_okey, nok);
        atomicAdd(&a.g->n_rec, (unsigned long long)n_inst);
    }
    for (uint32_t i0 = blockIdx.x * blockDim.x; i0 < n_items; i0 += gridDim.x * blockDim.x) {  // (uniform)
        const uint32_t i = i0 + threadIdx.x;
        const bool lane_live = i < n_items;
        const uint32_t q = lane_live ? (GEN ? a.defer[i] : i) : 0u;  // instance (a run of the flow's packets)
        fluere_record& rec = S.rec[threadIdx.x];
        uint8_t kind = K_ACTIVE;
        unsigned long long cie = 0, cex = 0;
        bool defer = false, rec_live = false;
        const uint32_t c = lane_live ? a.ist[q] : 0u;
        const uint8_t role = (lane_live && a.shard_mode) ? a.irole[c] : (uint8_t)R_RECORD;
        if (lane_live && role != R_RECORD) {
            // a piece of the flow's annex (lead / head / tail), not a record:
            // built in this thread's (unused) record slot, then copied out
            const ExMeta mc = a.sm[c];
            fluere_flow_piece& pc = *reinterpret_cast<fluere_flow_piece*>(&S.rec[threadIdx.x]);
            Parsed P;
            if (role != R_LEAD) {
                ex_parse<GEN>(a, mc.gidx, P);
                defer = !GEN && P.cls == 2;
            }
            if (!defer) {
                memset(&pc, 0, sizeof pc);
                piece_of(a.aggs[q], pc);
                pc.first = mc.gidx;
                pc.first_time = mc.t;
                if (role != R_LEAD) {  // fill_seed's fields (device.h)
                    const PktInfo& pi = P.pi;
#pragma unroll
                    for (int k = 0; k < 4; k++)
#pragma unroll
                        for (int b = 0; b < 4; b++) {
                            pc.src[4 * k + b] = (uint8_t)(pi.rsip[k] >> (24 - 8 * b));
                            pc.dst[4 * k + b] = (uint8_t)(pi.rdip[k] >> (24 - 8 * b));
                        }
                    pc.v6 = pi.rv6; pc.prot = pi.rprot; pc.tos = pi.rtos; pc.dir = mc.dir;
                    pc.src_port = pi.rsp; pc.dst_port = pi.rdp;
                }
                fluere_flow_annex& ax = a.annex[a.ikey[c]];
                if (role == R_LEAD) ax.lead = pc;
                if (role == R_HEAD || role == R_HEAD_TAIL) ax.head = pc;
                if (role == R_TAIL) ax.tail = pc;
            }
        } else if (lane_live) {
            const ExMeta mc = a.sm[c];
            if (a.seeds) {  // sharded Mode B: the creating packet is on another shard
                const Seed sd = a.seeds[q];
                memset(&rec, 0, sizeof rec);
#pragma unroll
                for (int k = 0; k < 16; k++) { rec.source[k] = sd.src[k]; rec.destination[k] = sd.dst[k]; }
                rec.src_v6 = rec.dst_v6 = sd.v6;
                rec.prot = sd.prot; rec.tos = sd.tos; rec.src_port = sd.sp; rec.dst_port = sd.dp;
                rec.first = mc.t;
            } else {
                Parsed P;
                ex_parse<GEN>(a, mc.gidx, P);
                defer = !GEN && P.cls == 2;
                if (!defer) fill_seed(rec, P);
            }
            if (!defer) {
                rec_live = true;
                if (a.shard_mode)  // the flow's last processed packet among its in-shard records (live mode)
                    atomicMax(reinterpret_cast<unsigned long long*>(&a.annex[a.ikey[c]].mid_last),
                              (unsigned long long)a.aggs[q].lastg + 1);
                const Agg g = a.aggs[q];
                const bool o = mc.dir != 0;  // orientation of the creating packet (selects: no indexed copy of g)
                const uint32_t p0 = g.pk[0], p1 = g.pk[1];
                const unsigned long long b0 = g.by[0], b1 = g.by[1];
                rec.d_pkts = p0 + p1;
                rec.d_octets = b0 + b1;
                rec.out_pkts = o ? p1 : p0;
                rec.in_pkts = o ? p0 : p1;
                rec.out_bytes = o ? b1 : b0;
                rec.in_bytes = o ? b0 : b1;
                rec.min_pkt = g.mnp;
                rec.max_pkt = g.mxp;
                rec.min_ttl = (uint8_t)g.mnt;
                rec.max_ttl = (uint8_t)g.mxt;
                for (int k = 0; k < 8; k++) rec.cnt[k] = g.fl[k];
                rec.cnt[8] = 0;
                rec.last = g.lastt;
                kind = a.ikind[c];
                cie = a.iie[c];
                cex = a.iex[c];
                rec.order_key = kind == K_ACTIVE ? NONE64 : a.ij[c];
            }
        }
        if (!GEN) {  // instances for the general parser: listed (wave-aggregated append)
            const uint64_t dm = __ballot(defer);
            if (dm) {
                const uint32_t lead = __builtin_ctzll(dm);
                uint32_t b0 = 0;
                if ((uint32_t)(threadIdx.x & 63) == lead) b0 = atomicAdd(a.n_defer, (uint32_t)__popcll(dm));
                b0 = __shfl(b0, lead, 64);
                if (defer)
                    a.defer[b0 + __builtin_amdgcn_mbcnt_hi((uint32_t)(dm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)dm, 0u))] = q;
            }
        }
        if (a.fixed) {  // (uniform) the record at base0 + q
            const unsigned long long pos = a.base0 + q;
            if (rec_live) {
                const OkeyRef o = okey_ref(a.g);
                if (okey_count(o, a.out_cap, pos, 1)) o.p[pos] = rec.order_key;
                if (a.mode_b && a.aux && pos < a.out_cap)
                    *reinterpret_cast<ulonglong2*>(a.aux + 2 * pos) =
                        make_ulonglong2(kind == K_SWEEP ? cex + 1 : 0ull, kind == K_SWEEP ? cie : 0ull);
                upd += rec.d_pkts;
                ended += rec.order_key != NONE64 ? 1 : 0;
            }
            if (GEN) {  // (few: each thread its own record)
                if (rec_live && pos < a.out_cap) {
                    const uint2* src = reinterpret_cast<const uint2*>(&rec);
                    uint2* dst = reinterpret_cast<uint2*>(a.out + pos);
                    for (uint32_t k = 0; k < sizeof(fluere_record) / 8; k++) dst[k] = src[k];
                }
                __syncthreads();  // (S.rec[t] is rebuilt by the next item)
            } else {
                emit_fixed_block(S, a.out, a.out_cap, rec_live, a.base0 + i0);
            }
            continue;
        }
        // (uniform: every thread of the block emits)
        emit_inplace_block(S, a.g, a.out, a.out_cap, rec_live, rec_live ? rec.d_pkts : 0u,
                           rec_live && rec.order_key != NONE64, a.mode_b ? a.aux : nullptr,
                           kind == K_SWEEP ? cex + 1 : 0ull, kind == K_SWEEP ? cie : 0ull, tot);
    }
    if (a.fixed) {  // the workgroup's updates / ended: one atomic pair
        upd = wave_sum(upd);
        ended = wave_sum(ended);
        if ((threadIdx.x & 63) == 0) {
            S.w[threadIdx.x >> 6][1] = upd;
            S.w[threadIdx.x >> 6][2] = ended;
        }
        __syncthreads();
        if (threadIdx.x == 0)
            for (int k = 0; k < EMIT_BLOCK / 64; k++) {
                tot[0] += S.w[k][1];
                tot[1] += S.w[k][2];
            }
    }
    if (threadIdx.x == 0) {
        if (tot[0]) atomicAdd(&a.g->n_updates, tot[0]);
        if (tot[1]) atomicAdd(&a.g->n_ended, tot[1]);
    }
}

__global__ void __launch_bounds__(256) k_ex_seed_req(uint32_t n_inst, const uint32_t* ist, const ExMeta* sm,
                                                     unsigned long long* req, uint32_t* q) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n_inst) {
        req[i] = sm[ist[i]].gidx;
        q[i] = i;
    }
}

unsigned gridn(uint64_t n, unsigned b) { return (unsigned)std::max<uint64_t>(1, (n + b - 1) / b); }

struct MailSrc {
    const void* p[MAIL_MAX];
    int bytes[MAIL_MAX];
    int n;
};
// One wave: the values, then (after the wave's system-scope fence) seq.
__global__ void __launch_bounds__(64) k_mail(MailSrc a, HostMail* m, uint32_t seq) {
    const int l = threadIdx.x;
    if (l < a.n) {
        const int b = a.bytes[l];
        const unsigned long long v = b == 8 ? *static_cast<const unsigned long long*>(a.p[l])
                                     : b == 4 ? (unsigned long long)*static_cast<const uint32_t*>(a.p[l])
                                              : (unsigned long long)*static_cast<const uint8_t*>(a.p[l]);
        __hip_atomic_store(&m->v[l], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __threadfence_system();
    if (l == 0) __hip_atomic_store(&m->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

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

int mail_fetch(HostMail* m, hipStream_t s, int n, const void* const* src, const int* bytes, unsigned long long* out) {
    if (n < 0 || n > MAIL_MAX) return FLUERE_E_ARG;
    static const bool no_mail = getenv("FLUERE_NO_MAIL") != nullptr;  // diagnostics: the copy + sync path
    if (!m || no_mail) {  // no mailbox: one copy per value, then a stream sync
        for (int i = 0; i < n; i++) {
            out[i] = 0;
            HIPCHECK(hipMemcpyAsync(&out[i], src[i], bytes[i], hipMemcpyDeviceToHost, s));
        }
        HIPCHECK(hipStreamSynchronize(s));
        return FLUERE_OK;
    }
    MailSrc a{};
    a.n = n;
    for (int i = 0; i < n; i++) {
        a.p[i] = src[i];
        a.bytes[i] = bytes[i];
    }
    const uint32_t seq = ++m->host_seq ? m->host_seq : ++m->host_seq;  // never 0 (the initial value)
    k_mail<<<1, 64, 0, s>>>(a, m, seq);
    HIPCHECK(hipGetLastError());
    for (uint32_t spin = 1;; spin++) {
        if (__atomic_load_n(&m->seq, __ATOMIC_ACQUIRE) == seq) break;
        if ((spin & 65535) == 0) {  // now and then (~ms): did the stream fail instead?
            const hipError_t q = hipStreamQuery(s);
            if (q == hipErrorNotReady) continue;
            if (__atomic_load_n(&m->seq, __ATOMIC_ACQUIRE) == seq) break;
            HIPCHECK(q);
            return FLUERE_E_HIP;  // the stream finished without writing seq: cannot happen
        }
    }
    for (int i = 0; i < n; i++) out[i] = __atomic_load_n(&m->v[i], __ATOMIC_RELAXED);
    return FLUERE_OK;
}

// One exact run, in phases (exact.h): the arena views and the host state
// between them.
struct ExactSession {
    ExactJob J;
    hipStream_t s;
    ExactResult R;
    uint64_t N = 0, n = 0;
    uint32_t n_keys = 0, n_inst = 0;
    bool mono = true;
    size_t tmp = 0;
    void* tp = nullptr;
    ExMeta *cm, *sm;
    const unsigned long long* ct = nullptr;  // or null: the replayed packets' times alone (capture order; J.dense_t)
    uint32_t *key, *skey;
    unsigned long long *re, *rf, *ne_rev, *nf_rev, *npr, *np_rev, *ej, *ij, *iie, *iex;
    unsigned long long *hi2, *tree;
    uint64_t tree_P = 0;
    uint32_t *val, *sval, *hf, *hpos, *heads, *link, *plink, *sflag, *iend, *incl, *ist, *alist, *ctr, *tbl;
    uint32_t *idx, *ikey;
    uint8_t *pr, *ikind, *irole;
    uint8_t* prp;  // the processed flags by sorted position (k_ex_members' own copy of pr)
    uint8_t *stamp, *kpass, *kdirty;
    uint32_t *elook, *ekp;
    uint32_t pass_no = 0;
    Agg* aggs;
    fluere_flow_annex* annex = nullptr;
    ChaseArgs ca;
};

void exact_free(ExactSession* S) { delete S; }

// The replayed packets' stable sort by flow (32-bit keys of at most end_bit
// bits, 32-bit values).  FLUERE_SORT_BITS > 0: rocprim's onesweep with that
// many bits a pass (10: two passes for up to 20-bit flow ids, where the
// gfx950 default of 8 takes three); 0: the library default.  The bits are
// the run's flow count's (ExactJob::key_bound), not the table capacity's.
#ifndef FLUERE_SORT_BITS
#define FLUERE_SORT_BITS 10  // (tcp_t1, 20-bit flow ids: 8 bits 3 passes ~300 us, 10 bits 2 passes ~254 us, 11 bits ~271 us)
#endif
static hipError_t sort_by_flow(void* tmp, size_t& tb, const uint32_t* key, uint32_t* skey, const uint32_t* val,
                               uint32_t* sval, int n, int end_bit, hipStream_t s) {
#if FLUERE_SORT_BITS > 0
    using OS = rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 16>, rocprim::kernel_config<1024, 16>,
                                                   FLUERE_SORT_BITS, rocprim::block_radix_rank_algorithm::match>;
    using Cfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, OS>;
    return rocprim::radix_sort_pairs<Cfg>(tmp, tb, key, skey, val, sval, (size_t)n, 0u, (unsigned)end_bit, s);
#else
    return prim_sort_pairs(tmp, tb, key, skey, val, sval, n, 0, end_bit, s);
#endif
}

// The arena exact_begin lays out for a job: phase 1 over every packet, phase
// 2 over at most every packet, and the rocPRIM temp storage at that size.
static size_t arena_bytes_calc(const ExactJob& J, uint64_t N, hipStream_t s, size_t* tmp_out);
// (the library's temp-size queries cost the host ~10 us a run, between the
// pass and the engine's first launch: the last sizes are kept)
static size_t arena_bytes(const ExactJob& J, uint64_t N, hipStream_t s, size_t* tmp_out) {
    struct Memo {
        uint64_t N;
        int nb, mode_b;
        size_t need, tmp;
    };
    static thread_local Memo memo = {~0ull, 0, 0, 0, 0};
    if (memo.N != N || memo.nb != J.nb || memo.mode_b != J.mode_b) {
        size_t t = 0;
        const size_t need = arena_bytes_calc(J, N, s, &t);
        memo = Memo{N, J.nb, J.mode_b, need, t};
    }
    if (tmp_out) *tmp_out = memo.tmp;
    return memo.need;
}
static size_t arena_bytes_calc(const ExactJob& J, uint64_t N, hipStream_t s, size_t* tmp_out) {
    const uint64_t P = J.mode_b ? tree_leaves(N) : 1;
    // ---- arena sizing: phase 1 (all packets) + phase 2 (replayed packets, at most N)
    auto bytes_for = [&](uint64_t n_all, uint64_t n, size_t tmp) {
        size_t b = 0;
        auto add = [&](size_t x) { b += ((x + 255) & ~(size_t)255) + 256; };
        add((n_all + EXM_PKTS * (size_t)J.nb) * sizeof(ExMeta));     // meta_blk (k_ex_meta's block regions)
        add(4 * (n_all / 256 + J.nb + 1)); add(4 * (n_all / 256 + J.nb + 1));  // bcount, bpos
        add(n * sizeof(ExMeta)); add(n * 4); add(n * 4);              // cm, key, val
        add(n * 4); add(n * 4); add(n * sizeof(ExMeta));              // skey, sval, sm
        add(n * 4); add(n * 4); add(n * 4);                           // hf, hpos, heads
        add(n * 8); add(n * 8); add(n * 8); add(n * 8);               // re, rf, ne_rev, nf_rev
        add(n); add(n * 8); add(n * 8); add(n * 8); add(n * 4);       // pr, npr, np_rev, ej, link
        add(n * 4);                                                   // plink
        add(n * 4); add(n * 4); add(n); add(n * 8); add(n * 8);       // sflag, iend, ikind, ij, iie
        add(n * 8);                                                   // iex
        add(n * 4); add(n * 4); add(n * 4);                           // incl, ist, alist
        add(n * sizeof(Agg)); add(16);                                // aggs, nruns/counters
        add(n * 4); add(n * 8);                                       // idx, hi2 (seed requests)
        add(n); add(n * 4);                                           // irole, ikey
        add(n);                                                       // prp
        add(n); add(n); add(n); add(n * 4); add(n * 4);               // stamp, kpass, kdirty, elook, ekp
        if (J.mode_b) add(2 * P * 8);                                 // tree
        add((n / 16 + 4) * 4);                                        // tbl
        add(tmp);
        return b;
    };
    // rocPRIM temp storage: the largest of the primitives at size N
    size_t tmp = 0, t = 0;
    {
        const int n = (int)N;
        (void)prim_exclusive_sum(nullptr, t, (uint32_t*)nullptr, (uint32_t*)nullptr, n, s); tmp = std::max(tmp, t);
        (void)prim_inclusive_sum(nullptr, t, (uint32_t*)nullptr, (uint32_t*)nullptr, n, s); tmp = std::max(tmp, t);
        (void)prim_sort_pairs(nullptr, t, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                           (uint32_t*)nullptr, (uint32_t*)nullptr, n, 0, 64, s);
        tmp = std::max(tmp, t);
        (void)prim_sort_pairs(nullptr, t, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                           (uint32_t*)nullptr, (uint32_t*)nullptr, n, 0, 32, s);
        tmp = std::max(tmp, t);
        (void)sort_by_flow(nullptr, t, nullptr, nullptr, nullptr, nullptr, n, 32, s);
        tmp = std::max(tmp, t);
        (void)prim_inclusive_min(nullptr, t, (unsigned long long*)nullptr, (unsigned long long*)nullptr, n, s);
        tmp = std::max(tmp, t);
        (void)prim_inclusive_max(nullptr, t, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                                n / 16 + 2, s);
        tmp = std::max(tmp, t);
    }
    if (tmp_out) *tmp_out = tmp;
    return bytes_for(N, N, tmp);
}

static uint64_t job_packets(const ExactJob& J) {
    uint64_t N = 0;
    if (J.ext_cm) N = J.ext_n;
    else
        for (int b = 0; b < J.nb; b++) N += J.h_batches[b].n;
    return N;
}

int exact_reserve(const ExactJob& J, hipStream_t s) {
    const uint64_t N = job_packets(J);
    if (!N) return FLUERE_OK;
    const size_t need = arena_bytes(J, N, s, nullptr);
    if (need <= *J.scratch_bytes) return FLUERE_OK;
    if (*J.scratch) {  // (the old arena may still be in use: hipFree waits for the device)
        hipFree(*J.scratch);
        *J.scratch = nullptr;
        *J.scratch_bytes = 0;
    }
    if (hipMalloc(J.scratch, need) != hipSuccess) return FLUERE_E_NOMEM;
    *J.scratch_bytes = need;
    return FLUERE_OK;
}

int exact_begin(const ExactJob& J, hipStream_t s, ExactSession** out) {
    *out = nullptr;
    const uint64_t N = job_packets(J);
    ExactSession* S = new (std::nothrow) ExactSession();
    if (!S) return FLUERE_E_NOMEM;
    S->J = J;
    S->s = s;
    S->N = N;
    *out = S;
    if (!N) return FLUERE_OK;
    const uint64_t P = J.mode_b ? tree_leaves(N) : 1;
    size_t tmp = 0;
    const size_t need = arena_bytes(J, N, s, &tmp);
    S->tmp = tmp;
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
    uint64_t nblk = 0;  // k_ex_meta blocks over every batch
    if (!J.ext_cm)
        for (int b = 0; b < J.nb; b++) nblk += J.h_batches[b].n ? gridn(J.h_batches[b].n, EXM_PKTS) : 0;
    ExMeta* meta = A.take<ExMeta>(nblk * EXM_PKTS);
    uint32_t* bcount = A.take<uint32_t>(nblk + 1);
    uint32_t* bpos = A.take<uint32_t>(nblk + 1);
    // ---- 1. metadata of every packet to replay, compacted in capture order
    if (!J.ext_cm && !J.dense_cm) {
        uint64_t blk = 0;
        for (int b = 0; b < J.nb; b++) {
            const Batch& B = J.h_batches[b];
            if (!B.n) continue;
            const uint32_t* ph = J.phash && (!J.mode_b || J.emap) ? J.phash + (B.first - J.phash_base) : nullptr;
            const ExMeta* hm = ph && J.emap && J.hot_meta ? J.hot_meta + (B.first - J.phash_base) : nullptr;
            k_ex_meta<<<gridn(B.n, EXM_PKTS), 256, 0, s>>>(B, J.T, J.macs, J.mode_b, J.complex, J.cbits, meta, bcount, blk, ph,
                                                           J.emap, hm);
            blk += gridn(B.n, EXM_PKTS);
        }
    }
    size_t tb = tmp;
    ExMeta* cm = S->cm = A.take<ExMeta>(N);
    uint32_t* key = S->key = A.take<uint32_t>(N);
    uint32_t* val = S->val = A.take<uint32_t>(N);
    uint32_t* skey = S->skey = A.take<uint32_t>(N);
    uint32_t* sval = S->sval = A.take<uint32_t>(N);
    ExMeta* sm = S->sm = A.take<ExMeta>(N);
    uint32_t* hf = S->hf = A.take<uint32_t>(N);
    uint32_t* hpos = S->hpos = A.take<uint32_t>(N);
    uint32_t* heads = S->heads = A.take<uint32_t>(N);
    unsigned long long* re = S->re = A.take<unsigned long long>(N);
    unsigned long long* rf = S->rf = A.take<unsigned long long>(N);
    unsigned long long* ne_rev = S->ne_rev = A.take<unsigned long long>(N);
    unsigned long long* nf_rev = S->nf_rev = A.take<unsigned long long>(N);
    uint8_t* pr = S->pr = A.take<uint8_t>(N);
    S->npr = A.take<unsigned long long>(N);
    S->np_rev = A.take<unsigned long long>(N);
    S->ej = A.take<unsigned long long>(N);
    S->link = A.take<uint32_t>(N);
    S->plink = A.take<uint32_t>(N);
    S->stamp = A.take<uint8_t>(N);
    S->kpass = A.take<uint8_t>(N);
    S->kdirty = A.take<uint8_t>(N);
    S->elook = A.take<uint32_t>(N);
    S->ekp = A.take<uint32_t>(N);
    S->sflag = A.take<uint32_t>(N);
    S->iend = A.take<uint32_t>(N);
    S->ikind = A.take<uint8_t>(N);
    S->ij = A.take<unsigned long long>(N);
    S->iie = A.take<unsigned long long>(N);
    S->iex = A.take<unsigned long long>(N);
    S->incl = A.take<uint32_t>(N);
    S->ist = A.take<uint32_t>(N);
    S->alist = A.take<uint32_t>(N);
    S->aggs = A.take<Agg>(N);
    uint32_t* ctr = S->ctr = A.take<uint32_t>(4);  // [0..1] aggregate lists, [1] non-monotonic (begin), [2] changed, [3] deferred records
    S->idx = A.take<uint32_t>(N);
    S->hi2 = A.take<unsigned long long>(N);
    S->irole = A.take<uint8_t>(N);
    S->ikey = A.take<uint32_t>(N);
    S->prp = A.take<uint8_t>(N);
    S->tree = J.mode_b ? A.take<unsigned long long>(2 * P) : nullptr;
    S->tbl = A.take<uint32_t>(N / 16 + 4);
    S->tree_P = P;
    void* tp = S->tp = A.take<char>(tmp);
    uint64_t n;
    if (J.ext_cm) {  // sharded Mode B owner: the shards' packets, already in capture order
        n = N;
        HIPCHECK(hipMemcpyAsync(cm, J.ext_cm, n * sizeof(ExMeta), hipMemcpyDeviceToDevice, s));
        k_ex_keys<<<gridn(n, 256), 256, 0, s>>>(n, cm, key, val);
    } else if (J.dense_cm) {  // one GPU, Mode B: the hot pass's metadata, every packet
        n = N;
        cm = S->cm = const_cast<ExMeta*>(J.dense_cm);
        S->ct = J.dense_t;
        // (no counter to clear before it: k_ex_tscan / k_ex_mono count the misses)
        k_ex_pidkeys<<<gridn(n, 256), 256, 0, s>>>(n, J.phash + (J.h_batches[0].first - J.phash_base), J.emap,
                                                   J.T.fmax, key, val, nullptr);
    } else {
        HIPCHECK(prim_exclusive_sum(tp, tb, bcount, bpos, (int)nblk, s));
        unsigned long long last[2] = {0, 0};
        const void* src[2] = {bpos + nblk - 1, bcount + nblk - 1};
        const int by[2] = {4, 4};
        int rc = mail_fetch(J.mail, s, 2, src, by, last);
        if (rc) return rc;
        n = last[0] + last[1];
        if (n) k_ex_compact<<<(unsigned)nblk, 256, 0, s>>>(meta, bcount, bpos, cm, key, val);
    }
    S->n = n;
    S->R.replayed = n;
    if (!n) return FLUERE_OK;
    const int in = (int)n;
    // ---- 2. sort by (key, index): a stable sort by key of the capture-order
    // packets (LSD radix: ceil(log2 fmax) bits, not key + index); key heads;
    // next eligible / FIN-RST
    int end_bit = 1;
    const uint64_t kb = J.key_bound ? std::min<uint64_t>(J.key_bound, J.T.fmax) : J.T.fmax;
    while (end_bit < 32 && (1ull << end_bit) < kb) end_bit++;
    tb = tmp;
    HIPCHECK(sort_by_flow(tp, tb, key, skey, val, sval, in, end_bit, s));
    // (re's space holds the sorted packets' flag bytes, rf's the scan's tile minima)
    k_ex_gather<<<gridn(n, 256 * GATHER_ITEMS), 256, 0, s>>>(n, skey, sval, cm, sm, hf, reinterpret_cast<uint8_t*>(re),
                                                                J.mode_b ? S->prp : nullptr);
    {
        int rc = next_scan(s, n, skey, reinterpret_cast<const uint8_t*>(re), 1u, 2u, 2, ne_rev, nf_rev, rf);
        if (rc) return rc;
    }
    {  // key positions and heads (rf: the tile totals, after next_scan's use)
        int rc = fc_run(s, n, hf, hpos, false, heads, rf);
        if (rc) return rc;
    }
    // Mode B: monotonicity and the time-bucket index in one pass (a max-scan
    // of range starts, no binary searches); small runs: the two kernels
    const uint64_t nb_dev = n / 16 + 1;
    const bool tscan = J.mode_b && n >= 64;
    {   // the counters, the range starts, the first guess of the processed set
        // (every valid packet; k_ex_gather set prp): one launch
        Fills f;
        f.add(ctr, 16, 0);
        if (tscan) f.add(S->idx, (nb_dev + 1) * 4, 0);
        if (J.mode_b) f.add(pr, n, 1);
        HIPCHECK(fill_many(f, s));
    }
    if (tscan) {
        uint32_t* starts = S->idx;  // (free until the seed requests; n >= nb + 1)
        k_ex_tscan<<<gridn(n, 256), 256, 0, s>>>(n, cm, S->ct, nb_dev, starts, ctr + 1, J.dense_cm ? key : nullptr,
                                                 ctr + 2);
        tb = tmp;
        HIPCHECK(prim_inclusive_max(tp, tb, starts, S->tbl, (int)(nb_dev + 1), s));
    } else if (J.mode_b) {
        k_ex_mono<<<gridn(n, 256), 256, 0, s>>>(n, cm, ctr + 1, J.dense_cm ? key : nullptr, ctr + 2);
    }
    // one host read: key count, monotonicity, the first and last times.  Mode
    // A (not shard mode) needs none of them on the host: the key count stays
    // on the device and the chase's grid covers the replayed packets (every
    // host round trip leaves the GPU idle for ~50-60 us: the wait, then the
    // next submission on an idle queue)
    unsigned long long hv[6] = {0, 0, 0, 0, 0, 0};
    const bool dev_keys = !J.mode_b && !J.shard_mode;
    if (dev_keys) {
        k_ex_nkeys<<<1, 64, 0, s>>>(hpos + n - 1, hf + n - 1, ctr + 3);
    } else {
        const void* src[6] = {hpos + n - 1, hf + n - 1, ctr + 1, &cm[0].t, &cm[n - 1].t, ctr + 2};  // (ctr[2]: dense misses)
        const int by[6] = {4, 4, 4, 8, 8, 4};
        int rc = mail_fetch(J.mail, s, J.mode_b ? (J.dense_cm ? 6 : 5) : 2, src, by, hv);
        if (rc) return rc;
        if (J.dense_cm && hv[5]) return EXACT_DENSE_MISS;  // a packet without a flow word: the k_ex_meta path
    }
    S->n_keys = (uint32_t)(hv[0] + hv[1]);
    S->R.keys = S->n_keys;
    S->mono = !hv[2];
    if (J.shard_mode) {
        if (S->n_keys > *J.annex_cap) {
            hipFree(*J.annex);
            *J.annex = nullptr;
            *J.annex_cap = 0;
            if (hipMalloc(J.annex, (size_t)S->n_keys * sizeof(fluere_flow_annex)) != hipSuccess) return FLUERE_E_NOMEM;
            *J.annex_cap = S->n_keys;
        }
        S->annex = *J.annex;
        S->R.annexes = S->n_keys;
    }
    // the time-bucket index of the non-decreasing times (about 16 packets a
    // bucket): a sweep point's lower_bound searches one bucket, not the capture
    uint64_t t0 = 0, bw = 1, nb = 0;
    if (J.mode_b && S->mono) {
        const unsigned long long tt[2] = {hv[3], hv[4]};
        t0 = tt[0];
        nb = nb_dev;
        bw = std::max<uint64_t>(1, (tt[1] - tt[0]) / nb + 1);  // nb * bw > the span (k_ex_tscan's buckets)
        if (!tscan) k_ex_tindex<<<gridn(nb + 1, 256), 256, 0, s>>>(n, cm, t0, bw, nb, S->tbl);
        HIPCHECK(hipGetLastError());
    }
    S->ca = ChaseArgs{n, S->n_keys, heads, sm, sval, ne_rev, nf_rev, J.mode_b, J.timeout_us, cm, S->np_rev,
                      (J.mode_b && !S->mono) ? S->tree : nullptr, P, S->tbl, t0, bw, nb, nullptr,
                      S->sflag, S->iend, S->ikind, S->ij, S->iie, S->iex, S->ej, S->link, S->plink,
                      J.shard_mode, S->irole, S->ikey, S->annex, J.annex_of, J.T.flow_key};
    if (dev_keys) S->ca.d_nkeys = ctr + 3;  // (ctr[3] is the records' defer count only after the chase)
    S->ca.ct = S->ct;
    return FLUERE_OK;
}

uint64_t exact_replayed(const ExactSession* S) { return S ? S->n : 0; }

int exact_pass(ExactSession* S, const unsigned long long* fext, uint8_t* pr_out, bool* changed) {
    const ExactJob& J = S->J;
    hipStream_t s = S->s;
    const uint64_t n = S->n;
    if (changed) *changed = false;
    if (!n) return FLUERE_OK;
    S->R.iterations++;
    S->ca.fext = fext;
    // the first pass guesses every replayed packet processed (exact_begin's
    // fill of pr): the next processed packet at or after k is k, no scan
    S->ca.np_all = J.mode_b && !fext && S->mono && S->pass_no == 0 && !pr_out ? 1 : 0;
    if (J.mode_b && !fext && !S->ca.np_all) {  // the sweep-point index over this pass's processed packets
        if (S->mono) {
            int rc = next_scan(s, n, nullptr, S->pr, 0xFFu, 0u, 1, S->np_rev, nullptr, S->npr);
            if (rc) return rc;
        } else {
            int rc = tree_build(n, S->cm, S->pr, S->tree, S->tree_P, s);
            if (rc) return rc;
        }
    }
    // incremental passes: non-decreasing times, the sweep points of this GPU
    static const bool no_inc = getenv("FLUERE_EXACT_NO_INC") != nullptr;  // (A/B)
    const bool inc = J.mode_b && !fext && !J.shard_mode && !no_inc;
    const uint32_t pid = ++S->pass_no;
    // this pass's fills in one launch: the changed counter k_ex_members counts
    // into, and the stamps (first pass), the dirty keys, or the start flags
    Fills fills;
    fills.add(S->ctr + 2, 4, 0);
    if (inc && pid < 255) fills.add(pid == 1 ? (void*)S->stamp : (void*)S->kdirty, pid == 1 ? n : S->n_keys, 0);
    else fills.add(S->sflag, n * 4, 0);
    HIPCHECK(fill_many(fills, s));
    if (inc && pid < 255) {
        if (pid == 1) {
            S->ca.kdirty = nullptr;
        } else {
            k_ex_check<<<gridn(n, 256), 256, 0, s>>>(n, S->sflag, S->elook, S->ekp, S->np_rev, S->hf, S->hpos, S->kdirty,
                                                     S->mono ? nullptr : S->tree, S->tree_P, S->sm, J.timeout_us);
            S->ca.kdirty = S->kdirty;
        }
        S->ca.stamp = S->stamp;
        S->ca.kpass = S->kpass;
        S->ca.elook = S->elook;
        S->ca.ekp = S->ekp;
        S->ca.pass_id = pid;
        k_ex_chase<<<gridn(S->ca.d_nkeys ? n : S->n_keys, 64), 64, 0, s>>>(S->ca);
        k_ex_flags<<<gridn(n, 256), 256, 0, s>>>(n, S->stamp, S->kpass, S->hf, S->hpos, S->sflag);
    } else {
        S->ca.stamp = nullptr;
        S->ca.kpass = nullptr;
        S->ca.kdirty = nullptr;
        S->ca.elook = S->ca.ekp = nullptr;
        k_ex_chase<<<gridn(S->ca.d_nkeys ? n : S->n_keys, 64), 64, 0, s>>>(S->ca);
    }
    {  // instance ordinals and starts (npr: the tile totals, after next_scan's use)
        int rc = fc_run(s, n, S->sflag, S->incl, true, S->ist, S->npr);
        if (rc) return rc;
    }
    if (J.mode_b)  // the processed set (Mode A needs none: every run is a record or a piece)
        k_ex_members<<<gridn(n, 256), 256, 0, s>>>(n, S->incl, S->ist, S->iend, S->sval, S->pr, S->prp, S->ctr + 2);
    HIPCHECK(hipGetLastError());
    if (pr_out) HIPCHECK(hipMemcpyAsync(pr_out, S->pr, n, hipMemcpyDeviceToDevice, s));
    if (!J.mode_b) return FLUERE_OK;
    unsigned long long ch = 0;
    const void* src[1] = {S->ctr + 2};
    const int by[1] = {4};
    int rc = mail_fetch(J.mail, s, 1, src, by, &ch);
    if (rc) return rc;
    if (changed) *changed = ch != 0;
    return FLUERE_OK;
}

int exact_seed_requests(ExactSession* S, unsigned long long* req, uint32_t* q, uint32_t* n_inst) {
    hipStream_t s = S->s;
    *n_inst = 0;
    if (!S->n) return FLUERE_OK;
    uint32_t ni = 0;
    HIPCHECK(hipMemcpyAsync(&ni, S->incl + S->n - 1, 4, hipMemcpyDeviceToHost, s));
    HIPCHECK(hipStreamSynchronize(s));
    S->n_inst = ni;
    if (ni) {
        // (creation index, instance) sorted by index: grouped by holder shard
        k_ex_seed_req<<<gridn(ni, 256), 256, 0, s>>>(ni, S->ist, S->sm, S->hi2, S->idx);
        size_t tb = S->tmp;
        HIPCHECK(prim_sort_pairs(S->tp, tb, S->hi2, req, S->idx, q, (int)ni, 0, 64, s));
    }
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(s));
    *n_inst = ni;
    return FLUERE_OK;
}

int exact_finish(ExactSession* S, const Seed* seeds, unsigned long long* aux_out) {
    const ExactJob& J = S->J;
    hipStream_t s = S->s;
    const uint64_t n = S->n;
    if (!n) return FLUERE_OK;
    // the instance count and the records already emitted: one host read, or
    // (Mode A with the record count known to the caller) none -- the
    // kernels read the count on the device and their grids cover n
    unsigned long long hv[2] = {0, 0};
    // (the record buffer is grown to the bound, kept below 4 GiB of HBM)
    const bool dev_inst = !J.mode_b && !J.shard_mode && !seeds && !aux_out && J.n_rec_known != ~0ull &&
                          (J.n_rec_known + n <= *J.d_recs_cap ||
                           (J.n_rec_known + n) * sizeof(fluere_record) <= (4ull << 30));
    const uint32_t* p_ninst = dev_inst ? S->incl + n - 1 : nullptr;
    if (dev_inst) {
        hv[0] = n;  // (an upper bound: every instance holds a packet)
        hv[1] = J.n_rec_known;
    } else {
        const void* src[2] = {S->incl + n - 1, reinterpret_cast<const char*>(J.g) + offsetof(Glob, n_rec)};
        const int by[2] = {4, 8};
        int rc = mail_fetch(J.mail, s, 2, src, by, hv);
        if (rc) return rc;
    }
    const uint32_t n_inst = (uint32_t)hv[0];
    const uint64_t n_rec0 = hv[1];
    // ---- 7a. the record buffer and (Mode B) the order words: grown first,
    // so that the counters and the order words are cleared in one launch
    const uint64_t want = n_rec0 + n_inst;
    if (want > *J.d_recs_cap) {  // grow, keeping the records already there
        fluere_record* nr = nullptr;
        if (hipMalloc(&nr, want * sizeof(fluere_record)) != hipSuccess) return FLUERE_E_NOMEM;
        if (n_rec0)
            HIPCHECK(hipMemcpyAsync(nr, *J.d_recs, n_rec0 * sizeof(fluere_record), hipMemcpyDeviceToDevice, s));
        HIPCHECK(hipStreamSynchronize(s));
        hipFree(*J.d_recs);
        *J.d_recs = nr;
        *J.d_recs_cap = want;
    }
    // Mode B: the order words beside the records (indexed like them); the
    // caller's aux_out is the slot of record n_rec0
    unsigned long long* aux = nullptr;
    Fills fills;
    fills.add(S->ctr, 16, 0);  // aggregate lists [0..1], the records' defer count [3]
    if (J.mode_b) {
        if (aux_out) {
            aux = aux_out - 2 * n_rec0;
        } else {
            if (!J.recaux || !J.recaux_cap) return FLUERE_E_ARG;
            if (want > *J.recaux_cap) {
                HIPCHECK(hipStreamSynchronize(s));  // (the old buffer may still be in use)
                hipFree(*J.recaux);
                *J.recaux = nullptr;
                *J.recaux_cap = 0;
                if (hipMalloc(J.recaux, std::max<uint64_t>(want, 1) * 16) != hipSuccess) return FLUERE_E_NOMEM;
                *J.recaux_cap = std::max<uint64_t>(want, 1);
            }
            fills.add(*J.recaux, n_rec0 * 16, 0);
            aux = *J.recaux;
        }
    }
    HIPCHECK(fill_many(fills, s));
    // ---- 6. per-instance aggregates over each instance's contiguous run
    if (n_inst) {
        k_ex_agg<<<gridn(n_inst, 256), 256, 0, s>>>(n_inst, S->ist, S->iend, S->sm, S->aggs, S->alist, S->ctr, p_ninst);
        k_ex_agg_wave<<<1024, 256, 0, s>>>(n_inst, S->ist, S->iend, S->sm, S->aggs, S->alist, S->ctr, p_ninst);
        k_ex_agg_block<<<256, 1024, 0, s>>>(n_inst, S->ist, S->iend, S->sm, S->aggs, S->alist, S->ctr, p_ninst);
    }
    HIPCHECK(hipGetLastError());
    S->R.instances = dev_inst ? 0 : n_inst;
    // ---- 7. records
    RecArgs ra{J.d_batches, J.nb, J.macs, J.mode_b, n_inst, S->aggs, S->ist, S->sm, S->iend, S->ikind,
               S->ij, S->iie, S->iex, J.g, *J.d_recs, *J.d_recs_cap, aux, p_ninst, S->idx, S->ctr + 3,
               J.shard_mode, S->irole, S->ikey, S->annex, seeds};
    {
        const char* e = getenv("FLUERE_REC_FIXED");  // (A/B)
        ra.fixed = !J.shard_mode && !(e && atoi(e) == 0);
        ra.base0 = n_rec0;
    }
    // runs <= n (every run holds a packet); records appended per block, Mode B
    // with their order words (fetch_records orders them: no device sort).
    // The instances whose creating packet needs the general parser are listed
    // by the first kernel and done by the second (grid-stride over the count).
    if (n_inst) {
        static const unsigned rec_wgs = getenv("FLUERE_REC_WGS") ? (unsigned)std::max(1, atoi(getenv("FLUERE_REC_WGS"))) : 1024u;  // (A/B)
        k_ex_records_t<false><<<std::min<unsigned>(gridn(n_inst, 256), rec_wgs), 256, 0, s>>>(ra);
        k_ex_records_t<true><<<std::min<unsigned>(gridn(n_inst, 256), 64), 256, 0, s>>>(ra);
    }
    HIPCHECK(hipGetLastError());
    // (every caller reads the run counters back with a stream-ordered copy)
    return FLUERE_OK;
}

const ExactResult& exact_result(const ExactSession* S) { return S->R; }

int exact_collect(const ExactJob& J, hipStream_t s, ExMeta* cm, uint64_t* n_out) {
    *n_out = 0;
    uint64_t nblk = 0;
    for (int b = 0; b < J.nb; b++) nblk += J.h_batches[b].n ? gridn(J.h_batches[b].n, EXM_PKTS) : 0;
    if (!nblk) return FLUERE_OK;
    ExMeta* meta = nullptr;
    uint32_t *bcount = nullptr, *bpos = nullptr;
    uint32_t* key = nullptr;
    uint32_t* val = nullptr;
    void* tp = nullptr;
    size_t tb = 0;
    (void)prim_exclusive_sum(nullptr, tb, bcount, bpos, (int)nblk, s);
    int rc = FLUERE_OK;
    const uint64_t N = nblk * EXM_PKTS;
    if (hipMalloc(&meta, N * sizeof(ExMeta)) != hipSuccess || hipMalloc(&bcount, nblk * 4) != hipSuccess ||
        hipMalloc(&bpos, nblk * 4) != hipSuccess || hipMalloc(&key, N * 4) != hipSuccess ||
        hipMalloc(&val, N * 4) != hipSuccess || hipMalloc(&tp, std::max<size_t>(tb, 16)) != hipSuccess)
        rc = FLUERE_E_NOMEM;
    if (rc == FLUERE_OK) {
        uint64_t blk = 0;
        for (int b = 0; b < J.nb; b++) {
            const Batch& B = J.h_batches[b];
            if (!B.n) continue;
            k_ex_meta<<<gridn(B.n, EXM_PKTS), 256, 0, s>>>(B, J.T, J.macs, 1, nullptr, nullptr, meta, bcount, blk, nullptr,
                                                           nullptr, nullptr);
            blk += gridn(B.n, EXM_PKTS);
        }
        unsigned long long last[2] = {0, 0};
        const void* src[2] = {bpos + nblk - 1, bcount + nblk - 1};
        const int by[2] = {4, 4};
        if (prim_exclusive_sum(tp, tb, bcount, bpos, (int)nblk, s) != hipSuccess ||
            mail_fetch(J.mail, s, 2, src, by, last) != FLUERE_OK)
            rc = FLUERE_E_HIP;
        else {
            k_ex_compact<<<(unsigned)nblk, 256, 0, s>>>(meta, bcount, bpos, cm, key, val);
            if (hipGetLastError() != hipSuccess || hipStreamSynchronize(s) != hipSuccess) rc = FLUERE_E_HIP;
            *n_out = last[0] + last[1];
        }
    }
    hipFree(meta); hipFree(bcount); hipFree(bpos); hipFree(key); hipFree(val); hipFree(tp);
    return rc;
}

int exact_run(const ExactJob& J, hipStream_t s, ExactResult* res) {
    ExactSession* S = nullptr;
    int rc = exact_begin(J, s, &S);
    if (rc == EXACT_DENSE_MISS) {
        exact_free(S);
        S = nullptr;
        ExactJob J2 = J;
        J2.dense_cm = nullptr;
        rc = exact_begin(J2, s, &S);
    }
    for (int pass = 0; rc == FLUERE_OK && S->n; pass++) {
        if (pass == MAX_PASSES) {
            rc = EXACT_FALLBACK;
            break;
        }
        bool changed = false;
        rc = exact_pass(S, nullptr, nullptr, &changed);
        if (!J.mode_b || !changed) break;
    }
    if (rc == FLUERE_OK && S->n) rc = exact_finish(S, nullptr, nullptr);
    if (res && S) *res = S->R;
    exact_free(S);
    return rc;
}

int flag_count(hipStream_t s, uint64_t n, const uint32_t* flags, uint32_t* out, bool inclusive, uint32_t* list,
               void* tmp) {
    return fc_run(s, n, flags, out, inclusive, list, tmp);
}

}  // namespace fl
