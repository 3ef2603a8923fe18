// order.hip -- the ended records in the reference's order, on the device.
#include "ctx.h"

// ---------------------------------------------------------------------------
// Ended-record order on the device, inside the run.  The reference appends a
// record when its flow ends, in packet order (offline_fluereflows.rs:155,171,
// inside the "Converted in" window :49-178), and its active flows after the
// loop (:182-191) in HashMap order.  The run's records leave as [ended, in
// the reference's order][active, any order]:
//  * Mode A: an ended record's order_key (its closing packet's index) is
//    unique -- a packet closes at most one instance of its key -- so its
//    place is the count of ended keys below it: one bit per packet, a
//    popcount scan, one scatter (of every record, or -- at most a quarter
//    ended -- of the ended ones and the actives they displace: k_ord_out);
//  * Mode B: a sweep ends several flows at one packet, in the BTreeMap's pop
//    order (exp, then push order) after a FIN/RST close (order words aux):
//    stable radix sorts by the packed order words, then by order_key, and a
//    gather of the records and their words.
// ---------------------------------------------------------------------------
// pass 1: every record's order_key into a compact array (one strided read
// of the 152-byte records; none when the emitters wrote the array: ok_in),
// the ended ones marked (Mode A: one bit per
// packet; Mode B: a count per closing packet and the largest group), and the
// active records counted per block of 256 (their places follow the ended
// prefix in record order: a scan of the block counts, no shared counter)
__global__ void __launch_bounds__(256) k_ord_keys(const fluere_record* r, uint64_t n, uint64_t base, int mode_b,
                                                  const unsigned long long* ok_in, unsigned long long* okey,
                                                  uint32_t* bits, uint32_t* cnt, uint32_t* gmax, uint32_t* blk_act) {
    __shared__ uint32_t s_act;
    if (threadIdx.x == 0) s_act = 0;
    __syncthreads();
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const bool live = i < n;
    const uint64_t k = live ? (ok_in ? ok_in[i] : r[i].order_key) : NONE64;
    if (live && !ok_in) okey[i] = k;
    const bool ended = k != NONE64;
    if (ended) {
        if (!mode_b) {
            atomicOr(&bits[(k - base) >> 5], 1u << ((k - base) & 31));
        } else {
            const uint32_t g = atomicAdd(&cnt[k - base], 1u) + 1u;
            if (g > 1) atomicMax(gmax, g);
        }
    }
    const uint64_t am = __ballot(live && !ended);
    if ((threadIdx.x & 63) == 0 && am) atomicAdd(&s_act, (uint32_t)__popcll(am));
    __syncthreads();
    if (threadIdx.x == 0) blk_act[blockIdx.x] = s_act;
}
__global__ void __launch_bounds__(256) k_ord_zero(uint32_t* cb, uint64_t nk, uint32_t* gmax) {
    const uint64_t i0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (i0 + 4 <= nk && (nk & 3) == 0) {
        *reinterpret_cast<uint4*>(cb + i0) = make_uint4(0, 0, 0, 0);
    } else {
        for (uint64_t i = i0; i < i0 + 4 && i < nk; i++) cb[i] = 0;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) *gmax = 0;
}
__global__ void __launch_bounds__(256) k_ord_popc(const uint32_t* bits, uint64_t nw, uint32_t* pc) {
    const uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (w < nw) pc[w] = __popc(bits[w]);
}
// Mode B: each closing packet's group members listed (mem[start[k] ..]), groups
// of two or more
__global__ void __launch_bounds__(256) k_ob_fill(const unsigned long long* okey, uint64_t n, uint64_t base,
                                                 uint32_t* cnt, const uint32_t* start, uint32_t* mem) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t k = okey[i];
    if (k == NONE64) return;
    if (start[k - base + 1] - start[k - base] == 1) return;  // a group of one: k_ord_move reads no members
    const uint32_t slot = atomicSub(&cnt[k - base], 1u) - 1u;
    mem[start[k - base] + slot] = (uint32_t)i;
}
// pass 2: each record's place, then the records (and Mode B's order words)
// moved there.  An ended record: Mode A, the ended keys below its own (bit
// rank); Mode B, its group's start plus its rank among the group by order
// words (exp + 1 after a FIN/RST close's 0, then the firing entry's creation:
// the BTreeMap's pop order, offline_fluereflows.rs:161-175).  An active
// record: after the ended prefix, in record order.  A wave moves its 64
// consecutive records together, 8-byte words in index order: every load
// instruction reads 512 contiguous bytes, every store writes whole 152-byte
// runs (a lane copying its own record, strided 152 bytes per lane, does not).
constexpr uint32_t REC_WORDS = sizeof(fluere_record) / 8;  // 19
__global__ void __launch_bounds__(256) k_ord_move(const fluere_record* r, const unsigned long long* aux, uint64_t n,
                                                  uint64_t base, const unsigned long long* okey, const uint32_t* bits,
                                                  const uint32_t* pre, const uint32_t* start, const uint32_t* mem,
                                                  const uint32_t* blk_pre, uint64_t n_ended, fluere_record* out,
                                                  unsigned long long* aux_out) {
    __shared__ uint32_t s_w[4];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const bool live = i < n;
    const uint64_t k = live ? okey[i] : NONE64;
    const bool ended = k != NONE64;
    // the active records' rank in the block (waves before this one, lanes before this lane)
    const uint64_t am = __ballot(live && !ended);
    if (lane == 0) s_w[w] = (uint32_t)__popcll(am);
    __syncthreads();
    uint32_t p = 0;
    if (live && !ended) {
        uint32_t before = 0;
        for (uint32_t q = 0; q < w; q++) before += s_w[q];
        p = (uint32_t)n_ended + blk_pre[blockIdx.x] + before +
            __builtin_amdgcn_mbcnt_hi((uint32_t)(am >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)am, 0u));
    } else if (ended && !start) {
        const uint64_t q = k - base;
        p = pre[q >> 5] + __popc(bits[q >> 5] & ((1u << (q & 31)) - 1u));
    } else if (ended) {
        const uint32_t s0 = start[k - base], s1 = start[k - base + 1];
        uint32_t rank = 0;
        if (s1 - s0 > 1) {
            const unsigned long long a0 = aux[2 * i], a1 = aux[2 * i + 1];
            for (uint32_t q = s0; q < s1; q++) {
                const uint32_t m = mem[q];
                const unsigned long long b0 = aux[2 * (size_t)m], b1 = aux[2 * (size_t)m + 1];
                rank += (b0 < a0 || (b0 == a0 && (b1 < a1 || (b1 == a1 && m < i)))) ? 1u : 0u;
            }
        }
        p = s0 + rank;
    }
    if (aux && live) {
        aux_out[2 * (size_t)p] = aux[2 * i];
        aux_out[2 * (size_t)p + 1] = aux[2 * i + 1];
    }
    const uint64_t w0 = i - lane;  // the wave's first record (whole waves: blockDim is a multiple of 64)
    if (w0 >= n) return;
    const uint32_t nr = (uint32_t)min<uint64_t>(64, n - w0);
    const unsigned long long* src = reinterpret_cast<const unsigned long long*>(r + w0);
    unsigned long long* dst = reinterpret_cast<unsigned long long*>(out);
    const uint32_t total = nr * REC_WORDS;
    for (uint32_t b = 0; b < total; b += 64) {  // (wave-uniform: every lane takes part in the shuffle)
        const uint32_t e = b + lane, ec = min(e, total - 1);
        const uint32_t j = ec / REC_WORDS, kk = ec - j * REC_WORDS;
        const uint32_t pj = __shfl(p, j, 64);
        if (e < total) dst[(size_t)pj * REC_WORDS + kk] = src[e];
    }
}

// Mode A with few ended records (at most a quarter): only they and the active
// records in the first n_ended places move.  k_ord_out copies the ended ones
// to their places in `out` and lists the holes they leave past n_ended;
// k_ord_fill moves the head's active records into those holes (the actives
// keep no order of their own: fetch_records sorts them); the ordered prefix
// is copied back.  About 4 x 152 B per ended record instead of 2 x 152 B per
// record.
// A wave copies the records of its lanes with `want` set, 8-byte words in
// order (as k_ord_move).  Called by every thread of the block.
__device__ __forceinline__ void wave_copy_recs(uint32_t* s_l, const fluere_record* r, uint64_t w0, bool want,
                                               uint32_t p, fluere_record* out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t m = __ballot(want);
    if (want) s_l[__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = lane;
    __syncthreads();
    const uint32_t total = (uint32_t)__popcll(m) * REC_WORDS;
    const unsigned long long* src = reinterpret_cast<const unsigned long long*>(r);
    unsigned long long* dst = reinterpret_cast<unsigned long long*>(out);
    for (uint32_t b = 0; b < total; b += 64) {  // (wave-uniform)
        const uint32_t e = b + lane, ec = min(e, total - 1);
        const uint32_t j = ec / REC_WORDS, kk = ec - j * REC_WORDS;
        const uint32_t L = s_l[j];
        const uint32_t pj = __shfl(p, L, 64);
        if (e < total) dst[(size_t)pj * REC_WORDS + kk] = src[(w0 + L) * REC_WORDS + kk];
    }
}
// the active records before record i (in the block's wave order)
__device__ __forceinline__ uint32_t act_before(uint32_t* s_w, uint64_t am, const uint32_t* blk_pre) {
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) s_w[w] = (uint32_t)__popcll(am);
    __syncthreads();
    uint32_t before = 0;
    for (uint32_t q = 0; q < w; q++) before += s_w[q];
    return blk_pre[blockIdx.x] + before +
           __builtin_amdgcn_mbcnt_hi((uint32_t)(am >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)am, 0u));
}
__global__ void __launch_bounds__(256) k_ord_out(const fluere_record* r, uint64_t n, uint64_t base,
                                                 const unsigned long long* okey, const uint32_t* bits,
                                                 const uint32_t* pre, const uint32_t* blk_pre, uint64_t n_ended,
                                                 fluere_record* out, uint32_t* holes, uint32_t* head_act) {
    __shared__ uint32_t s_w[4];
    __shared__ uint32_t s_l[4][64];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const bool live = i < n;
    const uint64_t k = live ? okey[i] : NONE64;
    const bool ended = k != NONE64;
    const uint32_t ab = act_before(s_w, __ballot(live && !ended), blk_pre);
    if (i == n_ended) *head_act = ab;  // the head's active records (n_ended < n)
    uint32_t p = 0;
    if (ended) {
        const uint64_t q = k - base;
        p = pre[q >> 5] + __popc(bits[q >> 5] & ((1u << (q & 31)) - 1u));
        if (i >= n_ended) holes[i - ab] = (uint32_t)i;  // ended records before i: i - ab
    }
    wave_copy_recs(s_l[w], r, i - lane, ended, p, out);
}
// the head's active records (i < n_ended; the i-th of them is its
// act_before) into the holes past n_ended, which start at ended rank
// n_ended - head_act
__global__ void __launch_bounds__(256) k_ord_fill(fluere_record* r, const unsigned long long* okey,
                                                  const uint32_t* blk_pre, uint64_t n_ended, const uint32_t* holes,
                                                  const uint32_t* head_act) {
    __shared__ uint32_t s_w[4];
    __shared__ uint32_t s_l[4][64];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const bool act = i < n_ended && okey[i] == NONE64;
    const uint32_t ab = act_before(s_w, __ballot(act), blk_pre);
    const uint32_t p = act ? holes[ab + (uint32_t)n_ended - *head_act] : 0u;
    wave_copy_recs(s_l[w], r, i - lane, act, p, r);
}

int ord_scratch(fluere_ctx* c, size_t need) {
    if (need <= c->d_ord_bytes) return FLUERE_OK;
    hipFree(c->d_ord);
    c->d_ord = nullptr;
    c->d_ord_bytes = 0;
    if (hipMalloc(&c->d_ord, need) != hipSuccess) return FLUERE_E_NOMEM;
    c->d_ord_bytes = need;
    return FLUERE_OK;
}

int grow_pair(void** a, void** b, uint64_t* cap_b, uint64_t cap_a, size_t unit) {
    if (*cap_b >= cap_a) return FLUERE_OK;
    hipFree(*b);
    *b = nullptr;
    *cap_b = 0;
    if (hipMalloc(b, cap_a * unit) != hipSuccess) return FLUERE_E_NOMEM;
    *cap_b = cap_a;
    (void)a;
    return FLUERE_OK;
}

// The active tail [ne, ne + m) of d_recs sorted by first packet (stable: the
// run's order among equal ones) into d_recs2 [0, m).
__global__ void k_act_keys(const fluere_record* r, uint64_t m, unsigned long long* keys, uint32_t* vals) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    keys[i] = r[i].first;
    vals[i] = (uint32_t)i;
}
__global__ void k_act_gather(const fluere_record* src, const uint32_t* perm, uint64_t m, fluere_record* dst) {
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;  // one word of one record
    if (e >= m * REC_WORDS) return;
    const uint64_t j = e / REC_WORDS, k = e - j * REC_WORDS;
    reinterpret_cast<uint64_t*>(dst)[e] = reinterpret_cast<const uint64_t*>(src)[(uint64_t)perm[j] * REC_WORDS + k];
}

int sort_actives(fluere_ctx* c, uint64_t ne, uint64_t m) {
    if (m >= (1ull << 31) || !m) return FLUERE_E_ARG;
    hipStream_t s = c->stream;
    int rc = grow_pair((void**)&c->d_recs, (void**)&c->d_recs2, &c->d_recs2_cap, c->d_recs_cap, sizeof(fluere_record));
    if (rc || c->d_recs2_cap < m) return rc ? rc : FLUERE_E_NOMEM;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    size_t tb = 0;
    (void)prim_sort_pairs(nullptr, tb, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                             (uint32_t*)nullptr, (uint32_t*)nullptr, (int)m, 0, 64, s);
    if ((rc = ord_scratch(c, 2 * al(m * 8) + 2 * al(m * 4) + al(tb)))) return rc;
    char* p = (char*)c->d_ord;
    auto take = [&](size_t bytes) { char* q = p; p += al(bytes); return q; };
    unsigned long long* k0 = (unsigned long long*)take(m * 8);
    unsigned long long* k1 = (unsigned long long*)take(m * 8);
    uint32_t* v0 = (uint32_t*)take(m * 4);
    uint32_t* v1 = (uint32_t*)take(m * 4);
    const fluere_record* act = c->d_recs + ne;
    k_act_keys<<<grid_for(m, 256), 256, 0, s>>>(act, m, k0, v0);
    size_t t = tb;
    HIPCHECK(prim_sort_pairs(p, t, k0, k1, v0, v1, (int)m, 0, 64, s));
    k_act_gather<<<grid_for(m * REC_WORDS, 256), 256, 0, s>>>(act, v1, m, c->d_recs2);
    HIPCHECK(hipGetLastError());
    return FLUERE_OK;
}

// Mode B with a large sweep group (an idle gap that ends thousands of flows
// at one packet): every record in the reference's order by stable LSD radix
// sorts -- by the firing entry's creation (aux[1]), then by exp + 1 (aux[0],
// 0 for a FIN/RST close), then by the ending packet (order_key; active
// records, NONE64, last) -- and one gather of the records and their words.
__global__ void k_ob_keys(const unsigned long long* okey, const unsigned long long* aux, uint64_t n, int word,
                          unsigned long long* keys, uint32_t* vals) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    keys[i] = word < 2 ? aux[2 * i + word] : okey[i];
    vals[i] = (uint32_t)i;
}
__global__ void k_ob_rekey(const unsigned long long* okey, const unsigned long long* aux, const uint32_t* perm,
                           uint64_t n, int word, unsigned long long* keys) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t j = perm[i];
    keys[i] = word < 2 ? aux[2 * (size_t)j + word] : okey[j];
}
__global__ void k_ob_gather_aux(const unsigned long long* aux, const uint32_t* perm, uint64_t n, unsigned long long* out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t j = perm[i];
    out[2 * i] = aux[2 * (size_t)j];
    out[2 * i + 1] = aux[2 * (size_t)j + 1];
}

static int order_sorted(fluere_ctx* c, uint64_t n, uint64_t n_ended, const unsigned long long* okey) {
    hipStream_t s = c->stream;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    size_t tb = 0;
    (void)prim_sort_pairs(nullptr, tb, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                             (uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0, 64, s);
    // (okey lives in the ordering scratch or the emitters' array: the keys get a buffer of their own)
    void* buf = nullptr;
    if (hipMalloc(&buf, 2 * al(n * 8) + 2 * al(n * 4) + al(tb)) != hipSuccess) return FLUERE_E_NOMEM;
    char* p = (char*)buf;
    auto take = [&](size_t bytes) { char* q = p; p += al(bytes); return q; };
    unsigned long long* k0 = (unsigned long long*)take(n * 8);
    unsigned long long* k1 = (unsigned long long*)take(n * 8);
    uint32_t* v0 = (uint32_t*)take(n * 4);
    uint32_t* v1 = (uint32_t*)take(n * 4);
    void* tmp = p;
    const unsigned g = grid_for(n, 256);
    int rc = FLUERE_OK;
    for (int word = 1; word >= -1 && rc == FLUERE_OK; word--) {  // aux[1], aux[0], order_key (word 2)
        const int w = word < 0 ? 2 : word;
        if (word == 1) k_ob_keys<<<g, 256, 0, s>>>(okey, c->d_recaux, n, w, k0, v0);
        else k_ob_rekey<<<g, 256, 0, s>>>(okey, c->d_recaux, v0, n, w, k0);
        size_t t = tb;
        if (prim_sort_pairs(tmp, t, k0, k1, v0, v1, (int)n, 0, 64, s) != hipSuccess) rc = FLUERE_E_HIP;
        std::swap(v0, v1);  // the permutation so far (stable: ties keep the last pass's order)
    }
    if (rc == FLUERE_OK) {
        k_act_gather<<<grid_for(n * REC_WORDS, 256), 256, 0, s>>>(c->d_recs, v0, n, c->d_recs2);
        k_ob_gather_aux<<<g, 256, 0, s>>>(c->d_recaux, v0, n, c->d_recaux2);
        if (hipGetLastError() != hipSuccess) rc = FLUERE_E_HIP;
    }
    HIPCHECK(ctx_sync(c));  // (then the scratch is released)
    hipFree(buf);
    if (rc) return rc;
    std::swap(c->d_recaux, c->d_recaux2);
    std::swap(c->d_recaux_cap, c->d_recaux2_cap);
    std::swap(c->d_recs, c->d_recs2);
    std::swap(c->d_recs_cap, c->d_recs2_cap);
    c->dev_ordered = true;
    c->dev_ordered_ended = n_ended;
    return FLUERE_OK;
}

// Orders the run's n records in d_recs (n_ended of them ended) as
// [ended][active]; Mode B with the order words in d_recaux.  Stream-ordered;
// Mode B reads its largest group (records ending at one packet) once.
// n_okey: the run's Glob::n_okey (the order-key array holds every record's
// key when it equals n).
int order_records(fluere_ctx* c, uint64_t n, uint64_t n_ended, bool mode_b, uint64_t n_okey) {
    c->dev_ordered = false;
    if (!n || !n_ended || n >= (1ull << 32)) return FLUERE_OK;
    hipStream_t s = c->stream;
    const uint64_t base = c->index_base, N = std::max<uint64_t>(c->n_total, 1);
    int rc = grow_pair((void**)&c->d_recs, (void**)&c->d_recs2, &c->d_recs2_cap, c->d_recs_cap, sizeof(fluere_record));
    if (rc) return rc;
    if (mode_b && !c->d_recaux) return FLUERE_OK;
    if (mode_b && (rc = grow_pair((void**)&c->d_recaux, (void**)&c->d_recaux2, &c->d_recaux2_cap, c->d_recaux_cap, 16)))
        return rc;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const unsigned gn = grid_for(n, 256);
    const uint64_t nw = N / 32 + 1;                 // Mode A: bit words
    const uint64_t nk = mode_b ? N + 1 : nw;        // the scanned array: Mode A bit counts, Mode B group counts
    size_t tb = 0, tb2 = 0;
    (void)prim_exclusive_sum(nullptr, tb, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)nk, s);
    (void)prim_exclusive_sum(nullptr, tb2, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)gn, s);
    tb = std::max(tb, tb2);
    // scratch: okey[n] | cnt-or-bits[nk] | pc[nw] | pre-or-start[nk] | mem[n] | blk[gn] | blk_pre[gn] | gmax | tmp
    if ((rc = ord_scratch(c, al(n * 8) + 2 * al(nk * 4) + al(nw * 4) + al(n * 4) + 2 * al(gn * 4) + al(16) + al(tb))))
        return rc;
    char* p = (char*)c->d_ord;
    auto take = [&](size_t bytes) { char* q = p; p += al(bytes); return q; };
    unsigned long long* okey = (unsigned long long*)take(n * 8);
    static const bool no_okey = getenv("FLUERE_NO_OKEY") != nullptr;
    const bool have_okey = !no_okey && c->d_okey && n_okey == n && n <= c->d_okey_cap;
    if (have_okey) okey = c->d_okey;
    uint32_t* cb = (uint32_t*)take(nk * 4);   // Mode A bits, Mode B counts
    uint32_t* pc = (uint32_t*)take(nw * 4);
    uint32_t* ps = (uint32_t*)take(nk * 4);   // Mode A bit-count prefix, Mode B group starts
    uint32_t* mem = (uint32_t*)take(n * 4);
    uint32_t* blk = (uint32_t*)take(gn * 4);
    uint32_t* blk_pre = (uint32_t*)take(gn * 4);
    uint32_t* gmax = (uint32_t*)take(16);
    void* tmp = p;
    // (one launch for both clears: each host submission here leaves the GPU idle)
    k_ord_zero<<<(unsigned)std::max<uint64_t>(1, (nk + 1023) / 1024), 256, 0, s>>>(cb, nk, gmax);
    k_ord_keys<<<gn, 256, 0, s>>>(c->d_recs, n, base, mode_b ? 1 : 0, have_okey ? c->d_okey : nullptr, okey, cb, cb,
                                  gmax, blk);
    size_t t = tb;
    HIPCHECK(prim_exclusive_sum(tmp, t, blk, blk_pre, (int)gn, s));
    if (!mode_b) {
        k_ord_popc<<<grid_for(nw, 256), 256, 0, s>>>(cb, nw, pc);
        t = tb;
        HIPCHECK(prim_exclusive_sum(tmp, t, pc, ps, (int)nw, s));
        static const bool all_move = getenv("FLUERE_ORD_MOVE_ALL") != nullptr;
        if (!all_move && n_ended * 4 <= n) {  // few ended: only they and the head's actives move (k_ord_out)
            k_ord_out<<<gn, 256, 0, s>>>(c->d_recs, n, base, okey, cb, ps, blk_pre, n_ended, c->d_recs2, mem, gmax);
            k_ord_fill<<<grid_for(n_ended, 256), 256, 0, s>>>(c->d_recs, okey, blk_pre, n_ended, mem, gmax);
            HIPCHECK(hipMemcpyAsync(c->d_recs, c->d_recs2, n_ended * sizeof(fluere_record), hipMemcpyDeviceToDevice, s));
            HIPCHECK(hipGetLastError());
            c->dev_ordered = true;
            c->dev_ordered_ended = n_ended;
            return FLUERE_OK;
        }
        k_ord_move<<<gn, 256, 0, s>>>(c->d_recs, nullptr, n, base, okey, cb, ps, nullptr, nullptr, blk_pre, n_ended,
                                      c->d_recs2, nullptr);
    } else {
        // the groups' starts (pc, unused in Mode B: the tile totals)
        if ((rc = flag_count(s, N + 1, cb, ps, false, nullptr, pc))) return rc;
        // the largest group: a sweep that ends thousands of flows at one packet
        // (an idle gap) would make the members' rank scans quadratic
        unsigned long long g = 0;
        const void* src[1] = {gmax};
        const int by[1] = {4};
        if ((rc = mail_fetch(c->h_mail, s, 1, src, by, &g))) return rc;
        if (g > 1024) return order_sorted(c, n, n_ended, okey);  // (rank scans would be quadratic)
        k_ob_fill<<<gn, 256, 0, s>>>(okey, n, base, cb, ps, mem);
        k_ord_move<<<gn, 256, 0, s>>>(c->d_recs, c->d_recaux, n, base, okey, nullptr, nullptr, ps, mem, blk_pre, n_ended,
                                      c->d_recs2, c->d_recaux2);
        std::swap(c->d_recaux, c->d_recaux2);
        std::swap(c->d_recaux_cap, c->d_recaux2_cap);
    }
    HIPCHECK(hipGetLastError());
    std::swap(c->d_recs, c->d_recs2);
    std::swap(c->d_recs_cap, c->d_recs2_cap);
    c->dev_ordered = true;
    c->dev_ordered_ended = n_ended;
    return FLUERE_OK;
}

// ---------------------------------------------------------------------------
// Mode A ordering enqueued behind k_finalize (SoArgs).  The host used to wait
// for the run's counters, then launch the ordering (bit marks, two library
// scans, the moves): its launches, the scans' host-side work and the wake-up
// left the GPU idle for most of the ~90 us the ordering took.  Here three
// kernels are queued with the pass; they read n_rec / n_ended on the device
// and act only when the run is complete (run_complete: the same test the
// speculative k_cleanup takes, and the host after it), so a run that needs
// the exact engine or Mode B finds d_recs untouched and orders it itself.
// Every place comes from prefix counts over two bit arrays -- no shared
// counters (same-address atomics from every CU serialize), no spinning:
//  * key bits: one per packet, set by k_finalize at each ended record's
//    closing packet; an ended record's place is the count of key bits below
//    its own;
//  * record bits: one per record, set by k_finalize when it is ended; E(i), the ended
//    records before record i, pairs the k-th hole (an ended record at or
//    past n_ended) with the k-th active record of the prefix.
//  k_so_scan  for both arrays, per word, the bits below it in its tile of
//             1024 words, and the tile totals; it also clears the other
//             arrays' dirty words for the next run (no memset);
//  k_so_out   (the tile totals scanned in LDS first) every ended record to its
//             place in d_recs2, a hole listed when it sits past the prefix; at
//             most a quarter ended only they move, else every record does
//             (the actives after the prefix in record order) and the host
//             swaps the buffers;
//  k_so_fill  the prefix's active records into the holes, then the ordered
//             prefix over d_recs (a workgroup per 64 records).
// Grids are any size: the record loops stride over the device counts.
__device__ __forceinline__ bool so_go(const SoArgs& a, uint64_t& n, uint64_t& ne, const unsigned long long*& ok) {
    const Glob& g = *a.g;
    n = g.n_rec;
    ne = g.n_ended;
    const OkeyRef o = okey_ref(a.g);
    ok = (o.p && g.n_okey == n && n <= o.cap) ? o.p : nullptr;
    return run_complete(g, *a.err, a.timeout_us, a.recs_cap) && n && ne && n < (1ull << 32);
}
__device__ __forceinline__ uint64_t so_key(const SoArgs& a, const unsigned long long* ok, uint64_t i) {
    return ok ? ok[i] : a.r[i].order_key;
}
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// s[0, T) = the exclusive prefix of src[0, T) (256 threads; ends with a barrier)
__device__ void lds_exclusive_scan(uint32_t* s, const uint32_t* src, uint32_t T) {
    __shared__ uint32_t s_w[4];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    for (uint32_t t = tid; t < T; t += 256) s[t] = src[t];
    __syncthreads();
    const uint32_t c = (T + 255) / 256, lo = min(T, tid * c), hi = min(T, lo + c);
    uint32_t sum = 0;
    for (uint32_t k = lo; k < hi; k++) sum += s[k];
    uint32_t incl = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d, 64);
        if ((int)lane >= d) incl += y;
    }
    if (lane == 63) s_w[wv] = incl;
    __syncthreads();
    uint32_t run = incl - sum;
    for (uint32_t q = 0; q < wv; q++) run += s_w[q];
    for (uint32_t k = lo; k < hi; k++) {
        const uint32_t v = s[k];
        s[k] = run;
        run += v;
    }
    __syncthreads();
}
// The listed records (lanes with `want` of the 64 at w0) to out[p], 8-byte
// words in order, by `nw` waves (the w-th takes every nw-th group of 64
// words): every load first, then every store -- one memory round trip, not
// one per 64 words.  Called by those waves alike (one list, block-uniform when
// nw > 1: the list is published with a barrier).
template <int NW>
__device__ __forceinline__ void copy_listed(uint32_t* s_l, const fluere_record* r, uint64_t w0, bool want,
                                            uint32_t p, fluere_record* out, uint32_t wv) {
    constexpr uint32_t IT = (REC_WORDS + NW - 1) / NW;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t m = __ballot(want);
    if (NW == 1 && !m) return;
    if (want && wv == 0) s_l[lanes_below(m)] = lane;
    if (NW > 1) {
        __syncthreads();
    } else {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    const uint32_t total = (uint32_t)__popcll(m) * REC_WORDS;
    const unsigned long long* src = reinterpret_cast<const unsigned long long*>(r);
    unsigned long long* dst = reinterpret_cast<unsigned long long*>(out);
    unsigned long long v[IT];
#pragma unroll
    for (uint32_t u = 0; u < IT; u++) {
        const uint32_t e = (u * NW + wv) * 64 + lane;
        if (e < total) {
            const uint32_t j = e / REC_WORDS, kk = e - j * REC_WORDS;
            v[u] = src[(w0 + s_l[j]) * REC_WORDS + kk];
        }
    }
#pragma unroll
    for (uint32_t u = 0; u < IT; u++) {
        const uint32_t b = (u * NW + wv) * 64;
        if (b < total) {  // (wave-uniform: every lane takes part in the shuffle)
            const uint32_t e = b + lane, ec = min(e, total - 1);
            const uint32_t j = ec / REC_WORDS, kk = ec - j * REC_WORDS;
            const uint32_t pj = __shfl(p, (int)s_l[j], 64);
            if (e < total) dst[(size_t)pj * REC_WORDS + kk] = v[u];
        }
    }
    if (NW > 1) {
        __syncthreads();  // (s_l is rewritten by the next call)
    } else {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}

// grid: the key tiles (a.kt) then the record tiles (a.rt), 1024 words each;
// 1024 threads
__global__ void __launch_bounds__(MB) k_so_scan(SoArgs a) {
    __shared__ uint32_t s_scan[MB / 64 + 1];
    for (uint64_t w = (uint64_t)blockIdx.x * MB + threadIdx.x; w < a.zn; w += (uint64_t)gridDim.x * MB) a.zbits[w] = 0;
    for (uint64_t w = (uint64_t)blockIdx.x * MB + threadIdx.x; w < a.zrn; w += (uint64_t)gridDim.x * MB) a.zrbits[w] = 0;
    uint64_t n, ne;
    const unsigned long long* ok;
    if (!so_go(a, n, ne, ok)) return;
    const bool rec = blockIdx.x >= a.kt;
    const uint64_t w = (uint64_t)(rec ? blockIdx.x - a.kt : blockIdx.x) * MB + threadIdx.x;
    const uint64_t nw = rec ? (n + 31) / 32 : a.nw;
    const uint32_t word = w < nw ? (rec ? a.rbits : a.bits)[w] : 0u;
    const uint32_t pre = block_exclusive_scan((uint32_t)__popc(word), s_scan);  // (at most 1023 x 32: fits 16 bits)
    if (w < nw) (rec ? a.rwpre : a.wpre)[w] = (uint16_t)pre;
    if (threadIdx.x == 0) a.tpre[blockIdx.x] = s_scan[MB / 64];
}

// dynamic LDS: (kt + rt) words, the tile prefixes
__global__ void __launch_bounds__(256) k_so_out(SoArgs a) {
    extern __shared__ uint32_t s_tp[];
    __shared__ uint32_t s_l[4][64];
    uint64_t n, ne;
    const unsigned long long* ok;
    if (!so_go(a, n, ne, ok)) return;
    lds_exclusive_scan(s_tp, a.tpre, a.kt + a.rt);  // key tiles, then record tiles (offset by the key total)
    const uint32_t* rtp = s_tp + a.kt;
    const uint32_t r0 = rtp[0];
    const bool few = ne * 4 <= n;
    // ended records before the prefix's end: E(ne)
    uint32_t e_ne = 0;
    if (few) e_ne = rtp[(ne >> 5) >> 10] - r0 + a.rwpre[ne >> 5] + (uint32_t)__popc(a.rbits[ne >> 5] & ((1u << (ne & 31)) - 1u));
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (uint64_t w0 = ((uint64_t)blockIdx.x * 4 + wv) * 64; w0 < n; w0 += (uint64_t)gridDim.x * 256) {
        const uint64_t i = w0 + lane;
        const bool live = i < n;
        const uint64_t k = live ? so_key(a, ok, i) : NONE64;
        const bool ended = k != NONE64;
        const uint64_t em = __ballot(ended);
        const uint32_t e_i = rtp[(w0 >> 5) >> 10] - r0 + a.rwpre[w0 >> 5] + lanes_below(em);  // E(i)
        uint32_t p = 0;
        if (ended) {
            const uint64_t q = k - a.base, w = q >> 5;
            p = s_tp[w >> 10] + a.wpre[w] + (uint32_t)__popc(a.bits[w] & ((1u << (q & 31)) - 1u));
        }
        if (few) {
            if (ended && i >= ne) a.holes[e_i - e_ne] = (uint32_t)i;
            copy_listed<1>(s_l[wv], a.r, w0, ended, p, a.r2, 0);
        } else {
            if (live && !ended) p = (uint32_t)ne + ((uint32_t)i - e_i);
            copy_listed<1>(s_l[wv], a.r, w0, live, p, a.r2, 0);
        }
    }
}

// dynamic LDS: rt words, the record tiles' prefixes; a workgroup per 64
// records of the prefix, its four waves sharing the copies
__global__ void __launch_bounds__(256) k_so_fill(SoArgs a) {
    extern __shared__ uint32_t s_tp[];
    __shared__ uint32_t s_l[64];
    uint64_t n, ne;
    const unsigned long long* ok;
    if (!so_go(a, n, ne, ok) || ne * 4 > n) return;
    lds_exclusive_scan(s_tp, a.tpre + a.kt, a.rt);
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (uint64_t w0 = (uint64_t)blockIdx.x * 64; w0 < ne; w0 += (uint64_t)gridDim.x * 64) {  // (block-uniform)
        const uint64_t j = w0 + lane;
        const bool ended = (a.rbits[j >> 5] >> (j & 31)) & 1u;
        const bool act = j < ne && !ended;
        const uint64_t em = __ballot(ended);
        const uint32_t e_j = s_tp[(w0 >> 5) >> 10] + a.rwpre[w0 >> 5] + lanes_below(em);
        const uint32_t p = act ? a.holes[(uint32_t)j - e_j] : 0u;  // the k-th active takes the k-th hole
        copy_listed<4>(s_l, a.r, w0, act, p, a.r, wv);  // (every hole lies past the prefix)
        const uint32_t nr = (uint32_t)min<uint64_t>(64, ne - w0);
        copy_listed<4>(s_l, a.r2, w0, lane < nr, (uint32_t)j, a.r, wv);  // then the ordered prefix over it
    }
}

void so_free(fluere_ctx* c) {
    hipFree(c->d_sob);
    hipFree(c->d_sos);
    hipFree(c->d_sorb);
    c->d_sorb = nullptr;
    c->sorb_cap = 0;
    c->d_sob = nullptr;
    c->d_sos = nullptr;
    c->sob_cap = 0;
    c->sos_bytes = 0;
}

// The launches and scratch of one run's ordering; flips the key bit arrays
// (call right before so_enqueue).  L.on = 0 when it does not apply.
constexpr uint64_t SO_MAX_TILES = 12288;  // key + record tiles: 48 KiB of tile prefixes in LDS

int so_plan(fluere_ctx* c, SoLaunch& L, unsigned long long timeout_us) {
    L.on = 0;
    const uint64_t N = std::max<uint64_t>(c->n_total, 1), nw = N / 32 + 1;
    const uint64_t kt = (nw + MB - 1) / MB;
    const uint64_t rw = (c->d_recs_cap + 63) / 64 * 2, rt = (rw + MB - 1) / MB;
    if (c->d_recs_cap >= (1ull << 32) || kt + rt > SO_MAX_TILES) return FLUERE_OK;  // (the prefixes live in LDS)
    int rc = grow_pair((void**)&c->d_recs, (void**)&c->d_recs2, &c->d_recs2_cap, c->d_recs_cap, sizeof(fluere_record));
    if (rc) return rc;
    hipStream_t s = c->stream;
    if (c->sob_cap < nw) {
        hipFree(c->d_sob);
        c->d_sob = nullptr;
        c->sob_cap = 0;
        const uint64_t cap = nw + nw / 4;
        if (hipMalloc(&c->d_sob, 2 * cap * 4) != hipSuccess) return FLUERE_E_NOMEM;
        HIPCHECK(hipMemsetAsync(c->d_sob, 0, 2 * cap * 4, s));
        c->sob_cap = cap;
        c->sob_dirty[0] = c->sob_dirty[1] = 0;
    }
    if (c->sorb_cap < rw) {
        hipFree(c->d_sorb);
        c->d_sorb = nullptr;
        c->sorb_cap = 0;
        const uint64_t cap = rw + rw / 4;
        if (hipMalloc(&c->d_sorb, 2 * cap * 4) != hipSuccess) return FLUERE_E_NOMEM;
        HIPCHECK(hipMemsetAsync(c->d_sorb, 0, 2 * cap * 4, s));
        c->sorb_cap = cap;
        c->sorb_dirty[0] = c->sorb_dirty[1] = 0;
    }
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t need = al(nw * 2) + al(rw * 2) + al((kt + rt) * 4) + al(c->d_recs_cap * 4);
    if (c->sos_bytes < need) {
        hipFree(c->d_sos);
        c->d_sos = nullptr;
        c->sos_bytes = 0;
        if (hipMalloc(&c->d_sos, need + need / 4) != hipSuccess) return FLUERE_E_NOMEM;
        c->sos_bytes = need + need / 4;
    }
    char* p = (char*)c->d_sos;
    auto take = [&](size_t bytes) { char* q = p; p += al(bytes); return q; };
    SoArgs& a = L.a;
    a.g = c->d_glob;
    a.err = tables_of(c).err;
    a.timeout_us = timeout_us;
    a.recs_cap = c->d_recs_cap;
    a.r = c->d_recs;
    a.r2 = c->d_recs2;
    a.base = c->index_base;
    a.nw = nw;
    a.kt = (uint32_t)kt;
    a.rt = (uint32_t)rt;
    a.wpre = (uint16_t*)take(nw * 2);
    a.rwpre = (uint16_t*)take(rw * 2);
    a.tpre = (uint32_t*)take((kt + rt) * 4);
    a.holes = (uint32_t*)take(c->d_recs_cap * 4);
    const int cur = c->sob_cur;
    a.bits = c->d_sob + (size_t)cur * c->sob_cap;
    a.zbits = c->d_sob + (size_t)(cur ^ 1) * c->sob_cap;
    a.zn = c->sob_dirty[cur ^ 1];
    c->sob_dirty[cur] = std::max(c->sob_dirty[cur], nw);
    c->sob_dirty[cur ^ 1] = 0;
    a.rbits = c->d_sorb + (size_t)cur * c->sorb_cap;
    a.zrbits = c->d_sorb + (size_t)(cur ^ 1) * c->sorb_cap;
    a.zrn = c->sorb_dirty[cur ^ 1];
    c->sorb_dirty[cur] = std::max(c->sorb_dirty[cur], rw);
    c->sorb_dirty[cur ^ 1] = 0;
    c->sob_cur = cur ^ 1;
    auto clampg = [](uint64_t n, unsigned per) {
        return (unsigned)std::min<uint64_t>(std::max<uint64_t>(grid_for(n, per), 8), 4096);
    };
    L.g_out = clampg(c->so_last_n, 256);
    L.g_fill = clampg(c->so_last_ne, 64);
    L.g_scan = (unsigned)(kt + rt);
    L.on = 1;
    return FLUERE_OK;
}

int so_enqueue(fluere_ctx* c, const SoLaunch& L) {
    hipStream_t s = c->stream;
    k_so_scan<<<L.g_scan, MB, 0, s>>>(L.a);
    k_so_out<<<L.g_out, 256, (L.a.kt + L.a.rt) * 4, s>>>(L.a);
    k_so_fill<<<L.g_fill, 256, L.a.rt * 4, s>>>(L.a);
    HIPCHECK(hipGetLastError());
    return FLUERE_OK;
}
