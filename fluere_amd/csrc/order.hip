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
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tb, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
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
    HIPCHECK(hipcub::DeviceRadixSort::SortPairs(p, t, k0, k1, v0, v1, (int)m, 0, 64, s));
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
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tb, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
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
        if (hipcub::DeviceRadixSort::SortPairs(tmp, t, k0, k1, v0, v1, (int)n, 0, 64, s) != hipSuccess) rc = FLUERE_E_HIP;
        std::swap(v0, v1);  // the permutation so far (stable: ties keep the last pass's order)
    }
    if (rc == FLUERE_OK) {
        k_act_gather<<<grid_for(n * REC_WORDS, 256), 256, 0, s>>>(c->d_recs, v0, n, c->d_recs2);
        k_ob_gather_aux<<<g, 256, 0, s>>>(c->d_recaux, v0, n, c->d_recaux2);
        if (hipGetLastError() != hipSuccess) rc = FLUERE_E_HIP;
    }
    HIPCHECK(hipStreamSynchronize(s));  // (then the scratch is released)
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
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tb, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)nk, s);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)gn, s);
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
    HIPCHECK(hipMemsetAsync(cb, 0, nk * 4, s));
    HIPCHECK(hipMemsetAsync(gmax, 0, 4, s));
    k_ord_keys<<<gn, 256, 0, s>>>(c->d_recs, n, base, mode_b ? 1 : 0, have_okey ? c->d_okey : nullptr, okey, cb, cb,
                                  gmax, blk);
    size_t t = tb;
    HIPCHECK(hipcub::DeviceScan::ExclusiveSum(tmp, t, blk, blk_pre, (int)gn, s));
    if (!mode_b) {
        k_ord_popc<<<grid_for(nw, 256), 256, 0, s>>>(cb, nw, pc);
        t = tb;
        HIPCHECK(hipcub::DeviceScan::ExclusiveSum(tmp, t, pc, ps, (int)nw, s));
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
        t = tb;
        HIPCHECK(hipcub::DeviceScan::ExclusiveSum(tmp, t, cb, ps, (int)(N + 1), s));
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
