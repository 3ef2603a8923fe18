// fluere_gpu.hip -- MI355X kernels and the C ABI (include/fluere_gpu.h) for
// the `fluere offline` hot path.
//
// Pipeline for one capture (all batches attached to a context):
//   k_parse_agg   one streaming pass over the pcap records in HBM: parse
//                 (parse_keys + parse_fluereflow), canonical flow key, exact
//                 dense flow id (flow_table.h), and the update_flow sums /
//                 min / max / flag counts / first-last packet indices,
//                 pre-aggregated in LDS per workgroup and flushed with
//                 coalesced atomics.                        <- roofline kernel
//   k_finalize    one thread per flow: if the order-free aggregate is exactly
//                 what the reference state machine would produce (certificate
//                 below) build the FluereRecord, else mark the flow complex.
//   complex flows (Mode A: no expiry can fire) and Mode B (capture span >=
//                 timeout, so expiries can fire): the exact state machine of
//                 exact.hip -- packets sorted by (flow, index), a per-flow
//                 pointer chase over flow instances (SYN gate, FIN/RST split,
//                 hard-timeout sweep), segmented reductions for the records.
//                 Mode B captures whose timestamps go backwards fall back to
//                 the sequential kernel (k_seq_*).
//
// Certificate (Mode A, per flow): first create-eligible packet == first
// packet of the flow (TCP: the first packet carries SYN) and no FIN/RST before
// the last packet.  Then the reference creates the flow at its first packet,
// every later packet updates it, and it is closed (if at all) by its last
// packet -- so the record is the order-free aggregate, with orientation / ports
// / tos / first taken from the first packet and `last` from the last one
// (offline_fluereflows.rs:97-157, flows.rs:11-42).
#include "ctx.h"

hipError_t fl_dmalloc(void** p, size_t bytes, int line) {
    static const bool log = getenv("FLUERE_ALLOC_LOG") != nullptr;
    if (!log) return (hipMalloc)(p, bytes);
    const auto t0 = std::chrono::steady_clock::now();
    const hipError_t e = (hipMalloc)(p, bytes);
    fprintf(stderr, "[fluere] hipMalloc line %d: %zu bytes, %.1f us\n", line, bytes,
            std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    return e;
}

static_assert(sizeof(fluere_record) == 152, "fluere_record ABI");
static_assert(sizeof(fluere_pkt_meta) == 128, "fluere_pkt_meta ABI");
static_assert(sizeof(fluere_flow_summary) == 256, "fluere_flow_summary ABI");
static_assert(sizeof(fluere_flow_piece) == 144, "fluere_flow_piece ABI");
static_assert(sizeof(fluere_flow_annex) == 512, "fluere_flow_annex ABI");
static_assert(sizeof(fluere_shard_header) == 64, "fluere_shard_header ABI");
static_assert(sizeof(fluere_raw_hdr) == 64, "fluere_raw_hdr ABI");

namespace {

// ---------------------------------------------------------------------------
// library seam: per-packet parse_keys / parse_fluereflow view
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_parse_batch(Batch B, fluere_pkt_meta* out, int mode) {
    uint64_t li = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (li >= B.n) return;
    Parsed P;
    if (mode == 0) {  // production: fast, middle, general (the k_slow sequence)
        const uint32_t off = B.offs[li];
        Win32 W;
        load_win32(B, off, W);
        parse_loaded32<1>(B, off, W, true, P);
    } else {
        parse_record(B, li, true, mode, P);
    }
    const PktInfo& pi = P.pi;
    fluere_pkt_meta m;
    memset(&m, 0, sizeof m);
    m.k_status = pi.kst;
    m.f_status = pi.fst;
    m.raw_used = pi.raw;
    const uint8_t* fr = B.bytes + B.offs[li] + 16;
    if (pi.kst == ST_OK) {
        m.key_v6 = pi.v6; m.key_proto = pi.kproto; m.key_sport = pi.ksp; m.key_dport = pi.kdp;
        for (int k = 0; k < 4; k++)
            for (int b = 0; b < 4; b++) {
                m.key_src[4 * k + b] = (uint8_t)(pi.sip[k] >> (24 - 8 * b));
                m.key_dst[4 * k + b] = (uint8_t)(pi.dip[k] >> (24 - 8 * b));
            }
        for (int b = 0; b < 6; b++) {
            m.key_dmac[b] = fr[pi.frame_off + b];
            m.key_smac[b] = fr[pi.frame_off + 6 + b];
        }
    }
    if (pi.fst == ST_OK) {
        m.rec_v6 = pi.rv6; m.rec_prot = pi.rprot; m.rec_tos = pi.rtos; m.rec_ttl = pi.rttl;
        for (int k = 0; k < 4; k++)
            for (int b = 0; b < 4; b++) {
                m.rec_src[4 * k + b] = (uint8_t)(pi.rsip[k] >> (24 - 8 * b));
                m.rec_dst[4 * k + b] = (uint8_t)(pi.rdip[k] >> (24 - 8 * b));
            }
        m.rec_sport = pi.rsp; m.rec_dport = pi.rdp; m.rec_pkt = pi.rpkt;
        m.doctets = pi.doctets;
        m.time = P.t;
        m.flags = pi.tflags;
    }
    out[li] = m;
}

// ---------------------------------------------------------------------------
// synthetic captures on the device
// ---------------------------------------------------------------------------
__global__ void k_synth_len(fluere_synth_cfg c, uint64_t first, uint64_t n, uint32_t* lens) {
    uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n) lens[j] = 16 + synth::frame_len(c, first + j);
}
__global__ void k_synth_write(fluere_synth_cfg c, uint64_t first, uint64_t n, uint8_t* bytes, const uint32_t* offs) {
    uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n) synth::write_record(c, first + j, bytes + offs[j]);
}


// test seam: insert canonical keys, return dense ids (flow dictionary checks)
__global__ void __launch_bounds__(256) k_dense_test(TableSet T, const uint32_t* keys, unsigned long long n,
                                                    uint32_t* out, uint32_t* slots) {
    unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    CKey k;
    for (int j = 0; j < 14; j++) k.w[j] = keys[i * 14 + j];
    out[i] = dense_of_key(T, k, true, slots, nullptr);
}

// test seam (fluere_debug_raw): one raw-fallback entry point of parse.h per
// byte string, exactly the device functions the parsers call
__global__ void __launch_bounds__(256) k_raw_probe(int fn, const uint8_t* bytes, const uint32_t* off, const uint32_t* len,
                                                   const uint32_t* arg, unsigned long long n, fluere_raw_hdr* out) {
    const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const G g{bytes + off[i]};
    const Span p{0, len[i]};
    RawHdr h;
    raw_new(h, 0, 0, 0, 0);
    bool some = false;
    switch (fn) {
    case FLUERE_RAW_FROM_RAW_PACKET: some = raw_from_raw_packet(g, p, arg[i] & 0xFF, h); break;
    case FLUERE_RAW_FROM_ETHERTYPE: some = raw_from_ethertype(g, p, arg[i] & 0xFFFF, h); break;
    case FLUERE_RAW_PARSE_ETHERTYPE: some = raw_parse_ethertype(g, p, arg[i] & 0xFFFF, h); break;
    case FLUERE_RAW_PARSE_PROTOCOL: some = raw_parse_protocol(g, p, arg[i] & 0xFF, h); break;
    case FLUERE_RAW_OPENVPN: some = raw_openvpn(g, p, h); break;
    case FLUERE_RAW_ICMP: some = raw_icmp(g, p, h); break;
    default: break;
    }
    fluere_raw_hdr r;
    memset(&r, 0, sizeof r);
    r.some = some;
    if (some) {
        r.has_src = h.has_src; r.has_dst = h.has_dst; r.ip_v6 = h.v6;
        for (int k = 0; k < 4; k++)
            for (int b = 0; b < 4; b++) {
                r.src[4 * k + b] = (uint8_t)(h.src[k] >> (24 - 8 * b));
                r.dst[4 * k + b] = (uint8_t)(h.dst[k] >> (24 - 8 * b));
            }
        r.src_port = h.sport; r.dst_port = h.dport; r.protocol = h.proto; r.length = h.length;
        r.has_flags = h.has_flags; r.flags = h.flags; r.has_version = h.has_version; r.version = h.version;
        r.has_ethertype = h.has_ethertype; r.ethertype = h.ethertype;
        r.has_payload = h.has_payload; r.payload_off = h.payload_off; r.payload_len = h.payload_len;
    }
    out[i] = r;
}



// Chunk descriptors (Batch::desc): one wave per chunk of 64 records.  Dense
// when the offsets are base + i * S with S in {16, 32, 48, 64, 80} and the
// chunk's span, read as 16-byte pieces from base, lies inside the readable
// buffer (nbytes + 80, the fluere_add_device_batch contract).
__global__ void __launch_bounds__(256) k_chunk_desc(const uint32_t* offs, uint64_t nbytes, uint64_t nd, uint2* desc) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint64_t ch = t / 64;
    const uint32_t lane = threadIdx.x & 63;
    if (ch >= nd) return;  // whole waves (blockDim is a multiple of 64)
    const uint32_t o = offs[ch * 64 + lane];
    const uint32_t base = __shfl(o, 0, 64), o1 = __shfl(o, 1, 64);
    const uint32_t S = o1 - base;
    const bool even = o == base + lane * S;
    const uint32_t npieces = (63u * S + 80u + 15u) / 16u;
    const bool dense = __all(even) && S >= 16u && S <= 80u && (S & 15u) == 0 &&
                       (uint64_t)base + 16ull * npieces <= nbytes + 80ull;
    if (lane == 0) desc[ch] = make_uint2(base, dense ? S : 0u);
}

// ---------------------------------------------------------------------------
// k_census: the shape of a newly attached capture, from a sample, for the
// choices its first run makes before any count exists (the hot kernel, the
// merge owner count, k_slow, the exact engine's filter words).  Reruns of the
// same batches use the last run's exact counts instead.
//   sample: one packet per stratum of n / s_n consecutive packets, at a hashed
//   position inside it (no aliasing with periodic flow assignments);
//   per sampled packet the hot parser, and for a keyed packet a 64-bit
//   fingerprint of its canonical key counted in an open-addressing table, so
//   the sample's distinct keys D and the keys seen once (f1) and twice (f2)
//   are maintained on the fly (count 0 -> 1: D, f1 up; 1 -> 2: f1 down, f2
//   up; 2 -> 3: f2 down).  The host extrapolates the capture's flow count
//   from them (census_flows).
// ---------------------------------------------------------------------------
struct CensusOut {
    unsigned long long seen, valid, slow, tcp, d, f1, f2, tmin, tmax;
};
constexpr uint32_t CENSUS_TBITS = 21;  // fingerprint table: 2^21 slots, >= 2x the largest sample
constexpr uint64_t CENSUS_MAX = 1ull << 20;
struct CensusArgs {
    Batch B;
    uint64_t s_n;  // samples of this batch
    unsigned long long* fp;
    uint32_t* cnt;
    CensusOut* out;
    int macs;
};
__global__ void __launch_bounds__(256) k_census(CensusArgs a) {
    __shared__ unsigned long long s_c[9];
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    if (tid < 9) s_c[tid] = tid == 7 ? NONE64 : 0ull;
    __syncthreads();
    const uint64_t j = (uint64_t)blockIdx.x * 256 + tid;
    const Batch& B = a.B;
    uint32_t cls = HOT_DROP, dd = 0, d1 = 0, d2 = 0;  // d1 / d2: +1, or -1 as 2
    bool tcp = false, live = j < a.s_n;
    unsigned long long t = 0;
    if (live) {
        const uint64_t lo = j * B.n / a.s_n, hi = (j + 1) * B.n / a.s_n;
        uint32_t r = (uint32_t)(j * 0x9E3779B97F4A7C15ull >> 32);
        r ^= r >> 15; r *= 0x2C1B3C6Du; r ^= r >> 12;
        const uint64_t li = lo + (hi > lo ? r % (uint32_t)(hi - lo) : 0u);
        // (clamped: the census may read a batch before the caller has
        // finished writing it -- only its predictions would be off)
        const uint32_t off = (uint32_t)min<uint64_t>(B.offs[li], B.nbytes);
        Win W;
        const uint8_t* p = B.bytes + off;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            uint4 q;
            __builtin_memcpy(&q, p + 16 * k, 16);
            W.w[4 * k + 0] = q.x; W.w[4 * k + 1] = q.y; W.w[4 * k + 2] = q.z; W.w[4 * k + 3] = q.w;
        }
        W.w[16] = W.w[17] = W.w[18] = W.w[19] = 0u;
        Hot h;
        cls = hot_parse(B, off, W, h);
        if (cls == HOT_OK) {
            tcp = h.proto == 6u;
            t = h.t;
            const uint32_t sp = h.ports >> 16, dp = h.ports & 0xFFFFu;
            bool gt = (h.sip > h.dip) | ((h.sip == h.dip) & (sp > dp));
            uint64_t mx = 0;
            if (a.macs) {  // the MAC pair joins the key (canonical order as in k_parse_agg<MACS>)
                const uint64_t dm = ((uint64_t)__builtin_amdgcn_perm(W.w[5], W.w[4], 0x00010203u) << 16) |
                                    __builtin_amdgcn_perm(W.w[5], W.w[4], 0x0C0C0405u);
                const uint64_t sm = ((uint64_t)__builtin_amdgcn_perm(W.w[6], W.w[5], 0x02030405u) << 16) |
                                    __builtin_amdgcn_perm(W.w[6], W.w[5], 0x0C0C0607u);
                if ((h.sip == h.dip) & (sp == dp)) gt = sm > dm;
                mx = (gt ? dm : sm) * 0xFF51AFD7ED558CCDull ^ (gt ? sm : dm);
            }
            const uint32_t k0 = gt ? h.dip : h.sip, k1 = gt ? h.sip : h.dip;
            const uint32_t k2 = gt ? __builtin_amdgcn_alignbit(h.ports, h.ports, 16) : h.ports;
            uint64_t f = ((uint64_t)k0 << 32 | k1) * 0x9E3779B97F4A7C15ull;
            f ^= ((uint64_t)k2 << 8 | h.proto) * 0xC2B2AE3D27D4EB4Full;
            f ^= mx * 0x165667B19E3779F9ull;
            f ^= f >> 29; f *= 0xBF58476D1CE4E5B9ull; f ^= f >> 32;
            f |= 1ull;  // (0 marks an empty slot)
            const uint32_t mask = (1u << CENSUS_TBITS) - 1;
            uint32_t e = (uint32_t)(f >> 40) & mask;
            for (int probe = 0; probe < 256; probe++) {
                const unsigned long long v = atomicCAS(&a.fp[e], 0ull, (unsigned long long)f);
                if (v == 0ull || v == f) {
                    const uint32_t old = atomicAdd(&a.cnt[e], 1u);
                    dd = old == 0;
                    d1 = old == 0 ? 1u : old == 1 ? 2u : 0u;
                    d2 = old == 1 ? 1u : old == 2 ? 2u : 0u;
                    break;
                }
                e = (e + 1) & mask;
            }
        }
    }
    // wave totals (ballots), then one LDS add per wave and counter
    const unsigned long long v[7] = {
        (unsigned long long)__popcll(__ballot(live)), (unsigned long long)__popcll(__ballot(cls == HOT_OK && live)),
        (unsigned long long)__popcll(__ballot(cls == HOT_SLOW && live)), (unsigned long long)__popcll(__ballot(tcp)),
        (unsigned long long)__popcll(__ballot(dd != 0)),
        (unsigned long long)__popcll(__ballot(d1 == 1)) - (unsigned long long)__popcll(__ballot(d1 == 2)),
        (unsigned long long)__popcll(__ballot(d2 == 1)) - (unsigned long long)__popcll(__ballot(d2 == 2))};
    unsigned long long tmn = (cls == HOT_OK && live) ? t : NONE64, tmx = (cls == HOT_OK && live) ? t : 0ull;
    for (int o = 32; o > 0; o >>= 1) {
        tmn = min(tmn, (unsigned long long)__shfl_xor(tmn, o, 64));
        tmx = max(tmx, (unsigned long long)__shfl_xor(tmx, o, 64));
    }
    if (lane == 0) {
        for (int k = 0; k < 7; k++)
            if (v[k]) atomicAdd(&s_c[k], v[k]);
        atomicMin(&s_c[7], tmn);
        atomicMax(&s_c[8], tmx);
    }
    __syncthreads();
    if (tid < 7 && s_c[tid]) atomicAdd(&a.out->seen + tid, s_c[tid]);
    if (tid == 7 && s_c[7] != NONE64) atomicMin(&a.out->tmin, s_c[7]);
    if (tid == 8 && s_c[8]) atomicMax(&a.out->tmax, s_c[8]);
}

}  // namespace

static unsigned long long* g_hot_dbg = nullptr;  // FLUERE_DEBUG: per-workgroup hot-kernel timestamps


// 512 B of private memory a lane, 1024-thread workgroups: more than any
// kernel of a run uses (k_merge_partials 304 B, k_compose 440 B); stores
// nothing (n is never 1)
__global__ void __launch_bounds__(1024) k_scratch_warm(uint8_t* out, uint32_t n) {
    volatile uint32_t buf[128];
    for (uint32_t i = 0; i < 128; i++) buf[(i * 7u + threadIdx.x) & 127u] = i;
    if (n == 1u) out[threadIdx.x] = (uint8_t)buf[threadIdx.x & 127u];
}

// the record counters of a run, zeroed by one launch (eight 8-byte memsets
// cost a host submission each while the GPU waits for them)
__global__ void k_reset_records(Glob* g) {
    if (threadIdx.x) return;
    g->n_rec = 0;
    g->n_complex = 0;
    g->n_complex_pkts = 0;
    g->n_heads = 0;
    g->n_updates = 0;
    g->n_ended = 0;
    g->n_fdefer = 0;
    g->n_okey = 0;
    g->n_bare = 0;
}
void reset_record_counters(fluere_ctx* c) {
    k_reset_records<<<1, 64, 0, c->stream>>>(c->d_glob);
}

// Host copy of device-resident records, ended prefix first in emission order
// (order_key: global index of the closing packet; with order words, sharded
// Mode B: then aux[0], aux[1]), then active flows.  After a one-GPU run the
// device has ordered the ended prefix already (order_records): only the
// active flows are sorted here, by first packet -- the reference emits them
// after its loop (offline_fluereflows.rs:182-191) in HashMap order, so any
// order is the reference's; this one is deterministic.
int fetch_records(fluere_ctx* c) {
    if (c->host_recs) return FLUERE_OK;
    static const bool hostprof = getenv("FLUERE_HOSTPROF") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    hipStream_t s = c->stream;
    const uint64_t n = c->dev_n_rec;
    c->recs.resize(n);
    c->aux.assign(c->has_aux ? 2 * n : 0, 0ull);
    // many active flows after a device ordering: sorted by first packet on the
    // device (stable radix sort, the host sort's order), into d_recs2
    const uint64_t ne0 = c->dev_ordered ? std::min<uint64_t>(c->dev_ordered_ended, n) : 0;
    const bool dev_act = c->dev_ordered && !c->has_aux && n - ne0 >= 4096 && sort_actives(c, ne0, n - ne0) == FLUERE_OK;
    if (dev_act) {
        if (ne0) HIPCHECK(hipMemcpyAsync(c->recs.data(), c->d_recs, ne0 * sizeof(fluere_record), hipMemcpyDeviceToHost, s));
        HIPCHECK(hipMemcpyAsync(c->recs.data() + ne0, c->d_recs2, (n - ne0) * sizeof(fluere_record), hipMemcpyDeviceToHost, s));
        HIPCHECK(ctx_sync(c));
        if (hostprof)
            fprintf(stderr, "[fluere] records: %llu to the host (%llu actives sorted on the device) %.1f ms\n",
                    (unsigned long long)n, (unsigned long long)(n - ne0),
                    1e3 * std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
        c->n_ended = ne0;
        c->host_recs = true;
        return FLUERE_OK;
    }
    if (n)
        HIPCHECK(hipMemcpyAsync(c->recs.data(), c->d_recs, n * sizeof(fluere_record), hipMemcpyDeviceToHost, s));
    if (n && c->has_aux)
        HIPCHECK(hipMemcpyAsync(c->aux.data(), c->d_recaux, 2 * n * 8, hipMemcpyDeviceToHost, s));
    HIPCHECK(ctx_sync(c));
    if (hostprof)
        fprintf(stderr, "[fluere] records: %llu to the host %.1f ms\n", (unsigned long long)n,
                1e3 * std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    if (c->dev_ordered) {
        const uint64_t ne = std::min<uint64_t>(c->dev_ordered_ended, n);
        auto& R = c->recs;
        std::vector<uint64_t> ix(n - ne);
        for (uint64_t i = 0; i < n - ne; i++) ix[i] = ne + i;
        std::stable_sort(ix.begin(), ix.end(), [&](uint64_t a, uint64_t b) { return R[a].first < R[b].first; });
        std::vector<fluere_record> act(n - ne);
        for (uint64_t i = 0; i < n - ne; i++) act[i] = R[ix[i]];
        std::copy(act.begin(), act.end(), R.begin() + ne);
        if (c->has_aux) {
            std::vector<unsigned long long> xa(2 * (n - ne));
            for (uint64_t i = 0; i < n - ne; i++) { xa[2 * i] = c->aux[2 * ix[i]]; xa[2 * i + 1] = c->aux[2 * ix[i] + 1]; }
            std::copy(xa.begin(), xa.end(), c->aux.begin() + 2 * ne);
        }
        c->n_ended = ne;
        c->host_recs = true;
        return FLUERE_OK;
    }
    std::vector<uint64_t> ix(n);
    for (uint64_t i = 0; i < n; i++) ix[i] = i;
    const auto& R = c->recs;
    const auto& X = c->aux;
    const bool ax = c->has_aux;
    std::stable_sort(ix.begin(), ix.end(), [&](uint64_t a, uint64_t b) {
        if (R[a].order_key != R[b].order_key) return R[a].order_key < R[b].order_key;
        if (ax && X[2 * a] != X[2 * b]) return X[2 * a] < X[2 * b];
        if (ax && X[2 * a + 1] != X[2 * b + 1]) return X[2 * a + 1] < X[2 * b + 1];
        return R[a].first < R[b].first;
    });
    std::vector<fluere_record> r2(n);
    std::vector<unsigned long long> x2(X.size());
    for (uint64_t i = 0; i < n; i++) {
        r2[i] = R[ix[i]];
        if (ax) { x2[2 * i] = X[2 * ix[i]]; x2[2 * i + 1] = X[2 * ix[i] + 1]; }
    }
    c->recs.swap(r2);
    c->aux.swap(x2);
    uint64_t ne = 0;
    for (auto& r : c->recs) if (r.order_key != NONE64) ne++;
    c->n_ended = ne;
    c->host_recs = true;
    return FLUERE_OK;
}


TableSet tables_of(fluere_ctx* c) {
    TableSet T;
    for (int t = 0; t < N_TABLES; t++) T.tab[t] = c->d_tab + (size_t)t * 2 * (c->C + 1);
    T.C = c->C;
    // (FLUERE_WIDE_TABLES: tests force the wide layout on small tables)
    T.wide = (c->C >= (1u << 24) || getenv("FLUERE_WIDE_TABLES") != nullptr) ? 1u : 0u;
    T.fmax = c->fmax;
    T.n_flows = c->d_nflows;
    T.err = c->d_nflows + 1;
    T.flow_key = c->d_flow_key;
    return T;
}

extern "C" int fluere_abi_version(void) { return FLUERE_ABI_VERSION; }

// The dictionary and the per-flow state for up to mf flows, empty: every
// table EMPTY, the accumulators at their identities (what k_cleanup leaves).
int alloc_flow_state(fluere_ctx* c, uint64_t mf) {
    uint32_t C = 1u << 16;
    while (C < 2 * mf && C < MAX_TABLE_SLOTS) C <<= 1;
    c->C = C;
    c->fmax = (uint32_t)std::min<uint64_t>(std::min<uint64_t>(mf, C), MAX_FLOWS);
    const size_t tab_words = (size_t)N_TABLES * 2 * (C + 1);
    if (hipMalloc(&c->d_tab, tab_words * 8) != hipSuccess) return FLUERE_E_NOMEM;
    const size_t F = c->fmax;
    const size_t acc_bytes = F * (4 * 2 + 8 * 2 + 4 * 4 + 4 * 8 + 8 * 4 + 4 * N_TABLES);
    if (hipMalloc(&c->d_acc, acc_bytes) != hipSuccess) return FLUERE_E_NOMEM;
    char* p = (char*)c->d_acc;
    auto take = [&](size_t bytes) { char* r = p; p += bytes; return r; };
    for (int q = 0; q < 2; q++) c->acc.by[q] = (unsigned long long*)take(F * 8);
    c->acc.fa = (unsigned long long*)take(F * 8);
    c->acc.fc = (unsigned long long*)take(F * 8);
    c->acc.fr = (unsigned long long*)take(F * 8);
    c->acc.la = (unsigned long long*)take(F * 8);
    for (int q = 0; q < 2; q++) c->acc.pk[q] = (uint32_t*)take(F * 4);
    for (int q = 0; q < 2; q++) c->acc.mn[q] = (uint32_t*)take(F * 4);
    for (int q = 0; q < 2; q++) c->acc.mx[q] = (uint32_t*)take(F * 4);
    for (int q = 0; q < 8; q++) c->acc.fl[q] = (uint32_t*)take(F * 4);
    c->acc.slots = (uint32_t*)take(F * 4 * N_TABLES);
    if (hipMalloc(&c->d_flow_key, F * 56) != hipSuccess) return FLUERE_E_NOMEM;
    if (hipMalloc(&c->d_complex, F) != hipSuccess) return FLUERE_E_NOMEM;
    if (hipMalloc(&c->d_fdefer, F * 4) != hipSuccess) return FLUERE_E_NOMEM;
    hipStream_t s = c->stream;
    k_fill_u64<<<grid_for(tab_words, 256), 256, 0, s>>>(c->d_tab, tab_words, EMPTY);
    k_fill_u64<<<grid_for(4 * F, 256), 256, 0, s>>>(c->acc.fa, 4 * F, NONE64);
    k_fill_u64<<<grid_for(F, 256), 256, 0, s>>>(c->acc.la, F, 0);
    k_fill_u64<<<grid_for(2 * F, 256), 256, 0, s>>>(c->acc.by[0], 2 * F, 0);
    k_fill_u32<<<grid_for(2 * F, 256), 256, 0, s>>>(c->acc.pk[0], 2 * F, 0);
    k_fill_u32<<<grid_for(2 * F, 256), 256, 0, s>>>(c->acc.mn[0], 2 * F, NONE32);
    k_fill_u32<<<grid_for(2 * F, 256), 256, 0, s>>>(c->acc.mx[0], 2 * F, 0);
    k_fill_u32<<<grid_for(8 * F, 256), 256, 0, s>>>(c->acc.fl[0], 8 * F, 0);
    k_fill_u32<<<grid_for(F * N_TABLES, 256), 256, 0, s>>>(c->acc.slots, F * N_TABLES, NONE32);
    HIPCHECK(hipMemsetAsync(c->d_complex, 0, F, s));
    HIPCHECK(hipGetLastError());
    return FLUERE_OK;
}

void free_flow_state(fluere_ctx* c) {
    hipFree(c->d_tab);
    hipFree(c->d_acc);
    hipFree(c->d_flow_key);
    hipFree(c->d_complex);
    hipFree(c->d_fdefer);
    c->d_tab = nullptr;
    c->d_acc = nullptr;
    c->d_flow_key = nullptr;
    c->d_complex = nullptr;
    c->d_fdefer = nullptr;
    // the lazily sized per-flow arrays follow the new capacity
    for (void** q : {(void**)&c->d_active, (void**)&c->d_pay, (void**)&c->d_annex_of, (void**)&c->d_sumpos}) {
        hipFree(*q);
        *q = nullptr;
    }
}

extern "C" int fluere_open(const fluere_opts* o, fluere_ctx** out) {
    if (!out) return FLUERE_E_ARG;
    *out = nullptr;
    fluere_ctx* c = new (std::nothrow) fluere_ctx();
    if (!c) return FLUERE_E_NOMEM;
    fluere_opts def{};
    def.timeout_ms = 600000;
    if (!o) o = &def;
    c->device = o->device;
    c->timeout_ms = o->timeout_ms;
    c->use_mac = o->use_mac ? 1 : 0;
    const uint64_t mf = o->max_flows ? o->max_flows : (1ull << 21);
    int rc = FLUERE_OK;
    auto fail = [&](int r) { rc = r; fluere_close(c); return r; };
    if (hipSetDevice(c->device) != hipSuccess) return fail(FLUERE_E_HIP);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, c->device) == hipSuccess) c->n_cu = std::min(prop.multiProcessorCount, MB);  // (slow-list regions: one per hot workgroup, <= MB)
    if (o->stream) c->stream = (hipStream_t)o->stream;
    else {
        if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return fail(FLUERE_E_HIP);
        c->own_stream = true;
    }
    if ((rc = alloc_flow_state(c, mf))) return fail(rc);
    if (hipMalloc(&c->d_glob, sizeof(Ctl) + sizeof(OkeyRef)) != hipSuccess) return fail(FLUERE_E_NOMEM);
    c->d_nflows = &reinterpret_cast<Ctl*>(c->d_glob)->n_flows;
    if (hipHostMalloc(&c->h_ctl, sizeof(Ctl)) != hipSuccess) return fail(FLUERE_E_NOMEM);
    memset(c->h_ctl, 0, sizeof(Ctl));
    if (hipHostMalloc(&c->h_mail, sizeof(HostMail)) != hipSuccess) return fail(FLUERE_E_NOMEM);
    memset(c->h_mail, 0, sizeof(HostMail));
    if (hipMalloc(&c->d_cbits, 1u << CBITS_LOG2) != hipSuccess) return fail(FLUERE_E_NOMEM);
    if (hipMalloc(&c->d_bctr, 8 * 8 * sizeof(unsigned long long)) != hipSuccess) return fail(FLUERE_E_NOMEM);
    if (hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
        hipEventCreate(&c->ev2) != hipSuccess ||
        hipEventCreate(&c->ev_ctl) != hipSuccess)
        return fail(FLUERE_E_HIP);
    // the hot kernels' timing events (carried by their dispatches): timing
    // only, so no system-scope fence when they are recorded -- with it the
    // stop event wrote back and invalidated the caches behind the hot kernel
    // (FLUERE_EV_FENCE=1: the default events, A/B)
    static const bool ev_fence = getenv("FLUERE_EV_FENCE") && atoi(getenv("FLUERE_EV_FENCE")) != 0;
    for (hipEvent_t& e : c->evh)
        if (hipEventCreateWithFlags(&e, ev_fence ? hipEventDefault : hipEventDisableSystemFence) != hipSuccess)
            return fail(FLUERE_E_HIP);
    hipStream_t s = c->stream;
    if (hipMemsetAsync(c->d_cbits, 0, 1u << CBITS_LOG2, s) != hipSuccess) return fail(FLUERE_E_HIP);
    // the stream's scratch (private memory) backing, sized now: the first
    // kernel that needs more than the queue has (the merge, 304 B a lane)
    // otherwise waits ~130 us in the first run for the runtime to grow it
    k_scratch_warm<<<1, 1024, 0, s>>>(c->d_cbits, 0u);
    if (hipGetLastError() != hipSuccess) return fail(FLUERE_E_HIP);
    {
        Ctl z{};
        z.g.tmin = NONE64;
        if (hipMemcpyAsync(c->d_glob, &z, sizeof z, hipMemcpyHostToDevice, s) != hipSuccess) return fail(FLUERE_E_HIP);
        if (hipMemsetAsync((char*)c->d_glob + sizeof(Ctl), 0, sizeof(OkeyRef), s) != hipSuccess) return fail(FLUERE_E_HIP);
    }
    if (hipStreamSynchronize(s) != hipSuccess) return fail(FLUERE_E_HIP);
    // the state above is what k_cleanup leaves: the first pass needs none
    c->precleaned = true;
    c->prev_nf = 0;
    (void)rc;
    *out = c;
    return FLUERE_OK;
}

// More flows than the context holds (the census's estimate): the reference's
// HashMap has no bound (offline_fluereflows.rs:61), so the dictionary and the
// per-flow state are reallocated, empty, for the estimate with headroom, up
// to MAX_FLOWS (2^26 flows; tables of 2^27 slots, ~40 GB of HBM).  Called
// between passes only (the flow state holds no results).
int grow_flow_state(fluere_ctx* c, uint64_t want) {
    const uint64_t mf = std::min<uint64_t>(std::max<uint64_t>(want, (uint64_t)c->fmax * 2), MAX_FLOWS);
    if (mf <= c->fmax) return FLUERE_OK;
    HIPCHECK(ctx_sync(c));
    // the larger state is allocated before the current one is released: when
    // HBM cannot hold it, the context keeps its capacity (a run that then
    // overflows reports FLUERE_E_TABLE_FULL, as without the growth)
    fluere_ctx old = {};
    old.d_tab = c->d_tab; old.d_acc = c->d_acc; old.d_flow_key = c->d_flow_key;
    old.d_complex = c->d_complex; old.d_fdefer = c->d_fdefer;
    const Acc acc = c->acc;
    const uint32_t C = c->C, fmax = c->fmax;
    c->d_tab = nullptr; c->d_acc = nullptr; c->d_flow_key = nullptr; c->d_complex = nullptr; c->d_fdefer = nullptr;
    const int rc = alloc_flow_state(c, mf);
    fluere_ctx* drop = rc ? c : &old;  // the state to free: the failed new one, or the old one
    hipFree(drop->d_tab);
    hipFree(drop->d_acc);
    hipFree(drop->d_flow_key);
    hipFree(drop->d_complex);
    hipFree(drop->d_fdefer);
    if (rc) {
        (void)hipGetLastError();
        c->d_tab = old.d_tab; c->d_acc = old.d_acc; c->d_flow_key = old.d_flow_key;
        c->d_complex = old.d_complex; c->d_fdefer = old.d_fdefer;
        c->acc = acc;
        c->C = C;
        c->fmax = fmax;
        return FLUERE_OK;
    }
    // the lazily sized per-flow arrays follow the new capacity
    for (void** q : {(void**)&c->d_active, (void**)&c->d_pay, (void**)&c->d_annex_of, (void**)&c->d_sumpos}) {
        hipFree(*q);
        *q = nullptr;
    }
    c->precleaned = true;  // (alloc_flow_state's fills are what a cleanup leaves)
    c->prev_nf = 0;
    c->last_nf = std::min<uint64_t>(c->last_nf, c->fmax);
    return FLUERE_OK;
}

void free_batches(fluere_ctx* c) {
    for (auto& hb : c->batches) {
        if (hb.own_bytes) hipFree(hb.own_bytes);
        if (hb.own_offs) hipFree(hb.own_offs);
        if (hb.own_desc) hipFree(hb.own_desc);
    }
    c->batches.clear();
    c->n_total = 0;
    c->batches_dirty = true;
    c->census_due = true;
}

extern "C" int fluere_close(fluere_ctx* c) {
    if (!c) return FLUERE_OK;
    if (c->stream) hipStreamSynchronize(c->stream);
    free_batches(c);
    free_flow_state(c);
    if (c->h_ctl) hipHostFree(c->h_ctl);
    if (c->h_mail) hipHostFree(c->h_mail);
    hipFree(c->d_glob);
    hipFree(c->d_cbits);
    hipFree(c->d_bctr);
    hipFree(c->d_phash);
    hipFree(c->d_emap);
    hipFree(c->d_batches);
    hipFree(c->d_recs);
    hipFree(c->d_slow);
    hipFree(c->d_stage);
    hipFree(c->d_exact);
    hipFree(c->d_annex);
    hipFree(c->d_wire_tmp);
    hipFree(c->d_v6map);
    hipFree(c->ar_d);
    hipFree(c->ar_offs);
    for (int i = 0; i < 8; i++) {
        if (c->ar_pin[i]) hipHostFree(c->ar_pin[i]);
        if (c->ar_ev[i]) hipEventDestroy(c->ar_ev[i]);
    }
    hipFree(c->d_need);
    hipFree(c->d_census);
    hipFree(c->d_recs2);
    hipFree(c->d_recaux2);
    hipFree(c->d_ord);
    so_free(c);
    hipFree(c->d_recaux);
    hipFree(c->d_okey);
    sweep_free(c);
    merge_pending_free(c);
    hipFree(c->d_exm);
    hipFree(c->d_exm_t);
    hipFree(c->d_sd);
    if (c->ev0) hipEventDestroy(c->ev0);
    if (c->ev1) hipEventDestroy(c->ev1);
    if (c->ev2) hipEventDestroy(c->ev2);
    for (hipEvent_t e : c->evh)
        if (e) hipEventDestroy(e);
    if (c->ev_ctl) hipEventDestroy(c->ev_ctl);
    if (c->graph) hipGraphExecDestroy(c->graph);
    free(c->graph_plan);
    if (c->own_stream && c->stream) hipStreamDestroy(c->stream);
    delete c;
    return FLUERE_OK;
}

// Clear flow state touched by the previous run (O(flows), not O(capacity)).
// Reset the flows of the previous run on the device (no host round trip):
// k_cleanup reads the flow count and the error word itself.
unsigned flow_grid(fluere_ctx* c) {
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(grid_for(c->fmax, 256), (uint64_t)c->n_cu * 16));
}
// Grid of the per-flow kernels that end on a done-counter (k_cleanup,
// k_finalize): grid-stride over n flows with at most 4 workgroups per CU, so
// a million-flow run counts ~1k workgroups done on the one word, not ~4k.
unsigned done_grid(fluere_ctx* c, uint64_t n) {
    static const uint64_t wpc = getenv("FLUERE_DONE_WPC") ? std::max(1, atoi(getenv("FLUERE_DONE_WPC"))) : 4;  // (A/B)
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(grid_for(n, 256), (uint64_t)c->n_cu * wpc));
}

// Sequential clear of the IPv4 chain's tables when the flows to clear would
// cost more as random 16-byte writes (two per flow) than 32 (C + 1) bytes
// written in order: more than (C + 1) / 16 flows.
int bulk_clean(const fluere_ctx* c, uint64_t nf) {
    static const int env = getenv("FLUERE_BULK_CLEAN") ? atoi(getenv("FLUERE_BULK_CLEAN")) : -1;
    if (env >= 0) return env;
    return nf != ~0ull && nf > ((uint64_t)c->C + 1) / 16 ? 1 : 0;
}

// Clears the flows of the last run and re-initialises every run counter
// (one launch; see k_cleanup).
int clear_flows(fluere_ctx* c) {
    hipStream_t s = c->stream;
    (void)hipGetLastError();
    CleanArgs a{tables_of(c), c->acc, c->d_complex, c->d_active, c->d_glob};
    static const int clean_abl = diag_knob("FLUERE_CLEAN_ABL");
    a.abl = clean_abl;
    a.bulk = bulk_clean(c, c->prev_nf == ~0ull ? c->last_nf : c->prev_nf);
    // grid: the last fetched run's flow count when known (k_cleanup is
    // grid-stride over the device count, so any grid is correct)
    const unsigned g = done_grid(c, c->prev_nf == ~0ull ? c->fmax : c->prev_nf);
    k_cleanup<<<g, 256, 0, s>>>(a, (size_t)N_TABLES * 2 * (c->C + 1));
    c->prev_nf = ~0ull;
    HIPCHECK(hipGetLastError());
    return FLUERE_OK;
}

// Poll the pinned host copy until the last kernel has published run seq
// (publish_ctl); now and then ask whether the stream failed instead.
int wait_published(fluere_ctx* c, uint32_t seq, Glob& g, uint32_t (&nf_err)[2]) {
    volatile uint32_t* seqp = &c->h_ctl->seq;
    if (__atomic_load_n(seqp, __ATOMIC_ACQUIRE) != seq) c->host_waits++;
    static const uint32_t qmask = getenv("FLUERE_QUERY_MASK") ? (uint32_t)atoi(getenv("FLUERE_QUERY_MASK")) : 65535u;
    for (uint32_t spin = 1;; spin++) {
        if (__atomic_load_n(seqp, __ATOMIC_ACQUIRE) == seq) break;
        if ((spin & qmask) == 0) {  // now and then (~ms): did the stream fail instead?
            const hipError_t q = hipStreamQuery(c->stream);
            if (q == hipErrorNotReady) continue;
            if (__atomic_load_n(seqp, __ATOMIC_ACQUIRE) == seq) break;
            HIPCHECK(q);
            return FLUERE_E_HIP;  // the stream finished without publishing: cannot happen
        }
    }
    g = c->h_ctl->g;
    nf_err[0] = c->h_ctl->n_flows;
    nf_err[1] = c->h_ctl->err;
    c->prev_nf = (nf_err[1] & (ERR_TABLE_FULL | ERR_SPIN)) ? ~0ull : nf_err[0];
    return FLUERE_OK;
}

// The run counters to the pinned host copy, stream-ordered (one wave: the
// words, the wave's system-scope fence, then seq), read by polling: no copy
// kernel and no blocking stream sync on the way back.
__global__ void __launch_bounds__(64) k_publish(const Glob* g, Ctl* host_ctl, uint32_t seq) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(g);
    uint32_t* dst = reinterpret_cast<uint32_t*>(host_ctl);
    constexpr uint32_t nw = offsetof(Ctl, seq) / 4;
    for (uint32_t i = threadIdx.x; i < nw; i += 64)
        __hip_atomic_store(dst + i, src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __threadfence_system();
    if (threadIdx.x == 0) __hip_atomic_store(&host_ctl->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

int read_glob(fluere_ctx* c, Glob& g) {
    const uint32_t seq = ++c->run_seq ? c->run_seq : ++c->run_seq;  // never 0
    k_publish<<<1, 64, 0, c->stream>>>(c->d_glob, c->h_ctl, seq);
    HIPCHECK(hipGetLastError());
    uint32_t nf_err[2];
    return wait_published(c, seq, g, nf_err);
}

extern "C" int fluere_reset(fluere_ctx* c) {
    if (!c) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    int rc = clear_flows(c);
    if (rc) return rc;
    HIPCHECK(ctx_sync(c));
    free_batches(c);
    c->recs.clear();
    c->have_results = false;
    return FLUERE_OK;
}

extern "C" int fluere_add_device_batch(fluere_ctx* c, const uint8_t* d_bytes, uint64_t nbytes,
                                       const uint32_t* d_offsets, uint64_t n, uint32_t snaplen, int swapped,
                                       int nsec_ts) {
    if (!c || (!d_bytes && n) || (!d_offsets && n) || nbytes >= (1ull << 32)) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    HostBatch hb;
    hb.b.bytes = d_bytes;
    hb.b.offs = d_offsets;
    hb.b.nbytes = nbytes;
    hb.b.n = n;
    hb.b.first = c->index_base + c->n_total;
    hb.b.snap = snaplen ? snaplen : 262144;
    hb.b.flags = (swapped ? 1u : 0u) | (nsec_ts ? 2u : 0u);
    c->batches.push_back(hb);
    c->batches_dirty = true;
    c->census_due = true;
    c->n_total += n;
    c->have_results = false;
    return prepare_capture(c);

}
int upload_batches(fluere_ctx* c) {
    if (!c->batches_dirty) return FLUERE_OK;
    c->batches_dirty = false;
    int nb = (int)c->batches.size();
    // chunk descriptors of batches attached since the last pass (index data,
    // like the offsets: built once per attached batch, from the offsets)
    for (auto& hb : c->batches) {
        const uint64_t nd = hb.b.n / 64;
        if (hb.b.desc || !nd) continue;
        if (hipMalloc(&hb.own_desc, nd * sizeof(uint2)) != hipSuccess) return FLUERE_E_NOMEM;
        k_chunk_desc<<<grid_for(nd * 64, 256), 256, 0, c->stream>>>(hb.b.offs, hb.b.nbytes, nd, hb.own_desc);
        HIPCHECK(hipGetLastError());
        hb.b.desc = hb.own_desc;
        hb.b.n_desc = nd;
    }
    if (nb > c->d_batches_cap) {
        hipFree(c->d_batches);
        c->d_batches = nullptr;
        int cap = std::max(16, nb);
        if (hipMalloc(&c->d_batches, sizeof(Batch) * cap) != hipSuccess) return FLUERE_E_NOMEM;
        c->d_batches_cap = cap;
    }
    std::vector<Batch> hb(nb);
    for (int i = 0; i < nb; i++) hb[i] = c->batches[i].b;
    if (nb) HIPCHECK(hipMemcpyAsync(c->d_batches, hb.data(), sizeof(Batch) * nb, hipMemcpyHostToDevice, c->stream));
    return FLUERE_OK;
}

// The capture's flow count from the census sample: D distinct keys among s of
// its N packets, f1 / f2 of them seen once / twice.  Chao's estimator for a
// sample drawn without replacement (q = s / N): F = D + f1^2 / (2 f2 s / (s - 1)
// + f1 q / (1 - q)); the whole capture (q = 1) gives D itself.
static uint64_t census_flows(uint64_t s, uint64_t N, double D, double f1, double f2) {
    if (s >= N || s < 2) return (uint64_t)D;
    const double q = (double)s / (double)N;
    const double den = 2.0 * f2 * (double)s / (double)(s - 1) + f1 * q / (1.0 - q);
    const double F = D + (den > 0 ? f1 * f1 / den : 0.0);
    return (uint64_t)std::min<double>(F + 0.5, (double)N);
}

// Census of newly attached batches (k_census; one host round trip, first pass
// after an attach only): sets the predictions a pass plans with -- the flow
// count (hot kernel, owners, grids), slow packets (k_slow), TCP in Mode A (the
// exact engine's filter words).  Live sessions keep the last batch's counts.
// FLUERE_CENSUS=0 disables it (A/B), =1 runs it before every pass (tests).
int census(fluere_ctx* c) {
    static const int env = getenv("FLUERE_CENSUS") ? atoi(getenv("FLUERE_CENSUS")) : -1;
    if (env == 1) c->census_due = true;
    if (!c->census_due || env == 0) return FLUERE_OK;
    c->census_due = false;
    if (c->reuse_ingest && c->runs > 0 && env != 1) return FLUERE_OK;
    const uint64_t N = c->n_total;
    if (!N) return FLUERE_OK;
    const uint64_t S = std::min<uint64_t>(N, CENSUS_MAX);
    hipStream_t s = c->stream;
    const size_t T = (size_t)1 << CENSUS_TBITS;
    if (!c->d_census && hipMalloc(&c->d_census, T * 12 + sizeof(CensusOut) + 64) != hipSuccess) return FLUERE_E_NOMEM;
    CensusArgs a{};
    a.fp = (unsigned long long*)c->d_census;
    a.cnt = (uint32_t*)(a.fp + T);
    a.out = (CensusOut*)(a.cnt + T);
    a.macs = c->use_mac;
    HIPCHECK(hipMemsetAsync(c->d_census, 0, T * 12 + sizeof(CensusOut), s));
    HIPCHECK(hipMemsetAsync(&a.out->tmin, 0xFF, 8, s));
    uint64_t done = 0, seen_n = 0;
    for (size_t i = 0; i < c->batches.size(); i++) {
        const Batch& B = c->batches[i].b;
        if (!B.n) continue;
        seen_n += B.n;
        const uint64_t upto = seen_n == N ? S : (uint64_t)((double)S * seen_n / N);
        a.B = B;
        a.s_n = std::min<uint64_t>(B.n, upto > done ? upto - done : 0);
        done += a.s_n;
        if (a.s_n) k_census<<<grid_for(a.s_n, 256), 256, 0, s>>>(a);
    }
    HIPCHECK(hipGetLastError());
    const void* src[9];
    int by[9];
    for (int k = 0; k < 9; k++) { src[k] = &a.out->seen + k; by[k] = 8; }
    unsigned long long v[9] = {};
    int rc = mail_fetch(c->h_mail, s, 9, src, by, v);
    if (rc) return rc;
    const uint64_t s_seen = v[0];
    const uint64_t F = census_flows(s_seen, N, (double)v[4], (double)v[5], (double)v[6]);
    for (int k = 0; k < 9; k++) c->census_v[k] = v[k];
    c->census_v[9] = F;
    c->census_ran++;
    // more flows than the context holds: grow it before the pass (live
    // sessions keep their capacity: their state is sized by it)
    if (!c->reuse_ingest && F + F / 4 > c->fmax && c->fmax < MAX_FLOWS && !getenv("FLUERE_NO_GROW")) {
        if ((rc = grow_flow_state(c, F + F / 2))) return rc;
    }
    // the predictions (the same fields a finished run sets)
    c->last_nf = std::min<uint64_t>(F, c->fmax);
    c->last_n_slow = v[2] ? std::max<uint64_t>(1, v[2] * N / std::max<uint64_t>(1, s_seen)) : 0;
    c->last_mode_b = (v[1] && v[8] >= v[7] && v[8] - v[7] >= c->timeout_ms * 1000ull) ? 1 : 0;
    c->last_n_complex = v[3] ? 1 : 0;  // TCP keys: flows the certificate may reject (filter words, 4 B/packet)
    return FLUERE_OK;
}

extern "C" int fluere_last_census(fluere_ctx* c, uint64_t* out, int n) {
    if (!c || !out || n < 0) return FLUERE_E_ARG;
    for (int k = 0; k < n && k < 10; k++) out[k] = c->census_v[k];
    return c->census_ran;
}

extern "C" int fluere_parse_batch(fluere_ctx* c, fluere_pkt_meta* d_out, uint64_t cap) {
    if (!c || !d_out || cap < c->n_total) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    const char* m = getenv("FLUERE_PARSE_MODE");
    int mode = (m && m[0] == '1') ? 1 : 0;
    for (auto& hb : c->batches) {
        if (!hb.b.n) continue;
        k_parse_batch<<<grid_for(hb.b.n, 256), 256, 0, c->stream>>>(hb.b, d_out + hb.b.first, mode);
    }
    HIPCHECK(hipGetLastError());
    HIPCHECK(ctx_sync(c));
    return FLUERE_OK;
}

// A pass = k_cleanup -> per batch (k_parse_agg, k_merge_partials) -> k_finalize
// -> one device->host copy of the run counters.  plan_pass does every
// allocation and computes every launch argument; enqueue_pass only launches,
// so a pass can be captured into a hipGraph and replayed while its plan is
// unchanged (byte-equal).
constexpr int PLAN_BATCHES = 8;
static_assert(sizeof(fluere_ctx::evh) == 2 * PLAN_BATCHES * sizeof(hipEvent_t), "a start / stop event pair per batch");
struct PassPlan {
    CleanArgs ca;
    unsigned clean_grid;
    size_t tab_words;
    int nb;
    AggArgs agg[PLAN_BATCHES];
    unsigned agg_grid[PLAN_BATCHES];
    uint32_t owners[PLAN_BATCHES];
    uint32_t slow_grid[PLAN_BATCHES];  // k_slow workgroups (its sets); 0: the merge tail takes the slow list
    int macs, abl;
    int spill;     // 1: the hot pass is k_parse_spill (many flows per window), not k_parse_agg
    int lean_merge;  // 1: runs without partials merge their owners in k_merge_spill (0: k_merge_partials, A/B)
    int one_merge;   // 1: one k_merge_spill over every batch of the pass (after all the hot passes)
    int exm;         // 1: k_parse_spill writes every packet's ExMeta (Mode B predicted: AggArgs::exm)
    int exm_t;       // 1: and every packet's time (AggArgs::exm_t; Mode B predicted)
    MergeSrc ms;     // the owner segments of every batch (k_merge_spill)
    int phash;     // 1: the hot pass writes the per-packet filter words (AggArgs::phash)
    int pid;       // 1: the merge writes each packet's flow over them (AggArgs::pid; k_parse_spill runs)
    int clean;     // 1: the pass starts with k_cleanup (0: the last fluere_run already cleared its flows)
    int spec;      // 1: k_finalize publishes the counters to the host itself, a speculative k_cleanup follows
    CleanArgs spec_ca;
    unsigned spec_grid;
    int finalize;  // fluere_run: k_finalize + counters copy
    FinArgs fa;
    unsigned fin_grid;
    SoLaunch so;   // the Mode A ordering behind k_finalize (spec runs; order.hip)
    Ctl* h_ctl;
    Glob* d_glob;
};

// Bytes of the hot kernel's staging area for one batch (Stage layout).
// Capacity of an owner segment (records per set and owner): a window's
// packets spread over the owners by hash, with 25 % headroom; bounded so
// record indices of the segments fit u32 (k_merge_partials' set tables).
static uint32_t owner_cap(size_t sets, uint32_t O) {
    const char* force = getenv("FLUERE_OWNER_CAP");  // tests: a small capacity sends spills to the overflow list
    // (a multiple of 32 records: every owner segment starts on a whole 128-B
    // line for the 24-byte records, so k_parse_spill's bins land as whole lines)
    uint64_t cap = force ? (uint64_t)std::max(1, atoi(force)) : ((uint64_t)SPILL_WG / O * 5 / 4 + 32 + 31) & ~31ull;
    while (cap > 16 && (uint64_t)sets * O * cap >= (1ull << 32)) cap /= 2;
    return (uint32_t)cap;
}

// k_slow's sets (one per SLOW_SET slow-list entries of a batch of n packets)
// and their owner-segment capacity, after `sets` hot sets; 0 sets when the
// record indices would not fit u32 (the merge tail then takes the slow list).
static void slow_shape(uint64_t n, size_t sets, uint32_t O, uint32_t& n_slow_sets, uint32_t& cap_s) {
    n_slow_sets = (uint32_t)((n + SLOW_SET - 1) / SLOW_SET);
    const char* force = getenv("FLUERE_OWNER_CAP");  // tests: a small capacity sends records to the overflow list
    // (a multiple of 32 records, as owner_cap: line-aligned segments of 24-byte records)
    cap_s = force ? (uint32_t)std::max(1, atoi(force)) : ((uint32_t)SLOW_SET / O * 5 / 4 + 32 + 31) & ~31u;
    const uint64_t rec0 = (uint64_t)sets * O * owner_cap(sets, O);
    while (cap_s > 8 && rec0 + (uint64_t)n_slow_sets * O * cap_s >= (1ull << 32)) cap_s /= 2;
    if (rec0 + (uint64_t)n_slow_sets * O * cap_s >= (1ull << 32)) n_slow_sets = 0;
}

static size_t stage_bytes(size_t cells, size_t sets, uint32_t O, unsigned grid, uint64_t n, bool macs, bool slow) {
    uint32_t ns = 0, cap_s = 0;
    if (slow) slow_shape(n, sets, O, ns, cap_s);
    const size_t all = sets + ns;
    return cells * (sizeof(Part) + (macs ? sizeof(uint4) : 0)) +
           (sets * O * owner_cap(sets, O) + (size_t)ns * O * cap_s + (size_t)grid * SPILL_WG + n) * spill_units(macs) *
               sizeof(Spill) +
           all * sizeof(unsigned long long) + 2 * (size_t)(O + 1) * all * sizeof(uint32_t) +
           (size_t)grid * WGS_N * sizeof(unsigned long long) + 64 + (macs ? 16 : 0);
}

// Merge owners (workgroups of k_merge_partials).  FLUERE_MAC_OWNERS caps them
// for MAC runs (diagnostics): fewer owners mean fewer owner-grouped write
// streams at the flush (C5u k_parse_agg 0.65 / 0.58 / 0.52 ms at 256 / 128 / 64
// owners) but a slower merge (step 0.97 / 1.14 / 3.3 ms), so all are used.
#ifndef FLUERE_MAC_OWNERS
#define FLUERE_MAC_OWNERS 2048
#endif
static uint32_t merge_owners(const fluere_ctx* c) {
    // enough owners that each one's share of the flows (the last run's count
    // as the estimate) fits its merge workgroup's 1024-entry LDS table at
    // <= 85 % load; at least one per CU.  No more than that: k_parse_spill's
    // per-owner LDS bins shrink as owners grow (BIN = 5461 / O records), and
    // at 2048 owners the 2-record bins cost realistic TCP (847k flows) 85 us of
    // hot kernel over 1024 owners (827 flows each); 1M flows at 1024 owners
    // (977 each) overflow the merge tables and cost 0.5 ms (r03ah)
    static const uint32_t o_min = getenv("FLUERE_MIN_OWNERS") ? (uint32_t)atoi(getenv("FLUERE_MIN_OWNERS")) : 256u;
    uint32_t o = o_min;
    while (o < (uint32_t)MAX_OWNERS && c->last_nf > 870ull * o) o *= 2;
    // between two powers of two: the smallest multiple of 256 owners whose mean
    // share stays <= 800 flows (1M flows: 1280 owners, bins of 4 records, not
    // 2048 owners with bins of 2)
    const uint64_t alt = ((c->last_nf + 799) / 800 + 255) / 256 * 256;
    if (alt > o_min && alt < o) o = (uint32_t)alt;
    static const int o_max = getenv("FLUERE_MAX_OWNERS") ? atoi(getenv("FLUERE_MAX_OWNERS")) : MAX_OWNERS;  // diagnostics
    const int cap = std::min(o_max, c->use_mac ? std::min(FLUERE_MAC_OWNERS, MAX_OWNERS) : MAX_OWNERS);
    // even: the flush's per-owner counters are 16-bit pairs (a CU count such as 304 stays)
    // (at least one per CU, unless FLUERE_MIN_OWNERS sets the floor itself)
    const int floor_o = getenv("FLUERE_MIN_OWNERS") ? (int)o_min : c->n_cu;
    uint32_t r = (uint32_t)std::max(2, std::min(std::max((int)o, floor_o), cap));
    r = (r + 1) & ~1u;
    return std::min<uint32_t>(r, (uint32_t)MAX_OWNERS);
}

static int plan_batches(fluere_ctx* c, PassPlan& P, bool allow_pid = true) {
    AggArgs a;
    memset(&a, 0, sizeof a);
    a.T = tables_of(c);
    a.A = c->acc;
    a.g = c->d_glob;
    a.macs = c->use_mac;
    // slow list: one region per hot workgroup (its steps x BLOCK packets),
    // then the per-workgroup counts
    auto hot_shape = [&](uint64_t n, unsigned& grid, uint64_t& steps) {
        const uint64_t want = (n + BLOCK * 8 - 1) / (BLOCK * 8);
        grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)c->n_cu));
        const uint64_t per = (n + grid - 1) / grid;
        steps = (per + BLOCK - 1) / BLOCK;
    };
    uint64_t maxn = 1;
    for (auto& hb : c->batches) {
        if (!hb.b.n) continue;
        unsigned grid;
        uint64_t steps;
        hot_shape(hb.b.n, grid, steps);
        maxn = std::max<uint64_t>(maxn, (uint64_t)grid * steps * BLOCK);
    }
    const uint64_t slow_words = 2 * maxn + MB;
    if (slow_words > c->d_slow_cap) {
        hipFree(c->d_slow);
        c->d_slow = nullptr;
        if (hipMalloc(&c->d_slow, slow_words * 4) != hipSuccess) return FLUERE_E_NOMEM;
        c->d_slow_cap = slow_words;
    }
    a.slow = c->d_slow;
    a.slow_cnt = c->d_slow + maxn;
    a.gen = c->d_slow + maxn + MB;
    a.slow_abl = diag_knob("FLUERE_SLOW_ABL");
    // k_slow when the last run had slow packets (a wrong guess costs only the
    // merge tail's slower path, or an empty launch)
    const int slow_env = getenv("FLUERE_SLOW_KERNEL") ? atoi(getenv("FLUERE_SLOW_KERNEL")) : -1;  // tests: force it
    a.slow_kernel = slow_env >= 0 ? slow_env : (c->last_n_slow > 0 ? 1 : 0);
    // k_slow over every packet, no hot kernel, when (nearly) every packet is of
    // the general parser's classes: the hot pass would only read each window
    // to list it for k_slow's second read (the slow config: 0.35 of 1.47 ms)
    // (tests set these between runs: read per plan, not cached)
    const int sa_env = getenv("FLUERE_SLOW_ALL") ? atoi(getenv("FLUERE_SLOW_ALL")) : -1;  // tests / A/B
    const bool slow_all =
        sa_env >= 0 ? sa_env != 0 : (c->n_total > 0 && (uint64_t)c->last_n_slow * 4 >= (uint64_t)c->n_total * 3);
    if (slow_all) a.slow_kernel = 1;
    a.slow_all = slow_all ? 1 : 0;
    // k_slow's IPv6 address ids (non-MAC runs): 4 slots per flow of capacity, at most 2^20
    if (a.slow_kernel && !c->use_mac) {
        uint32_t C = 1u << 12;
        while (C < (1u << 20) && C < 4ull * c->fmax) C <<= 1;
        if (C != c->v6C) {
            hipFree(c->d_v6map);
            c->d_v6map = nullptr;
            c->v6C = 0;
            if (hipMalloc(&c->d_v6map, (size_t)(C + 1) * (3 * 8 + 16) + 16) != hipSuccess) return FLUERE_E_NOMEM;
            c->v6C = C;
        }
        unsigned long long* k = (unsigned long long*)c->d_v6map;
        a.v6.tab[0] = k;
        a.v6.tab[1] = k + (C + 1);
        a.v6.tab[2] = k + 2 * (size_t)(C + 1);
        a.v6.addr_of = (uint4*)(k + ((3 * (size_t)(C + 1) + 1) & ~(size_t)1));  // (16-byte aligned)
        a.v6.C = C;
    }
    // per-packet filter words for the exact engine when the last run replayed
    // complex flows in Mode A (a prediction: without them k_ex_meta parses
    // every packet; 4 bytes per packet written by the hot pass)
    const int phash_env = getenv("FLUERE_PHASH") ? atoi(getenv("FLUERE_PHASH")) : -1;  // tests / A/B
    P.phash = !c->use_mac && (phash_env >= 0 ? phash_env : (c->last_n_complex > 0 && !c->last_mode_b)) ? 1 : 0;
    // k_parse_spill runs (every valid packet a record the merge resolves) that
    // will replay packets (complex flows in Mode A, or Mode B): the merge
    // writes each packet's flow over its filter word, so k_ex_meta walks no
    // dictionary (a prediction, like the filter words)
    {
        int nbat = 0;
        for (auto& hb : c->batches) nbat += hb.b.n ? 1 : 0;
        const int pid_env = getenv("FLUERE_PID") ? atoi(getenv("FLUERE_PID")) : -1;  // tests / A/B
        const bool want = pid_env >= 0 ? pid_env != 0 : (c->last_n_complex > 0 || c->last_mode_b);
        P.pid = (allow_pid && P.spill && !c->use_mac && nbat <= PLAN_BATCHES && want) ? 1 : 0;
        if (P.pid) P.phash = 1;
        if (slow_all) P.pid = P.phash = 0;  // (no hot pass writes the words)
        if (P.pid && !c->d_emap &&
            hipMalloc(&c->d_emap, ((size_t)PLAN_BATCHES << 21) * sizeof(uint32_t)) != hipSuccess)
            return FLUERE_E_NOMEM;
    }
    // Mode B predicted (the last run's): the hot pass also writes every
    // packet's replay metadata in capture order, so the exact engine skips its
    // k_ex_meta pass over the packets (used when every packet was valid and
    // none needed the general parser; FLUERE_EXM=0: A/B).  Complex flows
    // predicted in Mode A: the same metadata, which k_ex_meta copies for the
    // replayed packets the hot parser took instead of parsing them again
    // (FLUERE_EXMA=1, forced on; off by default: on the realistic TCP mix
    // k_ex_meta went from 249 to 194 us but the hot pass's 320 MB of extra
    // writes cost 68 us)
    {
        static const int exm_env = getenv("FLUERE_EXM") ? atoi(getenv("FLUERE_EXM")) : -1;
        const char* exma = getenv("FLUERE_EXMA");
        const bool want = c->last_mode_b ? exm_env != 0 : (exma && atoi(exma) > 0);
        P.exm = (P.pid && P.spill && !c->use_mac && want) ? 1 : 0;
        P.exm_t = P.exm && c->last_mode_b ? 1 : 0;
        // (an optional speed-up: without the memory the run goes on without it;
        // the times array only where Mode B reads it)
        if (P.exm && c->n_total > c->exm_cap) {
            hipFree(c->d_exm);
            c->d_exm = nullptr;
            c->exm_cap = 0;
            if (hipMalloc(&c->d_exm, c->n_total * sizeof(ExMeta)) == hipSuccess) c->exm_cap = c->n_total;
            else (void)hipGetLastError();
        }
        if (P.exm_t && c->n_total > c->exm_t_cap) {
            hipFree(c->d_exm_t);
            c->d_exm_t = nullptr;
            c->exm_t_cap = 0;
            if (hipMalloc(&c->d_exm_t, c->n_total * 8) == hipSuccess) c->exm_t_cap = c->n_total;
            else (void)hipGetLastError();
        }
        if (c->n_total > c->exm_cap) P.exm = 0;
        if (!P.exm || c->n_total > c->exm_t_cap) P.exm_t = 0;
    }
    if (P.phash && c->n_total > c->phash_cap) {
        hipFree(c->d_phash);
        c->d_phash = nullptr;
        c->phash_cap = 0;
        if (hipMalloc(&c->d_phash, c->n_total * 4) != hipSuccess) return FLUERE_E_NOMEM;
        c->phash_cap = c->n_total;
    }
    if (getenv("FLUERE_DEBUG")) {
        if (!g_hot_dbg && hipMalloc(&g_hot_dbg, 4096 * 8 * 8) != hipSuccess) g_hot_dbg = nullptr;
        a.dbg = g_hot_dbg;
    }
    // staging for the largest batch (every batch reuses it, in stream order)
    // One owner merge per pass (k_merge_spill over every batch's segments) when
    // no batch stages partials: each batch keeps a staging area of its own.
    // Otherwise every batch is merged right after its hot pass and reuses one.
    int nbat = 0;
    for (auto& hb : c->batches) nbat += hb.b.n ? 1 : 0;
    P.one_merge = P.lean_merge && (P.spill || slow_all) && nbat > 1 && nbat <= MS_BATCHES ? 1 : 0;
    size_t need_max = 0, need_sum = 0;
    std::vector<size_t> stage_off;
    for (auto& hb : c->batches) {
        if (!hb.b.n) continue;
        uint64_t want = (hb.b.n + BLOCK * 8 - 1) / (BLOCK * 8);
        unsigned grid = slow_all ? 0u : (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)c->n_cu));
        const uint64_t per = (hb.b.n + std::max(grid, 1u) - 1) / std::max(grid, 1u);
        const uint64_t steps = (per + BLOCK - 1) / BLOCK;
        const uint32_t W = (uint32_t)std::max<uint64_t>(1, (steps + WIN_ITERS - 1) / WIN_ITERS);
        const size_t sets = (size_t)grid * W, cells = sets * NS;
        const uint32_t O = merge_owners(c);
        const size_t sb = (stage_bytes(cells, sets, O, grid, hb.b.n, c->use_mac, a.slow_kernel != 0) + 255) & ~(size_t)255;
        stage_off.push_back(P.one_merge ? need_sum : 0);
        need_sum += sb;
        need_max = std::max(need_max, sb);
    }
    if (P.one_merge) need_max = need_sum;
    if (need_max > c->d_stage_bytes) {
        hipFree(c->d_stage);
        c->d_stage = nullptr;
        c->d_stage_bytes = 0;
        if (hipMalloc(&c->d_stage, need_max) != hipSuccess) return FLUERE_E_NOMEM;
        c->d_stage_bytes = need_max;
    }
    P.nb = 0;
    for (auto& hb : c->batches) {
        if (!hb.b.n) continue;
        a.B = hb.b;
        char* stage = (char*)c->d_stage + stage_off[P.nb];
        // the batch's counters: Glob's for a pass of one batch, else its own (zeroed per pass)
        a.bc = nbat > 1 ? c->d_bctr + 8 * (size_t)P.nb : &c->d_glob->n_slow;
        a.slow_n = a.bc;
        uint64_t want = (hb.b.n + BLOCK * 8 - 1) / (BLOCK * 8);
        unsigned grid = slow_all ? 0u : (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)c->n_cu));
        // staging: one set per (workgroup, window) -- k_parse_agg's loop bounds
        const uint64_t per = (hb.b.n + std::max(grid, 1u) - 1) / std::max(grid, 1u);
        const uint64_t steps = (per + BLOCK - 1) / BLOCK;
        const uint32_t W = (uint32_t)std::max<uint64_t>(1, (steps + WIN_ITERS - 1) / WIN_ITERS);
        const size_t sets = (size_t)grid * W, cells = sets * NS;
        const uint32_t O = merge_owners(c);
        a.slow_region = (uint32_t)(steps * BLOCK);
        // k_slow's sets after the hot kernel's (only when it runs)
        uint32_t n_slow_sets = 0, cap_s = 0;
        if (a.slow_kernel) slow_shape(hb.b.n, sets, O, n_slow_sets, cap_s);
        AggArgs ab = a;
        ab.slow_kernel = n_slow_sets ? a.slow_kernel : 0;
        ab.phash = P.phash ? c->d_phash + (hb.b.first - c->index_base) : nullptr;
        ab.pid = P.pid ? c->d_phash : nullptr;
        ab.emap = P.pid ? c->d_emap : nullptr;
        ab.pid_base = c->index_base;
        ab.pid_batch = (uint32_t)P.nb;
        ab.exm = P.exm ? c->d_exm + (hb.b.first - c->index_base) : nullptr;
        ab.exm_t = P.exm_t ? c->d_exm_t + (hb.b.first - c->index_base) : nullptr;
        const size_t all = sets + n_slow_sets;
        Stage& S = ab.S;
        // layout (16-byte aligned pieces): parts | owner segments (hot, k_slow) | spill_raw | spill | base | off | soff
        S.part = (Part*)stage;
        S.cap_o = owner_cap(sets, O);
        S.cap_s = cap_s;
        S.slow_rec0 = (unsigned long long)sets * O * S.cap_o;
        S.dspill = (Spill*)(S.part + cells);
        S.spill_raw = S.dspill + (sets * O * S.cap_o + (size_t)n_slow_sets * O * cap_s) * spill_units(c->use_mac);
        S.spill = S.spill_raw + (size_t)grid * SPILL_WG * spill_units(c->use_mac);
        S.spill_cap = hb.b.n;  // overflow-list records (32 B, or 64 B with MACs; the segments' are packed, seg.h)
        S.base = (unsigned long long*)(S.spill + hb.b.n * spill_units(c->use_mac));
        S.off = (uint32_t*)(S.base + all);
        S.soff = S.off + (size_t)(O + 1) * all;
        S.wgs = (unsigned long long*)(((uintptr_t)(S.soff + (size_t)(O + 1) * all) + 7) & ~(uintptr_t)7);
        S.partx = c->use_mac ? (uint4*)(((uintptr_t)(S.wgs + (size_t)grid * WGS_N) + 15) & ~(uintptr_t)15) : nullptr;
        S.n_wg = grid;
        S.W = W;
        S.O = O;
        S.n_hot = (uint32_t)sets;
        S.n_sets = (uint32_t)all;
        S.no_parts = (P.spill || slow_all) ? 1u : 0u;
        if (P.nb < MS_BATCHES) {
            SegSrc& sg = P.ms.b[P.nb];
            sg.dspill = S.dspill;
            sg.soff = S.soff;
            sg.base = S.base;
            sg.spill = S.spill;
            sg.bc = ab.bc;
            sg.slow_rec0 = S.slow_rec0;
            sg.first = hb.b.first;
            sg.cap_o = S.cap_o;
            sg.cap_s = S.cap_s;
            sg.n_sets = S.n_sets;
            sg.n_hot = S.n_hot;
            sg.slow_kernel = (uint32_t)ab.slow_kernel;
            P.ms.nb = P.nb + 1;
        }
        if (P.nb < PLAN_BATCHES) {
            P.agg[P.nb] = ab;
            P.agg_grid[P.nb] = grid;
            P.slow_grid[P.nb] = n_slow_sets;
            P.owners[P.nb] = O;
        }
        P.nb++;
    }
    return FLUERE_OK;
}

// k_parse_spill when the last run's flows would overflow k_parse_agg's LDS
// table in most windows: the distinct keys a workgroup window of w packets
// sees out of F flows, F (1 - e^(-w/F)), above twice the table's slots
// (C3/C4-like captures: ~45k-60k keys per window, 92-95 % of the packets
// past the table).  A prediction from the last run: either kernel is exact.
static int spill_mode(const fluere_ctx* c) {
    const int env = getenv("FLUERE_SPILL_MODE") ? atoi(getenv("FLUERE_SPILL_MODE")) : -1;  // tests: force either kernel
    if (merge_owners(c) < 128) return 0;  // bins of more than 32 (MACS: 16) records: more than a wave per bin
    if (env >= 0) return env;
    const double F = (double)c->last_nf;
    if (F <= 0) return 0;
    uint64_t nmax = 0;
    for (auto& hb : c->batches) nmax = std::max<uint64_t>(nmax, hb.b.n);
    const double w = std::min<double>((double)WIN_ITERS * BLOCK, (double)nmax / std::max(1, c->n_cu));
    return F * (1.0 - std::exp(-w / F)) > 2.0 * (c->use_mac ? NS_MAC : NS) ? 1 : 0;
}

// k_merge_spill for the runs without partials (not MAC runs: their 48-byte
// records stay with k_merge_partials); FLUERE_LEAN_MERGE=0: k_merge_partials
// for every run (A/B)
static int lean_merge(const fluere_ctx* c) {
    const int env = getenv("FLUERE_LEAN_MERGE") ? atoi(getenv("FLUERE_LEAN_MERGE")) : -1;
    return !c->use_mac && env != 0 ? 1 : 0;
}

static int plan_pass(fluere_ctx* c, PassPlan& P, bool finalize) {
    memset(&P, 0, sizeof P);  // byte-comparable (padding included)
    int rc;
    if ((rc = upload_batches(c))) return rc;  // host -> device, only when the batches changed
    if ((rc = census(c))) return rc;          // a new capture: its shape from a sample
    P.ca = CleanArgs{tables_of(c), c->acc, c->d_complex, c->d_active, c->d_glob};
    static const int clean_abl = diag_knob("FLUERE_CLEAN_ABL");
    P.ca.abl = clean_abl;
    P.ca.bulk = bulk_clean(c, c->prev_nf == ~0ull ? c->last_nf : c->prev_nf);
    // cleanup grid: the last fetched run's flow count when known (k_cleanup is
    // grid-stride over the device count, so any grid is correct)
    P.clean_grid = done_grid(c, c->prev_nf == ~0ull ? c->fmax : c->prev_nf);
    P.tab_words = (size_t)N_TABLES * 2 * (c->C + 1);
    P.clean = c->precleaned ? 0 : 1;
    P.spill = spill_mode(c);
    P.lean_merge = lean_merge(c);
    if ((rc = plan_batches(c, P))) return rc;
    static const int abl = diag_knob("FLUERE_ABLATE");
    P.macs = c->use_mac;
    P.abl = abl;
    P.finalize = finalize ? 1 : 0;
    P.h_ctl = c->h_ctl;
    P.d_glob = c->d_glob;
    if (finalize) {
        // speculative Mode A finalize over the device-side flow count
        // (sized for the expected flows: a speculative finalize past the
        // buffer runs again after growing it)
        const uint64_t want = std::max<uint64_t>(1u << 16, c->last_nf + c->last_nf / 4);
        if ((rc = ensure_recs(c, std::max<uint64_t>(c->d_recs_cap, std::min<uint64_t>(c->fmax, want))))) return rc;
        P.fa = FinArgs{c->d_batches, (int)c->batches.size(), tables_of(c), c->acc, c->d_glob,
                       c->d_recs,    c->d_complex,           c->use_mac,   c->d_recs_cap};
        P.fa.timeout_us = c->timeout_ms * 1000ull;
        P.fa.cbits = c->d_cbits;
        P.fa.defer = c->d_fdefer;
        P.spec_ca = P.ca;
        P.spec_ca.spec = 1;
        P.spec_ca.bulk = bulk_clean(c, c->last_nf);  // (this run's flows: the last run's count as the guess)
        P.spec_ca.timeout_us = c->timeout_ms * 1000ull;
        P.spec_ca.recs_cap = c->d_recs_cap;
        // grid-stride over the device flow count: any grid is correct; size
        // them for the last known flow count (k_finalize's workgroups also
        // count themselves done on one counter before the last one publishes)
        const uint64_t guess = c->last_nf ? c->last_nf : c->fmax;
        P.fin_grid = std::max(8u, done_grid(c, guess));
        P.spec_grid = P.fin_grid;
    }
    return FLUERE_OK;
}

static int enqueue_batches(fluere_ctx* c, const PassPlan& P) {
    hipStream_t s = c->stream;
    // the batches' own counters (AggArgs::bc; a pass of one batch uses Glob's, which k_cleanup zeroed)
    if (P.nb > 1) HIPCHECK(hipMemsetAsync(c->d_bctr, 0, 8 * 8 * (size_t)P.nb, s));
    for (int i = 0; i < P.nb; i++) {
        const AggArgs& a = P.agg[i];
        const unsigned grid = P.agg_grid[i];
        const void* fn = hot_kernel(P.spill, P.macs, P.abl);
        // HIP events carried by the dispatch itself (start / stop timestamps of
        // the hot kernel): separate event markers would each add a gap to the
        // stream; one pair per batch (summed: the pass's hot-kernel time).
        void* args[] = {const_cast<AggArgs*>(&a)};
        static const bool hostprof = getenv("FLUERE_HOSTPROF") != nullptr;
        const auto t0 = std::chrono::steady_clock::now();
        hipEvent_t e0 = c->evh[2 * i], e1 = c->evh[2 * i + 1];
        static const int ev_abl = diag_knob("FLUERE_EV_ABL");  // diagnostics: 1 no timing events (kernel_ms invalid)
        // FLUERE_EV_REC=1 (A/B): the events recorded on the stream around a plain launch
        static const bool ev_rec = getenv("FLUERE_EV_REC") && atoi(getenv("FLUERE_EV_REC")) != 0;
        if (grid && ev_abl == 1) {
            HIPCHECK(hipLaunchKernel(fn, dim3(grid), dim3(BLOCK), args, 0, s));
        } else if (grid && ev_rec) {
            HIPCHECK(hipEventRecord(e0, s));
            HIPCHECK(hipLaunchKernel(fn, dim3(grid), dim3(BLOCK), args, 0, s));
            HIPCHECK(hipEventRecord(e1, s));
        } else if (grid) {
            HIPCHECK(hipExtLaunchKernel(fn, dim3(grid), dim3(BLOCK), args, 0, s, e0, e1, 0));
        }
        const auto t1 = std::chrono::steady_clock::now();
        // the slow list into k_slow's owner segments, before the merge reads them
        // (every packet without a hot kernel: k_slow carries the timing events)
        if (a.slow_kernel) {
            if (a.v6.C) HIPCHECK(hipMemsetAsync(a.v6.tab[0], 0xFF, (size_t)(a.v6.C + 1) * 3 * 8, s));  // every key EMPTY
            if (grid) {
                k_slow<<<P.slow_grid[i], SB, 0, s>>>(a);
            } else {
                HIPCHECK(hipExtLaunchKernel((const void*)k_slow, dim3(P.slow_grid[i]), dim3(SB), args, 0, s, e0, e1,
                                            0));
            }
        }
        // at most one merge workgroup per CU, each taking owners in turn
        // + the slow list (unless k_slow took it).  Runs without partials
        // (k_parse_spill, k_slow): the lean owner merge, then the tail alone
        // (overflow list, general-parser packets, run statistics)
        const dim3 mgrid(std::min<uint32_t>(P.owners[i], (uint32_t)c->n_cu));
        if (P.one_merge) {
            // (after the last batch's hot pass: below)
        } else if (P.lean_merge && a.S.no_parts) {
            MergeSrc one = P.ms;
            one.b[0] = P.ms.b[i];
            one.nb = 1;
            void* margs[] = {const_cast<AggArgs*>(&a), &one};
            HIPCHECK(hipLaunchKernel((const void*)k_merge_spill, mgrid, dim3(MB), margs, 0, s));
            AggArgs at = a;
            at.tail_only = 1;
            at.dbg = nullptr;  // (FLUERE_DEBUG: the phase clocks are k_merge_spill's)
            void* targs[] = {&at};
            HIPCHECK(hipLaunchKernel(merge_kernel(P.macs), dim3((uint32_t)c->n_cu), dim3(MB), targs, 0, s));
        } else {
            HIPCHECK(hipLaunchKernel(merge_kernel(P.macs), mgrid, dim3(MB), args, 0, s));
        }
        if (hostprof) {
            const auto t2 = std::chrono::steady_clock::now();
            auto us = [](auto x, auto y) { return std::chrono::duration<double, std::micro>(y - x).count(); };
            fprintf(stderr, "[fluere] launch: hot %.1f merge %.1f us\n", us(t0, t1), us(t1, t2));
        }
    }
    if (P.one_merge) {
        // one owner merge over every batch's segments (each flow resolved and
        // accumulated once per pass), then each batch's tail: its overflow list,
        // general-parser packets and run statistics
        void* margs[] = {const_cast<AggArgs*>(&P.agg[0]), const_cast<MergeSrc*>(&P.ms)};
        HIPCHECK(hipLaunchKernel((const void*)k_merge_spill, dim3(std::min<uint32_t>(P.owners[0], (uint32_t)c->n_cu)),
                                 dim3(MB), margs, 0, s));
        for (int i = 0; i < P.nb; i++) {
            AggArgs at = P.agg[i];
            at.tail_only = 1;
            at.dbg = nullptr;
            void* targs[] = {&at};
            HIPCHECK(hipLaunchKernel(merge_kernel(P.macs), dim3((uint32_t)c->n_cu), dim3(MB), targs, 0, s));
        }
    }
    HIPCHECK(hipGetLastError());
    return FLUERE_OK;
}

static int enqueue_pass(fluere_ctx* c, const PassPlan& P) {
    hipStream_t s = c->stream;
    if (P.clean) k_cleanup<<<P.clean_grid, 256, 0, s>>>(P.ca, P.tab_words);
    c->precleaned = false;
    int rc;
    if ((rc = enqueue_batches(c, P))) return rc;
    if (P.finalize) {
        k_finalize<<<P.fin_grid, 256, 0, s>>>(P.fa);
        if (P.spec) {
            // k_finalize's last workgroup writes the counters to the pinned
            // host copy and publishes P.fa.seq; the speculative cleanup follows
            if (P.so.on && (rc = so_enqueue(c, P.so))) return rc;
            k_cleanup<<<P.spec_grid, 256, 0, s>>>(P.spec_ca, P.tab_words);
        } else {
            HIPCHECK(hipMemcpyAsync(P.h_ctl, P.d_glob, sizeof(Ctl), hipMemcpyDeviceToHost, s));
        }
    }
    HIPCHECK(hipGetLastError());
    return FLUERE_OK;
}

// The same pass as an explicit hipGraph (linear chain of nodes).  Built node by
// node rather than by stream capture: a captured hipEventRecord yields no
// timestamps on this runtime, explicit event-record nodes do.  `P` must stay
// alive and unchanged while the graph exists (kernel nodes point at its args).
static int build_pass_graph(fluere_ctx* c, PassPlan& P, hipGraphExec_t* out) {
    if (P.one_merge) return FLUERE_E_ARG;  // (a pass merged once runs direct launches)
    hipGraph_t g = nullptr;
    HIPCHECK(hipGraphCreate(&g, 0));
    hipGraphNode_t prev = nullptr, n = nullptr;
    bool ok = true;
    auto dep = [&]() { return prev ? 1 : 0; };
    auto kernel = [&](const void* fn, unsigned grid, unsigned block, void** args) {
        if (!ok) return;
        hipKernelNodeParams kp{};
        kp.func = const_cast<void*>(fn);
        kp.gridDim = dim3(grid);
        kp.blockDim = dim3(block);
        kp.sharedMemBytes = 0;
        kp.kernelParams = args;
        kp.extra = nullptr;
        ok = hipGraphAddKernelNode(&n, g, prev ? &prev : nullptr, dep(), &kp) == hipSuccess;
        prev = n;
    };
    auto event = [&](hipEvent_t e) {
        if (!ok) return;
        ok = hipGraphAddEventRecordNode(&n, g, prev ? &prev : nullptr, dep(), e) == hipSuccess;
        prev = n;
    };
    void* a_clean[] = {&P.ca, &P.tab_words};
    if (P.clean) kernel((const void*)k_cleanup, P.clean_grid, 256, a_clean);
    void* a_agg[PLAN_BATCHES][1];
    for (int i = 0; i < P.nb && ok; i++) {
        if (i == 0 && P.nb > 1) {  // the batches' own counters (AggArgs::bc)
            hipMemsetParams mp{};
            mp.dst = c->d_bctr;
            mp.elementSize = 4;
            mp.width = 16 * (size_t)P.nb;
            mp.height = 1;
            mp.pitch = 0;
            mp.value = 0;
            ok = hipGraphAddMemsetNode(&n, g, &prev, 1, &mp) == hipSuccess;
            prev = n;
        }
        event(c->evh[2 * i]);
        a_agg[i][0] = &P.agg[i];
        const void* fn = hot_kernel(P.spill, P.macs, P.abl);
        if (P.agg_grid[i]) kernel(fn, P.agg_grid[i], BLOCK, a_agg[i]);
        if (P.agg_grid[i]) event(c->evh[2 * i + 1]);
        if (P.agg[i].slow_kernel && P.agg[i].v6.C && ok) {
            hipMemsetParams mp{};
            mp.dst = P.agg[i].v6.tab[0];
            mp.elementSize = 4;
            mp.width = (size_t)(P.agg[i].v6.C + 1) * 3 * 2;
            mp.height = 1;
            mp.pitch = 0;
            mp.value = 0xFFFFFFFFu;
            ok = hipGraphAddMemsetNode(&n, g, &prev, 1, &mp) == hipSuccess;
            prev = n;
        }
        if (P.agg[i].slow_kernel) kernel((const void*)k_slow, P.slow_grid[i], SB, a_agg[i]);
        if (!P.agg_grid[i]) event(c->evh[2 * i + 1]);
        kernel(merge_kernel(P.macs),
               std::min<uint32_t>(P.owners[i], (uint32_t)c->n_cu), MB, a_agg[i]);
    }
    void* a_fin[] = {&P.fa};
    if (P.finalize) {
        kernel((const void*)k_finalize, P.fin_grid, 256, a_fin);
        if (ok) {
            ok = hipGraphAddMemcpyNode1D(&n, g, &prev, 1, P.h_ctl, P.d_glob, sizeof(Ctl), hipMemcpyDeviceToHost) ==
                 hipSuccess;
            prev = n;
        }
    }
    if (ok) ok = hipGraphInstantiate(out, g, nullptr, nullptr, 0) == hipSuccess;
    hipGraphDestroy(g);
    (void)hipGetLastError();
    return ok ? FLUERE_OK : FLUERE_E_HIP;
}

// The last pass's hot-kernel launches: their summed device time (HIP events
// carried by each dispatch), or the span from the first one's start to the
// last one's end.
static int hot_times(fluere_ctx* c, float* sum, float* span) {
    const int nb = std::max(1, std::min(c->plan_nb, PLAN_BATCHES));
    *sum = 0;
    for (int i = 0; i < nb; i++) {
        float ms = 0;
        if (hipEventElapsedTime(&ms, c->evh[2 * i], c->evh[2 * i + 1]) != hipSuccess) return FLUERE_E_HIP;
        *sum += ms;
    }
    if (span && hipEventElapsedTime(span, c->evh[0], c->evh[2 * nb - 1]) != hipSuccess) return FLUERE_E_HIP;
    return FLUERE_OK;
}

void debug_counters(fluere_ctx* c, const Glob* have) {
    if (!getenv("FLUERE_DEBUG")) return;  // diagnostics only: synchronises the stream
    Glob g;
    if (have) g = *have;
    else if (hipMemcpyAsync(&g, c->d_glob, sizeof g, hipMemcpyDeviceToHost, c->stream) != hipSuccess) return;
    if (hipStreamSynchronize(c->stream) != hipSuccess) return;
    fprintf(stderr, "[fluere] valid %llu dropped %llu slow %llu LDS-table overflow packets %llu\n", g.valid, g.dropped,
            g.n_slow, g.n_kc_miss);
    fprintf(stderr, "[fluere] per-WG clock: total %.0f flush %.0f wait-for-waves %.0f | merge scan %.0f ids %.0f\n",
            g.cyc_total / 256.0, g.cyc_flush / 256.0, g.cyc_flush0 / 256.0, g.cyc_m_scan / 256.0, g.cyc_m_ids / 256.0);
    if (g_hot_dbg) {
        // per XCD (workgroup b runs on XCD b % 8): mean / max workgroup time, mean flush, mean end
        std::vector<unsigned long long> w(256 * 8);
        if (hipMemcpy(w.data(), g_hot_dbg, w.size() * 8, hipMemcpyDeviceToHost) == hipSuccess) {
            unsigned long long t0 = ~0ull;
            for (int b = 0; b < 256; b++) t0 = std::min(t0, w[b * 8]);
            unsigned long long t1 = 0, smax = 0, loops = 0, iters = 0;
            for (int b = 0; b < 256; b++) {
                t1 = std::max(t1, w[b * 8 + 3]);
                smax = std::max(smax, w[b * 8]);
                loops += w[b * 8 + 7] & 0xFFFFFFFFull;
                iters += w[b * 8 + 7] >> 32;
            }
            fprintf(stderr, "[fluere] WG starts spread %.1f us, first start -> last end %.1f us; probe loop %llu wave-chunks, %llu iterations\n",
                    (smax - t0) / 100.0, (t1 - t0) / 100.0, loops, iters);
            {
                // merge kernel phases (owner workgroups 0..255), mean us from its first start
                std::vector<unsigned long long> m(256 * 8);
                if (hipMemcpy(m.data(), g_hot_dbg + 4096 * 8 - 2048, m.size() * 8, hipMemcpyDeviceToHost) == hipSuccess) {
                    unsigned long long m0 = ~0ull;
                    for (int b = 0; b < 256; b++) m0 = std::min(m0, m[b * 8]);
                    double ph[8] = {0}, mx[8] = {0};
                    for (int b = 0; b < 256; b++)
                        for (int k = 0; k < 8; k++) {
                            ph[k] += (m[b * 8 + k] - m0) / 100.0 / 256;
                            mx[k] = std::max(mx[k], (m[b * 8 + k] - m0) / 100.0);
                        }
                    {  // the spread of the owners' record phase over the workgroups (the kernel waits for the slowest)
                        std::vector<double> pr;
                        for (int b = 0; b < 256; b++) pr.push_back((m[b * 8 + 3] - m[b * 8 + 2]) / 100.0);
                        std::sort(pr.begin(), pr.end());
                        fprintf(stderr, "[fluere] merge record phase per workgroup (us): min %.1f p10 %.1f p50 %.1f p90 %.1f p99 %.1f max %.1f\n",
                                pr[0], pr[25], pr[128], pr[230], pr[253], pr[255]);
                    }
                    fprintf(stderr, "[fluere] merge phases (mean/max us): init %.1f/%.1f offs+scan %.1f/%.1f parts %.1f/%.1f "
                            "claims %.1f/%.1f n_flows %.1f/%.1f ids %.1f/%.1f global %.1f/%.1f\n",
                            ph[1], mx[1], ph[2], mx[2], ph[3], mx[3], ph[7], mx[7], ph[6], mx[6], ph[4], mx[4], ph[5], mx[5]);
                }
            }
            for (int x = 0; x < 8; x++) {
                double sd = 0, md = 0, sf = 0, se = 0, p1 = 0, p2 = 0, p3 = 0;
                for (int b = x; b < 256; b += 8) {
                    const unsigned long long* q = &w[b * 8];
                    const double d = (q[3] - q[0]) / 100.0;
                    sd += d; md = std::max(md, d);
                    sf += (q[2] - q[1]) / 100.0;
                    se += (q[1] - t0) / 100.0;
                    p1 += (q[4] - q[1]) / 100.0;
                    p2 += (q[5] - q[4]) / 100.0;
                    p3 += (q[6] - q[5]) / 100.0;
                }
                fprintf(stderr, "[fluere]   XCD %d: sort %.1f offs %.1f parts %.1f | ", x, p1 / 32, p2 / 32, p3 / 32);
                fprintf(stderr, "[fluere]   XCD %d: WG mean %.1f max %.1f us, loop end mean %.1f us, flush mean %.1f us\n", x,
                        sd / 32, md, se / 32, sf / 32);
            }
        }
    }
}

int init_glob(fluere_ctx* c) {
    Glob g{};
    g.tmin = NONE64;
    HIPCHECK(hipMemcpyAsync(c->d_glob, &g, sizeof g, hipMemcpyHostToDevice, c->stream));
    return FLUERE_OK;
}

extern "C" int fluere_parse_aggregate(fluere_ctx* c) {
    if (!c) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    // diagnostics only (FLUERE_KEEP_DICT): keep the flow dictionary across runs so
    // key-cache misses become read-only dictionary hits (results accumulate)
    static const bool keep = diag_knob("FLUERE_KEEP_DICT") != 0;
    static int runs = 0;
    const bool kept = keep && runs++ > 0;
    int rc = kept ? init_glob(c) : clear_flows(c);  // clear_flows re-initialises the counters too
    if (rc) return rc;
    c->pass_in_run = false;
    PassPlan P;
    memset(&P, 0, sizeof P);
    if ((rc = upload_batches(c))) return rc;
    if ((rc = census(c))) return rc;
    P.spill = spill_mode(c);
    P.lean_merge = lean_merge(c);
    if ((rc = plan_batches(c, P, false))) return rc;
    if (P.nb > PLAN_BATCHES) return FLUERE_E_ARG;
    static const int abl = diag_knob("FLUERE_ABLATE");
    P.macs = c->use_mac;
    P.abl = abl;
    c->plan_nb = P.nb;
    c->plan_spill = P.spill;
    c->plan_slow_all = P.nb > 0 && P.agg[0].slow_all;
    c->precleaned = false;
    c->runs++;
    rc = enqueue_batches(c, P);
    debug_counters(c);
    return rc;
}

extern "C" const char* fluere_last_hot_kernel(fluere_ctx* c) {
    if (c && c->plan_slow_all) return "k_slow";
    return c && c->plan_spill ? "k_parse_spill" : "k_parse_agg";
}

// Device time of the last pass's hot-kernel launches, summed (HIP events on
// the context stream, carried by each dispatch).
extern "C" double fluere_last_kernel_ms(fluere_ctx* c) {
    if (!c) return -1.0;
    float ms = -1.0f;
    const int nb = std::max(1, std::min(c->plan_nb, PLAN_BATCHES));
    if (hipEventSynchronize(c->evh[2 * nb - 1]) != hipSuccess) return -1.0;
    if (hot_times(c, &ms, nullptr) != FLUERE_OK) return -1.0;
    return ms;
}

// Duration of the last pass: after fluere_run, its host wall time (submission
// to results); after fluere_parse_aggregate, the device time of its hot
// kernel launches (HIP events on the context stream; no other markers).
extern "C" double fluere_last_pass_ms(fluere_ctx* c) {
    if (!c) return -1.0;
    float ms = -1.0f;
    if (c->pass_in_run) return c->last_run_ms;
    const int nb = std::max(1, std::min(c->plan_nb, PLAN_BATCHES));
    float sum = 0;
    if (hipEventSynchronize(c->evh[2 * nb - 1]) != hipSuccess) return -1.0;
    if (hot_times(c, &sum, &ms) != FLUERE_OK) return -1.0;
    return ms;
}

// The attached capture made ready for its first pass, at attach time (not in
// live sessions, whose batches are their runs): the chunk descriptors, the
// census (k_census), and every buffer the first pass would otherwise allocate
// while the GPU waits, sized from the census -- the staging of the owner count
// and hot kernel it implies, the slow list, the filter words, the record
// buffers for its flow estimate, the exact engine's arena when TCP is present,
// the ordering scratch.  A failed reservation is retried by the run itself.
int prepare_capture(fluere_ctx* c) {
    if (c->reuse_ingest || !c->n_total) return FLUERE_OK;
    static const bool hostprof = getenv("FLUERE_HOSTPROF") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    int rc = upload_batches(c);
    if (!rc) rc = census(c);
    if (rc) return rc;
    if (hostprof)
        fprintf(stderr, "[fluere] attach: upload + census %.1f ms\n",
                1e3 * std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    PassPlan P;
    memset(&P, 0, sizeof P);
    P.spill = spill_mode(c);
    P.lean_merge = lean_merge(c);
    if (plan_batches(c, P) != FLUERE_OK) return FLUERE_OK;  // (stage, slow list, filter words, IPv6 ids)
    const uint64_t N = c->n_total;
    const bool tcp = c->last_n_complex != 0;
    const uint64_t want = std::min<uint64_t>(c->fmax, c->last_nf + c->last_nf / 4 + (tcp ? N / 2 : 0) + 1024);
    if (ensure_recs(c, want) != FLUERE_OK) return FLUERE_OK;
    if (grow_pair((void**)&c->d_recs, (void**)&c->d_recs2, &c->d_recs2_cap, c->d_recs_cap, sizeof(fluere_record)))
        return FLUERE_OK;
    if (c->last_mode_b) {
        if (c->d_recaux_cap < c->d_recs_cap) {
            hipFree(c->d_recaux);
            c->d_recaux = nullptr;
            c->d_recaux_cap = 0;
            if (hipMalloc(&c->d_recaux, c->d_recs_cap * 16) != hipSuccess) return FLUERE_OK;
            c->d_recaux_cap = c->d_recs_cap;
        }
        if (grow_pair((void**)&c->d_recaux, (void**)&c->d_recaux2, &c->d_recaux2_cap, c->d_recaux_cap, 16))
            return FLUERE_OK;
    }
    if (tcp || c->last_mode_b) {
        const int nb = (int)c->batches.size();
        std::vector<Batch> hb(nb);
        for (int i = 0; i < nb; i++) hb[i] = c->batches[i].b;
        ExactJob J{c->d_batches, hb.data(), nb, tables_of(c), c->use_mac, c->last_mode_b, c->timeout_ms * 1000ull,
                   c->d_complex, c->d_glob, &c->d_recs, &c->d_recs_cap, &c->d_exact, &c->d_exact_bytes};
        if (exact_reserve(J, c->stream) != FLUERE_OK) return FLUERE_OK;
    }
    {   // order_records' scratch (Mode B's bound covers Mode A's)
        auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
        const uint64_t n = c->d_recs_cap, gn = (n + 255) / 256, nw = N / 32 + 1;
        size_t tb = 0;
        (void)prim_exclusive_sum(nullptr, tb, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)(N + 1),
                                               c->stream);
        (void)ord_scratch(c, al(n * 8) + 2 * al((N + 1) * 4) + al(nw * 4) + al(n * 4) + 2 * al(gn * 4) + al(16) +
                                 al(tb));
    }
    return FLUERE_OK;
}

// The order-key array at the record buffer's capacity (without it
// order_records reads the keys from the records).  Only before the run's
// records are emitted: a new array holds no keys.
static int okey_fit(fluere_ctx* c) {
    const uint64_t cap = c->d_recs_cap;
    if (c->d_okey_cap < cap) {
        hipFree(c->d_okey);
        c->d_okey = nullptr;
        c->d_okey_cap = 0;
        if (hipMalloc(&c->d_okey, cap * 8) == hipSuccess) c->d_okey_cap = cap;
        else (void)hipGetLastError();
        c->okref = OkeyRef{c->d_okey, c->d_okey_cap};
        HIPCHECK(hipMemcpyAsync((char*)c->d_glob + sizeof(Ctl), &c->okref, sizeof(OkeyRef), hipMemcpyHostToDevice,
                                c->stream));
        // keys counted into the old array are not in this one
        HIPCHECK(hipMemsetAsync((char*)c->d_glob + offsetof(Glob, n_okey), 0, 8, c->stream));
    }
    return FLUERE_OK;
}

int ensure_recs(fluere_ctx* c, uint64_t need) {
    if (need <= c->d_recs_cap) return okey_fit(c);
    hipFree(c->d_recs);
    c->d_recs = nullptr;
    uint64_t cap = std::max<uint64_t>(need, 1024);
    if (hipMalloc(&c->d_recs, cap * sizeof(fluere_record)) != hipSuccess) return FLUERE_E_NOMEM;
    c->d_recs_cap = cap;
    return okey_fit(c);
}

extern "C" int fluere_run(fluere_ctx* c, fluere_stats* st) {
    if (!c) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    (void)hipGetLastError();  // launch checks below see only this run's errors
    hipStream_t s = c->stream;
    int rc;
    // device timing: events carried by the hot-kernel dispatches only (each event marker
    // costs a gap on the stream); the run's total is host wall time
    c->pass_in_run = true;
    c->has_aux = false;
    c->dev_ordered = false;
    c->aux.clear();
    const auto t_run0 = std::chrono::steady_clock::now();
    const TableSet T = tables_of(c);
    const int nb = (int)c->batches.size();
    const uint64_t timeout_us = c->timeout_ms * 1000ull;
    // One pass: cleanup, hot kernel + merge per batch, speculative Mode A
    // finalize over the device-side flow count, counters to the host.  In the
    // common case the whole run is this one submission and one host round
    // trip; it is replayed from a hipGraph while its plan is unchanged.
    PassPlan P;
    if ((rc = plan_pass(c, P, true))) return rc;
    c->plan_nb = P.nb;
    c->plan_spill = P.spill;
    c->plan_slow_all = P.nb > 0 && P.agg[0].slow_all;
    const auto t_plan = std::chrono::steady_clock::now();
    // hipGraph replay is opt-in (FLUERE_GRAPH=1): measured on MI355X / ROCm 7.2
    // it is slower than these few direct launches (C2 step 0.264 vs 0.257 ms)
    static const bool want_graph = getenv("FLUERE_GRAPH") != nullptr && getenv("FLUERE_DEBUG") == nullptr;
    const bool use_graph = want_graph && !c->graph_off && P.nb <= PLAN_BATCHES;
    if (P.nb > PLAN_BATCHES) {  // more batches than a plan holds: direct launches, in chunks
        if (P.clean) k_cleanup<<<P.clean_grid, 256, 0, s>>>(P.ca, P.tab_words);
        c->precleaned = false;
        std::vector<HostBatch> all = c->batches;
        int last_chunk_nb = 1;
        for (size_t i = 0; i < all.size(); i += PLAN_BATCHES) {
            c->batches.assign(all.begin() + i, all.begin() + std::min(all.size(), i + PLAN_BATCHES));
            PassPlan Q;
            memset(&Q, 0, sizeof Q);
            Q.macs = P.macs;
            Q.abl = P.abl;
            Q.spill = P.spill;
            Q.lean_merge = P.lean_merge;
            rc = plan_batches(c, Q, false);
            if (!rc) rc = enqueue_batches(c, Q);
            if (rc) break;
            last_chunk_nb = Q.nb;
        }
        c->batches = all;
        c->batches_dirty = true;
        if (rc) return rc;
        c->plan_nb = last_chunk_nb;  // device timing covers the last chunk only
        k_finalize<<<P.fin_grid, 256, 0, s>>>(P.fa);
        HIPCHECK(hipMemcpyAsync(c->h_ctl, c->d_glob, sizeof(Ctl), hipMemcpyDeviceToHost, s));
    } else if (use_graph) {
        if (!c->graph || !c->graph_plan || memcmp(c->graph_plan, &P, sizeof P) != 0) {
            if (c->graph) hipGraphExecDestroy(c->graph);
            c->graph = nullptr;
            if (!c->graph_plan) c->graph_plan = malloc(sizeof(PassPlan));
            memcpy(c->graph_plan, &P, sizeof P);  // the graph's kernel nodes read their args from here
            if (build_pass_graph(c, *reinterpret_cast<PassPlan*>(c->graph_plan), &c->graph) != FLUERE_OK) {
                c->graph = nullptr;  // no graphs on this runtime: direct launches from now on
                c->graph_off = 1;
            }
        }
        if (c->graph) {
            HIPCHECK(hipGraphLaunch(c->graph, s));
            c->precleaned = false;
        } else if ((rc = enqueue_pass(c, P))) return rc;
    } else {
        P.spec = 1;
        P.fa.host_ctl = c->h_ctl;
        P.fa.seq = ++c->run_seq ? c->run_seq : ++c->run_seq;  // never 0 (the initial value)
        // the ordering behind k_finalize when the last run was complete with
        // ended records (the steady state of a repeated workload)
        static const bool so_off = getenv("FLUERE_SO") && atoi(getenv("FLUERE_SO")) == 0;
        if (!so_off && c->so_next && (rc = so_plan(c, P.so, timeout_us))) return rc;
        if (P.so.on) {  // k_finalize sets the key bits
            P.fa.kbits = P.so.a.bits;
            P.fa.kbase = P.so.a.base;
            P.fa.rbits = P.so.a.rbits;
        }
        if ((rc = enqueue_pass(c, P))) return rc;
    }
    c->prev_nf = ~0ull;  // the pass cleared the flows: unknown until the fetch below
    // the exact engine's arena for the capture, allocated on the host while
    // the GPU runs the pass, when its flows are expected to need it (TCP in
    // Mode A, or Mode B: the census or the last run)
    if ((c->last_n_complex || c->last_mode_b) && P.spec) {
        std::vector<Batch> hb(nb);
        for (int i = 0; i < nb; i++) hb[i] = c->batches[i].b;
        ExactJob J{c->d_batches, hb.data(), nb, T, c->use_mac, c->last_mode_b, timeout_us, c->d_complex, c->d_glob,
                   &c->d_recs, &c->d_recs_cap, &c->d_exact, &c->d_exact_bytes};
        if ((rc = exact_reserve(J, s))) return rc;
    }
    Glob g;
    uint32_t nf_err[2];
    const auto t_enq = std::chrono::steady_clock::now();
    if (P.spec) {
        // k_finalize publishes the counters in the pinned host copy; poll it
        // (a blocking wait would add ~15 us of wake-up latency to every run)
        if ((rc = wait_published(c, P.fa.seq, g, nf_err))) return rc;
    } else {
        HIPCHECK(ctx_sync(c));
        g = c->h_ctl->g;
        nf_err[0] = c->h_ctl->n_flows;
        nf_err[1] = c->h_ctl->err;
        c->prev_nf = (nf_err[1] & (ERR_TABLE_FULL | ERR_SPIN)) ? ~0ull : nf_err[0];
    }
    const auto t_sync = std::chrono::steady_clock::now();
    // the speculative cleanup behind the copy clears the flows exactly when
    // the run needs no more device work (the same test, on the same counters)
    const bool spec_cleared = P.spec && run_complete(g, nf_err[1], P.spec_ca.timeout_us, P.spec_ca.recs_cap);
    c->so_next = spec_cleared && g.n_ended > 0;
    c->so_last_n = g.n_rec;
    c->so_last_ne = g.n_ended;
    if (!(nf_err[1] & (ERR_TABLE_FULL | ERR_SPIN))) c->last_nf = nf_err[0];
    // (a pass of k_slow over every packet lists none: the prediction stays)
    c->last_n_slow = c->plan_slow_all ? std::max<uint64_t>(g.n_slow, c->n_total) : g.n_slow;
    debug_counters(c, &g);
    FinArgs fa = P.fa;
    fa.kbits = nullptr;     // (and set no ordering bits)
    fa.rbits = nullptr;
    fa.host_ctl = nullptr;  // re-launches below read the counters back with copies
    if (nf_err[1] & (ERR_TABLE_FULL | ERR_SPIN)) return FLUERE_E_TABLE_FULL;
    if (nf_err[1] & ERR_FLOWS_FULL) return FLUERE_E_TABLE_FULL;
    uint32_t nf = std::min(nf_err[0], c->fmax);
    // Mode B if any flow could expire inside the capture (offline_fluereflows.rs:161-175)
    bool modeB = g.valid && (g.tmax - g.tmin) >= timeout_us;
    uint64_t n_ended = 0, n_rec = 0, updates = 0;
    fluere_stats out{};
    if (!modeB) {
        const uint64_t n_defer = g.n_fdefer;
        if (g.n_rec + n_defer > c->d_recs_cap) {  // more flows than the record buffer: grow and finalize again
            reset_record_counters(c);
            if ((rc = ensure_recs(c, nf))) return rc;
            fa.out = c->d_recs;
            fa.out_cap = c->d_recs_cap;
            k_finalize<<<flow_grid(c), 256, 0, s>>>(fa);
            HIPCHECK(hipGetLastError());
        }
        // certified flows whose first packet needs the general parser
        // (IPv6, VXLAN, IPv4 options, ...): k_finalize listed them
        if (n_defer)
            k_finalize_gen<<<(unsigned)std::min<uint64_t>(flow_grid(c), grid_for(n_defer, 256)), 256, 0, s>>>(fa);
        if (n_defer || g.n_rec > c->d_recs_cap) {
            HIPCHECK(hipGetLastError());
            HIPCHECK(hipEventRecord(c->ev2, s));
            if ((rc = read_glob(c, g))) return rc;
        }
        if (g.n_complex) {
            // flows the certificate rejected: the exact state machine (exact.hip)
            std::vector<Batch> hb(nb);
            for (int i = 0; i < nb; i++) hb[i] = c->batches[i].b;
            ExactJob J{c->d_batches, hb.data(), nb, T, c->use_mac, 0, timeout_us, c->d_complex, c->d_glob,
                       &c->d_recs, &c->d_recs_cap, &c->d_exact, &c->d_exact_bytes};
            J.cbits = c->d_cbits;
            J.mail = c->h_mail;
            J.n_rec_known = g.n_rec;  // (g: this run's counters after finalize)
            J.key_bound = nf;
            if (P.phash) {
                J.phash = c->d_phash;
                J.phash_base = c->index_base;
                J.emap = P.pid ? c->d_emap : nullptr;
                if (P.exm && P.pid) J.hot_meta = c->d_exm;
            }
            ExactResult er{};
            if ((rc = exact_run(J, s, &er))) return rc < 0 ? rc : FLUERE_E_HIP;
            out.passes = er.iterations;
            HIPCHECK(hipEventRecord(c->ev2, s));
            if ((rc = read_glob(c, g))) return rc;
        }
        // records stay on the device, the ended prefix ordered there
        n_rec = g.n_rec;
        n_ended = g.n_ended;
        updates = g.n_updates;
        c->dev_n_rec = n_rec;
        c->host_recs = false;
        out.complex_flows = g.n_complex;
        if (spec_cleared && P.so.on) {
            // ordered on the device behind k_finalize (k_so_*)
            if (n_ended && n_rec < (1ull << 32)) {
                if (n_ended * 4 > n_rec) {  // every record moved to d_recs2
                    std::swap(c->d_recs, c->d_recs2);
                    std::swap(c->d_recs_cap, c->d_recs2_cap);
                }
                c->dev_ordered = true;
                c->dev_ordered_ended = n_ended;
            }
        } else if ((rc = order_records(c, n_rec, n_ended, false, g.n_okey))) {
            return rc;
        }
    } else {
        // exact global state machine (the speculative Mode A results are discarded):
        // in parallel (exact.hip) when the timestamps are non-decreasing, else
        // the sequential kernel below
        reset_record_counters(c);
        std::vector<Batch> hb(nb);
        for (int i = 0; i < nb; i++) hb[i] = c->batches[i].b;
        ExactJob J{c->d_batches, hb.data(), nb, T, c->use_mac, 1, timeout_us, c->d_complex, c->d_glob,
                   &c->d_recs, &c->d_recs_cap, &c->d_exact, &c->d_exact_bytes};
        J.mail = c->h_mail;
        J.key_bound = nf;
        if (P.pid) {  // every valid packet's flow from the merge (AggArgs::pid)
            J.phash = c->d_phash;
            J.phash_base = c->index_base;
            J.emap = c->d_emap;
        }
        // every packet's metadata from the hot pass (all valid, none for the general parser)
        if (P.exm && g.valid == c->n_total && g.dropped == 0 && g.n_slow == 0) {
            J.dense_cm = c->d_exm;
            if (P.exm_t) J.dense_t = c->d_exm_t;
        }
        if (P.exm && P.pid) J.hot_meta = c->d_exm;  // (k_ex_meta, when the dense path is not taken)
        J.recaux = &c->d_recaux;  // the records' order words (fetch_records orders by them)
        J.recaux_cap = &c->d_recaux_cap;
        ExactResult er{};
        rc = getenv("FLUERE_SEQ_MODE_B") ? EXACT_FALLBACK : exact_run(J, s, &er);
        if (rc < 0) return rc;
        out.passes = er.iterations;
        if (rc == FLUERE_OK) {
            HIPCHECK(hipEventRecord(c->ev2, s));
            if ((rc = read_glob(c, g))) return rc;
            c->has_aux = er.replayed != 0;
            n_rec = g.n_rec;
            n_ended = g.n_ended;
            updates = g.n_updates;
            c->dev_n_rec = n_rec;
            c->host_recs = false;
            out.sequential_mode = 1;
            if (c->has_aux && (rc = order_records(c, n_rec, n_ended, true, g.n_okey))) return rc;
        } else {
        uint64_t N = c->n_total;
        SeqMeta* meta = nullptr;
        HeapEnt* heap = nullptr;
        fluere_record* cur = nullptr;
        if (!c->d_active && hipMalloc(&c->d_active, c->fmax) != hipSuccess) return FLUERE_E_NOMEM;
        uint8_t* cdir = nullptr;
        if (hipMalloc(&meta, std::max<uint64_t>(N, 1) * sizeof(SeqMeta)) != hipSuccess ||
            hipMalloc(&heap, std::max<uint64_t>(N, 1) * sizeof(HeapEnt)) != hipSuccess ||
            hipMalloc(&cur, std::max<uint32_t>(nf, 1) * sizeof(fluere_record)) != hipSuccess ||
            hipMalloc(&cdir, std::max<uint32_t>(nf, 1)) != hipSuccess) {
            hipFree(meta); hipFree(heap); hipFree(cur); hipFree(cdir);
            return FLUERE_E_NOMEM;
        }
        HIPCHECK(hipMemsetAsync(c->d_active, 0, c->fmax, s));
        for (auto& hb : c->batches) {
            if (!hb.b.n) continue;
            SeqMetaArgs ma{hb.b, T, meta, c->index_base, c->use_mac};
            k_seq_meta<<<grid_for(hb.b.n, 256), 256, 0, s>>>(ma);
        }
        if ((rc = ensure_recs(c, g.valid + 1))) return rc;
        SeqArgs sa{c->d_batches, nb, meta, N, c->d_active, cdir, cur, heap, c->d_recs, c->d_recs_cap,
                   c->d_glob, timeout_us, c->index_base, nf, c->use_mac};
        k_seq_run<<<1, 64, 0, s>>>(sa);
        HIPCHECK(hipGetLastError());
        HIPCHECK(hipMemcpyAsync(&g, c->d_glob, sizeof g, hipMemcpyDeviceToHost, s));
        HIPCHECK(ctx_sync(c));
        n_rec = g.n_rec;
        n_ended = g.n_heads;
        c->recs.resize(n_rec);
        if (n_rec)
            HIPCHECK(hipMemcpyAsync(c->recs.data(), c->d_recs, n_rec * sizeof(fluere_record), hipMemcpyDeviceToHost, s));
        HIPCHECK(hipEventRecord(c->ev2, s));
        HIPCHECK(ctx_sync(c));
        for (uint64_t i = n_ended; i < n_rec; i++) c->recs[i].order_key = NONE64;
        hipFree(meta); hipFree(heap); hipFree(cur); hipFree(cdir);
        for (auto& r : c->recs) updates += r.d_pkts;
        c->host_recs = true;
        c->dev_n_rec = n_rec;
        c->dev_ordered = false;
        out.sequential_mode = 2;
        }
    }
    // the complex-flow filter is per run: clear the bits the speculative finalize set
    if (g.n_complex) HIPCHECK(hipMemsetAsync(c->d_cbits, 0, 1u << CBITS_LOG2, s));
    c->last_n_complex = g.n_complex;
    c->last_mode_b = modeB ? 1 : 0;
    c->runs++;
    c->n_ended = n_ended;
    c->have_results = true;
    float ms_parse = 0;
    {
        const int e = hot_times(c, &ms_parse, nullptr);
        if (e != FLUERE_OK && getenv("FLUERE_HIP_VERBOSE")) fprintf(stderr, "[fluere] hot-kernel timing events failed\n");
        (void)hipGetLastError();  // a timing failure is not a run failure
    }
    const double ms_total =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_run0).count();
    c->last_run_ms = ms_total;
    out.packets = c->n_total;
    out.valid = g.valid;
    out.dropped_parse = g.dropped;
    out.flows = nf;
    out.records = n_rec;
    out.ended = n_ended;
    out.parse_ms = ms_parse;
    out.total_ms = ms_total;
    out.updates = updates;
    if (st) *st = out;
    // The run's per-flow state is not needed any more (records are kept in
    // d_recs): clear it now, asynchronously, so the next pass starts with the
    // hot kernel and the cleanup overlaps the caller's turnaround.
    if (spec_cleared || clear_flows(c) == FLUERE_OK) {
        c->precleaned = true;
        c->prev_nf = 0;
    }
    static const bool hostprof = getenv("FLUERE_HOSTPROF") != nullptr;
    if (hostprof) {
        static auto t_prev_exit = std::chrono::steady_clock::now();
        const auto t_exit = std::chrono::steady_clock::now();
        auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
        fprintf(stderr, "[fluere] host: since last exit %.1f | plan %.1f enqueue %.1f | sync wait %.1f | after sync %.1f us\n",
                us(t_prev_exit, t_run0), us(t_run0, t_plan), us(t_plan, t_enq), us(t_enq, t_sync), us(t_sync, t_exit));
        t_prev_exit = t_exit;
    }
    return FLUERE_OK;
}

extern "C" int fluere_get_records(fluere_ctx* c, fluere_record** out, uint64_t* n, uint64_t* n_ended) {
    if (!c || !out || !n) return FLUERE_E_ARG;
    if (!c->have_results) return FLUERE_E_STATE;
    int rc = fetch_records(c);
    if (rc) return rc;
    *n = c->recs.size();
    if (n_ended) *n_ended = c->n_ended;
    *out = (fluere_record*)malloc(std::max<size_t>(1, c->recs.size()) * sizeof(fluere_record));
    if (!*out) return FLUERE_E_NOMEM;
    if (!c->recs.empty()) memcpy(*out, c->recs.data(), c->recs.size() * sizeof(fluere_record));
    return FLUERE_OK;
}

extern "C" void fluere_records_free(fluere_record* r) { free(r); }

extern "C" int fluere_get_record_order(fluere_ctx* c, uint64_t* aux, uint64_t n) {
    if (!c || (!aux && n)) return FLUERE_E_ARG;
    if (!c->have_results) return FLUERE_E_STATE;
    int rc = fetch_records(c);
    if (rc) return rc;
    if (n != c->recs.size()) return FLUERE_E_ARG;
    for (uint64_t i = 0; i < n; i++) {
        aux[2 * i] = c->has_aux ? c->aux[2 * i] : 0;
        aux[2 * i + 1] = c->has_aux ? c->aux[2 * i + 1] : 0;
    }
    return FLUERE_OK;
}

// ---------------------------------------------------------------------------
// synthetic captures
// ---------------------------------------------------------------------------
extern "C" uint64_t fluere_synth_range_bytes(const fluere_synth_cfg* cfg, uint64_t first, uint64_t n) {
    if (!cfg) return 0;
    if (cfg->kind != FLUERE_SYNTH_IMIX && !synth::tcp_kind(cfg->kind) && cfg->kind != FLUERE_SYNTH_SLOW) return n * 80;
    uint64_t s = 0;
    for (uint64_t i = first; i < first + n; i++) s += 16 + synth::frame_len(*cfg, i);
    return s;
}

extern "C" uint64_t fluere_synth_file_size(const fluere_synth_cfg* cfg) {
    return cfg ? 24 + fluere_synth_range_bytes(cfg, 0, cfg->n_packets) : 0;
}

extern "C" int fluere_synth_host(const fluere_synth_cfg* cfg, uint8_t* file, uint64_t cap) {
    if (!cfg || !file) return FLUERE_E_ARG;
    if (cap < fluere_synth_file_size(cfg)) return FLUERE_E_ARG;
    uint32_t hdr[6] = {0xa1b2c3d4u, 2u | (4u << 16), 0, 0, synth::kSnap, 1};
    memcpy(file, hdr, 24);
    uint64_t off = 24;
    for (uint64_t i = 0; i < cfg->n_packets; i++) off += synth::write_record(*cfg, i, file + off);
    return FLUERE_OK;
}

extern "C" int fluere_synth_device(const fluere_synth_cfg* cfg, uint64_t first, uint64_t n, uint8_t* d_bytes,
                                   uint32_t* d_offsets, void* stream) {
    if (!cfg || !d_bytes || !d_offsets) return FLUERE_E_ARG;
    hipStream_t s = (hipStream_t)stream;
    if (!n) return FLUERE_OK;
    uint32_t* lens = nullptr;
    HIPCHECK(hipMalloc(&lens, n * 4));
    k_synth_len<<<grid_for(n, 256), 256, 0, s>>>(*cfg, first, n, lens);
    size_t tb = 0;
    void* tmp = nullptr;
    prim_exclusive_sum(nullptr, tb, lens, d_offsets, (int)n, s);
    if (hipMalloc(&tmp, std::max<size_t>(tb, 16)) != hipSuccess) { hipFree(lens); return FLUERE_E_NOMEM; }
    prim_exclusive_sum(tmp, tb, lens, d_offsets, (int)n, s);
    k_synth_write<<<grid_for(n, 256), 256, 0, s>>>(*cfg, first, n, d_bytes, d_offsets);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(s));
    hipFree(tmp);
    hipFree(lens);
    return FLUERE_OK;
}

extern "C" int fluere_debug_dense_ids(fluere_ctx* c, const uint32_t* d_keys, uint64_t n, uint32_t* d_out) {
    if (!c || (!d_keys && n) || (!d_out && n)) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    if (n) k_dense_test<<<grid_for(n, 256), 256, 0, c->stream>>>(tables_of(c), d_keys, n, d_out, c->acc.slots);
    HIPCHECK(hipGetLastError());
    HIPCHECK(ctx_sync(c));
    uint32_t nf_err[2];
    HIPCHECK(hipMemcpy(nf_err, c->d_nflows, 8, hipMemcpyDeviceToHost));
    return nf_err[1] ? FLUERE_E_TABLE_FULL : FLUERE_OK;
}

extern "C" int fluere_debug_raw(int fn, const uint8_t* d_bytes, const uint32_t* d_off, const uint32_t* d_len,
                                const uint32_t* d_arg, uint64_t n, fluere_raw_hdr* d_out, void* stream) {
    if (fn < FLUERE_RAW_FROM_RAW_PACKET || fn > FLUERE_RAW_ICMP) return FLUERE_E_ARG;
    if (n && (!d_bytes || !d_off || !d_len || !d_arg || !d_out)) return FLUERE_E_ARG;
    hipStream_t s = (hipStream_t)stream;
    if (n) k_raw_probe<<<grid_for(n, 256), 256, 0, s>>>(fn, d_bytes, d_off, d_len, d_arg, n, d_out);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(s));
    return FLUERE_OK;
}
