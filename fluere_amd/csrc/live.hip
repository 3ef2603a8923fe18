// live.hip -- live mode on batched capture (fluere_live_*).
#include "ctx.h"

// ===========================================================================
// live mode (src/net/live_fluereflow.rs:196-376) on batched capture
// ===========================================================================
// A session keeps the flows that are open across batches: a flow dictionary
// of its own (a second context's tables) and, per flow, the open instance as a
// piece (seed + order-free aggregate).  Each batch runs the shard machinery of
// the multi-GPU path with one owner (parse, order-free aggregate, the exact
// state machine for order-dependent flows, summaries + annexes) and is
// composed into the session state like the next shard of a capture.  The
// checks the reference runs after a processed packet run once per batch,
// after its last processed packet: the interval export with the idle-timeout
// scan flow.last < time - timeout (:306-358); at the end, the duration scan
// (:361-373) and the flush of every active flow (:379-392).
namespace {

struct LiveArgs {
    const uint8_t* blk;
    unsigned long long cap, cap_annex, block_bytes;
    TableSet Tp;
    uint32_t* pslots;
    fluere_flow_piece* P;
    uint8_t* P_open;
    fluere_record* out;
    unsigned long long* ctr;  // [0] records out, [1] 1 + index of the batch's last processed packet
    unsigned long long out_cap;
};

__device__ __forceinline__ void live_emit(const LiveArgs& a, const fluere_flow_piece& f, unsigned long long order) {
    fluere_record r;
    record_of_piece(f, order, r);
    const unsigned long long pos = atomicAdd(&a.ctr[0], 1ull);
    if (pos < a.out_cap) a.out[pos] = r;
}

// one thread per flow of the batch: compose its piece of the state machine
// with the session's open instance (the owner composition of k_compose with
// the session state as the previous shards)
__global__ void __launch_bounds__(256) k_live_compose(LiveArgs a) {
    uint8_t* blocks = const_cast<uint8_t*>(a.blk);
    const fluere_shard_header* h = blk_hdr(blocks, a.block_bytes, 0);
    const unsigned long long nf = min((unsigned long long)h->n_flows, a.cap);
    const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nf) return;
    const fluere_flow_summary& s = blk_sum(blocks, a.block_bytes, 0)[i];
    CKey k;
    for (int j = 0; j < 14; j++) k.w[j] = s.key[j];
    const uint32_t p = dense_of_key(a.Tp, k, true, a.pslots, nullptr);
    if (p == FAIL || p >= a.Tp.fmax) return;  // (the error word is set)
    fluere_flow_piece F = a.P[p];
    bool open = a.P_open[p] != 0;
    const bool open_in = open;
    fluere_flow_piece A, H, T;
    bool has_f0, has_H, has_T;
    unsigned long long f0, lastp = 0;
    if (s.annex == NONE32) {
        piece_of_summary(s, A);
        has_f0 = s.finrst_min != NONE64;
        f0 = s.finrst_min;
        has_H = s.first_create != NONE64;
        H = A;
        has_T = false;
        if (open_in || has_H) lastp = s.last + 1;  // every packet processed, or none (SYN-gated)
    } else {
        const fluere_flow_annex& x = blk_annex(blocks, a.block_bytes, a.cap, 0)[s.annex];
        has_f0 = x.flags & 1;
        f0 = x.f0;
        has_H = x.flags & 4;
        has_T = x.flags & 8;
        piece_clear(A);
        if (x.flags & 2) piece_add(A, x.lead);
        if (has_H) piece_add(A, x.head);
        H = x.head;
        T = x.tail;
        if (open_in) lastp = A.last + 1;
        else if (has_H) lastp = H.last + 1;
        lastp = max(lastp, (unsigned long long)x.mid_last);
        if (has_T) lastp = max(lastp, T.last + 1);
    }
    if (open) {
        piece_add(F, A);
        if (has_f0) {
            live_emit(a, F, f0);
            open = false;
        }
    } else if (has_f0) {
        if (has_H) live_emit(a, H, f0);
    } else if (has_H) {
        F = H;
        open = true;
    }
    if (has_f0 && has_T) {
        F = T;
        open = true;
    }
    a.P[p] = F;
    a.P_open[p] = open ? 1 : 0;
    if (lastp) atomicMax(&a.ctr[1], lastp);
}

// idle-timeout / duration scan (lim: flow.last < lim expires) or the final flush (all)
__global__ void __launch_bounds__(256) k_live_scan(LiveArgs a, unsigned long long lim, int all) {
    const uint32_t np = min(*a.Tp.n_flows, a.Tp.fmax);
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < np; p += gridDim.x * blockDim.x) {
        if (!a.P_open[p]) continue;
        const fluere_flow_piece F = a.P[p];
        if (!all && !(F.last_time < lim)) continue;
        live_emit(a, F, NONE64);
        a.P_open[p] = 0;
    }
}

// session dictionary compaction: the open flows' keys and pieces out ...
__global__ void __launch_bounds__(256) k_live_collect(LiveArgs a, const uint8_t* flow_key, uint8_t* ckey,
                                                      fluere_flow_piece* cpiece, unsigned long long* cnt) {
    const uint32_t np = min(*a.Tp.n_flows, a.Tp.fmax);
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < np; p += gridDim.x * blockDim.x) {
        if (!a.P_open[p]) continue;
        const unsigned long long i = atomicAdd(cnt, 1ull);
        const uint4* src = reinterpret_cast<const uint4*>(flow_key + (size_t)p * 56);
        uint2* dst = reinterpret_cast<uint2*>(ckey + i * 56);
        const uint2* s2 = reinterpret_cast<const uint2*>(src);
        for (int k = 0; k < 7; k++) dst[k] = s2[k];
        cpiece[i] = a.P[p];
        a.P_open[p] = 0;
    }
}
// ... and back into the cleared dictionary (new dense ids)
__global__ void __launch_bounds__(256) k_live_reinsert(LiveArgs a, const uint8_t* ckey, const fluere_flow_piece* cpiece,
                                                       unsigned long long n) {
    const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    CKey k;
    const uint32_t* kw = reinterpret_cast<const uint32_t*>(ckey + i * 56);
    for (int j = 0; j < 14; j++) k.w[j] = kw[j];
    const uint32_t p = dense_of_key(a.Tp, k, true, a.pslots, nullptr);
    if (p == FAIL || p >= a.Tp.fmax) return;  // (the error word is set)
    a.P[p] = cpiece[i];
    a.P_open[p] = 1;
}

__global__ void k_live_time(const Batch* bs, int nb, unsigned long long gi, int macs, unsigned long long* t) {
    if (threadIdx.x || blockIdx.x) return;
    Parsed P;
    parse_global(bs, nb, gi, macs != 0, P);
    *t = P.t;
}

}  // namespace

struct fluere_live {
    fluere_ctx* batch = nullptr;    // the current batch: packets, flows, export
    fluere_ctx* persist = nullptr;  // the session's flow dictionary (its tables only)
    fluere_flow_piece* P = nullptr;
    uint8_t* P_open = nullptr;
    uint8_t* blk = nullptr;
    uint64_t cap = 1024, cap_annex = 256, blk_bytes = 0;
    fluere_record* out = nullptr;
    uint64_t out_cap = 0;
    unsigned long long* ctr = nullptr;
    uint64_t base = 0;              // global index of the batch's first packet
    uint64_t timeout_ms = 600000;
    int use_mac = 0;
    bool last_have = false;         // the last batch had a processed packet ...
    uint64_t last_time = 0;         // ... at this time (the checks' `time`)
    bool export_due = false;        // an interval elapsed: export after the next processed packet
    std::vector<fluere_record> pending;  // FIN/RST-closed records since the last export
    uint64_t persist_nf = 0;        // flows in the session dictionary (open or not)
    uint8_t* ckey = nullptr;        // compaction scratch: open flows' keys and pieces
    fluere_flow_piece* cpiece = nullptr;
    uint64_t ccap = 0;
};

extern "C" int fluere_live_open(const fluere_opts* o, fluere_live** out) {
    if (!out) return FLUERE_E_ARG;
    *out = nullptr;
    fluere_opts def{};
    def.timeout_ms = 600000;
    if (!o) o = &def;
    fluere_live* lv = new (std::nothrow) fluere_live();
    if (!lv) return FLUERE_E_NOMEM;
    int rc = fluere_open(o, &lv->batch);
    if (!rc) lv->batch->reuse_ingest = true;  // one batch per call: keep the ingest buffers
    if (!rc) rc = fluere_open(o, &lv->persist);
    const uint64_t pmax = lv->persist ? lv->persist->fmax : 0;
    if (!rc && (hipMalloc(&lv->P, pmax * sizeof(fluere_flow_piece)) != hipSuccess ||
                hipMalloc(&lv->P_open, pmax) != hipSuccess || hipMalloc(&lv->ctr, 16) != hipSuccess))
        rc = FLUERE_E_NOMEM;
    if (!rc && hipMemset(lv->P_open, 0, pmax) != hipSuccess) rc = FLUERE_E_HIP;
    if (rc) {
        fluere_live_close(lv);
        return rc;
    }
    lv->timeout_ms = o->timeout_ms;
    lv->use_mac = o->use_mac ? 1 : 0;
    *out = lv;
    return FLUERE_OK;
}

extern "C" int fluere_live_close(fluere_live* lv) {
    if (!lv) return FLUERE_OK;
    fluere_close(lv->batch);
    fluere_close(lv->persist);
    hipFree(lv->P);
    hipFree(lv->P_open);
    hipFree(lv->blk);
    hipFree(lv->out);
    hipFree(lv->ctr);
    hipFree(lv->ckey);
    hipFree(lv->cpiece);
    delete lv;
    return FLUERE_OK;
}

static LiveArgs live_args(fluere_live* lv) {
    LiveArgs a{lv->blk, lv->cap, lv->cap_annex, lv->blk_bytes, tables_of(lv->persist), lv->persist->acc.slots,
               lv->P, lv->P_open, lv->out, lv->ctr, lv->out_cap};
    return a;
}

// records [0, ctr[0]) of lv->out -> host (appended to v)
static int live_take(fluere_live* lv, std::vector<fluere_record>& v) {
    hipStream_t s = lv->batch->stream;
    unsigned long long n = 0;
    HIPCHECK(hipMemcpyAsync(&n, lv->ctr, 8, hipMemcpyDeviceToHost, s));
    HIPCHECK(hipStreamSynchronize(s));
    if (n > lv->out_cap) return FLUERE_E_NOMEM;
    const size_t at = v.size();
    v.resize(at + n);
    if (n) HIPCHECK(hipMemcpyAsync(v.data() + at, lv->out, n * sizeof(fluere_record), hipMemcpyDeviceToHost, s));
    HIPCHECK(hipMemsetAsync(lv->ctr, 0, 8, s));
    HIPCHECK(hipStreamSynchronize(s));
    return FLUERE_OK;
}

static int live_ensure_out(fluere_live* lv, uint64_t need) {
    if (need <= lv->out_cap) return FLUERE_OK;
    hipFree(lv->out);
    lv->out = nullptr;
    lv->out_cap = 0;
    if (hipMalloc(&lv->out, need * sizeof(fluere_record)) != hipSuccess) return FLUERE_E_NOMEM;
    lv->out_cap = need;
    return FLUERE_OK;
}

// an export's records: the FIN/RST-closed ones since the last export in their
// order (the packet that closed them), then the scan's
static int live_export(fluere_live* lv, std::vector<fluere_record>& scan, fluere_record** recs, uint64_t* n,
                       uint64_t* n_ordered) {
    std::stable_sort(lv->pending.begin(), lv->pending.end(),
                     [](const fluere_record& x, const fluere_record& y) { return x.order_key < y.order_key; });
    const uint64_t total = lv->pending.size() + scan.size();
    *recs = (fluere_record*)malloc(std::max<uint64_t>(total, 1) * sizeof(fluere_record));
    if (!*recs) return FLUERE_E_NOMEM;
    if (!lv->pending.empty()) memcpy(*recs, lv->pending.data(), lv->pending.size() * sizeof(fluere_record));
    if (!scan.empty()) memcpy(*recs + lv->pending.size(), scan.data(), scan.size() * sizeof(fluere_record));
    *n = total;
    if (n_ordered) *n_ordered = lv->pending.size();
    lv->pending.clear();
    return FLUERE_OK;
}

// The session dictionary keeps a key until it is compacted: flows closed by
// FIN/RST or expired by a scan leave the reference's active_flow
// (live_fluereflow.rs:299,336,371), so the session's state is bounded by its
// open flows.  When the dictionary cannot take a batch's new flows, the open
// flows are re-inserted into a cleared dictionary.
static int live_compact(fluere_live* lv) {
    fluere_ctx* pc = lv->persist;
    hipStream_t s = lv->batch->stream;
    const uint64_t fmax = pc->fmax;
    if (lv->ccap < fmax) {
        hipFree(lv->ckey);
        hipFree(lv->cpiece);
        lv->ckey = nullptr;
        lv->cpiece = nullptr;
        lv->ccap = 0;
        if (hipMalloc(&lv->ckey, fmax * 56) != hipSuccess ||
            hipMalloc(&lv->cpiece, fmax * sizeof(fluere_flow_piece)) != hipSuccess)
            return FLUERE_E_NOMEM;
        lv->ccap = fmax;
    }
    LiveArgs a = live_args(lv);
    HIPCHECK(hipMemsetAsync(lv->ctr + 1, 0, 8, s));
    k_live_collect<<<flow_grid(pc), 256, 0, s>>>(a, pc->d_flow_key, lv->ckey, lv->cpiece, lv->ctr + 1);
    unsigned long long n = 0;
    HIPCHECK(hipMemcpyAsync(&n, lv->ctr + 1, 8, hipMemcpyDeviceToHost, s));
    HIPCHECK(hipStreamSynchronize(s));
    int rc = clear_flows(pc);  // (on the dictionary context's stream)
    if (rc) return rc;
    HIPCHECK(hipStreamSynchronize(pc->stream));
    if (n) k_live_reinsert<<<grid_for(n, 256), 256, 0, s>>>(a, lv->ckey, lv->cpiece, n);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(s));
    lv->persist_nf = n;
    return FLUERE_OK;
}

static int live_batch(fluere_live* lv, const uint8_t* pcap, uint64_t nbytes, const uint64_t* rec_off, uint64_t n_recs,
                      int do_export, fluere_record** recs, uint64_t* n, uint64_t* n_ordered, int* exported);

extern "C" int fluere_live_batch(fluere_live* lv, const uint8_t* pcap, uint64_t nbytes, int do_export,
                                 fluere_record** recs, uint64_t* n, uint64_t* n_ordered, int* exported) {
    return live_batch(lv, pcap, nbytes, nullptr, 0, do_export, recs, n, n_ordered, exported);
}

extern "C" int fluere_live_batch_indexed(fluere_live* lv, const uint8_t* pcap, uint64_t nbytes, const uint64_t* rec_off,
                                         uint64_t n_recs, int do_export, fluere_record** recs, uint64_t* n,
                                         uint64_t* n_ordered, int* exported) {
    if (!rec_off && n_recs) return FLUERE_E_ARG;
    return live_batch(lv, pcap, nbytes, rec_off ? rec_off : (const uint64_t*)"", n_recs, do_export, recs, n, n_ordered,
                      exported);
}

static int live_batch(fluere_live* lv, const uint8_t* pcap, uint64_t nbytes, const uint64_t* rec_off, uint64_t n_recs,
                      int do_export, fluere_record** recs, uint64_t* n, uint64_t* n_ordered, int* exported) {
    if (!lv || !pcap || !recs || !n) return FLUERE_E_ARG;
    *recs = nullptr;
    *n = 0;
    if (n_ordered) *n_ordered = 0;
    if (exported) *exported = 0;
    fluere_ctx* c = lv->batch;
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    int rc;
    static const bool hostprof = getenv("FLUERE_HOSTPROF") != nullptr;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto ms = [](auto x, auto y) { return std::chrono::duration<double, std::milli>(y - x).count(); };
    const auto t0 = now();
    auto t1 = t0, t2 = t0, t3 = t0, t4 = t0;
    if ((rc = fluere_reset(c))) return rc;
    if ((rc = fluere_set_index_base(c, lv->base))) return rc;
    if (rec_off && !is_pcapng(pcap, nbytes)) rc = add_host_pcap_indexed(c, pcap, nbytes, rec_off, n_recs);
    else rc = fluere_add_host_pcap(c, pcap, nbytes);
    if (rc) return rc;
    lv->base += c->n_total;
    lv->last_have = false;
    if (c->n_total) {
        t1 = now();
        if ((rc = fluere_parse_aggregate(c))) return rc;
        if (hostprof) HIPCHECK(hipStreamSynchronize(s));
        t2 = now();
        uint64_t need_nf = 0;
        for (;;) {  // one owner: the whole batch
            const uint64_t bb = fluere_shard_block_bytes(lv->cap, lv->cap_annex);
            if (bb > lv->blk_bytes) {
                hipFree(lv->blk);
                lv->blk = nullptr;
                lv->blk_bytes = 0;
                if (hipMalloc(&lv->blk, bb) != hipSuccess) return FLUERE_E_NOMEM;
                lv->blk_bytes = bb;
            }
            uint64_t need = 0, need_a = 0;
            if ((rc = fluere_export_device(c, lv->blk, 1, 0, lv->cap, lv->cap_annex, &need, &need_a))) return rc;
            need_nf = need;
            if (need <= lv->cap && need_a <= lv->cap_annex) break;
            while (lv->cap < need) lv->cap *= 2;
            while (lv->cap_annex < need_a) lv->cap_annex *= 2;
        }
        // the records that opened and closed inside this batch
        const size_t at = lv->pending.size();
        lv->pending.resize(at + c->local_n_rec);
        if (c->local_n_rec)
            HIPCHECK(hipMemcpyAsync(lv->pending.data() + at, c->d_recs, c->local_n_rec * sizeof(fluere_record),
                                    hipMemcpyDeviceToHost, s));
        c->local_n_rec = c->local_updates = c->local_ended = 0;
        t3 = now();
        // room for the batch's flows in the session dictionary (need: the
        // batch's flow count, one owner): compact it first when short
        if (lv->persist_nf + need_nf > lv->persist->fmax) {
            if ((rc = live_compact(lv))) return rc;
            if (lv->persist_nf + need_nf > lv->persist->fmax) return FLUERE_E_TABLE_FULL;  // too many open flows
        }
        if ((rc = live_ensure_out(lv, lv->cap + lv->persist->fmax))) return rc;
        HIPCHECK(hipMemsetAsync(lv->ctr, 0, 16, s));
        LiveArgs a = live_args(lv);
        a.block_bytes = fluere_shard_block_bytes(lv->cap, lv->cap_annex);
        k_live_compose<<<grid_for(lv->cap, 256), 256, 0, s>>>(a);
        HIPCHECK(hipGetLastError());
        unsigned long long tend = 0;
        HIPCHECK(hipMemcpyAsync(&tend, lv->ctr + 1, 8, hipMemcpyDeviceToHost, s));
        uint32_t pnf[2] = {0, 0};
        HIPCHECK(hipMemcpyAsync(pnf, lv->persist->d_nflows, 8, hipMemcpyDeviceToHost, s));
        if ((rc = live_take(lv, lv->pending))) return rc;
        if (pnf[1]) return FLUERE_E_TABLE_FULL;  // (cannot happen: room was made above)
        lv->persist_nf = pnf[0];
        if (tend) {
            k_live_time<<<1, 64, 0, s>>>(c->d_batches, (int)c->batches.size(), tend - 1, c->use_mac, lv->ctr + 1);
            HIPCHECK(hipMemcpyAsync(&lv->last_time, lv->ctr + 1, 8, hipMemcpyDeviceToHost, s));
            HIPCHECK(hipStreamSynchronize(s));
            lv->last_have = true;
        }
        t4 = now();
        if (hostprof)
            fprintf(stderr, "[fluere] live batch: ingest %.2f parse+aggregate %.2f export %.2f compose+take %.2f ms\n",
                    ms(t0, t1), ms(t1, t2), ms(t2, t3), ms(t3, t4));
    }
    // the interval check runs after a processed packet: an interval that
    // elapsed in a batch without one exports at the next batch with one
    if (do_export) lv->export_due = true;
    if (!lv->export_due || !lv->last_have) return FLUERE_OK;
    lv->export_due = false;
    std::vector<fluere_record> scan;
    const auto t5 = now();
    if (lv->timeout_ms > 0) {
        LiveArgs a = live_args(lv);
        a.block_bytes = fluere_shard_block_bytes(lv->cap, lv->cap_annex);
        k_live_scan<<<flow_grid(lv->persist), 256, 0, s>>>(a, lv->last_time - lv->timeout_ms * 1000ull, 0);
        HIPCHECK(hipGetLastError());
        if ((rc = live_take(lv, scan))) return rc;
    }
    if (exported) *exported = 1;
    const auto t6 = now();
    rc = live_export(lv, scan, recs, n, n_ordered);
    if (hostprof)
        fprintf(stderr, "[fluere] live export: scan+take %.2f (%zu records) order+copy %.2f ms (%llu records)\n",
                ms(t5, t6), scan.size(), ms(t6, now()), (unsigned long long)*n);
    return rc;
}

extern "C" int fluere_live_finish(fluere_live* lv, int duration_end, fluere_record** recs, uint64_t* n,
                                  uint64_t* n_ordered) {
    if (!lv || !recs || !n) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(lv->batch->device));
    hipStream_t s = lv->batch->stream;
    int rc;
    if ((rc = live_ensure_out(lv, lv->cap + lv->persist->fmax))) return rc;
    std::vector<fluere_record> tail;
    LiveArgs a = live_args(lv);
    a.block_bytes = fluere_shard_block_bytes(lv->cap, lv->cap_annex);
    if (duration_end && lv->last_have) {  // the duration scan (no timeout > 0 guard, :364-366)
        k_live_scan<<<flow_grid(lv->persist), 256, 0, s>>>(a, lv->last_time - lv->timeout_ms * 1000ull, 0);
        HIPCHECK(hipGetLastError());
        if ((rc = live_take(lv, tail))) return rc;
    }
    k_live_scan<<<flow_grid(lv->persist), 256, 0, s>>>(a, 0, 1);  // every active flow (:379-383)
    HIPCHECK(hipGetLastError());
    if ((rc = live_take(lv, tail))) return rc;
    return live_export(lv, tail, recs, n, n_ordered);
}
