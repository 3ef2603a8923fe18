// ctx.h -- the host-side context of the library (fluere_ctx) and the host
// helpers its translation units share (fluere_gpu.hip: lifecycle, planning,
// runs; ingest.hip; order.hip; shard.hip; live.hip).
#pragma once
#include "kern.h"

// ===========================================================================
// host side
// ===========================================================================

struct HostBatch {
    Batch b{};
    void* own_bytes = nullptr;
    void* own_offs = nullptr;
    uint2* own_desc = nullptr;  // chunk descriptors (built by upload_batches)
};

namespace fl {
struct MergePending;
}

struct fluere_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    // Ingest arena (live sessions: a batch per call): the device image, its
    // record offsets and the pinned staging chunks are kept and reused instead
    // of allocated per batch (hipHostMalloc of the staging alone cost ms)
    bool reuse_ingest = false;
    uint8_t* ar_d = nullptr;
    uint64_t ar_d_cap = 0;
    uint32_t* ar_offs = nullptr;
    uint64_t ar_offs_cap = 0;
    uint8_t* ar_pin[8] = {};
    hipEvent_t ar_ev[8] = {};
    uint64_t timeout_ms = 600000;
    int use_mac = 0;
    uint32_t C = 0, fmax = 0;
    int n_cu = 256;
    std::vector<HostBatch> batches;
    uint64_t n_total = 0;
    uint64_t index_base = 0;
    // device state
    unsigned long long* d_tab = nullptr;
    void* d_acc = nullptr;
    Acc acc{};
    uint32_t* d_nflows = nullptr;  // [0] n_flows, [1] err (inside the d_glob allocation: Ctl)
    Glob* d_glob = nullptr;        // Ctl
    unsigned long long* d_bctr = nullptr;  // per-batch counters of a pass of several batches (AggArgs::bc), 8 x 8 words
    Ctl* h_ctl = nullptr;          // pinned host copy
    HostMail* h_mail = nullptr;    // pinned mailbox of the exact engine's host reads (exact.h)
    bool batches_dirty = true;
    uint8_t* d_flow_key = nullptr;
    uint8_t* d_complex = nullptr;
    uint32_t* d_fdefer = nullptr;  // k_finalize -> k_finalize_gen: flows for the general parser [fmax]
    uint8_t* d_cbits = nullptr;    // complex-flow filter of the exact engine (1 << CBITS_LOG2 bytes)
    uint8_t* d_active = nullptr;
    Batch* d_batches = nullptr;
    int d_batches_cap = 0;
    fluere_record* d_recs = nullptr;
    uint64_t d_recs_cap = 0;
    void* d_pay = nullptr;      // FirstPay[fmax] (merge)
    uint32_t* d_slow = nullptr; // slow-path packet list (one batch)
    uint64_t d_slow_cap = 0;
    uint32_t* d_sd = nullptr;   // merge scratch (summary -> dense id)
    uint64_t d_sd_cap = 0;
    void* d_stage = nullptr;    // hot-kernel partial aggregates (Stage)
    void* d_exact = nullptr;    // exact state machine scratch (exact.hip)
    size_t d_exact_bytes = 0;
    // multi-GPU export: annexes of the shard's order-dependent flows, their
    // index per flow, the largest per-owner counts; the final records the
    // export produced (kept through the owner merge)
    fluere_flow_annex* d_annex = nullptr;
    uint64_t d_annex_cap = 0;
    uint32_t* d_annex_of = nullptr;
    uint32_t* d_sumpos = nullptr;                // [fmax] summary position of each flow in its owner's block
    void* d_v6map = nullptr;                     // k_slow's IPv6 address-id map (V6Map: 3 key levels, addr_of)
    uint32_t v6C = 0;
    void* d_wire_tmp = nullptr;                  // fluere_wire_pack scratch (sizes, scan, offsets, scan temp)
    size_t d_wire_tmp_bytes = 0;
    void* d_need = nullptr;
    uint64_t merge_cap = 0;                      // the last merge's block capacity and shard count
    uint32_t merge_shards = 0;
    struct SweepState* sw = nullptr;             // sharded Mode B (fluere_sweep_*)
    unsigned long long* d_recaux = nullptr;      // sharded Mode B: 2 order words per record
    uint64_t d_recaux_cap = 0;
    bool has_aux = false;                        // the results carry order words (d_recaux)
    std::vector<unsigned long long> aux;         // host copy, in the order of recs
    uint64_t local_n_rec = 0, local_updates = 0, local_ended = 0;
    size_t d_stage_bytes = 0;
    bool generic_dirty = false;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
    // start / stop of each hot-kernel launch of the last pass (batch i: evh[2i],
    // evh[2i + 1]; carried by the dispatch itself, hipExtLaunchKernel)
    hipEvent_t evh[2 * 8] = {};
    hipEvent_t ev_ctl = nullptr;                // after a run's counter copy (the speculative cleanup follows)
    uint64_t last_nf = 0;                       // flows of the last completed run (sizing only)
    uint64_t last_n_slow = 0;                   // slow-list packets of the last run (k_slow prediction)
    uint64_t last_n_complex = 0;                // complex flows of the last run, and whether it was Mode B:
    int last_mode_b = 0;                        //   the phash prediction (the exact engine's Mode A filter)
    uint32_t* d_phash = nullptr;                // per packet: ckey_bucket or PH_PARSE (AggArgs::phash), then the
    uint64_t phash_cap = 0;                     //   merge's flow words (AggArgs::pid)
    uint32_t* d_emap = nullptr;                 // merge entry -> dense id (AggArgs::emap), PLAN_BATCHES << 21 words
    bool async_nf = false;                      // fluere_export_async left the shard's flow count in h_ctl->pad[0]
    bool pass_in_run = false;
    bool precleaned = false;                    // the flow state is clear (k_cleanup already enqueued)
    uint32_t run_seq = 0;                       // number of the last run that publishes its counters (Ctl::seq)
    int plan_nb = 0;                            // batches of the last pass
    int plan_spill = 0;                         // the last pass's hot kernel was k_parse_spill
    int plan_slow_all = 0;                      // ... or k_slow over every packet (no hot kernel)
    double last_run_ms = 0;                     // host wall time of the last fluere_run
    // census of a newly attached capture (k_census): due when batches were
    // attached since the last pass; its sample counts and flow estimate
    bool census_due = false;
    uint64_t runs = 0;                          // passes run on this context
    void* d_census = nullptr;                   // fingerprint table, counts, CensusOut
    unsigned long long census_v[10] = {};       // CensusOut + the flow estimate (fluere_last_census)
    int census_ran = 0;
    // hipGraph of the last fluere_run pass, replayed while the plan is unchanged
    hipGraphExec_t graph = nullptr;
    void* graph_plan = nullptr;                 // PassPlan the graph was captured from
    int graph_off = 0;                          // 1: graphs disabled (env or a failed capture)
    uint64_t prev_nf = ~0ull;                   // flows of the last fetched run (cleanup grid); ~0: unknown
    // results
    std::vector<fluere_record> recs;  // host copy of the records (made on demand)
    uint64_t n_ended = 0;
    bool have_results = false;
    bool host_recs = false;          // recs holds the last results
    uint64_t dev_n_rec = 0;          // records of the last results in d_recs (Mode A / merge order: by order_key)
    // the device ordered the ended prefix (order_records): [ended, in the
    // reference's order][active]; the second buffers are the scatter targets
    bool dev_ordered = false;
    uint64_t dev_ordered_ended = 0;
    fluere_record* d_recs2 = nullptr;
    uint64_t d_recs2_cap = 0;
    unsigned long long* d_recaux2 = nullptr;
    uint64_t d_recaux2_cap = 0;
    void* d_ord = nullptr;           // order_records scratch
    size_t d_ord_bytes = 0;
    unsigned long long* d_okey = nullptr;  // the records' order keys, written by the emitters (OkeyRef)
    uint64_t d_okey_cap = 0;
    OkeyRef okref{};                       // its device copy follows the Ctl in d_glob
    // the ordering enqueued behind k_finalize (order.hip: so_plan): two bit
    // arrays used in turn (each run clears the other's dirty words), scratch
    uint32_t* d_sob = nullptr;       // [2][sob_cap] key bit words
    uint64_t sob_cap = 0;
    uint64_t sob_dirty[2] = {0, 0};  // words a past run may have set, per array
    uint32_t* d_sorb = nullptr;      // [2][sorb_cap] record bit words
    uint64_t sorb_cap = 0;
    uint64_t sorb_dirty[2] = {0, 0};
    int sob_cur = 0;
    void* d_sos = nullptr;           // wpre | tpre | ctr | holes
    size_t sos_bytes = 0;
    // the owner merge of the device-agreed sharded step (shard.hip)
    fl::MergePending* merge_p = nullptr;
    std::chrono::steady_clock::time_point merge_t0{};
    uint64_t host_waits = 0;                    // blocking host waits on the stream (ctx_sync, wait_published polls)
    unsigned long long* d_exm_t = nullptr;  // Mode B predicted: the packets' times beside d_exm (AggArgs::exm_t)
    ExMeta* d_exm = nullptr;         // Mode B predicted: the hot pass's per-packet replay metadata (AggArgs::exm)
    uint64_t exm_t_cap = 0;       // packets d_exm_t holds
    uint64_t exm_cap = 0;         // packets d_exm holds
    bool so_next = false;            // the last run was complete with ended records: enqueue the ordering
    uint64_t so_last_n = 0, so_last_ne = 0;
};

// The Mode A ordering enqueued behind k_finalize, before the host has read
// the run's counters (order.hip).  Its kernels read the counters on the
// device and do nothing unless the run is complete (run_complete, the same
// test as the speculative k_cleanup's) with ended records.
struct SoArgs {
    const Glob* g;
    const uint32_t* err;
    unsigned long long timeout_us, recs_cap;
    fluere_record* r;   // d_recs
    fluere_record* r2;  // d_recs2 (capacity >= recs_cap)
    uint64_t base;      // the capture's first packet index
    uint64_t nw;        // key bit words of this run: N / 32 + 1
    uint32_t kt, rt;    // tiles of 1024 words: key bits, record bits
    uint32_t* bits;     // [nw] key bits: one per packet, zero on entry
    uint32_t* zbits;    // the other key array: its first zn words cleared for the next run
    uint64_t zn;
    uint16_t* wpre;     // [nw] key bits below each word within its tile
    uint32_t* rbits;    // record bits: one per record, set by k_finalize when ended (zero on entry)
    uint32_t* zrbits;   // the other record array: its first zrn words cleared for the next run
    uint64_t zrn;
    uint16_t* rwpre;    // their per-word prefixes within a tile
    uint32_t* tpre;     // [kt + rt] tile totals, then their exclusive prefixes
    uint32_t* holes;    // [recs_cap] the ended records at or past n_ended, by rank
};
struct SoLaunch {
    SoArgs a;
    unsigned g_scan, g_out, g_fill;
    int on;
};


// Ablation knobs that give wrong results (FLUERE_ABLATE, FLUERE_SLOW_ABL,
// FLUERE_CLEAN_ABL, FLUERE_KEEP_DICT) are read only by diagnostic builds
// (`make variant NAME=x DEFS="-DFLUERE_DIAG=1"`); the product library ignores them.
#ifndef FLUERE_DIAG
#define FLUERE_DIAG 0
#endif
inline int diag_knob(const char* name) {
    if (!FLUERE_DIAG) return 0;
    const char* v = getenv(name);
    if (!v) return 0;
    // a number is taken as given (FLUERE_ABLATE=0: the full kernel); any other
    // value switches the knob on
    char* end = nullptr;
    const long x = strtol(v, &end, 10);
    return end != v ? (int)x : 1;
}

// host helpers shared by the translation units
int upload_batches(fluere_ctx* c);  // fluere_gpu.hip
TableSet tables_of(fluere_ctx* c);  // fluere_gpu.hip
void reset_record_counters(fluere_ctx* c);  // fluere_gpu.hip
unsigned flow_grid(fluere_ctx* c);  // fluere_gpu.hip
unsigned done_grid(fluere_ctx* c, uint64_t n);  // fluere_gpu.hip
int clear_flows(fluere_ctx* c);
// hipStreamSynchronize of the context stream, counted (fluere_host_waits)
inline hipError_t ctx_sync(fluere_ctx* c) {
    c->host_waits++;
    return hipStreamSynchronize(c->stream);
}  // fluere_gpu.hip
int wait_published(fluere_ctx* c, uint32_t seq, Glob& g, uint32_t (&nf_err)[2]);  // fluere_gpu.hip
int read_glob(fluere_ctx* c, Glob& g);  // fluere_gpu.hip
int prepare_capture(fluere_ctx* c);  // fluere_gpu.hip
int fetch_records(fluere_ctx* c);  // fluere_gpu.hip
int ensure_recs(fluere_ctx* c, uint64_t need);  // fluere_gpu.hip
int census(fluere_ctx* c);  // fluere_gpu.hip
int init_glob(fluere_ctx* c);  // fluere_gpu.hip
void debug_counters(fluere_ctx* c, const Glob* have = nullptr);  // fluere_gpu.hip
void free_batches(fluere_ctx* c);  // fluere_gpu.hip
int alloc_flow_state(fluere_ctx* c, uint64_t mf);  // fluere_gpu.hip
void free_flow_state(fluere_ctx* c);  // fluere_gpu.hip
int grow_flow_state(fluere_ctx* c, uint64_t want);  // fluere_gpu.hip
int bulk_clean(const fluere_ctx* c, uint64_t nf);  // fluere_gpu.hip
void sweep_free(fluere_ctx* c);  // shard.hip
void merge_pending_free(fluere_ctx* c);  // shard.hip
int grow_recs_keep(fluere_ctx* c, uint64_t need, uint64_t keep);  // shard.hip
int grow_pair(void** a, void** b, uint64_t* cap_b, uint64_t cap_a, size_t unit);  // order.hip
int ord_scratch(fluere_ctx* c, size_t need);  // order.hip
int order_records(fluere_ctx* c, uint64_t n, uint64_t n_ended, bool mode_b, uint64_t n_okey);  // order.hip
int sort_actives(fluere_ctx* c, uint64_t ne, uint64_t m);  // order.hip
int so_plan(fluere_ctx* c, SoLaunch& L, unsigned long long timeout_us);  // order.hip
int so_enqueue(fluere_ctx* c, const SoLaunch& L);                        // order.hip
void so_free(fluere_ctx* c);                                             // order.hip
int add_host_pcap_indexed(fluere_ctx* c, const uint8_t* file, uint64_t nbytes, const uint64_t* rec_off, uint64_t n_recs);  // ingest.hip

// order.hip
__global__ void __launch_bounds__(256) k_ord_keys(const fluere_record* r, uint64_t n, uint64_t base, int mode_b, const unsigned long long* ok_in, unsigned long long* okey, uint32_t* bits, uint32_t* cnt, uint32_t* gmax, uint32_t* blk_act);
__global__ void __launch_bounds__(256) k_ord_popc(const uint32_t* bits, uint64_t nw, uint32_t* pc);
__global__ void __launch_bounds__(256) k_ob_fill(const unsigned long long* okey, uint64_t n, uint64_t base, uint32_t* cnt, const uint32_t* start, uint32_t* mem);
__global__ void __launch_bounds__(256) k_ord_move(const fluere_record* r, const unsigned long long* aux, uint64_t n, uint64_t base, const unsigned long long* okey, const uint32_t* bits, const uint32_t* pre, const uint32_t* start, const uint32_t* mem, const uint32_t* blk_pre, uint64_t n_ended, fluere_record* out, unsigned long long* aux_out);
__global__ void __launch_bounds__(256) k_ord_out(const fluere_record* r, uint64_t n, uint64_t base, const unsigned long long* okey, const uint32_t* bits, const uint32_t* pre, const uint32_t* blk_pre, uint64_t n_ended, fluere_record* out, uint32_t* holes, uint32_t* head_act);
__global__ void __launch_bounds__(256) k_ord_fill(fluere_record* r, const unsigned long long* okey, const uint32_t* blk_pre, uint64_t n_ended, const uint32_t* holes, const uint32_t* head_act);
__global__ void k_act_keys(const fluere_record* r, uint64_t m, unsigned long long* keys, uint32_t* vals);
__global__ void k_act_gather(const fluere_record* src, const uint32_t* perm, uint64_t m, fluere_record* dst);

