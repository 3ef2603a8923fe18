// exact.h -- the exact offline state machine on the GPU (exact.hip).
//
// Reference: fluereflow_fileparse's packet loop, src/net/offline_fluereflows.rs:
// 68-184: flow creation only by a non-TCP packet or a SYN (:101-113), update
// (flows.rs:11-42), close by FIN/RST (:152-157), and the hard-timeout sweep of
// the expiry wheel, whose entries are pushed once per creation and never
// removed, so a stale entry evicts a later flow of the same oriented key
// (:103-107, :161-175).
//
// Used for the flows whose record depends on packet order (Mode A: the
// certificate in fluere_gpu.hip rejected them) and, when the capture's span
// reaches the timeout, for every flow (Mode B).  See exact.hip for the method.
#pragma once
#include "device.h"

namespace fl {

// One replayed packet (32 bytes).
struct ExMeta {
    uint64_t t, gidx;
    uint32_t d, pkt, doct;
    uint8_t dir, tflags, ttl, bits;  // bits: 1 create-eligible, 2 FIN or RST
};
static_assert(sizeof(ExMeta) == 32, "ExMeta layout");

// FluereRecord seed of a creating packet (fill_seed's fields that the
// aggregate does not give): shipped from the shard that holds the packet to
// the key's owner in sharded Mode B.  40 bytes.
struct Seed {
    uint8_t src[16], dst[16];
    uint16_t sp, dp;
    uint8_t v6, prot, tos, pad;
};
static_assert(sizeof(Seed) == 40, "Seed layout");

// Max segment tree over the processed packets' times (exact.hip): P leaves
// (a power of two >= n), tree[P + k] = t_k + 1 for a processed packet k, else
// 0.  tree_first(tree, P, k0, x): the first leaf k >= k0 whose value is >= x,
// or ~0 -- the sweep point of an entry (k0 = its creation, x = exp + 1) in any
// timestamp order.
uint64_t tree_leaves(uint64_t n);
int tree_build(uint64_t n, const ExMeta* cm, const uint8_t* pr, unsigned long long* tree, uint64_t P, hipStream_t s);
__device__ __forceinline__ uint64_t tree_first(const unsigned long long* tree, uint64_t P, uint64_t k0,
                                               unsigned long long x) {
    if (k0 >= P) return ~0ull;
    uint64_t i = P + k0;
    if (tree[i] >= x) return k0;
    for (;;) {
        while (i & 1) i >>= 1;  // climb while a right child (the root ends it: i == 1 -> 0)
        if (i == 0) return ~0ull;
        i += 1;                 // the right sibling's subtree holds the next leaves
        if (tree[i] >= x) {
            while (i < P) i = tree[2 * i] >= x ? 2 * i : 2 * i + 1;
            return i - P;
        }
    }
}

// A pinned host mailbox for the few device scalars a run needs on the host
// (counts that size the next launches): one wave copies them in and then
// writes seq; the host spins on seq.  A hipMemcpyAsync + hipStreamSynchronize
// round trip costs a copy kernel and the blocking wake-up (measured 20-45 us
// of idle GPU per round trip on MI355X in the exact engine's timeline).
struct alignas(64) HostMail {
    uint32_t seq;       // written by the device last
    uint32_t host_seq;  // the host's last request (never written by the device)
    unsigned long long v[14];
};
constexpr int MAIL_MAX = 14;
// out[i] = the `bytes[i]`-byte (1, 4 or 8) value at device address src[i],
// stream-ordered after the work enqueued on s; m null: copies + a stream sync.
int mail_fetch(HostMail* m, hipStream_t s, int n, const void* const* src, const int* bytes, unsigned long long* out);

struct ExactJob {
    const Batch* d_batches;  // device copy of the batches
    const Batch* h_batches;  // host copy (per-batch launches)
    int nb;
    TableSet T;              // the flow dictionary of the run (every valid key present)
    int macs;
    int mode_b;              // expiries can fire: replay every valid packet with the sweep
    uint64_t timeout_us;
    const uint8_t* complex;  // Mode A: replay the flows d with complex[d] != 0
    Glob* g;                 // run counters: n_rec / n_updates / n_ended are added to
    fluere_record** d_recs;  // record buffer (grown when needed; records already in it are kept)
    uint64_t* d_recs_cap;
    void** scratch;          // device scratch arena, reused across runs
    size_t* scratch_bytes;
    // Shard mode (multi-GPU export): replay the complex[] flows from "no
    // flow" over this shard's packets; instances that open and close inside
    // the shard become records, the lead / head / tail pieces go to one annex
    // per flow (fluere_flow_annex), annex_of[d] = its index.
    int shard_mode;
    fluere_flow_annex** annex;  // grown to the number of replayed flows
    uint64_t* annex_cap;
    uint32_t* annex_of;         // [fmax], NONE32 for flows without an annex (the caller fills it)
    // Sharded Mode B owner (fluere_sweep_*): the replayed packets are the
    // shards' (ext_n of them, capture order, d = this context's dense ids)
    // instead of a parse of the batches.
    const ExMeta* ext_cm = nullptr;
    uint64_t ext_n = 0;
    // One GPU, Mode B: every packet's replay metadata written by the hot pass
    // in capture order (AggArgs::exm; every packet valid, none for the general
    // parser): no k_ex_meta pass; the flows come from the merge's words
    // (phash + emap, which must be set)
    const ExMeta* dense_cm = nullptr;
    // or null: with dense_cm, the packets' times alone (AggArgs::exm_t)
    const unsigned long long* dense_t = nullptr;
    // Mode A: the complex-flow filter (device.h ckey_bucket), or null
    const uint8_t* cbits = nullptr;
    // pinned mailbox for the host's scalar reads (null: copies + stream syncs)
    HostMail* mail = nullptr;
    // Mode B without a caller-provided aux_out (one GPU): the records' order
    // words, grown to the record count (records already there keep zeros)
    unsigned long long** recaux = nullptr;
    uint64_t* recaux_cap = nullptr;
    // Mode A: the records already emitted (the caller's fresh counters), or ~0
    // (exact_finish reads them): lets exact_finish skip its host read
    uint64_t n_rec_known = ~0ull;
    // Mode A: the hot pass's per-packet filter words (AggArgs::phash), packet
    // B.first - phash_base of each batch first, or null
    const uint32_t* phash = nullptr;
    uint64_t phash_base = 0;
    // or null: the words also carry the merge's flows (PH_ID / PH_EREF,
    // device.h), emap its entries' dense ids (Mode A and Mode B)
    const uint32_t* emap = nullptr;
    // or null: the hot pass's per-packet replay metadata, indexed like phash
    // (AggArgs::exm; d == 0 marks a packet the hot parser took): k_ex_meta
    // copies it for a packet with a merge word instead of parsing it again
    const ExMeta* hot_meta = nullptr;
    // the run's flow count when the host knows it (every dense id below it),
    // else 0 (T.fmax bounds them): the sort by flow takes only its bits
    uint64_t key_bound = 0;
};

struct ExactResult {
    uint64_t replayed;    // packets replayed
    uint64_t keys;        // flows replayed
    uint64_t instances;   // flow records (instances) produced
    int iterations;       // Mode B: passes until the processed-packet set was stable
    uint64_t annexes;     // shard mode: annexes written (= keys)
};

// 0 on success; EXACT_FALLBACK when Mode B cannot be done in parallel here
// (timestamps not non-decreasing over the valid packets, or no fixed point
// within the pass limit): the caller runs the sequential kernel; else FLUERE_E_*.
constexpr int EXACT_FALLBACK = 1;
// exact_begin: a packet of the dense metadata has no flow word (exact_run
// then begins again with k_ex_meta)
constexpr int EXACT_DENSE_MISS = 2;
int exact_run(const ExactJob& job, hipStream_t s, ExactResult* res);
// Grow the job's scratch arena (J.scratch) to what exact_begin lays out for
// it, ahead of the run (host-side allocation while the GPU works).
int exact_reserve(const ExactJob& job, hipStream_t s);

// exact_run in phases, for the sharded Mode B owner, whose sweep points and
// seeds come from the shards between the phases:
//   exact_begin   replayed packets -> sorted per key, heads, next-eligible /
//                 next-FIN scans (the job is copied; its pointers must live on)
//   exact_pass    one chase + members pass; fext (device, capture order): the
//                 sweep point of every packet, or null to compute them here;
//                 pr_out (device, may be null): processed flag per packet;
//                 *changed: the processed set changed (Mode B)
//   exact_seed_requests  the creating packets' indices of the instances,
//                 ascending (req) with their instance ordinals (q)
//   exact_finish  records; seeds (device, by instance ordinal) or null to
//                 parse the creating packets; aux_out (device, 2 per record)
//                 or null: Mode B records keep order_key = the ending packet's
//                 index and aux = {0 FIN/RST | exp + 1 sweep, firing creation}
struct ExactSession;
int exact_begin(const ExactJob& job, hipStream_t s, ExactSession** out);
uint64_t exact_replayed(const ExactSession* S);
int exact_pass(ExactSession* S, const unsigned long long* fext, uint8_t* pr_out, bool* changed);
int exact_seed_requests(ExactSession* S, unsigned long long* req, uint32_t* q, uint32_t* n_inst);
int exact_finish(ExactSession* S, const Seed* seeds, unsigned long long* aux_out);
const ExactResult& exact_result(const ExactSession* S);
// Every valid packet of the job's batches (its flows in J.T) as ExMeta, in
// capture order, into cm (room for every packet); *n = how many.
int exact_collect(const ExactJob& job, hipStream_t s, ExMeta* cm, uint64_t* n);
void exact_free(ExactSession* S);

// out[p] = the sum of flags[0..p) (or [0..p] inclusive), 32-bit words; with a
// list, list[out_exclusive[p]] = p where flags[p] != 0 (0/1 flags).  tmp: one
// word per 4096 items.  Stream-ordered (a reduce and a scan kernel).
int flag_count(hipStream_t s, uint64_t n, const uint32_t* flags, uint32_t* out, bool inclusive, uint32_t* list,
               void* tmp);

}  // namespace fl
