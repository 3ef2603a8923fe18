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
int exact_run(const ExactJob& job, hipStream_t s, ExactResult* res);

}  // namespace fl
