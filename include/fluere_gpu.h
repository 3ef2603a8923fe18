/*
 * fluere_gpu.h -- C ABI of the MI355X-native `fluere offline` hot path.
 *
 * Plain pointers and sizes only; no torch or HIP types in the signatures
 * (streams are passed as void*, hipStream_t underneath).  A Rust host links
 * this through `extern "C"` (INTEGRATION.md shows the bindgen-free stub).
 *
 * Reference interfaces replaced (paths relative to SkuldNorniern/fluere):
 *   fluere_offline_file   <- pub async fn fluereflow_fileparse(arg: Args)
 *                            src/net/offline_fluereflows.rs:26 (mode seam,
 *                            called from execute_mode src/lib.rs:61)
 *   fluere_parse_batch    <- pub fn parse_keys(packet) src/net/parser/keys.rs:98
 *                            + pub fn parse_fluereflow(packet)
 *                            src/net/parser/fluereflows.rs:30 (library seam,
 *                            batched; re-exported at src/net/parser/mod.rs:15,17)
 *   fluere_run / fluere_get_records
 *                         <- the loop body of offline_fluereflows.rs:68-184:
 *                            update_flow (src/net/flows.rs:11) + the active /
 *                            expiry tables (:60-62) + the final flush (:182-184)
 *   fluere_record         <- FluereRecord fluereflow/src/types/fluereflow.rs:31-60
 *   fluere_write_csv      <- fluere_exporter src/utils/fluere_csv_exporter.rs:5
 *
 * Error convention: every call returns 0 on success, a negative FLUERE_E_*
 * code on failure (never panics or aborts).  Per-packet NetError results
 * (src/net/mod.rs:28-36) surface as fluere_pkt_meta.k_status / f_status.
 */
#ifndef FLUERE_GPU_H
#define FLUERE_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FLUERE_ABI_VERSION 1

enum fluere_status {
    FLUERE_OK = 0,
    FLUERE_E_ARG = -1,         /* bad argument */
    FLUERE_E_IO = -2,          /* file open/read/write failed (FluereError::IoError) */
    FLUERE_E_PCAP = -3,        /* not a pcap or pcapng capture (FluereError::PcapError) */
    FLUERE_E_HIP = -4,         /* HIP runtime error / no device */
    FLUERE_E_NOMEM = -5,       /* device or host allocation failed */
    FLUERE_E_TABLE_FULL = -6,  /* flow dictionary capacity exceeded: reopen with larger max_flows */
    FLUERE_E_UNSUPPORTED = -7, /* no exact result on this path (sharded sweep without a fixed point; never seen) */
    FLUERE_E_STATE = -8        /* call order violated */
};
/* Positive status (not an error): fluere_merge_gathered merged the summaries
 * of a capture whose span reaches the timeout; its records come from the
 * sweep composition (fluere_sweep_*). */
#define FLUERE_NEED_SWEEP 1
/* Positive status: fluere_merge_gathered_finish found the device-agreed step's
 * merge unusable (a block cut short, order-dependent flows, or the span
 * reaching the timeout); redo the step with the host-driven sequence. */
#define FLUERE_RETRY 2

/* NetError per packet (src/net/mod.rs:28-36). */
enum fluere_pkt_status {
    FLUERE_PKT_OK = 0,
    FLUERE_PKT_EMPTY = 1,         /* NetError::EmptyPacket */
    FLUERE_PKT_INVALID = 2,       /* NetError::InvalidPacket */
    FLUERE_PKT_UNKNOWN_ETHER = 3  /* NetError::UnknownEtherType */
};

/* The fluereflow record with a C layout.  IpAddr is {v6 flag, 16 bytes}
 * (IPv4 in the first 4).  cnt[] = fin, syn, rst, psh, ack, urg, ece, cwr, ns. */
typedef struct fluere_record {
    uint8_t src_v6, dst_v6, prot, tos;
    uint8_t min_ttl, max_ttl;
    uint16_t src_port, dst_port;
    uint8_t source[16];
    uint8_t destination[16];
    uint16_t pad0;
    uint32_t d_pkts, min_pkt, max_pkt, in_pkts, out_pkts;
    uint32_t cnt[9];
    uint64_t d_octets, first, last, in_bytes, out_bytes;
    /* emission order: ended records carry the global index of the packet that
     * closed them (FIN/RST or the sweep); active records carry UINT64_MAX. */
    uint64_t order_key;
} fluere_record; /* 152 bytes */

/* Per-packet view of parse_keys + parse_fluereflow (library seam). 128 B. */
typedef struct fluere_pkt_meta {
    uint8_t k_status, f_status, key_v6, key_proto;
    uint16_t key_sport, key_dport;
    uint8_t key_src[16], key_dst[16];
    uint8_t key_smac[6], key_dmac[6];
    uint8_t rec_v6, rec_prot, rec_tos, rec_ttl;
    uint8_t rec_src[16], rec_dst[16];
    uint16_t rec_sport, rec_dport;
    uint32_t rec_pkt;
    uint64_t doctets;
    uint64_t time;
    uint16_t flags; /* bit i = parse_flags()[i], fin..ns */
    uint8_t raw_used;
    uint8_t pad[13];
} fluere_pkt_meta;

typedef struct fluere_opts {
    int device;            /* HIP device ordinal */
    void* stream;          /* hipStream_t to run on (NULL: the library creates one) */
    uint64_t timeout_ms;   /* -t (Args.parameters.timeout), default 600000 */
    int use_mac;           /* -M (Args.parameters.use_mac) */
    uint64_t max_flows;    /* initial flow dictionary capacity (0: 1<<21).  Like the
                              reference's HashMap (offline_fluereflows.rs:61, no bound),
                              a capture whose sampled census shows more flows grows it
                              before its first pass, up to 2^26 (kept when HBM cannot
                              hold the larger tables); live sessions keep it fixed, and
                              so does FLUERE_NO_GROW=1 (then a run past it fails with
                              FLUERE_E_TABLE_FULL) */
} fluere_opts;

typedef struct fluere_stats {
    uint64_t packets;          /* pcap records handed to the device */
    uint64_t valid;            /* passed parse_keys and parse_fluereflow */
    uint64_t updates;          /* valid and not dropped by the TCP SYN gate */
    uint64_t dropped_parse;    /* parse_keys or parse_fluereflow returned Err */
    uint64_t unsupported;      /* always 0: every parser class runs on the GPU (kept for the ABI layout) */
    uint64_t flows;            /* distinct canonical flow keys */
    uint64_t complex_flows;    /* flows resolved by the exact per-flow state machine */
    uint64_t records;          /* emitted records */
    uint64_t ended;            /* records in the ended prefix */
    uint32_t sequential_mode;  /* 0: no expiry can fire; 1: expiry sweep, parallel; 2: expiry sweep, sequential
                                  kernel (forced: FLUERE_SEQ_MODE_B) */
    uint32_t passes;           /* passes of the exact chase (Mode B: until the processed set is stable) */
    double parse_ms;           /* device time of the fused parse+key+aggregate kernel */
    double total_ms;           /* wall time of the whole run (fluere_run: host clock, submission to results) */
} fluere_stats;

typedef struct fluere_ctx fluere_ctx;

int fluere_abi_version(void);
int fluere_open(const fluere_opts* opts, fluere_ctx** out);
int fluere_close(fluere_ctx* ctx);
/* Forget all packets and flows (keeps allocations). */
int fluere_reset(fluere_ctx* ctx);

/* ---- ingress ------------------------------------------------------------- */
/* Index a classic pcap held in host memory: record offsets (relative to the
 * buffer) follow libpcap offline semantics (stop at the first bad record).
 * offsets may be NULL to count.  Returns number of records or <0.  A pcapng
 * capture is counted (offsets must be NULL: its records are not contiguous
 * classic records). */
int64_t fluere_pcap_index(const uint8_t* file, uint64_t nbytes, uint64_t* offsets, uint64_t cap);

/* Attach a device-resident batch: `d_bytes` holds pcap records (the 24-byte
 * file header excluded or not: offsets decide), `d_offsets[i]` is the byte
 * offset of record i's 16-byte header inside d_bytes.  Batches must be
 * appended in capture order; the library does not copy them and they must
 * stay valid until fluere_reset/fluere_close.  nbytes < 4 GiB, and the
 * buffer must stay readable 80 bytes past nbytes (every record is read as
 * one unconditional 80-byte window: header + first 64 frame bytes).  snaplen: the file header's snaplen (0: 262144);
 * swapped: byte-swapped pcap; nsec_ts: nanosecond timestamps. */
int fluere_add_device_batch(fluere_ctx* ctx, const uint8_t* d_bytes, uint64_t nbytes,
                            const uint32_t* d_offsets, uint64_t n_packets, uint32_t snaplen, int swapped,
                            int nsec_ts);

/* Copy a host pcap file image to the device (owned by ctx) and attach it.
 * The bytes stream through pinned staging chunks (copies overlap the next
 * chunk) while the record index is built on the host in one pass.  A pcapng
 * image (libpcap reads both) is first rewritten as classic records with
 * microsecond timestamps. */
int fluere_add_host_pcap(fluere_ctx* ctx, const uint8_t* file, uint64_t nbytes);
/* The same, reading the capture file straight into the staging chunks
 * (Capture::from_file, offline_fluereflows.rs:44). */
int fluere_add_pcap_file(fluere_ctx* ctx, const char* path);

/* ---- compute ------------------------------------------------------------- */
/* Per-packet parse_keys/parse_fluereflow of every attached packet into a
 * device array of n fluere_pkt_meta (test / library seam). */
int fluere_parse_batch(fluere_ctx* ctx, fluere_pkt_meta* d_out, uint64_t cap);

/* Run the hot path over every attached batch: parse + flow key + aggregate
 * + state machine.  Asynchronous on the ctx stream except where the exact
 * state machine needs host decisions. */
int fluere_run(fluere_ctx* ctx, fluere_stats* stats);

/* Only the parse+key+aggregate pass over the attached batches (k_parse_agg,
 * then k_merge_partials, which also runs the general parser over the packets
 * the hot kernel left to it); leaves the flow table populated. Asynchronous. */
int fluere_parse_aggregate(fluere_ctx* ctx);
/* Device time (HIP events on the ctx stream) of the last hot-kernel launch
 * (k_parse_agg or k_parse_spill, the roofline kernel) of the last fluere_run /
 * fluere_parse_aggregate, ms. */
double fluere_last_kernel_ms(fluere_ctx* ctx);
/* After fluere_run: its host wall time (submission to results), ms.  After
 * fluere_parse_aggregate: device time of the hot kernel + merge, ms. */
double fluere_last_pass_ms(fluere_ctx* ctx);
/* The hot kernel of the last pass: "k_parse_agg" (LDS flow table) or
 * "k_parse_spill" (many flows per window: per-owner LDS bins), chosen from
 * the flow count: the census of a newly attached capture (its first pass), or
 * the previous run's exact count (reruns).  Static string. */
const char* fluere_last_hot_kernel(fluere_ctx* ctx);
/* The census of the capture attached last (k_census, one sampled pass run
 * before the first pass after an attach): out[0..9] = packets sampled, hot-
 * parser keyed, slow class, TCP, distinct keys in the sample, keys seen once,
 * twice, min / max time (us), estimated flows of the capture.  Returns how
 * many censuses the context has run (0: none yet). */
int fluere_last_census(fluere_ctx* ctx, uint64_t* out, int n);

/* Records of the last fluere_run, host memory, ended prefix first (in the
 * reference's emission order), then active flows.  Caller frees with
 * fluere_records_free. */
int fluere_get_records(fluere_ctx* ctx, fluere_record** out, uint64_t* n, uint64_t* n_ended);
void fluere_records_free(fluere_record* recs);

/* ---- multi-GPU exchange (one process per GPU; RCCL moves the bytes) ----- */
/* Packet-range sharding: rank r attaches packets [b_r, e_r) of the capture
 * with fluere_set_index_base(ctx, b_r) first, so every index is global.
 * After fluere_parse_aggregate every rank exports its flows into one block
 * per owner rank (owner = hash of the canonical key); one all-to-all over
 * xGMI (RCCL) delivers to every owner the blocks of all ranks, in rank order;
 * each owner merges its flows and builds their records.  No reference
 * counterpart (the reference is single-threaded); the records equal the
 * reference's on the whole capture.
 *
 * A summary carries a flow's order-free aggregate in one shard.  A flow whose
 * record depends on packet order inside the shard (a FIN/RST before its last
 * packet there, or a first packet that cannot create it) also carries an
 * annex: the state machine of offline_fluereflows.rs:97-157 run over the
 * shard's packets of the flow from "no flow": the lead piece (packets before
 * the first create-eligible one, up to the first FIN/RST), the head instance
 * (created in the shard, closed by that first FIN/RST or still open), the
 * tail instance (open at the shard's end, after the first FIN/RST).  Records
 * of instances that open and close between the two are final: the shard
 * keeps them.  The owner composes summaries and annexes in shard order. */
typedef struct fluere_flow_summary {
    uint32_t key[14];           /* canonical key words (DESIGN.md "Flow key") */
    uint32_t pkts[2];           /* per canonical direction */
    uint64_t bytes[2];
    uint32_t min_pkt, max_pkt, min_ttl, max_ttl;
    uint32_t flag_cnt[8];       /* fin syn rst psh ack urg ece cwr */
    uint64_t first_all, first_create, finrst_min, last; /* global packet indices */
    uint64_t first_time, last_time; /* times of packets first_create / last */
    uint16_t first_sport, first_dport; /* FluereRecord fields of the creating packet */
    uint8_t first_dir, first_prot, first_tos, first_v6;
    uint8_t first_src[16], first_dst[16];
    uint32_t annex;             /* index of the flow's annex in the same block, or UINT32_MAX */
    uint32_t shard;             /* exporting rank */
    uint64_t pad[4];
} fluere_flow_summary;          /* 256 bytes */

/* A run of a flow's packets inside one shard: update_flow's order-free fields
 * over the run, and (head / tail) the FluereRecord seed of its first packet. */
typedef struct fluere_flow_piece {
    uint32_t pkts[2];           /* per canonical direction */
    uint64_t bytes[2];
    uint32_t min_pkt, max_pkt, min_ttl, max_ttl;
    uint32_t flag_cnt[8];
    uint64_t last, last_time;   /* the run's last packet: global index, time */
    uint64_t first, first_time; /* the run's first packet: global index, time */
    uint8_t src[16], dst[16];   /* seed: FluereRecord source / destination, */
    uint8_t v6, prot, tos, dir; /*       family, prot, tos, canonical direction */
    uint16_t src_port, dst_port;
} fluere_flow_piece;            /* 144 bytes */

typedef struct fluere_flow_annex {
    uint32_t key[14];
    uint32_t flags;             /* 1 a FIN/RST in the shard (f0), 2 lead, 4 head, 8 tail */
    uint32_t pad;
    uint64_t f0;                /* global index of the shard's first FIN/RST of the flow */
    fluere_flow_piece lead, head, tail;
    uint64_t mid_last;          /* 1 + index of the last packet of the instances that open and close
                                   inside the shard (their records stay there); 0: none */
} fluere_flow_annex;            /* 512 bytes */

/* Block header; the run counters are the exporting shard's (the same in each
 * of its blocks). */
typedef struct {
    uint64_t n_flows;           /* summaries for this owner (> cap: the block was cut short) */
    uint64_t n_annex;           /* annexes for this owner (> cap_annex: cut short) */
    uint64_t tmin, tmax, valid, dropped;
    uint32_t err, shard;
    uint64_t n_bare_complex;    /* order-dependent flows of this shard exported WITHOUT their annexes
                                   (fluere_export_async): the owner cannot compose them, the step is
                                   redone with annexes (fluere_merge_gathered_async's retry word) */
} fluere_shard_header;          /* 64 bytes */

/* Flow capacity of the context (max_flows clamped to the table size). */
uint64_t fluere_capacity(fluere_ctx* ctx);
/* Records attached to the context (every batch). */
uint64_t fluere_total_packets(fluere_ctx* ctx);
int fluere_set_index_base(fluere_ctx* ctx, uint64_t first_global_index);

/* Bytes of one block: header, cap summaries, cap_annex annexes. */
uint64_t fluere_shard_block_bytes(uint64_t cap, uint64_t cap_annex);
/* After fluere_parse_aggregate: export this shard (rank `shard`) into n_owners
 * consecutive blocks at d_blocks (block o for owner rank o).  Runs the exact
 * state machine over the shard's order-dependent flows first (their final
 * records stay in this context).  *need / *need_annex (host, may be NULL): the
 * largest per-owner counts, so a caller sees when cap / cap_annex were too
 * small (the block header holds them too).  Synchronises the context stream. */
int fluere_export_device(fluere_ctx* ctx, void* d_blocks, uint32_t n_owners, uint32_t shard, uint64_t cap,
                         uint64_t cap_annex, uint64_t* need, uint64_t* need_annex);
/* The common case of fluere_export_device without a host round trip (no
 * annexes): d_info (device memory, 6 x uint64) receives {largest per-owner
 * summary count, annex count, order-dependent flows, flow count, 2^62 - the
 * earliest valid time, the latest valid time} (the last two 0 without a valid
 * packet).  The caller reduces d_info over the ranks (MAX, on the context's
 * stream) and reads it once: if the capture's span (latest - earliest) reaches
 * the timeout, the merge is completed by the sweep composition below (no
 * annexes); else if any rank has order-dependent flows every rank calls
 * fluere_export_device instead; if a count exceeds cap / cap_annex every rank
 * exports again with larger blocks. */
int fluere_export_async(fluere_ctx* ctx, void* d_blocks, uint32_t n_owners, uint32_t shard, uint64_t cap,
                        uint64_t cap_annex, unsigned long long* d_info);
/* Owner side: merge n_shards blocks (block r from rank r, consecutive, as an
 * all-to-all leaves them) into this context's (cleared) flow table and build
 * the owner's records; the context keeps the final records its own export
 * produced, so fluere_get_records returns every record this rank holds.
 * FLUERE_E_ARG if a block was cut short.  FLUERE_NEED_SWEEP (> 0) if the
 * capture's span reaches the timeout: the flows are merged but have no record
 * yet; every rank completes the merge with the fluere_sweep_* sequence. */
int fluere_merge_gathered(fluere_ctx* ctx, const void* d_blocks, uint32_t n_shards, uint64_t cap,
                          uint64_t cap_annex, fluere_stats* stats);
/* The same merge for a step agreed on the device (no host round trip before
 * it): fluere_merge_gathered_async enqueues the merge and sets d_retry (device,
 * one uint64) to 1 when its result cannot stand -- a block cut short, a flow
 * whose record depends on packet order (annexes), the span reaching the
 * timeout; the ranks reduce it (MAX) on the stream and read it once (the
 * step's one host round trip).  fluere_merge_gathered_finish then returns
 * FLUERE_OK with the stats, or FLUERE_RETRY: every rank redoes the step with
 * fluere_parse_aggregate, fluere_export_async / fluere_export_device and
 * fluere_merge_gathered (dist.py).  Replaces the host decision on the gathered
 * export counts (the reference has no sharding: offline_fluereflows.rs:49-191
 * is one sequential pass). */
int fluere_merge_gathered_async(fluere_ctx* ctx, const void* d_blocks, uint32_t n_shards, uint64_t cap,
                                uint64_t cap_annex, unsigned long long* d_retry);
int fluere_merge_gathered_finish(fluere_ctx* ctx, fluere_stats* stats);
/* Blocking host waits on the context's stream so far (stream syncs, polls of
 * a counter copy that was not yet published): the host round trips a step
 * takes (tests). */
uint64_t fluere_host_waits(fluere_ctx* ctx);

/* The compact wire encoding of the blocks (what the all-to-all moves): each
 * summary as a variable-length record that leaves out absent and zero fields
 * (an IPv4 5-tuple key in 12 bytes; no seed for a flow without a creating
 * packet; only the non-zero flag counts), behind a u32 offset table; annexes
 * verbatim.  A flow of the C4 recipe takes ~90-110 bytes instead of 256.
 * fluere_wire_bound: the largest wire block of one owner.
 * fluere_wire_pack (exporting side, after the export, enqueued on the context
 * stream): the n_owners blocks at d_blocks -> their wire blocks, contiguous in
 * owner order, at d_wire (n_owners * fluere_wire_bound bytes); d_sizes (device,
 * n_owners x uint64) receives each wire block's bytes -- the all-to-all's split
 * sizes.  fluere_wire_unpack (owner side, before fluere_merge_gathered): the
 * n_shards (<= 64) received wire blocks, contiguous in shard order with
 * sizes[s] (host) bytes each, -> the wide blocks at d_blocks (n_shards *
 * fluere_shard_block_bytes), every summary at its exported position. */
uint64_t fluere_wire_bound(uint64_t cap, uint64_t cap_annex);
int fluere_wire_pack(fluere_ctx* ctx, const void* d_blocks, uint32_t n_owners, uint64_t cap, uint64_t cap_annex,
                     void* d_wire, unsigned long long* d_sizes);
int fluere_wire_unpack(fluere_ctx* ctx, const void* d_wire, uint32_t n_shards, const uint64_t* sizes, uint64_t cap,
                       uint64_t cap_annex, void* d_blocks);
/* The same in fixed slots, for the device-agreed step (no split sizes on the
 * host): block b of d_slots (n x slot_bytes, slot_bytes a multiple of 16) in
 * [b * slot_bytes, (b + 1) * slot_bytes) behind a 16-byte prefix holding its
 * bytes; a block that does not fit sends only the prefix (bytes = UINT64_MAX),
 * and its owner unpacks it as a block cut short (the merge's retry word asks
 * for the redo).  The caller sizes the slots from the last host-driven step's
 * wire sizes; the all-to-all moves equal slot_bytes blocks. */
int fluere_wire_pack_slots(fluere_ctx* ctx, const void* d_blocks, uint32_t n_owners, uint64_t cap, uint64_t cap_annex,
                           uint64_t slot_bytes, void* d_slots);
int fluere_wire_unpack_slots(fluere_ctx* ctx, const void* d_slots, uint32_t n_shards, uint64_t slot_bytes, uint64_t cap,
                             uint64_t cap_annex, void* d_blocks);

/* ---- the hard-timeout sweep across shards (offline_fluereflows.rs:103-119,
 * 161-175): an expiry entry pushed at a flow's creation fires at the first
 * processed packet of the WHOLE capture with t >= exp, so shards are coupled.
 * Every rank is both a holder (of its packet range) and an owner (of its
 * flows, as in the merge); after fluere_merge_gathered returned
 * FLUERE_NEED_SWEEP (the export made without annexes), every rank runs:
 *   1. fluere_sweep_pack (holder): counts[o] = this shard's valid packets of
 *      owner o's flows; with d_send, their 32-byte records, owner-major,
 *      capture order within an owner.  All-to-all (split sizes from counts).
 *   2. fluere_sweep_load (owner): the records received, shard-major (counts[s]
 *      from shard s).
 *   3. a fixed point over the processed packets, per pass:
 *      a. fluere_sweep_index (holder): apply the owners' processed flags
 *         (d_pr: 1 byte per packed packet in the pack order, as the reverse
 *         all-to-all of step e leaves them; NULL on the first pass); *max_time
 *         = 1 + the latest processed packet's time (0: none).  All-gather.
 *      b. fluere_sweep_queries (holder): sweep points of its create-eligible
 *         packets; those past its own processed packets become queries to the
 *         first later shard whose max_time reaches exp: qcounts[r]; with d_q,
 *         the queries (8 bytes each, grouped by shard).  All-to-all.
 *      c. fluere_sweep_answer (answering shard): n queries -> packet indices
 *         (8 bytes each, same order).  All-to-all back.
 *      d. fluere_sweep_points (holder): the answers -> d_f, 8 bytes per packed
 *         packet (the pack order).  All-to-all (as step 1, 8-byte elements).
 *      e. fluere_sweep_chase (owner): the exact chase with those sweep points;
 *         d_pr: 1 byte per loaded packet (processed); *changed.  MAX over the
 *         ranks; reverse all-to-all of d_pr; stop when no rank changed.
 *   4. fluere_sweep_seed_requests (owner): the creating packets of its flow
 *      instances (8-byte global indices, ascending), counts[r] per holder
 *      (rank_first[r] = first global index of rank r, n_ranks + 1 entries).
 *      All-to-all; fluere_sweep_seeds (holder): 40-byte FluereRecord seeds,
 *      same order; all-to-all back.
 *   5. fluere_sweep_finish (owner): the records (fluere_get_records).  Their
 *      order is global: order_key = the index of the packet that ended them,
 *      then fluere_get_record_order's two words {0 for a FIN/RST close, else
 *      exp + 1; the creation index of the firing entry}. */
int fluere_sweep_pack(fluere_ctx* ctx, uint32_t n_owners, uint64_t* counts, void* d_send);
int fluere_sweep_load(fluere_ctx* ctx, const void* d_recv, uint32_t n_shards, const uint64_t* counts);
int fluere_sweep_index(fluere_ctx* ctx, const uint8_t* d_pr, uint64_t* max_time);
int fluere_sweep_queries(fluere_ctx* ctx, uint32_t n_ranks, uint32_t rank, const uint64_t* max_times,
                         uint64_t* qcounts, void* d_q);
int fluere_sweep_answer(fluere_ctx* ctx, const void* d_q, uint64_t n, void* d_ans);
int fluere_sweep_points(fluere_ctx* ctx, const void* d_ans, void* d_f);
int fluere_sweep_chase(fluere_ctx* ctx, const void* d_f, void* d_pr, int* changed);
int fluere_sweep_seed_requests(fluere_ctx* ctx, uint32_t n_ranks, const uint64_t* rank_first, uint64_t* counts,
                               void* d_req);
int fluere_sweep_seeds(fluere_ctx* ctx, const void* d_req, uint64_t n, void* d_seeds);
int fluere_sweep_finish(fluere_ctx* ctx, const void* d_seeds, fluere_stats* stats);
/* Two order words per record, in fluere_get_records' order (n = its count):
 * non-zero only after fluere_sweep_finish. */
int fluere_get_record_order(fluere_ctx* ctx, uint64_t* aux, uint64_t n);

/* ---- live mode (src/net/live_fluereflow.rs:196-376) on batched capture --- */
/* A live session: packets arrive in batches (a classic pcap image each: the
 * records a capture ring delivered since the last call); flows stay open
 * across batches.  Per packet the reference runs parse_keys /
 * parse_fluereflow, the SYN gate (:226-269), update_flow (:288) and the
 * FIN/RST close with the plugin hand-off (:290-303); there is no expiry wheel.
 * The checks it runs after each processed packet run here once per batch,
 * after the batch's last processed packet, with that packet's time:
 *   fluere_live_batch(do_export = 1): the interval export (:306-358): flows
 *     with flow.last < time - timeout expire (when timeout > 0), and the
 *     FIN/RST-closed records since the last export plus the expired ones are
 *     returned (*exported = 1) -- one CSV file / one plugin hand-off batch;
 *   fluere_live_finish: the duration scan (duration_end, :361-373: the same
 *     test without the timeout > 0 guard), then every flow still active, as
 *     the last export (:379-392).
 * Returned records: the first *n_ordered in the reference's order (the
 * packet that closed them; order_key = its global index), the rest in the
 * reference's HashMap order (unspecified; order_key = UINT64_MAX).  Free with
 * fluere_records_free.  opts->max_flows bounds the session's distinct flows. */
typedef struct fluere_live fluere_live;
int fluere_live_open(const fluere_opts* opts, fluere_live** out);
int fluere_live_close(fluere_live* lv);
int fluere_live_batch(fluere_live* lv, const uint8_t* pcap, uint64_t nbytes, int do_export, fluere_record** recs,
                      uint64_t* n, uint64_t* n_ordered, int* exported);
int fluere_live_finish(fluere_live* lv, int duration_end, fluere_record** recs, uint64_t* n, uint64_t* n_ordered);
/* fluere_live_batch for a batch whose record offsets the capture side already
 * holds (a capture ring hands over packets one by one, headers included):
 * rec_off[i] = byte offset of record i's 16-byte header in pcap.  The host
 * then skips libpcap's walk over the headers, a pointer chase that costs one
 * memory latency per record (~0.1 us for IMIX-sized records, the live-mode
 * ingest bound); the records are checked against the offsets with independent
 * loads instead.  Same result as fluere_live_batch: the batch ends at the
 * first record that does not start where the previous one ended, or whose
 * caplen the walk would refuse. */
int fluere_live_batch_indexed(fluere_live* lv, const uint8_t* pcap, uint64_t nbytes, const uint64_t* rec_off,
                              uint64_t n_recs, int do_export, fluere_record** recs, uint64_t* n, uint64_t* n_ordered,
                              int* exported);

/* Test seam: insert n canonical keys (14 u32 words each, device memory) into
 * the flow dictionary and write each key's dense flow id. */
int fluere_debug_dense_ids(fluere_ctx* ctx, const uint32_t* d_keys, uint64_t n, uint32_t* d_out);

/* Test seam (parser probe): run the device restatement of one entry point of
 * the raw fallback (src/net/parser/raw, reached from parse_ports ports.rs:47,
 * the parse_keys eager chain keys.rs:279-296 and parse_fluereflow
 * fluereflows.rs:148-195) over n byte strings, so the reference's own unit
 * tests of those functions pin the GPU code directly:
 *   FLUERE_RAW_FROM_RAW_PACKET  RawProtocolHeader::from_raw_packet(p, arg as u8)  raw/mod.rs:152
 *   FLUERE_RAW_FROM_ETHERTYPE   RawProtocolHeader::from_ethertype(p, arg as u16)  raw/mod.rs:330
 *   FLUERE_RAW_PARSE_ETHERTYPE  ethertypes::parse_ethertype(p, arg)               raw/ethertypes/mod.rs:20
 *   FLUERE_RAW_PARSE_PROTOCOL   protocols::parse_protocol(p, arg)                 raw/protocols/mod.rs:48
 *   FLUERE_RAW_OPENVPN          OpenVpnParser::parse_packet                       raw/protocols/openvpn.rs:155
 *   FLUERE_RAW_ICMP             IcmpParser::parse_packet                          raw/protocols/icmp.rs:10
 * String i is d_bytes[d_off[i], d_off[i] + d_len[i]) (device memory); the
 * result (Some / None and the RawProtocolHeader fields) goes to d_out[i]. */
enum {
    FLUERE_RAW_FROM_RAW_PACKET = 0,
    FLUERE_RAW_FROM_ETHERTYPE = 1,
    FLUERE_RAW_PARSE_ETHERTYPE = 2,
    FLUERE_RAW_PARSE_PROTOCOL = 3,
    FLUERE_RAW_OPENVPN = 4,
    FLUERE_RAW_ICMP = 5
};
typedef struct fluere_raw_hdr {
    uint8_t some;                      /* Option<RawProtocolHeader>::is_some() */
    uint8_t has_src, has_dst, ip_v6;   /* src_ip / dst_ip: Some, and IpAddr::V6 */
    uint8_t src[16], dst[16];          /* IPv4 in the first 4 bytes */
    uint16_t src_port, dst_port;
    uint8_t protocol, has_flags, flags, has_version;
    uint8_t version, has_ethertype, has_payload, pad0;
    uint16_t length, ethertype;
    uint32_t payload_off, payload_len; /* payload = the string's bytes [off, off + len) */
    uint32_t pad1;
} fluere_raw_hdr;                      /* 64 bytes */
int fluere_debug_raw(int fn, const uint8_t* d_bytes, const uint32_t* d_off, const uint32_t* d_len,
                     const uint32_t* d_arg, uint64_t n, fluere_raw_hdr* d_out, void* stream);

/* ---- egress -------------------------------------------------------------- */
/* Write the CSV exactly as fluere_exporter does (header + one row per record). */
int fluere_write_csv(const fluere_record* recs, uint64_t n, const char* path);
/* Format into a caller buffer; returns bytes needed (buf may be NULL). */
uint64_t fluere_format_csv(const fluere_record* recs, uint64_t n, char* buf, uint64_t cap);

/* The whole `fluere offline` mode: read pcap, run, write
 * <out_dir>/<file_stem>_converted.csv (offline_fluereflows.rs:44-58,186-190). */
int fluere_offline_file(const char* pcap_path, uint64_t timeout_ms, int use_mac, const char* out_dir,
                        fluere_stats* stats);

/* ---- synthetic captures (bench / tests) ---------------------------------- */
typedef struct fluere_synth_cfg {
    uint64_t seed;
    uint64_t n_packets;
    uint32_t n_flows;
    uint32_t kind;       /* FLUERE_SYNTH_* */
    uint32_t rev_pct;    /* % of packets sent in the reverse direction */
    uint32_t pad;
} fluere_synth_cfg;

enum {
    FLUERE_SYNTH_UDP64 = 0,     /* 64-B Ethernet/IPv4/UDP */
    FLUERE_SYNTH_IMIX = 1,      /* 64/576/1500 (7:4:1), TCP+UDP, SYN first, FIN/RST last */
    FLUERE_SYNTH_VLAN64 = 2,    /* 802.1Q-tagged 64-B IPv4/UDP, MAC pairs */
    FLUERE_SYNTH_MAC64 = 3,     /* untagged 64-B IPv4/UDP, MAC pairs */
    FLUERE_SYNTH_TCP = 4,       /* IMIX sizes; TCP with handshakes, 4-way closes (the peer's packets after the
                                   first FIN), RSTs, reopened keys, mid-stream starts, elephants; and UDP */
    FLUERE_SYNTH_SLOW = 5       /* the general parser's classes: IMIX schedule at 128/576/1500 B, per flow
                                   IPv6 (1/2), VXLAN-encapsulated IPv4 (1/4) or IPv4 with options (1/4) */,
    FLUERE_SYNTH_TCP_BACKTIME = 6 /* FLUERE_SYNTH_TCP with 1 % of the timestamps up to 5 ms early (out of order) */
};

/* Size of the synthetic pcap file (24-B header + records). */
uint64_t fluere_synth_file_size(const fluere_synth_cfg* cfg);
/* Write the whole synthetic pcap file into host memory. */
int fluere_synth_host(const fluere_synth_cfg* cfg, uint8_t* file, uint64_t cap);
/* Generate packets [first, first+n) directly in device memory as a batch
 * (bytes + offsets), identical to the host image.  d_bytes needs
 * fluere_synth_range_bytes(); d_offsets n entries. */
uint64_t fluere_synth_range_bytes(const fluere_synth_cfg* cfg, uint64_t first, uint64_t n);
int fluere_synth_device(const fluere_synth_cfg* cfg, uint64_t first, uint64_t n, uint8_t* d_bytes,
                        uint32_t* d_offsets, void* stream);

#ifdef __cplusplus
}
#endif
#endif
