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
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <hipcub/hipcub.hpp>

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/fluere_gpu.h"
#include "device.h"
#include "exact.h"
#include "pcapng.h"
#include "synth.h"

// FLUERE_ALLOC_LOG (diagnostics): every device allocation of the library, with
// its source line and time -- the allocations a run makes while the GPU waits
static hipError_t fl_dmalloc(void** p, size_t bytes, int line) {
    static const bool log = getenv("FLUERE_ALLOC_LOG") != nullptr;
    if (!log) return (hipMalloc)(p, bytes);
    const auto t0 = std::chrono::steady_clock::now();
    const hipError_t e = (hipMalloc)(p, bytes);
    fprintf(stderr, "[fluere] hipMalloc line %d: %zu bytes, %.1f us\n", line, bytes,
            std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    return e;
}
#define hipMalloc(p, bytes) fl_dmalloc(reinterpret_cast<void**>(p), (bytes), __LINE__)

using namespace fl;

static_assert(sizeof(fluere_record) == 152, "fluere_record ABI");
static_assert(sizeof(fluere_pkt_meta) == 128, "fluere_pkt_meta ABI");
static_assert(sizeof(fluere_flow_summary) == 256, "fluere_flow_summary ABI");
static_assert(sizeof(fluere_flow_piece) == 144, "fluere_flow_piece ABI");
static_assert(sizeof(fluere_flow_annex) == 512, "fluere_flow_annex ABI");
static_assert(sizeof(fluere_shard_header) == 64, "fluere_shard_header ABI");
static_assert(sizeof(fluere_raw_hdr) == 64, "fluere_raw_hdr ABI");

namespace {

// ---------------------------------------------------------------------------
// k_parse_agg: the hot kernel
// ---------------------------------------------------------------------------
// Per-window partial aggregates of the hot kernel's LDS flow tables, one "set"
// per (workgroup, window), SoA over [set * NS + cell].  Within a set the
// cells are grouped by merge owner (owner = hash(key) % O), so the owner of a
// flow reads only its own segment of every set.  Written with plain stores;
// merged per flow by k_merge_partials.
// One staged partial: 80 bytes, written and read as five 16-byte accesses.
struct alignas(16) Part {
    uint32_t k0, k1, k2, tag;     // key words; tag = proto << 24 (0xFF << 24: k0 is a dense id)
    uint32_t h, pk, by0, by1;     // key hash; packets per direction (16-bit halves); bytes per direction
    uint32_t mn0, mn1, mx0, mx1;  // min / max pkt, min / max ttl
    uint32_t fl[4];               // flag pairs, 16-bit halves
    uint32_t pos[4];              // first any / first create / first FIN-RST (NONE32) and last+1 (0), window-relative
};
static_assert(sizeof(Part) == 80, "Part layout");

// A spilled packet: a valid hot-path packet whose key found no LDS slot (more
// flows in a workgroup's window than the table holds).  32 bytes; written
// raw per workgroup during the window, grouped by merge owner at the flush,
// merged by its owner like a one-packet partial.
struct alignas(16) Spill {
    uint32_t k0, k1, k2, tag;     // LDS key words (tag = proto << 24)
    uint32_t doct, pt, loc, fl;   // pt = pkt | ttl << 16 | elig << 24; fl = tf | dir << 8 (| set << 9: overflow list)
};
static_assert(sizeof(Spill) == 32, "Spill layout");
// MAC kernels: a spilled packet takes two records: {k0, k1, k2, tag},
// {m0, m1, m2, key hash}, {doct, pt, loc, fl}, padding.
__host__ __device__ constexpr int spill_units(bool macs) { return macs ? 2 : 1; }

struct Stage {
    Part* part;                   // [set * NS + cell]
    uint32_t* off;                // [(O + 1) * n_sets]: off[o * n_sets + set] = first cell of owner o's flows
    unsigned long long* base;     // [set] global index of the window's first packet
    // Spilled packets are stored as planes of 16-byte words (word w of every
    // record together), so a wave's loads and stores of one word are contiguous.
    // A spilled packet is stored where its merge owner reads it: segment o of
    // its set holds up to cap_o records (32 B, 64 B with MACs: whole sectors),
    // soff[o][set] of them.  The rare packets past cap_o (a key spilling a
    // whole window) are appended raw per workgroup (planes of 16-byte words)
    // and listed at the flush in spill (the overflow list, n_spill records).
    Spill* dspill;                // [set][owner][cap_o] records
    uint32_t cap_o;
    Spill* spill_raw;             // [workgroup][word][WIN_ITERS * BLOCK] this window's overflow, arrival order
    Spill* spill;                 // [spill_cap] the overflow list (one record each; fl bits 9.. = set)
    unsigned long long spill_cap; // records of spill (the batch's packet count)
    uint32_t* soff;               // [O * n_sets]: records in owner o's segment of set s
    uint4* partx;                 // MAC runs: [set * NS + cell] the partial's MAC words and key hash
    unsigned long long* wgs;      // [workgroup][WGS_N] run statistics of each hot-kernel workgroup (plain
                                  // stores; k_merge_partials sums them: no contended atomics at the end)
    uint32_t W;                   // sets per workgroup
    uint32_t O;                   // merge owners (k_merge_partials workgroups)
    uint32_t no_parts;            // the hot pass staged no partials (k_parse_spill, or k_slow alone): the merge
                                  // reads the owner segments only
    uint32_t n_sets;              // sets: the hot kernel's n_hot, then k_slow's (when it runs)
    uint32_t n_wg;                // hot-kernel workgroups
    uint32_t n_hot;               // the hot kernel's sets (n_wg * W)
    uint32_t cap_s;               // k_slow sets: records per owner segment
    unsigned long long slow_rec0; // k_slow sets: their segments start at this record of dspill
};
// per-workgroup statistics: valid, dropped, LDS-table misses, tmin, tmax, cycles total / flush / wave wait
constexpr int WGS_N = 8;

// IPv6 address ids (k_slow): each distinct address of a pass gets an id from
// a write-once chain of three 64-bit levels (the protocol of flow_table.h's
// dictionary): A[addr words 0,1] -> sa, B[sa << 32 | word 2] -> sb,
// C[sb << 32 | word 3] -> id; the level-C inserter writes addr_of[id].  An
// IPv6 5-tuple then travels like an IPv4 one, as three words (id of the lower
// address, id of the higher, ports) with bit 0 of its tag set, through the
// merge owners' segments and LDS tables; the owner rebuilds the full key once
// per flow (a later launch reads addr_of).  Cleared before every pass that
// uses it; a full chain falls back to the dictionary walk per packet.
struct V6Map {
    unsigned long long* tab[3];  // (C + 1) keys each (slot C: the word EMPTY)
    uint4* addr_of;              // [C + 1]
    uint32_t C;                  // power of two; 0: no map
};
constexpr uint32_t V6_TAG = 1u;  // tag bit 0: the key words are (address id, address id, ports)

__device__ __forceinline__ uint32_t v6_level(unsigned long long* keys, uint32_t C, uint64_t w, bool& fresh) {
    fresh = false;
    if (w == EMPTY) return C;
    uint32_t h = (uint32_t)mix64(w) & (C - 1);
    for (int p = 0; p < 64; p++) {
        const unsigned long long k = keys[h];  // (a stale load shows EMPTY for a filled slot, never another key)
        if (k == w) return h;
        if (k == EMPTY) {
            const unsigned long long old = atomicCAS(&keys[h], EMPTY, (unsigned long long)w);
            if (old == EMPTY) { fresh = true; return h; }
            if (old == w) return h;
        }
        h = (h + 1) & (C - 1);
    }
    return FAIL;
}
// ids of two addresses, their levels interleaved (two lookups per round trip)
__device__ __forceinline__ void v6_ids(const V6Map& M, const uint32_t* a, const uint32_t* b, uint32_t& ia, uint32_t& ib) {
    bool fa, fb;
    uint32_t sa = v6_level(M.tab[0], M.C, ((uint64_t)a[0] << 32) | a[1], fa);
    uint32_t sb = v6_level(M.tab[0], M.C, ((uint64_t)b[0] << 32) | b[1], fb);
    if (sa != FAIL) sa = v6_level(M.tab[1], M.C, ((uint64_t)sa << 32) | a[2], fa);
    if (sb != FAIL) sb = v6_level(M.tab[1], M.C, ((uint64_t)sb << 32) | b[2], fb);
    if (sa != FAIL) sa = v6_level(M.tab[2], M.C, ((uint64_t)sa << 32) | a[3], fa);
    if (sb != FAIL) sb = v6_level(M.tab[2], M.C, ((uint64_t)sb << 32) | b[3], fb);
    if (sa != FAIL && fa) M.addr_of[sa] = make_uint4(a[0], a[1], a[2], a[3]);
    if (sb != FAIL && fb) M.addr_of[sb] = make_uint4(b[0], b[1], b[2], b[3]);
    ia = sa;
    ib = sb;
}

struct AggArgs {
    Batch B;
    TableSet T;
    Acc A;
    Stage S;
    Glob* g;
    uint32_t* slow;            // packets (batch-local indices) the hot parser left to the general parser:
                               // workgroup b's in slow[b * slow_region, + slow_cnt[b])
    unsigned long long* slow_n;  // their total (the merge's "any slow packet" test)
    V6Map v6;                  // k_slow's IPv6 address ids (C = 0: none)
    uint32_t* gen;             // k_slow: the slow packets parse_fast / parse_mid leave to the general parser
                               // (batch-local indices, Glob::n_gen of them; the merge tail takes them)
    uint32_t* slow_cnt;
    uint32_t slow_region;      // packets a hot workgroup can see (its steps x BLOCK)
    int slow_abl;              // diagnostics only (FLUERE_SLOW_ABL, wrong results): 1 no dictionary, 2 no parse,
                               // 3 no spill records (k_slow)
    int slow_kernel;           // the slow list is k_slow's (launched before the merge), not the merge tail's
    int macs;
    unsigned long long* dbg;   // diagnostics (FLUERE_DEBUG): per workgroup {start, flush start, flush end, end} wall clock
    uint32_t* phash;           // or null: per packet of the batch, its ckey_bucket or PH_PARSE (device.h), for
                               // the exact engine's filter (k_ex_meta reads it instead of parsing every packet)
    // or null: the merge writes each resolved packet's flow (PH_ID / PH_EREF,
    // device.h) over its word in pid[global index - pid_base], and its
    // entries' dense ids to emap (k_ex_meta then walks no dictionary)
    uint32_t* pid;
    uint32_t* emap;
    uint64_t pid_base;
    uint32_t pid_batch;
    int slow_all;              // k_slow takes every packet of the batch (no hot kernel: captures of the general
                               // parser's classes, where the hot pass would only list them)
};

// Front end of the hot kernel: Ethernet / IPv4 (ihl 5) / TCP or UDP parsed
// from the record window in registers, with selects instead of branches.
// Everything else (other ethertypes and IP protocols, IPv4 options, VXLAN,
// short or truncated frames) is left to the general parser (slow_packets, in k_merge_partials),
// which computes the same result for these packets too; this is only the
// common case of parse_keys + parse_fluereflow (keys.rs:98-343,
// fluereflows.rs:30-199, ports.rs:7-58, flags.rs:13-38) written out for it.
// Record bytes (16-B pcap header + frame) used, as window words w[k] = bytes
// [4k, 4k+4) little-endian: 0-11 header, 28-29 ethertype, 30 version/ihl,
// 32-33 total length, 38 ttl, 39 protocol, 42-49 addresses, 50-53 ports,
// 58-65 the VXLAN probe (keys.rs:188), 63 TCP flags.
struct Hot {
    uint64_t t;                   // parse_microseconds (time.rs:5-7)
    uint32_t sip, dip, ports;     // big-endian addresses; src_port << 16 | dst_port
    uint32_t proto, doct, pkt, ttl, tf;
};
enum : uint32_t { HOT_OK = 0, HOT_DROP = 1, HOT_SLOW = 2 };

__device__ __forceinline__ uint32_t hot_parse(const Batch& B, uint32_t off, const Win& W, Hot& h) {
    const bool sw = B.flags & 1;
    const uint32_t sec = sw ? bswap32(W.w[0]) : W.w[0];
    uint32_t frac = sw ? bswap32(W.w[1]) : W.w[1];
    const uint32_t incl = sw ? bswap32(W.w[2]) : W.w[2];
    if (B.flags & 2) frac /= 1000u;  // nanosecond capture (wave-uniform)
    h.t = (uint64_t)sec * 1000000ull + frac;
    const uint32_t L = min(incl, B.snap);
    const uint32_t w7 = W.w[7], w8 = W.w[8], w9 = W.w[9];
    const uint32_t tl = __builtin_amdgcn_perm(0u, w8, 0x0C0C0001u);
    const uint32_t proto = w9 >> 24;
    // Ipv4Packet::payload() length: min(total_length - 20, caplen - 34)
    const uint32_t pe = min(tl > 20u ? tl - 20u : 0u, L > 34u ? L - 34u : 0u);
    // (bitwise, not short-circuit: no branches).  The VXLAN probe reads the
    // 8 bytes after the UDP header view (record bytes 58..65, keys.rs:188);
    // only bytes 58..63 are tested here, so the hot parser needs record bytes
    // 0..63 alone (a 64-byte window): a packet whose bytes 58..63 read
    // 08 00 00 00 00 00 goes to the general parser, which decides exactly
    // (a TCP header never matches: its data offset is not 0).
    const bool vx = (pe >= 16u) & ((W.w[14] >> 16) == 0x0008u) & (W.w[15] == 0u);
    const bool whole = (uint64_t)off + 16u + L <= B.nbytes;  // else a truncated last record
    const bool shape = whole & (L >= 34u) & ((w7 & 0x000FFFFFu) == 0x00050008u) & ((proto == 6u) | (proto == 17u)) & !vx;
    const bool tcp = proto == 6u;
    // TCP: ports need 20 payload bytes (InvalidPacket); UDP: 8 (InvalidPacket),
    // and exactly 8 leaves an empty "UDP" payload (EmptyPacket, keys.rs:182-184)
    const bool ok = pe >= (tcp ? 20u : 9u);
    h.sip = __builtin_amdgcn_perm(W.w[11], W.w[10], 0x02030405u);
    h.dip = __builtin_amdgcn_perm(W.w[12], W.w[11], 0x02030405u);
    h.ports = __builtin_amdgcn_perm(W.w[13], W.w[12], 0x02030405u);
    h.proto = proto;
    h.doct = max(tl, 20u);  // Ipv4Packet::packet_size()
    h.ttl = (w9 >> 16) & 0xFFu;
    const bool dns = !tcp & (((h.ports >> 16) == 53u) | ((h.ports & 0xFFFFu) == 53u));  // fluereflows.rs:255-291
    h.pkt = dns ? pe : tl;
    h.tf = tcp ? W.w[15] >> 24 : 0u;
    // 802.1Q frames: vlan_keys (keys.rs:417-435) reads the bytes after the tag
    // as a whole Ethernet header, so the key parse fails (the packet is
    // skipped) unless frame bytes 30..31 read 0x0800 / 0x86DD; frames shorter
    // than 32 bytes fail as well.  Those are dropped here, not listed slow.
    const uint32_t in_et = W.w[11] >> 16;  // frame bytes 30, 31
    const bool vlan_drop =
        whole & ((w7 & 0xFFFFu) == 0x0081u) & ((L < 32u) | ((in_et != 0x0008u) & (in_et != 0xDD86u)));
    return shape ? (ok ? HOT_OK : HOT_DROP) : (vlan_drop ? HOT_DROP : HOT_SLOW);
}

// Workgroup barrier for LDS-only hand-offs: waits for this wave's LDS
// operations, not for its outstanding global loads (__syncthreads would drain
// the prefetched windows).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Per-workgroup LDS flow table (k_parse_agg), two parts:
//  * key table, LK entries of 16 bytes (3 key words + proto | state | slot),
//    each written once per launch: claim (CAS of the state word) -> take an
//    aggregate slot from an LDS counter -> key words -> publish.  Load stays
//    low (<= NS / LK), so probe chains are short; two entries per probe step.
//  * NS aggregate slots: the flow's update_flow aggregates for the current
//    window and, once resolved, its dense id.
// The hot loop never needs the dense id: ids are resolved (global dictionary
// walk, all lanes in parallel) only when a window is flushed.  Keys that get
// no slot (more than NS flows in this workgroup) or no key entry take the
// global path per packet (dictionary walk + global atomics).
//   non-MAC kernels: key = (lo_ip, hi_ip, lo_port<<16|hi_port), proto
//   MAC kernels:     key = (dense id, 0, 0), proto 0xFF (the dictionary is
//                    walked per packet; the table only pre-aggregates)
constexpr int LK_BITS = 11;
constexpr int LK = 1 << LK_BITS;        // key entries (32 KiB)
#ifndef FLUERE_NS
#define FLUERE_NS 1200
#endif
constexpr int NS = FLUERE_NS;                // aggregate slots (68 B each, 80 KiB)
constexpr int LK_STEPS = 16;            // probe steps of two entries
#ifndef FLUERE_HOT_PK
#define FLUERE_HOT_PK 1
#endif
#ifndef FLUERE_FLUSH_LINEAR
#define FLUERE_FLUSH_LINEAR 0  // diagnostics only (wrong results): partials in slot order
#endif
#ifndef FLUERE_DENSE_POLICY
#define FLUERE_DENSE_POLICY "nt"  // cache policy of the dense chunk loads (streamed once)
#endif
#ifndef FLUERE_PROBE2
#define FLUERE_PROBE2 1  // 1: two-choice pairs (the inline probe reads both candidate pairs); 0: one pair, linear
#endif
#ifndef FLUERE_AGG_UNCOND
#define FLUERE_AGG_UNCOND 2  // bit 0: min/max, bit 1: first positions as unconditional atomics
#endif
constexpr int PK = FLUERE_HOT_PK;       // packets per lane per hot-loop iteration
static_assert(WIN_ITERS % PK == 0, "a window holds whole iterations");
constexpr uint32_t LT_READY = 1u << 23, LT_CLAIM = 1u << 22, LT_SLOT = LT_CLAIM - 1;
constexpr int MAX_OWNERS = 2048;
// Per-owner counters of a window in LDS, two 16-bit counters per word: counts
// and segment starts of one window stay below 65536 (<= 61440 packets, <= NS
// slots), so a half never carries into its neighbour.
__device__ __forceinline__ uint32_t own_get(const uint32_t* arr, uint32_t o) {
    return (arr[o >> 1] >> ((o & 1) * 16)) & 0xFFFFu;
}
__device__ __forceinline__ uint32_t own_add(uint32_t* arr, uint32_t o) {
    return (atomicAdd(&arr[o >> 1], 1u << ((o & 1) * 16)) >> ((o & 1) * 16)) & 0xFFFFu;
}
__device__ __forceinline__ void own_set(uint32_t* arr, uint32_t o, uint32_t v) {  // (no concurrent writer of the word)
    const uint32_t sh = (o & 1) * 16;
    arr[o >> 1] = (arr[o >> 1] & ~(0xFFFFu << sh)) | (v << sh);
}
constexpr int OWN_WORDS = (MAX_OWNERS + 2) / 2;
constexpr int SPILL_WG = WIN_ITERS * BLOCK;  // raw spilled packets per workgroup (one window)
constexpr int NS_MAC = 768;  // MAC kernels: slots (the key table holds LK / 2 keys + sidecars)

// merge owner of a flow: the top 24 hash bits scaled to [0, O) (multiply-shift)
__device__ __forceinline__ uint32_t owner_of(uint32_t h, uint32_t O) {
    return (uint32_t)(((uint64_t)(h >> 8) * O) >> 24);
}

__device__ __forceinline__ uint32_t lt_hash(uint32_t k0, uint32_t k1, uint32_t k2, uint32_t tag) {
    uint32_t h = (k0 * 0x9E3779B1u) ^ (k1 * 0x85EBCA77u) ^ (k2 * 0xC2B2AE3Du) ^ tag;
    h ^= h >> 16;
    h *= 0x7FEB352Du;
    h ^= h >> 15;
    return h;
}

// MAC kernels (-M): the flow key is the 5-tuple words plus the canonical MAC
// pair packed in three words, m0 = lo MAC bytes 0..3, m1 = lo MAC bytes 4..5
// << 16 | hi MAC bytes 4..5, m2 = hi MAC bytes 0..3 (dictionary words 10..13
// of the canonical key, flow_table.h).  Key tables keep the MAC words in a
// sidecar entry whose w = 1 marks it written.
__device__ __forceinline__ uint32_t mac_hash(uint32_t h, uint32_t m0, uint32_t m1, uint32_t m2) {
    return h ^ lt_hash(m0, m1, m2, 0x5BD1E995u);
}
// The dictionary key of a MAC-kernel key (same words as flow_of with macs).
__device__ __forceinline__ void mac_ckey(uint32_t k0, uint32_t k1, uint32_t k2, uint32_t tag, uint32_t m0,
                                         uint32_t m1, uint32_t m2, CKey& k) {
#pragma unroll
    for (int j = 0; j < 14; j++) k.w[j] = 0;
    k.w[0] = k0;
    k.w[4] = k1;
    k.w[8] = k2;
    k.w[9] = (2u << 8) | (tag >> 24);
    k.w[10] = m0;
    k.w[11] = m1 & 0xFFFF0000u;
    k.w[12] = m2;
    k.w[13] = m1 << 16;
}

// ABL (diagnostics only): 5 every LDS-table miss written to its lane's own
// contiguous run (4 consecutive misses of a lane fill one 128-B line; wrong
// results: the merge never sees them) -- the store pattern of per-owner bins;
// 4 every LDS-table miss appended to the workgroup's
// raw buffer (coalesced, wave-aggregated) instead of its owner segment (still
// correct: the overflow list); 0 full kernel; 1 parse + canonical key only; 2 + LDS key
// table, no aggregation; 3 aggregation into hashed slots without the key table
template <int ABL, bool MACS>
__global__ void __launch_bounds__(BLOCK) k_parse_agg(AggArgs a) {
    // LDS flow table.  Per slot: packets (low 32) and bytes (high 32) per
    // canonical direction in one u64 (one ds_add_u64 per packet; a window
    // holds <= 61440 packets of <= 65535 bytes, so neither half wraps);
    // {min pkt, min ttl, max pkt, max ttl}; window-relative positions
    // {first, first create-eligible, first FIN/RST, last + 1}; flag pairs.
    __shared__ uint4 s_key[LK];
    __shared__ unsigned long long s_pb[2][NS];
    __shared__ uint4 s_mm[NS], s_pos[NS];
    __shared__ uint32_t s_fl[4][NS];
    __shared__ uint32_t s_sk[NS];  // key entry of each slot
    __shared__ uint4 s_slab[BLOCK / 64][160];  // per wave: half a dense chunk's span (32 x 80 B)
    __shared__ uint32_t s_nslot, s_chunk, s_nspill;
    __shared__ uint32_t s_own[OWN_WORDS];   // flush: per-owner slot counts -> segment starts (packed, own_get)
    __shared__ uint32_t s_scnt[OWN_WORDS];  // spilled packets per owner (this window) -> segment starts (packed)
    __shared__ unsigned long long s_sbase;
    __shared__ unsigned long long s_cnt[5], s_tmin, s_tmax;
    __shared__ uint32_t s_slow;  // this workgroup's slow-list entries
    const int tid = threadIdx.x;
    // MAC kernels: LK / 2 key entries, each with its MAC sidecar at + LK / 2
    constexpr int LKL = MACS ? LK / 2 : LK, LKL_BITS = MACS ? LK_BITS - 1 : LK_BITS;
    constexpr uint32_t NSL = MACS ? NS_MAC : NS;
    constexpr int SPU = spill_units(MACS);
    for (int e = tid; e < LK; e += BLOCK) s_key[e] = make_uint4(0, 0, 0, 0);
    for (int e = tid; e < NS; e += BLOCK) {
        s_pb[0][e] = s_pb[1][e] = 0;
        s_mm[e] = make_uint4(NONE32, NONE32, 0, 0);
        s_pos[e] = make_uint4(NONE32, NONE32, NONE32, 0);
        s_fl[0][e] = s_fl[1][e] = s_fl[2][e] = s_fl[3][e] = 0;
    }
    if (tid < 5) s_cnt[tid] = 0;
    if (tid == 0) s_slow = 0;
    if (tid == 0) { s_tmin = NONE64; s_tmax = 0; s_nslot = 0; s_chunk = 0; s_nspill = 0; }
    for (int o = tid; o < OWN_WORDS; o += BLOCK) s_scnt[o] = 0;
    __syncthreads();

    const Batch& B = a.B;
    const uint64_t n = B.n;
#ifndef FLUERE_HOT_ORDER
#define FLUERE_HOT_ORDER 1
#endif
    // Packet order.  Step st of workgroup b covers BLOCK consecutive packets:
    //   ORDER 1 (interleaved): packets (st * G + b) * BLOCK + [0, BLOCK) -- all
    //     workgroups stream one moving region of the capture together;
    //   ORDER 0 (contiguous): workgroup b owns the range [b * per, (b+1) * per).
    // Positions inside a window are relative to the window's first packet
    // (at most WIN_ITERS * G * BLOCK apart: they fit u32).
    const uint64_t G = gridDim.x;
    const uint64_t per = (n + G - 1) / G;
    const uint64_t stride = FLUERE_HOT_ORDER ? G * BLOCK : BLOCK;
    const uint64_t beg = FLUERE_HOT_ORDER ? (uint64_t)blockIdx.x * BLOCK : per * blockIdx.x;
    const uint64_t end = FLUERE_HOT_ORDER ? n : min(n, beg + per);
    unsigned long long c_valid = 0, c_drop = 0, c_miss = 0, tmin = NONE64, tmax = 0;
    uint32_t d_loops = 0, d_iters = 0;  // diagnostics (per wave, uniform)
    uint32_t d_abl5 = 0;                // diagnostics (ABL 5): this lane's misses
    const uint64_t nsteps = end > beg ? (end - beg + stride - 1) / stride : 0;
    uint64_t wbase = beg;
    uint32_t win = 0;  // this workgroup's window (set blockIdx.x * W + win)

    // PK packets per lane per iteration (steps st .. st+PK-1), processed
    // phase by phase so that the LDS round trips of the PK packets overlap
    // (every phase issues its reads for all PK packets before using any).
    // Packets the hot parser declines, and packets of keys that find no LDS
    // slot, are appended to the slow list: slow_packets runs the general
    // parser and the global path for them (nothing rare is inlined here).
    struct PS {
        Hot h;
        uint32_t dir, lo_ip, hi_ip, kports, k0, k1, k2, tag, e, e2, slot;
        uint32_t m0, m1, m2;  // MAC kernels: the canonical MAC pair (mac_ckey)
        int state, steps;
        bool valid, slow;
    };
    auto process = [&](const Win (&W)[PK], const uint32_t (&off)[PK], const uint64_t (&li)[PK], const bool (&live)[PK]) {
        PS q[PK];
#pragma unroll
        for (int u = 0; u < PK; u++) {
            Hot& h = q[u].h;
            const uint32_t cls = live[u] ? hot_parse(B, off[u], W[u], h) : HOT_DROP;
            c_drop += (live[u] & (cls == HOT_DROP)) ? 1 : 0;
            q[u].valid = live[u] & (cls == HOT_OK);
            q[u].slow = live[u] & (cls == HOT_SLOW);
            // canonical key: lower endpoint (ip, port[, mac]) first (flow_table.h)
            const uint32_t sp = h.ports >> 16, dp = h.ports & 0xFFFFu;
            bool gt = (h.sip > h.dip) | ((h.sip == h.dip) & (sp > dp));
            uint64_t smac = 0, dmac = 0;
            if (MACS) {
                const uint32_t d_hi = __builtin_amdgcn_perm(W[u].w[5], W[u].w[4], 0x00010203u);  // frame bytes 0..3
                const uint32_t d_lo = __builtin_amdgcn_perm(W[u].w[5], W[u].w[4], 0x0C0C0405u);  // frame bytes 4..5
                const uint32_t s_hi = __builtin_amdgcn_perm(W[u].w[6], W[u].w[5], 0x02030405u);  // frame bytes 6..9
                const uint32_t s_lo = __builtin_amdgcn_perm(W[u].w[6], W[u].w[5], 0x0C0C0607u);  // frame bytes 10..11
                dmac = ((uint64_t)d_hi << 16) | d_lo;
                smac = ((uint64_t)s_hi << 16) | s_lo;
                if ((h.sip == h.dip) & (sp == dp)) gt = smac > dmac;
            }
            q[u].dir = gt ? 1u : 0u;
            q[u].lo_ip = gt ? h.dip : h.sip;
            q[u].hi_ip = gt ? h.sip : h.dip;
            q[u].kports = gt ? __builtin_amdgcn_alignbit(h.ports, h.ports, 16) : h.ports;
            q[u].k0 = q[u].lo_ip;
            q[u].k1 = q[u].hi_ip;
            q[u].k2 = q[u].kports;
            q[u].tag = h.proto << 24;
            if (!MACS && a.phash && live[u])
                a.phash[li[u]] = q[u].valid ? ckey_bucket_v4(q[u].k0, q[u].k1, q[u].k2, h.proto) : PH_PARSE;
            q[u].m0 = q[u].m1 = q[u].m2 = 0;
            if (MACS) {  // the MAC pair joins the key (the dictionary is walked once per slot, at the flush)
                const uint64_t lom = gt ? dmac : smac, him = gt ? smac : dmac;
                q[u].m0 = (uint32_t)(lom >> 16);
                q[u].m1 = ((uint32_t)(lom & 0xFFFF) << 16) | (uint32_t)(him & 0xFFFF);
                q[u].m2 = (uint32_t)(him >> 16);
            }
        }
        if (ABL == 1) {
#pragma unroll
            for (int u = 0; u < PK; u++)
                if (q[u].valid)
                    asm volatile("" ::"v"(q[u].lo_ip ^ q[u].hi_ip ^ q[u].kports ^ q[u].h.proto ^ q[u].h.doct ^
                                          q[u].h.pkt ^ q[u].h.ttl ^ q[u].dir));
            return;
        }
        // find or claim the key entries.  First probe of every packet inline
        // (the common case: a published entry at the home position); the
        // wave-uniform retry loop runs only while some lane still searches (a
        // lane that lost a claim, or saw an entry being written, reads the
        // pair again next step).
        // Probe sequence of a key: pair e1, pair e2, then linear from e2 + 2
        // (write-once table, so lookups and inserts follow one sequence).
        // Two-choice placement keeps nearly every key in one of its first two
        // pairs; both are read inline, so the retry loop below runs only for
        // inserts and for the rare key placed further on.
        uint32_t hk[PK];
        uint4 kp[PK][4];
#pragma unroll
        for (int u = 0; u < PK; u++) {
            hk[u] = lt_hash(q[u].k0, q[u].k1, q[u].k2, q[u].tag);
            if (MACS) hk[u] = mac_hash(hk[u], q[u].m0, q[u].m1, q[u].m2);
            const uint32_t e1 = hk[u] & (LKL - 2);  // even: entries e, e+1 per step
            uint32_t e2 = (hk[u] >> 12) * 0x9E3779B1u >> (32 - LKL_BITS + 1) << 1;
            e2 = FLUERE_PROBE2 ? (e2 == e1 ? e1 ^ 2u : e2) : (e1 + 2) & (LKL - 1);
            q[u].e = e1;
            q[u].e2 = e2;
            kp[u][0] = s_key[e1];
            kp[u][1] = s_key[e1 + 1];
            kp[u][2] = FLUERE_PROBE2 ? s_key[e2] : make_uint4(0, 0, 0, 0);
            kp[u][3] = FLUERE_PROBE2 ? s_key[e2 + 1] : make_uint4(0, 0, 0, 0);
        }
        bool searching = false;
#pragma unroll
        for (int u = 0; u < PK; u++) {
            bool m[4];
#pragma unroll
            for (int k = 0; k < 4; k++)
                m[k] = ((kp[u][k].w & (0xFF000000u | LT_READY)) == (q[u].tag | LT_READY)) & (kp[u][k].x == q[u].k0) &
                       (kp[u][k].y == q[u].k1) & (kp[u][k].z == q[u].k2);
            if (MACS) {
                // the sidecar of an entry whose 5-tuple words match (read after the
                // entry, so a published entry's sidecar is seen written)
                bool hit = false;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    if (m[k] & !hit) {
                        const uint32_t ek = (k < 2 ? q[u].e : q[u].e2) + (k & 1);
                        const uint4 xs = s_key[LKL + ek];
                        m[k] = (xs.w == 1u) & (xs.x == q[u].m0) & (xs.y == q[u].m1) & (xs.z == q[u].m2);
                        hit = m[k];
                    } else {
                        m[k] = false;
                    }
                }
            }
            const uint32_t sw = m[0] ? kp[u][0].w : m[1] ? kp[u][1].w : m[2] ? kp[u][2].w : kp[u][3].w;
            q[u].slot = sw & LT_SLOT;
            const bool found = m[0] | m[1] | m[2] | m[3];
            q[u].state = q[u].valid ? (found ? 1 : 0) : 2;  // 0 searching, 1 found (slot < NS, or NS: no slot), 2 none
            const bool full1 = (kp[u][0].w & kp[u][1].w & LT_READY) != 0;
            const bool full2 = (kp[u][2].w & kp[u][3].w & LT_READY) != 0;
            // where the search goes on: the first pair of the sequence not yet
            // known to be full of other keys
            q[u].steps = full1 ? (full2 ? 2 : 1) : 0;
            q[u].e = full1 ? (full2 ? (q[u].e2 + 2) & (LKL - 1) : q[u].e2) : q[u].e;
            if (ABL == 3) {  // diagnostics: aggregation without the key table (wrong slots)
                q[u].slot = lt_hash(q[u].k0, q[u].k1, q[u].k2, q[u].tag) % 1000u;
                q[u].state = q[u].valid ? 1 : 2;
            }
            searching |= q[u].state == 0;
        }
        // every aggregate slot taken (more flows in this window than NS): a
        // key not in its two inline pairs spills at once -- inserting it
        // would gain nothing, and the search through a full table costs a
        // dozen LDS round trips per chunk
        if (searching && s_nslot >= NSL) {
#pragma unroll
            for (int u = 0; u < PK; u++)
                if (q[u].state == 0) q[u].state = 2;
            searching = false;
        }
        if (ABL != 3 && __ballot(searching)) {
            d_loops++;
            for (int it = 0; it < 2 * LK_STEPS; it++) {
                d_iters++;
                bool more = false;
#pragma unroll
                for (int u = 0; u < PK; u++) {
                    PS& r = q[u];
                    if (r.state == 0) {
                        const uint4 ka = s_key[r.e], kb = s_key[r.e + 1];
                        bool ma = (ka.w & (0xFF000000u | LT_READY)) == (r.tag | LT_READY) && ka.x == r.k0 &&
                                  ka.y == r.k1 && ka.z == r.k2;
                        bool mb = (kb.w & (0xFF000000u | LT_READY)) == (r.tag | LT_READY) && kb.x == r.k0 &&
                                  kb.y == r.k1 && kb.z == r.k2;
                        if (MACS) {
                            const uint4 xa = s_key[LKL + r.e], xb = s_key[LKL + r.e + 1];
                            ma = ma && xa.w == 1u && xa.x == r.m0 && xa.y == r.m1 && xa.z == r.m2;
                            mb = mb && xb.w == 1u && xb.x == r.m0 && xb.y == r.m1 && xb.z == r.m2;
                        }
                        if (ma || mb) {
                            r.slot = (ma ? ka.w : kb.w) & LT_SLOT;
                            r.state = 1;
                        } else if ((ka.w & LT_READY) && (kb.w & LT_READY)) {
                            if (++r.steps == LK_STEPS) r.state = 2;
                            else r.e = r.steps == 1 ? r.e2 : (r.e + 2) & (LKL - 1);
                        } else {
                            // first free entry of the pair; an entry being written (CLAIM) is re-read next step
                            const uint32_t f = (ka.w == 0) ? r.e : ((ka.w & LT_READY) && kb.w == 0 ? r.e + 1 : LKL);
                            if (f < LKL && atomicCAS(&s_key[f].w, 0u, LT_CLAIM) == 0u) {
                                uint32_t sl = atomicAdd(&s_nslot, 1u);
                                if (sl >= NSL) sl = NSL;  // no slot left: the key is kept, its packets spill
                                s_key[f].x = r.k0;
                                s_key[f].y = r.k1;
                                s_key[f].z = r.k2;
                                if (MACS) s_key[LKL + f] = make_uint4(r.m0, r.m1, r.m2, 1u);
                                if (sl < NSL) s_sk[sl] = f;
                                __threadfence_block();
                                atomicExch(&s_key[f].w, r.tag | LT_READY | (sl < NSL ? sl : LT_SLOT));
                                r.slot = sl;
                                r.state = 1;
                            }
                        }
                    }
                    more |= r.state == 0;
                }
                if (__ballot(more) == 0) break;
            }
        }
        bool agg[PK];
#pragma unroll
        for (int u = 0; u < PK; u++) {
            agg[u] = q[u].valid & (q[u].state == 1) & (q[u].slot < NSL);
            // a valid packet whose key has no LDS slot spills: a 32-byte record
            // (64 with MACs) straight into its merge owner's segment of this
            // set; past the segment's capacity, to this workgroup's raw
            // overflow buffer (wave-aggregated append; listed at the flush)
            const bool miss = q[u].valid & !agg[u];
            c_miss += miss ? 1 : 0;
            bool ovf = false;
            if (miss) {
                const Hot& h = q[u].h;
                const uint32_t loc = (uint32_t)(li[u] - wbase);
                const bool elig = (h.proto != 6u) | ((h.tf & 2u) != 0);
                const uint4 w_key = make_uint4(q[u].k0, q[u].k1, q[u].k2, q[u].tag);
                const uint4 w_pay = make_uint4(h.doct, h.pkt | (h.ttl << 16) | ((elig ? 1u : 0u) << 24), loc,
                                               h.tf | (q[u].dir << 8));
                const uint32_t ow = owner_of(hk[u], a.S.O);
                const uint32_t pos = ABL == 4 ? 0xFFFFFFFFu : ABL == 5 ? 0u : own_add(s_scnt, ow);
                if (ABL == 5) {
                    uint4* dst = reinterpret_cast<uint4*>(a.S.spill_raw) + (size_t)blockIdx.x * SPILL_WG * 2 +
                                 ((size_t)threadIdx.x * WIN_ITERS + (d_abl5++ % WIN_ITERS)) * 2;
                    dst[0] = w_key;
                    dst[1] = w_pay;
                } else if (pos < a.S.cap_o) {
                    uint4* dst = reinterpret_cast<uint4*>(a.S.dspill) +
                                 (((size_t)(blockIdx.x * a.S.W + win) * a.S.O + ow) * a.S.cap_o + pos) * (2 * SPU);
                    dst[0] = w_key;
                    if (MACS) {
                        dst[1] = make_uint4(q[u].m0, q[u].m1, q[u].m2, hk[u]);
                        dst[2] = w_pay;
                    } else {
                        dst[1] = w_pay;
                    }
                } else {
                    ovf = true;
                }
                c_valid++;
                tmin = min(tmin, (unsigned long long)h.t);
                tmax = max(tmax, (unsigned long long)h.t);
            }
            const uint64_t mm_ = __ballot(ovf);
            if (mm_) {
                const uint32_t lead = __builtin_ctzll(mm_);
                uint32_t b0 = 0;
                if ((uint32_t)(threadIdx.x & 63) == lead) b0 = atomicAdd(&s_nspill, (uint32_t)__popcll(mm_));
                b0 = __shfl(b0, lead, 64);
                if (ovf) {
                    const Hot& h = q[u].h;
                    const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(mm_ >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)mm_, 0u));
                    const uint32_t loc = (uint32_t)(li[u] - wbase);
                    const bool elig = (h.proto != 6u) | ((h.tf & 2u) != 0);
                    uint4* dst = reinterpret_cast<uint4*>(a.S.spill_raw) + (size_t)blockIdx.x * SPILL_WG * 2 * SPU + b0 + r;
                    dst[0] = make_uint4(q[u].k0, q[u].k1, q[u].k2, q[u].tag);
                    if (MACS) dst[SPILL_WG] = make_uint4(q[u].m0, q[u].m1, q[u].m2, hk[u]);
                    dst[(MACS ? 2 : 1) * SPILL_WG] = make_uint4(h.doct, h.pkt | (h.ttl << 16) | ((elig ? 1u : 0u) << 24),
                                                                loc, h.tf | (q[u].dir << 8));
                }
            }
            const bool slow = q[u].slow;
            // slow list: wave-aggregated append into this workgroup's region
            // (an LDS cursor; one global atomic per wave on a single counter
            // serialised an all-slow capture: 1.9 ms for 10M packets)
            const uint64_t sm = __ballot(slow);
            if (sm) {
                const uint32_t lead = __builtin_ctzll(sm);
                uint32_t b0 = 0;
                if ((uint32_t)(threadIdx.x & 63) == lead) b0 = atomicAdd(&s_slow, (uint32_t)__popcll(sm));
                b0 = __shfl(b0, lead, 64);
                if (slow) {
                    const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(sm >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)sm, 0u));
                    a.slow[(size_t)blockIdx.x * a.slow_region + b0 + r] = (uint32_t)li[u];
                }
            }
        }
        if (ABL == 2) {  // diagnostics: key table only
#pragma unroll
            for (int u = 0; u < PK; u++) asm volatile("" ::"v"(q[u].slot));
            return;
        }
        // update_flow (flows.rs:11-42), order-free part.  Guard reads of every
        // packet first (a slot index of 0 for lanes without an update keeps
        // them unconditional), then the atomics: min / max and first
        // positions change rarely, so they are written only where the packet
        // moves the value (a stale guard can only cost a redundant atomic,
        // never skip a needed one: the values move monotonically).
        uint4 mm[PK];
        uint2 ps[PK];
#pragma unroll
        for (int u = 0; u < PK; u++) {
            const uint32_t sl = agg[u] ? q[u].slot : 0u;
            if (!(FLUERE_AGG_UNCOND & 1)) mm[u] = s_mm[sl];
            if (!(FLUERE_AGG_UNCOND & 2)) ps[u] = *reinterpret_cast<const uint2*>(&s_pos[sl]);
        }
#pragma unroll
        for (int u = 0; u < PK; u++) {
            if (!agg[u]) continue;
            const Hot& h = q[u].h;
            const uint32_t slot = q[u].slot;
            c_valid++;
            tmin = min(tmin, (unsigned long long)h.t);
            tmax = max(tmax, (unsigned long long)h.t);
            const uint32_t tf = h.tf;
            const uint32_t loc = (uint32_t)(li[u] - wbase);
            atomicAdd(&s_pb[q[u].dir][slot], ((unsigned long long)h.doct << 32) | 1ull);
            atomicMax(&s_pos[slot].w, loc + 1);
            if (FLUERE_AGG_UNCOND & 1) {
                atomicMin(&s_mm[slot].x, h.pkt);
                atomicMin(&s_mm[slot].y, h.ttl);
                atomicMax(&s_mm[slot].z, h.pkt);
                atomicMax(&s_mm[slot].w, h.ttl);
            } else {
                if (h.pkt < mm[u].x) atomicMin(&s_mm[slot].x, h.pkt);
                if (h.ttl < mm[u].y) atomicMin(&s_mm[slot].y, h.ttl);
                if (h.pkt > mm[u].z) atomicMax(&s_mm[slot].z, h.pkt);
                if (h.ttl > mm[u].w) atomicMax(&s_mm[slot].w, h.ttl);
            }
            // a flow is created by any non-TCP packet or a SYN (offline_fluereflows.rs:101-113)
            const bool elig = (h.proto != 6u) | ((tf & 2u) != 0);
            if (FLUERE_AGG_UNCOND & 2) {
                atomicMin(&s_pos[slot].x, loc);
                atomicMin(&s_pos[slot].y, elig ? loc : NONE32);
            } else {
                if (loc < ps[u].x) atomicMin(&s_pos[slot].x, loc);
                if (elig & (loc < ps[u].y)) atomicMin(&s_pos[slot].y, loc);
            }
            if (tf) {
#pragma unroll
                for (int qq = 0; qq < 4; qq++) {
                    const uint32_t w = ((tf >> (2 * qq)) & 1) | (((tf >> (2 * qq + 1)) & 1) << 16);
                    if (w) atomicAdd(&s_fl[qq][slot], w);
                }
                if (tf & 5) atomicMin(&s_pos[slot].z, loc);  // FIN or RST
            }
        }
    };
    unsigned long long cyc_flush = 0, cyc_flush0 = 0, cyc_wait = 0, cyc_start = clock64(), rt_start = wall_clock64();
    uint32_t ovf_total = 0;  // (thread 0) overflow records of every window
    auto flush = [&]() {
        // the window's partial aggregates -> this workgroup's staging set
        // (plain coalesced stores, lane per slot); k_merge_partials merges them
        const unsigned long long fw = clock64();
        if (a.dbg && tid == 0 && win == 0) a.dbg[blockIdx.x * 8 + 1] = wall_clock64();
        // every wave's spill stores have completed (vmcnt) before the barrier
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        const unsigned long long f0 = clock64();  // flush proper (fw..f0: waiting for the slowest wave)
        cyc_wait += f0 - fw;
        const Stage& S = a.S;
        const uint32_t set = blockIdx.x * S.W + win;
        const uint32_t ns = min(s_nslot, NSL), O = S.O;
        if (tid == 0) s_chunk = 0;  // every wave has drawn its last chunk of the window
        // counting sort of this window's flows by merge owner; a thread keeps
        // its slots' (at most two) owners and hashes in registers
        constexpr int SPT = (NS + BLOCK - 1) / BLOCK;  // slots per thread
        for (uint32_t o = tid; o < OWN_WORDS; o += BLOCK) s_own[o] = 0;
        lds_barrier();
        uint32_t own[SPT], hh[SPT];
        uint4 kks[SPT];
#pragma unroll
        for (int k = 0; k < SPT; k++) {
            own[k] = NONE32;
            hh[k] = 0;
        }
#pragma unroll
        for (int k = 0; k < SPT; k++) {
            const uint32_t e = tid + k * BLOCK;
            if (e >= ns || (s_pb[0][e] | s_pb[1][e]) == 0) continue;
            kks[k] = s_key[s_sk[e]];
            hh[k] = lt_hash(kks[k].x, kks[k].y, kks[k].z, kks[k].w & 0xFF000000u);
            if (MACS) {  // the MAC words travel beside the partial (S.partx); same hash as the hot loop's
                const uint4 xs = s_key[LKL + s_sk[e]];
                hh[k] = mac_hash(hh[k], xs.x, xs.y, xs.z);
            }
            own[k] = owner_of(hh[k], O);
            own_add(s_own, own[k]);
        }
        lds_barrier();
        if (a.dbg && tid == 0 && win == 0) a.dbg[blockIdx.x * 8 + 4] = wall_clock64();
        // exclusive scan of the slot counts over the owners (one wave, an
        // even run of owners per lane, so no two lanes write one packed word)
        static_assert(MAX_OWNERS % 2 == 0, "owner runs cover whole words");
        if (tid < 64) {
            uint32_t* arr = s_own;
            const uint32_t l = tid & 63;
            const uint32_t per = 2 * ((O + 127) / 128);
            uint32_t sum = 0;
            for (uint32_t q = 0; q < per; q++) {
                const uint32_t o = l * per + q;
                if (o < O) sum += own_get(arr, o);
            }
            uint32_t incl = sum;
#pragma unroll
            for (int dlt = 1; dlt < 64; dlt <<= 1) {
                const uint32_t y = __shfl_up(incl, dlt, 64);
                if (l >= dlt) incl += y;
            }
            uint32_t run = incl - sum;
            for (uint32_t q = 0; q < per; q++) {
                const uint32_t o = l * per + q;
                if (o < O) {
                    const uint32_t v = own_get(arr, o);
                    own_set(arr, o, run);
                    run += v;
                }
            }
            if (l == 63) own_set(arr, O, incl);
        }
        const uint32_t nsp = s_nspill;  // overflow records of this window
        if (tid == 128) s_sbase = nsp ? atomicAdd(&a.g->n_spill, (unsigned long long)nsp) : 0ull;
        if (tid == 0) ovf_total += nsp;
        lds_barrier();
        for (uint32_t o = tid; o <= O; o += BLOCK) {
            S.off[(size_t)o * S.n_sets + set] = own_get(s_own, o);
            if (o < O) S.soff[(size_t)o * S.n_sets + set] = min(own_get(s_scnt, o), S.cap_o);
        }
        if (tid == 0) S.base[set] = B.first + wbase;
        lds_barrier();
        if (a.dbg && tid == 0 && win == 0) a.dbg[blockIdx.x * 8 + 5] = wall_clock64();
        // overflow records -> the overflow list (the raw records were written
        // by other waves of this workgroup: nontemporal loads, which bypass
        // the CU's L1); the set goes into fl's high bits
        if (nsp) {
            const uint4* raw = reinterpret_cast<const uint4*>(S.spill_raw) + (size_t)blockIdx.x * SPILL_WG * 2 * SPU;
            const unsigned long long sb = s_sbase;
            // SU records per thread per round, all loads issued first (one
            // round trip per round instead of one per record)
            constexpr int SU = 4;
            typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
            const uint32_t last = nsp ? nsp - 1 : 0;  // (loads stay inside the buffer even if hoisted)
            constexpr int SW = MACS ? 3 : 2;  // 16-byte words per spilled packet
            for (uint32_t i0 = 0; i0 < nsp; i0 += SU * BLOCK) {
                u32x4 av[SU][SW];
#pragma unroll
                for (int u = 0; u < SU; u++) {
                    const uint32_t i = i0 + u * BLOCK + tid;
                    const u32x4* src = reinterpret_cast<const u32x4*>(raw + min(i, last));
#pragma unroll
                    for (int w = 0; w < SW; w++) av[u][w] = __builtin_nontemporal_load(src + (size_t)w * SPILL_WG);
                }
                // every load of the round issued before the first use (the
                // compiler would sink a guarded record's loads into its branch)
#pragma unroll
                for (int u = 0; u < SU; u++)
#pragma unroll
                    for (int w = 0; w < SW; w++) asm volatile("" ::"v"(av[u][w]));
#pragma unroll
                for (int u = 0; u < SU; u++) {
                    const uint32_t i = i0 + u * BLOCK + tid;
                    if (i >= nsp) continue;
                    av[u][SW - 1].w |= set << 9;
                    uint4* dst = reinterpret_cast<uint4*>(S.spill) + (sb + i) * (size_t)(2 * SPU);
#pragma unroll
                    for (int w = 0; w < SW; w++) dst[w] = make_uint4(av[u][w].x, av[u][w].y, av[u][w].z, av[u][w].w);
                }
            }
        }
#pragma unroll
        for (int k = 0; k < SPT; k++) {
            const uint32_t e = tid + k * BLOCK;
            if (own[k] == NONE32) continue;
            const unsigned long long p0 = s_pb[0][e], p1 = s_pb[1][e];
            const uint4 kk = kks[k];
            const uint32_t tag = kk.w & 0xFF000000u;
            const uint32_t h = hh[k];
            const size_t o = (size_t)set * NS + (FLUERE_FLUSH_LINEAR ? e : own_add(s_own, own[k]));
            uint4* dst = reinterpret_cast<uint4*>(S.part + o);
            if (FLUERE_FLUSH_LINEAR == 2 && kk.x != 0x12345678u) continue;  // diagnostics: no stores
            dst[0] = make_uint4(kk.x, kk.y, kk.z, tag);
            dst[1] = make_uint4(h, (uint32_t)(p0 & 0xFFFF) | ((uint32_t)(p1 & 0xFFFF) << 16), (uint32_t)(p0 >> 32),
                                (uint32_t)(p1 >> 32));
            const uint4 mm = s_mm[e];
            dst[2] = make_uint4(mm.x, mm.y, mm.z, mm.w);
            dst[3] = make_uint4(s_fl[0][e], s_fl[1][e], s_fl[2][e], s_fl[3][e]);
            dst[4] = s_pos[e];
            if (MACS) {  // (re-read from LDS: registers are scarce across the spill scatter)
                const uint4 xs = s_key[LKL + s_sk[e]];
                S.partx[o] = make_uint4(xs.x, xs.y, xs.z, h);
            }
            s_pb[0][e] = s_pb[1][e] = 0;
            s_mm[e] = make_uint4(NONE32, NONE32, 0, 0);
            s_pos[e] = make_uint4(NONE32, NONE32, NONE32, 0);
            s_fl[0][e] = s_fl[1][e] = s_fl[2][e] = s_fl[3][e] = 0;
        }
        lds_barrier();
        if (a.dbg && tid == 0 && win == 0) a.dbg[blockIdx.x * 8 + 6] = wall_clock64();
        for (uint32_t o = tid; o < OWN_WORDS; o += BLOCK) s_scnt[o] = 0;
        if (tid == 0) s_nspill = 0;
        lds_barrier();
        const unsigned long long f1 = clock64() - f0;
        if (a.dbg && tid == 0 && win == 0) a.dbg[blockIdx.x * 8 + 2] = wall_clock64();
        if (win == 0) cyc_flush0 = f1;
        cyc_flush += f1;
        wbase += stride * WIN_ITERS;
        win++;
    };
    const uint64_t lastp = n - 1;  // loads past the end re-read the last packet (in bounds)
    // Window by window.  A window is WIN_ITERS steps of this workgroup, i.e.
    // WIN_ITERS * WAVES wave-chunks of 64 packets; the chunks are dealt to the
    // waves dynamically (an LDS counter) so the waves of a workgroup finish a
    // window together (static assignment left waves idle for ~10% of the
    // kernel while the slowest one finished).  Per chunk the offset of the
    // wave's next chunk is prefetched (one register of carry), the window is
    // loaded and consumed in the same iteration and pinned (pin_win) so its
    // loads form one round trip; only offsets cross the back edge.
    static_assert(PK == 1, "dynamic chunks: one packet per lane per iteration");
    constexpr uint32_t WAVES = BLOCK / 64;
    const uint32_t lane = tid & 63;
    uint4* slab = s_slab[__builtin_amdgcn_readfirstlane(tid >> 6)];
    auto grab = [&]() {
        uint32_t v = 0;
        if (lane == 0) v = atomicAdd(&s_chunk, 1u);
        return __builtin_amdgcn_readfirstlane(v);
    };
    // a per-lane zero the compiler cannot see through: keeps the (uniform)
    // descriptor loads on the vector memory path (vmcnt), so they never hold
    // up the LDS waits (lgkmcnt) of the processing as a scalar load would
    uint32_t vzero;
    asm volatile("v_mov_b32 %0, 0" : "=v"(vzero));
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    for (uint64_t ws = 0; ws < nsteps; ws += WIN_ITERS) {
        const uint32_t nch = (uint32_t)min<uint64_t>(WIN_ITERS, nsteps - ws) * WAVES;
        auto li_of = [&](uint32_t c) -> uint64_t {
            return beg + (ws + c / WAVES) * stride + (uint64_t)(c % WAVES) * 64 + lane;
        };
        // descriptor of chunk c (Batch::desc): a vector load, every lane the same word
        auto desc_of = [&](uint32_t c) -> uint2 {
            const uint64_t ch = (li_of(c) - lane) >> 6;
            if (c >= nch || ch >= B.n_desc) return make_uint2(0, 0);
            return B.desc[ch + vzero];
        };
        // Software pipeline, one chunk deep: while chunk c is processed the
        // loads of the wave's next chunk cn are in flight.  Dense chunks: six
        // coalesced nontemporal 16-byte loads per lane cover the chunk's span
        // (64 windows at stride <= 80 B); they are transposed to per-lane
        // windows through the wave's LDS slab.  Sparse chunks: the record
        // offsets are loaded one chunk ahead, the windows when processed.
        // The loads are issued unconditionally (inline asm; a chunk that does
        // not need them points them at one cached line), so no branch merges
        // registers that are still being loaded: such a merge makes the
        // compiler copy them, which waits for them and drains the pipeline.
        // Their completion is waited for explicitly (vmcnt(0) at the top).
        u32x4 v[5];
        uint32_t osp;
        auto issue = [&](uint32_t c, uint2 d) {
            const bool dense = d.y != 0;
            const uint64_t li = min(li_of(c), lastp);
            const uint8_t* g = dense ? B.bytes + d.x : reinterpret_cast<const uint8_t*>(B.offs + (li & ~63ull));
            const uint32_t np = dense ? (63u * d.y + 80u + 15u) / 16u : 1u;
#pragma unroll
            for (int k = 0; k < 5; k++) {
                const uint8_t* p = g + 16u * min(k * 64u + lane, np - 1u);
                asm volatile("global_load_dwordx4 %0, %1, off " FLUERE_DENSE_POLICY : "=v"(v[k]) : "v"(p) : "memory");
            }
            const uint32_t* po = dense ? B.offs : B.offs + li;
            asm volatile("global_load_dword %0, %1, off" : "=v"(osp) : "v"(po) : "memory");
        };
        uint32_t c = grab();
        uint2 dc = desc_of(c);
        dc.x = __builtin_amdgcn_readfirstlane(dc.x);
        dc.y = __builtin_amdgcn_readfirstlane(dc.y);
        issue(c, dc);
        uint32_t cn = grab();
        uint2 dn_v = desc_of(cn);
        while (c < nch) {
            const uint32_t c2 = grab();
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // chunk c's loads (issue) and dn_v
            const uint2 dn = make_uint2(__builtin_amdgcn_readfirstlane(dn_v.x), __builtin_amdgcn_readfirstlane(dn_v.y));
            Win W[1];
            uint32_t o1[1];
            const uint64_t lis[1] = {li_of(c)};
            bool live[1];
            if (dc.y) {
                // two halves of 32 records through a 160-piece slab: half h
                // needs pieces [2hS, 2hS + 160) of the span, record i its
                // five pieces at slab byte (i & 31) * S (16-byte aligned)
                uint4 r[2][5];
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const uint32_t p0 = 2u * h * dc.y;
#pragma unroll
                    for (int k = 0; k < 5; k++) {
                        const uint32_t sl = k * 64u + lane - p0;
                        if (sl < 160u) slab[sl] = make_uint4(v[k].x, v[k].y, v[k].z, v[k].w);
                    }
                    __builtin_amdgcn_wave_barrier();
                    asm volatile("" ::: "memory");
                    const uint4* sp = reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(slab) + (lane & 31u) * dc.y);
#pragma unroll
                    for (int k = 0; k < 5; k++) r[h][k] = sp[k];
                    __builtin_amdgcn_wave_barrier();
                    asm volatile("" ::: "memory");
                }
                const bool hi = lane >= 32u;
#pragma unroll
                for (int k = 0; k < 5; k++) {
                    W[0].w[4 * k + 0] = hi ? r[1][k].x : r[0][k].x;
                    W[0].w[4 * k + 1] = hi ? r[1][k].y : r[0][k].y;
                    W[0].w[4 * k + 2] = hi ? r[1][k].z : r[0][k].z;
                    W[0].w[4 * k + 3] = hi ? r[1][k].w : r[0][k].w;
                }
                o1[0] = dc.x + lane * dc.y;
                live[0] = true;  // dense chunks are whole
                pin_win(W[0]);
            } else {
                // the record's first 64 bytes (four 16-byte loads): all the
                // hot parser reads; an 80-byte window straddles one more
                // 64-byte memory segment for 3 in 16 alignments
                o1[0] = osp;
                const uint8_t* p = B.bytes + osp;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    uint4 q;
                    __builtin_memcpy(&q, p + 16 * k, 16);
                    W[0].w[4 * k + 0] = q.x; W[0].w[4 * k + 1] = q.y; W[0].w[4 * k + 2] = q.z; W[0].w[4 * k + 3] = q.w;
                }
                W[0].w[16] = W[0].w[17] = W[0].w[18] = W[0].w[19] = 0u;
                live[0] = lis[0] < end;
                pin_win(W[0]);
            }
            // pinned in each branch: after the merge no wait covers the window
            issue(cn < nch ? cn : c, cn < nch ? dn : make_uint2(0, 0));
            dn_v = desc_of(c2);
            process(W, o1, lis, live);
            c = cn;
            dc = dn;
            cn = c2;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last (unused) issue
        flush();
    }
    // sets of windows this workgroup did not have: empty segments
    for (uint32_t w = win; w < a.S.W; w++) {
        const uint32_t set = blockIdx.x * a.S.W + w;
        for (uint32_t oo = tid; oo <= a.S.O; oo += BLOCK) {
            a.S.off[(size_t)oo * a.S.n_sets + set] = 0;
            if (oo < a.S.O) a.S.soff[(size_t)oo * a.S.n_sets + set] = 0;
        }
    }
    // statistics: one record per workgroup (plain stores), summed by k_merge_partials
    if ((tid & 63) == 0 && d_loops && a.dbg) {
        atomicAdd(&s_cnt[3], (unsigned long long)d_loops);
        atomicAdd(&s_cnt[4], (unsigned long long)d_iters);
    }
    // wave reductions (shuffles), then one LDS atomic per wave and counter (a
    // 64-bit LDS atomic from every lane compiles to a 64-step lane loop)
    {
        uint32_t cv = (uint32_t)c_valid, cd = (uint32_t)c_drop, cm = (uint32_t)c_miss;
        unsigned long long tn = tmin, tx = tmax;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            cv += __shfl_xor(cv, o, 64);
            cd += __shfl_xor(cd, o, 64);
            cm += __shfl_xor(cm, o, 64);
            tn = min(tn, (unsigned long long)__shfl_xor(tn, o, 64));
            tx = max(tx, (unsigned long long)__shfl_xor(tx, o, 64));
        }
        if ((tid & 63) == 0) {
            if (cv) atomicAdd(&s_cnt[0], (unsigned long long)cv);
            if (cd) atomicAdd(&s_cnt[1], (unsigned long long)cd);
            if (cm) atomicAdd(&s_cnt[2], (unsigned long long)cm);
            if (cv) { atomicMin(&s_tmin, tn); atomicMax(&s_tmax, tx); }
        }
    }
    lds_barrier();  // LDS only: the flush's stores need not have completed here
    if (tid == 0) {
        unsigned long long* st = a.S.wgs + (size_t)blockIdx.x * WGS_N;
        st[0] = s_cnt[0];
        st[1] = s_cnt[1];
        st[2] = s_cnt[2];
        st[3] = s_cnt[0] ? s_tmin : NONE64;
        st[4] = s_cnt[0] ? s_tmax : 0;
        st[5] = clock64() - cyc_start;
        st[6] = cyc_flush;
        st[7] = cyc_wait;
        a.slow_cnt[blockIdx.x] = s_slow;
        if (s_slow) atomicAdd(a.slow_n, (unsigned long long)s_slow);
        // spills in owner segments: every LDS-table miss but the overflow
        if (s_cnt[2] > ovf_total) atomicAdd(&a.g->n_dspill, s_cnt[2] - ovf_total);
        if (a.dbg) {
            const unsigned long long rt_end = wall_clock64();
            a.dbg[blockIdx.x * 8 + 0] = rt_start;
            a.dbg[blockIdx.x * 8 + 3] = rt_end;
            a.dbg[blockIdx.x * 8 + 7] = s_cnt[3] | (s_cnt[4] << 32);  // probe loops | iterations
        }
    }
}

// ---------------------------------------------------------------------------
// k_parse_spill: the hot pass for captures with many flows per window (the
// last run sent more than half of its packets past k_parse_agg's LDS table:
// C3/C4-like IMIX with 100k-1M flows).  No key table: every valid packet
// becomes a 32-byte record for its merge owner, staged in an LDS bin per
// owner (O x BIN records, 128 KiB); a full bin leaves as one contiguous run
// of its owner's segment, written cooperatively by the wave that completed
// it (2*BIN lanes per bin: 16-byte pieces, whole lines per instruction).
// k_parse_agg's scattered per-packet 32-byte stores into the owner segments
// were ~90 us of C3's 0.44-ms kernel (ablation: the same stores coalesced).
// The merge, the segments and the sets are k_parse_agg's (no partials).
// ---------------------------------------------------------------------------
constexpr int SPB_WORDS = 8192;  // LDS bins: 16-byte words (128 KiB), 2 per record
__device__ __forceinline__ uint32_t own_add_n(uint32_t* arr, uint32_t o, uint32_t n) {
    return (atomicAdd(&arr[o >> 1], n << ((o & 1) * 16)) >> ((o & 1) * 16)) & 0xFFFFu;
}

// MACS (-M): the canonical MAC pair joins the key; a record is four 16-byte
// words -- key, MAC words + hash, payload, zero (k_parse_agg<MACS>'s spills)
template <bool MACS>
__global__ void __launch_bounds__(BLOCK) k_parse_spill(AggArgs a) {
    constexpr uint32_t RU = MACS ? 4u : 2u;  // 16-byte words per record
    __shared__ uint4 s_bin[SPB_WORDS];
    __shared__ uint32_t s_cl[MAX_OWNERS], s_wr[MAX_OWNERS];  // per bin: slots claimed / records written
    __shared__ uint32_t s_scnt[OWN_WORDS];                   // per owner: records in its segment (packed)
    __shared__ uint32_t s_chunk, s_nspill, s_slow;
    __shared__ unsigned long long s_sbase, s_cnt[3], s_tmin, s_tmax;
    const int tid = threadIdx.x;
    const Stage& S = a.S;
    const Batch& B = a.B;
    const uint32_t O = S.O;
    const uint32_t BIN = (uint32_t)(SPB_WORDS / RU) / O;  // records per bin: 16 (256 owners) .. 2 (2048); MACS: 8 .. 1
    const uint32_t PPB = RU * BIN;                         // 16-byte pieces per bin
    for (uint32_t o = tid; o < MAX_OWNERS; o += BLOCK) s_cl[o] = s_wr[o] = 0;
    for (uint32_t o = tid; o < OWN_WORDS; o += BLOCK) s_scnt[o] = 0;
    if (tid < 3) s_cnt[tid] = 0;
    if (tid == 0) { s_tmin = NONE64; s_tmax = 0; s_chunk = 0; s_nspill = 0; s_slow = 0; }
    __syncthreads();
    const uint64_t n = B.n, G = gridDim.x, stride = G * BLOCK, beg = (uint64_t)blockIdx.x * BLOCK;
    const uint64_t nsteps = n > beg ? (n - beg + stride - 1) / stride : 0;
    const uint64_t lastp = n - 1;
    const uint32_t lane = tid & 63;
    constexpr uint32_t WAVES = BLOCK / 64;
    unsigned long long c_valid = 0, c_drop = 0, tmin = NONE64, tmax = 0;
    uint64_t wbase = beg;
    uint32_t win = 0, ovf_total = 0;
    const unsigned long long rt_start = wall_clock64();
    // a lane's overflow record (its owner segment is full): the workgroup's
    // raw buffer, listed at the window flush (k_parse_agg's overflow list)
    auto overflow = [&](uint32_t q, uint32_t h, uint4 v) {
        uint4* dst = reinterpret_cast<uint4*>(S.spill_raw) + (size_t)blockIdx.x * SPILL_WG * RU + (size_t)h * SPILL_WG + q;
        *dst = v;
    };
    for (uint64_t ws = 0; ws < nsteps; ws += WIN_ITERS) {
        const uint32_t set = blockIdx.x * S.W + win;
        const uint32_t nch = (uint32_t)min<uint64_t>(WIN_ITERS, nsteps - ws) * WAVES;
        uint4* seg0 = reinterpret_cast<uint4*>(S.dspill) + (size_t)set * O * S.cap_o * RU;
        auto li_of = [&](uint32_t c) -> uint64_t {
            return beg + (ws + c / WAVES) * stride + (uint64_t)(c % WAVES) * 64 + lane;
        };
        // the record offset of this lane's packet of chunk c (dense chunks: computed)
        auto off_of = [&](uint32_t c) -> uint32_t {
            const uint64_t li = min(li_of(c), lastp);
            const uint64_t ch = (li_of(c) - lane) >> 6;
            uint2 d = make_uint2(0, 0);
            if (ch < B.n_desc) d = B.desc[ch];
            return d.y ? d.x + lane * d.y : B.offs[li];
        };
        uint32_t c = 0;
        if (lane == 0) c = atomicAdd(&s_chunk, 1u);
        c = __builtin_amdgcn_readfirstlane(c);
        uint32_t off = c < nch ? off_of(c) : 0u;
        while (c < nch) {
            uint32_t cn = 0;
            if (lane == 0) cn = atomicAdd(&s_chunk, 1u);
            cn = __builtin_amdgcn_readfirstlane(cn);
            const uint64_t li = li_of(c);
            const bool live = li < n;
            Win W;
            {
                const uint8_t* p = B.bytes + off;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    uint4 q;
                    __builtin_memcpy(&q, p + 16 * k, 16);
                    W.w[4 * k + 0] = q.x; W.w[4 * k + 1] = q.y; W.w[4 * k + 2] = q.z; W.w[4 * k + 3] = q.w;
                }
                W.w[16] = W.w[17] = W.w[18] = W.w[19] = 0u;
            }
            const uint32_t off_n = cn < nch ? off_of(cn) : 0u;  // the next chunk's offset, in flight
            pin_win(W);
            Hot h;
            const uint32_t cls = live ? hot_parse(B, off, W, h) : HOT_DROP;
            c_drop += (live & (cls == HOT_DROP)) ? 1 : 0;
            const bool valid = live & (cls == HOT_OK);
            const bool slow = live & (cls == HOT_SLOW);
            // canonical key (lower endpoint first, flow_table.h; MACS: the MAC breaks a tie)
            const uint32_t sp = h.ports >> 16, dp = h.ports & 0xFFFFu;
            bool gt = (h.sip > h.dip) | ((h.sip == h.dip) & (sp > dp));
            uint32_t m0 = 0, m1 = 0, m2 = 0;
            if (MACS) {
                const uint64_t dmac = ((uint64_t)__builtin_amdgcn_perm(W.w[5], W.w[4], 0x00010203u) << 16) |
                                      __builtin_amdgcn_perm(W.w[5], W.w[4], 0x0C0C0405u);  // frame bytes 0..5
                const uint64_t smac = ((uint64_t)__builtin_amdgcn_perm(W.w[6], W.w[5], 0x02030405u) << 16) |
                                      __builtin_amdgcn_perm(W.w[6], W.w[5], 0x0C0C0607u);  // frame bytes 6..11
                if ((h.sip == h.dip) & (sp == dp)) gt = smac > dmac;
                const uint64_t lom = gt ? dmac : smac, him = gt ? smac : dmac;
                m0 = (uint32_t)(lom >> 16);
                m1 = ((uint32_t)(lom & 0xFFFF) << 16) | (uint32_t)(him & 0xFFFF);
                m2 = (uint32_t)(him >> 16);
            }
            const uint4 w_key = make_uint4(gt ? h.dip : h.sip, gt ? h.sip : h.dip,
                                           gt ? __builtin_amdgcn_alignbit(h.ports, h.ports, 16) : h.ports, h.proto << 24);
            const bool elig = (h.proto != 6u) | ((h.tf & 2u) != 0);
            const uint4 w_pay = make_uint4(h.doct, h.pkt | (h.ttl << 16) | ((elig ? 1u : 0u) << 24), (uint32_t)(li - wbase),
                                           h.tf | ((gt ? 1u : 0u) << 8));
            uint32_t hk = lt_hash(w_key.x, w_key.y, w_key.z, w_key.w);
            if (MACS) hk = mac_hash(hk, m0, m1, m2);
            const uint4 w_mac = make_uint4(m0, m1, m2, hk);
            const uint32_t o = owner_of(hk, O);
            if (!MACS && a.phash && live) a.phash[li] = valid ? ckey_bucket_v4(w_key.x, w_key.y, w_key.z, h.proto) : PH_PARSE;
            if (valid) {
                c_valid++;
                tmin = min(tmin, (unsigned long long)h.t);
                tmax = max(tmax, (unsigned long long)h.t);
            }
            // claim a bin slot, write the record, count it written; a lane whose
            // bin is full retries once the bin's completer has flushed it
            bool pend = valid;
            for (int it = 0; it < (1 << 16); it++) {
                if (__ballot(pend) == 0) break;
                uint32_t done = NONE32;
                if (pend) {
                    const uint32_t slot = atomicAdd(&s_cl[o], 1u);
                    if (slot < BIN) {
                        uint4* b = &s_bin[(o * BIN + slot) * RU];
                        b[0] = w_key;
                        if (MACS) {
                            b[1] = w_mac;
                            b[2] = w_pay;
                            b[3] = make_uint4(0, 0, 0, 0);
                        } else {
                            b[1] = w_pay;
                        }
                        __threadfence_block();
                        if (atomicAdd(&s_wr[o], 1u) + 1 == BIN) done = o;
                        pend = false;
                    }
                }
                // the bins completed this round: their segment positions, then
                // the wave writes them out, 2*BIN lanes per bin
                uint32_t pos = 0;
                if (done != NONE32) pos = own_add_n(s_scnt, done, BIN);
                uint64_t fm = __ballot(done != NONE32);
                while (fm) {
                    const uint32_t j = lane / PPB, pc = lane % PPB;  // this lane: piece pc of the j-th bin of the group
                    uint64_t m = fm;
                    for (uint32_t k = 0; k < j && m; k++) m &= m - 1;
                    const bool act = m != 0 && j < 64 / PPB;  // (64 % PPB != 0: the spare lanes idle)
                    const uint32_t src = act ? (uint32_t)__builtin_ctzll(m) : 0u;
                    const uint32_t bo = __shfl(done, src, 64), bp = __shfl(pos, src, 64);
                    const uint32_t r = pc / RU, hh = pc % RU;
                    const bool ovf = act && bp + r >= S.cap_o;
                    uint32_t q = 0;  // (the overflow slot: from the record's first lane, every lane shuffling)
                    if (ovf && hh == 0) q = atomicAdd(&s_nspill, 1u);
                    q = __shfl(q, lane & ~(RU - 1), 64);
                    if (act) {
                        const uint4 v = s_bin[(bo * BIN + r) * RU + hh];
                        if (!ovf) seg0[((size_t)bo * S.cap_o + bp + r) * RU + hh] = v;
                        else overflow(q, hh, v);  // past the segment's capacity: the overflow list
                    }
                    // drop the group's bins (the first 64 / PPB set bits)
                    for (uint32_t k = 0; k < 64 / PPB && fm; k++) fm &= fm - 1;
                }
                if (done != NONE32) {  // (the wave's reads of the bin come first: LDS order)
                    atomicExch(&s_wr[done], 0u);
                    atomicExch(&s_cl[done], 0u);
                }
                if (__ballot(pend)) __builtin_amdgcn_s_sleep(1);
            }
            if (pend) atomicOr(a.T.err, ERR_SPIN);  // (cannot happen: a full bin's completer flushes it)
            // slow list: wave-aggregated append into this workgroup's region
            const uint64_t sm = __ballot(slow);
            if (sm) {
                const uint32_t lead = __builtin_ctzll(sm);
                uint32_t b0 = 0;
                if (lane == lead) b0 = atomicAdd(&s_slow, (uint32_t)__popcll(sm));
                b0 = __shfl(b0, lead, 64);
                if (slow)
                    a.slow[(size_t)blockIdx.x * a.slow_region + b0 +
                           __builtin_amdgcn_mbcnt_hi((uint32_t)(sm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)sm, 0u))] = (uint32_t)li;
            }
            c = cn;
            off = off_n;
        }
        // ---- window flush: the partly filled bins, then the set's segment counts
        __syncthreads();
        for (uint32_t o = tid; o < O; o += BLOCK) {
            const uint32_t k = s_wr[o];
            if (!k) continue;
            const uint32_t p0 = own_add_n(s_scnt, o, k);
            for (uint32_t r = 0; r < k; r++) {
                const uint4* v = &s_bin[(o * BIN + r) * RU];
                if (p0 + r < S.cap_o) {
                    uint4* d = seg0 + ((size_t)o * S.cap_o + p0 + r) * RU;
#pragma unroll
                    for (uint32_t u = 0; u < RU; u++) d[u] = v[u];
                } else {
                    const uint32_t q = atomicAdd(&s_nspill, 1u);
#pragma unroll
                    for (uint32_t u = 0; u < RU; u++) overflow(q, u, v[u]);
                }
            }
            s_cl[o] = s_wr[o] = 0;
        }
        __syncthreads();  // (every overflow record written before the list copy below)
        const uint32_t nsp = s_nspill;
        if (tid == 128) s_sbase = nsp ? atomicAdd(&a.g->n_spill, (unsigned long long)nsp) : 0ull;
        if (tid == 0) { ovf_total += nsp; S.base[set] = B.first + wbase; s_chunk = 0; }
        for (uint32_t o = tid; o <= O; o += BLOCK) {
            S.off[(size_t)o * S.n_sets + set] = 0;  // no partials
            if (o < O) S.soff[(size_t)o * S.n_sets + set] = min(own_get(s_scnt, o), S.cap_o);
        }
        __syncthreads();
        if (nsp) {  // overflow records -> the overflow list (the set in fl's high bits)
            const uint4* raw = reinterpret_cast<const uint4*>(S.spill_raw) + (size_t)blockIdx.x * SPILL_WG * RU;
            const unsigned long long sb = s_sbase;
            constexpr uint32_t PAY = RU == 4 ? 2u : 1u;  // the payload word (its fl field carries the set)
            for (uint32_t i = tid; i < nsp; i += BLOCK) {
                // (written by other waves of this workgroup: nontemporal loads bypass the CU's L1)
                typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
                uint4* dst = reinterpret_cast<uint4*>(S.spill) + (sb + i) * RU;
#pragma unroll
                for (uint32_t u = 0; u < RU; u++) {
                    const u32x4 kk = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(raw + u * SPILL_WG + i));
                    dst[u] = make_uint4(kk.x, kk.y, kk.z, kk.w | (u == PAY ? (set << 9) : 0u));
                }
            }
        }
        for (uint32_t o = tid; o < OWN_WORDS; o += BLOCK) s_scnt[o] = 0;
        if (tid == 0) s_nspill = 0;
        __syncthreads();
        wbase += stride * WIN_ITERS;
        win++;
    }
    // sets of windows this workgroup did not have: empty segments
    for (uint32_t w = win; w < S.W; w++) {
        const uint32_t set = blockIdx.x * S.W + w;
        for (uint32_t oo = tid; oo <= O; oo += BLOCK) {
            S.off[(size_t)oo * S.n_sets + set] = 0;
            if (oo < O) S.soff[(size_t)oo * S.n_sets + set] = 0;
        }
    }
    // statistics (k_parse_agg's per-workgroup record; every valid packet is a "miss")
    {
        uint32_t cv = (uint32_t)c_valid, cd = (uint32_t)c_drop;
        unsigned long long tn = tmin, tx = tmax;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            cv += __shfl_xor(cv, o, 64);
            cd += __shfl_xor(cd, o, 64);
            tn = min(tn, (unsigned long long)__shfl_xor(tn, o, 64));
            tx = max(tx, (unsigned long long)__shfl_xor(tx, o, 64));
        }
        if (lane == 0) {
            if (cv) atomicAdd(&s_cnt[0], (unsigned long long)cv);
            if (cd) atomicAdd(&s_cnt[1], (unsigned long long)cd);
            if (cv) { atomicMin(&s_tmin, tn); atomicMax(&s_tmax, tx); }
        }
    }
    __syncthreads();
    if (tid == 0) {
        unsigned long long* st = S.wgs + (size_t)blockIdx.x * WGS_N;
        st[0] = s_cnt[0];
        st[1] = s_cnt[1];
        st[2] = s_cnt[0];
        st[3] = s_cnt[0] ? s_tmin : NONE64;
        st[4] = s_cnt[0] ? s_tmax : 0;
        st[5] = st[6] = st[7] = 0;
        a.slow_cnt[blockIdx.x] = s_slow;
        if (s_slow) atomicAdd(a.slow_n, (unsigned long long)s_slow);
        if (s_cnt[0] > ovf_total) atomicAdd(&a.g->n_dspill, s_cnt[0] - ovf_total);
        if (a.dbg) {
            a.dbg[blockIdx.x * 8 + 0] = rt_start;
            a.dbg[blockIdx.x * 8 + 1] = a.dbg[blockIdx.x * 8 + 2] = a.dbg[blockIdx.x * 8 + 3] = wall_clock64();
            a.dbg[blockIdx.x * 8 + 7] = 0;
        }
    }
}

// One flow's merged update_flow aggregate -> the global accumulators of dense
// id d (flows.rs:11-42).  Positions are global packet indices.
struct FlowPart {
    uint32_t pk[2];
    unsigned long long by[2];
    uint32_t mn[2], mx[2];
    uint32_t fl[8];
    unsigned long long fa, fc, fr, la;  // NONE64 / 0 when absent (la = last + 1)
};

__device__ __forceinline__ void part_to_global(const Acc& A, uint32_t d, const FlowPart& f) {
#pragma unroll
    for (int q = 0; q < 2; q++) {
        if (f.pk[q]) {
            atomicAdd(&A.pk[q][d], f.pk[q]);
            atomicAdd(&A.by[q][d], f.by[q]);
        }
        if (f.mn[q] < A.mn[q][d]) atomicMin(&A.mn[q][d], f.mn[q]);
        if (f.mx[q] > A.mx[q][d]) atomicMax(&A.mx[q][d], f.mx[q]);
    }
#pragma unroll
    for (int q = 0; q < 8; q++)
        if (f.fl[q]) atomicAdd(&A.fl[q][d], f.fl[q]);
    if (f.fa != NONE64) atomicMin(&A.fa[d], f.fa);
    if (f.fc != NONE64) atomicMin(&A.fc[d], f.fc);
    if (f.fr != NONE64) atomicMin(&A.fr[d], f.fr);
    if (f.la) atomicMax(&A.la[d], f.la - 1);
}

__device__ __forceinline__ void part_of_stage(const Part& p, unsigned long long base, FlowPart& f) {
    f.pk[0] = p.pk & 0xFFFF;
    f.pk[1] = p.pk >> 16;
    f.by[0] = p.by0;
    f.by[1] = p.by1;
    f.mn[0] = p.mn0;
    f.mn[1] = p.mn1;
    f.mx[0] = p.mx0;
    f.mx[1] = p.mx1;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        f.fl[2 * q] = p.fl[q] & 0xFFFF;
        f.fl[2 * q + 1] = p.fl[q] >> 16;
    }
    f.fa = p.pos[0] == NONE32 ? NONE64 : base + p.pos[0];
    f.fc = p.pos[1] == NONE32 ? NONE64 : base + p.pos[1];
    f.fr = p.pos[2] == NONE32 ? NONE64 : base + p.pos[2];
    f.la = p.pos[3] ? base + p.pos[3] : 0;
}

// A spilled packet as a one-packet partial (update_flow of one packet,
// flows.rs:11-42, with positions as global packet indices).
__device__ __forceinline__ void spill_to_part(uint32_t doct, uint32_t pt, uint32_t loc, uint32_t fl,
                                              unsigned long long base, FlowPart& f) {
    const uint32_t dir = (fl >> 8) & 1, tf = fl & 0xFF;
    const uint32_t pkt = pt & 0xFFFF, ttl = (pt >> 16) & 0xFF;
    const unsigned long long gi = base + loc;
    f.pk[0] = dir ? 0 : 1;
    f.pk[1] = dir ? 1 : 0;
    f.by[0] = dir ? 0 : doct;
    f.by[1] = dir ? doct : 0;
    f.mn[0] = f.mx[0] = pkt;
    f.mn[1] = f.mx[1] = ttl;
#pragma unroll
    for (int q = 0; q < 8; q++) f.fl[q] = (tf >> q) & 1;
    f.fa = gi;
    f.fc = ((pt >> 24) & 1) ? gi : NONE64;
    f.fr = (tf & 5) ? gi : NONE64;
    f.la = gi + 1;
}

// One general-parser packet as a one-packet partial (update_flow's
// order-free fields; positions are global packet indices, la = last + 1).
__device__ __forceinline__ void pkt_to_part(const PktInfo& pi, uint8_t dir, unsigned long long gi, FlowPart& f) {
    const uint32_t tf = pi.tflags;
    f.pk[0] = dir ? 0 : 1;
    f.pk[1] = dir ? 1 : 0;
    f.by[0] = dir ? 0 : (unsigned long long)pi.doctets;
    f.by[1] = dir ? (unsigned long long)pi.doctets : 0;
    f.mn[0] = f.mx[0] = pi.rpkt;
    f.mn[1] = f.mx[1] = pi.rttl;
#pragma unroll
    for (int q = 0; q < 8; q++) f.fl[q] = (tf >> q) & 1;
    f.fa = gi;
    f.fc = (pi.rprot != 6 || (tf & 2)) ? gi : NONE64;
    f.fr = (tf & 5) ? gi : NONE64;
    f.la = gi + 1;
}

// The canonical key of an IPv6 5-tuple staged as address ids (V6Map).
__device__ __forceinline__ void v6_ckey(const V6Map& M, uint32_t ia, uint32_t ib, uint32_t ports, uint32_t tag, CKey& k) {
    const uint4 a = M.addr_of[ia], b = M.addr_of[ib];
#pragma unroll
    for (int j = 0; j < 14; j++) k.w[j] = 0;
    k.w[0] = a.x; k.w[1] = a.y; k.w[2] = a.z; k.w[3] = a.w;
    k.w[4] = b.x; k.w[5] = b.y; k.w[6] = b.z; k.w[7] = b.w;
    k.w[8] = ports;
    k.w[9] = (1u << 8) | (tag >> 24);
}

// Dense id of a staged key (flow_table.h dictionary; tag 0xFF: the key is the
// id; tag bit 0: an IPv6 5-tuple as address ids).
__device__ __forceinline__ uint32_t staged_id(const TableSet& T, const V6Map& M, uint32_t k0, uint32_t k1, uint32_t k2,
                                              uint32_t tag, uint32_t* slots) {
    CKey k;
    if (tag & V6_TAG) {
        v6_ckey(M, k0, k1, k2, tag, k);
        return dense_of_key(T, k, true, slots, nullptr);
    }
    if (tag == 0xFF000000u) return k0;
#pragma unroll
    for (int j = 0; j < 14; j++) k.w[j] = 0;
    k.w[0] = k0;
    k.w[4] = k1;
    k.w[8] = k2;
    k.w[9] = tag >> 24;
    return dense_of_key(T, k, true, slots, nullptr);
}

// k_merge_partials: the flow-table merge of the hot kernel's staged partials.
// Flow f belongs to workgroup owner(hash(f)); each owner scans the compact
// hash array (L2-resident), merges its flows' partials in LDS, resolves each
// key ONCE in the dictionary (no key has two inserters, so no claim waits)
// and applies one uncontended atomic update per field.  Partials of flows that
// find no LDS entry merge straight into the global accumulators.
constexpr int MB = 1024;   // merge kernel block
constexpr int MT = 1024;   // merge table entries (120 B each)
constexpr int MCH = 1024;  // sets per scan chunk
#ifndef FLUERE_MERGE_NOPART
#define FLUERE_MERGE_NOPART 0  // diagnostics only (wrong results with partials): the spill path's code alone
#endif
#ifndef FLUERE_MERGE_TAIL
#define FLUERE_MERGE_TAIL 1  // diagnostics only (0: no tail, wrong results): the register cost of the tail
#endif
#ifndef FLUERE_MERGE_ABL
#define FLUERE_MERGE_ABL 0  // diagnostics only (wrong results): 1 records loaded, no table; 2 probe, no updates
#endif
#ifndef FLUERE_MERGE_GUARD
#define FLUERE_MERGE_GUARD 1  // read-before-atomic for min / max / positions (0: unconditional)
#endif

// Exclusive scan of one value per thread over a 1024-thread block; returns
// this thread's prefix, and leaves the block total in scratch[MB / 64].
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* scratch) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    uint32_t incl = v;
#pragma unroll
    for (int dlt = 1; dlt < 64; dlt <<= 1) {
        const uint32_t y = __shfl_up(incl, dlt, 64);
        if (lane >= dlt) incl += y;
    }
    if (lane == 63) scratch[wv] = incl;
    __syncthreads();
    if (tid == 0) {
        uint32_t r = 0;
        for (int w = 0; w < MB / 64; w++) {
            const uint32_t t = scratch[w];
            scratch[w] = r;
            r += t;
        }
        scratch[MB / 64] = r;
    }
    __syncthreads();
    return scratch[wv] + incl - v;
}
// ---------------------------------------------------------------------------
// finalize (certified flows -> records; others -> complex)
// ---------------------------------------------------------------------------
struct FinArgs {
    const Batch* bs;
    int nb;
    TableSet T;
    Acc A;
    Glob* g;
    fluere_record* out;
    uint8_t* complex;
    int macs;
    uint64_t out_cap;
    Ctl* host_ctl;   // non-null: the last workgroup writes the run counters to this pinned host copy,
    uint32_t seq;    // then host_ctl->seq = seq (the host polls it: no copy, no event on the way back)
    unsigned long long timeout_us;  // non-zero: skip the flows when expiries can fire (Mode B redoes every flow)
    uint8_t* cbits = nullptr;       // the exact engine's complex-flow filter (ckey_bucket: a byte per bucket), or null
    uint32_t* defer = nullptr;      // k_finalize: certified flows whose first packet needs the general
                                    // parser (Glob::n_fdefer of them), finalized by k_finalize_gen
};

// A flow's order-free aggregate (the accumulators of one dense id).
struct AccVals {
    unsigned long long fa, fc, fr, la;
    uint32_t pk[2];
    unsigned long long by[2];
    uint32_t mn[2], mx[2], fl[8];
};

__device__ __forceinline__ void load_acc(const Acc& A, uint32_t d, AccVals& v) {
    v.fa = A.fa[d]; v.fc = A.fc[d]; v.fr = A.fr[d]; v.la = A.la[d];
#pragma unroll
    for (int q = 0; q < 2; q++) {
        v.pk[q] = A.pk[q][d];
        v.by[q] = A.by[q][d];
        v.mn[q] = A.mn[q][d];
        v.mx[q] = A.mx[q][d];
    }
#pragma unroll
    for (int q = 0; q < 8; q++) v.fl[q] = A.fl[q][d];
}

// Certified flow d -> its record; false when d has no record here (TCP flow
// without a SYN: dropped; complex: marked for the per-flow state machine;
// GEN false: a first packet the register parser declines is listed for
// k_finalize_gen, whose general parser would cost k_finalize its occupancy).
template <bool GEN>
__device__ __forceinline__ bool finalize_vals(const FinArgs& a, uint32_t d, const AccVals& v, fluere_record& r,
                                              bool& cplx, unsigned long long& cplx_pkts) {
    const unsigned long long fa = v.fa, fc = v.fc, fr = v.fr, la = v.la;
    if (fc == NONE64) return false;  // TCP flow without any SYN: every packet is dropped (:101-113)
    bool certified = fc == fa && (fr == NONE64 || fr == la);
    if (!certified) {
        a.complex[d] = 1;
        if (a.cbits) {
            const uint32_t b = ckey_bucket(reinterpret_cast<const uint32_t*>(a.T.flow_key + (size_t)d * 56));
            a.cbits[b] = 1;
        }
        cplx = true;
        cplx_pkts = v.pk[0] + v.pk[1];
        return false;
    }
    const bool macs = a.macs != 0;
    // the first and the last packet: both offsets, then both windows, in flight together
    const int bp = find_batch(a.bs, a.nb, fc), bq = find_batch(a.bs, a.nb, la);
    const Batch& BP = a.bs[bp];
    const Batch& BQ = a.bs[bq];
    const uint32_t op = BP.offs[fc - BP.first], oq = BQ.offs[la - BQ.first];
    Win WP;
    load_win(BP, op, WP);
    const uint64_t t_last = record_time(BQ, oq);  // the last packet: its time only
    pin_win(WP);
    Parsed P;
    if constexpr (GEN) {
        parse_loaded(BP, op, WP, macs, 0, P);
    } else {
        parse_loaded_fast(BP, op, WP, macs, P);
        if (P.cls == 2) {  // IPv6, VXLAN, IPv4 options: parse_mid over the 128-byte window
            Win32 W32;
            load_win32(BP, op, W32);
            parse_loaded32<0>(BP, op, W32, macs, P);
        }
        if (P.cls == 2) {  // the general parser's classes (ARP, VLAN, raw fallback ...)
            a.defer[atomicAdd(&a.g->n_fdefer, 1ull)] = d;
            return false;
        }
    }
    const uint8_t cd = canon_dir(P, macs);
    fill_seed(r, P);
    const uint32_t p0 = v.pk[0], p1 = v.pk[1];
    const unsigned long long b0 = v.by[0], b1 = v.by[1];
    r.d_pkts = p0 + p1;
    r.d_octets = b0 + b1;
    r.out_pkts = cd ? p1 : p0; r.in_pkts = cd ? p0 : p1;
    r.out_bytes = cd ? b1 : b0; r.in_bytes = cd ? b0 : b1;
    r.min_pkt = v.mn[0]; r.max_pkt = v.mx[0];
    r.min_ttl = (uint8_t)v.mn[1]; r.max_ttl = (uint8_t)v.mx[1];
    for (int q = 0; q < 8; q++) r.cnt[q] = v.fl[q];
    r.cnt[8] = 0;
    r.last = t_last;
    r.order_key = (fr == la) ? la : NONE64;
    return true;
}

template <bool GEN>
__device__ __forceinline__ bool finalize_one(const FinArgs& a, uint32_t d, fluere_record& r, bool& cplx,
                                             unsigned long long& cplx_pkts) {
    AccVals v;
    load_acc(a.A, d, v);
    return finalize_vals<GEN>(a, d, v, r, cplx, cplx_pkts);
}

// emit + complex-flow counters of one wave's flows (every lane of the wave)
__device__ __forceinline__ void finalize_emit(EmitLds& S, const FinArgs& a, const fluere_record& r, bool want, bool cplx,
                                              unsigned long long cplx_pkts) {
    emit_record_block(S, a.g, a.out, a.out_cap, r, want);
    const uint64_t cm = __ballot(cplx);
    if (cm) {
        const unsigned long long pk = wave_sum(cplx_pkts);
        if ((uint32_t)(threadIdx.x & 63) == (uint32_t)__builtin_ctzll(cm)) {
            atomicAdd(&a.g->n_complex, (unsigned long long)__popcll(cm));
            atomicAdd(&a.g->n_complex_pkts, pk);
        }
    }
}

// (MACS: a run with MAC keys -- the entries' MAC sidecars; a kernel of its own
// so the 5-tuple runs keep 16 KiB of LDS and none of the MAC paths' code)
template <bool MACS>
__global__ void __launch_bounds__(MB) k_merge_partials(AggArgs a) {
    __shared__ uint4 m_key[MT];
    __shared__ uint4 m_kx[MACS ? MT : 1];  // MAC runs: the MAC sidecar of each entry (w = 1 once written)
    __shared__ uint32_t m_pk[2][MT], m_mn[2][MT], m_mx[2][MT], m_fl[8][MT];
    __shared__ unsigned long long m_by[2][MT], m_fa[MT], m_fc[MT], m_fr[MT], m_la[MT];
    __shared__ uint32_t m_nclaim, m_base;
    // per set of the current chunk: this owner's first record (index into the
    // partials or the spill planes), its start in the flattened index space,
    // and the window's first packet (relative to the batch): a record's
    // loads then depend on LDS reads only
    __shared__ uint32_t m_lo[MCH], m_start[MCH], m_wb[MCH], m_scan[MB / 64 + 1];
    // per group of 64 flattened indices: the set holding its first index (the
    // spill records' wave-uniform search, one LDS read instead of a binary search)
    constexpr uint32_t MGRP = 2048;
    __shared__ uint16_t m_grp[MGRP];
    const int tid = threadIdx.x;
    const unsigned long long c0 = clock64();
    if (a.dbg && tid == 0) a.dbg[4096 * 8 - 2048 + blockIdx.x * 8 + 0] = wall_clock64();
    // loads issued before the LDS initialisation (their latency overlaps it):
    // this owner's segment bounds of the first set chunk, and the run counters
    const unsigned long long n_spill_all = __hip_atomic_load(&a.g->n_spill, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long n_dspill_all = __hip_atomic_load(&a.g->n_dspill, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long n_slow_all = __hip_atomic_load(a.slow_n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    constexpr bool macs = MACS;
    const Stage& S = a.S;
    auto reduce_stats = [&]() {
        // the hot kernel's per-workgroup statistics -> the run counters (one wave)
        unsigned long long v[WGS_N] = {0, 0, 0, NONE64, 0, 0, 0, 0};
        for (uint32_t w = tid; w < S.n_wg; w += 64) {
            const unsigned long long* st = S.wgs + (size_t)w * WGS_N;
#pragma unroll
            for (int k = 0; k < WGS_N; k++) v[k] = k == 3 ? min(v[k], st[k]) : k == 4 ? max(v[k], st[k]) : v[k] + st[k];
        }
#pragma unroll
        for (int k = 0; k < WGS_N; k++)
            for (int d = 32; d >= 1; d >>= 1) {
                const unsigned long long o = __shfl_xor(v[k], d, 64);
                v[k] = k == 3 ? min(v[k], o) : k == 4 ? max(v[k], o) : v[k] + o;
            }
        if (tid == 0) {
            Glob* g = a.g;
            if (v[0]) atomicAdd(&g->valid, v[0]);
            if (v[1]) atomicAdd(&g->dropped, v[1]);
            if (v[2]) atomicAdd(&g->n_kc_miss, v[2]);
            if (v[0]) { atomicMin(&g->tmin, v[3]); atomicMax(&g->tmax, v[4]); }
            atomicAdd(&g->cyc_total, v[5]);
            atomicAdd(&g->cyc_flush, v[6]);
            atomicAdd(&g->cyc_flush0, v[7]);
        }
    };
    // Owners o = blockIdx.x, + gridDim.x, ...: the grid is at most one workgroup
    // per CU (one merge table fills a CU's LDS), so a workgroup merges several
    // owners in turn rather than being dispatched again for each.
    // Owner blockIdx.x first; with more owners than workgroups the rest are
    // claimed from a counter (Glob::n_owner), so a workgroup that finishes
    // early takes the next one (owners' record phases spread, e.g. C3 99-199
    // us).  No counter when every workgroup has one owner.
    __shared__ uint32_t s_me;
    if (tid == 0) s_me = blockIdx.x;
    __syncthreads();
    const int pass0 = S.no_parts ? 1 : 0;  // (no partials: the segments' pass alone)
    for (uint32_t me = s_me; me < S.O; me = s_me) {
        // the first chunk's bounds, loaded before the LDS initialisation
        // (partials: their offsets; no partials: the segments' counts)
        uint32_t pre_lo[MCH / MB], pre_hi[MCH / MB];
        unsigned long long pre_wb[MCH / MB];
    #pragma unroll
        for (int q = 0; q < MCH / MB; q++) {
            const uint32_t set = tid * (MCH / MB) + q;
            const bool in = set < a.S.n_sets;
            pre_lo[q] = in && !pass0 ? a.S.off[(size_t)me * a.S.n_sets + set] : 0;
            pre_hi[q] = !in ? 0 : pass0 ? a.S.soff[(size_t)me * a.S.n_sets + set] : a.S.off[(size_t)(me + 1) * a.S.n_sets + set];
            pre_wb[q] = in ? a.S.base[set] : 0;
        }
        for (int e = tid; e < MT; e += MB) {
            m_key[e] = make_uint4(0, 0, 0, 0);
            if (MACS) m_kx[e] = make_uint4(0, 0, 0, 0);
            m_pk[0][e] = m_pk[1][e] = 0;
            m_by[0][e] = m_by[1][e] = 0;
            m_mn[0][e] = m_mn[1][e] = NONE32;
            m_mx[0][e] = m_mx[1][e] = 0;
    #pragma unroll
            for (int q = 0; q < 8; q++) m_fl[q][e] = 0;
            m_fa[e] = m_fc[e] = m_fr[e] = NONE64;
            m_la[e] = 0;
        }
        __syncthreads();
        if (a.dbg && tid == 0) a.dbg[4096 * 8 - 2048 + blockIdx.x * 8 + 1] = wall_clock64();
        // This owner's segment of every set, flattened: per chunk of MCH sets, an
        // exclusive scan of the segment lengths; threads then take partials from
        // the flattened index space (binary search for the set), so every thread
        // has about (partials / MB) of them with all their loads in flight.
        // Pass 0 takes the staged partials, pass 1 the spilled packets in this
        // owner's segments (each a one-packet partial), through the same
        // machinery; the overflow list is the tail's.
        const int passes = n_dspill_all ? 2 : 1;  // no spills: one pass
        for (int pass = FLUERE_MERGE_NOPART ? 1 : pass0; pass < passes; pass++)
        for (uint32_t c0s = 0; c0s < S.n_sets; c0s += MCH) {
            const uint32_t nset = min((uint32_t)MCH, S.n_sets - c0s);
            const uint32_t* offs = pass ? S.soff : S.off;
            uint32_t len[MCH / MB], tot = 0;
    #pragma unroll
            for (int q = 0; q < MCH / MB; q++) {
                const uint32_t set = c0s + tid * (MCH / MB) + q;
                uint32_t lo = 0, hi = 0;
                unsigned long long wb = 0, rb = 0;
                if (pass == pass0 && c0s == 0) {  // prefetched
                    lo = pre_lo[q];
                    hi = pre_hi[q];
                    wb = pre_wb[q];
                } else if (set < c0s + nset) {
                    lo = pass ? 0u : offs[(size_t)me * S.n_sets + set];
                    hi = offs[(size_t)(pass ? me : me + 1) * S.n_sets + set];  // pass 1: the segment's count
                    wb = S.base[set];
                }
                rb = !pass ? (unsigned long long)set * NS
                     : set < S.n_hot ? ((unsigned long long)set * S.O + me) * S.cap_o
                                     : S.slow_rec0 + ((unsigned long long)(set - S.n_hot) * S.O + me) * S.cap_s;
                m_lo[tid * (MCH / MB) + q] = (uint32_t)(rb + lo);
                m_wb[tid * (MCH / MB) + q] = (uint32_t)(wb - a.B.first);
                len[q] = hi - lo;
                tot += len[q];
            }
            uint32_t run = block_exclusive_scan(tot, m_scan) ;
            const uint32_t total = m_scan[MB / 64];  // (block_exclusive_scan ends with a barrier)
            const bool grp = pass == 1 && total <= 64u * MGRP;
    #pragma unroll
            for (int q = 0; q < MCH / MB; q++) {
                m_start[tid * (MCH / MB) + q] = run;
                if (grp && len[q])
                    for (uint32_t g = (run + 63) >> 6; g <= (run + len[q] - 1) >> 6; g++)
                        m_grp[g] = (uint16_t)(tid * (MCH / MB) + q);
                run += len[q];
            }
            __syncthreads();
            if (a.dbg && tid == 0 && c0s == 0 && pass == 0) a.dbg[4096 * 8 - 2048 + blockIdx.x * 8 + 2] = wall_clock64();
            // one record (a staged partial or a spilled packet): find or claim
            // its merge entry, then the update (or the global path)
            auto merge_rec = [&](uint32_t h, uint32_t k0, uint32_t k1, uint32_t k2, uint32_t tag, uint32_t x0,
                                 uint32_t x1, uint32_t x2, const FlowPart& f) {
                    // find or claim the merge entry (same protocol as the hot kernel)
                    uint32_t e = (h * 0x85EBCA77u) >> 22;  // 10 bits: MT == 1024
                    int state = 0, probes = 0;
                    for (int it = 0; it < 128; it++) {
                        if (state == 0) {
                            const uint4 kk = m_key[e];
                            bool xm = true;
                            if (macs) {  // MAC words
                                const uint4 xx = m_kx[MACS ? e : 0];
                                xm = xx.w == 1u && xx.x == x0 && xx.y == x1 && xx.z == x2;
                            }
                            if (kk.w & LT_READY) {
                                if (kk.w == (tag | LT_READY) && kk.x == k0 && kk.y == k1 && kk.z == k2 && xm) state = 1;
                                else if (++probes == 64) state = 2;
                                else e = (e + 1) & (MT - 1);
                            } else if (kk.w == 0 && atomicCAS(&m_key[e].w, 0u, LT_CLAIM) == 0u) {
                                m_key[e].x = k0;
                                m_key[e].y = k1;
                                m_key[e].z = k2;
                                if (MACS) m_kx[e] = make_uint4(x0, x1, x2, 1u);
                                __threadfence_block();
                                atomicExch(&m_key[e].w, tag | LT_READY);
                                state = 1;
                            }
                        }
                        if (__ballot(state == 0) == 0) break;
                    }
                    if (state == 1) {
                        // Many records land on one entry (a flow's partials from every
                        // set, its spilled packets), and LDS atomics on one address
                        // serialise: min / max and first / last positions are read
                        // first and written only where the record moves them (values
                        // move monotonically, so a stale read costs at most a
                        // redundant atomic).
    #if FLUERE_MERGE_GUARD
                        const uint32_t gmn0 = m_mn[0][e], gmn1 = m_mn[1][e], gmx0 = m_mx[0][e], gmx1 = m_mx[1][e];
                        const unsigned long long gfa = m_fa[e], gfc = m_fc[e], gla = m_la[e];
    #else
                        const uint32_t gmn0 = NONE32, gmn1 = NONE32, gmx0 = 0, gmx1 = 0;
                        const unsigned long long gfa = NONE64, gfc = NONE64, gla = 0;
    #endif
    #pragma unroll
                        for (int q = 0; q < 2; q++) {
                            if (f.pk[q]) {
                                atomicAdd(&m_pk[q][e], f.pk[q]);
                                atomicAdd(&m_by[q][e], f.by[q]);
                            }
                            if (f.mn[q] < (q ? gmn1 : gmn0) || !FLUERE_MERGE_GUARD) atomicMin(&m_mn[q][e], f.mn[q]);
                            if (f.mx[q] > (q ? gmx1 : gmx0) || !FLUERE_MERGE_GUARD) atomicMax(&m_mx[q][e], f.mx[q]);
                        }
    #pragma unroll
                        for (int q = 0; q < 8; q++)
                            if (f.fl[q]) atomicAdd(&m_fl[q][e], f.fl[q]);
                        if (f.fa != NONE64 && f.fa < gfa) atomicMin(&m_fa[e], f.fa);
                        if (f.fc != NONE64 && f.fc < gfc) atomicMin(&m_fc[e], f.fc);
                        if (f.fr != NONE64) atomicMin(&m_fr[e], f.fr);
                        if (f.la && (f.la > gla || !FLUERE_MERGE_GUARD)) atomicMax(&m_la[e], f.la);
                    } else {
                        uint32_t d;
                        if (macs && tag != 0xFF000000u) {
                            CKey ck;
                            mac_ckey(k0, k1, k2, tag, x0, x1, x2, ck);
                            d = dense_of_key(a.T, ck, true, a.A.slots, nullptr);
                        } else {
                            d = staged_id(a.T, a.v6, k0, k1, k2, tag, a.A.slots);
                        }
                        if (d != FAIL && d < a.T.fmax) part_to_global(a.A, d, f);
                    }
            };
            if (pass == 1) {
                // Spilled packets, the lean path (MAC runs: 64-byte records,
                // the MAC words and the hash beside the key): the merge is
                // instruction-bound (PMC on C3: 28 % of wave time issuing at
                // 4 waves per SIMD, 14k VALU + 7k SALU instructions per wave),
                // so no binary search per record (the wave's first index is
                // searched once, each lane steps forward over the few sets
                // its index is past) and update_flow of one packet written
                // out directly instead of through a FlowPart.
                // the set of flattened index id (the wave's smallest index
                // searched once, each lane stepping forward past the few sets
                // its index is beyond)
                auto set_of = [&](uint32_t id) -> uint32_t {
                    const uint32_t iw = __builtin_amdgcn_readfirstlane(id);
                    uint32_t lo_i = 0, hi_i = nset - 1;
                    if (grp) {
                        lo_i = m_grp[iw >> 6];  // (the set of the group's first index: a lower bound)
                    } else {
                        while (lo_i < hi_i) {
                            const uint32_t mid = (lo_i + hi_i + 1) >> 1;
                            if (m_start[mid] <= iw) lo_i = mid;
                            else hi_i = mid - 1;
                        }
                    }
                    while (lo_i + 1 < nset && m_start[lo_i + 1] <= id) lo_i++;
                    return lo_i;
                };
                // one record ahead: the next iteration's record is loaded
                // while this one is probed and aggregated in LDS
                constexpr uint32_t RW = MACS ? 4u : 2u;  // 16-byte words per record
                uint32_t lo_n = 0;
                uint4 n0 = make_uint4(0, 0, 0, 0), n1 = n0, nx = n0;
                if ((uint32_t)tid < total) {
                    lo_n = set_of(tid);
                    const uint4* src = reinterpret_cast<const uint4*>(S.dspill) +
                                       ((size_t)m_lo[lo_n] + ((uint32_t)tid - m_start[lo_n])) * RW;
                    n0 = src[0];
                    n1 = src[MACS ? 2 : 1];
                    if (MACS) nx = src[1];
                }
                for (uint32_t idx = tid; idx < total; idx += MB) {
                    const uint32_t lo_i = lo_n;
                    const uint4 v0 = n0, v1 = n1, vx = nx;  // key, payload, (MACS) MAC words + hash
                    if (idx + MB < total) {
                        lo_n = set_of(idx + MB);
                        const uint4* src = reinterpret_cast<const uint4*>(S.dspill) +
                                           ((size_t)m_lo[lo_n] + (idx + MB - m_start[lo_n])) * RW;
                        n0 = src[0];
                        n1 = src[MACS ? 2 : 1];
                        if (MACS) nx = src[1];
                    }
                    const unsigned long long gi = a.B.first + m_wb[lo_i] + v1.z;
                    const uint32_t k0 = v0.x, k1 = v0.y, k2 = v0.z, tag = v0.w;
                    if (FLUERE_MERGE_ABL == 1) {  // diagnostics: the loads alone
                        if ((k0 ^ k1 ^ k2 ^ v1.x ^ v1.y) == 0x12345678u) atomicAdd(&m_pk[0][0], 1u);
                        continue;
                    }
                    const uint32_t h = MACS ? vx.w : lt_hash(k0, k1, k2, tag);
                    uint32_t e = (h * 0x85EBCA77u) >> 22;  // 10 bits: MT == 1024
                    int state = 0, probes = 0;
                    for (int it = 0; it < 128; it++) {  // find or claim (the hot kernel's protocol)
                        if (state == 0) {
                            const uint4 kk = m_key[e];
                            bool xm = true;
                            if (MACS) {  // the MAC words (the sidecar is written before the entry is published)
                                const uint4 xx = m_kx[MACS ? e : 0];
                                xm = xx.w == 1u && xx.x == vx.x && xx.y == vx.y && xx.z == vx.z;
                            }
                            if (kk.w & LT_READY) {
                                if (kk.w == (tag | LT_READY) && kk.x == k0 && kk.y == k1 && kk.z == k2 && xm) state = 1;
                                else if (++probes == 64) state = 2;
                                else e = (e + 1) & (MT - 1);
                            } else if (kk.w == 0 && atomicCAS(&m_key[e].w, 0u, LT_CLAIM) == 0u) {
                                m_key[e].x = k0;
                                m_key[e].y = k1;
                                m_key[e].z = k2;
                                if (MACS) m_kx[MACS ? e : 0] = make_uint4(vx.x, vx.y, vx.z, 1u);
                                __threadfence_block();
                                atomicExch(&m_key[e].w, tag | LT_READY);
                                state = 1;
                            }
                        }
                        if (__ballot(state == 0) == 0) break;
                    }
                    const uint32_t dir = (v1.w >> 8) & 1u, tf = v1.w & 0xFFu;
                    const uint32_t pkt = v1.y & 0xFFFFu, ttl = (v1.y >> 16) & 0xFFu;
                    if (FLUERE_MERGE_ABL == 2) {  // diagnostics: the probe, no updates
                        if (state == 1 && pkt == 0x1234u) atomicAdd(&m_pk[0][e], 1u);
                        continue;
                    }
                    if (a.pid && state == 1) a.pid[gi - a.pid_base] = PH_EREF | (a.pid_batch << 21) | (me << 10) | e;
                    if (state == 1) {  // update_flow of one packet (flows.rs:11-42), order-free part
                        atomicAdd(&m_pk[dir][e], 1u);
                        atomicAdd(&m_by[dir][e], (unsigned long long)v1.x);
                        const uint32_t gmn0 = m_mn[0][e], gmn1 = m_mn[1][e], gmx0 = m_mx[0][e], gmx1 = m_mx[1][e];
                        const unsigned long long gfa = m_fa[e], gfc = m_fc[e], gla = m_la[e];
                        if (pkt < gmn0) atomicMin(&m_mn[0][e], pkt);
                        if (ttl < gmn1) atomicMin(&m_mn[1][e], ttl);
                        if (pkt > gmx0) atomicMax(&m_mx[0][e], pkt);
                        if (ttl > gmx1) atomicMax(&m_mx[1][e], ttl);
                        for (uint32_t t = tf; t; t &= t - 1) atomicAdd(&m_fl[__builtin_ctz(t)][e], 1u);
                        if (gi < gfa) atomicMin(&m_fa[e], gi);
                        if (((v1.y >> 24) & 1u) && gi < gfc) atomicMin(&m_fc[e], gi);
                        if (tf & 5u) atomicMin(&m_fr[e], gi);
                        if (gi + 1 > gla) atomicMax(&m_la[e], gi + 1);
                    } else {  // no entry within 64 probes: the global path
                        FlowPart f;
                        spill_to_part(v1.x, v1.y, v1.z, v1.w, a.B.first + m_wb[lo_i], f);
                        uint32_t d;
                        if (MACS && tag != 0xFF000000u) {
                            CKey ck;
                            mac_ckey(k0, k1, k2, tag, vx.x, vx.y, vx.z, ck);
                            d = dense_of_key(a.T, ck, true, a.A.slots, nullptr);
                        } else {
                            d = staged_id(a.T, a.v6, k0, k1, k2, tag, a.A.slots);
                        }
                        if (d != FAIL && d < a.T.fmax) part_to_global(a.A, d, f);
                        if (a.pid && d != FAIL && d < a.T.fmax) a.pid[gi - a.pid_base] = PH_ID | d;
                    }
                }
                __syncthreads();
                continue;
            }
            if (FLUERE_MERGE_NOPART) continue;
            for (uint32_t idx = tid; idx < total; idx += MB) {
                uint32_t lo_i = 0, hi_i = nset - 1;  // last set with start <= idx
                while (lo_i < hi_i) {
                    const uint32_t mid = (lo_i + hi_i + 1) >> 1;
                    if (m_start[mid] <= idx) lo_i = mid;
                    else hi_i = mid - 1;
                }
                const unsigned long long base = a.B.first + m_wb[lo_i];
                uint32_t h, k0, k1, k2, tag, x0 = 0, x1 = 0, x2 = 0;
                FlowPart f;
                if (pass == 0) {
                    const size_t o = (size_t)m_lo[lo_i] + (idx - m_start[lo_i]);
                    Part p;
                    const uint4* src = reinterpret_cast<const uint4*>(S.part + o);
                    uint4 v[5];
    #pragma unroll
                    for (int q = 0; q < 5; q++) v[q] = src[q];
                    __builtin_memcpy(&p, v, sizeof p);
                    h = p.h; k0 = p.k0; k1 = p.k1; k2 = p.k2; tag = p.tag;
                    if (macs) {
                        const uint4 xx = S.partx[o];
                        x0 = xx.x; x1 = xx.y; x2 = xx.z;
                    }
                    part_of_stage(p, base, f);
                } else {
                    const size_t o = (size_t)m_lo[lo_i] + (idx - m_start[lo_i]);
                    const uint4* src = reinterpret_cast<const uint4*>(S.dspill) + o * (size_t)(macs ? 4 : 2);
                    const uint4 v0 = src[0], v1 = src[1];
                    k0 = v0.x; k1 = v0.y; k2 = v0.z; tag = v0.w;
                    if (macs) {  // {key}, {MAC words, hash}, {payload}
                        const uint4 v2 = src[2];
                        x0 = v1.x; x1 = v1.y; x2 = v1.z;
                        h = v1.w;
                        spill_to_part(v2.x, v2.y, v2.z, v2.w, base, f);
                    } else {
                        h = lt_hash(k0, k1, k2, tag);
                        spill_to_part(v1.x, v1.y, v1.z, v1.w, base, f);
                    }
                }
                merge_rec(h, k0, k1, k2, tag, x0, x1, x2, f);
            }
            __syncthreads();
        }
        // Dense ids: thread per entry (MT == MB).  The owner is the only inserter
        // of its keys, so a claim (EMPTY -> PENDING) normally succeeds at once;
        // the new ids of the whole workgroup come from ONE atomicAdd on the flow
        // counter (a single hot address: per-flow increments would serialise).
        if (a.dbg && tid == 0) a.dbg[4096 * 8 - 2048 + blockIdx.x * 8 + 3] = wall_clock64();
        static_assert(MT == MB, "one merge entry per thread");
        if (tid == 0) m_nclaim = 0;
        __syncthreads();
        const unsigned long long c1 = clock64();
        const int e = tid;
        const uint4 kk = m_key[e];
        const bool have = (kk.w & LT_READY) != 0;
        const uint32_t tag = kk.w & 0xFF000000u;
        uint32_t d = FAIL, s0 = FAIL, s1 = FAIL, rank = 0;
        bool claimed = false, wait = false;
        unsigned long long* val = nullptr;
        if (have) {
            if (kk.w & V6_TAG) {  // an IPv6 5-tuple from k_slow: the full key from the address ids
                CKey ck;
                v6_ckey(a.v6, kk.x, kk.y, kk.z, tag, ck);
                d = dense_of_key(a.T, ck, true, a.A.slots, &a.g->generic_used);
            } else if (tag == 0xFF000000u) {
                d = kk.x;  // MAC kernels' partials carry dense ids
            } else if (macs) {  // a spilled MAC-kernel key: one dictionary walk per flow and owner
                const uint4 xx = m_kx[MACS ? e : 0];
                CKey ck;
                mac_ckey(kk.x, kk.y, kk.z, tag, xx.x, xx.y, xx.z, ck);
                d = dense_of_key(a.T, ck, true, a.A.slots, nullptr);
            } else if (!v4_fast(a.T, tag >> 24)) {  // wide tables: protocols other than TCP / UDP
                d = staged_id(a.T, a.v6, kk.x, kk.y, kk.z, tag, a.A.slots);
            } else {       // IPv4 5-tuple: flow_table.h chain T0 (ip pair) -> T1 (slot, ports, proto)
                unsigned long long v = EMPTY;
                v4_slots(a.T, kk.x, kk.y, kk.z, tag >> 24, true, s0, s1, &v);
                if (s1 != FAIL) {
                    val = &a.T.tab[1][2 * s1 + 1];
                    if (v >= PENDING) v = atomicCAS(val, EMPTY, PENDING);
                    if (v == EMPTY) {
                        claimed = true;
                        rank = atomicAdd(&m_nclaim, 1u);
                    } else if (v == PENDING) {
                        wait = true;
                    } else {
                        d = (uint32_t)v;
                    }
                }
            }
        }
        __syncthreads();
        if (a.dbg && tid == 0) a.dbg[4096 * 8 - 2048 + blockIdx.x * 8 + 7] = wall_clock64();
        if (tid == 0) m_base = m_nclaim ? atomicAdd(a.T.n_flows, m_nclaim) : 0;
        __syncthreads();
        if (a.dbg && tid == 0) a.dbg[4096 * 8 - 2048 + blockIdx.x * 8 + 6] = wall_clock64();
        if (claimed) {
            d = m_base + rank;
            if (d >= a.T.fmax) {
                atomicOr(a.T.err, ERR_FLOWS_FULL);
                d = FAIL;
            } else {
                uint32_t* dst = (uint32_t*)(a.T.flow_key + (size_t)d * 56);
    #pragma unroll
                for (int k = 0; k < 14; k++) dst[k] = k == 0 ? kk.x : k == 4 ? kk.y : k == 8 ? kk.z : k == 9 ? tag >> 24 : 0;
    #pragma unroll
                for (int j = 0; j < N_TABLES; j++) a.A.slots[(size_t)d * N_TABLES + j] = j == 0 ? s0 : j == 1 ? s1 : NONE32;
            }
            atomicExch(val, (unsigned long long)d);
        }
        for (int sp = 0; sp < (1 << 20); sp++) {  // a claim held elsewhere: poll (wave-uniform)
            if (__ballot(wait) == 0) break;
            if (wait) {
                const unsigned long long v = __hip_atomic_load(val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (v != PENDING && v != EMPTY) {
                    d = (uint32_t)v;
                    wait = false;
                }
            }
            if (__ballot(wait) != 0) __builtin_amdgcn_s_sleep(16);
        }
        if (wait) atomicOr(a.T.err, ERR_SPIN);
        if (a.dbg && tid == 0) a.dbg[4096 * 8 - 2048 + blockIdx.x * 8 + 4] = wall_clock64();
        if (a.emap) a.emap[((size_t)a.pid_batch << 21) | ((size_t)me << 10) | (uint32_t)e] = (have && d < a.T.fmax) ? d : FAIL;
        if (have && d != FAIL && d < a.T.fmax) {
            FlowPart f;
    #pragma unroll
            for (int q = 0; q < 2; q++) {
                f.pk[q] = m_pk[q][e];
                f.by[q] = m_by[q][e];
                f.mn[q] = m_mn[q][e];
                f.mx[q] = m_mx[q][e];
            }
    #pragma unroll
            for (int q = 0; q < 8; q++) f.fl[q] = m_fl[q][e];
            f.fa = m_fa[e];
            f.fc = m_fc[e];
            f.fr = m_fr[e];
            f.la = m_la[e];
            part_to_global(a.A, d, f);
        }
        if (a.dbg && tid == 0) a.dbg[4096 * 8 - 2048 + blockIdx.x * 8 + 5] = wall_clock64();
        if (tid == 0 && a.dbg) {  // diagnostics: contended atomics, debug runs only
            atomicAdd(&a.g->cyc_m_scan, c1 - c0);
            atomicAdd(&a.g->cyc_m_ids, clock64() - c1);
        }
        __syncthreads();  // (the next owner re-initialises the table)
        if (tid == 0) s_me = S.O > gridDim.x ? gridDim.x + (uint32_t)atomicAdd(&a.g->n_owner, 1ull) : S.O;
        __syncthreads();
    }
    // the hot kernel's per-workgroup statistics -> the run counters (one wave
    // of the last workgroup, off the other owners' critical path)
    if (blockIdx.x == gridDim.x - 1 && tid < 64) reduce_stats();
    // k_slow ran: its general-parser list (flat); else the whole slow list
    const unsigned long long n_gen_all =
        a.slow_kernel ? __hip_atomic_load(&a.g->n_gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
    const bool tail_slow = a.slow_kernel ? n_gen_all != 0 : n_slow_all != 0;
    if (FLUERE_MERGE_TAIL && (tail_slow || n_spill_all)) {
        // The tail: the overflow list (spills past their owner segment's
        // capacity: full keys, no parse) and the packets for the general
        // parser: the whole slow list (packets the hot kernel left over: IPv6,
        // IPv4 options, ARP, VXLAN, VLAN, other IP protocols, short frames),
        // or, when k_slow ran, the ones parse_fast / parse_mid left to it.
        // Each record: dense id from the dictionary, then update_flow's
        // order-free part pre-aggregated per dense id in this workgroup's LDS
        // entries (reused: the owner's flows are in the global accumulators);
        // an id with no entry within 32 probes takes the global atomics.
        // Grid-stride over device-side counts (no host round trip).
        __syncthreads();
        for (int e = tid; e < MT; e += MB) {
            m_key[e].x = NONE32;
            m_pk[0][e] = m_pk[1][e] = 0;
            m_by[0][e] = m_by[1][e] = 0;
            m_mn[0][e] = m_mn[1][e] = NONE32;
            m_mx[0][e] = m_mx[1][e] = 0;
#pragma unroll
            for (int q = 0; q < 8; q++) m_fl[q][e] = 0;
            m_fa[e] = m_fc[e] = m_fr[e] = NONE64;
            m_la[e] = 0;
        }
        // single-word keys (the dense id): a CAS claims or finds an entry,
        // nothing to publish, so the bounded probe needs no other lane
        auto put = [&](uint32_t d, const FlowPart& f) {
            uint32_t e = (d * 0x9E3779B1u) >> 22;  // 10 bits: MT == 1024
            for (int pr = 0; pr < 32; pr++) {
                const uint32_t k = atomicCAS(&m_key[e].x, NONE32, d);
                if (k == NONE32 || k == d) {
#pragma unroll
                    for (int q = 0; q < 2; q++) {
                        if (f.pk[q]) {
                            atomicAdd(&m_pk[q][e], f.pk[q]);
                            atomicAdd(&m_by[q][e], f.by[q]);
                        }
                        atomicMin(&m_mn[q][e], f.mn[q]);
                        atomicMax(&m_mx[q][e], f.mx[q]);
                    }
#pragma unroll
                    for (int q = 0; q < 8; q++)
                        if (f.fl[q]) atomicAdd(&m_fl[q][e], f.fl[q]);
                    if (f.fa != NONE64) atomicMin(&m_fa[e], f.fa);
                    if (f.fc != NONE64) atomicMin(&m_fc[e], f.fc);
                    if (f.fr != NONE64) atomicMin(&m_fr[e], f.fr);
                    if (f.la) atomicMax(&m_la[e], f.la);
                    return;
                }
                e = (e + 1) & (MT - 1);
            }
            part_to_global(a.A, d, f);
        };
        const unsigned long long gstride = (unsigned long long)gridDim.x * MB;
        for (unsigned long long i = (unsigned long long)blockIdx.x * MB + tid; i < n_spill_all; i += gstride) {
            const uint4* src = reinterpret_cast<const uint4*>(S.spill) + i * (macs ? 4 : 2);
            const uint4 v0 = src[0], v1 = src[1];
            uint32_t x0 = 0, x1 = 0, x2 = 0;
            uint4 pay = v1;
            if (macs) {
                pay = src[2];
                x0 = v1.x; x1 = v1.y; x2 = v1.z;
            }
            FlowPart f;
            const unsigned long long wbase = S.base[pay.w >> 9];
            spill_to_part(pay.x, pay.y, pay.z, pay.w, wbase, f);
            uint32_t d;
            if (macs && v0.w != 0xFF000000u) {
                CKey ck;
                mac_ckey(v0.x, v0.y, v0.z, v0.w, x0, x1, x2, ck);
                d = dense_of_key(a.T, ck, true, a.A.slots, nullptr);
            } else {
                d = staged_id(a.T, a.v6, v0.x, v0.y, v0.z, v0.w, a.A.slots);
            }
            if (d != FAIL && d < a.T.fmax) put(d, f);
            if (a.pid && d != FAIL && d < a.T.fmax) a.pid[wbase + pay.z - a.pid_base] = PH_ID | d;
        }
        if (tail_slow) {
            // the hot workgroups' regions, flattened: exclusive scan of their counts
            const uint32_t nwg = S.n_wg;  // <= MB
            const uint32_t cnt = tid < (int)nwg ? a.slow_cnt[tid] : 0u;
            const uint32_t st0 = block_exclusive_scan(cnt, m_scan);
            if (tid < (int)nwg) m_start[tid] = st0;
            __syncthreads();
            const unsigned long long n = a.slow_kernel ? n_gen_all : (unsigned long long)m_scan[MB / 64];
            unsigned long long c_valid = 0, c_drop = 0, tmin = NONE64, tmax = 0;
            for (unsigned long long i = (unsigned long long)blockIdx.x * MB + tid; i < n; i += gstride) {
                uint64_t li;
                if (a.slow_kernel) {
                    li = a.gen[i];
                } else {
                    uint32_t lo_w = 0, hi_w = nwg - 1;  // last region with start <= i
                    while (lo_w < hi_w) {
                        const uint32_t mid = (lo_w + hi_w + 1) >> 1;
                        if (m_start[mid] <= i) lo_w = mid;
                        else hi_w = mid - 1;
                    }
                    li = a.slow[(size_t)lo_w * a.slow_region + (i - m_start[lo_w])];
                }
                if (a.slow_abl == 2) { c_drop += li == NONE32; continue; }
                Parsed P;
                parse_record(a.B, li, macs, 1, P);
                if (P.cls) { c_drop++; continue; }
                c_valid++;
                tmin = min(tmin, (unsigned long long)P.t);
                tmax = max(tmax, (unsigned long long)P.t);
                uint8_t dir = 0;
                const uint32_t d = a.slow_abl == 1 ? (P.pi.sip[3] ^ P.pi.dip[3] ^ P.pi.ksp) % 8192u
                                                   : flow_of(a.T, P, macs, true, dir, a.A.slots, &a.g->generic_used);
                if (d == FAIL || d >= a.T.fmax) continue;
                FlowPart f;
                pkt_to_part(P.pi, dir, a.B.first + li, f);
                put(d, f);
                if (a.pid) a.pid[a.B.first + li - a.pid_base] = PH_ID | d;
            }
            // run counters: one set of atomics per wave
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                c_valid += __shfl_xor(c_valid, o, 64);
                c_drop += __shfl_xor(c_drop, o, 64);
                tmin = min(tmin, (unsigned long long)__shfl_xor(tmin, o, 64));
                tmax = max(tmax, (unsigned long long)__shfl_xor(tmax, o, 64));
            }
            if ((tid & 63) == 0) {
                if (c_valid) { atomicAdd(&a.g->valid, c_valid); atomicMin(&a.g->tmin, tmin); atomicMax(&a.g->tmax, tmax); }
                if (c_drop) atomicAdd(&a.g->dropped, c_drop);
            }
        }
        __syncthreads();
        for (int e = tid; e < MT; e += MB) {
            const uint32_t d = m_key[e].x;
            if (d == NONE32) continue;
            FlowPart f;
#pragma unroll
            for (int q = 0; q < 2; q++) {
                f.pk[q] = m_pk[q][e];
                f.by[q] = m_by[q][e];
                f.mn[q] = m_mn[q][e];
                f.mx[q] = m_mx[q][e];
            }
#pragma unroll
            for (int q = 0; q < 8; q++) f.fl[q] = m_fl[q][e];
            f.fa = m_fa[e];
            f.fc = m_fc[e];
            f.fr = m_fr[e];
            f.la = m_la[e];
            part_to_global(a.A, d, f);
        }
    }
}

// ---------------------------------------------------------------------------
// k_slow: the slow list (packets the hot parser left over) when the last run
// had one (the host predicts it; otherwise k_merge_partials' tail takes it).
// Runs between the hot kernel and the merge.  Workgroup b takes slow-list
// entries [b * SLOW_SET, (b + 1) * SLOW_SET) of the hot workgroups' regions
// flattened, as staging set n_hot + b.  Per packet: the 128-byte window,
// parse_fast / parse_mid in registers (the rest -- ARP, VLAN, short frames,
// drops -- go to a list for the general parser in the merge tail: inlined
// here, its registers would cost every packet occupancy); then a spill
// record into its merge owner's segment of the set, like the hot kernel's
// LDS-table misses: an IPv4 key as its words (no dictionary walk here: the
// owner resolves each key once), any other key (IPv6, -M, the raw fallback's
// protocol 255) as its dense id from the dictionary.  k_merge_partials then
// aggregates them with the hot kernel's partials.
// ---------------------------------------------------------------------------
constexpr int SB = 256;                      // k_slow block
constexpr uint32_t SLOW_SET = SPILL_WG / 4;  // slow-list entries per k_slow workgroup (one set)
__global__ void __launch_bounds__(SB) k_slow(AggArgs a) {
    __shared__ uint32_t s_start[MB + 1];
    __shared__ uint32_t s_scnt[OWN_WORDS];  // records per owner (packed 16-bit: a set has <= SLOW_SET)
    const int tid = threadIdx.x;
    const bool macs = a.macs != 0;
    const Stage& S = a.S;
    const uint32_t O = S.O;
    const uint32_t set = S.n_hot + blockIdx.x;
    const int spu = spill_units(macs);
    for (int o = tid; o < OWN_WORDS; o += SB) s_scnt[o] = 0;
    // the hot workgroups' regions, flattened (wave 0: an exclusive scan, an
    // even run of regions per lane)
    const uint32_t nwg = S.n_wg;  // <= MB
    if (tid < 64 && !a.slow_all) {
        const uint32_t per = (nwg + 63) / 64;
        uint32_t sum = 0;
        for (uint32_t q = 0; q < per; q++) {
            const uint32_t w = tid * per + q;
            if (w < nwg) sum += a.slow_cnt[w];
        }
        uint32_t incl = sum;
#pragma unroll
        for (int dlt = 1; dlt < 64; dlt <<= 1) {
            const uint32_t y = __shfl_up(incl, dlt, 64);
            if (tid >= dlt) incl += y;
        }
        uint32_t run = incl - sum;
        for (uint32_t q = 0; q < per; q++) {
            const uint32_t w = tid * per + q;
            if (w < nwg) {
                s_start[w] = run;
                run += a.slow_cnt[w];
            }
        }
        if (tid == 63) s_start[MB] = incl;
    }
    __syncthreads();
    const unsigned long long n = a.slow_all ? a.B.n : s_start[MB];
    const unsigned long long i0 = (unsigned long long)blockIdx.x * SLOW_SET;
    const unsigned long long i1 = min(n, i0 + SLOW_SET);
    unsigned long long c_valid = 0, c_drop = 0, c_seg = 0, tmin = NONE64, tmax = 0;
    for (unsigned long long ib = i0; ib < i1; ib += SB) {  // (uniform)
        const unsigned long long i = ib + tid;
        bool rec = false, gen = false;
        uint32_t ow = 0, gli = 0;
        Parsed P;
        uint4 wk = make_uint4(0, 0, 0, 0), wx = make_uint4(0, 0, 0, 0), wp = make_uint4(0, 0, 0, 0);
        if (i < i1) {
            uint32_t li = (uint32_t)i;
            if (!a.slow_all) {
                uint32_t lo_w = 0, hi_w = nwg - 1;  // last region with start <= i
                while (lo_w < hi_w) {
                    const uint32_t mid = (lo_w + hi_w + 1) >> 1;
                    if (s_start[mid] <= i) lo_w = mid;
                    else hi_w = mid - 1;
                }
                li = a.slow[(size_t)lo_w * a.slow_region + (i - s_start[lo_w])];
            }
            const uint32_t off = a.B.offs[li];
            Win32 W;
            load_win32(a.B, off, W);
            pin_win32(W);
            if (a.slow_abl == 2) {  // diagnostics: no parse (wrong results)
                P.cls = 0;
                P.t = W.w[0];
                P.pi.v6 = 0; P.pi.kproto = 17; P.pi.sip[0] = W.w[9] & 0xF; P.pi.dip[0] = W.w[10] & 0xF;
                P.pi.sip[1] = P.pi.sip[2] = P.pi.sip[3] = P.pi.dip[1] = P.pi.dip[2] = P.pi.dip[3] = 0;
                P.pi.ksp = (uint16_t)(W.w[11] & 7); P.pi.kdp = (uint16_t)(W.w[12] & 7);
                P.pi.tflags = 0; P.pi.rprot = 17; P.pi.doctets = W.w[13] & 0xFFFF; P.pi.rpkt = W.w[14] & 0xFFFF; P.pi.rttl = 1;
                P.smac = P.dmac = 0;
            } else {
                parse_loaded32<0>(a.B, off, W, macs, P);
            }
            gen = P.cls == 2;
            if (gen) {
                gli = li;
            } else if (P.cls) {
                c_drop++;
            } else {
                c_valid++;
                tmin = min(tmin, (unsigned long long)P.t);
                tmax = max(tmax, (unsigned long long)P.t);
                const PktInfo& pi = P.pi;
                uint8_t dir = 0;
                CKey k;
                canon_key(P, macs, k, dir);
                uint32_t h;
                uint32_t ia = FAIL, ib = FAIL;
                if (!macs && pi.v6 && a.v6.C) v6_ids(a.v6, &k.w[0], &k.w[4], ia, ib);
                if (!macs && !pi.v6 && pi.kproto != 0xFF) {
                    // an IPv4 key: its words, as the hot kernel's spills carry them
                    wk = make_uint4(k.w[0], k.w[4], k.w[8], (uint32_t)pi.kproto << 24);
                    h = lt_hash(wk.x, wk.y, wk.z, wk.w);
                    rec = true;
                } else if (ia != FAIL && ib != FAIL) {
                    // an IPv6 key: the ids of its two addresses (no dictionary walk here)
                    wk = make_uint4(ia, ib, k.w[8], ((uint32_t)pi.kproto << 24) | V6_TAG);
                    h = lt_hash(wk.x, wk.y, wk.z, wk.w);
                    rec = true;
                } else {
                    const uint32_t d = a.slow_abl == 1 ? (k.w[3] ^ k.w[7] ^ k.w[8]) % 8192u  // diagnostics: no dictionary
                                                       : dense_of_key(a.T, k, true, a.A.slots, &a.g->generic_used);
                    wk = make_uint4(d, 0, 0, 0xFF000000u);
                    h = lt_hash(d, 0, 0, 0xFF000000u);
                    rec = d != FAIL && d < a.T.fmax;
                }
                const uint32_t tf = pi.tflags;
                const bool elig = (pi.rprot != 6) | ((tf & 2u) != 0);
                wp = make_uint4(pi.doctets, pi.rpkt | ((uint32_t)pi.rttl << 16) | ((elig ? 1u : 0u) << 24), li,
                                tf | ((uint32_t)dir << 8));
                wx = make_uint4(0, 0, 0, h);
                ow = owner_of(h, O);
            }
        }
        // the general parser's packets: the merge tail's list (wave-aggregated append)
        const uint64_t gm = __ballot(gen);
        if (gm) {
            const uint32_t lead = __builtin_ctzll(gm);
            unsigned long long b0 = 0;
            if ((uint32_t)(tid & 63) == lead) b0 = atomicAdd(&a.g->n_gen, (unsigned long long)__popcll(gm));
            b0 = __shfl(b0, lead, 64);
            if (gen) a.gen[b0 + __builtin_amdgcn_mbcnt_hi((uint32_t)(gm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)gm, 0u))] = gli;
        }
        if (a.slow_abl == 3) rec = false;  // diagnostics: no spill records
        const uint32_t pos = rec ? own_add(s_scnt, ow) : 0u;
        const bool ovf = rec && pos >= S.cap_s;
        if (rec && !ovf) {
            uint4* dst = reinterpret_cast<uint4*>(S.dspill) +
                         (S.slow_rec0 + ((size_t)blockIdx.x * O + ow) * S.cap_s + pos) * (2 * spu);
            dst[0] = wk;
            if (macs) {
                dst[1] = wx;
                dst[2] = wp;
            } else {
                dst[1] = wp;
            }
            c_seg++;
        }
        // past the segment's capacity: the overflow list (wave-aggregated append; rare)
        const uint64_t om = __ballot(ovf);
        if (om) {
            const uint32_t lead = __builtin_ctzll(om);
            unsigned long long b0 = 0;
            if ((uint32_t)(tid & 63) == lead) b0 = atomicAdd(&a.g->n_spill, (unsigned long long)__popcll(om));
            b0 = __shfl(b0, lead, 64);
            if (ovf) {
                const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(om >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)om, 0u));
                uint4* dst = reinterpret_cast<uint4*>(S.spill) + (b0 + r) * (size_t)(2 * spu);
                wp.w |= set << 9;
                dst[0] = wk;
                if (macs) {
                    dst[1] = wx;
                    dst[2] = wp;
                } else {
                    dst[1] = wp;
                }
            }
        }
    }
    __syncthreads();
    // this set's segments: record counts, no partials, positions relative to the batch
    for (uint32_t o = tid; o <= O; o += SB) {
        S.off[(size_t)o * S.n_sets + set] = 0;
        if (o < O) S.soff[(size_t)o * S.n_sets + set] = min(own_get(s_scnt, o), S.cap_s);
    }
    if (tid == 0) S.base[set] = a.B.first;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        c_valid += __shfl_xor(c_valid, o, 64);
        c_drop += __shfl_xor(c_drop, o, 64);
        c_seg += __shfl_xor(c_seg, o, 64);
        tmin = min(tmin, (unsigned long long)__shfl_xor(tmin, o, 64));
        tmax = max(tmax, (unsigned long long)__shfl_xor(tmax, o, 64));
    }
    if ((tid & 63) == 0) {
        if (c_valid) { atomicAdd(&a.g->valid, c_valid); atomicMin(&a.g->tmin, tmin); atomicMax(&a.g->tmax, tmax); }
        if (c_drop) atomicAdd(&a.g->dropped, c_drop);
        if (c_seg) atomicAdd(&a.g->n_dspill, c_seg);
    }
}

// one thread per flow, grid-stride (uniform per workgroup) over the
// device-side flow count
// The last workgroup to finish (counter *done) copies the run counters (Glob,
// n_flows, err) to the pinned host copy, then publishes seq there (the host
// polls it: no copy kernel, no event on the way back).
__device__ void publish_ctl(Glob* g, unsigned long long* done, Ctl* host_ctl, uint32_t seq) {
    __shared__ unsigned long long p_rank;
    // Every wave waits for its own counter atomics to be performed (they are
    // device-scope: at the coherence point once acknowledged), then the
    // workgroup counts itself done.  No agent-scope fence per workgroup: it
    // writes back the XCD's L2 (the records just stored) and ~1-4k
    // workgroups serialised on it (C4 k_finalize 327 -> 192 us with the grid
    // capped; the records reach later kernels at the launch boundary).
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) p_rank = atomicAdd(done, 1ull);
    __syncthreads();
    if (p_rank != gridDim.x - 1) return;
    __threadfence();
    const uint32_t* src = reinterpret_cast<const uint32_t*>(g);
    uint32_t* dst = reinterpret_cast<uint32_t*>(host_ctl);
    constexpr uint32_t nw = offsetof(Ctl, seq) / 4;
    for (uint32_t i = threadIdx.x; i < nw; i += blockDim.x)
        __hip_atomic_store(dst + i, __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(&host_ctl->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// k_finalize: one thread per flow (grid-stride); records appended per
// workgroup (emit_record_block).
// The record is built in place in the block's LDS staging (S.rec[thread]):
// held in registers it took the kernel to 250 VGPRs (2 waves per SIMD).
__global__ void __launch_bounds__(EMIT_BLOCK) k_finalize(FinArgs a) {
    const Glob& gg = *a.g;
    const bool mode_b = a.timeout_us && gg.valid && gg.tmax - gg.tmin >= a.timeout_us;
    const uint32_t nf = mode_b ? 0u : min(*a.T.n_flows, a.T.fmax);
    __shared__ EmitLds S;
    __shared__ unsigned long long s_tot[4];  // updates, ended, complex flows, their packets (this workgroup)
    if (threadIdx.x < 4) s_tot[threadIdx.x] = 0;
    unsigned long long tot[2] = {0, 0}, n_cplx = 0, cplx_all = 0;  // (thread 0's totals: updates, ended)
    for (uint32_t d0 = blockIdx.x * blockDim.x; d0 < nf; d0 += gridDim.x * blockDim.x) {
        const uint32_t d = d0 + threadIdx.x;
        fluere_record& r = S.rec[threadIdx.x];
        bool cplx = false;
        unsigned long long cplx_pkts = 0;
        const bool want = d < nf && finalize_one<false>(a, d, r, cplx, cplx_pkts);
        emit_inplace_block(S, a.g, a.out, a.out_cap, want, want ? r.d_pkts : 0u, want && r.order_key != NONE64, nullptr, 0,
                           0, tot);
        n_cplx += cplx ? 1 : 0;
        cplx_all += cplx_pkts;
    }
    // the workgroup's counters: one set of global atomics (per-block or
    // per-wave atomics on these few words serialised a million-flow run)
    n_cplx = wave_sum(n_cplx);
    cplx_all = wave_sum(cplx_all);
    if ((threadIdx.x & 63) == 0 && n_cplx) {
        atomicAdd(&s_tot[2], n_cplx);
        atomicAdd(&s_tot[3], cplx_all);
    }
    if (threadIdx.x == 0) {
        s_tot[0] = tot[0];
        s_tot[1] = tot[1];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (s_tot[0]) atomicAdd(&a.g->n_updates, s_tot[0]);
        if (s_tot[1]) atomicAdd(&a.g->n_ended, s_tot[1]);
        if (s_tot[2]) {
            atomicAdd(&a.g->n_complex, s_tot[2]);
            atomicAdd(&a.g->n_complex_pkts, s_tot[3]);
        }
    }
    if (a.host_ctl) publish_ctl(a.g, &a.g->fin_done, a.host_ctl, a.seq);
}

// k_finalize_gen: the flows k_finalize listed (first packet outside the
// register parser's classes), with the general parser.
__global__ void __launch_bounds__(EMIT_BLOCK) k_finalize_gen(FinArgs a) {
    const uint32_t n = (uint32_t)min(a.g->n_fdefer, (unsigned long long)a.T.fmax);
    __shared__ EmitLds S;
    for (uint32_t i0 = blockIdx.x * blockDim.x; i0 < n; i0 += gridDim.x * blockDim.x) {
        const uint32_t i = i0 + threadIdx.x;
        fluere_record r;
        bool cplx = false;
        unsigned long long cplx_pkts = 0;
        const bool want = i < n && finalize_one<true>(a, a.defer[i], r, cplx, cplx_pkts);
        finalize_emit(S, a, r, want, cplx, cplx_pkts);
    }
}

// ---------------------------------------------------------------------------
// Mode B, sequential fallback (timestamps not non-decreasing): the exact
// global state machine on one thread (expiries can fire)
// ---------------------------------------------------------------------------
struct SeqMeta {
    uint32_t d;       // dense flow id, NONE32 = not a valid packet
    uint8_t dir, tflags, rprot_tcp, ttl;
    uint32_t pkt, doctets;
    uint64_t t;
};

struct SeqMetaArgs {
    Batch B;
    TableSet T;
    SeqMeta* meta;
    uint64_t base;
    int macs;
};

__global__ void __launch_bounds__(256) k_seq_meta(SeqMetaArgs a) {
    uint64_t li = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (li >= a.B.n) return;
    const bool macs = a.macs != 0;
    Parsed P;
    parse_record(a.B, li, macs, 0, P);
    SeqMeta m;
    m.d = NONE32;
    m.dir = 0; m.tflags = 0; m.rprot_tcp = 0; m.ttl = 0; m.pkt = 0; m.doctets = 0; m.t = P.t;
    if (P.cls == 0) {
        uint8_t dir;
        uint32_t d = flow_of(a.T, P, macs, false, dir, nullptr, nullptr);
        m.d = d == FAIL ? NONE32 : d;
        m.dir = dir; m.tflags = P.pi.tflags; m.rprot_tcp = P.pi.rprot == 6; m.ttl = P.pi.rttl;
        m.pkt = P.pi.rpkt; m.doctets = P.pi.doctets;
    }
    a.meta[a.B.first + li - a.base] = m;
}

struct HeapEnt {
    unsigned long long exp, seq;
    uint32_t d;
    uint32_t dir;
};

struct SeqArgs {
    const Batch* bs;
    int nb;
    const SeqMeta* meta;
    unsigned long long n;
    uint8_t* active;   // [fmax]
    uint8_t* cdir;     // [fmax]
    fluere_record* cur;  // [fmax]
    HeapEnt* heap;     // capacity n
    fluere_record* out;
    unsigned long long out_cap;
    Glob* g;
    unsigned long long timeout_us;
    uint64_t base;
    uint32_t n_flows;
    int macs;
};

__device__ __forceinline__ bool h_less(const HeapEnt& x, const HeapEnt& y) {
    return x.exp < y.exp || (x.exp == y.exp && x.seq < y.seq);
}

__global__ void __launch_bounds__(64) k_seq_run(SeqArgs a) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    unsigned long long hn = 0, seq = 0, nout = 0;
    auto emit = [&](const fluere_record& r) {
        if (nout < a.out_cap) { a.out[nout] = r; a.out[nout].order_key = nout; }
        nout++;
    };
    for (unsigned long long gi = 0; gi < a.n; gi++) {  // offline_fluereflows.rs:68-176
        SeqMeta m = a.meta[gi];
        if (m.d == NONE32) continue;
        uint32_t d = m.d;
        bool rev;
        if (a.active[d]) {
            rev = m.dir != a.cdir[d];
        } else {
            if (m.rprot_tcp && !(m.tflags & 2)) continue;  // :101-113 (no sweep either)
            Parsed P;
            parse_global(a.bs, a.nb, gi + a.base, a.macs != 0, P);
            fill_seed(a.cur[d], P);
            a.active[d] = 1;
            a.cdir[d] = m.dir;
            HeapEnt e{m.t + a.timeout_us, seq++, d, m.dir};
            unsigned long long i = hn++;
            a.heap[i] = e;
            while (i) {
                unsigned long long p = (i - 1) / 2;
                if (!h_less(a.heap[i], a.heap[p])) break;
                HeapEnt t = a.heap[i]; a.heap[i] = a.heap[p]; a.heap[p] = t; i = p;
            }
            rev = false;
        }
        fluere_record& r = a.cur[d];
        PktInfo pi;
        pi.doctets = m.doctets; pi.rpkt = m.pkt; pi.rttl = m.ttl; pi.tflags = m.tflags;
        update_flow(r, rev, pi, m.t);
        if (m.tflags & 5) { emit(r); a.active[d] = 0; }
        while (hn && a.heap[0].exp <= m.t) {  // :161-175
            HeapEnt top = a.heap[0];
            // the entry holds the creator Key: it removes whatever flow is now
            // stored under that exact (oriented) key
            if (a.active[top.d] && a.cdir[top.d] == top.dir) { emit(a.cur[top.d]); a.active[top.d] = 0; }
            a.heap[0] = a.heap[--hn];
            unsigned long long i = 0;
            for (;;) {
                unsigned long long l = 2 * i + 1, rr = l + 1, mm = i;
                if (l < hn && h_less(a.heap[l], a.heap[mm])) mm = l;
                if (rr < hn && h_less(a.heap[rr], a.heap[mm])) mm = rr;
                if (mm == i) break;
                HeapEnt t = a.heap[i]; a.heap[i] = a.heap[mm]; a.heap[mm] = t; i = mm;
            }
        }
    }
    unsigned long long ended = nout;
    for (uint32_t d = 0; d < a.n_flows; d++)
        if (a.active[d]) {
            if (nout < a.out_cap) { a.out[nout] = a.cur[d]; a.out[nout].order_key = NONE64; }
            nout++;
        }
    a.g->n_rec = nout;
    a.g->n_heads = ended;  // reused: number of ended records
}

// ---------------------------------------------------------------------------
// cleanup: clear exactly the table slots and accumulators this run touched
// ---------------------------------------------------------------------------
struct CleanArgs {
    TableSet T;
    Acc A;
    uint8_t* complex;
    uint8_t* active;
    Glob* g;
    // speculative cleanup (enqueued right behind a run's counter copy): clear
    // only if the run needs no further device work -- no table error, no
    // complex flow, no expiry inside the capture (Mode B), records fitted.
    // fluere_run takes the same decision on the host from the copied counters.
    int spec;
    unsigned long long timeout_us, recs_cap;
    int abl = 0;  // diagnostics only (FLUERE_CLEAN_ABL, wrong results): 1 no table clears, 2 no accumulator clears
    // 1: tables 0 and 1 (the IPv4 chain) are cleared whole, sequentially,
    // instead of two random 16-byte entries per flow (runs with many flows)
    int bulk = 0;
};

__device__ __host__ __forceinline__ bool run_complete(const Glob& g, uint32_t err, unsigned long long timeout_us,
                                                      unsigned long long recs_cap) {
    const bool modeB = g.valid && (g.tmax - g.tmin) >= timeout_us;
    return !(err & (ERR_TABLE_FULL | ERR_SPIN | ERR_FLOWS_FULL)) && !modeB && g.n_complex == 0 && g.n_rec <= recs_cap &&
           g.n_fdefer == 0;
}

__device__ __forceinline__ void cleanup_one(const CleanArgs& a, uint32_t d, bool tables) {
    // the flow's chain slots (an IPv4 flow uses 2 of the N_TABLES): read as
    // 8-byte pairs, cleared only where set
    uint2* row = reinterpret_cast<uint2*>(a.A.slots + (size_t)d * N_TABLES);
    static_assert(N_TABLES % 2 == 0, "slot rows are whole 8-byte pairs");
    uint2 sv[N_TABLES / 2];
#pragma unroll
    for (int t = 0; t < N_TABLES / 2; t++) sv[t] = (a.bulk && t == 0) ? make_uint2(NONE32, NONE32) : row[t];
#pragma unroll
    for (int t = 0; t < N_TABLES / 2; t++) {
        const uint32_t s0 = sv[t].x, s1 = sv[t].y;
        // one 16-byte store per entry {key, value} (two 8-byte stores were two
        // partial writes of the same random line)
        if (tables && !(a.abl & 1) && s0 != NONE32)
            *reinterpret_cast<ulonglong2*>(&a.T.tab[2 * t][2 * s0]) = make_ulonglong2(EMPTY, EMPTY);
        if (tables && !(a.abl & 1) && s1 != NONE32)
            *reinterpret_cast<ulonglong2*>(&a.T.tab[2 * t + 1][2 * s1]) = make_ulonglong2(EMPTY, EMPTY);
        if (!a.bulk && (s0 & s1) != NONE32) row[t] = make_uint2(NONE32, NONE32);  // (bulk: every claim rewrites its row)
    }
    if (a.abl & 2) return;
    a.A.pk[0][d] = a.A.pk[1][d] = 0;
    a.A.by[0][d] = a.A.by[1][d] = 0;
    a.A.mn[0][d] = a.A.mn[1][d] = NONE32;
    a.A.mx[0][d] = a.A.mx[1][d] = 0;
    for (int q = 0; q < 8; q++) a.A.fl[q][d] = 0;
    a.A.fa[d] = a.A.fc[d] = a.A.fr[d] = NONE64;
    a.A.la[d] = 0;
    a.complex[d] = 0;
    if (a.active) a.active[d] = 0;
}

// Reset the flows of the last run, grid-stride over the device-side count.
// After a failed run (error word set) some table slots may have no dense id,
// so every table word is cleared instead of the recorded chains.
// The workgroup that finishes last re-initialises the run counters (Glob,
// n_flows, err): every other workgroup has read n_flows / err before it
// counted itself done, so nobody can see the reset early.
__global__ void __launch_bounds__(256) k_cleanup(CleanArgs a, size_t tab_words) {
    if (a.spec && !run_complete(*a.g, *a.T.err, a.timeout_us, a.recs_cap)) return;  // every workgroup decides alike
    const bool failed = (*a.T.err & (ERR_TABLE_FULL | ERR_SPIN)) != 0;
    const uint32_t nf = failed ? a.T.fmax : min(*a.T.n_flows, a.T.fmax);
    const size_t stride = (size_t)gridDim.x * blockDim.x, t0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (size_t d = t0; d < nf; d += stride) cleanup_one(a, (uint32_t)d, !failed);
    if (failed)
        for (size_t w = t0; w < tab_words; w += stride) a.T.tab[0][w] = EMPTY;  // tables are contiguous
    else if (a.bulk)  // tables 0 and 1: 2 (C + 1) entries of 16 bytes
        for (size_t w = t0; w < 2 * ((size_t)a.T.C + 1); w += stride)
            reinterpret_cast<ulonglong2*>(a.T.tab[0])[w] = make_ulonglong2(EMPTY, EMPTY);
    __shared__ unsigned long long s_rank;
    __syncthreads();
    // (no fence: what the last workgroup resets, every workgroup read before
    // its work, and its count comes after that work; the stores reach the
    // next kernel at the launch boundary.  A per-workgroup agent-scope fence
    // writes back the XCD's L2 and serialised thousands of workgroups.)
    if (threadIdx.x == 0) s_rank = atomicAdd(&a.g->clean_done, 1ull);
    __syncthreads();
    if (s_rank != gridDim.x - 1) return;
    __threadfence();
    unsigned long long* w = reinterpret_cast<unsigned long long*>(a.g);
    const size_t nw = sizeof(Ctl) / 8;  // Glob + counters (+ padding)
    for (size_t i = threadIdx.x; i < nw; i += blockDim.x)
        w[i] = i == offsetof(Glob, tmin) / 8 ? NONE64 : 0ull;
}

__global__ void k_fill_u64(unsigned long long* p, size_t n, unsigned long long v) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}
__global__ void k_fill_u32(uint32_t* p, size_t n, uint32_t v) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

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

// ---------------------------------------------------------------------------
// multi-GPU exchange (include/fluere_gpu.h): every shard exports summaries and
// annexes bucketed by owner; each owner merges its flows and composes, in
// shard order, the flows whose record depends on packet order
// ---------------------------------------------------------------------------
// owner rank of a canonical key (the same on every rank)
__device__ __forceinline__ uint32_t key_owner(const uint32_t* key, uint32_t n_owners) {
    uint64_t h = 0x9E3779B97F4A7C15ull;
#pragma unroll
    for (int j = 0; j < 14; j++) h = synth::mix64(h ^ key[j]);
    return (uint32_t)(((h >> 32) * (uint64_t)n_owners) >> 32);
}

__device__ __forceinline__ void export_one(const FinArgs& a, fluere_flow_summary& s, uint32_t d) {
    const Acc& A = a.A;
    memset(&s, 0, sizeof s);
    const uint32_t* key = (const uint32_t*)(a.T.flow_key + (size_t)d * 56);
    for (int j = 0; j < 14; j++) s.key[j] = key[j];
    s.pkts[0] = A.pk[0][d]; s.pkts[1] = A.pk[1][d];
    s.bytes[0] = A.by[0][d]; s.bytes[1] = A.by[1][d];
    s.min_pkt = A.mn[0][d]; s.max_pkt = A.mx[0][d]; s.min_ttl = A.mn[1][d]; s.max_ttl = A.mx[1][d];
    for (int q = 0; q < 8; q++) s.flag_cnt[q] = A.fl[q][d];
    s.first_all = A.fa[d]; s.first_create = A.fc[d]; s.finrst_min = A.fr[d]; s.last = A.la[d];
    const bool macs = a.macs != 0;
    if (s.first_create != NONE64) {
        Parsed P;
        parse_global(a.bs, a.nb, s.first_create, macs, P);
        fluere_record sd;
        fill_seed(sd, P);
        s.first_dir = canon_dir(P, macs);
        s.first_sport = sd.src_port; s.first_dport = sd.dst_port;
        s.first_prot = sd.prot; s.first_tos = sd.tos; s.first_v6 = sd.src_v6;
        for (int k = 0; k < 16; k++) { s.first_src[k] = sd.source[k]; s.first_dst[k] = sd.destination[k]; }
        s.first_time = P.t;
    }
    s.last_time = time_global(a.bs, a.nb, s.last);
    s.annex = NONE32;
}

// A flow's local order dependence (shard side): trivial when its first FIN/RST
// (if any) is its last packet and its first packet can create it (or none
// can) -- then the summary alone determines its part of the state machine.
__global__ void __launch_bounds__(256) k_local_cert(FinArgs a, uint32_t* annex_of) {
    const uint32_t nf = min(*a.T.n_flows, a.T.fmax);
    for (uint32_t d0 = blockIdx.x * blockDim.x; d0 < nf; d0 += gridDim.x * blockDim.x) {
        const uint32_t d = d0 + threadIdx.x;
        bool cplx = false;
        if (d < nf) {
            const unsigned long long fa = a.A.fa[d], fc = a.A.fc[d], fr = a.A.fr[d], la = a.A.la[d];
            cplx = !((fr == NONE64 || fr == la) && (fc == fa || fc == NONE64));
            a.complex[d] = cplx ? 1 : 0;
            annex_of[d] = NONE32;
        }
        const uint64_t cm = __ballot(cplx);
        if (cm && (uint32_t)(threadIdx.x & 63) == (uint32_t)__builtin_ctzll(cm))
            atomicAdd(&a.g->n_complex, (unsigned long long)__popcll(cm));
    }
}

struct ExportArgs {
    FinArgs fa;
    uint8_t* blocks;
    uint32_t n_owners, shard;
    uint64_t cap, cap_annex, block_bytes;
    const uint32_t* annex_of;
    const fluere_flow_annex* annex;
    uint32_t* sumpos;  // [fmax]: each flow's summary position in its owner's block (the sweep's packet tags)
};
__device__ __forceinline__ fluere_shard_header* blk_hdr(uint8_t* blocks, uint64_t block_bytes, uint32_t o) {
    return reinterpret_cast<fluere_shard_header*>(blocks + (size_t)o * block_bytes);
}
__device__ __forceinline__ fluere_flow_summary* blk_sum(uint8_t* blocks, uint64_t block_bytes, uint32_t o) {
    return reinterpret_cast<fluere_flow_summary*>(blocks + (size_t)o * block_bytes + sizeof(fluere_shard_header));
}
__device__ __forceinline__ fluere_flow_annex* blk_annex(uint8_t* blocks, uint64_t block_bytes, uint64_t cap, uint32_t o) {
    return reinterpret_cast<fluere_flow_annex*>(blocks + (size_t)o * block_bytes + sizeof(fluere_shard_header) +
                                                cap * sizeof(fluere_flow_summary));
}

__global__ void k_export_hdr(ExportArgs a) {
    const uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= a.n_owners) return;
    fluere_shard_header h{};
    const Glob* g = a.fa.g;
    h.tmin = g->tmin; h.tmax = g->tmax; h.valid = g->valid; h.dropped = g->dropped;
    h.err = *a.fa.T.err;
    h.shard = a.shard;
    *blk_hdr(a.blocks, a.block_bytes, o) = h;
}

__global__ void __launch_bounds__(256) k_export_owners(ExportArgs a) {
    const uint32_t nf = min(*a.fa.T.n_flows, a.fa.T.fmax);
    for (uint32_t d = blockIdx.x * blockDim.x + threadIdx.x; d < nf; d += gridDim.x * blockDim.x) {
        fluere_flow_summary s;
        export_one(a.fa, s, d);
        s.shard = a.shard;
        const uint32_t o = key_owner(s.key, a.n_owners);
        fluere_shard_header* h = blk_hdr(a.blocks, a.block_bytes, o);
        const unsigned long long pos = atomicAdd(reinterpret_cast<unsigned long long*>(&h->n_flows), 1ull);
        const uint32_t ax = a.annex ? a.annex_of[d] : NONE32;  // (no annexes yet: a speculative export)
        if (ax != NONE32) {
            const unsigned long long apos = atomicAdd(reinterpret_cast<unsigned long long*>(&h->n_annex), 1ull);
            if (apos < a.cap_annex) {
                blk_annex(a.blocks, a.block_bytes, a.cap, o)[apos] = a.annex[ax];
                s.annex = (uint32_t)apos;
            }
        }
        if (pos < a.cap) blk_sum(a.blocks, a.block_bytes, o)[pos] = s;
        a.sumpos[d] = (uint32_t)pos;
    }
}

// need[0..1]: the largest per-owner summary / annex counts; info (may be
// null): the same, then the shard's order-dependent flows and its flow count
// (fluere_export_async: reduced over the ranks on the device, read once).
__global__ void k_export_need(ExportArgs a, unsigned long long* need, unsigned long long* info) {
    if (threadIdx.x || blockIdx.x) return;
    unsigned long long m0 = 0, m1 = 0;
    for (uint32_t o = 0; o < a.n_owners; o++) {
        const fluere_shard_header* h = blk_hdr(a.blocks, a.block_bytes, o);
        m0 = max(m0, (unsigned long long)h->n_flows);
        m1 = max(m1, (unsigned long long)h->n_annex);
    }
    need[0] = m0;
    need[1] = m1;
    if (info) {
        const Glob* g = a.fa.g;
        info[0] = m0;
        info[1] = m1;
        info[2] = g->n_complex;
        info[3] = min(*a.fa.T.n_flows, a.fa.T.fmax);
        // the capture span, reducible with MAX: 2^62 - tmin and tmax (0: no valid packet)
        info[4] = g->valid ? (1ull << 62) - g->tmin : 0ull;
        info[5] = g->valid ? g->tmax : 0ull;
    }
}

struct FirstPay {
    unsigned long long t_first, t_last;
    uint16_t sp, dp;
    uint8_t dir, prot, tos, v6;
    uint8_t src[16], dst[16];
};

struct MergeArgs {
    TableSet T;
    Acc A;
    unsigned long long n;  // n_shards * cap summary slots
    uint32_t* sd;
    FirstPay* pay;
    Glob* g;
    fluere_record* out;
    uint8_t* complex;
    uint64_t out_cap;
    // the gathered blocks: summary i is entry i % cap of block i / cap (the
    // block of rank i / cap); entries past the block's n_flows are absent
    const uint8_t* blocks;
    unsigned long long cap, cap_annex, block_bytes;
    Ctl* host_ctl;   // non-null: k_merge_finalize publishes the counters (publish_ctl)
    uint32_t seq;
    unsigned long long timeout_us;
};

// summary i of a merge; null when absent
__device__ __forceinline__ const fluere_flow_summary* merge_input(const MergeArgs& a, unsigned long long i) {
    if (i >= a.n) return nullptr;
    uint8_t* blocks = const_cast<uint8_t*>(a.blocks);
    const uint32_t b = (uint32_t)(i / a.cap);
    const unsigned long long j = i % a.cap;
    if (j >= min((unsigned long long)blk_hdr(blocks, a.block_bytes, b)->n_flows, a.cap)) return nullptr;
    return blk_sum(blocks, a.block_bytes, b) + j;
}
__device__ __forceinline__ const fluere_flow_annex* merge_annex(const MergeArgs& a, unsigned long long i, uint32_t k) {
    return blk_annex(const_cast<uint8_t*>(a.blocks), a.block_bytes, a.cap, (uint32_t)(i / a.cap)) + k;
}

__global__ void __launch_bounds__(256) k_merge_insert(MergeArgs a) {
    unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < a.n && i % a.cap == 0) {  // the block's run counters
        const fluere_shard_header* h = blk_hdr(const_cast<uint8_t*>(a.blocks), a.block_bytes, (uint32_t)(i / a.cap));
        if (h->valid) {
            atomicAdd(&a.g->valid, (unsigned long long)h->valid);
            atomicMin(&a.g->tmin, (unsigned long long)h->tmin);
            atomicMax(&a.g->tmax, (unsigned long long)h->tmax);
        }
        if (h->dropped) atomicAdd(&a.g->dropped, (unsigned long long)h->dropped);
        if (h->err) atomicOr(a.T.err, h->err);
        if (h->n_flows > a.cap || h->n_annex > a.cap_annex) atomicOr(a.T.err, ERR_CAPACITY);  // cut short
    }
    const fluere_flow_summary* sp = merge_input(a, i);
    if (!sp) {
        if (i < a.n) a.sd[i] = FAIL;
        return;
    }
    const fluere_flow_summary& s = *sp;
    CKey k;
    for (int j = 0; j < 14; j++) k.w[j] = s.key[j];
    uint32_t d = dense_of_key(a.T, k, true, a.A.slots, &a.g->generic_used);
    a.sd[i] = d;
    if (d == FAIL || d >= a.T.fmax) return;
    const Acc& A = a.A;
    for (int q = 0; q < 2; q++) {
        if (s.pkts[q]) { atomicAdd(&A.pk[q][d], s.pkts[q]); atomicAdd(&A.by[q][d], (unsigned long long)s.bytes[q]); }
    }
    atomicMin(&A.mn[0][d], s.min_pkt); atomicMax(&A.mx[0][d], s.max_pkt);
    atomicMin(&A.mn[1][d], s.min_ttl); atomicMax(&A.mx[1][d], s.max_ttl);
    for (int q = 0; q < 8; q++) if (s.flag_cnt[q]) atomicAdd(&A.fl[q][d], s.flag_cnt[q]);
    atomicMin(&A.fa[d], (unsigned long long)s.first_all);
    atomicMin(&A.fc[d], (unsigned long long)s.first_create);
    atomicMin(&A.fr[d], (unsigned long long)s.finrst_min);
    atomicMax(&A.la[d], (unsigned long long)s.last);
}

__global__ void __launch_bounds__(256) k_merge_payload(MergeArgs a) {
    unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    uint32_t d = a.sd[i];
    if (d == FAIL || d >= a.T.fmax) return;
    const fluere_flow_summary& s = *merge_input(a, i);
    // packet indices are global and unique: exactly one shard holds each
    if (s.first_create != NONE64 && s.first_create == a.A.fc[d]) {
        FirstPay& p = a.pay[d];
        p.t_first = s.first_time;
        p.sp = s.first_sport; p.dp = s.first_dport;
        p.dir = s.first_dir; p.prot = s.first_prot; p.tos = s.first_tos; p.v6 = s.first_v6;
        for (int k = 0; k < 16; k++) { p.src[k] = s.first_src[k]; p.dst[k] = s.first_dst[k]; }
    }
    if (s.last == a.A.la[d]) a.pay[d].t_last = s.last_time;
}

__device__ __forceinline__ void merge_finalize_one(const MergeArgs& a, uint32_t d, fluere_record& r, bool& want,
                                                   bool& cplx) {
    const Acc& A = a.A;
    unsigned long long fa = A.fa[d], fc = A.fc[d], fr = A.fr[d], la = A.la[d];
    if (fc == NONE64) return;
    if (!(fc == fa && (fr == NONE64 || fr == la))) {
        a.complex[d] = 1;
        cplx = true;
        return;
    }
    const FirstPay p = a.pay[d];
    memset(&r, 0, sizeof r);
    r.src_v6 = r.dst_v6 = p.v6;
    for (int k = 0; k < 16; k++) { r.source[k] = p.src[k]; r.destination[k] = p.dst[k]; }
    r.prot = p.prot; r.tos = p.tos; r.src_port = p.sp; r.dst_port = p.dp;
    uint32_t p0 = A.pk[0][d], p1 = A.pk[1][d];
    unsigned long long b0 = A.by[0][d], b1 = A.by[1][d];
    r.d_pkts = p0 + p1;
    r.d_octets = b0 + b1;
    r.out_pkts = p.dir ? p1 : p0; r.in_pkts = p.dir ? p0 : p1;
    r.out_bytes = p.dir ? b1 : b0; r.in_bytes = p.dir ? b0 : b1;
    r.min_pkt = A.mn[0][d]; r.max_pkt = A.mx[0][d];
    r.min_ttl = (uint8_t)A.mn[1][d]; r.max_ttl = (uint8_t)A.mx[1][d];
    for (int q = 0; q < 8; q++) r.cnt[q] = A.fl[q][d];
    r.first = p.t_first;
    r.last = p.t_last;
    r.order_key = (fr == la) ? la : NONE64;
    want = true;
}

// grid-stride over the flows counted on the device (no host round trip)
__global__ void __launch_bounds__(EMIT_BLOCK) k_merge_finalize(MergeArgs a) {
    // a capture whose span reaches the timeout: no record here, the sweep
    // composition (fluere_sweep_*) builds them all
    const Glob* g = a.g;
    const bool expiry = g->valid && g->tmax >= g->tmin && g->tmax - g->tmin >= a.timeout_us;
    const uint32_t nf = expiry ? 0u : min(*a.T.n_flows, a.T.fmax);
    __shared__ EmitLds S;
    for (uint32_t d0 = blockIdx.x * blockDim.x; d0 < nf; d0 += gridDim.x * blockDim.x) {
        const uint32_t d = d0 + threadIdx.x;
        fluere_record r;
        bool want = false, cplx = false;
        if (d < nf) merge_finalize_one(a, d, r, want, cplx);
        emit_record_block(S, a.g, a.out, a.out_cap, r, want);
        const uint64_t cm = __ballot(cplx);
        if (cm && (uint32_t)(threadIdx.x & 63) == (uint32_t)__builtin_ctzll(cm))
            atomicAdd(&a.g->n_complex, (unsigned long long)__popcll(cm));
    }
    if (a.host_ctl) publish_ctl(a.g, &a.g->fin_done, a.host_ctl, a.seq);
}

// ---- composition of the order-dependent flows at their owner ----------------
// the owner's summaries of complex flows, as (flow << 8 | shard, summary index)
__global__ void __launch_bounds__(256) k_comp_collect(MergeArgs a, unsigned long long* keys, uint32_t* vals) {
    const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const uint32_t d = a.sd[i];
    if (d == FAIL || d >= a.T.fmax || !a.complex[d]) return;
    const unsigned long long pos = atomicAdd(&a.g->n_keys, 1ull);
    keys[pos] = ((unsigned long long)d << 8) | (i / a.cap);
    vals[pos] = (uint32_t)i;
}

__device__ __forceinline__ void piece_clear(fluere_flow_piece& p) {
    memset(&p, 0, sizeof p);
    p.min_pkt = p.min_ttl = NONE32;
}
__device__ __forceinline__ void piece_add(fluere_flow_piece& f, const fluere_flow_piece& x) {
    for (int q = 0; q < 2; q++) { f.pkts[q] += x.pkts[q]; f.bytes[q] += x.bytes[q]; }
    f.min_pkt = min(f.min_pkt, x.min_pkt); f.max_pkt = max(f.max_pkt, x.max_pkt);
    f.min_ttl = min(f.min_ttl, x.min_ttl); f.max_ttl = max(f.max_ttl, x.max_ttl);
    for (int q = 0; q < 8; q++) f.flag_cnt[q] += x.flag_cnt[q];
    if (x.pkts[0] + x.pkts[1] && (f.pkts[0] + f.pkts[1] == x.pkts[0] + x.pkts[1] || x.last > f.last)) {
        f.last = x.last;
        f.last_time = x.last_time;
    }
}
// a trivial shard summary as one piece (its seed: the creating packet)
__device__ __forceinline__ void piece_of_summary(const fluere_flow_summary& s, fluere_flow_piece& p) {
    p.pkts[0] = s.pkts[0]; p.pkts[1] = s.pkts[1];
    p.bytes[0] = s.bytes[0]; p.bytes[1] = s.bytes[1];
    p.min_pkt = s.min_pkt; p.max_pkt = s.max_pkt; p.min_ttl = s.min_ttl; p.max_ttl = s.max_ttl;
    for (int q = 0; q < 8; q++) p.flag_cnt[q] = s.flag_cnt[q];
    p.last = s.last; p.last_time = s.last_time;
    p.first = s.first_create; p.first_time = s.first_time;
    for (int k = 0; k < 16; k++) { p.src[k] = s.first_src[k]; p.dst[k] = s.first_dst[k]; }
    p.v6 = s.first_v6; p.prot = s.first_prot; p.tos = s.first_tos; p.dir = s.first_dir;
    p.src_port = s.first_sport; p.dst_port = s.first_dport;
}
__device__ __forceinline__ void record_of_piece(const fluere_flow_piece& f, unsigned long long order, fluere_record& r) {
    memset(&r, 0, sizeof r);
    r.src_v6 = r.dst_v6 = f.v6;
    for (int k = 0; k < 16; k++) { r.source[k] = f.src[k]; r.destination[k] = f.dst[k]; }
    r.prot = f.prot; r.tos = f.tos; r.src_port = f.src_port; r.dst_port = f.dst_port;
    const uint32_t o = f.dir;
    r.d_pkts = f.pkts[0] + f.pkts[1];
    r.d_octets = f.bytes[0] + f.bytes[1];
    r.out_pkts = f.pkts[o]; r.in_pkts = f.pkts[1 - o];
    r.out_bytes = f.bytes[o]; r.in_bytes = f.bytes[1 - o];
    r.min_pkt = f.min_pkt; r.max_pkt = f.max_pkt;
    r.min_ttl = (uint8_t)f.min_ttl; r.max_ttl = (uint8_t)f.max_ttl;
    for (int q = 0; q < 8; q++) r.cnt[q] = f.flag_cnt[q];
    r.first = f.first_time;
    r.last = f.last_time;
    r.order_key = order;
}

// One thread per complex flow: offline_fluereflows.rs:97-157 over the shards
// in order, each shard as (A = its packets up to its first FIN/RST, f0, H =
// the instance it creates from "no flow" up to f0, T = the instance open at
// its end after f0).  Entering with a flow F open: F += A, closed at f0 (then
// T, if any, is open).  Entering with none: H is emitted at f0 (or stays open
// without f0), then T.
__global__ void __launch_bounds__(64) k_compose(MergeArgs a, const unsigned long long* keys, const uint32_t* vals,
                                                unsigned long long n) {
    const unsigned long long p = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n || (p > 0 && (keys[p - 1] >> 8) == (keys[p] >> 8))) return;
    const unsigned long long d = keys[p] >> 8;
    fluere_flow_piece F;
    bool open = false;
    for (unsigned long long q = p; q < n && (keys[q] >> 8) == d; q++) {
        const unsigned long long i = vals[q];
        const fluere_flow_summary& s = *merge_input(a, i);
        fluere_flow_piece A, H, T;
        bool has_f0, has_H, has_T;
        unsigned long long f0;
        if (s.annex == NONE32) {
            piece_of_summary(s, A);
            has_f0 = s.finrst_min != NONE64;
            f0 = s.finrst_min;
            has_H = s.first_create != NONE64;  // == first_all (the local certificate held)
            H = A;
            has_T = false;
        } else if (s.annex >= a.cap_annex) {  // a corrupt block: never read past its annexes
            atomicOr(a.T.err, ERR_CAPACITY);
            return;
        } else {
            const fluere_flow_annex& x = *merge_annex(a, i, s.annex);
            has_f0 = x.flags & 1;
            f0 = x.f0;
            has_H = x.flags & 4;
            has_T = x.flags & 8;
            piece_clear(A);
            if (x.flags & 2) piece_add(A, x.lead);
            if (has_H) piece_add(A, x.head);
            H = x.head;
            T = x.tail;
        }
        fluere_record r;
        if (open) {
            piece_add(F, A);
            if (has_f0) {
                record_of_piece(F, f0, r);
                emit_record(a.g, a.out, a.out_cap, r);
                open = false;
            }
        } else if (has_f0) {
            if (has_H) {
                record_of_piece(H, f0, r);
                emit_record(a.g, a.out, a.out_cap, r);
            }
        } else if (has_H) {
            F = H;
            open = true;
        }
        if (has_f0 && has_T) {
            F = T;
            open = true;
        }
    }
    if (open) {
        fluere_record r;
        record_of_piece(F, NONE64, r);
        emit_record(a.g, a.out, a.out_cap, r);
    }
}

// ---- the compact wire encoding of export blocks ------------------------------
// A wide block (fluere_flow_summary, 256 B each) carries every field at full
// width.  On the wire each summary is a variable-length record: a descriptor
// word says which fields are present and how wide; absent fields (zero
// counters, flag counts, a first FIN/RST, a first packet that differs from the
// creating one, the seed of a flow with no creating packet) take no bytes, and
// an IPv4 5-tuple key takes 12 bytes instead of 56.  Wire block of one owner:
// the block header, a u32 offset table (one per summary, relative to the
// records), the records (4-byte aligned), the annexes verbatim (16-byte
// aligned).  The owner expands every received block back to the wide layout,
// at the same positions, before fluere_merge_gathered.
enum : uint32_t {
    WB_PK0 = 1u << 18, WB_PK1 = 1u << 19, WB_WBY = 1u << 20, WB_WMM = 1u << 21, WB_FC = 1u << 22,
    WB_FA = 1u << 23,  WB_FR = 1u << 24,  WB_AX = 1u << 25,  WB_DIR = 1u << 26, WB_V6 = 1u << 27,
    WB_LADDR = 1u << 28, WB_FULLKEY = 1u << 29,
};
constexpr uint32_t WIRE_REC_MAX = 4 + 56 + 8 + 16 + 20 + 32 + 16 + 16 + 16 + 4 + 32 + 4;  // 224
constexpr uint32_t WIRE_MAX_BLOCKS = 64;  // shards of one unpack (kernel-argument offsets)

__device__ __forceinline__ bool wire_short_key(const fluere_flow_summary& s) {
    uint32_t o = s.key[9] >> 10;
#pragma unroll
    for (int j = 0; j < 14; j++)
        if (j != 0 && j != 4 && j != 8 && j != 9) o |= s.key[j];
    return o == 0;
}
__device__ __forceinline__ bool wire_long_addr(const fluere_flow_summary& s) {
    uint32_t o = s.first_v6;
#pragma unroll
    for (int k = 4; k < 16; k++) o |= s.first_src[k] | s.first_dst[k];
    return o != 0;
}
__device__ __forceinline__ uint32_t wire_desc(const fluere_flow_summary& s) {
    uint32_t fm = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) fm |= (s.flag_cnt[q] ? 1u : 0u) << q;
    uint32_t d = (s.key[9] & 0x3FFu) | (fm << 10);
    d |= s.pkts[0] ? WB_PK0 : 0u;
    d |= s.pkts[1] ? WB_PK1 : 0u;
    d |= (s.bytes[0] > 0xFFFFFFFFull || s.bytes[1] > 0xFFFFFFFFull) ? WB_WBY : 0u;
    d |= (s.min_pkt > 0xFFFFu || s.max_pkt > 0xFFFFu || s.min_ttl > 0xFFu || s.max_ttl > 0xFFu) ? WB_WMM : 0u;
    d |= s.first_create != NONE64 ? WB_FC : 0u;
    d |= s.first_all != s.first_create ? WB_FA : 0u;
    d |= s.finrst_min != NONE64 ? WB_FR : 0u;
    d |= s.annex != NONE32 ? WB_AX : 0u;
    d |= s.first_dir ? WB_DIR : 0u;
    d |= s.first_v6 ? WB_V6 : 0u;
    d |= wire_long_addr(s) ? WB_LADDR : 0u;
    d |= wire_short_key(s) ? 0u : WB_FULLKEY;
    return d;
}
__device__ __forceinline__ uint32_t wire_bytes(uint32_t d) {
    const uint32_t by = (d & WB_WBY) ? 8u : 4u;
    uint32_t n = 4 + ((d & WB_FULLKEY) ? 56u : 12u);
    n += (d & WB_PK0) ? 4u + by : 0u;
    n += (d & WB_PK1) ? 4u + by : 0u;
    n += (d & WB_WMM) ? 20u : 8u;  // min / max pkt, ttl (+ prot, tos)
    n += 4u * __popc((d >> 10) & 0xFFu);
    n += 8u + 8u;  // last, last_time
    n += (d & WB_FA) ? 8u : 0u;
    n += (d & WB_FR) ? 8u : 0u;
    n += (d & WB_FC) ? 8u + 8u + 4u + ((d & WB_LADDR) ? 32u : 8u) : 0u;  // first_create, first_time, ports, addresses
    n += (d & WB_AX) ? 4u : 0u;
    return n;
}
struct WirePut {
    uint32_t* p;
    __device__ __forceinline__ void u32(uint32_t v) { *p++ = v; }
    __device__ __forceinline__ void u64(unsigned long long v) { p[0] = (uint32_t)v; p[1] = (uint32_t)(v >> 32); p += 2; }
    __device__ __forceinline__ void bytes(const uint8_t* b, int n) {
        for (int k = 0; k < n; k += 4) u32(b[k] | (b[k + 1] << 8) | (b[k + 2] << 16) | ((uint32_t)b[k + 3] << 24));
    }
};
struct WireGet {
    const uint32_t* p;
    __device__ __forceinline__ uint32_t u32() { return *p++; }
    __device__ __forceinline__ unsigned long long u64() {
        const unsigned long long v = p[0] | ((unsigned long long)p[1] << 32);
        p += 2;
        return v;
    }
    __device__ __forceinline__ void bytes(uint8_t* b, int n) {
        for (int k = 0; k < n; k += 4) {
            const uint32_t v = u32();
            b[k] = (uint8_t)v; b[k + 1] = (uint8_t)(v >> 8); b[k + 2] = (uint8_t)(v >> 16); b[k + 3] = (uint8_t)(v >> 24);
        }
    }
};
__device__ __forceinline__ void wire_put(const fluere_flow_summary& s, uint32_t d, uint32_t* dst) {
    WirePut w{dst};
    w.u32(d);
    if (d & WB_FULLKEY) {
#pragma unroll
        for (int j = 0; j < 14; j++) w.u32(s.key[j]);
    } else {
        w.u32(s.key[0]); w.u32(s.key[4]); w.u32(s.key[8]);
    }
#pragma unroll
    for (int q = 0; q < 2; q++)
        if (d & (q ? WB_PK1 : WB_PK0)) {
            w.u32(s.pkts[q]);
            if (d & WB_WBY) w.u64(s.bytes[q]);
            else w.u32((uint32_t)s.bytes[q]);
        }
    if (d & WB_WMM) {
        w.u32(s.min_pkt); w.u32(s.max_pkt); w.u32(s.min_ttl); w.u32(s.max_ttl);
        w.u32((uint32_t)s.first_prot | ((uint32_t)s.first_tos << 8));
    } else {
        w.u32(s.min_pkt | (s.max_pkt << 16));
        w.u32(s.min_ttl | (s.max_ttl << 8) | ((uint32_t)s.first_prot << 16) | ((uint32_t)s.first_tos << 24));
    }
#pragma unroll
    for (int q = 0; q < 8; q++)
        if ((d >> (10 + q)) & 1) w.u32(s.flag_cnt[q]);
    w.u64(s.last);
    w.u64(s.last_time);
    if (d & WB_FA) w.u64(s.first_all);
    if (d & WB_FR) w.u64(s.finrst_min);
    if (d & WB_FC) {
        w.u64(s.first_create);
        w.u64(s.first_time);
        w.u32(s.first_sport | ((uint32_t)s.first_dport << 16));
        const int na = (d & WB_LADDR) ? 16 : 4;
        w.bytes(s.first_src, na);
        w.bytes(s.first_dst, na);
    }
    if (d & WB_AX) w.u32(s.annex);
}
__device__ __forceinline__ void wire_get(const uint32_t* src, uint32_t shard, fluere_flow_summary& s) {
    memset(&s, 0, sizeof s);
    WireGet w{src};
    const uint32_t d = w.u32();
    if (d & WB_FULLKEY) {
#pragma unroll
        for (int j = 0; j < 14; j++) s.key[j] = w.u32();
    } else {
        s.key[0] = w.u32(); s.key[4] = w.u32(); s.key[8] = w.u32();
        s.key[9] = d & 0x3FFu;
    }
#pragma unroll
    for (int q = 0; q < 2; q++)
        if (d & (q ? WB_PK1 : WB_PK0)) {
            s.pkts[q] = w.u32();
            s.bytes[q] = (d & WB_WBY) ? w.u64() : (unsigned long long)w.u32();
        }
    if (d & WB_WMM) {
        s.min_pkt = w.u32(); s.max_pkt = w.u32(); s.min_ttl = w.u32(); s.max_ttl = w.u32();
        const uint32_t x = w.u32();
        s.first_prot = (uint8_t)x; s.first_tos = (uint8_t)(x >> 8);
    } else {
        const uint32_t a = w.u32(), b = w.u32();
        s.min_pkt = a & 0xFFFFu; s.max_pkt = a >> 16;
        s.min_ttl = b & 0xFFu; s.max_ttl = (b >> 8) & 0xFFu; s.first_prot = (uint8_t)(b >> 16); s.first_tos = (uint8_t)(b >> 24);
    }
#pragma unroll
    for (int q = 0; q < 8; q++) s.flag_cnt[q] = ((d >> (10 + q)) & 1) ? w.u32() : 0u;
    s.last = w.u64();
    s.last_time = w.u64();
    s.first_create = NONE64;
    s.finrst_min = NONE64;
    const unsigned long long fa = (d & WB_FA) ? w.u64() : 0ull;
    if (d & WB_FR) s.finrst_min = w.u64();
    if (d & WB_FC) {
        s.first_create = w.u64();
        s.first_time = w.u64();
        const uint32_t pp = w.u32();
        s.first_sport = (uint16_t)pp; s.first_dport = (uint16_t)(pp >> 16);
        const int na = (d & WB_LADDR) ? 16 : 4;
        w.bytes(s.first_src, na);
        w.bytes(s.first_dst, na);
    }
    s.first_all = (d & WB_FA) ? fa : s.first_create;
    s.first_dir = (d & WB_DIR) ? 1 : 0;
    s.first_v6 = (d & WB_V6) ? 1 : 0;
    s.annex = (d & WB_AX) ? w.u32() : NONE32;
    s.shard = shard;
}

struct WireArgs {
    const uint8_t* blocks;       // wide blocks (pack: the export's; unpack: the merge's)
    uint8_t* wblocks;
    const uint8_t* wire;
    uint8_t* wwire;
    uint64_t cap, cap_annex, block_bytes;
    uint32_t n_blocks;
    unsigned long long* sz;      // pack: [n_blocks * cap + 1] record bytes (0: absent)
    unsigned long long* scan;    // pack: exclusive sum of sz
    unsigned long long* woff;    // [n_blocks + 1]: offset of each wire block (device)
    unsigned long long* sizes;   // pack: [n_blocks] bytes of each wire block (the caller's device buffer)
    unsigned long long off_h[WIRE_MAX_BLOCKS + 1];  // unpack: offset of each received wire block, then the end
};
__device__ __forceinline__ uint64_t wire_table_bytes(uint64_t n) { return (4 * n + 15) & ~15ull; }
__device__ __forceinline__ uint64_t blk_count(const uint8_t* blocks, uint64_t block_bytes, uint32_t b, uint64_t cap) {
    return min((unsigned long long)reinterpret_cast<const fluere_shard_header*>(blocks + (size_t)b * block_bytes)->n_flows,
               (unsigned long long)cap);
}
__device__ __forceinline__ uint64_t blk_acount(const uint8_t* blocks, uint64_t block_bytes, uint32_t b, uint64_t cap_annex) {
    return min((unsigned long long)reinterpret_cast<const fluere_shard_header*>(blocks + (size_t)b * block_bytes)->n_annex,
               (unsigned long long)cap_annex);
}

// pack 1: each summary's record bytes (0 for the absent slots past n_flows)
__global__ void __launch_bounds__(256) k_wire_size(WireArgs a) {
    const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned long long n = (unsigned long long)a.n_blocks * a.cap;
    if (i > n) return;
    unsigned long long v = 0;
    if (i < n) {
        const uint32_t b = (uint32_t)(i / a.cap);
        const uint64_t j = i % a.cap;
        if (j < blk_count(a.blocks, a.block_bytes, b, a.cap)) {
            const fluere_flow_summary* s = reinterpret_cast<const fluere_flow_summary*>(
                a.blocks + (size_t)b * a.block_bytes + sizeof(fluere_shard_header)) + j;
            v = wire_bytes(wire_desc(*s));
        }
    }
    a.sz[i] = v;
}
// pack 2 (one thread): each wire block's size and offset
__global__ void k_wire_offsets(WireArgs a) {
    if (threadIdx.x || blockIdx.x) return;
    unsigned long long off = 0;
    for (uint32_t b = 0; b < a.n_blocks; b++) {
        const uint64_t n = blk_count(a.blocks, a.block_bytes, b, a.cap);
        const uint64_t na = blk_acount(a.blocks, a.block_bytes, b, a.cap_annex);
        const uint64_t rec = a.scan[(size_t)(b + 1) * a.cap] - a.scan[(size_t)b * a.cap];
        const uint64_t bytes = sizeof(fluere_shard_header) + wire_table_bytes(n) + ((rec + 15) & ~15ull) +
                               na * sizeof(fluere_flow_annex);
        a.woff[b] = off;
        a.sizes[b] = bytes;
        off += bytes;
    }
    a.woff[a.n_blocks] = off;
}
// pack 3: header, offset table and record of each summary (thread per summary slot)
__global__ void __launch_bounds__(256) k_wire_pack(WireArgs a) {
    const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (unsigned long long)a.n_blocks * a.cap) return;
    const uint32_t b = (uint32_t)(i / a.cap);
    const uint64_t j = i % a.cap;
    const uint8_t* wb = a.blocks + (size_t)b * a.block_bytes;
    uint8_t* out = a.wwire + a.woff[b];
    const uint64_t n = blk_count(a.blocks, a.block_bytes, b, a.cap);
    if (j == 0) *reinterpret_cast<fluere_shard_header*>(out) = *reinterpret_cast<const fluere_shard_header*>(wb);
    if (j >= n) return;
    const uint32_t rel = (uint32_t)(a.scan[i] - a.scan[(size_t)b * a.cap]);
    reinterpret_cast<uint32_t*>(out + sizeof(fluere_shard_header))[j] = rel;
    const fluere_flow_summary& s = *(reinterpret_cast<const fluere_flow_summary*>(wb + sizeof(fluere_shard_header)) + j);
    wire_put(s, wire_desc(s), reinterpret_cast<uint32_t*>(out + sizeof(fluere_shard_header) + wire_table_bytes(n) + rel));
}
// pack 4 / unpack 2: the annexes, verbatim (thread per 16-byte word)
__global__ void __launch_bounds__(256) k_wire_annex(WireArgs a, int unpack) {
    const uint32_t b = blockIdx.y;
    const uint8_t* hdrp = unpack ? a.wire + a.off_h[b] : a.blocks + (size_t)b * a.block_bytes;
    const fluere_shard_header& h = *reinterpret_cast<const fluere_shard_header*>(hdrp);
    const uint64_t n = min((unsigned long long)h.n_flows, (unsigned long long)a.cap);
    const uint64_t na = min((unsigned long long)h.n_annex, (unsigned long long)a.cap_annex);
    const uint64_t words = na * sizeof(fluere_flow_annex) / 16;
    const uint8_t* wide_ax = (unpack ? a.wblocks : a.blocks) + (size_t)b * a.block_bytes + sizeof(fluere_shard_header) +
                             a.cap * sizeof(fluere_flow_summary);
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < words; k += (uint64_t)gridDim.x * blockDim.x) {
        if (!unpack) {
            const uint64_t rec = a.scan[(size_t)(b + 1) * a.cap] - a.scan[(size_t)b * a.cap];
            uint8_t* wax = a.wwire + a.woff[b] + sizeof(fluere_shard_header) + wire_table_bytes(n) + ((rec + 15) & ~15ull);
            reinterpret_cast<uint4*>(wax)[k] = reinterpret_cast<const uint4*>(wide_ax)[k];
        } else {
            // the received block's records end at the start of its annexes: total - annex bytes
            const uint8_t* wax = a.wire + a.off_h[b + 1] - na * sizeof(fluere_flow_annex);
            reinterpret_cast<uint4*>(const_cast<uint8_t*>(wide_ax))[k] = reinterpret_cast<const uint4*>(wax)[k];
        }
    }
}
// unpack 1: the wide block header and summaries (thread per summary slot)
__global__ void __launch_bounds__(256) k_wire_unpack(WireArgs a) {
    const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (unsigned long long)a.n_blocks * a.cap) return;
    const uint32_t b = (uint32_t)(i / a.cap);
    const uint64_t j = i % a.cap;
    const uint8_t* in = a.wire + a.off_h[b];
    const fluere_shard_header& h = *reinterpret_cast<const fluere_shard_header*>(in);
    uint8_t* wb = a.wblocks + (size_t)b * a.block_bytes;
    if (j == 0) *reinterpret_cast<fluere_shard_header*>(wb) = h;
    const uint64_t n = min((unsigned long long)h.n_flows, (unsigned long long)a.cap);
    if (j >= n) return;
    const uint32_t rel = reinterpret_cast<const uint32_t*>(in + sizeof(fluere_shard_header))[j];
    fluere_flow_summary s;
    wire_get(reinterpret_cast<const uint32_t*>(in + sizeof(fluere_shard_header) + wire_table_bytes(n) + rel), h.shard, s);
    *(reinterpret_cast<fluere_flow_summary*>(wb + sizeof(fluere_shard_header)) + j) = s;
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

unsigned grid_for(uint64_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

}  // namespace

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

// ===========================================================================
// host side
// ===========================================================================
static unsigned long long* g_hot_dbg = nullptr;  // FLUERE_DEBUG: per-workgroup hot-kernel timestamps

struct HostBatch {
    Batch b{};
    void* own_bytes = nullptr;
    void* own_offs = nullptr;
    uint2* own_desc = nullptr;  // chunk descriptors (built by upload_batches)
};

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
    hipEvent_t evk0 = nullptr, evk1 = nullptr;  // around the last k_parse_agg launch
    hipEvent_t evk_first = nullptr;             // before the first k_parse_agg launch of the pass
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
};

static int prepare_capture(fluere_ctx* c);

// 512 B of private memory a lane, 1024-thread workgroups: more than any
// kernel of a run uses (k_merge_partials 304 B, k_compose 440 B); stores
// nothing (n is never 1)
__global__ void __launch_bounds__(1024) k_scratch_warm(uint8_t* out, uint32_t n) {
    volatile uint32_t buf[128];
    for (uint32_t i = 0; i < 128; i++) buf[(i * 7u + threadIdx.x) & 127u] = i;
    if (n == 1u) out[threadIdx.x] = (uint8_t)buf[threadIdx.x & 127u];
}
static int sort_actives(fluere_ctx* c, uint64_t ne, uint64_t m);

static void reset_record_counters(fluere_ctx* c) {
    char* g = (char*)c->d_glob;
    for (size_t off : {offsetof(Glob, n_rec), offsetof(Glob, n_complex), offsetof(Glob, n_complex_pkts),
                       offsetof(Glob, n_heads), offsetof(Glob, n_updates), offsetof(Glob, n_ended),
                       offsetof(Glob, n_fdefer), offsetof(Glob, n_okey)})
        hipMemsetAsync(g + off, 0, 8, c->stream);
}

// Host copy of device-resident records, ended prefix first in emission order
// (order_key: global index of the closing packet; with order words, sharded
// Mode B: then aux[0], aux[1]), then active flows.  After a one-GPU run the
// device has ordered the ended prefix already (order_records): only the
// active flows are sorted here, by first packet -- the reference emits them
// after its loop (offline_fluereflows.rs:182-191) in HashMap order, so any
// order is the reference's; this one is deterministic.
static int fetch_records(fluere_ctx* c) {
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
        HIPCHECK(hipStreamSynchronize(s));
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
    HIPCHECK(hipStreamSynchronize(s));
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

static void sweep_free(fluere_ctx* c);

static TableSet tables_of(fluere_ctx* c) {
    TableSet T;
    for (int t = 0; t < N_TABLES; t++) T.tab[t] = c->d_tab + (size_t)t * 2 * (c->C + 1);
    T.C = c->C;
    T.fmax = c->fmax;
    T.n_flows = c->d_nflows;
    T.err = c->d_nflows + 1;
    T.flow_key = c->d_flow_key;
    return T;
}

extern "C" int fluere_abi_version(void) { return FLUERE_ABI_VERSION; }

// The dictionary and the per-flow state for up to mf flows, empty: every
// table EMPTY, the accumulators at their identities (what k_cleanup leaves).
static int alloc_flow_state(fluere_ctx* c, uint64_t mf) {
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

static void free_flow_state(fluere_ctx* c) {
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
    if (hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
        hipEventCreate(&c->ev2) != hipSuccess || hipEventCreate(&c->evk0) != hipSuccess ||
        hipEventCreate(&c->evk1) != hipSuccess || hipEventCreate(&c->evk_first) != hipSuccess ||
        hipEventCreate(&c->ev_ctl) != hipSuccess)
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
static int grow_flow_state(fluere_ctx* c, uint64_t want) {
    const uint64_t mf = std::min<uint64_t>(std::max<uint64_t>(want, (uint64_t)c->fmax * 2), MAX_FLOWS);
    if (mf <= c->fmax) return FLUERE_OK;
    HIPCHECK(hipStreamSynchronize(c->stream));
    free_flow_state(c);
    int rc = alloc_flow_state(c, mf);
    if (rc) return rc;
    c->precleaned = true;  // (alloc_flow_state's fills are what a cleanup leaves)
    c->prev_nf = 0;
    c->last_nf = std::min<uint64_t>(c->last_nf, c->fmax);
    return FLUERE_OK;
}

static void free_batches(fluere_ctx* c) {
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
    hipFree(c->d_recaux);
    hipFree(c->d_okey);
    sweep_free(c);
    hipFree(c->d_sd);
    if (c->ev0) hipEventDestroy(c->ev0);
    if (c->ev1) hipEventDestroy(c->ev1);
    if (c->ev2) hipEventDestroy(c->ev2);
    if (c->evk0) hipEventDestroy(c->evk0);
    if (c->evk1) hipEventDestroy(c->evk1);
    if (c->evk_first) hipEventDestroy(c->evk_first);
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
static unsigned flow_grid(fluere_ctx* c) {
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(grid_for(c->fmax, 256), (uint64_t)c->n_cu * 16));
}
// Grid of the per-flow kernels that end on a done-counter (k_cleanup,
// k_finalize): grid-stride over n flows with at most 4 workgroups per CU, so
// a million-flow run counts ~1k workgroups done on the one word, not ~4k.
static unsigned done_grid(fluere_ctx* c, uint64_t n) {
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(grid_for(n, 256), (uint64_t)c->n_cu * 4));
}

// Sequential clear of the IPv4 chain's tables when the flows to clear would
// cost more as random 16-byte writes (two per flow) than 32 (C + 1) bytes
// written in order: more than (C + 1) / 16 flows.
static int bulk_clean(const fluere_ctx* c, uint64_t nf) {
    static const int env = getenv("FLUERE_BULK_CLEAN") ? atoi(getenv("FLUERE_BULK_CLEAN")) : -1;
    if (env >= 0) return env;
    return nf != ~0ull && nf > ((uint64_t)c->C + 1) / 16 ? 1 : 0;
}

// Clears the flows of the last run and re-initialises every run counter
// (one launch; see k_cleanup).
static int clear_flows(fluere_ctx* c) {
    hipStream_t s = c->stream;
    (void)hipGetLastError();
    CleanArgs a{tables_of(c), c->acc, c->d_complex, c->d_active, c->d_glob};
    static const int clean_abl = getenv("FLUERE_CLEAN_ABL") ? atoi(getenv("FLUERE_CLEAN_ABL")) : 0;
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
static int wait_published(fluere_ctx* c, uint32_t seq, Glob& g, uint32_t (&nf_err)[2]) {
    volatile uint32_t* seqp = &c->h_ctl->seq;
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

static int read_glob(fluere_ctx* c, Glob& g) {
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
    HIPCHECK(hipStreamSynchronize(c->stream));
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

// libpcap offline walk: stop at the first truncated or
// oversized record.  Returns records, fills offsets (relative to file start).
static int64_t pcap_walk(const uint8_t* f, uint64_t nbytes, uint64_t* offs, uint64_t cap, uint32_t* snap_out,
                         int* swapped_out, int* nsec_out) {
    if (!f || nbytes < 24) return FLUERE_E_PCAP;
    uint32_t magic;
    memcpy(&magic, f, 4);
    int sw = 0, ns = 0;
    if (magic == 0xa1b2c3d4u) {
    } else if (magic == 0xd4c3b2a1u) sw = 1;
    else if (magic == 0xa1b23c4du) ns = 1;
    else if (magic == 0x4d3cb2a1u) { sw = 1; ns = 1; }
    else return FLUERE_E_PCAP;
    auto rd = [&](uint64_t o) { uint32_t v; memcpy(&v, f + o, 4); return sw ? __builtin_bswap32(v) : v; };
    uint32_t snap = rd(16);
    const uint32_t kMax = 262144;
    if (snap == 0 || snap > kMax) snap = kMax;
    if (snap_out) *snap_out = snap;
    if (swapped_out) *swapped_out = sw;
    if (nsec_out) *nsec_out = ns;
    uint64_t off = 24;
    int64_t n = 0;
    while (off + 16 <= nbytes) {
        uint32_t incl = rd(off + 8);
        if (incl > kMax || off + 16 + (uint64_t)incl > nbytes) break;
        if (offs && (uint64_t)n < cap) offs[n] = off;
        n++;
        off += 16 + (uint64_t)incl;
    }
    return n;
}

extern "C" int64_t fluere_pcap_index(const uint8_t* file, uint64_t nbytes, uint64_t* offsets, uint64_t cap) {
    if (file && is_pcapng(file, nbytes)) {  // pcapng: the record count (offsets exist for classic files only)
        if (offsets) return FLUERE_E_ARG;
        std::vector<uint8_t> classic;
        const int rc = pcapng_to_pcap(file, nbytes, classic);
        if (rc) return rc;
        return pcap_walk(classic.data(), classic.size(), nullptr, 0, nullptr, nullptr, nullptr);
    }
    return pcap_walk(file, nbytes, offsets, cap, nullptr, nullptr, nullptr);
}

// ---------------------------------------------------------------------------
// Host ingress.  The capture streams to the device in order through pinned
// staging chunks (the copy of one chunk overlaps filling the next), and the
// record index is built on the host from the staged bytes: libpcap offline
// semantics (stop at the first bad or truncated record).  The record chain is
// a pointer chase (each header gives the next one's offset), latency-bound
// once the bytes have left the cache, so each reader thread walks its own
// chunk as it fills it (in L2-sized pieces), from a record start it
// recognises (a run of plausible headers); the calling thread then only
// checks that the true chain meets the reader's: a chunk whose guessed start
// was wrong is walked from the true position until the chains meet (or to
// its end).  The whole capture lands in one device allocation; batches
// (< 4 GiB each, u32 offsets) are sub-ranges.
// ---------------------------------------------------------------------------
constexpr uint32_t kSnapMax = 262144;
constexpr uint64_t kMaxBatch = (1ull << 32) - (1ull << 20);

// Staging slots: reader threads fill slot k % kIngestSlots with chunk k
// (pread from the file, or a copy of the host buffer) while the calling
// thread indexes the chunks in order and enqueues their H2D copies.
constexpr int kIngestSlots = 8;  // at most; FLUERE_INGEST_SLOTS / _READERS (diagnostics) pick fewer
static uint64_t ingest_chunk() {  // staging chunk bytes (FLUERE_INGEST_CHUNK_MB: diagnostics)
    static const uint64_t v =
        (uint64_t)(getenv("FLUERE_INGEST_CHUNK_MB") ? std::max(1, std::min(64, atoi(getenv("FLUERE_INGEST_CHUNK_MB")))) : 4) << 20;
    return v;
}
static int ingest_slots() {
    static const int v = getenv("FLUERE_INGEST_SLOTS") ? std::max(2, std::min(kIngestSlots, atoi(getenv("FLUERE_INGEST_SLOTS")))) : 8;
    return v;
}
static int ingest_readers() {
    static const int v = getenv("FLUERE_INGEST_READERS") ? std::max(1, std::min(16, atoi(getenv("FLUERE_INGEST_READERS")))) : 8;
    return v;
}
constexpr uint64_t kFillPiece = 512ull << 10;  // a reader fills and walks this much at a time (in L2)
constexpr int kSyncRun = 8;                    // plausible headers in a row that make a record start

// One chunk's record chain as its reader walked it (offsets chunk-relative).
struct ChunkChain {
    std::vector<uint32_t> so;  // record starts
    int64_t start = -1;        // the first record start taken; -1 none yet, -2 none found
    uint64_t next = 0;         // where the chain continues (may lie past the chunk)
    uint64_t scan = 0;         // the record-start search position
    bool stopped = false;      // the chain met a record libpcap's walk stops at
};

struct Ingest {
    fluere_ctx* c;
    uint64_t size = 0;
    uint8_t* d = nullptr;
    uint8_t* pin[kIngestSlots] = {};
    hipEvent_t ev[kIngestSlots] = {};
    bool busy[kIngestSlots] = {};
    int nslots = 2;
    int sw = 0, ns = 0;
    uint32_t snap = kSnapMax;
    uint64_t pos = 24;
    bool stopped = false;
    uint8_t tail[16];
    // the record index: pieces of the chains the readers walked, and of the
    // calling thread's own walk (absolute offsets, seq64), in capture order
    struct Piece {
        int64_t chunk;  // -1: seq64[i0, i0 + n)
        size_t i0, n;
    };
    std::vector<Piece> pieces;
    std::vector<uint64_t> seq64;
    std::vector<ChunkChain> chains;  // per chunk, when the readers walk
    uint64_t nrec = 0;
    uint32_t snap_file = kSnapMax;   // the global header's snaplen (record-start plausibility)
    std::vector<size_t> cut;         // first record of each batch
    std::vector<uint64_t> cut_base;  // byte offset of each batch
    // the capture side's record offsets (fluere_live_batch_indexed): the
    // chunks are only copied; finish() checks the records against them in
    // the source image (independent loads, not the walk's pointer chase)
    const uint8_t* src = nullptr;
    const uint64_t* given = nullptr;
    uint64_t given_n = 0;

    explicit Ingest(fluere_ctx* cc) : c(cc) {}
    ~Ingest() {
        for (int i = 0; i < kIngestSlots; i++)
            if (busy[i]) hipEventSynchronize(ev[i]);  // no copy may read a freed staging chunk
        if (c->reuse_ingest) return;  // the arena keeps them
        for (int i = 0; i < kIngestSlots; i++) {
            if (ev[i]) hipEventDestroy(ev[i]);
            if (pin[i]) hipHostFree(pin[i]);
        }
        if (d) hipFree(d);  // still owned here unless finish() handed it over
    }
    int begin(uint64_t nbytes) {
        if (nbytes < 24) return FLUERE_E_PCAP;
        size = nbytes;
        nslots = ingest_slots();
        const int ns_ = (int)std::min<uint64_t>(nslots, (nbytes + ingest_chunk() - 1) / ingest_chunk());
        const auto ta = std::chrono::steady_clock::now();
        if (c->reuse_ingest) {
            static_assert(kIngestSlots == 8, "arena slots");
            if (nbytes + 256 > c->ar_d_cap) {
                const uint64_t cap = std::max<uint64_t>(nbytes + 256, c->ar_d_cap * 3 / 2);
                hipFree(c->ar_d);
                c->ar_d = nullptr;
                c->ar_d_cap = 0;
                if (hipMalloc(&c->ar_d, cap) != hipSuccess) return FLUERE_E_NOMEM;
                c->ar_d_cap = cap;
            }
            d = c->ar_d;
            for (int i = 0; i < ns_; i++) {
                if (!c->ar_pin[i] && hipHostMalloc(&c->ar_pin[i], ingest_chunk(), hipHostMallocDefault) != hipSuccess)
                    return FLUERE_E_NOMEM;
                if (!c->ar_ev[i] && hipEventCreateWithFlags(&c->ar_ev[i], hipEventDisableTiming) != hipSuccess)
                    return FLUERE_E_HIP;
                pin[i] = c->ar_pin[i];
                ev[i] = c->ar_ev[i];
            }
            return FLUERE_OK;
        }
        if (hipMalloc(&d, nbytes + 256) != hipSuccess) return FLUERE_E_NOMEM;
        const auto tb = std::chrono::steady_clock::now();
        for (int i = 0; i < ns_; i++) {
            if (hipHostMalloc(&pin[i], ingest_chunk(), hipHostMallocDefault) != hipSuccess) return FLUERE_E_NOMEM;
            if (hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess) return FLUERE_E_HIP;
        }
        if (getenv("FLUERE_HOSTPROF"))
            fprintf(stderr, "[fluere] ingest setup: device buffer %.1f ms, %d pinned slots of %llu MiB %.1f ms\n",
                    1e3 * std::chrono::duration<double>(tb - ta).count(), ns_, (unsigned long long)(ingest_chunk() >> 20),
                    1e3 * std::chrono::duration<double>(std::chrono::steady_clock::now() - tb).count());
        return FLUERE_OK;
    }
    // staging slot for chunk k, free once its previous copy has completed
    uint8_t* slot(uint64_t k) {
        const int i = (int)(k % nslots);
        if (busy[i]) {
            hipEventSynchronize(ev[i]);
            busy[i] = false;
        }
        return pin[i];
    }
    // Every chunk of [0, nbytes): fill(dst, offset, len) brings bytes into a
    // staging slot (reader threads), feed() indexes and copies them in order.
    template <class Fill>
    int run(uint64_t nbytes, Fill fill) {
        const uint64_t nch = (nbytes + ingest_chunk() - 1) / ingest_chunk();
        if (nch <= 1) {  // one chunk: no threads
            for (uint64_t k = 0; k < nch; k++) {
                const uint64_t cs = k * ingest_chunk(), len = std::min(ingest_chunk(), nbytes - cs);
                if (!fill(slot(k), cs, len)) return FLUERE_E_IO;
                const int rc = feed(k, cs, len);
                if (rc) return rc;
            }
            return FLUERE_OK;
        }
        const int NS = nslots, NR = ingest_readers();
        // the global header first: the readers' walks need its byte order
        if (!given) {
            if (!fill(pin[0], 0, 24)) return FLUERE_E_IO;
            if (int rc = global_header(pin[0])) return rc;
            chains.resize(nch);
        }
        std::atomic<int64_t> filled[kIngestSlots];
        for (auto& f : filled) f.store(-1);
        std::atomic<int64_t> fed{-1};
        std::atomic<bool> fail{false}, stop{false};
        auto reader = [&](int t) {
            for (uint64_t k = t; k < nch && !stop.load(); k += NR) {
                const int i = (int)(k % NS);
                // the slot's previous chunk (k - slots) indexed and its copy done
                while ((int64_t)k - NS > fed.load() && !stop.load()) std::this_thread::yield();
                if (stop.load()) return;
                if (k >= (uint64_t)NS && hipEventSynchronize(ev[i]) != hipSuccess) { fail = true; stop = true; return; }
                const uint64_t cs = k * ingest_chunk(), len = std::min(ingest_chunk(), nbytes - cs);
                if (given) {
                    if (!fill(pin[i], cs, len)) { fail = true; stop = true; return; }
                } else {
                    ChunkChain& ch = chains[k];
                    ch.so.reserve(len / 128 + 64);
                    if (k == 0) ch.start = ch.next = 24;
                    for (uint64_t f = 0; f < len; f += kFillPiece) {
                        const uint64_t pl = std::min(kFillPiece, len - f);
                        if (!fill(pin[i] + f, cs + f, pl)) { fail = true; stop = true; return; }
                        chain_walk(pin[i], cs, f + pl, len, ch);
                    }
                }
                filled[i].store((int64_t)k);
            }
        };
        static const bool hostprof = getenv("FLUERE_HOSTPROF") != nullptr;
        const auto t0 = std::chrono::steady_clock::now();
        double wait_s = 0, feed_s = 0;
        std::vector<std::thread> th;
        for (int t = 0; t < NR; t++) th.emplace_back(reader, t);
        int rc = FLUERE_OK;
        for (uint64_t k = 0; k < nch && !rc; k++) {
            const int i = (int)(k % NS);
            const auto w0 = std::chrono::steady_clock::now();
            while (filled[i].load() != (int64_t)k && !fail.load()) std::this_thread::yield();
            const auto w1 = std::chrono::steady_clock::now();
            if (fail.load()) { rc = FLUERE_E_IO; break; }
            const uint64_t cs = k * ingest_chunk(), len = std::min(ingest_chunk(), nbytes - cs);
            rc = feed(k, cs, len);
            fed.store((int64_t)k);
            wait_s += std::chrono::duration<double>(w1 - w0).count();
            feed_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - w1).count();
        }
        stop = true;
        for (auto& t : th) t.join();
        if (hostprof)
            fprintf(stderr, "[fluere] ingest %llu chunks, %d slots, %d readers: %.1f ms (main waits %.1f, indexes+enqueues %.1f)\n",
                    (unsigned long long)nch, NS, NR,
                    1e3 * std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(), 1e3 * wait_s,
                    1e3 * feed_s);
        return rc;
    }
    uint32_t rd32(const uint8_t* p) const {
        uint32_t v;
        memcpy(&v, p, 4);
        return sw ? __builtin_bswap32(v) : v;
    }
    int global_header(const uint8_t* b) {  // pcap global header (libpcap offline)
        uint32_t magic;
        memcpy(&magic, b, 4);
        if (magic == 0xa1b2c3d4u) {
        } else if (magic == 0xd4c3b2a1u) sw = 1;
        else if (magic == 0xa1b23c4du) ns = 1;
        else if (magic == 0x4d3cb2a1u) { sw = 1; ns = 1; }
        else return FLUERE_E_PCAP;
        snap = rd32(b + 16);
        if (snap == 0 || snap > kSnapMax) snap = kSnapMax;
        snap_file = snap;
        return FLUERE_OK;
    }
    // Is q (chunk-relative, bytes [0, avail) present) the start of kSyncRun
    // plausible record headers in a row?  1 yes, 0 no, -1 not enough bytes
    // yet.  Plausible: caplen within the snaplen and the wire length, a
    // nonzero wire length, a sub-second fraction in range.  Only a speed
    // question: a wrong guess costs the calling thread a walk, never a result.
    int plausible_run(const uint8_t* b, uint64_t q, uint64_t avail, uint64_t len) const {
        const uint32_t frac_max = ns ? 1000000000u : 1000000u;
        for (int d = 0; d < kSyncRun; d++) {
            if (q >= len) return d > 0 ? 1 : 0;  // the run leaves the chunk
            if (q + 16 > avail) return avail == len ? (d > 0 ? 1 : 0) : -1;
            const uint32_t frac = rd32(b + q + 4), incl = rd32(b + q + 8), orig = rd32(b + q + 12);
            if (frac >= frac_max || incl > snap_file || incl > orig || orig == 0 || orig > (1u << 20)) return 0;
            q += 16 + (uint64_t)incl;
        }
        return 1;
    }
    // reader side: extend chunk [cs, cs + len)'s chain over its bytes [0, avail)
    void chain_walk(const uint8_t* b, uint64_t cs, uint64_t avail, uint64_t len, ChunkChain& ch) const {
        if (ch.start == -2) return;
        if (ch.start < 0) {
            // a record starts within the first kSnapMax + 16 bytes of any chunk
            const uint64_t lim = std::min<uint64_t>(len, kSnapMax + 32);
            while (ch.scan < lim) {
                const int r = plausible_run(b, ch.scan, avail, len);
                if (r < 0) return;  // wait for the next piece
                if (r > 0) break;
                ch.scan++;
            }
            if (ch.scan >= lim) { ch.start = -2; return; }
            ch.start = (int64_t)ch.scan;
            ch.next = ch.scan;
        }
        uint64_t p = ch.next;
        while (!ch.stopped && p + 16 <= avail) {
            const uint32_t incl = rd32(b + p + 8);
            if (incl > kSnapMax || cs + p + 16 + (uint64_t)incl > size) {
                ch.stopped = true;
                break;
            }
            ch.so.push_back((uint32_t)p);
            p += 16 + (uint64_t)incl;
        }
        ch.next = p;
    }
    void push_rec(uint64_t off) {
        if (pieces.empty() || pieces.back().chunk >= 0) pieces.push_back({-1, seq64.size(), 0});
        seq64.push_back(off);
        pieces.back().n++;
        nrec++;
    }
    // calling thread: the true chain met chunk k's at its record j (or its end)
    void take_chain(uint64_t k, uint64_t cs, size_t j) {
        const ChunkChain& ch = chains[k];
        const size_t n = ch.so.size() - j;
        const uint64_t end = cs + ch.next;
        if (n) {
            if (end - cut_base.back() > kMaxBatch)  // a 4-GiB batch boundary inside: place it record by record
                for (size_t i = j; i < ch.so.size(); i++) {
                    const uint64_t e = cs + (i + 1 < ch.so.size() ? ch.so[i + 1] : ch.next);
                    if (e - cut_base.back() > kMaxBatch) {
                        cut.push_back(nrec + (i - j));
                        cut_base.push_back(cs + ch.so[i]);
                    }
                }
            pieces.push_back({(int64_t)k, j, n});
            nrec += n;
        }
        pos = end;
        if (ch.stopped) stopped = true;
    }
    // chunk k = bytes [cs, cs + len) of the capture, already in slot(k)
    int feed(uint64_t k, uint64_t cs, uint64_t len) {
        const uint8_t* b = pin[k % nslots];
        if (cs == 0) {
            if (int rc = global_header(b)) return rc;
            cut.push_back(0);
            cut_base.push_back(24);
        }
        const uint64_t ce = cs + len;
        uint8_t h[16];
        const ChunkChain* ch = k < chains.size() && chains[k].start >= 0 ? &chains[k] : nullptr;
        size_t j = 0;
        while (!given && !stopped && pos + 16 <= ce) {
            if (ch && pos >= cs) {  // has the true chain met the reader's?
                const uint64_t r = pos - cs;
                while (j < ch->so.size() && ch->so[j] < r) j++;
                if (j < ch->so.size() ? ch->so[j] == r : r == ch->next) {
                    take_chain(k, cs, j);
                    break;
                }
            }
            const uint8_t* hp;
            if (pos >= cs) {
                hp = b + (pos - cs);
            } else {  // header straddles the previous chunk (its last 16 bytes are in tail)
                for (int j = 0; j < 16; j++) h[j] = pos + j >= cs ? b[pos + j - cs] : tail[16 - (cs - (pos + j))];
                hp = h;
            }
            const uint32_t incl = rd32(hp + 8);
            if (incl > kSnapMax || pos + 16 + (uint64_t)incl > size) {
                stopped = true;
                break;
            }
            if (pos + 16 + incl - cut_base.back() > kMaxBatch) {
                cut.push_back(nrec);
                cut_base.push_back(pos);
            }
            push_rec(pos);
            pos += 16 + (uint64_t)incl;
        }
        if (pos + 16 > size) stopped = true;
        if (len >= 16) memcpy(tail, b + len - 16, 16);
        else {  // short final chunk: shift it into the tail
            memmove(tail, tail + len, 16 - len);
            memcpy(tail + 16 - len, b, len);
        }
        const int i = (int)(k % nslots);
        HIPCHECK(hipMemcpyAsync(d + cs, b, len, hipMemcpyHostToDevice, c->stream));
        HIPCHECK(hipEventRecord(ev[i], c->stream));
        busy[i] = true;
        return FLUERE_OK;
    }
    // libpcap's walk over the given offsets, the same stop rules: record i is
    // taken while it starts where record i - 1 ended and its caplen is one the
    // walk takes.  Each record's test needs only its own header and the one
    // before, so threads test ranges of records at once (independent loads);
    // the first failing record ends the batch.
    void walk_given() {
        const uint64_t n = given_n;
        auto incl_of = [&](uint64_t i) -> uint64_t {
            const uint64_t o = given[i];
            return o + 16 <= size ? rd32(src + o + 8) : ~0ull;
        };
        auto ok = [&](uint64_t i, uint64_t prev_end) {
            const uint64_t o = given[i], incl = incl_of(i);
            return o == prev_end && o + 16 <= size && incl <= kSnapMax && o + 16 + incl <= size;
        };
        const int T = n >= (1u << 16) ? 8 : 1;
        std::vector<uint64_t> first_bad(T, n);
        auto part = [&](int t) {
            const uint64_t i0 = n * t / T, i1 = n * (t + 1) / T;
            uint64_t prev_end = 24;
            if (i0 > 0) {
                const uint64_t pi = incl_of(i0 - 1);
                prev_end = pi == ~0ull ? ~0ull : given[i0 - 1] + 16 + pi;
            }
            for (uint64_t i = i0; i < i1; i++) {
                if (i + 32 < i1 && given[i + 32] + 16 <= size) __builtin_prefetch(src + given[i + 32]);
                if (!ok(i, prev_end)) { first_bad[t] = i; return; }
                prev_end = given[i] + 16 + incl_of(i);
            }
        };
        if (T == 1) {
            part(0);
        } else {
            std::vector<std::thread> th;
            for (int t = 0; t < T; t++) th.emplace_back(part, t);
            for (auto& x : th) x.join();
        }
        const uint64_t m = *std::min_element(first_bad.begin(), first_bad.end());
        pos = 24;
        for (uint64_t i = 0; i < m; i++) {
            const uint64_t end = i + 1 < m ? given[i + 1] : given[i] + 16 + incl_of(i);
            if (end - cut_base.back() > kMaxBatch) {
                cut.push_back(nrec);
                cut_base.push_back(given[i]);
            }
            push_rec(given[i]);
            pos = end;
        }
    }
    // records [g0, g1) of the index, batch-relative
    void fill_rel(uint32_t* out, size_t g0, size_t g1, const std::vector<size_t>& pstart) const {
        if (g0 >= g1) return;
        size_t pi = (size_t)(std::upper_bound(pstart.begin(), pstart.end(), g0) - pstart.begin()) - 1;
        size_t q = (size_t)(std::upper_bound(cut.begin(), cut.end(), g0) - cut.begin()) - 1;
        size_t g = g0;
        while (g < g1) {
            const Piece& P = pieces[pi];
            const size_t e = std::min(g1, pstart[pi + 1]);
            while (g < e) {
                while (q + 1 < cut.size() && cut[q + 1] <= g) q++;
                const size_t lim = q + 1 < cut.size() ? std::min(e, cut[q + 1]) : e;
                const uint64_t sub = cut_base[q];
                size_t i = P.i0 + (g - pstart[pi]);
                if (P.chunk < 0) {
                    for (; g < lim; g++, i++) out[g - g0] = (uint32_t)(seq64[i] - sub);
                } else {
                    const uint32_t* so = chains[P.chunk].so.data();
                    const uint64_t base = (uint64_t)P.chunk * ingest_chunk() - sub;  // mod 2^64
                    for (; g < lim; g++, i++) out[g - g0] = (uint32_t)(base + so[i]);
                }
            }
            pi++;
        }
    }
    // the index as batches of the context (device bytes handed over)
    int finish() {
        const auto tf = std::chrono::steady_clock::now();
        if (given && !cut.empty()) walk_given();
        HIPCHECK(hipMemsetAsync(d + size, 0, 256, c->stream));
        const size_t n = nrec;
        uint32_t* d_offs = nullptr;
        if (c->reuse_ingest) {
            if (std::max<size_t>(n, 1) > c->ar_offs_cap) {
                const uint64_t cap = std::max<uint64_t>(std::max<size_t>(n, 1), c->ar_offs_cap * 3 / 2);
                hipFree(c->ar_offs);
                c->ar_offs = nullptr;
                c->ar_offs_cap = 0;
                if (hipMalloc(&c->ar_offs, cap * 4) != hipSuccess) return FLUERE_E_NOMEM;
                c->ar_offs_cap = cap;
            }
            d_offs = c->ar_offs;
        } else if (hipMalloc(&d_offs, std::max<size_t>(n, 1) * 4) != hipSuccess) {
            return FLUERE_E_NOMEM;
        }
        // batch-relative u32 offsets, written into the staging slots (pinned)
        // a slot's worth at a time, by threads when there are many
        std::vector<size_t> pstart(pieces.size() + 1, 0);
        for (size_t q = 0; q < pieces.size(); q++) pstart[q + 1] = pstart[q] + pieces[q].n;
        const size_t per = ingest_chunk() / 4;
        for (size_t g0 = 0, part = 0; g0 < n; g0 += per, part++) {
            const size_t g1 = std::min(n, g0 + per);
            const int i = (int)(part % nslots);
            if (!pin[i]) {
                if (c->reuse_ingest) {
                    if (!c->ar_pin[i] && hipHostMalloc(&c->ar_pin[i], ingest_chunk(), hipHostMallocDefault) != hipSuccess)
                        return FLUERE_E_NOMEM;
                    if (!c->ar_ev[i] && hipEventCreateWithFlags(&c->ar_ev[i], hipEventDisableTiming) != hipSuccess)
                        return FLUERE_E_HIP;
                    pin[i] = c->ar_pin[i];
                    ev[i] = c->ar_ev[i];
                } else {
                    if (hipHostMalloc(&pin[i], ingest_chunk(), hipHostMallocDefault) != hipSuccess) return FLUERE_E_NOMEM;
                    if (hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess) return FLUERE_E_HIP;
                }
            }
            if (busy[i]) HIPCHECK(hipEventSynchronize(ev[i]));
            uint32_t* out = reinterpret_cast<uint32_t*>(pin[i]);
            const int T = g1 - g0 >= (1u << 20) ? 8 : 1;
            if (T == 1) {
                fill_rel(out, g0, g1, pstart);
            } else {
                std::vector<std::thread> th;
                for (int t = 0; t < T; t++) {
                    const size_t a = g0 + (g1 - g0) * t / T, e = g0 + (g1 - g0) * (t + 1) / T;
                    th.emplace_back([this, out, a, e, g0, &pstart] { fill_rel(out + (a - g0), a, e, pstart); });
                }
                for (auto& x : th) x.join();
            }
            HIPCHECK(hipMemcpyAsync(d_offs + g0, out, (g1 - g0) * 4, hipMemcpyHostToDevice, c->stream));
            HIPCHECK(hipEventRecord(ev[i], c->stream));
            busy[i] = true;
        }
        HIPCHECK(hipStreamSynchronize(c->stream));  // staging slots free
        if (getenv("FLUERE_HOSTPROF"))
            fprintf(stderr, "[fluere] ingest finish (%llu records, %zu pieces): %.1f ms\n", (unsigned long long)n,
                    pieces.size(), 1e3 * std::chrono::duration<double>(std::chrono::steady_clock::now() - tf).count());
        for (int i = 0; i < kIngestSlots; i++) busy[i] = false;
        bool first = true;
        for (size_t q = 0; q < cut.size(); q++) {
            const size_t i0 = cut[q], i1 = q + 1 < cut.size() ? cut[q + 1] : n;
            if (i1 == i0) continue;
            const uint64_t base = cut_base[q];
            // the last batch ends with its last indexed record (pos), not at the
            // end of the file: a corrupt tail after a bad record header is not
            // part of any batch (and cannot push it past the 4 GiB offset range)
            const uint64_t endb = q + 1 < cut.size() ? cut_base[q + 1] : pos;
            HostBatch hb;
            hb.own_bytes = first && !c->reuse_ingest ? d : nullptr;  // one allocation for every batch
            hb.own_offs = first && !c->reuse_ingest ? d_offs : nullptr;
            first = false;
            hb.b.bytes = d + base;
            hb.b.offs = d_offs + i0;
            hb.b.nbytes = endb - base;
            hb.b.n = i1 - i0;
            hb.b.first = c->index_base + c->n_total;
            hb.b.snap = snap;
            hb.b.flags = (sw ? 1u : 0u) | (ns ? 2u : 0u);
            c->batches.push_back(hb);
            c->batches_dirty = true;
            c->census_due = true;
            c->n_total += hb.b.n;
        }
        if (c->reuse_ingest) {
            d = nullptr;  // the arena's
        } else if (first) {  // no records: nothing attached
            hipFree(d_offs);
        } else {
            d = nullptr;  // owned by the first batch now
        }
        c->have_results = false;
        return FLUERE_OK;
    }
};

// A classic pcap image with its record offsets known (live batches).
static int add_host_pcap_indexed(fluere_ctx* c, const uint8_t* file, uint64_t nbytes, const uint64_t* rec_off,
                                 uint64_t n_recs) {
    Ingest in(c);
    in.src = file;
    in.given = rec_off;
    in.given_n = n_recs;
    int rc = in.begin(nbytes);
    if (rc) return rc;
    rc = in.run(nbytes, [&](uint8_t* dst, uint64_t cs, uint64_t len) {
        memcpy(dst, file + cs, len);
        return true;
    });
    return rc ? rc : in.finish();
}

extern "C" int fluere_add_host_pcap(fluere_ctx* c, const uint8_t* file, uint64_t nbytes) {
    if (!c || !file) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    if (is_pcapng(file, nbytes)) {  // libpcap reads pcapng too (pcapng.h)
        std::vector<uint8_t> classic;
        const int rc = pcapng_to_pcap(file, nbytes, classic);
        if (rc) return rc;
        return fluere_add_host_pcap(c, classic.data(), classic.size());
    }
    Ingest in(c);
    int rc = in.begin(nbytes);
    if (rc) return rc;
    rc = in.run(nbytes, [&](uint8_t* dst, uint64_t cs, uint64_t len) {
        memcpy(dst, file + cs, len);
        return true;
    });
    if (!rc) rc = in.finish();
    return rc ? rc : prepare_capture(c);
}

// File ingress for fluere_offline_file: read() straight into the pinned
// staging chunks (no intermediate copy of the capture in host memory).
extern "C" int fluere_add_pcap_file(fluere_ctx* c, const char* path) {
    if (!c || !path) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return FLUERE_E_IO;
    struct stat stt;
    if (fstat(fd, &stt) != 0) { close(fd); return FLUERE_E_IO; }
    const uint64_t nbytes = (uint64_t)stt.st_size;
    {
        uint8_t head[4] = {0, 0, 0, 0};
        if (nbytes >= 4 && pread(fd, head, 4, 0) == 4 && is_pcapng(head, 4)) {
            // pcapng: read whole, rewrite as a classic image (pcapng.h)
            std::vector<uint8_t> raw(nbytes);
            uint64_t got = 0;
            while (got < nbytes) {
                const ssize_t r = pread(fd, raw.data() + got, nbytes - got, (off_t)got);
                if (r <= 0) { close(fd); return FLUERE_E_IO; }
                got += (uint64_t)r;
            }
            close(fd);
            return fluere_add_host_pcap(c, raw.data(), nbytes);
        }
    }
    Ingest in(c);
    int rc = in.begin(nbytes);
    if (!rc)
        rc = in.run(nbytes, [&](uint8_t* dst, uint64_t cs, uint64_t len) {
            uint64_t got = 0;
            while (got < len) {
                const ssize_t r = pread(fd, dst + got, len - got, (off_t)(cs + got));
                if (r <= 0) return false;
                got += (uint64_t)r;
            }
            return true;
        });
    close(fd);
    if (!rc) rc = in.finish();
    return rc ? rc : prepare_capture(c);
}

static int upload_batches(fluere_ctx* c) {
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
static int census(fluere_ctx* c) {
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
    HIPCHECK(hipStreamSynchronize(c->stream));
    return FLUERE_OK;
}

// A pass = k_cleanup -> per batch (k_parse_agg, k_merge_partials) -> k_finalize
// -> one device->host copy of the run counters.  plan_pass does every
// allocation and computes every launch argument; enqueue_pass only launches,
// so a pass can be captured into a hipGraph and replayed while its plan is
// unchanged (byte-equal).
constexpr int PLAN_BATCHES = 8;
static int ensure_recs(fluere_ctx* c, uint64_t need);
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
    int phash;     // 1: the hot pass writes the per-packet filter words (AggArgs::phash)
    int pid;       // 1: the merge writes each packet's flow over them (AggArgs::pid; k_parse_spill runs)
    int clean;     // 1: the pass starts with k_cleanup (0: the last fluere_run already cleared its flows)
    int spec;      // 1: k_finalize publishes the counters to the host itself, a speculative k_cleanup follows
    CleanArgs spec_ca;
    unsigned spec_grid;
    int finalize;  // fluere_run: k_finalize + counters copy
    FinArgs fa;
    unsigned fin_grid;
    Ctl* h_ctl;
    Glob* d_glob;
};

// Bytes of the hot kernel's staging area for one batch (Stage layout).
// Capacity of an owner segment (records per set and owner): a window's
// packets spread over the owners by hash, with 25 % headroom; bounded so
// record indices of the segments fit u32 (k_merge_partials' set tables).
static uint32_t owner_cap(size_t sets, uint32_t O) {
    const char* force = getenv("FLUERE_OWNER_CAP");  // tests: a small capacity sends spills to the overflow list
    uint64_t cap = force ? (uint64_t)std::max(1, atoi(force)) : (uint64_t)SPILL_WG / O * 5 / 4 + 32;
    while (cap > 16 && (uint64_t)sets * O * cap >= (1ull << 32)) cap /= 2;
    return (uint32_t)cap;
}

// k_slow's sets (one per SLOW_SET slow-list entries of a batch of n packets)
// and their owner-segment capacity, after `sets` hot sets; 0 sets when the
// record indices would not fit u32 (the merge tail then takes the slow list).
static void slow_shape(uint64_t n, size_t sets, uint32_t O, uint32_t& n_slow_sets, uint32_t& cap_s) {
    n_slow_sets = (uint32_t)((n + SLOW_SET - 1) / SLOW_SET);
    const char* force = getenv("FLUERE_OWNER_CAP");  // tests: a small capacity sends records to the overflow list
    cap_s = force ? (uint32_t)std::max(1, atoi(force)) : SLOW_SET / O * 5 / 4 + 32;
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
    // per-owner LDS bins shrink as owners grow (BIN = 4096 / O records), and
    // at 2048 owners the 2-record bins cost realistic TCP (847k flows) 85 us of
    // hot kernel over 1024 owners (827 flows each); 1M flows at 1024 owners
    // (977 each) overflow the merge tables and cost 0.5 ms (r03ah)
    static const uint32_t o_min = getenv("FLUERE_MIN_OWNERS") ? (uint32_t)atoi(getenv("FLUERE_MIN_OWNERS")) : 256u;
    uint32_t o = o_min;
    while (o < (uint32_t)MAX_OWNERS && c->last_nf > 870ull * o) o *= 2;
    static const int o_max = getenv("FLUERE_MAX_OWNERS") ? atoi(getenv("FLUERE_MAX_OWNERS")) : MAX_OWNERS;  // diagnostics
    const int cap = std::min(o_max, c->use_mac ? std::min(FLUERE_MAC_OWNERS, MAX_OWNERS) : MAX_OWNERS);
    // a power of two: k_parse_spill writes a wave's completed bins in groups of
    // 64 / (2 * BIN) lanes with BIN = 4096 / O (a CU count such as 304 rounds up)
    uint32_t r = (uint32_t)std::max(1, std::min(std::max((int)o, c->n_cu), cap));
    while (r & (r - 1)) r += r & (~r + 1);
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
    a.slow_n = &c->d_glob->n_slow;
    a.slow_abl = getenv("FLUERE_SLOW_ABL") ? atoi(getenv("FLUERE_SLOW_ABL")) : 0;
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
    size_t need_max = 0;
    for (auto& hb : c->batches) {
        if (!hb.b.n) continue;
        uint64_t want = (hb.b.n + BLOCK * 8 - 1) / (BLOCK * 8);
        unsigned grid = slow_all ? 0u : (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)c->n_cu));
        const uint64_t per = (hb.b.n + std::max(grid, 1u) - 1) / std::max(grid, 1u);
        const uint64_t steps = (per + BLOCK - 1) / BLOCK;
        const uint32_t W = (uint32_t)std::max<uint64_t>(1, (steps + WIN_ITERS - 1) / WIN_ITERS);
        const size_t sets = (size_t)grid * W, cells = sets * NS;
        const uint32_t O = merge_owners(c);
        need_max = std::max(need_max, stage_bytes(cells, sets, O, grid, hb.b.n, c->use_mac, a.slow_kernel != 0));
    }
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
        const size_t all = sets + n_slow_sets;
        Stage& S = ab.S;
        // layout (16-byte aligned pieces): parts | owner segments (hot, k_slow) | spill_raw | spill | base | off | soff
        S.part = (Part*)c->d_stage;
        S.cap_o = owner_cap(sets, O);
        S.cap_s = cap_s;
        S.slow_rec0 = (unsigned long long)sets * O * S.cap_o;
        S.dspill = (Spill*)(S.part + cells);
        S.spill_raw = S.dspill + (sets * O * S.cap_o + (size_t)n_slow_sets * O * cap_s) * spill_units(c->use_mac);
        S.spill = S.spill_raw + (size_t)grid * SPILL_WG * spill_units(c->use_mac);
        S.spill_cap = hb.b.n;  // records (32 B, or 64 B with MACs)
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

static int plan_pass(fluere_ctx* c, PassPlan& P, bool finalize) {
    memset(&P, 0, sizeof P);  // byte-comparable (padding included)
    int rc;
    if ((rc = upload_batches(c))) return rc;  // host -> device, only when the batches changed
    if ((rc = census(c))) return rc;          // a new capture: its shape from a sample
    P.ca = CleanArgs{tables_of(c), c->acc, c->d_complex, c->d_active, c->d_glob};
    static const int clean_abl = getenv("FLUERE_CLEAN_ABL") ? atoi(getenv("FLUERE_CLEAN_ABL")) : 0;
    P.ca.abl = clean_abl;
    P.ca.bulk = bulk_clean(c, c->prev_nf == ~0ull ? c->last_nf : c->prev_nf);
    // cleanup grid: the last fetched run's flow count when known (k_cleanup is
    // grid-stride over the device count, so any grid is correct)
    P.clean_grid = done_grid(c, c->prev_nf == ~0ull ? c->fmax : c->prev_nf);
    P.tab_words = (size_t)N_TABLES * 2 * (c->C + 1);
    P.clean = c->precleaned ? 0 : 1;
    P.spill = spill_mode(c);
    if ((rc = plan_batches(c, P))) return rc;
    static const int abl = getenv("FLUERE_ABLATE") ? atoi(getenv("FLUERE_ABLATE")) : 0;
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
    for (int i = 0; i < P.nb; i++) {
        const AggArgs& a = P.agg[i];
        if (i > 0) HIPCHECK(hipMemsetAsync(&c->d_glob->n_slow, 0, 40, s));  // n_slow, n_spill, n_dspill, n_gen, n_owner (k_cleanup zeroed them for batch 0)
        const unsigned grid = P.agg_grid[i];
        const void* fn = P.spill ? (P.macs ? (const void*)k_parse_spill<true> : (const void*)k_parse_spill<false>)
                       : P.macs ? (const void*)k_parse_agg<0, true>
                         : P.abl == 1 ? (const void*)k_parse_agg<1, false>
                         : P.abl == 2 ? (const void*)k_parse_agg<2, false>
                         : P.abl == 3 ? (const void*)k_parse_agg<3, false>
                         : P.abl == 4 ? (const void*)k_parse_agg<4, false>
                         : P.abl == 5 ? (const void*)k_parse_agg<5, false>
                                      : (const void*)k_parse_agg<0, false>;
        // HIP events carried by the dispatch itself (start / stop timestamps of
        // the hot kernel): separate event markers would each add a gap to the
        // stream.  The first batch of a multi-batch pass starts evk_first.
        void* args[] = {const_cast<AggArgs*>(&a)};
        static const bool hostprof = getenv("FLUERE_HOSTPROF") != nullptr;
        const auto t0 = std::chrono::steady_clock::now();
        hipEvent_t e0 = (i == 0 && P.nb > 1) ? c->evk_first : c->evk0;
        if (grid)
            HIPCHECK(hipExtLaunchKernel(fn, dim3(grid), dim3(BLOCK), args, 0, s, e0, c->evk1, 0));
        const auto t1 = std::chrono::steady_clock::now();
        // the slow list into k_slow's owner segments, before the merge reads them
        // (every packet without a hot kernel: k_slow carries the timing events)
        if (a.slow_kernel) {
            if (a.v6.C) HIPCHECK(hipMemsetAsync(a.v6.tab[0], 0xFF, (size_t)(a.v6.C + 1) * 3 * 8, s));  // every key EMPTY
            if (grid) {
                k_slow<<<P.slow_grid[i], SB, 0, s>>>(a);
            } else {
                HIPCHECK(hipExtLaunchKernel((const void*)k_slow, dim3(P.slow_grid[i]), dim3(SB), args, 0, s, e0, c->evk1,
                                            0));
            }
        }
        // at most one merge workgroup per CU, each taking owners in turn
        if (P.macs) k_merge_partials<true><<<std::min<uint32_t>(P.owners[i], (uint32_t)c->n_cu), MB, 0, s>>>(a);
        else k_merge_partials<false><<<std::min<uint32_t>(P.owners[i], (uint32_t)c->n_cu), MB, 0, s>>>(a);  // + the slow list (unless k_slow took it)
        if (hostprof) {
            const auto t2 = std::chrono::steady_clock::now();
            auto us = [](auto x, auto y) { return std::chrono::duration<double, std::micro>(y - x).count(); };
            fprintf(stderr, "[fluere] launch: hot %.1f merge %.1f us\n", us(t0, t1), us(t1, t2));
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
        if (i > 0) {
            hipMemsetParams mp{};
            mp.dst = &c->d_glob->n_slow;
            mp.elementSize = 4;
            mp.width = 10;  // n_slow, n_spill, n_dspill, n_gen, n_owner
            mp.height = 1;
            mp.pitch = 16;
            mp.value = 0;
            ok = hipGraphAddMemsetNode(&n, g, &prev, 1, &mp) == hipSuccess;
            prev = n;
        }
        if (i == 0 && P.nb > 1) event(c->evk_first);
        event(c->evk0);
        a_agg[i][0] = &P.agg[i];
        const void* fn = P.spill ? (P.macs ? (const void*)k_parse_spill<true> : (const void*)k_parse_spill<false>)
                       : P.macs ? (const void*)k_parse_agg<0, true>
                                : P.abl == 1 ? (const void*)k_parse_agg<1, false>
                                : P.abl == 2 ? (const void*)k_parse_agg<2, false>
                                : P.abl == 3 ? (const void*)k_parse_agg<3, false>
                                : P.abl == 4 ? (const void*)k_parse_agg<4, false>
                                : P.abl == 5 ? (const void*)k_parse_agg<5, false>
                                             : (const void*)k_parse_agg<0, false>;
        if (P.agg_grid[i]) kernel(fn, P.agg_grid[i], BLOCK, a_agg[i]);
        if (P.agg_grid[i]) event(c->evk1);
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
        if (!P.agg_grid[i]) event(c->evk1);
        kernel(P.macs ? (const void*)k_merge_partials<true> : (const void*)k_merge_partials<false>,
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

// First-batch start event of the last pass (evk0 itself for one batch).
static hipEvent_t pass_start_event(fluere_ctx* c) { return c->plan_nb > 1 ? c->evk_first : c->evk0; }

static void debug_counters(fluere_ctx* c, const Glob* have = nullptr) {
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

static int init_glob(fluere_ctx* c) {
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
    static const bool keep = getenv("FLUERE_KEEP_DICT") != nullptr;
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
    if ((rc = plan_batches(c, P, false))) return rc;
    if (P.nb > PLAN_BATCHES) return FLUERE_E_ARG;
    static const int abl = getenv("FLUERE_ABLATE") ? atoi(getenv("FLUERE_ABLATE")) : 0;
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

// Duration of the last k_parse_agg launch (HIP events on the context stream).
extern "C" double fluere_last_kernel_ms(fluere_ctx* c) {
    if (!c) return -1.0;
    float ms = -1.0f;
    if (hipEventSynchronize(c->evk1) != hipSuccess) return -1.0;
    if (hipEventElapsedTime(&ms, c->evk0, c->evk1) != hipSuccess) return -1.0;
    return ms;
}

// Duration of the last pass: after fluere_run, its host wall time (submission
// to results); after fluere_parse_aggregate, the device time of its hot
// kernel launches (HIP events on the context stream; no other markers).
extern "C" double fluere_last_pass_ms(fluere_ctx* c) {
    if (!c) return -1.0;
    float ms = -1.0f;
    if (c->pass_in_run) return c->last_run_ms;
    if (hipEventSynchronize(c->evk1) != hipSuccess) return -1.0;
    if (hipEventElapsedTime(&ms, pass_start_event(c), c->evk1) != hipSuccess) return -1.0;
    return ms;
}

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

static int ord_scratch(fluere_ctx* c, size_t need) {
    if (need <= c->d_ord_bytes) return FLUERE_OK;
    hipFree(c->d_ord);
    c->d_ord = nullptr;
    c->d_ord_bytes = 0;
    if (hipMalloc(&c->d_ord, need) != hipSuccess) return FLUERE_E_NOMEM;
    c->d_ord_bytes = need;
    return FLUERE_OK;
}

static int grow_pair(void** a, void** b, uint64_t* cap_b, uint64_t cap_a, size_t unit) {
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

static int sort_actives(fluere_ctx* c, uint64_t ne, uint64_t m) {
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

// Orders the run's n records in d_recs (n_ended of them ended) as
// [ended][active]; Mode B with the order words in d_recaux.  Stream-ordered;
// Mode B reads its largest group (records ending at one packet) once.
// n_okey: the run's Glob::n_okey (the order-key array holds every record's
// key when it equals n).
static int order_records(fluere_ctx* c, uint64_t n, uint64_t n_ended, bool mode_b, uint64_t n_okey) {
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
        if (g > 1024) return FLUERE_OK;  // (fetch_records orders them on the host)
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

// The attached capture made ready for its first pass, at attach time (not in
// live sessions, whose batches are their runs): the chunk descriptors, the
// census (k_census), and every buffer the first pass would otherwise allocate
// while the GPU waits, sized from the census -- the staging of the owner count
// and hot kernel it implies, the slow list, the filter words, the record
// buffers for its flow estimate, the exact engine's arena when TCP is present,
// the ordering scratch.  A failed reservation is retried by the run itself.
static int prepare_capture(fluere_ctx* c) {
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
        (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tb, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)(N + 1),
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

static int ensure_recs(fluere_ctx* c, uint64_t need) {
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
    // device timing: evk0 / evk1 around the hot kernel only (each event marker
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
        for (size_t i = 0; i < all.size(); i += PLAN_BATCHES) {
            c->batches.assign(all.begin() + i, all.begin() + std::min(all.size(), i + PLAN_BATCHES));
            PassPlan Q;
            memset(&Q, 0, sizeof Q);
            Q.macs = P.macs;
            Q.abl = P.abl;
            Q.spill = P.spill;
            rc = plan_batches(c, Q, false);
            if (!rc) rc = enqueue_batches(c, Q);
            if (rc) break;
        }
        c->batches = all;
        c->batches_dirty = true;
        if (rc) return rc;
        c->plan_nb = 1;  // device timing covers the last chunk only
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
        HIPCHECK(hipStreamSynchronize(s));
        g = c->h_ctl->g;
        nf_err[0] = c->h_ctl->n_flows;
        nf_err[1] = c->h_ctl->err;
        c->prev_nf = (nf_err[1] & (ERR_TABLE_FULL | ERR_SPIN)) ? ~0ull : nf_err[0];
    }
    const auto t_sync = std::chrono::steady_clock::now();
    // the speculative cleanup behind the copy clears the flows exactly when
    // the run needs no more device work (the same test, on the same counters)
    const bool spec_cleared = P.spec && run_complete(g, nf_err[1], P.spec_ca.timeout_us, P.spec_ca.recs_cap);
    if (!(nf_err[1] & (ERR_TABLE_FULL | ERR_SPIN))) c->last_nf = nf_err[0];
    // (a pass of k_slow over every packet lists none: the prediction stays)
    c->last_n_slow = c->plan_slow_all ? std::max<uint64_t>(g.n_slow, c->n_total) : g.n_slow;
    debug_counters(c, &g);
    FinArgs fa = P.fa;
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
            if (P.phash) {
                J.phash = c->d_phash;
                J.phash_base = c->index_base;
                J.emap = P.pid ? c->d_emap : nullptr;
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
        if ((rc = order_records(c, n_rec, n_ended, false, g.n_okey))) return rc;
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
        if (P.pid) {  // every valid packet's flow from the merge (AggArgs::pid)
            J.phash = c->d_phash;
            J.phash_base = c->index_base;
            J.emap = c->d_emap;
        }
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
        HIPCHECK(hipStreamSynchronize(s));
        n_rec = g.n_rec;
        n_ended = g.n_heads;
        c->recs.resize(n_rec);
        if (n_rec)
            HIPCHECK(hipMemcpyAsync(c->recs.data(), c->d_recs, n_rec * sizeof(fluere_record), hipMemcpyDeviceToHost, s));
        HIPCHECK(hipEventRecord(c->ev2, s));
        HIPCHECK(hipStreamSynchronize(s));
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
        const hipError_t e = hipEventElapsedTime(&ms_parse, pass_start_event(c), c->evk1);
        if (e != hipSuccess && getenv("FLUERE_HIP_VERBOSE"))
            fprintf(stderr, "[fluere] parse timing events: %s\n", hipGetErrorString(e));
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
    hipcub::DeviceScan::ExclusiveSum(nullptr, tb, lens, d_offsets, (int)n, s);
    if (hipMalloc(&tmp, std::max<size_t>(tb, 16)) != hipSuccess) { hipFree(lens); return FLUERE_E_NOMEM; }
    hipcub::DeviceScan::ExclusiveSum(tmp, tb, lens, d_offsets, (int)n, s);
    k_synth_write<<<grid_for(n, 256), 256, 0, s>>>(*cfg, first, n, d_bytes, d_offsets);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(s));
    hipFree(tmp);
    hipFree(lens);
    return FLUERE_OK;
}

// ---------------------------------------------------------------------------
// multi-GPU merge
// ---------------------------------------------------------------------------
extern "C" uint64_t fluere_capacity(fluere_ctx* c) { return c ? c->fmax : 0; }
extern "C" uint64_t fluere_total_packets(fluere_ctx* c) { return c ? c->n_total : 0; }

extern "C" int fluere_set_index_base(fluere_ctx* c, uint64_t base) {
    if (!c) return FLUERE_E_ARG;
    if (!c->batches.empty()) return FLUERE_E_STATE;
    c->index_base = base;
    return FLUERE_OK;
}

extern "C" uint64_t fluere_shard_block_bytes(uint64_t cap, uint64_t cap_annex) {
    return sizeof(fluere_shard_header) + cap * sizeof(fluere_flow_summary) + cap_annex * sizeof(fluere_flow_annex);
}

// Record buffer of at least `need` records, keeping the first `keep`.
static int grow_recs_keep(fluere_ctx* c, uint64_t need, uint64_t keep) {
    if (need <= c->d_recs_cap) return FLUERE_OK;
    fluere_record* nr = nullptr;
    const uint64_t cap = std::max<uint64_t>(need, 1024);
    if (hipMalloc(&nr, cap * sizeof(fluere_record)) != hipSuccess) return FLUERE_E_NOMEM;
    if (keep) HIPCHECK(hipMemcpyAsync(nr, c->d_recs, keep * sizeof(fluere_record), hipMemcpyDeviceToDevice, c->stream));
    HIPCHECK(hipStreamSynchronize(c->stream));
    hipFree(c->d_recs);
    c->d_recs = nr;
    c->d_recs_cap = cap;
    return FLUERE_OK;
}

extern "C" int fluere_export_device(fluere_ctx* c, void* d_blocks, uint32_t n_owners, uint32_t shard, uint64_t cap,
                                    uint64_t cap_annex, uint64_t* need, uint64_t* need_annex) {
    if (!c || !d_blocks || !n_owners || !cap) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    int rc;
    if ((rc = upload_batches(c))) return rc;
    const TableSet T = tables_of(c);
    const int nb = (int)c->batches.size();
    if (!c->d_annex_of && hipMalloc(&c->d_annex_of, (size_t)c->fmax * 4) != hipSuccess) return FLUERE_E_NOMEM;
    if (!c->d_sumpos && hipMalloc(&c->d_sumpos, (size_t)c->fmax * 4) != hipSuccess) return FLUERE_E_NOMEM;
    if (!c->d_need && hipMalloc(&c->d_need, 16) != hipSuccess) return FLUERE_E_NOMEM;
    FinArgs fa{c->d_batches, nb, T, c->acc, c->d_glob, nullptr, c->d_complex, c->use_mac};
    // 1. flows whose part of the state machine depends on packet order here
    reset_record_counters(c);
    k_local_cert<<<flow_grid(c), 256, 0, s>>>(fa, c->d_annex_of);
    // 3. summaries (+ annexes) into the owners' blocks, enqueued behind it
    //    speculatively: with no order-dependent flow (the common case) the
    //    export needs ONE host round trip
    ExportArgs ea{fa, (uint8_t*)d_blocks, n_owners, shard, cap, cap_annex, fluere_shard_block_bytes(cap, cap_annex),
                  c->d_annex_of, (const fluere_flow_annex*)c->d_annex, c->d_sumpos};
    auto enqueue_export = [&](bool annexes) -> int {
        ea.annex = annexes ? (const fluere_flow_annex*)c->d_annex : nullptr;
        k_export_hdr<<<grid_for(n_owners, 64), 64, 0, s>>>(ea);
        k_export_owners<<<flow_grid(c), 256, 0, s>>>(ea);
        k_export_need<<<1, 64, 0, s>>>(ea, (unsigned long long*)c->d_need, nullptr);
        HIPCHECK(hipGetLastError());
        return FLUERE_OK;
    };
    if ((rc = enqueue_export(false))) return rc;
    struct {
        Ctl ctl;
        unsigned long long nd[2];
    } back;
    HIPCHECK(hipMemcpyAsync(&back.ctl, c->d_glob, sizeof back.ctl, hipMemcpyDeviceToHost, s));
    HIPCHECK(hipMemcpyAsync(back.nd, c->d_need, 16, hipMemcpyDeviceToHost, s));
    HIPCHECK(hipStreamSynchronize(s));
    Glob g = back.ctl.g;
    if (!(back.ctl.err & (ERR_TABLE_FULL | ERR_SPIN))) c->last_nf = back.ctl.n_flows;  // (merge owner estimate)
    // 2. order-dependent flows: their annexes (and the records that open and
    //    close in this shard) from the exact state machine, then the export again
    if (g.n_complex) {
        std::vector<Batch> hb(nb);
        for (int i = 0; i < nb; i++) hb[i] = c->batches[i].b;
        ExactJob J{c->d_batches, hb.data(), nb, T, c->use_mac, 0, c->timeout_ms * 1000ull, c->d_complex, c->d_glob,
                   &c->d_recs, &c->d_recs_cap, &c->d_exact, &c->d_exact_bytes,
                   1, &c->d_annex, &c->d_annex_cap, c->d_annex_of};
        J.mail = c->h_mail;
        ExactResult er{};
        if ((rc = exact_run(J, s, &er))) return rc < 0 ? rc : FLUERE_E_HIP;
        if ((rc = enqueue_export(true))) return rc;
        HIPCHECK(hipMemcpyAsync(&g, c->d_glob, sizeof g, hipMemcpyDeviceToHost, s));
        HIPCHECK(hipMemcpyAsync(back.nd, c->d_need, 16, hipMemcpyDeviceToHost, s));
        HIPCHECK(hipStreamSynchronize(s));
    }
    if (need) *need = back.nd[0];
    if (need_annex) *need_annex = back.nd[1];
    // the final records this shard produced (kept through the merge)
    c->local_n_rec = g.n_rec;
    c->local_updates = g.n_updates;
    c->local_ended = g.n_ended;
    return FLUERE_OK;
}

// The common-case export without a host round trip: the certificate and the
// summaries (no annexes) are enqueued, and d_info (device, 4 x u64) receives
// {largest per-owner summary count, annex count, order-dependent flows, flow
// count}.  The caller reduces d_info over the ranks (MAX) on the context's
// stream and reads it once; if any rank has order-dependent flows, every rank
// runs fluere_export_device instead (annexes), and blocks that were too small
// are exported again with larger capacities.
extern "C" int fluere_export_async(fluere_ctx* c, void* d_blocks, uint32_t n_owners, uint32_t shard, uint64_t cap,
                                   uint64_t cap_annex, unsigned long long* d_info) {
    if (!c || !d_blocks || !n_owners || !cap || !d_info) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    int rc;
    if ((rc = upload_batches(c))) return rc;
    const int nb = (int)c->batches.size();
    if (!c->d_annex_of && hipMalloc(&c->d_annex_of, (size_t)c->fmax * 4) != hipSuccess) return FLUERE_E_NOMEM;
    if (!c->d_sumpos && hipMalloc(&c->d_sumpos, (size_t)c->fmax * 4) != hipSuccess) return FLUERE_E_NOMEM;
    if (!c->d_need && hipMalloc(&c->d_need, 16) != hipSuccess) return FLUERE_E_NOMEM;
    FinArgs fa{c->d_batches, nb, tables_of(c), c->acc, c->d_glob, nullptr, c->d_complex, c->use_mac};
    reset_record_counters(c);
    k_local_cert<<<flow_grid(c), 256, 0, s>>>(fa, c->d_annex_of);
    ExportArgs ea{fa, (uint8_t*)d_blocks, n_owners, shard, cap, cap_annex, fluere_shard_block_bytes(cap, cap_annex),
                  c->d_annex_of, nullptr, c->d_sumpos};
    k_export_hdr<<<grid_for(n_owners, 64), 64, 0, s>>>(ea);
    k_export_owners<<<flow_grid(c), 256, 0, s>>>(ea);
    k_export_need<<<1, 64, 0, s>>>(ea, (unsigned long long*)c->d_need, d_info);
    HIPCHECK(hipGetLastError());
    c->local_n_rec = c->local_updates = c->local_ended = 0;  // (no order-dependent flow: no local record)
    // the shard's flow count, for the next pass's owner count: read after the
    // merge's wait (a spare word of the pinned control copy)
    HIPCHECK(hipMemcpyAsync(&c->h_ctl->pad[0], c->d_nflows, 4, hipMemcpyDeviceToHost, s));
    c->async_nf = true;
    return FLUERE_OK;
}

// ---- the compact wire encoding (include/fluere_gpu.h) -------------------------
extern "C" uint64_t fluere_wire_bound(uint64_t cap, uint64_t cap_annex) {
    return sizeof(fluere_shard_header) + ((4 * cap + 15) & ~15ull) + ((cap * WIRE_REC_MAX + 15) & ~15ull) +
           cap_annex * sizeof(fluere_flow_annex);
}

extern "C" int fluere_wire_pack(fluere_ctx* c, const void* d_blocks, uint32_t n_owners, uint64_t cap, uint64_t cap_annex,
                                void* d_wire, unsigned long long* d_sizes) {
    if (!c || !d_blocks || !d_wire || !d_sizes || !n_owners || !cap) return FLUERE_E_ARG;
    if (cap * WIRE_REC_MAX >= (1ull << 32)) return FLUERE_E_ARG;  // u32 record offsets within a block
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const uint64_t n = (uint64_t)n_owners * cap;
    size_t tb = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tb, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                           (int)(n + 1), s);
    const size_t need = 2 * (n + 1) * 8 + (size_t)(n_owners + 1) * 8 + ((tb + 255) & ~(size_t)255);
    if (need > c->d_wire_tmp_bytes) {
        hipFree(c->d_wire_tmp);
        c->d_wire_tmp = nullptr;
        c->d_wire_tmp_bytes = 0;
        if (hipMalloc(&c->d_wire_tmp, need) != hipSuccess) return FLUERE_E_NOMEM;
        c->d_wire_tmp_bytes = need;
    }
    WireArgs a{};
    a.blocks = (const uint8_t*)d_blocks;
    a.wwire = (uint8_t*)d_wire;
    a.cap = cap;
    a.cap_annex = cap_annex;
    a.block_bytes = fluere_shard_block_bytes(cap, cap_annex);
    a.n_blocks = n_owners;
    char* t = (char*)c->d_wire_tmp;
    void* tmp = t;
    a.sz = (unsigned long long*)(t + ((tb + 255) & ~(size_t)255));
    a.scan = a.sz + (n + 1);
    a.woff = a.scan + (n + 1);
    a.sizes = d_sizes;
    k_wire_size<<<grid_for(n + 1, 256), 256, 0, s>>>(a);
    HIPCHECK(hipcub::DeviceScan::ExclusiveSum(tmp, tb, a.sz, a.scan, (int)(n + 1), s));
    k_wire_offsets<<<1, 64, 0, s>>>(a);
    k_wire_pack<<<grid_for(n, 256), 256, 0, s>>>(a);
    const unsigned ax = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(64, cap_annex * 32 / 256));
    k_wire_annex<<<dim3(ax, n_owners), 256, 0, s>>>(a, 0);
    HIPCHECK(hipGetLastError());
    return FLUERE_OK;
}

extern "C" int fluere_wire_unpack(fluere_ctx* c, const void* d_wire, uint32_t n_shards, const uint64_t* sizes,
                                  uint64_t cap, uint64_t cap_annex, void* d_blocks) {
    if (!c || !d_wire || !d_blocks || !sizes || !n_shards || n_shards > WIRE_MAX_BLOCKS || !cap) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    WireArgs a{};
    a.wire = (const uint8_t*)d_wire;
    a.wblocks = (uint8_t*)d_blocks;
    a.cap = cap;
    a.cap_annex = cap_annex;
    a.block_bytes = fluere_shard_block_bytes(cap, cap_annex);
    a.n_blocks = n_shards;
    unsigned long long off = 0;
    for (uint32_t b = 0; b < n_shards; b++) {
        if (sizes[b] < sizeof(fluere_shard_header)) return FLUERE_E_ARG;
        a.off_h[b] = off;
        off += sizes[b];
    }
    a.off_h[n_shards] = off;
    const uint64_t n = (uint64_t)n_shards * cap;
    k_wire_unpack<<<grid_for(n, 256), 256, 0, s>>>(a);
    const unsigned ax = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(64, cap_annex * 32 / 256));
    k_wire_annex<<<dim3(ax, n_shards), 256, 0, s>>>(a, 1);
    HIPCHECK(hipGetLastError());
    return FLUERE_OK;
}

extern "C" int fluere_merge_gathered(fluere_ctx* c, const void* d_blocks, uint32_t n_shards, uint64_t cap,
                                     uint64_t cap_annex, fluere_stats* st) {
    if (!c || (!d_blocks && n_shards) || (n_shards && !cap)) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    int rc;
    const uint64_t n = (uint64_t)n_shards * cap;
    const uint64_t keep = c->local_n_rec;
    if ((rc = clear_flows(c))) return rc;
    c->precleaned = false;
    {   // the records this rank's export produced stay first in d_recs
        const unsigned long long cnt[3] = {keep, c->local_updates, c->local_ended};
        char* gb = (char*)c->d_glob;
        HIPCHECK(hipMemcpyAsync(gb + offsetof(Glob, n_rec), &cnt[0], 8, hipMemcpyHostToDevice, s));
        HIPCHECK(hipMemcpyAsync(gb + offsetof(Glob, n_updates), &cnt[1], 16, hipMemcpyHostToDevice, s));
    }
    if (!c->d_pay && hipMalloc(&c->d_pay, (size_t)c->fmax * sizeof(FirstPay)) != hipSuccess) return FLUERE_E_NOMEM;
    if (std::max<uint64_t>(n, 1) > c->d_sd_cap) {
        hipFree(c->d_sd);
        c->d_sd = nullptr;
        c->d_sd_cap = 0;
        if (hipMalloc(&c->d_sd, std::max<uint64_t>(n, 1) * 4) != hipSuccess) return FLUERE_E_NOMEM;
        c->d_sd_cap = std::max<uint64_t>(n, 1);
    }
    if ((rc = grow_recs_keep(c, keep + std::min<uint64_t>(std::max<uint64_t>(n, 1), c->fmax), keep))) return rc;
    const auto t0 = std::chrono::steady_clock::now();
    const uint32_t seq = ++c->run_seq ? c->run_seq : ++c->run_seq;  // never 0 (the initial value)
    MergeArgs ma{tables_of(c), c->acc, n, c->d_sd, (FirstPay*)c->d_pay, c->d_glob, c->d_recs, c->d_complex,
                 c->d_recs_cap, (const uint8_t*)d_blocks, cap, cap_annex, fluere_shard_block_bytes(cap, cap_annex),
                 c->h_ctl, seq, c->timeout_ms * 1000ull};
    if (n) {
        k_merge_insert<<<grid_for(n, 256), 256, 0, s>>>(ma);
        k_merge_payload<<<grid_for(n, 256), 256, 0, s>>>(ma);
    }
    k_merge_finalize<<<flow_grid(c), 256, 0, s>>>(ma);
    HIPCHECK(hipGetLastError());
    Glob g;
    uint32_t nf_err[2];
    if ((rc = wait_published(c, seq, g, nf_err))) return rc;
    if (c->async_nf) {
        c->last_nf = c->h_ctl->pad[0];
        c->async_nf = false;
    }
    if (nf_err[1] & ERR_CAPACITY) return FLUERE_E_ARG;  // a shard had more flows than its block holds
    if (nf_err[1]) return FLUERE_E_TABLE_FULL;
    const uint64_t timeout_us = c->timeout_ms * 1000ull;
    const bool expiry = g.valid && g.tmax >= g.tmin && g.tmax - g.tmin >= timeout_us;
    if (g.n_complex && !expiry) {
        // the order-dependent flows: compose the shards' pieces in shard order
        unsigned long long *keys = nullptr, *keys2 = nullptr;
        uint32_t *vals = nullptr, *vals2 = nullptr;
        void* tmp = nullptr;
        size_t tb = 0;
        const uint64_t m = n;
        if (hipMalloc(&keys, m * 8) != hipSuccess || hipMalloc(&keys2, m * 8) != hipSuccess ||
            hipMalloc(&vals, m * 4) != hipSuccess || hipMalloc(&vals2, m * 4) != hipSuccess) {
            hipFree(keys); hipFree(keys2); hipFree(vals); hipFree(vals2);
            return FLUERE_E_NOMEM;
        }
        HIPCHECK(hipMemsetAsync(&c->d_glob->n_keys, 0, 8, s));
        k_comp_collect<<<grid_for(n, 256), 256, 0, s>>>(ma, keys, vals);
        unsigned long long nk = 0;
        HIPCHECK(hipMemcpyAsync(&nk, &c->d_glob->n_keys, 8, hipMemcpyDeviceToHost, s));
        HIPCHECK(hipStreamSynchronize(s));
        // records: the certified ones + at most one per shard piece
        if ((rc = grow_recs_keep(c, g.n_rec + 2 * nk, g.n_rec))) return rc;
        ma.out = c->d_recs;
        ma.out_cap = c->d_recs_cap;
        int end_bit = 8;
        while (end_bit < 64 && (1ull << (end_bit - 8)) <= c->fmax) end_bit++;
        (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tb, keys, keys2, vals, vals2, (int)nk, 0, end_bit, s);
        if (hipMalloc(&tmp, std::max<size_t>(tb, 16)) != hipSuccess) {
            hipFree(keys); hipFree(keys2); hipFree(vals); hipFree(vals2);
            return FLUERE_E_NOMEM;
        }
        HIPCHECK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, keys, keys2, vals, vals2, (int)nk, 0, end_bit, s));
        if (nk) k_compose<<<grid_for(nk, 64), 64, 0, s>>>(ma, keys2, vals2, nk);
        HIPCHECK(hipGetLastError());
        HIPCHECK(hipMemcpyAsync(&g, c->d_glob, sizeof g, hipMemcpyDeviceToHost, s));
        HIPCHECK(hipStreamSynchronize(s));
        hipFree(tmp); hipFree(keys); hipFree(keys2); hipFree(vals); hipFree(vals2);
    }
    const uint32_t nf = std::min(nf_err[0], c->fmax);
    c->dev_n_rec = g.n_rec;
    c->host_recs = false;
    c->dev_ordered = false;
    c->have_results = true;
    c->local_n_rec = c->local_updates = c->local_ended = 0;
    fluere_stats out{};
    out.valid = g.valid;
    out.dropped_parse = g.dropped;
    out.flows = nf;
    out.records = g.n_rec;
    out.ended = g.n_ended;
    out.complex_flows = g.n_complex;
    out.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    out.updates = g.n_updates;
    if (st) *st = out;
    // the hard-timeout sweep (offline_fluereflows.rs:161-175): the records
    // come from the sweep composition (fluere_sweep_*), which reads the
    // summary -> flow mapping of this merge
    c->merge_cap = cap;
    c->merge_shards = n_shards;
    c->has_aux = false;
    if (expiry) return FLUERE_NEED_SWEEP;
    return FLUERE_OK;
}

// ---------------------------------------------------------------------------
// sharded Mode B: the hard-timeout sweep composed across shards
// ---------------------------------------------------------------------------
// When the capture's span reaches the timeout, an expiry entry pushed at a
// creation fires at the first *processed* packet of the whole capture with
// t >= exp (offline_fluereflows.rs:103-119,161-175): shards are coupled.  The
// composition (driven by fluere_amd/dist.py):
//   1. every shard (holder) ships the metadata of its valid packets to the
//      keys' owners (32 B each, capture order within an owner): each owner
//      then holds every packet of its keys, in capture order;
//   2. per pass, every holder computes the sweep point of each of its
//      create-eligible packets over the packets processed so far -- first in
//      its own shard (max segment tree over the processed times), else by a
//      query to the first later shard whose latest processed time reaches
//      exp -- and ships the points to the owners, who run the exact chase
//      (exact.hip) and send back which packets were processed; repeated until
//      no owner's processed set changes (the single-GPU fixed point);
//   3. the owners ask the holders for the FluereRecord seeds of the creating
//      packets and build the records; their order stays global (order_key =
//      the ending packet's index plus two order words, fluere_get_record_order).
struct SweepState {
    // holder (this shard's packets)
    ExMeta* hcm = nullptr;              // valid packets, capture order (d = local flow)
    uint64_t hn = 0;
    uint32_t* hperm = nullptr;          // pack position -> local index
    uint8_t* hpr = nullptr;             // processed (local index)
    unsigned long long* hF = nullptr;   // sweep point (local index)
    unsigned long long* tree = nullptr;
    uint64_t P = 0;
    uint32_t* qk = nullptr;             // the local index of each query (grouped by target shard)
    uint64_t nq = 0;
    uint32_t n_owners = 0;
    std::vector<uint64_t> counts;       // packets per owner
    // owner (its keys' packets from every shard)
    ExMeta* ocm = nullptr;
    uint64_t on = 0;
    ExactSession* es = nullptr;
    unsigned long long* req = nullptr;  // creating packets of the instances (ascending)
    uint32_t* reqq = nullptr;           // their instance ordinals
    uint32_t n_inst = 0;
    Seed* seeds = nullptr;              // by instance ordinal
    int passes = 0;
    // scratch
    uint32_t *k1 = nullptr, *k2 = nullptr, *v1 = nullptr;
    unsigned long long* misc = nullptr; // small device scratch (counts)
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    uint32_t* err = nullptr;
};

static void sweep_free(fluere_ctx* c) {
    SweepState* w = c->sw;
    if (!w) return;
    hipFree(w->hcm); hipFree(w->hperm); hipFree(w->hpr); hipFree(w->hF); hipFree(w->tree); hipFree(w->qk);
    hipFree(w->ocm); hipFree(w->req); hipFree(w->reqq); hipFree(w->seeds);
    hipFree(w->k1); hipFree(w->k2); hipFree(w->v1); hipFree(w->misc); hipFree(w->tmp); hipFree(w->err);
    if (w->es) exact_free(w->es);
    delete w;
    c->sw = nullptr;
}

static int sw_tmp(SweepState* w, size_t need) {
    if (need <= w->tmp_bytes) return FLUERE_OK;
    hipFree(w->tmp);
    w->tmp = nullptr;
    w->tmp_bytes = 0;
    if (hipMalloc(&w->tmp, need) != hipSuccess) return FLUERE_E_NOMEM;
    w->tmp_bytes = need;
    return FLUERE_OK;
}

static int bits_for(uint64_t v) {  // radix sort width for keys in [0, v]
    int b = 1;
    while (b < 64 && (v >> b)) b++;
    return b;
}

__global__ void __launch_bounds__(256) k_sw_owner(const ExMeta* cm, uint64_t n, const uint8_t* flow_key,
                                                  uint32_t n_owners, uint32_t* okey, uint32_t* val) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    okey[k] = key_owner(reinterpret_cast<const uint32_t*>(flow_key + (size_t)cm[k].d * 56), n_owners);
    val[k] = (uint32_t)k;
}

// counts[r] = entries equal to r among n sorted keys, r < m
__global__ void k_sw_kcount(const uint32_t* keys, uint64_t n, uint32_t m, unsigned long long* counts) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= m) return;
    auto lb = [&](uint32_t v) {
        uint64_t lo = 0, hi = n;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (keys[mid] < v) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    };
    counts[r] = lb(r + 1) - lb(r);
}

// the packet records for the owners: d = the flow's summary position in its block
__global__ void __launch_bounds__(256) k_sw_pack(const ExMeta* cm, const uint32_t* perm, uint64_t n,
                                                 const uint32_t* sumpos, ExMeta* out) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    ExMeta m = cm[perm[p]];
    m.d = sumpos[m.d];
    out[p] = m;
}

// owner: (shard s, summary position j) -> this context's flow id (the merge's sd)
__global__ void __launch_bounds__(256) k_sw_load(const ExMeta* in, uint64_t n, const unsigned long long* seg,
                                                 uint32_t n_shards, const uint32_t* sd, uint64_t cap, uint32_t fmax,
                                                 ExMeta* out, uint32_t* err) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t sh = 0;
    while (sh + 1 < n_shards && seg[sh + 1] <= i) sh++;
    ExMeta m = in[i];
    const uint32_t d = m.d < cap ? sd[sh * cap + m.d] : FAIL;
    if (d == FAIL || d >= fmax) {
        atomicOr(err, 1u);
        m.d = 0;
    } else {
        m.d = d;
    }
    out[i] = m;
}

__global__ void __launch_bounds__(256) k_sw_feedback(const uint8_t* back, const uint32_t* perm, uint64_t n, uint8_t* pr) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n) pr[perm[p]] = back[p];
}

// sweep point of every create-eligible packet, in this shard or a query
__global__ void __launch_bounds__(256) k_sw_points(const ExMeta* cm, uint64_t n, const unsigned long long* tree,
                                                   uint64_t P, unsigned long long timeout_us, uint32_t rank,
                                                   uint32_t n_ranks, const unsigned long long* maxt,
                                                   unsigned long long* F, uint32_t* tkey, uint32_t* val) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const ExMeta m = cm[k];
    unsigned long long f = NONE64;
    uint32_t target = n_ranks;  // none
    const unsigned long long exp = m.t + timeout_us < m.t ? NONE64 : m.t + timeout_us;
    if ((m.bits & 1) && exp != NONE64) {
        const uint64_t j = tree_first(tree, P, k, exp + 1);
        if (j < n) f = cm[j].gidx;
        else
            for (uint32_t r = rank + 1; r < n_ranks; r++)
                if (maxt[r] >= exp + 1) { target = r; break; }
    }
    F[k] = f;
    tkey[k] = target;
    val[k] = (uint32_t)k;
}

__global__ void __launch_bounds__(256) k_sw_qpack(const ExMeta* cm, const uint32_t* qk, uint64_t nq,
                                                  unsigned long long timeout_us, unsigned long long* q) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nq) q[i] = cm[qk[i]].t + timeout_us;  // (queried only when it does not saturate)
}

__global__ void __launch_bounds__(256) k_sw_answer(const unsigned long long* q, uint64_t nq, const unsigned long long* tree,
                                                   uint64_t P, const ExMeta* cm, uint64_t n, unsigned long long* ans) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq) return;
    const uint64_t j = tree_first(tree, P, 0, q[i] + 1);
    ans[i] = j < n ? cm[j].gidx : NONE64;
}

__global__ void __launch_bounds__(256) k_sw_fill(const unsigned long long* ans, const uint32_t* qk, uint64_t nq,
                                                 unsigned long long* F) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nq) F[qk[i]] = ans[i];
}

__global__ void __launch_bounds__(256) k_sw_fpack(const unsigned long long* F, const uint32_t* perm, uint64_t n,
                                                  unsigned long long* out) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n) out[p] = F[perm[p]];
}

// requests (ascending packet indices) per holder shard: first[r] .. first[r + 1]
__global__ void k_sw_rcount(const unsigned long long* req, uint64_t n, const unsigned long long* first, uint32_t n_ranks,
                            unsigned long long* counts) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_ranks) return;
    auto lb = [&](unsigned long long v) {
        uint64_t lo = 0, hi = n;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (req[mid] < v) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    };
    counts[r] = lb(first[r + 1]) - lb(first[r]);
}

__global__ void __launch_bounds__(256) k_sw_seed(const Batch* bs, int nb, const unsigned long long* req, uint64_t n,
                                                 int macs, Seed* out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Parsed P;
    parse_global(bs, nb, req[i], macs != 0, P);
    fluere_record r;
    fill_seed(r, P);
    Seed sd;
    for (int k = 0; k < 16; k++) { sd.src[k] = r.source[k]; sd.dst[k] = r.destination[k]; }
    sd.sp = r.src_port; sd.dp = r.dst_port;
    sd.v6 = r.src_v6; sd.prot = r.prot; sd.tos = r.tos; sd.pad = 0;
    out[i] = sd;
}

__global__ void __launch_bounds__(256) k_sw_seed_scatter(const Seed* in, const uint32_t* q, uint64_t n, Seed* out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[q[i]] = in[i];
}

static int sw_state(fluere_ctx* c) {
    if (!c->sw) {
        c->sw = new (std::nothrow) SweepState();
        if (!c->sw) return FLUERE_E_NOMEM;
        if (hipMalloc(&c->sw->misc, 4096 * 8) != hipSuccess || hipMalloc(&c->sw->err, 4) != hipSuccess)
            return FLUERE_E_NOMEM;
    }
    return FLUERE_OK;
}

extern "C" int fluere_sweep_pack(fluere_ctx* c, uint32_t n_owners, uint64_t* counts, void* d_send) {
    if (!c || !n_owners || n_owners > 4096 || !counts) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    int rc;
    if ((rc = sw_state(c))) return rc;
    SweepState* w = c->sw;
    if (!d_send || w->n_owners != n_owners || !w->hcm) {
        // (re)index: this shard's valid packets and their owners
        sweep_free(c);
        if ((rc = sw_state(c))) return rc;
        w = c->sw;
        if ((rc = upload_batches(c))) return rc;
        const uint64_t N = c->n_total;
        const uint64_t M = std::max<uint64_t>(N, 1);
        w->P = tree_leaves(M);
        if (hipMalloc(&w->hcm, M * sizeof(ExMeta)) != hipSuccess || hipMalloc(&w->hperm, M * 4) != hipSuccess ||
            hipMalloc(&w->hpr, M) != hipSuccess || hipMalloc(&w->hF, M * 8) != hipSuccess ||
            hipMalloc(&w->tree, 2 * w->P * 8) != hipSuccess || hipMalloc(&w->qk, M * 4) != hipSuccess ||
            hipMalloc(&w->k1, M * 4) != hipSuccess || hipMalloc(&w->k2, M * 4) != hipSuccess ||
            hipMalloc(&w->v1, M * 4) != hipSuccess)
            return FLUERE_E_NOMEM;
        std::vector<Batch> hb(c->batches.size());
        for (size_t i = 0; i < hb.size(); i++) hb[i] = c->batches[i].b;
        ExactJob J{c->d_batches, hb.data(), (int)hb.size(), tables_of(c), c->use_mac, 1, c->timeout_ms * 1000ull,
                   nullptr, c->d_glob, nullptr, nullptr, nullptr, nullptr};
        if ((rc = exact_collect(J, s, w->hcm, &w->hn))) return rc;
        const uint64_t n = w->hn;
        HIPCHECK(hipMemsetAsync(w->misc, 0, n_owners * 8, s));
        if (n) {
            k_sw_owner<<<grid_for(n, 256), 256, 0, s>>>(w->hcm, n, c->d_flow_key, n_owners, w->k1, w->v1);
            size_t tb = 0;
            (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tb, w->k1, w->k2, w->v1, w->hperm, (int)n, 0,
                                                     bits_for(n_owners), s);
            if ((rc = sw_tmp(w, tb))) return rc;
            HIPCHECK(hipcub::DeviceRadixSort::SortPairs(w->tmp, tb, w->k1, w->k2, w->v1, w->hperm, (int)n, 0,
                                                        bits_for(n_owners), s));
            k_sw_kcount<<<grid_for(n_owners, 256), 256, 0, s>>>(w->k2, n, n_owners, w->misc);
            HIPCHECK(hipMemsetAsync(w->hpr, 1, n, s));  // first guess: every valid packet is processed
        }
        w->counts.assign(n_owners, 0);
        HIPCHECK(hipMemcpyAsync(w->counts.data(), w->misc, n_owners * 8, hipMemcpyDeviceToHost, s));
        HIPCHECK(hipGetLastError());
        HIPCHECK(hipStreamSynchronize(s));
        w->n_owners = n_owners;
    }
    for (uint32_t o = 0; o < n_owners; o++) counts[o] = w->counts[o];
    if (d_send && w->hn) {
        k_sw_pack<<<grid_for(w->hn, 256), 256, 0, s>>>(w->hcm, w->hperm, w->hn, c->d_sumpos, (ExMeta*)d_send);
        HIPCHECK(hipGetLastError());
        HIPCHECK(hipStreamSynchronize(s));
    }
    return FLUERE_OK;
}

extern "C" int fluere_sweep_load(fluere_ctx* c, const void* d_recv, uint32_t n_shards, const uint64_t* counts) {
    if (!c || !c->sw || !n_shards || n_shards > 4095 || !counts) return FLUERE_E_ARG;
    if (n_shards != c->merge_shards || !c->d_sd) return FLUERE_E_STATE;
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    SweepState* w = c->sw;
    std::vector<unsigned long long> seg(n_shards + 1, 0);
    for (uint32_t r = 0; r < n_shards; r++) seg[r + 1] = seg[r] + counts[r];
    const uint64_t n = seg[n_shards];
    if (n && !d_recv) return FLUERE_E_ARG;
    hipFree(w->ocm);
    w->ocm = nullptr;
    if (hipMalloc(&w->ocm, std::max<uint64_t>(n, 1) * sizeof(ExMeta)) != hipSuccess) return FLUERE_E_NOMEM;
    w->on = n;
    HIPCHECK(hipMemcpyAsync(w->misc, seg.data(), (n_shards + 1) * 8, hipMemcpyHostToDevice, s));
    HIPCHECK(hipMemsetAsync(w->err, 0, 4, s));
    if (n)
        k_sw_load<<<grid_for(n, 256), 256, 0, s>>>((const ExMeta*)d_recv, n, w->misc, n_shards, c->d_sd,
                                                   c->merge_cap, c->fmax, w->ocm, w->err);
    uint32_t err = 0;
    HIPCHECK(hipMemcpyAsync(&err, w->err, 4, hipMemcpyDeviceToHost, s));
    HIPCHECK(hipStreamSynchronize(s));
    if (err) return FLUERE_E_ARG;  // a packet of a flow the merge does not hold
    if (w->es) exact_free(w->es);
    w->es = nullptr;
    w->passes = 0;
    std::vector<Batch> hb(c->batches.size());
    for (size_t i = 0; i < hb.size(); i++) hb[i] = c->batches[i].b;
    ExactJob J{c->d_batches, hb.data(), (int)hb.size(), tables_of(c), c->use_mac, 1, c->timeout_ms * 1000ull,
               nullptr, c->d_glob, &c->d_recs, &c->d_recs_cap, &c->d_exact, &c->d_exact_bytes};
    J.ext_cm = w->ocm;
    J.ext_n = n;
    J.mail = c->h_mail;
    ExactSession* es = nullptr;
    int rc = exact_begin(J, s, &es);
    w->es = es;
    return rc;
}

extern "C" int fluere_sweep_index(fluere_ctx* c, const uint8_t* d_pr, uint64_t* max_time) {
    if (!c || !c->sw || !max_time) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    SweepState* w = c->sw;
    const uint64_t n = w->hn;
    if (d_pr && n) k_sw_feedback<<<grid_for(n, 256), 256, 0, s>>>(d_pr, w->hperm, n, w->hpr);
    int rc = tree_build(n, w->hcm, w->hpr, w->tree, w->P, s);
    if (rc) return rc;
    unsigned long long root = 0;
    HIPCHECK(hipMemcpyAsync(&root, w->tree + 1, 8, hipMemcpyDeviceToHost, s));
    HIPCHECK(hipStreamSynchronize(s));
    *max_time = n ? root : 0;  // 1 + the latest processed packet's time (0: none)
    return FLUERE_OK;
}

extern "C" int fluere_sweep_queries(fluere_ctx* c, uint32_t n_ranks, uint32_t rank, const uint64_t* max_times,
                                    uint64_t* qcounts, void* d_q) {
    if (!c || !c->sw || !n_ranks || n_ranks > 4095 || rank >= n_ranks || !max_times || !qcounts) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    SweepState* w = c->sw;
    const uint64_t n = w->hn;
    const unsigned long long T = c->timeout_ms * 1000ull;
    if (!d_q) {
        HIPCHECK(hipMemcpyAsync(w->misc, max_times, n_ranks * 8, hipMemcpyHostToDevice, s));
        HIPCHECK(hipMemsetAsync(w->misc + 2048, 0, (n_ranks + 1) * 8, s));
        std::vector<uint64_t> cnt(n_ranks + 1, 0);
        w->nq = 0;
        if (n) {
            k_sw_points<<<grid_for(n, 256), 256, 0, s>>>(w->hcm, n, w->tree, w->P, T, rank, n_ranks, w->misc, w->hF,
                                                         w->k1, w->v1);
            // queries grouped by target shard (n_ranks: none), capture order within one
            size_t tb = 0;
            (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tb, w->k1, w->k2, w->v1, w->qk, (int)n, 0,
                                                     bits_for(n_ranks), s);
            int rc = sw_tmp(w, tb);
            if (rc) return rc;
            HIPCHECK(hipcub::DeviceRadixSort::SortPairs(w->tmp, tb, w->k1, w->k2, w->v1, w->qk, (int)n, 0,
                                                        bits_for(n_ranks), s));
            k_sw_kcount<<<grid_for(n_ranks + 1, 256), 256, 0, s>>>(w->k2, n, n_ranks + 1, w->misc + 2048);
            HIPCHECK(hipGetLastError());
            HIPCHECK(hipMemcpyAsync(cnt.data(), w->misc + 2048, (n_ranks + 1) * 8, hipMemcpyDeviceToHost, s));
            HIPCHECK(hipStreamSynchronize(s));
        }
        for (uint32_t r = 0; r < n_ranks; r++) { qcounts[r] = cnt[r]; w->nq += cnt[r]; }
        return FLUERE_OK;
    }
    for (uint32_t r = 0; r < n_ranks; r++) qcounts[r] = 0;
    uint64_t nq = w->nq;
    if (nq) k_sw_qpack<<<grid_for(nq, 256), 256, 0, s>>>(w->hcm, w->qk, nq, T, (unsigned long long*)d_q);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(s));
    return FLUERE_OK;
}

extern "C" int fluere_sweep_answer(fluere_ctx* c, const void* d_q, uint64_t n, void* d_ans) {
    if (!c || !c->sw || (n && (!d_q || !d_ans))) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    SweepState* w = c->sw;
    if (n)
        k_sw_answer<<<grid_for(n, 256), 256, 0, s>>>((const unsigned long long*)d_q, n, w->tree, w->P, w->hcm, w->hn,
                                                     (unsigned long long*)d_ans);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(s));
    return FLUERE_OK;
}

extern "C" int fluere_sweep_points(fluere_ctx* c, const void* d_ans, void* d_f) {
    if (!c || !c->sw || (c->sw->nq && !d_ans) || (c->sw->hn && !d_f)) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    SweepState* w = c->sw;
    if (w->nq) k_sw_fill<<<grid_for(w->nq, 256), 256, 0, s>>>((const unsigned long long*)d_ans, w->qk, w->nq, w->hF);
    if (w->hn) k_sw_fpack<<<grid_for(w->hn, 256), 256, 0, s>>>(w->hF, w->hperm, w->hn, (unsigned long long*)d_f);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(s));
    return FLUERE_OK;
}

extern "C" int fluere_sweep_chase(fluere_ctx* c, const void* d_f, void* d_pr, int* changed) {
    if (!c || !c->sw || !c->sw->es || !changed) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    SweepState* w = c->sw;
    if (w->on && (!d_f || !d_pr)) return FLUERE_E_ARG;
    if (++w->passes > 64) return FLUERE_E_UNSUPPORTED;  // no fixed point (cannot happen: the system is causal)
    bool ch = false;
    int rc = exact_pass(w->es, (const unsigned long long*)d_f, (uint8_t*)d_pr, &ch);
    *changed = ch ? 1 : 0;
    return rc;
}

extern "C" int fluere_sweep_seed_requests(fluere_ctx* c, uint32_t n_ranks, const uint64_t* rank_first,
                                          uint64_t* counts, void* d_req) {
    if (!c || !c->sw || !c->sw->es || !n_ranks || n_ranks > 4095 || !rank_first || !counts) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    SweepState* w = c->sw;
    if (!d_req) {
        hipFree(w->req); hipFree(w->reqq);
        w->req = nullptr; w->reqq = nullptr;
        const uint64_t M = std::max<uint64_t>(w->on, 1);
        if (hipMalloc(&w->req, M * 8) != hipSuccess || hipMalloc(&w->reqq, M * 4) != hipSuccess) return FLUERE_E_NOMEM;
        int rc = exact_seed_requests(w->es, w->req, w->reqq, &w->n_inst);
        if (rc) return rc;
        HIPCHECK(hipMemcpyAsync(w->misc, rank_first, (n_ranks + 1) * 8, hipMemcpyHostToDevice, s));
        k_sw_rcount<<<grid_for(n_ranks, 256), 256, 0, s>>>(w->req, w->n_inst, w->misc, n_ranks, w->misc + 2048);
        HIPCHECK(hipGetLastError());
        std::vector<unsigned long long> cnt(n_ranks);
        HIPCHECK(hipMemcpyAsync(cnt.data(), w->misc + 2048, n_ranks * 8, hipMemcpyDeviceToHost, s));
        HIPCHECK(hipStreamSynchronize(s));
        uint64_t tot = 0;
        for (uint32_t r = 0; r < n_ranks; r++) { counts[r] = cnt[r]; tot += cnt[r]; }
        if (tot != w->n_inst) return FLUERE_E_ARG;  // a creating packet outside every shard's range
        return FLUERE_OK;
    }
    if (w->n_inst) HIPCHECK(hipMemcpyAsync(d_req, w->req, (size_t)w->n_inst * 8, hipMemcpyDeviceToDevice, s));
    HIPCHECK(hipStreamSynchronize(s));
    return FLUERE_OK;
}

extern "C" int fluere_sweep_seeds(fluere_ctx* c, const void* d_req, uint64_t n, void* d_seeds) {
    if (!c || (n && (!d_req || !d_seeds))) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    int rc;
    if ((rc = upload_batches(c))) return rc;
    if (n)
        k_sw_seed<<<grid_for(n, 256), 256, 0, s>>>(c->d_batches, (int)c->batches.size(), (const unsigned long long*)d_req,
                                                   n, c->use_mac, (Seed*)d_seeds);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(s));
    return FLUERE_OK;
}

extern "C" int fluere_sweep_finish(fluere_ctx* c, const void* d_seeds, fluere_stats* st) {
    if (!c || !c->sw || !c->sw->es) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    SweepState* w = c->sw;
    const uint32_t ni = w->n_inst;
    if (ni && !d_seeds) return FLUERE_E_ARG;
    hipFree(w->seeds);
    w->seeds = nullptr;
    if (hipMalloc(&w->seeds, std::max<uint32_t>(ni, 1) * sizeof(Seed)) != hipSuccess) return FLUERE_E_NOMEM;
    if (ni) k_sw_seed_scatter<<<grid_for(ni, 256), 256, 0, s>>>((const Seed*)d_seeds, w->reqq, ni, w->seeds);
    // the records of this rank: only the sweep's (the merge emitted none)
    Glob g;
    HIPCHECK(hipMemcpyAsync(&g, c->d_glob, sizeof g, hipMemcpyDeviceToHost, s));
    HIPCHECK(hipStreamSynchronize(s));
    const uint64_t want = g.n_rec + ni;
    if (want > c->d_recaux_cap) {
        hipFree(c->d_recaux);
        c->d_recaux = nullptr;
        c->d_recaux_cap = 0;
        if (hipMalloc(&c->d_recaux, std::max<uint64_t>(want, 1) * 16) != hipSuccess) return FLUERE_E_NOMEM;
        c->d_recaux_cap = std::max<uint64_t>(want, 1);
    }
    if (g.n_rec) HIPCHECK(hipMemsetAsync(c->d_recaux, 0, g.n_rec * 16, s));
    int rc = exact_finish(w->es, w->seeds, c->d_recaux + 2 * g.n_rec);
    if (rc) return rc;
    HIPCHECK(hipMemcpyAsync(&g, c->d_glob, sizeof g, hipMemcpyDeviceToHost, s));
    HIPCHECK(hipStreamSynchronize(s));
    c->dev_n_rec = g.n_rec;
    c->host_recs = false;
    c->dev_ordered = false;
    c->has_aux = true;
    c->have_results = true;
    if (st) {
        fluere_stats out{};
        out.valid = g.valid;
        out.dropped_parse = g.dropped;
        out.records = g.n_rec;
        out.ended = g.n_ended;
        out.updates = g.n_updates;
        out.complex_flows = exact_result(w->es).keys;
        out.sequential_mode = 1;
        *st = out;
    }
    exact_free(w->es);
    w->es = nullptr;
    return FLUERE_OK;
}

extern "C" int fluere_debug_dense_ids(fluere_ctx* c, const uint32_t* d_keys, uint64_t n, uint32_t* d_out) {
    if (!c || (!d_keys && n) || (!d_out && n)) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    if (n) k_dense_test<<<grid_for(n, 256), 256, 0, c->stream>>>(tables_of(c), d_keys, n, d_out, c->acc.slots);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(c->stream));
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
