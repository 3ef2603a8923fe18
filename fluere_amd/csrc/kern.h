// kern.h -- device-side structures and helpers of the one-GPU pass shared by
// its kernel translation units (hot.hip, merge.hip, shard.hip, fluere_gpu.hip)
// and the host code that fills their arguments.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include "prim.h"

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
#include "seg.h"

// FLUERE_ALLOC_LOG (diagnostics): every device allocation of the library, with
// its source line and time (fluere_gpu.hip) -- the allocations a run makes while
// the GPU waits
hipError_t fl_dmalloc(void** p, size_t bytes, int line);
#define hipMalloc(p, bytes) fl_dmalloc(reinterpret_cast<void**>(p), (bytes), __LINE__)

using namespace fl;

namespace fl {

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
// A lean partial (k_parse_agg without MACs): a flow whose window carried no TCP
// flag, no FIN/RST and whose first packet could create it (every UDP flow)
// is staged as its first 48 bytes only -- tag | PART_LEAN; word 2 = {min pkt |
// max pkt << 16, min ttl | max ttl << 8, first, last + 1} -- 40 % fewer flush
// bytes (20 -> 12 MB for C2) and dirty lines behind the kernel.
constexpr uint32_t PART_LEAN = 2u;

// A spilled packet: a valid hot-path packet whose key found no LDS slot (more
// flows in a workgroup's window than the table holds).  32 bytes; written
// raw per workgroup during the window, grouped by merge owner at the flush,
// merged by its owner like a one-packet partial.
struct alignas(16) Spill {
    uint32_t k0, k1, k2, tag;     // LDS key words (tag = proto << 24)
    uint32_t doct, pt, loc, fl;   // pt = pkt | ttl << 16 | elig << 24; fl = tf | dir << 8 (| set << 9: overflow list;
                                  // set SPILL_BATCH_REL: loc is relative to the batch's first packet)
};
static_assert(sizeof(Spill) == 32, "Spill layout");
constexpr uint32_t SPILL_BATCH_REL = 0x7FFFFFu;
// (the packed owner-segment records: seg.h)
__host__ __device__ constexpr int spill_units(bool macs) { return macs ? 2 : 1; }

struct Stage {
    Part* part;                   // [set * NS + cell]
    uint32_t* off;                // [(O + 1) * n_sets]: off[o * n_sets + set] = first cell of owner o's flows
    unsigned long long* base;     // [set] global index of the window's first packet
    // Spilled packets are stored as planes of 16-byte words (word w of every
    // record together), so a wave's loads and stores of one word are contiguous.
    // A spilled packet is stored where its merge owner reads it: segment o of
    // its set holds up to cap_o records (24 B packed, seg_pack; 64 B with MACs),
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
    unsigned long long* slow_n;  // their total (the merge's "any slow packet" test): bc[0]
    // the batch's counters {slow-list packets, overflow-list records, owner-segment
    // spills, general-parser list, merge owners claimed}: Glob::n_slow.. for a pass of
    // one batch, else the batch's own area (their merges can run after every batch)
    unsigned long long* bc;
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
    // Mode B predicted (k_parse_spill): every packet's replay metadata, this
    // batch's first packet first (capture order over the capture: the exact
    // engine's k_ex_meta pass is skipped), or null
    ExMeta* exm;
    unsigned long long* exm_t;  // or null: the packets' times alone (8 B, capture order) beside exm
    int tail_only;             // k_merge_partials: no owners (k_merge_spill merged them), only the run
                               // statistics and the tail (overflow list, general-parser packets)
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
__device__ __forceinline__ uint32_t own_add_n(uint32_t* arr, uint32_t o, uint32_t n) {
    return (atomicAdd(&arr[o >> 1], n << ((o & 1) * 16)) >> ((o & 1) * 16)) & 0xFFFFu;
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

// part_to_global for a flow whose accumulators have no other writer in the
// run (k_merge_spill, when no tail adds to them): plain stores over the
// identities k_cleanup left
__device__ __forceinline__ void part_store_global(const Acc& A, uint32_t d, const FlowPart& f) {
#pragma unroll
    for (int q = 0; q < 2; q++) {
        A.pk[q][d] = f.pk[q];
        A.by[q][d] = f.by[q];
        A.mn[q][d] = f.mn[q];
        A.mx[q][d] = f.mx[q];
    }
#pragma unroll
    for (int q = 0; q < 8; q++) A.fl[q][d] = f.fl[q];
    A.fa[d] = f.fa;
    A.fc[d] = f.fc;
    A.fr[d] = f.fr;
    A.la[d] = f.la ? f.la - 1 : 0;
}

__device__ __forceinline__ void part_of_stage(const Part& p, unsigned long long base, FlowPart& f) {
    if (p.tag & PART_LEAN) {  // {min | max pkt << 16, min | max ttl << 8, first, last + 1}
        f.pk[0] = p.pk & 0xFFFF;
        f.pk[1] = p.pk >> 16;
        f.by[0] = p.by0;
        f.by[1] = p.by1;
        f.mn[0] = p.mn0 & 0xFFFF;
        f.mx[0] = p.mn0 >> 16;
        f.mn[1] = p.mn1 & 0xFF;
        f.mx[1] = (p.mn1 >> 8) & 0xFF;
#pragma unroll
        for (int q = 0; q < 8; q++) f.fl[q] = 0;
        f.fa = f.fc = base + p.mx0;
        f.fr = NONE64;
        f.la = base + p.mx1;
        return;
    }
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
    uint32_t* kbits = nullptr;      // k_finalize: the ordering's key bits (SoArgs::bits), set at each ended
    unsigned long long kbase = 0;   //   record's closing packet (index - kbase), or null
    uint32_t* rbits = nullptr;      //   and its record bits (SoArgs::rbits), set at each ended record
};

// A flow's order-free aggregate (the accumulators of one dense id).
struct AccVals {
    unsigned long long fa, fc, fr, la;
    uint32_t pk[2];
    unsigned long long by[2];
    uint32_t mn[2], mx[2], fl[8];
};

// one thread per flow, grid-stride (uniform per workgroup) over the
// device-side flow count
// The last workgroup to finish (counter *done) copies the run counters (Glob,
// n_flows, err) to the pinned host copy, then publishes seq there (the host
// polls it: no copy kernel, no event on the way back).
__device__ inline void publish_ctl(Glob* g, unsigned long long* done, Ctl* host_ctl, uint32_t seq) {
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

// flow pieces (multi-GPU composition, live sessions)
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

inline unsigned grid_for(uint64_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

#ifndef FLUERE_SB
#define FLUERE_SB 256
#endif
constexpr int SB = FLUERE_SB;                // k_slow block
constexpr uint32_t SLOW_SET = SPILL_WG / 4;  // slow-list entries per k_slow workgroup (one set)

// kernels of the pass launched from other translation units
// merge.hip
__global__ void __launch_bounds__(SB) k_slow(AggArgs a);
__global__ void __launch_bounds__(EMIT_BLOCK) k_finalize(FinArgs a);
__global__ void __launch_bounds__(EMIT_BLOCK) k_finalize_gen(FinArgs a);
__global__ void __launch_bounds__(256) k_seq_meta(SeqMetaArgs a);
__global__ void __launch_bounds__(64) k_seq_run(SeqArgs a);
__global__ void __launch_bounds__(256) k_cleanup(CleanArgs a, size_t tab_words);
__global__ void k_fill_u64(unsigned long long* p, size_t n, unsigned long long v);
__global__ void k_fill_u32(uint32_t* p, size_t n, uint32_t v);
// k_merge_spill's input: the owner segments of every batch of a pass (one
// merge per pass; a batch's staging is its own)
struct SegSrc {
    const Spill* dspill;
    const uint32_t* soff;
    const unsigned long long* base;
    Spill* spill;                 // the batch's overflow list (records without an aggregate slot)
    unsigned long long* bc;       // the batch's counters (AggArgs::bc)
    unsigned long long slow_rec0, first;
    uint32_t cap_o, cap_s, n_sets, n_hot;
    uint32_t slow_kernel;         // the batch's slow list went to k_slow (its tail: the general-parser list)
};
constexpr int MS_BATCHES = 8;
struct MergeSrc {
    SegSrc b[MS_BATCHES];
    int nb;
};
__global__ void __launch_bounds__(MB) k_merge_spill(AggArgs a, MergeSrc ms);
// templated kernels: their host stubs, by configuration
const void* hot_kernel(int spill, int macs, int abl);  // hot.hip: k_parse_agg / k_parse_spill
const void* merge_kernel(int macs);                     // merge.hip: k_merge_partials

}  // namespace fl
