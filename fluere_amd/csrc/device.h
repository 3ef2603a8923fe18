// device.h -- device-side types and helpers shared by the MI355X kernels of
// fluere_gpu.hip (hot path, finalize, merge) and exact.hip (the exact state
// machine): batches, per-flow accumulators, run counters, the per-packet
// front end (parse_keys + parse_fluereflow over a record window), canonical
// flow keys and the flow dictionary lookup, record building.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../include/fluere_gpu.h"
#include "flow_table.h"
#include "parse.h"

namespace fl {

constexpr int BLOCK = 1024;      // hot kernel: one 16-wave workgroup per CU
// LDS aggregates are flushed every WIN_ITERS steps of BLOCK packets: a window
// holds at most 61440 packets, so the 16-bit per-direction packet and flag
// counts and the u32 per-direction byte sums (<= 65535 B per packet) cannot wrap.
constexpr int WIN_ITERS = 60;
constexpr uint32_t NONE32 = 0xFFFFFFFFu;
constexpr unsigned long long NONE64 = ~0ull;
constexpr uint64_t IDX_MASK = (1ull << 40) - 1;

// Chunk descriptor (one per 64 records, built when a batch is attached, from
// its offsets): x = offset of the chunk's first record, y = the records'
// common stride when the 64 records are evenly spaced with a stride of at
// most 80 B, a multiple of 16 ("dense": the hot kernel reads the chunk's span
// with five coalesced loads per lane and reads no offsets), else 0 ("sparse":
// per-record windows at the record offsets).
struct Batch {
    const uint8_t* bytes;
    const uint32_t* offs;
    const uint2* desc;    // [n_desc] or null
    uint64_t n_desc;      // n / 64 (whole chunks)
    uint64_t nbytes;
    uint64_t n;
    uint64_t first;  // global index of packet 0
    uint32_t snap;
    uint32_t flags;  // bit0 byte-swapped headers, bit1 nanosecond timestamps
};

struct Acc {
    uint32_t* pk[2];
    unsigned long long* by[2];
    uint32_t* mn[2];  // min pkt, min ttl
    uint32_t* mx[2];  // max pkt, max ttl
    uint32_t* fl[8];  // fin syn rst psh ack urg ece cwr
    unsigned long long* fa;  // first packet (any)
    unsigned long long* fc;  // first create-eligible packet
    unsigned long long* fr;  // first FIN/RST packet
    unsigned long long* la;  // last packet
    uint32_t* slots;         // [fmax][N_TABLES] chain slots (cleanup)
};

struct Glob {
    unsigned long long valid, dropped, raw;
    unsigned long long tmin, tmax;
    unsigned long long n_rec;
    unsigned long long n_complex, n_complex_pkts;
    unsigned long long n_keys, n_heads;
    unsigned long long generic_used;
    unsigned long long n_slow;
    unsigned long long n_spill;  // k_parse_agg: the batch's overflow-list records (cursor); next to n_slow
    unsigned long long n_dspill; // k_parse_agg: the batch's spills in owner segments; next to n_spill
    unsigned long long n_gen;    // k_slow: the batch's general-parser list (cursor); next to n_dspill
    unsigned long long n_owner;  // k_merge_partials: owners claimed by its workgroups; next to n_gen
    unsigned long long n_updates, n_ended;  // over emitted records: sum of d_pkts, ended (order_key set)
    unsigned long long n_kc_miss;  // diagnostics: hot-kernel packets that found no LDS table entry
    unsigned long long cyc_total, cyc_flush, cyc_flush0;  // diagnostics: thread-0 clock sums over workgroups
    unsigned long long cyc_m_scan, cyc_m_ids;             // diagnostics: k_merge_partials phases
    unsigned long long clean_done;                        // k_cleanup: workgroups finished
    unsigned long long fin_done;                          // k_finalize: workgroups finished
    unsigned long long n_fdefer;                          // k_finalize: certified flows left to k_finalize_gen
    unsigned long long n_okey;                            // emitters: order keys written beside the records
    unsigned long long n_bare;                            // owner merge: order-dependent flows gathered without annexes
};
static_assert(offsetof(Glob, n_spill) == offsetof(Glob, n_slow) + 8 && offsetof(Glob, n_dspill) == offsetof(Glob, n_slow) + 16 &&
                  offsetof(Glob, n_gen) == offsetof(Glob, n_slow) + 24 && offsetof(Glob, n_owner) == offsetof(Glob, n_slow) + 32,
              "n_slow, n_spill, n_dspill, n_gen, n_owner are reset together");
// One device allocation holds Glob and the dictionary counters right after it
// (n_flows, err), so a run ends with ONE small device->host copy.
struct Ctl {
    Glob g;
    uint32_t n_flows, err;
    uint32_t seq;  // host copy only: k_finalize's last workgroup writes the run's number here last
    uint32_t pad[13];
};

// The records' order keys, one word per record slot in an array beside the
// record buffer (order_records reads them instead of one word of every
// 152-byte record).  Its pointer sits where the Ctl allocation ends, outside
// what k_cleanup clears; {nullptr, 0} until the host sizes it.  Glob::n_okey
// counts the words written since the run counters were reset: the array
// holds the run's keys when it equals n_rec.
struct OkeyRef {
    unsigned long long* p;
    unsigned long long cap;
};
__device__ __forceinline__ OkeyRef okey_ref(const Glob* g) {
    return *reinterpret_cast<const OkeyRef*>(reinterpret_cast<const char*>(g) + sizeof(Ctl));
}
// records [base, base + n) emitted: how many of them have an order-key slot
__device__ __forceinline__ unsigned long long okey_count(const OkeyRef& o, uint64_t cap, unsigned long long base,
                                                         unsigned long long n) {
    const unsigned long long lim = min((unsigned long long)cap, o.cap);
    return base >= lim ? 0ull : min(n, lim - base);
}

#define HIPCHECK(x)                                                                                  \
    do {                                                                                             \
        hipError_t e_ = (x);                                                                         \
        if (e_ != hipSuccess) {                                                                      \
            if (getenv("FLUERE_HIP_VERBOSE"))                                                        \
                fprintf(stderr, "[fluere] %s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return FLUERE_E_HIP;                                                                     \
        }                                                                                            \
    } while (0)

// ---------------------------------------------------------------------------
// per-packet front end shared by every kernel
// ---------------------------------------------------------------------------
struct Parsed {
    PktInfo pi;
    uint64_t t;
    uint64_t smac, dmac;  // big-endian packed MACs of the keyed frame
    uint32_t L;
    uint8_t cls;          // 0 valid, 1 dropped (NetError)
};

__device__ __forceinline__ uint32_t hdr_word(uint32_t w, bool swapped) { return swapped ? bswap32(w) : w; }

// Five unconditional 16-byte loads (unaligned global_load_dwordx4): record
// header + the first 64 frame bytes.  Unconditional so the compiler can count
// outstanding loads and keep the next packet's window in flight; batches are
// readable 80 bytes past their end (fluere_add_device_batch contract).
__device__ __forceinline__ void load_win(const Batch& B, uint32_t off, Win& W) {
    const uint8_t* p = B.bytes + off;
#pragma unroll
    for (int c = 0; c < 5; c++) {
        uint4 v;
        __builtin_memcpy(&v, p + 16 * c, 16);
        W.w[4 * c + 0] = v.x; W.w[4 * c + 1] = v.y; W.w[4 * c + 2] = v.z; W.w[4 * c + 3] = v.w;
    }
}

// Pins a loaded window at this point: every word is "used" here, so the
// compiler cannot sink the five loads into the parser's branches (which turns
// one memory round trip per packet into three dependent ones).
__device__ __forceinline__ void pin_win(const Win& W) {
    asm volatile("" ::"v"(W.w[0]), "v"(W.w[1]), "v"(W.w[2]), "v"(W.w[3]), "v"(W.w[4]), "v"(W.w[5]), "v"(W.w[6]),
                 "v"(W.w[7]), "v"(W.w[8]), "v"(W.w[9]));
    asm volatile("" ::"v"(W.w[10]), "v"(W.w[11]), "v"(W.w[12]), "v"(W.w[13]), "v"(W.w[14]), "v"(W.w[15]),
                 "v"(W.w[16]), "v"(W.w[17]), "v"(W.w[18]), "v"(W.w[19]));
}

__device__ __forceinline__ void pin_win32(const Win32& W) {
#pragma unroll
    for (int k = 0; k < 32; k += 8)
        asm volatile("" ::"v"(W.w[k]), "v"(W.w[k + 1]), "v"(W.w[k + 2]), "v"(W.w[k + 3]), "v"(W.w[k + 4]),
                     "v"(W.w[k + 5]), "v"(W.w[k + 6]), "v"(W.w[k + 7]));
}

__device__ __forceinline__ uint64_t mac_be(const uint8_t* p) {
    uint64_t m = 0;
    for (int k = 0; k < 6; k++) m = (m << 8) | p[k];
    return m;
}

// mode: 0 production (fast path first), 1 general parser only.  INL: the
// general parser inlined (k_slow) instead of called out of line.
template <bool INL = false>
__device__ __forceinline__ void parse_loaded(const Batch& B, uint32_t off, const Win& W, bool macs, int mode, Parsed& P,
                                             const uint8_t* staged = nullptr, uint32_t staged_n = 0);
template <bool INL = false>
__device__ __forceinline__ void parse_record(const Batch& B, uint64_t li, bool macs, int mode, Parsed& P) {
    uint32_t off = B.offs[li];
    Win W;
    load_win(B, off, W);
    parse_loaded<INL>(B, off, W, macs, mode, P);
}
// The record at batch offset off, its window W already loaded.
template <bool INL>
__device__ __forceinline__ void parse_loaded(const Batch& B, uint32_t off, const Win& W, bool macs, int mode, Parsed& P,
                                             const uint8_t* staged, uint32_t staged_n) {
    bool sw = B.flags & 1;
    uint32_t sec = hdr_word(W.w[0], sw), frac = hdr_word(W.w[1], sw), incl = hdr_word(W.w[2], sw);
    uint32_t L = min(incl, B.snap);
    uint64_t avail = B.nbytes > (uint64_t)off + 16 ? B.nbytes - off - 16 : 0;
    if (L > avail) L = (uint32_t)avail;
    P.L = L;
    P.t = (uint64_t)sec * 1000000ull + ((B.flags & 2) ? frac / 1000u : frac);  // time.rs:5-7
    const uint8_t* fr = B.bytes + off + 16;
    bool fast = (mode == 0) && parse_fast(W, L, P.pi);
    if (!fast) {
        if constexpr (INL) {
            parse_general_inl(fr, L, P.pi, staged, min(staged_n, L));
        } else {
            PktInfo g;  // only this copy lives on the stack (parse_general is out of line)
            parse_general(fr, L, g);
            P.pi = g;
        }
    }
    const PktInfo& pi = P.pi;
    P.cls = (pi.kst != ST_OK || pi.fst != ST_OK) ? 1 : 0;
    P.smac = P.dmac = 0;
    if (macs && P.cls == 0) {
        if (fast) {
            // frame bytes 0..12 = record bytes 16..28
            uint64_t d = 0, s = 0;
            for (int k = 0; k < 6; k++) d = (d << 8) | W.b(16 + k);
            for (int k = 0; k < 6; k++) s = (s << 8) | W.b(22 + k);
            P.dmac = d; P.smac = s;
        } else {
            P.dmac = mac_be(fr + pi.frame_off);
            P.smac = mac_be(fr + pi.frame_off + 6);
        }
    }
}

// The record at batch offset off through the register parser alone (no
// general parser in the caller's code: its registers and stack would cost the
// whole kernel occupancy); P.cls = 2 when parse_fast declines the packet.
__device__ __forceinline__ void parse_loaded_fast(const Batch& B, uint32_t off, const Win& W, bool macs, Parsed& P) {
    const bool sw = B.flags & 1;
    const uint32_t sec = hdr_word(W.w[0], sw), frac = hdr_word(W.w[1], sw), incl = hdr_word(W.w[2], sw);
    uint32_t L = min(incl, B.snap);
    const uint64_t avail = B.nbytes > (uint64_t)off + 16 ? B.nbytes - off - 16 : 0;
    if (L > avail) L = (uint32_t)avail;
    P.L = L;
    P.t = (uint64_t)sec * 1000000ull + ((B.flags & 2) ? frac / 1000u : frac);  // time.rs:5-7
    P.smac = P.dmac = 0;
    if (!parse_fast(W, L, P.pi)) {
        P.cls = 2;
        return;
    }
    const PktInfo& pi = P.pi;
    P.cls = (pi.kst != ST_OK || pi.fst != ST_OK) ? 1 : 0;
    if (macs && P.cls == 0) {  // frame bytes 0..12 = record bytes 16..28
        uint64_t d = 0, s = 0;
        for (int k = 0; k < 6; k++) d = (d << 8) | W.b(16 + k);
        for (int k = 0; k < 6; k++) s = (s << 8) | W.b(22 + k);
        P.dmac = d;
        P.smac = s;
    }
}

// The packets the hot parser leaves over (k_slow; k_parse_batch's production
// mode): the record at batch offset off with its 128-byte window W loaded --
// parse_fast, then parse_mid, then (GEN = 1) the general parser out of line;
// GEN = 0 leaves the rest to the caller (P.cls = 2: the general parser's).
template <int GEN>
__device__ __forceinline__ void parse_loaded32(const Batch& B, uint32_t off, const Win32& W, bool macs, Parsed& P) {
    const bool sw = B.flags & 1;
    const uint32_t sec = hdr_word(W.w[0], sw), frac = hdr_word(W.w[1], sw), incl = hdr_word(W.w[2], sw);
    uint32_t L = min(incl, B.snap);
    const uint64_t avail = B.nbytes > (uint64_t)off + 16 ? B.nbytes - off - 16 : 0;
    if (L > avail) L = (uint32_t)avail;
    P.L = L;
    P.t = (uint64_t)sec * 1000000ull + ((B.flags & 2) ? frac / 1000u : frac);  // time.rs:5-7
    Win W20;
#pragma unroll
    for (int k = 0; k < 20; k++) W20.w[k] = W.w[k];
    const bool fast = parse_fast(W20, L, P.pi);
    const bool mid = !fast && parse_mid(W, L, P.pi);
    const uint8_t* fr = B.bytes + off + 16;
    P.smac = P.dmac = 0;
    if (!fast && !mid) {
        if constexpr (GEN == 0) {
            P.cls = 2;
            return;
        } else {
            PktInfo g;
            parse_general(fr, L, g);
            P.pi = g;
        }
    }
    const PktInfo& pi = P.pi;
    P.cls = (pi.kst != ST_OK || pi.fst != ST_OK) ? 1 : 0;
    if (macs && P.cls == 0) {
        if (fast || mid) {
            // the keyed frame at frame byte 0 or 50 (VXLAN inner): record bytes 16.. / 66..
            const bool in = pi.frame_off != 0;
            uint64_t d = 0, s = 0;
#pragma unroll
            for (int k = 0; k < 6; k++) d = (d << 8) | (in ? W.b(66 + k) : W.b(16 + k));
#pragma unroll
            for (int k = 0; k < 6; k++) s = (s << 8) | (in ? W.b(72 + k) : W.b(22 + k));
            P.dmac = d;
            P.smac = s;
        } else {
            P.dmac = mac_be(fr + pi.frame_off);
            P.smac = mac_be(fr + pi.frame_off + 6);
        }
    }
}

// The 128-byte window of the record at off: pieces 0..4 always (a batch is
// readable 80 bytes past its end), 5..7 where they stay inside that (a record
// short enough to need the clamp never reads them: parse_mid needs L >= 34 of
// a whole record).
__device__ __forceinline__ void load_win32(const Batch& B, uint32_t off, Win32& W) {
    const uint8_t* p = B.bytes + off;
    const uint64_t room = B.nbytes + 80 > (uint64_t)off ? B.nbytes + 80 - off : 0;
#pragma unroll
    for (int c = 0; c < 8; c++) {
        const uint8_t* q = (c < 5 || (uint64_t)(16 * c + 16) <= room) ? p + 16 * c : p + 64;
        uint4 v;
        __builtin_memcpy(&v, q, 16);
        W.w[4 * c + 0] = v.x; W.w[4 * c + 1] = v.y; W.w[4 * c + 2] = v.z; W.w[4 * c + 3] = v.w;
    }
}

__device__ __forceinline__ int find_batch(const Batch* bs, int nb, uint64_t gi) {
    int b = 0;
    while (b + 1 < nb && bs[b + 1].first <= gi) b++;
    return b;
}

__device__ __forceinline__ uint8_t canon_dir(const Parsed& P, bool macs) {
    const PktInfo& pi = P.pi;
    return src_gt_dst(pi.sip, pi.dip, pi.ksp, pi.kdp, P.smac, P.dmac, pi.v6, macs) ? 1 : 0;
}

// Canonical key of a parsed packet.  dir = 1 when the packet travels from the
// higher endpoint to the lower one.
__device__ __forceinline__ void canon_key(const Parsed& P, bool macs, CKey& k, uint8_t& dir) {
    const PktInfo& pi = P.pi;
    bool gt = src_gt_dst(pi.sip, pi.dip, pi.ksp, pi.kdp, P.smac, P.dmac, pi.v6, macs);
    dir = gt ? 1 : 0;
    uint32_t lop = gt ? pi.kdp : pi.ksp, hip = gt ? pi.ksp : pi.kdp;
    uint64_t lom = gt ? P.dmac : P.smac, him = gt ? P.smac : P.dmac;
#pragma unroll
    for (int j = 0; j < 4; j++) {  // per-word selects keep the IP arrays in registers
        k.w[j] = gt ? pi.dip[j] : pi.sip[j];
        k.w[4 + j] = gt ? pi.sip[j] : pi.dip[j];
    }
    k.w[8] = (lop << 16) | hip;
    uint32_t kind = (pi.v6 ? 1u : 0u) | (macs ? 2u : 0u);
    k.w[9] = (kind << 8) | pi.kproto;
    k.w[10] = macs ? (uint32_t)(lom >> 16) : 0; k.w[11] = macs ? (uint32_t)(lom & 0xFFFF) << 16 : 0;
    k.w[12] = macs ? (uint32_t)(him >> 16) : 0; k.w[13] = macs ? (uint32_t)(him & 0xFFFF) << 16 : 0;
}

// Exact dense flow id of a canonical key (flow_table.h chains).
__device__ __forceinline__ uint32_t dense_of_key(const TableSet& T, const CKey& k, bool insert, uint32_t* chain_out,
                                                 unsigned long long* generic_used) {
    const uint32_t kind = k.w[9] >> 8;
    const bool v6 = kind & 1, macs = kind & 2;
    uint32_t chain[N_TABLES];
    for (int j = 0; j < N_TABLES; j++) chain[j] = NONE32;
    uint32_t s;
    int ft;
    unsigned long long v = EMPTY;
    if (!v6 && !macs && v4_fast(T, k.w[9] & 0xFF)) {
        uint32_t s0;
        v4_slots(T, k.w[0], k.w[4], k.w[8], k.w[9] & 0xFF, insert, s0, s, &v);
        if (s0 == FAIL || s == FAIL) return FAIL;
        chain[0] = s0;
        chain[1] = s;
        ft = 1;
    } else {
        if (generic_used && insert) *generic_used = 1;
        // 32-bit units: kind|proto, ports, lo_ip, hi_ip, [lo_mac, hi_mac]
        uint32_t u[13];
        u[0] = k.w[9];
        u[1] = k.w[8];
        const uint32_t m0 = k.w[10], m1 = k.w[11] | (k.w[12] >> 16), m2 = (k.w[12] << 16) | (k.w[13] >> 16);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            u[2 + j] = v6 ? k.w[j] : (j == 0 ? k.w[0] : j == 1 ? k.w[4] : j == 2 ? m0 : m1);
            u[6 + j] = v6 ? k.w[4 + j] : (j == 0 ? m2 : 0);
        }
        u[10] = m0; u[11] = m1; u[12] = m2;
        const int m = v6 ? (macs ? 13 : 10) : 7;
        s = tab_slot(T, 2, ((uint64_t)u[0] << 32) | u[1], insert, &v);
        if (s == FAIL) return FAIL;
        chain[2] = s;
        ft = 2;
#pragma unroll
        for (int j = 2; j < 13; j++) {
            if (j < m) {
                s = tab_slot(T, j + 1, ((uint64_t)s << 32) | u[j], insert, &v);
                if (s == FAIL) return FAIL;
                chain[j + 1] = s;
                ft = j + 1;
            }
        }
    }
    return dense_id(T, ft, s, insert, k, chain, chain_out, v);
}

__device__ __forceinline__ uint32_t flow_of(const TableSet& T, const Parsed& P, bool macs, bool insert,
                                           uint8_t& dir, uint32_t* chain_out, unsigned long long* generic_used) {
    CKey k;
    canon_key(P, macs, k, dir);
    return dense_of_key(T, k, insert, chain_out, generic_used);
}

// Bucket of a canonical key in the exact engine's complex-flow filter (a
// bitmap of CBITS bits, set for every flow the certificate rejects): a packet
// whose key's bit is clear belongs to no complex flow, so the replay skips its
// dictionary walk.
constexpr uint32_t CBITS_LOG2 = 22;  // complex-flow filter: one byte per bucket (plain stores, no atomics)
__device__ __forceinline__ uint32_t ckey_bucket(const uint32_t* w) {
    uint32_t h = 0x2545F491u;
#pragma unroll
    for (int j = 0; j < 14; j++) {
        h = (h ^ w[j]) * 0x9E3779B1u;
        h ^= h >> 15;
    }
    return h >> (32 - CBITS_LOG2);
}

// ckey_bucket of an IPv4 non-MAC canonical key (the hot kernels' key words:
// lower ip, higher ip, lower port << 16 | higher port, protocol)
__device__ __forceinline__ uint32_t ckey_bucket_v4(uint32_t lo, uint32_t hi, uint32_t ports, uint32_t proto) {
    const uint32_t w[14] = {lo, 0, 0, 0, hi, 0, 0, 0, ports, proto, 0, 0, 0, 0};
    return ckey_bucket(w);
}
// Per-packet filter words of the hot pass (AggArgs::phash): the packet's
// ckey_bucket, or PH_PARSE (the hot parser did not key it: the exact engine
// parses the packet itself).
constexpr uint32_t PH_PARSE = 0xFFFFFFFFu;
// The same words after the merge (flow ids per packet, k_parse_spill runs with
// AggArgs::pid): a packet the merge resolved carries its dense id (PH_ID | d),
// or its merge entry (PH_EREF | batch << 21 | owner << 10 | entry), whose
// dense id the merge's id phase writes to emap[batch << 21 | owner << 10 |
// entry].  Buckets stay below 2^22, dense ids below 2^26 (MAX_FLOWS).
constexpr uint32_t PH_ID = 0x80000000u, PH_EREF = 0x40000000u;
__device__ __forceinline__ uint32_t ph_flow(uint32_t w, const uint32_t* emap) {  // dense id, or FAIL
    if (w == PH_PARSE || !(w & (PH_ID | PH_EREF))) return FAIL;
    return (w & PH_ID) ? (w & 0x03FFFFFFu) : emap[w & 0x00FFFFFFu];
}

// Append one record (Mode A paths): position, updates and ended counters.
__device__ __forceinline__ void emit_record(Glob* g, fluere_record* out, uint64_t cap, const fluere_record& r) {
    const unsigned long long pos = atomicAdd(&g->n_rec, 1ull);
    if (pos < cap) out[pos] = r;
    const OkeyRef o = okey_ref(g);
    if (okey_count(o, cap, pos, 1)) {
        o.p[pos] = r.order_key;
        atomicAdd(&g->n_okey, 1ull);
    }
    atomicAdd(&g->n_updates, (unsigned long long)r.d_pkts);
    if (r.order_key != NONE64) atomicAdd(&g->n_ended, 1ull);
}

__device__ inline void fill_seed(fluere_record& r, const Parsed& P) {
    const PktInfo& pi = P.pi;
    memset(&r, 0, sizeof r);
    r.src_v6 = r.dst_v6 = pi.rv6;
    for (int k = 0; k < 4; k++) {
        uint32_t s = pi.rsip[k], d = pi.rdip[k];
        for (int b = 0; b < 4; b++) {
            r.source[4 * k + b] = (uint8_t)(s >> (24 - 8 * b));
            r.destination[4 * k + b] = (uint8_t)(d >> (24 - 8 * b));
        }
    }
    r.prot = pi.rprot; r.tos = pi.rtos;
    r.src_port = pi.rsp; r.dst_port = pi.rdp;
    r.min_pkt = r.max_pkt = pi.rpkt;
    r.min_ttl = r.max_ttl = pi.rttl;
    r.first = r.last = P.t;
}

__device__ __forceinline__ void parse_global(const Batch* bs, int nb, uint64_t gi, bool macs, Parsed& P) {
    int b = find_batch(bs, nb, gi);
    parse_record(bs[b], gi - bs[b].first, macs, 0, P);
}
// The register parser alone (parse_loaded_fast): P.cls = 2 when it declines.
__device__ __forceinline__ void parse_global_fast(const Batch* bs, int nb, uint64_t gi, bool macs, Parsed& P) {
    const int b = find_batch(bs, nb, gi);
    const Batch& B = bs[b];
    const uint32_t off = B.offs[gi - B.first];
    Win W;
    load_win(B, off, W);
    parse_loaded_fast(B, off, W, macs, P);
}

// parse_microseconds (time.rs:5-7) of the record at batch offset off: the
// record header alone (a record's `last` needs no parse of its frame).
__device__ __forceinline__ uint64_t record_time(const Batch& B, uint32_t off) {
    uint2 h;
    __builtin_memcpy(&h, B.bytes + off, 8);  // (record offsets need not be aligned)
    const bool sw = B.flags & 1;
    const uint32_t sec = hdr_word(h.x, sw), frac = hdr_word(h.y, sw);
    return (uint64_t)sec * 1000000ull + ((B.flags & 2) ? frac / 1000u : frac);
}
__device__ __forceinline__ uint64_t time_global(const Batch* bs, int nb, uint64_t gi) {
    const int b = find_batch(bs, nb, gi);
    return record_time(bs[b], bs[b].offs[gi - bs[b].first]);
}

// Wave-aggregated emit_record: one atomic per counter per wave (a thread-per-
// flow kernel that hits the three run counters per flow serialises on them).
// All lanes of the wave must call it (want = this lane has a record).
__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ void emit_record_wave(Glob* g, fluere_record* out, uint64_t cap, const fluere_record& r,
                                                 bool want) {
    const uint64_t m = __ballot(want);
    if (!m) return;
    const uint64_t em = __ballot(want && r.order_key != NONE64);
    const unsigned long long upd = wave_sum(want ? (unsigned long long)r.d_pkts : 0ull);
    const uint32_t lead = __builtin_ctzll(m);
    unsigned long long base = 0;
    if ((uint32_t)(threadIdx.x & 63) == lead) {
        base = atomicAdd(&g->n_rec, (unsigned long long)__popcll(m));
        atomicAdd(&g->n_updates, upd);
        if (em) atomicAdd(&g->n_ended, (unsigned long long)__popcll(em));
    }
    base = __shfl(base, lead, 64);
    const OkeyRef o = okey_ref(g);
    const unsigned long long nok = okey_count(o, cap, base, (unsigned long long)__popcll(m));
    if ((uint32_t)(threadIdx.x & 63) == lead && nok) atomicAdd(&g->n_okey, nok);
    if (want) {
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        if (base + rank < cap) out[base + rank] = r;
        if (rank < nok) o.p[base + rank] = r.order_key;
    }
}

// Block-level emit_record (256-thread blocks; every thread of the block calls
// it, with uniform control flow): one set of counter atomics per block, the
// block's records staged in LDS and written out as coalesced 8-byte words.
// (A 152-byte record stored per lane, lane by lane, made the 1M-flow C4
// finalize spend ~0.35 ms on its record writes.)
constexpr int EMIT_BLOCK = 256;
struct EmitLds {
    unsigned long long w[EMIT_BLOCK / 64][3];  // per wave: records (-> exclusive prefix), updates, ended
    unsigned long long base, n;
    fluere_record rec[EMIT_BLOCK];
    uint16_t slot[EMIT_BLOCK];                 // emit_inplace_block: the k-th record's thread
};
// aux (optional): two order words per record, written beside it (Mode B:
// {0 for a FIN/RST close, else exp + 1; the firing entry's creation}).
__device__ __forceinline__ void emit_record_block(EmitLds& S, Glob* g, fluere_record* out, uint64_t cap,
                                                  const fluere_record& r, bool want,
                                                  unsigned long long* aux = nullptr, unsigned long long a0 = 0,
                                                  unsigned long long a1 = 0) {
    static_assert(sizeof(fluere_record) % 8 == 0, "records are whole 8-byte words");
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t m = __ballot(want), em = __ballot(want && r.order_key != NONE64);
    const unsigned long long upd = wave_sum(want ? (unsigned long long)r.d_pkts : 0ull);
    if (lane == 0) {
        S.w[w][0] = __popcll(m);
        S.w[w][1] = upd;
        S.w[w][2] = __popcll(em);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t[3] = {0, 0, 0};
        for (int k = 0; k < EMIT_BLOCK / 64; k++) {
            const unsigned long long nk = S.w[k][0];
            t[1] += S.w[k][1];
            t[2] += S.w[k][2];
            S.w[k][0] = t[0];  // exclusive prefix of the records
            t[0] += nk;
        }
        S.base = t[0] ? atomicAdd(&g->n_rec, t[0]) : 0ull;
        S.n = t[0];
        if (t[1]) atomicAdd(&g->n_updates, t[1]);
        if (t[2]) atomicAdd(&g->n_ended, t[2]);
        const unsigned long long nok = okey_count(okey_ref(g), cap, S.base, t[0]);
        if (nok) atomicAdd(&g->n_okey, nok);
    }
    __syncthreads();
    if (want) {
        const uint32_t i = S.w[w][0] + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        S.rec[i] = r;
        const OkeyRef o = okey_ref(g);
        if (okey_count(o, cap, S.base + i, 1)) o.p[S.base + i] = r.order_key;
        if (aux && S.base + i < cap)
            *reinterpret_cast<ulonglong2*>(aux + 2 * (S.base + i)) = make_ulonglong2(a0, a1);
    }
    __syncthreads();
    const unsigned long long base = S.base;
    const unsigned long long n = base < cap ? min(S.n, cap - base) : 0ull;  // (records past the capacity: counted only)
    constexpr uint32_t RW = sizeof(fluere_record) / 8;
    const uint2* src = reinterpret_cast<const uint2*>(S.rec);
    uint2* dst = reinterpret_cast<uint2*>(out + base);
    for (uint32_t i = threadIdx.x; i < n * RW; i += EMIT_BLOCK) dst[i] = src[i];
    __syncthreads();  // S is rewritten by the next call
}

// emit_record_block for records built in place, thread t's in S.rec[t] (a
// kernel that builds its record field by field in LDS holds no 38-word record
// in registers): the copy gathers the wanted slots in thread order.
// tot (optional): thread 0 adds the block's updates / ended counts there
// instead of one pair of global atomics per call (the caller adds its totals
// once: thousands of blocks on two words serialised k_finalize).
__device__ __forceinline__ void emit_inplace_block(EmitLds& S, Glob* g, fluere_record* out, uint64_t cap, bool want,
                                                   uint32_t d_pkts, bool ended, unsigned long long* aux = nullptr,
                                                   unsigned long long a0 = 0, unsigned long long a1 = 0,
                                                   unsigned long long* tot = nullptr, uint32_t* rbits = nullptr) {
    const uint32_t w = threadIdx.x >> 6;
    const uint64_t m = __ballot(want), em = __ballot(want && ended);
    const unsigned long long upd = wave_sum(want ? (unsigned long long)d_pkts : 0ull);
    if ((threadIdx.x & 63) == 0) {
        S.w[w][0] = __popcll(m);
        S.w[w][1] = upd;
        S.w[w][2] = __popcll(em);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t[3] = {0, 0, 0};
        for (int k = 0; k < EMIT_BLOCK / 64; k++) {
            const unsigned long long nk = S.w[k][0];
            t[1] += S.w[k][1];
            t[2] += S.w[k][2];
            S.w[k][0] = t[0];
            t[0] += nk;
        }
        S.base = t[0] ? atomicAdd(&g->n_rec, t[0]) : 0ull;
        S.n = t[0];
        const unsigned long long nok = okey_count(okey_ref(g), cap, S.base, t[0]);
        if (nok) atomicAdd(&g->n_okey, nok);
        if (tot) {
            tot[0] += t[1];
            tot[1] += t[2];
        } else {
            if (t[1]) atomicAdd(&g->n_updates, t[1]);
            if (t[2]) atomicAdd(&g->n_ended, t[2]);
        }
    }
    __syncthreads();
    if (want) {
        const uint32_t i = S.w[w][0] + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        S.slot[i] = (uint16_t)threadIdx.x;
        const OkeyRef o = okey_ref(g);
        if (okey_count(o, cap, S.base + i, 1)) o.p[S.base + i] = S.rec[threadIdx.x].order_key;
        if (rbits && ended && S.base + i < cap) atomicOr(&rbits[(S.base + i) >> 5], 1u << ((S.base + i) & 31));
        if (aux && S.base + i < cap)
            *reinterpret_cast<ulonglong2*>(aux + 2 * (S.base + i)) = make_ulonglong2(a0, a1);
    }
    __syncthreads();
    const unsigned long long base = S.base;
    const unsigned long long n = base < cap ? min(S.n, cap - base) : 0ull;
    constexpr uint32_t RW = sizeof(fluere_record) / 8;
    uint2* dst = reinterpret_cast<uint2*>(out + base);
    for (uint32_t i = threadIdx.x; i < n * RW; i += EMIT_BLOCK) {
        const uint32_t k = i / RW, wd = i - k * RW;
        dst[i] = reinterpret_cast<const uint2*>(&S.rec[S.slot[k]])[wd];
    }
    __syncthreads();
}

__device__ __forceinline__ void update_flow(fluere_record& r, bool rev, const PktInfo& pi, uint64_t t) {
    // src/net/flows.rs:11-42 (u32 counters wrap like the release build)
    r.d_pkts += 1;
    r.d_octets += pi.doctets;
    r.max_pkt = max(r.max_pkt, pi.rpkt);
    r.min_pkt = min(r.min_pkt, pi.rpkt);
    r.max_ttl = max(r.max_ttl, pi.rttl);
    r.min_ttl = min(r.min_ttl, pi.rttl);
    for (int q = 0; q < 8; q++) r.cnt[q] += (pi.tflags >> q) & 1;
    r.last = t;
    if (rev) { r.in_pkts += 1; r.in_bytes += pi.doctets; }
    else { r.out_pkts += 1; r.out_bytes += pi.doctets; }
}

}  // namespace fl
