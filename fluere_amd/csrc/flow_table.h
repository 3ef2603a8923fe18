// flow_table.h -- exact flow dictionary for MI355X.
//
// The reference keys its active-flow HashMap by the full Key
// (src/net/types/key.rs:5-14: two IpAddr, two ports, protocol, two MACs) and
// looks a packet up under Key and its reverse (offline_fluereflows.rs:97-130).
// On the device both directions map to one *canonical* key (lower endpoint
// first, endpoint = (ip, port, mac)) plus a direction bit, and the canonical
// key is turned into a dense flow id through a chain of write-once hash
// tables whose entries are single 64-bit words:
//
//   IPv4, no MAC:  T0[(lo_ip << 32) | hi_ip]                      -> s0
//                  T1[(s0 << 40) | (lo_port << 24) | (hi_port << 8) | proto] -> s1 -> dense id
//                  (T1's probe starts at a hash of the whole key, so both
//                  tables' first probes travel together: v4_slots)
//                  (tables of 2^24 slots and more, "wide": T1[(s0 << 33) |
//                  (ports << 1) | udp] for TCP and UDP, every other protocol
//                  through the generic chain -- v4_t1_word)
//   otherwise:     the canonical key serialised to 32-bit units; level 0 takes
//                  units 0 and 1, level k >= 1 takes (s_{k-1} << 32) | unit k+1.
//
// Each level is exact (the stored word *is* the key material), so the chain
// is an injective map without any full-key compare, and every cross-workgroup
// interaction is a 64-bit CAS whose returned value is authoritative: a plain
// (possibly stale) load can only show EMPTY for a filled slot, never a wrong
// key, because slots are written once.  No release/acquire hand-off between
// workgroups is needed inside the launch (MI355X_MICROARCH.md, inter-workgroup
// visibility).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fl {

constexpr uint64_t EMPTY = ~0ull;
constexpr uint64_t PENDING = ~0ull - 1;
constexpr int N_TABLES = 14;        // 0,1: IPv4 fast chain; 2..13: generic levels 0..11
constexpr int MAX_PROBE = 4096;
constexpr uint32_t FAIL = 0xFFFFFFFFu;

enum : uint32_t { ERR_TABLE_FULL = 1, ERR_FLOWS_FULL = 2, ERR_SPIN = 4, ERR_CAPACITY = 8 };

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

constexpr uint32_t MAX_TABLE_SLOTS = 1u << 27;  // per table (T1 words keep s0 in 31 bits when wide)
constexpr uint32_t MAX_FLOWS = 1u << 26;        // dense ids (the exact engine packs id << 38 | position)

struct TableSet {
    unsigned long long* tab[N_TABLES];  // (C + 1) entries of {key, val}; entry C holds the word EMPTY
    uint32_t C;                          // power of two, <= MAX_TABLE_SLOTS
    uint32_t wide;                       // the IPv4 chain's wide level-1 words (C >= 2^24, v4_t1_word)
    uint32_t fmax;                       // dense id capacity
    uint32_t* n_flows;
    uint32_t* err;
    uint8_t* flow_key;                   // [fmax][56] canonical key of each dense id
};

// Returns the slot of `w` in table t, inserting it if absent (insert=true).
// Each probe loads the whole 16-byte entry {key, val}; *val_out receives the
// value word seen with the matching key (possibly stale: EMPTY/PENDING), so a
// final-level lookup of a published flow costs one round trip.
// h0: the probe's first slot (tab_slot: the word's own hash).
__device__ __forceinline__ uint32_t tab_slot_at(const TableSet& T, int t, uint64_t w, uint32_t h0, bool insert,
                                               unsigned long long* val_out = nullptr) {
    unsigned long long* tab = T.tab[t];
    if (val_out) *val_out = EMPTY;
    if (w == EMPTY) return T.C;  // the sentinel word has a dedicated slot
    uint32_t h = h0 & (T.C - 1);
    for (int p = 0; p < MAX_PROBE; p++) {
        const ulonglong2 e = *reinterpret_cast<const ulonglong2*>(&tab[2 * h]);
        if (e.x == w) {
            if (val_out) *val_out = e.y;
            return h;
        }
        if (e.x == EMPTY) {
            if (!insert) return FAIL;
            unsigned long long old = atomicCAS(&tab[2 * h], EMPTY, (unsigned long long)w);
            if (old == EMPTY || old == w) return h;
        }
        h = (h + 1) & (T.C - 1);
    }
    atomicOr(T.err, ERR_TABLE_FULL);
    return FAIL;
}
__device__ __forceinline__ uint32_t tab_slot(const TableSet& T, int t, uint64_t w, bool insert,
                                            unsigned long long* val_out = nullptr) {
    return tab_slot_at(T, t, w, (uint32_t)mix64(w), insert, val_out);
}

// The IPv4 fast chain's second-level word.  Tables of fewer than 2^24 slots
// keep s0 (which can be the sentinel slot C) in 24 bits beside the ports and
// the protocol; larger tables ("wide", 8M flows and more) keep s0 in 31 bits,
// the ports and one protocol bit: TCP and UDP only (v4_fast), every other
// protocol takes the generic chain.  A key always takes the same chain, so
// either is exact.  (TableSet::wide also forces the wide layout on small
// tables: FLUERE_WIDE_TABLES, a test seam for these paths.)
__device__ __forceinline__ bool v4_fast(const TableSet& T, uint32_t proto) {
    return !T.wide || proto == 6u || proto == 17u;
}
__device__ __forceinline__ uint64_t v4_t1_word(const TableSet& T, uint32_t s0, uint32_t ports, uint32_t proto) {
    return !T.wide ? ((uint64_t)s0 << 40) | ((uint64_t)ports << 8) | proto
                   : ((uint64_t)s0 << 33) | ((uint64_t)ports << 1) | (proto == 17u ? 1u : 0u);
}

// The IPv4 fast chain in one round trip: T1's probe starts at a hash of the
// whole key (lo_ip, hi_ip, ports, proto), not of its word, which holds T0's
// slot s0 -- so the first probes of both tables are in flight together, and
// T1's word is compared once s0 is known.  (The word still decides: a slot
// holds exactly one word, and a key always starts its probe at one place.)
__device__ __forceinline__ uint32_t v4_t1_start(uint32_t lo, uint32_t hi, uint32_t ports, uint32_t proto) {
    return (uint32_t)mix64((((uint64_t)lo << 32) | hi) ^ mix64(((uint64_t)ports << 8) | proto | (1ull << 48)));
}
__device__ __forceinline__ void v4_slots(const TableSet& T, uint32_t lo, uint32_t hi, uint32_t ports, uint32_t proto,
                                         bool insert, uint32_t& s0, uint32_t& s1, unsigned long long* v) {
    const uint64_t w0 = ((uint64_t)lo << 32) | hi;
    const uint32_t h1 = v4_t1_start(lo, hi, ports, proto) & (T.C - 1);
    const ulonglong2 e1 = *reinterpret_cast<const ulonglong2*>(&T.tab[1][2 * h1]);  // (in flight with T0's probe)
    s1 = FAIL;
    *v = EMPTY;
    s0 = tab_slot(T, 0, w0, insert);
    if (s0 == FAIL) return;
    const uint64_t w1 = v4_t1_word(T, s0, ports, proto);
    if (w1 != EMPTY && e1.x == w1) {  // the first probe hit
        s1 = h1;
        *v = e1.y;
        return;
    }
    s1 = tab_slot_at(T, 1, w1, h1, insert, v);
}

// Canonical key: 14 little-endian u32 words (also fluere_flow_summary.key):
//   w[0..4) lo_ip, w[4..8) hi_ip (big-endian numeric words, IPv4 in w[0] / w[4])
//   w[8]  = lo_port << 16 | hi_port
//   w[9]  = kind << 8 | proto          (kind bit0: IPv6, bit1: MACs in key)
//   w[10] = lo_mac[0..4) BE, w[11] = lo_mac[4..6) BE << 16
//   w[12] = hi_mac[0..4) BE, w[13] = hi_mac[4..6) BE << 16
struct CKey {
    uint32_t w[14];
};

// Dense id of a final-level slot; the first caller assigns it.
//
// CDNA waves have no independent thread scheduling, and a retry loop whose
// exit is per-lane proved fragile here, so the only loop is wave-uniform
// (exit decided by a ballot).  In each iteration every lane that still needs
// an id makes ONE attempt: CAS EMPTY->PENDING; the winner takes a dense id
// and publishes it in the same branch, lanes that read a published id are
// done, lanes that read PENDING retry next iteration (the claimer -- in this
// wave or another -- publishes right after its claim, so the bounded retry
// terminates).  Everything another workgroup can observe is a 64-bit atomic
// (memory-side on MI355X, coherent across XCDs).
__device__ __forceinline__ uint32_t dense_id(const TableSet& T, int t, uint32_t s, bool insert, const CKey& key,
                                             const uint32_t (&chain)[N_TABLES], uint32_t* chain_out,
                                             unsigned long long v0) {
    // v0: the value word loaded with the key (stale reads can only show
    // EMPTY/PENDING, never a wrong id)
    unsigned long long* val = &T.tab[t][2 * s + 1];
    if (v0 < PENDING) return (uint32_t)v0;
    if (!insert) {
        v0 = atomicOr(val, 0ull);
        return v0 < PENDING ? (uint32_t)v0 : FAIL;
    }
    uint32_t res = FAIL;
    bool need = true, try_cas = true;
    for (int spins = 0; spins < (1 << 20); spins++) {
        if (__ballot(need) == 0) break;
        if (need) {
            // Claim attempts are CAS; after a lost claim (PENDING) the lane polls
            // with coherent atomic loads, so the many waiting workgroups do not
            // queue read-modify-writes in front of the claimer's publish.  Only a
            // CAS that returned EMPTY claims; a poll reading EMPTY retries the CAS.
            const bool cas = try_cas;
            unsigned long long v = cas ? atomicCAS(val, EMPTY, PENDING)
                                       : __hip_atomic_load(val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            try_cas = v == EMPTY;
            if (cas && v == EMPTY) {
                uint32_t d = atomicAdd(T.n_flows, 1u);
                if (d >= T.fmax) {
                    atomicOr(T.err, ERR_FLOWS_FULL);
                    d = FAIL;
                } else {
                    uint32_t* dst = (uint32_t*)(T.flow_key + (size_t)d * 56);
#pragma unroll
                    for (int k = 0; k < 14; k++) dst[k] = key.w[k];
                    if (chain_out) {  // table slots of this flow's chain, for O(flows) cleanup
#pragma unroll
                        for (int j = 0; j < N_TABLES; j++) chain_out[(size_t)d * N_TABLES + j] = chain[j];
                    }
                }
                atomicExch(val, (unsigned long long)d);
                res = d;
                need = false;
            } else if (v != PENDING && v != EMPTY) {
                res = (uint32_t)v;
                need = false;
            }
        }
        if (__ballot(need) != 0) {  // back off: ~0.1 us, then ~0.5 us, then ~2 us between polls
            if (spins < 4) __builtin_amdgcn_s_sleep(4);
            else if (spins < 16) __builtin_amdgcn_s_sleep(16);
            else __builtin_amdgcn_s_sleep(64);
        }
    }
    if (need) atomicOr(T.err, ERR_SPIN);
    return res;
}

// Endpoint comparison (ip, port, mac) lexicographic in key-field order;
// returns true when src > dst (the packet travels hi -> lo).
__device__ __forceinline__ bool src_gt_dst(const uint32_t* sip, const uint32_t* dip, uint32_t sp, uint32_t dp,
                                          uint64_t smac, uint64_t dmac, bool v6, bool macs) {
    if (sip[0] != dip[0]) return sip[0] > dip[0];
    if (v6) {
#pragma unroll
        for (int k = 1; k < 4; k++)
            if (sip[k] != dip[k]) return sip[k] > dip[k];
    }
    if (sp != dp) return sp > dp;
    if (macs && smac != dmac) return smac > dmac;
    return false;
}

}  // namespace fl
