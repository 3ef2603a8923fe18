// parse.h -- device-side restatement of parse_keys + parse_fluereflow.
//
// Reference: src/net/parser/keys.rs:98-435 (parse_keys and helpers),
// src/net/parser/fluereflows.rs:30-388 (parse_fluereflow), ports.rs:7-58,
// flags.rs:13-38, tos.rs:3-30, time.rs:5-7.  pnet 0.35 view semantics as in
// SURVEY.md Appendix A.
//
// Two implementations of the same function:
//   * parse_fast: Ethernet/IPv4 with ihl == 5 and no VXLAN prefix -- every
//     field sits at a static offset inside the 80-byte record window that the
//     kernel loads with five 16-byte loads, so the parse is pure VALU on
//     registers.  This is every packet of the benchmark captures.
//   * parse_general: everything else the GPU supports (IPv4 options, IPv6,
//     ARP, VXLAN decapsulation, the 802.1Q misparse, ICMPv6/GRE port
//     quirks), reading bytes from global memory (L1/L2 hits: the window was
//     just loaded), including the src/net/parser/raw fallback.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fl {

enum : uint8_t { ST_OK = 0, ST_EMPTY = 1, ST_INVALID = 2, ST_UNKNOWN_ETHER = 3 };

// Result of both parsers for one packet.
struct PktInfo {
    uint8_t kst, fst;       // parse_keys / parse_fluereflow status
    uint8_t v6;             // key family (IpAddr::V6)
    uint8_t rv6;            // record family
    uint8_t kproto;         // Key.protocol
    uint16_t ksp, kdp;      // Key ports
    uint32_t sip[4], dip[4];  // Key IPs, big-endian words (IPv4 in [0])
    uint32_t frame_off;     // start of the keyed Ethernet frame inside the packet (VXLAN inner)
    uint8_t rprot, rtos, rttl, tflags;  // FluereRecord prot/tos/min_ttl, TCP flags byte (fin..cwr bits)
    uint16_t rsp, rdp;      // FluereRecord ports
    uint32_t rsip[4], rdip[4];  // FluereRecord source / destination
    uint32_t rpkt;          // FluereRecord min_pkt (= max_pkt)
    uint32_t doctets;       // packet_size() of the L3 view
    uint8_t raw;            // the src/net/parser/raw fallback produced key or record fields
};

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// DSCP -> TOS (tos.rs:3-30); unmapped -> 0 (fluereflows.rs:300-301, 352-353).
__device__ __forceinline__ uint8_t dscp_to_tos(uint32_t d) {
    // mapped set {0,8,10,...,40 step 2 from 8, 46, 48, 56}
    const uint64_t mask = (1ull << 0) | (1ull << 8) | (1ull << 10) | (1ull << 12) | (1ull << 14) | (1ull << 16) |
                          (1ull << 18) | (1ull << 20) | (1ull << 22) | (1ull << 24) | (1ull << 26) | (1ull << 28) |
                          (1ull << 30) | (1ull << 32) | (1ull << 34) | (1ull << 36) | (1ull << 38) | (1ull << 40) |
                          (1ull << 46) | (1ull << 48) | (1ull << 56);
    return ((mask >> (d & 63)) & 1) && d < 64 ? (uint8_t)(d * 4) : 0;
}

// ---------------------------------------------------------------------------
// Fast path over a register window: w[k] holds record bytes [4k, 4k+4)
// (little-endian words), record = 16-byte pcap header + frame.
// ---------------------------------------------------------------------------
struct Win {
    uint32_t w[20];
    __device__ __forceinline__ uint32_t b(int k) const { return (w[k >> 2] >> (8 * (k & 3))) & 0xFF; }
    __device__ __forceinline__ uint32_t be16(int k) const { return (b(k) << 8) | b(k + 1); }
    __device__ __forceinline__ uint32_t be32(int k) const { return (be16(k) << 16) | be16(k + 2); }
};

// Returns true if the packet was fully handled by the fast path (info filled,
// including drops); false -> run parse_general.  F = 16 (frame offset).
__device__ __forceinline__ bool parse_fast(const Win& W, uint32_t L, PktInfo& o) {
    constexpr int F = 16;
    if (L < 34) return false;
    if (W.be16(F + 12) != 0x0800 || (W.b(F + 14) & 0x0F) != 5) return false;
    uint32_t tl = W.be16(F + 16);
    uint32_t plen = tl > 20 ? tl - 20 : 0;
    uint32_t pe = min(plen, L - 34);  // Ipv4Packet::payload() length
    uint32_t proto = W.b(F + 23);
    if (pe >= 16) {                    // VXLAN probe on UDP-view payload (keys.rs:188)
        if (W.be32(F + 42) == 0x08000000u && W.be32(F + 46) == 0x00006400u) return false;
    }
    o.frame_off = 0;
    o.v6 = 0;
    o.rv6 = 0;
    o.kproto = (uint8_t)proto;
    o.sip[0] = W.be32(F + 26); o.dip[0] = W.be32(F + 30);
    o.sip[1] = o.sip[2] = o.sip[3] = 0;
    o.dip[1] = o.dip[2] = o.dip[3] = 0;
    for (int k = 0; k < 4; k++) { o.rsip[k] = o.sip[k]; o.rdip[k] = o.dip[k]; }
    o.kst = ST_OK;
    o.fst = ST_OK;
    o.raw = 0;
    // keys.rs:182-184: "UDP" payload (ip payload[8..]) empty -> EmptyPacket
    if (pe == 8) o.kst = ST_EMPTY;
    // parse_ports (ports.rs:7-58)
    uint32_t p01 = W.be16(F + 34), p23 = W.be16(F + 36);
    uint32_t sp = 0, dp = 0;
    bool perr = false;
    switch (proto) {
    case 0: case 1: case 2: case 4: case 47: case 50: case 51: case 58: break;
    case 6: if (pe >= 20) { sp = p01; dp = p23; } else perr = true; break;
    case 17: if (pe >= 8) { sp = p01; dp = p23; } else perr = true; break;
    case 53: if (pe >= 8) { sp = p01; dp = p23; } else { sp = dp = 53; } break;
    default:
        if (pe >= 4) {  // TCP view, UDP view, or raw generic/0x36 pattern (raw/mod.rs:247-305)
            if (pe < 8 && proto == 0x36) { sp = W.b(F + 34); dp = W.b(F + 35); }
            else { sp = p01; dp = p23; }
        }
    }
    if (perr) o.kst = ST_INVALID;
    o.ksp = (uint16_t)sp; o.kdp = (uint16_t)dp;
    if (proto == 47 && pe >= 4) { o.ksp = (uint16_t)p23; o.kdp = 0; }  // keys.rs:367-379
    // parse_fluereflow -> ipv4_packet (fluereflows.rs:249-336)
    o.doctets = max(tl, 20u);
    o.rttl = (uint8_t)W.b(F + 22);
    if (proto == 17 && pe >= 8 && (p23 == 53 || p01 == 53)) {  // DNS special case :255-291
        o.rsp = (uint16_t)p01; o.rdp = (uint16_t)p23;
        o.rpkt = pe;  // udp.packet_size()
        o.rprot = 17; o.rtos = 0; o.tflags = 0;
        return true;
    }
    o.rsp = perr ? 0 : (uint16_t)sp;
    o.rdp = perr ? 0 : (uint16_t)dp;
    o.rpkt = tl;
    o.rprot = (uint8_t)proto;
    o.rtos = dscp_to_tos(W.b(F + 15) >> 2);
    o.tflags = (proto == 6 && pe >= 20) ? (uint8_t)W.b(F + 34 + 13) : 0;
    return true;
}

// ---------------------------------------------------------------------------
// Middle path over a 128-byte register window (record bytes 0..127): the
// classes the hot parser leaves to k_slow that still have every field inside
// the window, parsed with selects instead of byte-serial reads:
//   * IPv4 with options (ihl 6..15), any IP protocol;
//   * IPv6 (no VXLAN prefix), any next header;
//   * VXLAN: outer Ethernet / IPv4 (ihl 5) / VXLAN header (keys.rs:186-200,
//     fluereflows.rs:100-110), inner Ethernet / IPv4 (ihl 5), any protocol.
// It computes exactly what parse_general computes for these packets, and only
// for valid ones: anything else (a drop, an empty UDP payload, a VXLAN prefix
// elsewhere, other ethertypes) returns false and takes parse_general.  Every
// byte it reads lies inside a span whose length it has checked, so bytes past
// the caplen (the next record) never decide a result.
// ---------------------------------------------------------------------------
struct Win32 {
    uint32_t w[32];
    __device__ __forceinline__ uint32_t b(int k) const { return (w[k >> 2] >> (8 * (k & 3))) & 0xFF; }
    __device__ __forceinline__ uint32_t be16(int k) const { return (b(k) << 8) | b(k + 1); }
    __device__ __forceinline__ uint32_t be32(int k) const { return (be16(k) << 16) | be16(k + 2); }
};

// byte k (< 16) / big-endian pair at k of a 16-byte view held as 4 little-endian words
__device__ __forceinline__ uint32_t view_b(const uint32_t (&v)[4], int k) { return (v[k >> 2] >> (8 * (k & 3))) & 0xFF; }
__device__ __forceinline__ uint32_t view_be16(const uint32_t (&v)[4], int k) { return (view_b(v, k) << 8) | view_b(v, k + 1); }

__device__ __forceinline__ bool parse_mid(const Win32& W, uint32_t L, PktInfo& o) {
    constexpr int F = 16;
    if (L < 34) return false;
    const uint32_t et = W.be16(F + 12);
    uint32_t v[4];  // the keyed L4 view: its first 16 bytes
    uint32_t pll, proto, doct, rpkt, ttl, tosb, frame_off = 0;
    uint32_t sip[4] = {0, 0, 0, 0}, dip[4] = {0, 0, 0, 0};
    bool v6 = false;
    if (et == 0x0800) {
        const uint32_t ihl = W.b(F + 14) & 0x0F;
        if (ihl < 5) return false;
        const uint32_t h = 4 * ihl, tl = W.be16(F + 16), plen = tl > h ? tl - h : 0, Pl = L - 14;
        const uint32_t pl0 = Pl <= h ? 0 : min(h + plen, Pl) - h;  // Ipv4Packet::payload() (v4_payload)
        // L4 bytes 0..15 at record byte 30 + h = 50 + 4s (s option words): words 12 + s .. 16 + s, shifted
        const uint32_t s = ihl - 5;
#pragma unroll
        for (int j = 0; j < 4; j++) v[j] = 0;
#pragma unroll
        for (uint32_t c = 0; c <= 10; c++)
#pragma unroll
            for (int j = 0; j < 4; j++)
                v[j] = s == c ? __builtin_amdgcn_alignbit(W.w[13 + c + j], W.w[12 + c + j], 16) : v[j];
        if (pl0 == 8) return false;  // empty "UDP" payload: EmptyPacket (keys.rs:182-184)
        const bool vx = pl0 >= 16 && v[2] == 0x00000008u && v[3] == 0x00640000u;  // is_vxlan (keys.rs:188)
        if (vx) {
            if (ihl != 5) return false;
            // inner Ethernet frame at frame byte 50, pl0 - 16 bytes long
            const uint32_t inl = pl0 - 16;
            if (inl < 14 || W.be16(F + 62) != 0x0800) return false;
            const uint32_t P2 = inl - 14;
            if (P2 < 20 || (W.b(F + 64) & 0x0F) != 5) return false;
            const uint32_t tl2 = W.be16(F + 66), plen2 = tl2 > 20 ? tl2 - 20 : 0;
            pll = P2 <= 20 ? 0 : min(20 + plen2, P2) - 20;
            proto = W.b(F + 73);
            ttl = W.b(F + 72);
            tosb = W.b(F + 65);
            sip[0] = W.be32(F + 76);
            dip[0] = W.be32(F + 80);
#pragma unroll
            for (int j = 0; j < 4; j++) v[j] = W.w[25 + j];  // inner L4 at record byte 100
            doct = 20 + plen2;  // v4_size
            rpkt = tl2;
            frame_off = 50;
        } else {
            pll = pl0;
            proto = W.b(F + 23);
            ttl = W.b(F + 22);
            tosb = W.b(F + 15);
            sip[0] = W.be32(F + 26);
            dip[0] = W.be32(F + 30);
            doct = h + plen;  // v4_size: 20 + options + (tl - h)
            rpkt = tl;
        }
    } else if (et == 0x86DD) {
        if (L < 54) return false;
        const uint32_t plf = W.be16(F + 18), Pl = L - 14;
        pll = Pl <= 40 ? 0 : min(40 + plf, Pl) - 40;  // v6_payload
#pragma unroll
        for (int j = 0; j < 4; j++) v[j] = __builtin_amdgcn_alignbit(W.w[18 + j], W.w[17 + j], 16);  // record byte 70
        if (pll == 8) return false;
        if (pll >= 16 && v[2] == 0x00000008u && v[3] == 0x00640000u) return false;
        v6 = true;
        proto = W.b(F + 20);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            sip[k] = W.be32(F + 22 + 4 * k);
            dip[k] = W.be32(F + 38 + 4 * k);
        }
        doct = 40 + plf;
        rpkt = plf;
        ttl = 0;
        tosb = (((W.b(F + 14) & 0x0F) << 4) | (W.b(F + 15) >> 4));  // traffic class
    } else {
        return false;
    }
    // parse_ports (ports.rs:7-58) over the L4 view
    const uint32_t p01 = view_be16(v, 0), p23 = view_be16(v, 2);
    uint32_t sp = 0, dp = 0;
    switch (proto) {
    case 0: case 1: case 2: case 4: case 47: case 50: case 51: case 58: break;
    case 6: if (pll < 20) return false; sp = p01; dp = p23; break;
    case 17: if (pll < 8) return false; sp = p01; dp = p23; break;
    case 53: if (pll >= 8) { sp = p01; dp = p23; } else { sp = dp = 53; } break;
    default:
        if (pll >= 4) {
            if (pll < 8 && proto == 0x36) { sp = view_b(v, 0); dp = view_b(v, 1); }
            else { sp = p01; dp = p23; }
        }
    }
    o.kst = ST_OK;
    o.fst = ST_OK;
    o.raw = 0;
    o.frame_off = frame_off;
    o.v6 = v6 ? 1 : 0;
    o.rv6 = o.v6;
    o.kproto = (uint8_t)proto;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        o.sip[k] = o.rsip[k] = sip[k];
        o.dip[k] = o.rdip[k] = dip[k];
    }
    o.ksp = (uint16_t)sp;
    o.kdp = (uint16_t)dp;
    if (!v6 && proto == 47 && pll >= 4) { o.ksp = (uint16_t)p23; o.kdp = 0; }                        // keys.rs:367-379
    if (v6 && proto == 58 && pll >= 4) { o.ksp = (uint16_t)view_b(v, 0); o.kdp = (uint16_t)view_b(v, 1); }  // keys.rs:403-409
    o.doctets = doct;
    o.rttl = (uint8_t)ttl;
    if (!v6 && proto == 17 && pll >= 8 && (p23 == 53 || p01 == 53)) {  // DNS (fluereflows.rs:255-291)
        o.rsp = (uint16_t)p01; o.rdp = (uint16_t)p23;
        o.rpkt = pll;
        o.rprot = 17; o.rtos = 0; o.tflags = 0;
        return true;
    }
    o.rsp = (uint16_t)sp; o.rdp = (uint16_t)dp;
    o.rpkt = rpkt;
    o.rprot = (uint8_t)proto;
    o.rtos = dscp_to_tos(tosb >> 2);
    o.tflags = (proto == 6 && pll >= 20) ? (uint8_t)view_b(v, 13) : 0;
    return true;
}

// ---------------------------------------------------------------------------
// General path: byte reads from global memory.  d = frame start, L = caplen.
// ---------------------------------------------------------------------------
// d: the frame in global memory.  s / sn: an optional staged copy of its
// first sn bytes (k_slow keeps one per lane in LDS: the parser's byte reads
// are a chain of dependent loads, an LDS round trip each instead of a global
// one); sn = 0 reads everything from d.
struct G {
    const uint8_t* d;
    const uint8_t* s = nullptr;
    uint32_t sn = 0;
    __device__ __forceinline__ uint32_t b(uint32_t k) const { return k < sn ? s[k] : d[k]; }
    __device__ __forceinline__ uint32_t be16(uint32_t k) const { return (b(k) << 8) | b(k + 1); }
    __device__ __forceinline__ uint32_t be32(uint32_t k) const { return (be16(k) << 16) | be16(k + 2); }
};

struct Span { uint32_t off, len; };

// pnet Ipv4Packet::payload() for an IPv4 view at [off, off+len)
__device__ __forceinline__ Span v4_payload(const G& g, Span i) {
    uint32_t h = (g.b(i.off) & 0x0F) * 4;
    uint32_t opt = h > 20 ? h - 20 : 0;
    uint32_t tl = g.be16(i.off + 2);
    uint32_t pl = tl > h ? tl - h : 0;
    uint32_t start = 20 + opt;
    if (i.len <= start) return {i.off, 0};
    uint32_t end = min(start + pl, i.len);
    return {i.off + start, end - start};
}
__device__ __forceinline__ uint32_t v4_size(const G& g, Span i) {
    uint32_t h = (g.b(i.off) & 0x0F) * 4;
    uint32_t tl = g.be16(i.off + 2);
    return 20 + (h > 20 ? h - 20 : 0) + (tl > h ? tl - h : 0);
}
__device__ __forceinline__ Span v6_payload(const G& g, Span i) {
    if (i.len <= 40) return {i.off, 0};
    uint32_t end = min(40u + g.be16(i.off + 4), i.len);
    return {i.off + 40, end - 40};
}
__device__ __forceinline__ bool is_vxlan(const G& g, Span u) {
    return u.len >= 8 && g.be32(u.off) == 0x08000000u && g.be32(u.off + 4) == 0x00006400u;
}

// ports.rs:7-58; returns false on NetError::InvalidPacket
__device__ __forceinline__ bool ports(const G& g, uint32_t proto, Span x, uint16_t& sp, uint16_t& dp) {
    sp = dp = 0;
    switch (proto) {
    case 0: case 1: case 2: case 4: case 47: case 50: case 51: case 58: return true;
    case 6: if (x.len < 20) return false; break;
    case 17: if (x.len < 8) return false; break;
    case 53: if (x.len < 8) { sp = dp = 53; return true; } break;
    default:
        if (x.len < 4) return true;
        if (x.len < 8 && proto == 0x36) { sp = (uint16_t)g.b(x.off); dp = (uint16_t)g.b(x.off + 1); return true; }
    }
    sp = (uint16_t)g.be16(x.off);
    dp = (uint16_t)g.be16(x.off + 2);
    return true;
}

__device__ __forceinline__ void ip4_words(const G& g, uint32_t off, uint32_t* w) {
    w[0] = g.be32(off); w[1] = w[2] = w[3] = 0;
}
__device__ __forceinline__ void ip6_words(const G& g, uint32_t off, uint32_t* w) {
    for (int k = 0; k < 4; k++) w[k] = g.be32(off + 4 * k);
}

// ipv4_keys (keys.rs:361-388)
__device__ __forceinline__ bool ipv4_keys(const G& g, Span i, PktInfo& o) {
    o.v6 = 0;
    ip4_words(g, i.off + 12, o.sip); ip4_words(g, i.off + 16, o.dip);
    o.kproto = (uint8_t)g.b(i.off + 9);
    Span pl = v4_payload(g, i);
    if (!ports(g, o.kproto, pl, o.ksp, o.kdp)) return false;
    if (o.kproto == 47 && pl.len >= 4) { o.ksp = (uint16_t)g.be16(pl.off + 2); o.kdp = 0; }
    return true;
}
// ipv6_keys (keys.rs:390-415)
__device__ __forceinline__ bool ipv6_keys(const G& g, Span i, PktInfo& o) {
    o.v6 = 1;
    ip6_words(g, i.off + 8, o.sip); ip6_words(g, i.off + 24, o.dip);
    o.kproto = (uint8_t)g.b(i.off + 6);
    Span pl = v6_payload(g, i);
    if (!ports(g, o.kproto, pl, o.ksp, o.kdp)) return false;
    if (o.kproto == 58 && pl.len >= 4) { o.ksp = (uint16_t)g.b(pl.off); o.kdp = (uint16_t)g.b(pl.off + 1); }
    return true;
}
// ---------------------------------------------------------------------------
// Raw fallback (src/net/parser/raw): the header the reference derives when
// pnet's typed views do not apply.  Byte reads from global memory; only
// packets outside the hot path get here.
// ---------------------------------------------------------------------------
struct RawHdr {
    bool has_src, has_dst, v6;
    uint32_t src[4], dst[4];
    uint16_t sport, dport;
    uint8_t proto;
    uint16_t length;  // u16 in RawProtocolHeader (raw/mod.rs)
    // Option fields the reference's tests assert (never read by the hot path;
    // flags only feed parse_flags of an empty slice, fluereflows.rs:151)
    bool has_flags, has_version, has_ethertype, has_payload;
    uint8_t flags, version;
    uint16_t ethertype;
    uint32_t payload_off, payload_len;  // payload = bytes [payload_off, +payload_len) of the G view
};

// raw/mod.rs:40-71 RawProtocolHeader::new (Option fields None)
__device__ __forceinline__ void raw_new(RawHdr& h, uint32_t sp, uint32_t dp, uint32_t proto, uint32_t len) {
    h.has_src = h.has_dst = h.v6 = false;
    for (int k = 0; k < 4; k++) h.src[k] = h.dst[k] = 0;
    h.sport = (uint16_t)sp; h.dport = (uint16_t)dp; h.proto = (uint8_t)proto; h.length = (uint16_t)len;
    h.has_flags = h.has_version = h.has_ethertype = h.has_payload = false;
    h.flags = h.version = 0;
    h.ethertype = 0;
    h.payload_off = h.payload_len = 0;
}
__device__ __forceinline__ void raw_payload(RawHdr& h, Span p, uint32_t off) {
    off = min(off, p.len);
    h.has_payload = true;
    h.payload_off = p.off + off;
    h.payload_len = p.len - off;
}

// protocols/icmp.rs:10-48
__device__ __forceinline__ bool raw_icmp(const G& g, Span p, RawHdr& h) {
    if (p.len < 4) return false;
    raw_new(h, g.b(p.off), g.b(p.off + 1), 1, p.len);
    if (p.len > 4) raw_payload(h, p, 4);
    h.has_flags = true; h.flags = (uint8_t)g.b(p.off);
    h.has_version = true; h.version = (uint8_t)g.b(p.off + 1);
    return true;
}

// protocols/openvpn.rs:155-220 (control packets :31-72, data packets :85-128)
__device__ __forceinline__ bool raw_openvpn(const G& g, Span p, RawHdr& h) {
    if (p.len < 9) return false;
    const uint32_t t = g.b(p.off);
    if (!((t >= 1 && t <= 9) || t == 0x40 || t == 0x41)) return false;
    raw_new(h, t, 0, 0x9B, p.len);
    raw_payload(h, p, 9);
    if (t == 6 || t == 9) {
        const Span ip = {p.off + 9, p.len - 9};
        if (ip.len >= 16 && ((g.b(ip.off) >> 4) & 0x0F) == 4) {
            h.has_src = h.has_dst = true;
            ip4_words(g, ip.off + 4, h.src); ip4_words(g, ip.off + 8, h.dst);
            h.sport = (uint16_t)g.be16(ip.off + 12); h.dport = (uint16_t)g.be16(ip.off + 14);
        }
    } else if (p.len >= 21 && (t == 0x40 || t == 0x41)) {
        h.has_src = h.has_dst = true;
        ip4_words(g, p.off + 9, h.src); ip4_words(g, p.off + 13, h.dst);
        h.sport = (uint16_t)g.be16(p.off + 17); h.dport = (uint16_t)g.be16(p.off + 19);
    }
    return true;
}

// protocols/mod.rs:48-84
__device__ __forceinline__ bool raw_parse_protocol(const G& g, Span p, uint32_t proto, RawHdr& h) {
    if (proto == 1 && raw_icmp(g, p, h)) return true;
    if (proto >= 170 && proto <= 172 && raw_openvpn(g, p, h)) return true;
    return raw_openvpn(g, p, h);
}

// raw/mod.rs:152-328 RawProtocolHeader::from_raw_packet
__device__ __attribute__((noinline)) bool raw_from_raw_packet(const G& g, Span p, uint32_t hint, RawHdr& h) {
    bool outer = false;
    uint32_t os = 0, od = 0, osp = 0, odp = 0, oproto = 0;
    if (p.len >= 20 && (g.b(p.off) >> 4) == 4) {
        const uint32_t hl = (g.b(p.off) & 0x0F) * 4;
        if (hl >= 20 && hl <= p.len) {
            outer = true;
            os = g.be32(p.off + 12); od = g.be32(p.off + 16);
            oproto = g.b(p.off + 9);
            if (hl + 4 <= p.len) { osp = g.be16(p.off + hl); odp = g.be16(p.off + hl + 2); }
        }
    }
    if (raw_parse_protocol(g, p, hint, h)) {
        if (outer) {  // fill what the protocol parser left unset from the outer IPv4 header
            if (!h.has_src) { h.has_src = true; h.src[0] = os; h.src[1] = h.src[2] = h.src[3] = 0; }
            if (!h.has_dst) { h.has_dst = true; h.dst[0] = od; h.dst[1] = h.dst[2] = h.dst[3] = 0; }
            if (h.sport == 0) h.sport = (uint16_t)osp;
            if (h.dport == 0) h.dport = (uint16_t)odp;
        }
        return true;
    }
    if (outer) {
        raw_new(h, osp, odp, oproto, p.len);
        raw_payload(h, p, 0);
        h.has_src = h.has_dst = true;
        h.src[0] = os; h.dst[0] = od;
        return true;
    }
    if (p.len < 4) return false;
    if (hint == 0x36) { raw_new(h, g.b(p.off), g.b(p.off + 1), hint, p.len); raw_payload(h, p, 2); }  // :271-283
    else { raw_new(h, g.be16(p.off), g.be16(p.off + 2), hint, p.len); raw_payload(h, p, hint == 0xb9 ? 4 : 0); }  // :249-304
    return true;
}

// ethertypes/vpn.rs:133-186 extract_ip_addresses
__device__ __forceinline__ void raw_extract_ips(const G& g, Span q, RawHdr& h) {
    if (q.len < 20) return;
    const uint32_t ver = g.b(q.off) >> 4;
    if (ver == 4) {
        h.has_src = h.has_dst = true; h.v6 = false;
        ip4_words(g, q.off + 12, h.src); ip4_words(g, q.off + 16, h.dst);
    } else if (ver == 6 && q.len >= 40) {
        h.has_src = h.has_dst = true; h.v6 = true;
        ip6_words(g, q.off + 8, h.src); ip6_words(g, q.off + 24, h.dst);
    }
}

// ethertypes/mod.rs:136-159 analyze_packet_structure -> payload start (len = none)
__device__ __forceinline__ uint32_t raw_custom_payload_start(const G& g, Span p) {
    const uint32_t b = g.b(p.off);
    const uint32_t hs = (b >= 0xB8 && b <= 0xBF) ? 8u : (b == 0x36 || b == 0x37) ? 6u : 4u;
    const bool has = (b >= 0xB8 && b <= 0xBF) || b == 0x36 || b == 0x37 || b == 0x6C || p.len > 4;
    return (has && p.len > hs) ? hs : 0xFFFFFFFFu;
}

// ethertypes/mod.rs:20-61 parse_ethertype.  Its 0x0806 arm (arp.rs:3-44) is
// unreachable from parse_fluereflow, which handles ARP itself; it is here so
// the reference's parse_ethertype tests pin this function whole.
__device__ __forceinline__ bool raw_parse_ethertype(const G& g, Span p, uint32_t et, RawHdr& h) {
    if (et == 0x0A08 || et == 0x4B65) {  // vpn.rs:15-56, :58-99
        if (p.len < 4) return false;
        raw_new(h, et == 0x0A08 ? 2186 : 19301, g.be16(p.off + 2), et == 0x0A08 ? 21 : 22, p.len);
        raw_payload(h, p, 4);
        raw_extract_ips(g, {p.off + 4, p.len - 4}, h);
        return true;
    }
    if (et == 0x0806) {  // arp.rs:3-44
        if (p.len < 28) return false;
        raw_new(h, g.be16(p.off + 6), 0, 0x08, p.len);
        h.has_src = h.has_dst = true;
        ip4_words(g, p.off + 14, h.src); ip4_words(g, p.off + 24, h.dst);
        h.has_ethertype = true; h.ethertype = 0x0806;
        return true;
    }
    if (et == 0x8847 || et == 0x8848) {  // mpls.rs:3-40
        if (p.len < 4) return false;
        const uint32_t label = (g.b(p.off) << 12) | (g.b(p.off + 1) << 4) | (g.b(p.off + 2) >> 4);
        raw_new(h, label & 0xFFFF, (g.b(p.off + 2) >> 1) & 7, 137, p.len);
        uint32_t off = 4;  // label stack walk (:18-26)
        if (!(g.b(p.off + 2) & 1))
            while (off + 4 <= p.len && !(g.b(p.off + off + 2) & 1)) off += 4;
        raw_payload(h, p, off);
        return true;
    }
    if (et == 0x12B5) {  // vxlan.rs:8-48
        if (p.len < 8 || !(g.be32(p.off) == 0x08000000u && g.be32(p.off + 4) == 0x00006400u)) return false;
        const uint32_t vni = (g.b(p.off + 4) << 16) | (g.b(p.off + 5) << 8) | g.b(p.off + 6);
        raw_new(h, 4789, vni & 0xFFFF, 0x12, p.len);
        raw_payload(h, p, 8);
        return true;
    }
    if (et == 0x88B8) {  // wireguard.rs:12-80
        if (p.len < 4) return false;
        const uint32_t t = g.b(p.off);
        if (t == 1 && p.len != 148) return false;
        if (t == 2 && p.len != 92) return false;
        if (t == 3 && p.len != 64) return false;
        if (t == 4 && p.len < 16) return false;
        if (t < 1 || t > 4) return false;
        raw_new(h, 0, 51820, t, p.len);
        raw_payload(h, p, 0);
        h.has_flags = true; h.flags = (uint8_t)t;
        h.has_version = true; h.version = 1;
        h.has_ethertype = true; h.ethertype = 0x88B8;
        return true;
    }
    if ((et >= 0xB800 && et <= 0xBFFF) || (et >= 0x3600 && et <= 0x36FF)) {  // mod.rs:107-134
        if (p.len < 4) return false;
        raw_new(h, g.be16(p.off), g.be16(p.off + 2), g.b(p.off), p.len);
        const uint32_t ps = raw_custom_payload_start(g, p);
        if (ps != 0xFFFFFFFFu) raw_payload(h, p, ps);
        return true;
    }
    return false;
}

// raw/mod.rs:330-349 RawProtocolHeader::from_ethertype
__device__ __forceinline__ bool raw_from_ethertype(const G& g, Span p, uint32_t et, RawHdr& h) {
    if (raw_parse_ethertype(g, p, et, h)) return true;
    if (et == 0x0800 && p.len >= 20) return raw_from_raw_packet(g, p, g.b(p.off + 9), h);
    return raw_from_raw_packet(g, p, et & 0xFF, h);
}

// arp_keys (keys.rs:345-359)
__device__ __forceinline__ void arp_keys(const G& g, Span a, PktInfo& o) {
    o.v6 = 0;
    ip4_words(g, a.off + 14, o.sip); ip4_words(g, a.off + 24, o.dip);
    o.ksp = o.kdp = 0; o.kproto = 4;
}
// vlan_keys (keys.rs:417-435): 0 ok, else NetError
__device__ __forceinline__ uint8_t vlan_keys(const G& g, Span v, PktInfo& o) {
    if (v.len < 4 + 14) return ST_INVALID;
    Span e = {v.off + 4, v.len - 4};
    uint32_t et = g.be16(e.off + 12);
    Span ip = {e.off + 14, e.len - 14};
    if (et == 0x0800) { if (ip.len < 20) return ST_INVALID; return ipv4_keys(g, ip, o) ? ST_OK : ST_INVALID; }
    if (et == 0x86DD) { if (ip.len < 40) return ST_INVALID; return ipv6_keys(g, ip, o) ? ST_OK : ST_INVALID; }
    return ST_UNKNOWN_ETHER;
}

// The general parser, inlined into its caller: k_slow, where every packet
// takes it (an out-of-line call saves and restores the callee's registers
// through scratch on every packet).
__device__ __forceinline__ void parse_general_inl(const uint8_t* d, uint32_t L, PktInfo& o, const uint8_t* staged = nullptr,
                                                  uint32_t staged_n = 0) {
    G g{d, staged, staged_n};
    o.kst = ST_OK; o.fst = ST_OK;
    o.v6 = 0; o.rv6 = 0; o.kproto = 0; o.ksp = o.kdp = 0;
    for (int k = 0; k < 4; k++) o.sip[k] = o.dip[k] = o.rsip[k] = o.rdip[k] = 0;
    o.frame_off = 0;
    o.rprot = o.rtos = o.rttl = o.tflags = 0;
    o.rsp = o.rdp = 0; o.rpkt = 0; o.doctets = 0;
    o.raw = 0;
    // ---------------- parse_keys (keys.rs:98-343)
    if (L == 0) o.kst = ST_EMPTY;
    else if (L < 14) o.kst = ST_INVALID;
    if (L < 14) { o.fst = ST_EMPTY; return; }  // fluereflows.rs:32-40
    uint32_t et = g.be16(12);
    Span P = {14, L - 14};
    Span pl = {14, 0};
    bool udp = false;
    uint8_t kouter = ST_OK, fouter = ST_OK;
    if (et == 0x86DD) {
        if (P.len < 40) { kouter = ST_EMPTY; fouter = ST_INVALID; }
        else { pl = v6_payload(g, P); udp = pl.len >= 8; }
    } else if (et == 0x0800) {
        if (P.len < 20) { kouter = ST_EMPTY; fouter = ST_INVALID; }
        else { pl = v4_payload(g, P); udp = pl.len >= 8; }
    } else if (et == 0x0806) {
        if (P.len < 28) kouter = ST_EMPTY;  // parse_fluereflow has no ARP arm here
    }
    Span kframe = {0, L}, fframe = {0, L};
    if (kouter == ST_OK && udp) {
        Span u = {pl.off + 8, pl.len - 8};
        if (u.len == 0) kouter = ST_EMPTY;  // keys.rs:182-184
        else if (is_vxlan(g, u)) {
            Span in = {u.off + 8, u.len - 8};
            if (in.len < 14) kouter = ST_EMPTY;  // keys.rs:192-193
            else kframe = in;
        }
    }
    if (fouter == ST_OK && udp) {
        Span u = {pl.off + 8, pl.len - 8};
        if (is_vxlan(g, u) && u.len - 8 >= 14) fframe = {u.off + 8, u.len - 8};  // fluereflows.rs:100-110
    }
    o.kst = kouter;
    if (kouter == ST_OK) {
        uint32_t et2 = g.be16(kframe.off + 12);
        Span P2 = {kframe.off + 14, kframe.len - 14};
        o.frame_off = kframe.off;
        if (et2 == 0x86DD) {
            if (P2.len < 40) o.kst = ST_EMPTY;
            else if (!ipv6_keys(g, P2, o)) o.kst = ST_INVALID;
        } else if (et2 == 0x0800) {
            if (P2.len < 20) o.kst = ST_EMPTY;
            else if (!ipv4_keys(g, P2, o)) o.kst = ST_INVALID;
        } else if (et2 == 0x0806 || et2 == 0x8035) {
            if (P2.len < 28) o.kst = ST_EMPTY;
            else arp_keys(g, P2, o);
        } else if (et2 == 0x8100) {
            if (P2.len < 4) o.kst = ST_EMPTY;
            else o.kst = vlan_keys(g, P2, o);
        } else {
            // keys.rs:252-313: the eager chain over the payload; the first Ok
            // wins: ipv4_keys, ipv6_keys, arp_keys, vlan_keys, then the raw
            // fallback (RawProtocolHeader::from_raw_packet with the low byte of
            // the ethertype as the protocol hint)
            uint8_t e = ST_INVALID;
            if (P2.len >= 20) e = ipv4_keys(g, P2, o) ? ST_OK : ST_INVALID;
            if (e != ST_OK && P2.len >= 40) e = ipv6_keys(g, P2, o) ? ST_OK : ST_INVALID;
            if (e != ST_OK && P2.len >= 28) { arp_keys(g, P2, o); e = ST_OK; }
            if (e != ST_OK && P2.len >= 4) e = vlan_keys(g, P2, o);
            if (e != ST_OK) {
                RawHdr h;
                o.raw = 1;
                if (raw_from_raw_packet(g, P2, et2 & 0xFF, h)) {
                    o.v6 = 0;  // from_raw_packet yields IPv4 addresses or none (0.0.0.0)
                    for (int k = 0; k < 4; k++) { o.sip[k] = h.src[k]; o.dip[k] = h.dst[k]; }
                    o.ksp = h.sport; o.kdp = h.dport; o.kproto = h.proto;
                    e = ST_OK;
                } else {
                    e = ST_UNKNOWN_ETHER;
                }
            }
            o.kst = e;
        }
    }
    // ---------------- parse_fluereflow (fluereflows.rs:30-199)
    if (fouter != ST_OK) { o.fst = fouter; return; }
    uint32_t et2 = g.be16(fframe.off + 12);
    Span P2 = {fframe.off + 14, fframe.len - 14};
    if (et2 == 0x0800) {
        if (P2.len < 20) { o.fst = ST_INVALID; return; }
        uint32_t proto = g.b(P2.off + 9);
        Span l4 = v4_payload(g, P2);
        o.doctets = v4_size(g, P2);
        o.rttl = (uint8_t)g.b(P2.off + 8);
        ip4_words(g, P2.off + 12, o.rsip); ip4_words(g, P2.off + 16, o.rdip);
        uint16_t sp, dp;
        bool ok = ports(g, proto, l4, sp, dp);
        if (proto == 17 && l4.len >= 8 && (g.be16(l4.off + 2) == 53 || g.be16(l4.off) == 53)) {
            o.rsp = (uint16_t)g.be16(l4.off); o.rdp = (uint16_t)g.be16(l4.off + 2);
            o.rpkt = l4.len; o.rprot = 17; o.rtos = 0; o.tflags = 0;
            return;
        }
        o.rsp = ok ? sp : 0; o.rdp = ok ? dp : 0;
        o.rpkt = g.be16(P2.off + 2);
        o.rprot = (uint8_t)proto;
        o.rtos = dscp_to_tos(g.b(P2.off + 1) >> 2);
        o.tflags = (proto == 6 && l4.len >= 20) ? (uint8_t)g.b(l4.off + 13) : 0;
    } else if (et2 == 0x86DD) {
        if (P2.len < 40) { o.fst = ST_INVALID; return; }
        uint32_t nh = g.b(P2.off + 6);
        Span l4 = v6_payload(g, P2);
        uint16_t sp, dp;
        if (!ports(g, nh, l4, sp, dp)) { o.fst = ST_INVALID; return; }
        uint32_t plf = g.be16(P2.off + 4);
        o.doctets = 40 + plf;
        ip6_words(g, P2.off + 8, o.rsip); ip6_words(g, P2.off + 24, o.rdip);
        o.rv6 = 1;
        o.rsp = sp; o.rdp = dp;
        o.rpkt = plf; o.rttl = 0; o.rprot = (uint8_t)nh;
        uint32_t tc = ((g.b(P2.off) & 0x0F) << 4) | (g.b(P2.off + 1) >> 4);
        o.rtos = dscp_to_tos(tc >> 2);
        o.tflags = (nh == 6 && l4.len >= 20) ? (uint8_t)g.b(l4.off + 13) : 0;
    } else if (et2 == 0x0806) {
        if (P2.len < 28) { o.fst = ST_INVALID; return; }
        o.doctets = 28; o.rpkt = 28; o.rprot = 4;
        ip4_words(g, P2.off + 14, o.rsip); ip4_words(g, P2.off + 24, o.rdip);
    } else {
        // fluereflows.rs:148-195: RawProtocolHeader::from_ethertype over the
        // whole frame; ttl None -> 0, tos 0, flags of an empty slice
        RawHdr h;
        o.raw = 1;
        if (!raw_from_ethertype(g, fframe, et2, h)) { o.fst = ST_UNKNOWN_ETHER; return; }
        o.rv6 = h.v6 ? 1 : 0;
        for (int k = 0; k < 4; k++) { o.rsip[k] = h.src[k]; o.rdip[k] = h.dst[k]; }
        o.doctets = h.length;
        o.rsp = h.sport; o.rdp = h.dport;
        o.rpkt = h.length; o.rttl = 0; o.rprot = h.proto; o.rtos = 0; o.tflags = 0;
    }
}

// Out of line for every other caller (one copy, no register pressure in the
// kernels whose packets rarely need it).
__device__ __attribute__((noinline)) void parse_general(const uint8_t* d, uint32_t L, PktInfo& o) {
    parse_general_inl(d, L, o);
}

}  // namespace fl
