// synth.h -- counter-based synthetic pcap generator.
//
// Every byte of packet i is a pure function of (cfg, i), so the host image
// (fluere_synth_host) and the device generator (fluere_synth_device) produce
// identical captures and any packet range can be generated independently on
// any GPU shard.  Compiled for host and device from the same source.
#pragma once
#include <stdint.h>

#include "../../include/fluere_gpu.h"

#ifndef FL_HD
#define FL_HD __host__ __device__ inline
#endif

namespace synth {

constexpr uint32_t kT0 = 1700000000u;  // capture start (s); +1 us per packet
constexpr uint32_t kSnap = 65535;

FL_HD uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
FL_HD uint64_t rnd(uint64_t seed, uint64_t stream, uint64_t i) {
    return mix64(mix64(seed + stream * 0x9E3779B97F4A7C15ull) + i * 0xD1B54A32D192ED03ull);
}

struct Flow {
    uint32_t a_ip, b_ip;
    uint16_t a_port, b_port;
    uint8_t proto;
    uint8_t closer;  // 0 none, 1 FIN+ACK, 2 RST (IMIX TCP flows only)
    uint8_t a_mac[6], b_mac[6];
};

FL_HD uint16_t pick_port(uint64_t r) {
    uint16_t p = (uint16_t)(1024 + r % 64000);
    return p == 4789 ? 4790 : p;  // 53 and 4789 never appear
}

FL_HD Flow flow(const fluere_synth_cfg& c, uint32_t f) {
    Flow F;
    F.a_ip = 0x0A000000u | (f & 0x7FFFFFu);                        // 10.0-127.x.x, unique per f
    F.b_ip = 0x0A800000u | (uint32_t)(rnd(c.seed, 3, f) & 0x7FFFFFu);  // 10.128-255.x.x
    F.a_port = pick_port(rnd(c.seed, 4, f));
    F.b_port = pick_port(rnd(c.seed, 5, f));
    F.proto = 17;
    F.closer = 0;
    if (c.kind == FLUERE_SYNTH_IMIX || c.kind == FLUERE_SYNTH_SLOW) {
        F.proto = (rnd(c.seed, 6, f) & 1) ? 6 : 17;
        if (F.proto == 6) {
            uint32_t r = (uint32_t)(rnd(c.seed, 15, f) % 100);
            F.closer = r < 20 ? 1 : (r < 25 ? 2 : 0);
        }
    }
    uint64_t ma = rnd(c.seed, 7, f), mb = rnd(c.seed, 8, f);
    for (int k = 0; k < 6; k++) {
        F.a_mac[k] = (uint8_t)(ma >> (8 * k));
        F.b_mac[k] = (uint8_t)(mb >> (8 * k));
    }
    F.a_mac[0] = (uint8_t)((F.a_mac[0] & 0xFC) | 0x02);  // unicast, locally administered
    F.b_mac[0] = (uint8_t)((F.b_mac[0] & 0xFC) | 0x02);
    return F;
}

FL_HD bool tcp_kind(uint32_t k) { return k == FLUERE_SYNTH_TCP || k == FLUERE_SYNTH_TCP_BACKTIME; }

// Capture time of packet i, microseconds after kT0: +1 us per packet; with
// FLUERE_SYNTH_TCP_BACKTIME 1 % of the packets carry a time up to 5 ms earlier
// (merged or multi-queue captures are slightly out of order).
FL_HD uint64_t time_us(const fluere_synth_cfg& c, uint64_t i) {
    if (c.kind == FLUERE_SYNTH_TCP_BACKTIME && rnd(c.seed, 32, i) % 100 == 0) {
        const uint64_t back = 1 + rnd(c.seed, 33, i) % 5000;
        return i >= back ? i - back : 0;
    }
    return i;
}

// Frame length of packet i (bytes on the wire, == caplen == orig_len).
FL_HD uint32_t frame_len(const fluere_synth_cfg& c, uint64_t i) {
    if (c.kind != FLUERE_SYNTH_IMIX && !tcp_kind(c.kind) && c.kind != FLUERE_SYNTH_SLOW) return 64;
    uint32_t r = (uint32_t)(rnd(c.seed, 14, i) % 12);
    return r < 7 ? (c.kind == FLUERE_SYNTH_SLOW ? 128 : 64) : (r < 11 ? 576 : 1500);
}

// Schedule: which flow packet i belongs to, its direction and TCP flags.
struct Slot {
    uint32_t f;
    uint8_t rev;
    uint8_t tcp_flags;
};

FL_HD Slot slot(const fluere_synth_cfg& c, uint64_t i) {
    Slot s;
    uint64_t F = c.n_flows ? c.n_flows : 1;
    s.rev = (uint8_t)((rnd(c.seed, 2, i) % 100) < c.rev_pct);
    s.tcp_flags = (uint8_t)(0x10 | ((rnd(c.seed, 16, i) & 1) ? 0x08 : 0));  // ACK (+PSH)
    if ((c.kind == FLUERE_SYNTH_IMIX || c.kind == FLUERE_SYNTH_SLOW) && c.n_packets >= 2 * F) {
        // [0, F): opening packet of flow i (forward; SYN for TCP)
        // [N-F, N): one packet per flow; TCP closers send FIN+ACK / RST here
        // otherwise: random flow, ACK (+PSH) for TCP
        if (i < F) {
            s.f = (uint32_t)i;
            s.rev = 0;
            s.tcp_flags = 0x02;
        } else if (i >= c.n_packets - F) {
            s.f = (uint32_t)(i - (c.n_packets - F));
            s.tcp_flags = 0xFF;  // resolved from the flow's closer kind
        } else {
            s.f = (uint32_t)(rnd(c.seed, 1, i) % F);
        }
        return s;
    }
    s.f = (uint32_t)(rnd(c.seed, 1, i) % F);
    return s;
}

FL_HD void put16(uint8_t* p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }
FL_HD void put32(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}
FL_HD void put32le(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}

// ---------------------------------------------------------------------------
// FLUERE_SYNTH_TCP: TCP as captures show it.  Packet i belongs to lane
// l = i % L (L = n_flows concurrent lanes) at lane position j = i / L; a lane
// runs a sequence of connections of a fixed length n (per lane), connection
// m = j / n, position k = j % n.  Lane types (rnd(seed, 20, l) % 100):
//   [0, 40)  TCP, 3-way handshake, data, 4-way close FIN -> ACK -> FIN -> ACK
//            (the closer is the client or the server); half of these lanes
//            reuse one 5-tuple for every connection (a closed key reopens)
//   [40, 50) TCP, handshake, data, RST (either side)
//   [50, 60) TCP, handshake, data, never closed
//   [60, 65) TCP, mid-stream: the lane's first connection starts without a
//            SYN (data, then the 4-way close); later connections are normal
//   [65, 100) UDP, both directions
// Lanes [0, E) (E = L / 64) carry 8 elephant flows: lane g of an elephant
// (g = l % 8) opens it with a SYN at its first packet; every other packet of
// those lanes is data, so each elephant holds ~1/512 of the capture.
// In every reference rule this exercises: the SYN gate drops the peer's ACK /
// FIN / ACK after the first FIN closed the flow (offline_fluereflows.rs:101-113,
// 152-157), RST closes, reopened keys, flows that never see a SYN.
// ---------------------------------------------------------------------------
struct Pkt {
    uint32_t a_ip, b_ip;        // client, server
    uint16_t a_port, b_port;
    uint8_t proto, rev, tflags;
    uint8_t a_mac[6], b_mac[6];
    uint8_t cls;                // FLUERE_SYNTH_SLOW: 0 IPv4, 1 IPv6, 2 VXLAN, 3 IPv4 with options
};

FL_HD void lane_macs(const fluere_synth_cfg& c, uint64_t l, Pkt& p) {
    uint64_t ma = rnd(c.seed, 7, l), mb = rnd(c.seed, 8, l);
    for (int k = 0; k < 6; k++) {
        p.a_mac[k] = (uint8_t)(ma >> (8 * k));
        p.b_mac[k] = (uint8_t)(mb >> (8 * k));
    }
    p.a_mac[0] = (uint8_t)((p.a_mac[0] & 0xFC) | 0x02);
    p.b_mac[0] = (uint8_t)((p.b_mac[0] & 0xFC) | 0x02);
}

FL_HD Pkt tcp_real(const fluere_synth_cfg& c, uint64_t i) {
    Pkt p;
    p.cls = 0;
    const uint64_t L = c.n_flows ? c.n_flows : 1;
    const uint64_t l = i % L, j = i / L;
    const uint64_t E = L / 64;
    const bool data_rev = (rnd(c.seed, 2, i) % 100) < c.rev_pct;
    const uint8_t data_flags = (uint8_t)(0x10 | ((rnd(c.seed, 16, i) & 1) ? 0x08 : 0));  // ACK (+PSH)
    if (l < E) {  // elephant g: lane g opens it
        const uint64_t g = l % 8;
        lane_macs(c, g, p);
        p.a_ip = 0x0A7F0000u | (uint32_t)g;
        p.b_ip = 0x0AFF0000u | (uint32_t)g;
        p.a_port = pick_port(rnd(c.seed, 4, g));
        p.b_port = 443;
        p.proto = 6;
        const bool open = l == g && j == 0;
        p.rev = open ? 0 : data_rev;
        p.tflags = open ? 0x02 : data_flags;
        return p;
    }
    lane_macs(c, l, p);
    const uint32_t type = (uint32_t)(rnd(c.seed, 20, l) % 100);
    const uint64_t lens[8] = {5, 7, 8, 12, 16, 24, 48, 200};
    const uint64_t n = lens[rnd(c.seed, 22, l) & 7];
    const uint64_t m = j / n, k = j % n;
    const bool reuse = type < 40 && (rnd(c.seed, 23, l) & 1);
    p.a_ip = 0x0A000000u | (uint32_t)(l & 0x7FFFFFu);
    p.b_ip = 0x0A800000u | (uint32_t)(rnd(c.seed, 3, l) & 0x7FFFFFu);
    p.a_port = pick_port(rnd(c.seed, 4, reuse ? l : l * 0x10001ull + m));
    p.b_port = pick_port(rnd(c.seed, 5, l));
    p.proto = type < 65 ? 6 : 17;
    p.rev = data_rev;
    p.tflags = data_flags;
    if (p.proto == 17) return p;
    const bool server_closes = rnd(c.seed, 24, l * 0x10001ull + m) & 1;
    const bool midstream = type >= 60 && m == 0;
    if (!midstream) {  // 3-way handshake
        if (k == 0) { p.rev = 0; p.tflags = 0x02; return p; }            // SYN
        if (k == 1) { p.rev = 1; p.tflags = 0x12; return p; }            // SYN+ACK
        if (k == 2) { p.rev = 0; p.tflags = 0x10; return p; }            // ACK
    }
    if (type < 40 || type >= 60) {  // 4-way close in the last four packets
        if (k + 4 >= n && n >= 7) {
            const uint64_t q = k + 4 - n;  // 0 FIN, 1 ACK, 2 FIN, 3 ACK
            const bool first_side = server_closes;  // rev of the first FIN
            p.rev = (q == 0 || q == 3) ? first_side : !first_side;
            p.tflags = (q == 0 || q == 2) ? 0x11 : 0x10;
            return p;
        }
    } else if (type < 50) {  // RST after the data
        if (k + 1 == n) { p.rev = server_closes; p.tflags = 0x04 | (rnd(c.seed, 25, i) & 1 ? 0x10 : 0); return p; }
    }
    return p;
}

// The header fields of packet i: the schedule of the kind.
FL_HD Pkt pkt(const fluere_synth_cfg& c, uint64_t i) {
    if (tcp_kind(c.kind)) return tcp_real(c, i);
    Pkt p;
    Slot s = slot(c, i);
    Flow F = flow(c, s.f);
    uint8_t tflags = s.tcp_flags;
    if (tflags == 0xFF)
        tflags = F.closer == 1 ? 0x11 : (F.closer == 2 ? 0x04 : (uint8_t)(0x10 | ((rnd(c.seed, 16, i) & 1) ? 0x08 : 0)));
    p.a_ip = F.a_ip; p.b_ip = F.b_ip; p.a_port = F.a_port; p.b_port = F.b_port;
    p.proto = F.proto; p.rev = s.rev; p.tflags = tflags;
    p.cls = 0;
    if (c.kind == FLUERE_SYNTH_SLOW) {
        const uint32_t r = (uint32_t)(rnd(c.seed, 30, s.f) & 3);
        p.cls = r < 2 ? 1 : (uint8_t)r;
    }
    for (int k = 0; k < 6; k++) { p.a_mac[k] = F.a_mac[k]; p.b_mac[k] = F.b_mac[k]; }
    return p;
}

// Writes the 16-byte pcap record header and the frame of packet i at dst.
// Returns bytes written (16 + frame_len).
FL_HD uint32_t write_record(const fluere_synth_cfg& c, uint64_t i, uint8_t* dst) {
    const uint32_t L0 = frame_len(c, i);
    uint32_t L = L0;
    const uint64_t ts = time_us(c, i);
    put32le(dst + 0, kT0 + (uint32_t)(ts / 1000000u));
    put32le(dst + 4, (uint32_t)(ts % 1000000u));
    put32le(dst + 8, L);
    put32le(dst + 12, L);
    uint8_t* e = dst + 16;
    const Pkt P = pkt(c, i);
    const uint8_t tflags = P.tflags;
    uint32_t sip = P.rev ? P.b_ip : P.a_ip, dip = P.rev ? P.a_ip : P.b_ip;
    uint16_t sp = P.rev ? P.b_port : P.a_port, dp = P.rev ? P.a_port : P.b_port;
    const uint8_t* smac = P.rev ? P.b_mac : P.a_mac;
    const uint8_t* dmac = P.rev ? P.a_mac : P.b_mac;
    for (int k = 0; k < 6; k++) { e[k] = dmac[k]; e[6 + k] = smac[k]; }
    uint32_t o = 12;
    if (c.kind == FLUERE_SYNTH_VLAN64) {
        put16(e + 12, 0x8100);
        put16(e + 14, (uint32_t)(rnd(c.seed, 17, P.a_ip & 0x7FFFFFu) & 0x0FFF));
        o = 16;
    }
    uint32_t dsel = (uint32_t)(rnd(c.seed, 10, i) & 3);  // DSCP 0, 10, 46, 1 (1 is unmapped -> tos 0)
    const uint32_t dscp = dsel == 0 ? 0 : dsel == 1 ? 10 : dsel == 2 ? 46 : 1;
    const uint8_t ttl = (uint8_t)(32 + rnd(c.seed, 9, i) % 97);
    if (P.cls == 2) {  // VXLAN: outer IPv4/UDP between two tunnel endpoints, then the inner frame
        put16(e + o, 0x0800);
        uint8_t* ip = e + o + 2;
        const uint32_t iplen = L - (o + 2);
        ip[0] = 0x45; ip[1] = 0;
        put16(ip + 2, iplen);
        put16(ip + 4, (uint32_t)(rnd(c.seed, 26, i) & 0xFFFF));
        put16(ip + 6, 0x4000);
        ip[8] = 64; ip[9] = 17;
        put16(ip + 10, 0);
        put32(ip + 12, 0xC0A80001u);  // 192.168.0.1 -> 192.168.0.2
        put32(ip + 16, 0xC0A80002u);
        uint32_t sum = 0;
        for (int k = 0; k < 20; k += 2) sum += ((uint32_t)ip[k] << 8) | ip[k + 1];
        while (sum >> 16) sum = (sum & 0xFFFF) + (sum >> 16);
        put16(ip + 10, ~sum & 0xFFFF);
        uint8_t* u = ip + 20;
        put16(u, 49152 + (uint32_t)(rnd(c.seed, 27, i) & 0x3FFF));
        put16(u + 2, 4789);
        put16(u + 4, iplen - 20);
        put16(u + 6, 0);
        const uint8_t vx[8] = {0x08, 0, 0, 0, 0, 0, 0x64, 0};  // the VXLAN header keys.rs:23 matches (VNI 100)
        for (int k = 0; k < 8; k++) u[8 + k] = vx[k];
        e = u + 16;  // inner Ethernet frame
        for (int k = 0; k < 6; k++) { e[k] = dmac[k]; e[6 + k] = smac[k]; }
        L = L - (uint32_t)(e - (dst + 16));  // inner frame length
    }
    uint8_t* l4;
    uint32_t l4len, hl;
    if (P.cls == 1) {  // IPv6: fd00::<v4 address> endpoints
        put16(e + o, 0x86DD);
        uint8_t* ip = e + o + 2;
        const uint32_t plen6 = L - (o + 2) - 40;
        put32(ip, 0x60000000u | (dscp << 22) | (uint32_t)(rnd(c.seed, 11, i) & 0xFFFFF));
        put16(ip + 4, plen6);
        ip[6] = P.proto;
        ip[7] = ttl;
        for (int h = 0; h < 2; h++) {
            uint8_t* a = ip + 8 + 16 * h;
            for (int k = 0; k < 16; k++) a[k] = 0;
            a[0] = 0xFD;
            put32(a + 12, h ? dip : sip);
        }
        l4 = ip + 40;
        l4len = plen6;
    } else {  // IPv4 (cls 3: one 4-byte option word, ihl 6)
        put16(e + o, 0x0800);
        uint8_t* ip = e + o + 2;
        const uint32_t iplen = L - (o + 2), ihl = P.cls == 3 ? 6 : 5;
        ip[0] = (uint8_t)(0x40 | ihl);
        ip[1] = (uint8_t)(dscp << 2);
        put16(ip + 2, iplen);
        put16(ip + 4, (uint32_t)(rnd(c.seed, 11, i) & 0xFFFF));
        put16(ip + 6, 0x4000);  // DF
        ip[8] = ttl;
        ip[9] = P.proto;
        put16(ip + 10, 0);
        put32(ip + 12, sip);
        put32(ip + 16, dip);
        if (ihl == 6) put32(ip + 20, 0x01010100u);  // NOP NOP NOP EOL
        uint32_t sum = 0;
        for (uint32_t k = 0; k < 4 * ihl; k += 2) sum += ((uint32_t)ip[k] << 8) | ip[k + 1];
        while (sum >> 16) sum = (sum & 0xFFFF) + (sum >> 16);
        put16(ip + 10, ~sum & 0xFFFF);
        l4 = ip + 4 * ihl;
        l4len = iplen - 4 * ihl;
    }
    put16(l4, sp);
    put16(l4 + 2, dp);
    if (P.proto == 6) {
        put32(l4 + 4, (uint32_t)rnd(c.seed, 18, i));
        put32(l4 + 8, (uint32_t)rnd(c.seed, 19, i));
        l4[12] = 0x50;
        l4[13] = tflags;
        put16(l4 + 14, 0xFFFF);
        put16(l4 + 16, 0);
        put16(l4 + 18, 0);
        hl = 20;
    } else {
        put16(l4 + 4, l4len);
        put16(l4 + 6, 0);
        hl = 8;
    }
    uint8_t* pay = l4 + hl;
    uint32_t plen = l4len - hl;
    uint64_t base = rnd(c.seed, 12, i);
    for (uint32_t k = 0; k < plen; k += 8) {
        uint64_t w = mix64(base + k * 0x9E3779B97F4A7C15ull);
        for (uint32_t b = 0; b < 8 && k + b < plen; b++) pay[k + b] = (uint8_t)(w >> (8 * b));
    }
    if (plen && pay[0] == 0x08) pay[0] = 0x09;  // never a VXLAN prefix
    return 16 + L0;
}

}  // namespace synth
