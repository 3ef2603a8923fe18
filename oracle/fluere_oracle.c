/*
 * fluere_oracle.c -- TEST INFRASTRUCTURE ONLY (see fluere_oracle.h).
 *
 * Plain-C restatement of the reference CPU path of `fluere offline`.
 * Every function cites the reference file:line it restates.  pnet 0.35
 * packet views are restated inline (SURVEY.md Appendix A "pnet derived
 * views"):
 *   EthernetPacket::new  len >= 14, payload = [14..]
 *   Ipv4Packet::new      len >= 20 (no version check), payload =
 *                        [20+opt .. min(20+opt+plen, len)], packet_size = 20+opt+plen
 *   Ipv6Packet::new      len >= 40, payload = [40 .. min(40+pl, len)], packet_size = 40+pl
 *   ArpPacket::new       len >= 28, payload = [], packet_size = 28
 *   UdpPacket::new       len >= 8,  payload = [8..], packet_size = len
 *   TcpPacket::new       len >= 20, flags = byte 13
 *   VlanPacket::new      len >= 4,  payload = [4..]
 *   GrePacket/Icmpv6Packet::new len >= 4
 */
#define _POSIX_C_SOURCE 199309L
#include "fluere_oracle.h"

#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef struct {
    const uint8_t* p;
    uint32_t n;
} span;

static span sp_make(const uint8_t* p, uint32_t n) { span s = {p, n}; return s; }
static span sp_from(span s, uint32_t off) { return off >= s.n ? sp_make(s.p, 0) : sp_make(s.p + off, s.n - off); }
static uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }

static const uint8_t VXLAN_HEADER[8] = {0x08, 0x00, 0x00, 0x00, 0x00, 0x00, 0x64, 0x00};

static void ip4(or_ip* ip, const uint8_t* b) { memset(ip, 0, sizeof *ip); memcpy(ip->b, b, 4); }
static void ip6(or_ip* ip, const uint8_t* b) { memset(ip, 0, sizeof *ip); ip->v6 = 1; memcpy(ip->b, b, 16); }

/* ---- pnet views -------------------------------------------------------- */
static uint32_t v4_opt(span i) { uint32_t h = (uint32_t)(i.p[0] & 0x0F) * 4; return h > 20 ? h - 20 : 0; }
static uint32_t v4_plen(span i) { uint32_t h = (uint32_t)(i.p[0] & 0x0F) * 4, tl = be16(i.p + 2); return tl > h ? tl - h : 0; }
static span v4_payload(span i) {
    uint32_t start = 20 + v4_opt(i);
    if (i.n <= start) return sp_make(i.p, 0);
    uint32_t end = start + v4_plen(i);
    if (end > i.n) end = i.n;
    return sp_make(i.p + start, end - start);
}
static uint64_t v4_size(span i) { return 20ull + v4_opt(i) + v4_plen(i); }
static span v6_payload(span i) {
    if (i.n <= 40) return sp_make(i.p, 0);
    uint32_t end = 40 + be16(i.p + 4);
    if (end > i.n) end = i.n;
    return sp_make(i.p + 40, end - 40);
}

/* ---- raw fallback: src/net/parser/raw ---------------------------------- */
/* RawProtocolHeader (raw/mod.rs:9-37), the fields the reference's own tests
 * and the hot path read; payload as a slice [payload_off, +payload_len) of
 * the parsed bytes (Some/None in has_payload). */
typedef or_raw_hdr raw_hdr;

/* raw/mod.rs:40-71 RawProtocolHeader::new (Option fields None) */
static void raw_new(raw_hdr* h, uint16_t sp, uint16_t dp, uint8_t proto, uint32_t len) {
    memset(h, 0, sizeof *h);
    h->sport = sp; h->dport = dp; h->proto = proto; h->length = (uint16_t)len;
}
static void raw_payload(raw_hdr* h, span p, uint32_t off) {
    h->has_payload = 1;
    h->payload_off = off < p.n ? off : p.n;
    h->payload_len = p.n - h->payload_off;
}

/* protocols/icmp.rs:10-48 IcmpParser::parse_packet */
static int raw_icmp(span p, raw_hdr* h) {
    if (p.n < 4) return 0;
    raw_new(h, p.p[0], p.p[1], 1, p.n);
    if (p.n > 4) raw_payload(h, p, 4);
    h->has_flags = 1; h->flags = p.p[0];     /* with_flags(icmp_type) */
    h->has_version = 1; h->version = p.p[1]; /* with_version(icmp_code) */
    return 1;
}

/* protocols/openvpn.rs:155-220 (parse_control_packet :31-72, parse_data_packet :85-128) */
static int raw_openvpn(span p, raw_hdr* h) {
    if (p.n < 9) return 0;
    uint8_t t = p.p[0];
    if (!((t >= 1 && t <= 9) || t == 0x40 || t == 0x41)) return 0;
    raw_new(h, t, 0, 0x9B, p.n);
    raw_payload(h, p, 9);
    if (t == 6 || t == 9) {
        span ip = sp_from(p, 9);
        if (ip.n >= 16 && ((ip.p[0] >> 4) & 0x0F) == 4) {
            h->has_src = h->has_dst = 1;
            ip4(&h->src, ip.p + 4);
            ip4(&h->dst, ip.p + 8);
            h->sport = be16(ip.p + 12);
            h->dport = be16(ip.p + 14);
        }
    } else if (p.n >= 21 && (t == 0x40 || t == 0x41)) {
        h->has_src = h->has_dst = 1;
        ip4(&h->src, p.p + 9);
        ip4(&h->dst, p.p + 13);
        h->sport = be16(p.p + 17);
        h->dport = be16(p.p + 19);
    }
    return 1;
}

/* protocols/mod.rs:48-84 parse_protocol */
static int raw_parse_protocol(span p, uint8_t proto, raw_hdr* h) {
    if (proto == 1 && raw_icmp(p, h)) return 1;
    if (proto >= 170 && proto <= 172 && raw_openvpn(p, h)) return 1;
    return raw_openvpn(p, h);
}

static void raw_fill_outer(raw_hdr* h, const or_ip* s, const or_ip* d, uint16_t sp, uint16_t dp) {
    if (!h->has_src) { h->has_src = 1; h->src = *s; }
    if (!h->has_dst) { h->has_dst = 1; h->dst = *d; }
    if (h->sport == 0) h->sport = sp;
    if (h->dport == 0) h->dport = dp;
}

/* raw/mod.rs:152-328 RawProtocolHeader::from_raw_packet */
static int raw_from_raw_packet(span p, uint8_t hint, raw_hdr* h) {
    int outer = 0;
    or_ip os, od;
    uint16_t osp = 0, odp = 0;
    uint8_t oproto = 0;
    if (p.n >= 20 && (p.p[0] >> 4) == 4) {
        uint32_t hl = (uint32_t)(p.p[0] & 0x0F) * 4;
        if (hl >= 20 && hl <= p.n) {
            outer = 1;
            ip4(&os, p.p + 12);
            ip4(&od, p.p + 16);
            oproto = p.p[9];
            if (hl + 4 <= p.n) { osp = be16(p.p + hl); odp = be16(p.p + hl + 2); }
        }
    }
    if (raw_parse_protocol(p, hint, h)) {
        if (outer) raw_fill_outer(h, &os, &od, osp, odp);
        return 1;
    }
    if (outer) {
        raw_new(h, osp, odp, oproto, p.n);
        raw_payload(h, p, 0);
        h->has_src = h->has_dst = 1; h->src = os; h->dst = od;
        return 1;
    }
    if (p.n < 4) return 0;
    if (hint == 0x36) { raw_new(h, p.p[0], p.p[1], hint, p.n); raw_payload(h, p, 2); }           /* :271-283 */
    else if (hint == 0xb9) { raw_new(h, be16(p.p), be16(p.p + 2), hint, p.n); raw_payload(h, p, 4); } /* :249-270 */
    else { raw_new(h, be16(p.p), be16(p.p + 2), hint, p.n); raw_payload(h, p, 0); }             /* :284-304 */
    return 1;
}

/* ethertypes/vpn.rs:133-186 extract_ip_addresses */
static void raw_extract_ips(span q, raw_hdr* h) {
    if (q.n < 20) return;
    if ((q.p[0] >> 4) == 4) { h->has_src = h->has_dst = 1; ip4(&h->src, q.p + 12); ip4(&h->dst, q.p + 16); return; }
    if ((q.p[0] >> 4) == 6 && q.n >= 40) { h->has_src = h->has_dst = 1; ip6(&h->src, q.p + 8); ip6(&h->dst, q.p + 24); }
}

/* ethertypes/mod.rs:136-159 analyze_packet_structure */
void or_raw_analyze_structure(const uint8_t* p, uint32_t n, uint32_t* header_size, int* has_payload) {
    uint8_t b = n ? p[0] : 0;
    if (b >= 0xB8 && b <= 0xBF) { *header_size = 8; *has_payload = 1; }
    else if (b == 0x36 || b == 0x37) { *header_size = 6; *has_payload = 1; }
    else if (b == 0x6C) { *header_size = 4; *has_payload = 1; }
    else { *header_size = 4; *has_payload = n > 4; }
}

/* ethertypes/mod.rs:20-61 parse_ethertype.  Its 0x0806 arm (arp.rs:3-44) is
 * unreachable from parse_fluereflow, which handles ARP itself; it is kept so
 * the reference's parse_ethertype tests pin this function whole. */
static int raw_parse_ethertype(span p, uint16_t et, raw_hdr* h) {
    if (et == 0x0A08 || et == 0x4B65) { /* vpn.rs:15-56, :58-99 */
        if (p.n < 4) return 0;
        raw_new(h, et == 0x0A08 ? 2186 : 19301, be16(p.p + 2), et == 0x0A08 ? 21 : 22, p.n);
        raw_payload(h, p, 4);
        raw_extract_ips(sp_from(p, 4), h);
        return 1;
    }
    if (et == 0x0806) { /* arp.rs:3-44 */
        if (p.n < 28) return 0;
        raw_new(h, be16(p.p + 6), 0, 0x08, p.n);
        h->has_src = h->has_dst = 1;
        ip4(&h->src, p.p + 14); ip4(&h->dst, p.p + 24);
        h->has_ethertype = 1; h->ethertype = 0x0806;
        return 1;
    }
    if (et == 0x8847 || et == 0x8848) { /* mpls.rs:3-40 */
        if (p.n < 4) return 0;
        uint32_t label = ((uint32_t)p.p[0] << 12) | ((uint32_t)p.p[1] << 4) | ((uint32_t)p.p[2] >> 4);
        raw_new(h, (uint16_t)label, (p.p[2] >> 1) & 7, 137, p.n);
        uint32_t off = 4;  /* label stack walk (:18-26) */
        if (!(p.p[2] & 1))
            while (off + 4 <= p.n && !(p.p[off + 2] & 1)) off += 4;
        raw_payload(h, p, off);
        return 1;
    }
    if (et == 0x12B5) { /* vxlan.rs:8-48 */
        if (p.n < 8 || memcmp(p.p, VXLAN_HEADER, 8) != 0) return 0;
        uint32_t vni = ((uint32_t)p.p[4] << 16) | ((uint32_t)p.p[5] << 8) | p.p[6];
        raw_new(h, 4789, (uint16_t)vni, 0x12, p.n);
        raw_payload(h, p, 8);
        return 1;
    }
    if (et == 0x88B8) { /* wireguard.rs:12-80 */
        if (p.n < 4) return 0;
        uint8_t t = p.p[0];
        if (t == 1 && p.n != 148) return 0;
        if (t == 2 && p.n != 92) return 0;
        if (t == 3 && p.n != 64) return 0;
        if (t == 4 && p.n < 16) return 0;
        if (t < 1 || t > 4) return 0;
        raw_new(h, 0, 51820, t, p.n);
        raw_payload(h, p, 0);
        h->has_flags = 1; h->flags = t;
        h->has_version = 1; h->version = 1;
        h->has_ethertype = 1; h->ethertype = 0x88B8;
        return 1;
    }
    if ((et >= 0xB800 && et <= 0xBFFF) || (et >= 0x3600 && et <= 0x36FF)) { /* mod.rs:107-134 */
        if (p.n < 4) return 0;
        raw_new(h, be16(p.p), be16(p.p + 2), p.p[0], p.n);
        uint32_t hs; int hp;
        or_raw_analyze_structure(p.p, p.n, &hs, &hp);
        if (hp && p.n > hs) raw_payload(h, p, hs);
        return 1;
    }
    return 0;
}

/* raw/mod.rs:330-349 RawProtocolHeader::from_ethertype */
static int raw_from_ethertype(span p, uint16_t et, raw_hdr* h) {
    if (raw_parse_ethertype(p, et, h)) return 1;
    if (et == 0x0800 && p.n >= 20) return raw_from_raw_packet(p, p.p[9], h);
    return raw_from_raw_packet(p, (uint8_t)et, h);
}

/* exported for the pinning tests (tests/test_oracle.py) */
int or_raw_from_raw_packet(const uint8_t* p, uint32_t n, uint8_t hint, or_raw_hdr* h) {
    return raw_from_raw_packet(sp_make(p, n), hint, h);
}
int or_raw_from_ethertype(const uint8_t* p, uint32_t n, uint16_t et, or_raw_hdr* h) {
    return raw_from_ethertype(sp_make(p, n), et, h);
}
int or_raw_parse_ethertype(const uint8_t* p, uint32_t n, uint16_t et, or_raw_hdr* h) {
    return raw_parse_ethertype(sp_make(p, n), et, h);
}
int or_raw_parse_protocol(const uint8_t* p, uint32_t n, uint8_t proto, or_raw_hdr* h) {
    return raw_parse_protocol(sp_make(p, n), proto, h);
}
int or_raw_openvpn(const uint8_t* p, uint32_t n, or_raw_hdr* h) { return raw_openvpn(sp_make(p, n), h); }
int or_raw_icmp(const uint8_t* p, uint32_t n, or_raw_hdr* h) { return raw_icmp(sp_make(p, n), h); }

/* ---- ports / flags / tos ------------------------------------------------ */
/* src/net/parser/ports.rs:7-58 */
static int parse_ports(uint8_t proto, span x, uint16_t* sp, uint16_t* dp, int* raw_used) {
    switch (proto) {
    case 0: case 1: case 2: case 4: case 47: case 50: case 51: case 58:
        *sp = *dp = 0; return OR_OK;
    case 6:
        if (x.n < 20) return OR_ERR_INVALID;
        *sp = be16(x.p); *dp = be16(x.p + 2); return OR_OK;
    case 17:
        if (x.n < 8) return OR_ERR_INVALID;
        *sp = be16(x.p); *dp = be16(x.p + 2); return OR_OK;
    case 53:
        if (x.n < 8) { *sp = *dp = 53; return OR_OK; }
        *sp = be16(x.p); *dp = be16(x.p + 2); return OR_OK;
    default: {
        if (x.n >= 8) { *sp = be16(x.p); *dp = be16(x.p + 2); return OR_OK; } /* TCP then UDP view */
        raw_hdr h;
        if (raw_used) *raw_used = 1;
        if (raw_from_raw_packet(x, proto, &h)) { *sp = h.sport; *dp = h.dport; }
        else { *sp = *dp = 0; }
        return OR_OK;
    }
    }
}

/* src/net/parser/flags.rs:13-38 */
static void parse_flags(uint8_t proto, span x, uint8_t f[9]) {
    memset(f, 0, 9);
    if (proto == 6 && x.n >= 20) {
        uint8_t b = x.p[13];
        for (int i = 0; i < 8; i++) f[i] = (b >> i) & 1;
    }
}

/* src/net/parser/tos.rs:3-30 (Err -> caller uses 0) */
static uint8_t dscp_to_tos(uint8_t dscp) {
    switch (dscp) {
    case 0: case 8: case 10: case 12: case 14: case 16: case 18: case 20: case 22: case 24:
    case 26: case 28: case 30: case 32: case 34: case 36: case 38: case 40: case 46: case 48:
    case 56:
        return (uint8_t)(dscp * 4);
    default:
        return 0;
    }
}

/* ---- parse_keys: src/net/parser/keys.rs ---------------------------------- */
typedef struct {
    or_ip s, d;
    uint16_t sp, dp;
    uint8_t proto;
} l3key;

/* keys.rs:361-388 */
static int ipv4_keys(span i, l3key* k, int* raw_used) {
    ip4(&k->s, i.p + 12); ip4(&k->d, i.p + 16);
    k->proto = i.p[9];
    span pl = v4_payload(i);
    int e = parse_ports(k->proto, pl, &k->sp, &k->dp, raw_used);
    if (e) return e;
    if (k->proto == 47 && pl.n >= 4) { k->sp = be16(pl.p + 2); k->dp = 0; }
    return OR_OK;
}

/* keys.rs:390-415 */
static int ipv6_keys(span i, l3key* k, int* raw_used) {
    ip6(&k->s, i.p + 8); ip6(&k->d, i.p + 24);
    k->proto = i.p[6];
    span pl = v6_payload(i);
    int e = parse_ports(k->proto, pl, &k->sp, &k->dp, raw_used);
    if (e) return e;
    if (k->proto == 58 && pl.n >= 4) { k->sp = pl.p[0]; k->dp = pl.p[1]; }
    return OR_OK;
}

/* keys.rs:345-359 */
static int arp_keys(span a, l3key* k) {
    ip4(&k->s, a.p + 14); ip4(&k->d, a.p + 24);
    k->sp = k->dp = 0; k->proto = 4;
    return OR_OK;
}

/* keys.rs:417-435 */
static int vlan_keys(span v, l3key* k, int* raw_used) {
    span e = sp_from(v, 4);
    if (e.n < 14) return OR_ERR_INVALID;
    uint16_t et = be16(e.p + 12);
    span ip = sp_from(e, 14);
    if (et == 0x0800) { if (ip.n < 20) return OR_ERR_INVALID; return ipv4_keys(ip, k, raw_used); }
    if (et == 0x86DD) { if (ip.n < 40) return OR_ERR_INVALID; return ipv6_keys(ip, k, raw_used); }
    return OR_ERR_UNKNOWN_ETHER;
}

/* keys.rs:107-139 (is_udp) and :144-198 (UDP payload, VXLAN decap).
 * Returns the frame to key on, or an error. */
static int keys_frame(span d, span* frame) {
    uint16_t et = be16(d.p + 12);
    span p = sp_from(d, 14);
    span pl = sp_make(d.p, 0);
    int is_udp = 0;
    if (et == 0x86DD) { if (p.n < 40) return OR_ERR_EMPTY; pl = v6_payload(p); is_udp = pl.n >= 8; }
    else if (et == 0x0800) { if (p.n < 20) return OR_ERR_EMPTY; pl = v4_payload(p); is_udp = pl.n >= 8; }
    else if (et == 0x0806) { if (p.n < 28) return OR_ERR_EMPTY; is_udp = 0; /* ARP payload is empty */ }
    *frame = d;
    if (is_udp) {
        span u = sp_from(pl, 8);
        if (u.n == 0) return OR_ERR_EMPTY; /* keys.rs:182-184 */
        if (u.n >= 8 && memcmp(u.p, VXLAN_HEADER, 8) == 0) {
            span in = sp_from(u, 8);
            if (in.n < 14) return OR_ERR_EMPTY; /* keys.rs:192-193 */
            *frame = in;
        }
    }
    return OR_OK;
}

int or_parse_keys(const uint8_t* dp, uint32_t len, or_key* key, or_key* rev, int* raw_used) {
    int dummy = 0;
    if (!raw_used) raw_used = &dummy;
    *raw_used = 0;
    if (len == 0) return OR_ERR_EMPTY;          /* keys.rs:100-102 */
    if (len < 14) return OR_ERR_INVALID;        /* keys.rs:104 */
    span fr;
    int e = keys_frame(sp_make(dp, len), &fr);
    if (e) return e;
    uint16_t et2 = be16(fr.p + 12);
    span p2 = sp_from(fr, 14);
    l3key k;
    memset(&k, 0, sizeof k);
    switch (et2) { /* keys.rs:205-314 */
    case 0x86DD:
        if (p2.n < 40) return OR_ERR_EMPTY;
        e = ipv6_keys(p2, &k, raw_used); break;
    case 0x0800:
        if (p2.n < 20) return OR_ERR_EMPTY;
        e = ipv4_keys(p2, &k, raw_used); break;
    case 0x0806: case 0x8035:
        if (p2.n < 28) return OR_ERR_EMPTY;
        e = arp_keys(p2, &k); break;
    case 0x8100:
        if (p2.n < 4) return OR_ERR_EMPTY;
        e = vlan_keys(p2, &k, raw_used); break;
    default: { /* keys.rs:252-313: first Ok of the eager chain wins */
        e = OR_ERR_INVALID;
        if (p2.n >= 20) e = ipv4_keys(p2, &k, raw_used);
        if (e && p2.n >= 40) e = ipv6_keys(p2, &k, raw_used);
        if (e && p2.n >= 28) e = arp_keys(p2, &k);
        if (e && p2.n >= 4) e = vlan_keys(p2, &k, raw_used);
        if (e) {
            raw_hdr h;
            *raw_used = 1;
            if (raw_from_raw_packet(p2, (uint8_t)et2, &h)) {
                memset(&k, 0, sizeof k);
                if (h.has_src) k.s = h.src; else memset(&k.s, 0, sizeof k.s);
                if (h.has_dst) k.d = h.dst; else memset(&k.d, 0, sizeof k.d);
                k.sp = h.sport; k.dp = h.dport; k.proto = h.proto;
                e = OR_OK;
            } else {
                e = OR_ERR_UNKNOWN_ETHER;
            }
        }
    }
    }
    if (e) return e;
    /* keys.rs:323-340 */
    memset(key, 0, sizeof *key);
    key->src = k.s; key->dst = k.d; key->sport = k.sp; key->dport = k.dp; key->proto = k.proto;
    memcpy(key->smac, fr.p + 6, 6);
    memcpy(key->dmac, fr.p, 6);
    memset(rev, 0, sizeof *rev);
    rev->src = k.d; rev->dst = k.s; rev->sport = k.dp; rev->dport = k.sp; rev->proto = k.proto;
    memcpy(rev->smac, fr.p, 6);
    memcpy(rev->dmac, fr.p + 6, 6);
    return OR_OK;
}

/* ---- parse_fluereflow: src/net/parser/fluereflows.rs --------------------- */
static void rec_seed(or_record* r, uint64_t t, uint16_t sp, uint16_t dp, uint32_t pkt, uint8_t ttl,
                     uint8_t prot, uint8_t tos) {
    /* FluereRecord::new(src, dst, 0, 0, t, t, sp, dp, pkt, pkt, ttl, ttl, 0.., prot, tos) */
    r->d_pkts = 0; r->d_octets = 0; r->first = r->last = t;
    r->src_port = sp; r->dst_port = dp;
    r->min_pkt = r->max_pkt = pkt;
    r->min_ttl = r->max_ttl = ttl;
    r->in_pkts = r->out_pkts = 0; r->in_bytes = r->out_bytes = 0;
    memset(r->cnt, 0, sizeof r->cnt);
    r->prot = prot; r->tos = tos;
}

int or_parse_fluereflow(const uint8_t* dp, uint32_t len, uint64_t sec, uint64_t usec, uint64_t* doctets,
                        uint8_t flags[9], or_record* rec, int* raw_used) {
    int dummy = 0;
    if (!raw_used) raw_used = &dummy;
    *raw_used = 0;
    memset(rec, 0, sizeof *rec);
    memset(flags, 0, 9);
    if (len < 14) return OR_ERR_EMPTY; /* fluereflows.rs:32-40 */
    span d = sp_make(dp, len);
    uint16_t et = be16(d.p + 12);
    span p = sp_from(d, 14), pl = sp_make(d.p, 0);
    int is_udp = 0;
    if (et == 0x86DD) { if (p.n < 40) return OR_ERR_INVALID; pl = v6_payload(p); is_udp = pl.n >= 8; }
    else if (et == 0x0800) { if (p.n < 20) return OR_ERR_INVALID; pl = v4_payload(p); is_udp = pl.n >= 8; }
    span fr = d;
    if (is_udp) { /* fluereflows.rs:62-110; an empty payload is not an error here */
        span u = sp_from(pl, 8);
        if (u.n >= 8 && memcmp(u.p, VXLAN_HEADER, 8) == 0) {
            span in = sp_from(u, 8);
            if (in.n >= 14) fr = in; /* else: fall back to the outer frame */
        }
    }
    uint64_t t = sec * 1000000ull + usec; /* time.rs:5-7 */
    uint16_t et2 = be16(fr.p + 12);
    span p2 = sp_from(fr, 14);
    if (et2 == 0x0800) { /* ipv4_packet fluereflows.rs:249-336 */
        if (p2.n < 20) return OR_ERR_INVALID;
        uint8_t proto = p2.p[9];
        span l4 = v4_payload(p2);
        ip4(&rec->source, p2.p + 12); ip4(&rec->destination, p2.p + 16);
        if (proto == 17 && l4.n >= 8 && (be16(l4.p + 2) == 53 || be16(l4.p) == 53)) {
            *doctets = v4_size(p2);
            rec_seed(rec, t, be16(l4.p), be16(l4.p + 2), l4.n /* udp.packet_size() */, p2.p[8], 17, 0);
            return OR_OK;
        }
        uint16_t sp = 0, dpt = 0;
        if (parse_ports(proto, l4, &sp, &dpt, raw_used)) { sp = 0; dpt = 0; }
        parse_flags(proto, l4, flags);
        *doctets = v4_size(p2);
        rec_seed(rec, t, sp, dpt, be16(p2.p + 2), p2.p[8], proto, dscp_to_tos(p2.p[1] >> 2));
        return OR_OK;
    }
    if (et2 == 0x86DD) { /* ipv6_packet fluereflows.rs:338-388 */
        if (p2.n < 40) return OR_ERR_INVALID;
        uint8_t nh = p2.p[6];
        span l4 = v6_payload(p2);
        uint16_t sp = 0, dpt = 0;
        int e = parse_ports(nh, l4, &sp, &dpt, raw_used);
        if (e) return e;
        parse_flags(nh, l4, flags);
        uint16_t plf = be16(p2.p + 4);
        *doctets = 40ull + plf;
        uint8_t tc = (uint8_t)(((p2.p[0] & 0x0F) << 4) | (p2.p[1] >> 4));
        ip6(&rec->source, p2.p + 8); ip6(&rec->destination, p2.p + 24);
        rec_seed(rec, t, sp, dpt, plf, 0, nh, dscp_to_tos(tc >> 2));
        return OR_OK;
    }
    if (et2 == 0x0806) { /* arp_packet fluereflows.rs:201-247 */
        if (p2.n < 28) return OR_ERR_INVALID;
        ip4(&rec->source, p2.p + 14); ip4(&rec->destination, p2.p + 24);
        *doctets = 28;
        rec_seed(rec, t, 0, 0, 28, 0, 4, 0);
        return OR_OK;
    }
    /* fluereflows.rs:148-195: raw fallback over the WHOLE frame */
    raw_hdr h;
    *raw_used = 1;
    if (!raw_from_ethertype(fr, et2, &h)) return OR_ERR_UNKNOWN_ETHER;
    if (h.has_src) rec->source = h.src; else memset(&rec->source, 0, sizeof rec->source);
    if (h.has_dst) rec->destination = h.dst; else memset(&rec->destination, 0, sizeof rec->destination);
    *doctets = h.length;
    rec_seed(rec, t, h.sport, h.dport, h.length, 0 /* ttl None */, h.proto, 0);
    return OR_OK; /* flags: parse_flags(f, &[]) is all zero */
}

/* ---- pcap (libpcap offline semantics) ----------------- */
static uint32_t rd32(const uint8_t* p, int swap) {
    uint32_t v = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
    if (swap) v = (v >> 24) | ((v >> 8) & 0xFF00) | ((v << 8) & 0xFF0000) | (v << 24);
    return v;
}

/* pcapng (libpcap pcap-ng.c, read by pcap_open_offline at microsecond
 * precision; third-party code, restated -- SURVEY Appendix C style):
 * blocks in file order; a Section Header Block sets the byte order and
 * forgets the interfaces (a later section in the other byte order ends the
 * capture: "sections with different byte orders"); an Enhanced / obsolete
 * Packet Block's caplen above the snapshot length (interface 0's snaplen) is
 * cut to it; Interface Description Blocks give if_tsresol
 * (option 9: 10^-b, or 2^-(b & 0x7f) when the high bit is set; default 10^-6),
 * if_tsoffset (option 14, seconds) and the snaplen (0 or above 262144 ->
 * 262144); Enhanced / obsolete Packet Blocks carry (interface, 64-bit time in
 * the interface's units, caplen, len, data); Simple Packet Blocks carry no
 * time (0) and caplen = min(len, block room, snaplen of interface 0); other
 * blocks are skipped.  A truncated or malformed block, an unknown interface
 * or caplen > 262144 ends the capture (pcap_next_ex error).  Time: sec =
 * t / res + tsoffset, usec = (t % res) * 10^6 / res. */
typedef struct { uint64_t res; int64_t off; uint32_t snap; } ng_if;

static uint32_t rdx32(const uint8_t* p, int sw) { uint32_t v; memcpy(&v, p, 4); return sw ? __builtin_bswap32(v) : v; }
static uint16_t rdx16(const uint8_t* p, int sw) { uint16_t v; memcpy(&v, p, 2); return sw ? __builtin_bswap16(v) : v; }

static int64_t or_pcapng_index(const uint8_t* f, uint64_t n, or_pcap_rec** out) {
    uint64_t cap = 1024, cnt = 0, pos = 0;
    or_pcap_rec* r = (or_pcap_rec*)malloc(cap * sizeof *r);
    ng_if ifs[256];
    int nif = 0, sw = 0, have_shb = 0, first_sw = -1;
    const uint32_t max_snap = 262144;
    while (pos + 12 <= n) {
        uint32_t type = rdx32(f + pos, sw);
        if (type == 0x0A0D0D0Au) {
            uint32_t bom;
            memcpy(&bom, f + pos + 8, 4);
            if (bom == 0x1A2B3C4Du) sw = 0;
            else if (bom == 0x4D3C2B1Au) sw = 1;
            else break;
            if (pos + 16 > n || rdx16(f + pos + 12, sw) != 1) break; /* major version 1 */
            if (first_sw < 0) first_sw = sw;
            else if (first_sw != sw) break;
            have_shb = 1;
            nif = 0;
        } else if (!have_shb) {
            break;
        }
        uint32_t total = rdx32(f + pos + 4, sw);
        if (total < 12 || (total & 3) || pos + total > n) break;
        const uint8_t* b = f + pos + 8;
        uint32_t blen = total - 12;
        int stop = 0;
        if (type == 1) { /* IDB */
            if (blen < 8 || nif == 256) { stop = 1; }
            else {
                ng_if x;
                x.res = 1000000; x.off = 0;
                x.snap = rdx32(b + 4, sw);
                if (x.snap == 0 || x.snap > max_snap) x.snap = max_snap;
                uint32_t o = 8;
                while (o + 4 <= blen) {
                    uint16_t code = rdx16(b + o, sw), len = rdx16(b + o + 2, sw);
                    if (code == 0) break;
                    if (o + 4 + len > blen) { stop = 1; break; }
                    if (code == 9 && len >= 1) {
                        uint8_t v = b[o + 4];
                        unsigned __int128 res = 1;
                        int e = v & 0x7f, bin = (v & 0x80) != 0;
                        for (int k = 0; k < e && res <= (unsigned __int128)UINT64_MAX; k++) res *= bin ? 2 : 10;
                        if (res > (unsigned __int128)UINT64_MAX) { stop = 1; break; }
                        x.res = (uint64_t)res;
                    } else if (code == 14 && len >= 8) {
                        uint64_t v = (uint64_t)rdx32(b + o + 4, sw) | ((uint64_t)rdx32(b + o + 8, sw) << 32);
                        if (sw) v = ((uint64_t)rdx32(b + o + 4, sw) << 32) | rdx32(b + o + 8, sw);
                        x.off = (int64_t)v;
                    }
                    o += 4 + ((len + 3u) & ~3u);
                }
                if (!stop) ifs[nif++] = x;
            }
        } else if (type == 6 || type == 2 || type == 3) { /* EPB, OPB, SPB */
            uint32_t ifid = 0, caplen, dataoff;
            uint64_t t = 0;
            if (type == 3) {
                if (blen < 4 || nif == 0) { stop = 1; }
                else {
                    uint32_t len = rdx32(b, sw);
                    caplen = len < blen - 4 ? len : blen - 4;
                    if (caplen > ifs[0].snap) caplen = ifs[0].snap;
                    dataoff = 4;
                }
            } else {
                if (blen < 20) { stop = 1; }
                else {
                    ifid = type == 6 ? rdx32(b, sw) : rdx16(b, sw);
                    t = ((uint64_t)rdx32(b + 4, sw) << 32) | rdx32(b + 8, sw);
                    caplen = rdx32(b + 12, sw);
                    dataoff = 20;
                    if (ifid >= (uint32_t)nif || caplen > blen - 20) stop = 1;
                    else if (caplen > ifs[0].snap) caplen = ifs[0].snap;
                }
            }
            if (!stop && caplen > max_snap) stop = 1;
            if (!stop) {
                const ng_if* x = &ifs[ifid];
                if (cnt == cap) { cap *= 2; r = (or_pcap_rec*)realloc(r, cap * sizeof *r); }
                r[cnt].data_off = pos + 8 + dataoff;
                r[cnt].caplen = caplen;
                uint64_t sec = type == 3 ? 0 : t / x->res;
                uint64_t frac = type == 3 ? 0 : t % x->res;
                r[cnt].ts_sec = (uint32_t)(sec + (uint64_t)x->off);
                r[cnt].ts_usec = (uint32_t)(((unsigned __int128)frac * 1000000u) / x->res);
                cnt++;
            }
        }
        if (stop) break;
        pos += total;
    }
    *out = r;
    return (int64_t)cnt;
}

int64_t or_pcap_index(const uint8_t* f, uint64_t n, or_pcap_rec** out) {
    *out = NULL;
    if (n >= 4 && rd32(f, 0) == 0x0A0D0D0Au) return or_pcapng_index(f, n, out);
    if (n < 24) return -1;
    uint32_t magic = rd32(f, 0);
    int swap = 0, nsec = 0;
    if (magic == 0xa1b2c3d4u) { }
    else if (magic == 0xd4c3b2a1u) swap = 1;
    else if (magic == 0xa1b23c4du) nsec = 1;
    else if (magic == 0x4d3cb2a1u) { swap = 1; nsec = 1; }
    else return -1;
    uint32_t snap = rd32(f + 16, swap);
    const uint32_t max_snap = 262144; /* libpcap MAXIMUM_SNAPLEN for DLT_EN10MB */
    if (snap == 0 || snap > max_snap) snap = max_snap;
    uint64_t cap = 1024, cnt = 0, off = 24;
    or_pcap_rec* r = (or_pcap_rec*)malloc(cap * sizeof *r);
    while (off + 16 <= n) {
        uint32_t incl = rd32(f + off + 8, swap);
        if (incl > max_snap) break;                /* "invalid packet capture length" */
        if (off + 16 + (uint64_t)incl > n) break;  /* truncated dump file */
        if (cnt == cap) { cap *= 2; r = (or_pcap_rec*)realloc(r, cap * sizeof *r); }
        r[cnt].data_off = off + 16;
        r[cnt].caplen = incl > snap ? snap : incl;
        r[cnt].ts_sec = rd32(f + off, swap);
        uint32_t frac = rd32(f + off + 4, swap);
        r[cnt].ts_usec = nsec ? frac / 1000 : frac;
        cnt++;
        off += 16 + (uint64_t)incl;
    }
    *out = r;
    return (int64_t)cnt;
}

static void key_to_meta(const or_key* k, or_pkt_meta* m) {
    m->key_v6 = k->src.v6;
    m->key_proto = k->proto;
    m->key_sport = k->sport; m->key_dport = k->dport;
    memcpy(m->key_src, k->src.b, 16); memcpy(m->key_dst, k->dst.b, 16);
    memcpy(m->key_smac, k->smac, 6); memcpy(m->key_dmac, k->dmac, 6);
}

int or_parse_batch(const uint8_t* file, uint64_t nbytes, or_pkt_meta* out, uint64_t cap, uint64_t* n_out) {
    or_pcap_rec* recs;
    int64_t n = or_pcap_index(file, nbytes, &recs);
    if (n < 0) return -1;
    if ((uint64_t)n > cap) n = (int64_t)cap;
    for (int64_t i = 0; i < n; i++) {
        or_pkt_meta* m = &out[i];
        memset(m, 0, sizeof *m);
        const uint8_t* d = file + recs[i].data_off;
        uint32_t L = recs[i].caplen;
        or_key k, rv;
        int raw_k = 0, raw_f = 0;
        m->k_status = (uint8_t)or_parse_keys(d, L, &k, &rv, &raw_k);
        if (m->k_status == OR_OK) key_to_meta(&k, m);
        uint64_t doct = 0;
        uint8_t fl[9];
        or_record rec;
        m->f_status = (uint8_t)or_parse_fluereflow(d, L, recs[i].ts_sec, recs[i].ts_usec, &doct, fl, &rec, &raw_f);
        if (m->f_status == OR_OK) {
            m->rec_v6 = rec.source.v6;
            m->rec_prot = rec.prot; m->rec_tos = rec.tos; m->rec_ttl = rec.min_ttl;
            memcpy(m->rec_src, rec.source.b, 16); memcpy(m->rec_dst, rec.destination.b, 16);
            m->rec_sport = rec.src_port; m->rec_dport = rec.dst_port;
            m->rec_pkt = rec.min_pkt;
            m->doctets = doct;
            m->time = rec.first;
            for (int b = 0; b < 9; b++) m->flags |= (uint16_t)(fl[b] << b);
        }
        m->raw_used = (uint8_t)((raw_k || raw_f) ? 1 : 0);
    }
    free(recs);
    *n_out = (uint64_t)n;
    return 0;
}

/* ---- offline state machine: src/net/offline_fluereflows.rs:60-184 -------- */
/* Key equality is over every field of Key (key.rs:5-14, derive(Eq, Hash)). */
typedef struct { uint8_t b[52]; } kbuf;
static void key_buf(const or_key* k, kbuf* o) {
    uint8_t* b = o->b;
    memset(o, 0, sizeof *o);
    b[0] = k->src.v6; memcpy(b + 1, k->src.b, 16); b[17] = (uint8_t)(k->sport >> 8); b[18] = (uint8_t)k->sport;
    b[19] = k->dst.v6; memcpy(b + 20, k->dst.b, 16); b[36] = (uint8_t)(k->dport >> 8); b[37] = (uint8_t)k->dport;
    b[38] = k->proto; memcpy(b + 39, k->smac, 6); memcpy(b + 45, k->dmac, 6);
}
static uint64_t kb_hash(const kbuf* k) {
    uint64_t h = 1469598103934665603ull;
    for (int i = 0; i < 52; i++) { h ^= k->b[i]; h *= 1099511628211ull; }
    return h ^ (h >> 29);
}

typedef struct {
    kbuf key;
    uint64_t seq;
    or_record rec;
    uint8_t used;
} slot;

typedef struct {
    slot* s;
    uint64_t cap, n;
} fmap;

static void fm_init(fmap* m, uint64_t cap) { m->cap = cap; m->n = 0; m->s = (slot*)calloc(cap, sizeof(slot)); }
static slot* fm_find(fmap* m, const kbuf* k) {
    uint64_t i = kb_hash(k) & (m->cap - 1);
    while (m->s[i].used) {
        if (memcmp(m->s[i].key.b, k->b, 52) == 0) return &m->s[i];
        i = (i + 1) & (m->cap - 1);
    }
    return NULL;
}
static slot* fm_insert(fmap* m, const kbuf* k);
static void fm_grow(fmap* m) {
    fmap g;
    fm_init(&g, m->cap * 2);
    for (uint64_t i = 0; i < m->cap; i++)
        if (m->s[i].used) { slot* t = fm_insert(&g, &m->s[i].key); t->seq = m->s[i].seq; t->rec = m->s[i].rec; }
    free(m->s);
    *m = g;
}
static slot* fm_insert(fmap* m, const kbuf* k) {
    if ((m->n + 1) * 2 > m->cap) fm_grow(m);
    uint64_t i = kb_hash(k) & (m->cap - 1);
    while (m->s[i].used) i = (i + 1) & (m->cap - 1);
    m->s[i].used = 1; m->s[i].key = *k; m->n++;
    return &m->s[i];
}
/* linear-probing delete with backward shift */
static void fm_erase(fmap* m, slot* s) {
    uint64_t i = (uint64_t)(s - m->s), j = i;
    m->s[i].used = 0;
    m->n--;
    for (;;) {
        j = (j + 1) & (m->cap - 1);
        if (!m->s[j].used) break;
        uint64_t h = kb_hash(&m->s[j].key) & (m->cap - 1);
        int move = (i <= j) ? (h <= i || h > j) : (h <= i && h > j);
        if (move) { m->s[i] = m->s[j]; m->s[j].used = 0; i = j; }
    }
}

/* BTreeMap<u64, Vec<Key>> swept in (exp asc, push order) == min-heap on (exp, seq) */
typedef struct { uint64_t exp, seq; kbuf key; } hent;
typedef struct { hent* a; uint64_t n, cap; } heap;
static int h_less(const hent* x, const hent* y) { return x->exp < y->exp || (x->exp == y->exp && x->seq < y->seq); }
static void h_push(heap* h, const hent* e) {
    if (h->n == h->cap) { h->cap = h->cap ? h->cap * 2 : 1024; h->a = (hent*)realloc(h->a, h->cap * sizeof(hent)); }
    uint64_t i = h->n++;
    h->a[i] = *e;
    while (i) { uint64_t p = (i - 1) / 2; if (!h_less(&h->a[i], &h->a[p])) break; hent t = h->a[i]; h->a[i] = h->a[p]; h->a[p] = t; i = p; }
}
static void h_pop(heap* h) {
    h->a[0] = h->a[--h->n];
    uint64_t i = 0;
    for (;;) {
        uint64_t l = 2 * i + 1, r = l + 1, m = i;
        if (l < h->n && h_less(&h->a[l], &h->a[m])) m = l;
        if (r < h->n && h_less(&h->a[r], &h->a[m])) m = r;
        if (m == i) break;
        hent t = h->a[i]; h->a[i] = h->a[m]; h->a[m] = t; i = m;
    }
}

static void push_rec(or_result* r, const or_record* x) {
    if (r->n == r->cap) { r->cap = r->cap ? r->cap * 2 : 1024; r->recs = (or_record*)realloc(r->recs, r->cap * sizeof(or_record)); }
    r->recs[r->n++] = *x;
}

static int cmp_seq(const void* a, const void* b) {
    uint64_t x = (*(const slot* const*)a)->seq, y = (*(const slot* const*)b)->seq;
    return x < y ? -1 : x > y;
}

int or_offline_buffer(const uint8_t* file, uint64_t nbytes, uint64_t timeout_ms, int use_mac, or_result* out) {
    memset(out, 0, sizeof *out);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    or_pcap_rec* recs;
    int64_t n = or_pcap_index(file, nbytes, &recs);
    if (n < 0) return -1;
    fmap A;
    fm_init(&A, 1024);
    heap E = {0};
    uint64_t seq = 0, create_seq = 0;
    for (int64_t i = 0; i < n; i++) { /* offline_fluereflows.rs:68 */
        const uint8_t* d = file + recs[i].data_off;
        uint32_t L = recs[i].caplen;
        or_key key, rev;
        int raw_k = 0, raw_f = 0;
        if (or_parse_keys(d, L, &key, &rev, &raw_k)) continue;                  /* :71-74 */
        if (!use_mac) {                                                          /* :76-79 */
            memset(key.smac, 0, 6); memset(key.dmac, 0, 6);
            memset(rev.smac, 0, 6); memset(rev.dmac, 0, 6);
        }
        uint64_t doctets;
        uint8_t fl[9];
        or_record fd;
        if (or_parse_fluereflow(d, L, recs[i].ts_sec, recs[i].ts_usec, &doctets, fl, &fd, &raw_f)) continue; /* :81-87 */
        uint64_t t = (uint64_t)recs[i].ts_sec * 1000000ull + recs[i].ts_usec;   /* :90-93 */
        kbuf kb, rb;
        key_buf(&key, &kb);
        key_buf(&rev, &rb);
        int is_rev;
        slot* fl_s = fm_find(&A, &kb);                                           /* :97-130 */
        if (fl_s) is_rev = 0;
        else if ((fl_s = fm_find(&A, &rb))) is_rev = 1;
        else {
            if (fd.prot == 6 && fl[1] == 0) continue;                            /* :101-113 */
            hent e;
            e.exp = t + timeout_ms * 1000ull;
            e.seq = seq++;
            e.key = kb;
            h_push(&E, &e);
            fl_s = fm_insert(&A, &kb);
            fl_s->seq = create_seq++;
            fl_s->rec = fd;
            is_rev = 0;
        }
        out->valid++;
        if (raw_k || raw_f) out->raw_used++;
        /* update_flow src/net/flows.rs:11-42 */
        or_record* f = &fl_s->rec;
        uint32_t pkt = fd.min_pkt;
        uint8_t ttl = fd.min_ttl;
        f->d_pkts += 1;
        f->d_octets += doctets;
        if (pkt > f->max_pkt) f->max_pkt = pkt;
        if (pkt < f->min_pkt) f->min_pkt = pkt;
        if (ttl > f->max_ttl) f->max_ttl = ttl;
        if (ttl < f->min_ttl) f->min_ttl = ttl;
        for (int b = 0; b < 9; b++) f->cnt[b] += fl[b];
        f->last = t;
        if (is_rev) { f->in_pkts += 1; f->in_bytes += doctets; }
        else { f->out_pkts += 1; f->out_bytes += doctets; }
        if (fl[0] == 1 || fl[2] == 1) {                                          /* :152-157 */
            push_rec(out, f);
            fm_erase(&A, fl_s);
        }
        while (E.n && E.a[0].exp <= t) {                                         /* :161-175 */
            slot* s = fm_find(&A, &E.a[0].key);
            if (s) { push_rec(out, &s->rec); fm_erase(&A, s); }
            h_pop(&E);
        }
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    out->loop_seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    out->packets = (uint64_t)n;
    out->n_ended = out->n;
    /* :182-184 active flows (HashMap order in the reference; creation order here) */
    slot** act = (slot**)malloc((A.n + 1) * sizeof(slot*));
    uint64_t k = 0;
    for (uint64_t i = 0; i < A.cap; i++) if (A.s[i].used) act[k++] = &A.s[i];
    qsort(act, k, sizeof(slot*), cmp_seq);
    for (uint64_t i = 0; i < k; i++) push_rec(out, &act[i]->rec);
    free(act);
    free(A.s);
    free(E.a);
    free(recs);
    return 0;
}

void or_result_free(or_result* r) { free(r->recs); memset(r, 0, sizeof *r); }

/* ---- live mode: src/net/live_fluereflow.rs:196-376 ---------------------- */
static void live_push(or_live_result* o, const or_record* r, uint8_t kind) {
    if (o->n == o->cap) {
        o->cap = o->cap ? 2 * o->cap : 1024;
        o->recs = (or_record*)realloc(o->recs, o->cap * sizeof *o->recs);
        o->interval = (uint32_t*)realloc(o->interval, o->cap * sizeof *o->interval);
        o->kind = (uint8_t*)realloc(o->kind, o->cap * sizeof *o->kind);
    }
    o->recs[o->n] = *r;
    o->interval[o->n] = UINT32_MAX;  /* set at the export that writes it */
    o->kind[o->n] = kind;
    o->n++;
}

/* expire the active flows whose last update is older than time - timeout
 * (u64 arithmetic wraps as in the release build); in creation order, the
 * reference's HashMap order is unspecified */
static int cmp_slot_seq(const void* a, const void* b) {
    const slot* x = (const slot*)a;
    const slot* y = (const slot*)b;
    return x->seq < y->seq ? -1 : x->seq > y->seq;
}
static void live_scan(fmap* A, uint64_t time, uint64_t timeout_ms, uint8_t kind, or_live_result* o) {
    const uint64_t lim = time - timeout_ms * 1000ull;
    slot* ex = (slot*)malloc((A->n + 1) * sizeof(slot));  /* copies: erasing shifts slots */
    uint64_t k = 0;
    for (uint64_t i = 0; i < A->cap; i++) if (A->s[i].used && A->s[i].rec.last < lim) ex[k++] = A->s[i];
    qsort(ex, k, sizeof(slot), cmp_slot_seq);
    for (uint64_t i = 0; i < k; i++) {
        live_push(o, &ex[i].rec, kind);
        fm_erase(A, fm_find(A, &ex[i].key));
    }
    free(ex);
}

int or_live_buffer(const uint8_t* file, uint64_t nbytes, const uint64_t* batch_end, const uint8_t* batch_export,
                   uint64_t n_batches, uint64_t timeout_ms, int use_mac, int duration_end, or_live_result* out) {
    memset(out, 0, sizeof *out);
    or_pcap_rec* recs;
    int64_t n = or_pcap_index(file, nbytes, &recs);
    if (n < 0) return -1;
    fmap A;
    fm_init(&A, 1024);
    uint64_t create_seq = 0, exported = 0;
    int64_t i = 0;
    int export_due = 0;  /* the interval elapsed: the export runs after the next processed packet */
    for (uint64_t b = 0; b < n_batches; b++) {
        int have = 0;      /* a processed packet in this batch (the checks run after one) */
        uint64_t time = 0; /* its timestamp: the `time` of the checks (:306-373) */
        for (; i < n && (uint64_t)i < batch_end[b]; i++) { /* :196-303 */
            const uint8_t* d = file + recs[i].data_off;
            uint32_t L = recs[i].caplen;
            or_key key, rev;
            int raw_k = 0, raw_f = 0;
            if (or_parse_keys(d, L, &key, &rev, &raw_k)) continue;              /* :204-207 */
            if (!use_mac) {                                                      /* :208-211 */
                memset(key.smac, 0, 6); memset(key.dmac, 0, 6);
                memset(rev.smac, 0, 6); memset(rev.dmac, 0, 6);
            }
            uint64_t doctets;
            uint8_t fl[9];
            or_record fd;
            if (or_parse_fluereflow(d, L, recs[i].ts_sec, recs[i].ts_usec, &doctets, fl, &fd, &raw_f)) continue; /* :213-219 */
            kbuf kb, rb;
            key_buf(&key, &kb);
            key_buf(&rev, &rb);
            int is_rev;
            slot* fl_s = fm_find(&A, &kb);                                       /* :224-269 */
            if (fl_s) is_rev = 0;
            else if ((fl_s = fm_find(&A, &rb))) is_rev = 1;
            else {
                if (fd.prot == 6 && fl[1] == 0) continue;                        /* SYN gate */
                fl_s = fm_insert(&A, &kb);
                fl_s->seq = create_seq++;
                fl_s->rec = fd;
                is_rev = 0;
            }
            const uint64_t t = (uint64_t)recs[i].ts_sec * 1000000ull + recs[i].ts_usec; /* :271-274 */
            or_record* f = &fl_s->rec;                                           /* update_flow :288 */
            uint32_t pkt = fd.min_pkt;
            uint8_t ttl = fd.min_ttl;
            f->d_pkts += 1;
            f->d_octets += doctets;
            if (pkt > f->max_pkt) f->max_pkt = pkt;
            if (pkt < f->min_pkt) f->min_pkt = pkt;
            if (ttl > f->max_ttl) f->max_ttl = ttl;
            if (ttl < f->min_ttl) f->min_ttl = ttl;
            for (int c = 0; c < 9; c++) f->cnt[c] += fl[c];
            f->last = t;
            if (is_rev) { f->in_pkts += 1; f->in_bytes += doctets; }
            else { f->out_pkts += 1; f->out_bytes += doctets; }
            if (fl[0] == 1 || fl[2] == 1) {                                      /* :296-302 plugin + records */
                live_push(out, f, 0);
                fm_erase(&A, fl_s);
            }
            have = 1;
            time = t;
        }
        if (batch_export[b]) export_due = 1;
        if (!have) continue;
        if (export_due) {                                                        /* :306-358 interval export */
            export_due = 0;
            if (timeout_ms > 0) live_scan(&A, time, timeout_ms, 1, out);
            for (uint64_t k = 0; k < out->n; k++) if (out->interval[k] == UINT32_MAX) out->interval[k] = (uint32_t)exported;
            exported++;
        }
        if (b + 1 == n_batches && duration_end) live_scan(&A, time, timeout_ms, 2, out); /* :361-373 */
    }
    /* :379-392 every flow still active, then the last export */
    slot** act = (slot**)malloc((A.n + 1) * sizeof(slot*));
    uint64_t k = 0;
    for (uint64_t j = 0; j < A.cap; j++) if (A.s[j].used) act[k++] = &A.s[j];
    qsort(act, k, sizeof(slot*), cmp_seq);
    for (uint64_t j = 0; j < k; j++) live_push(out, &act[j]->rec, 3);
    free(act);
    for (uint64_t j = 0; j < out->n; j++) if (out->interval[j] == UINT32_MAX) out->interval[j] = (uint32_t)exported;
    out->n_exports = exported + 1;
    out->packets = (uint64_t)n;
    free(A.s);
    free(recs);
    return 0;
}

uint64_t or_record_size(void) { return sizeof(or_record); }

void or_live_free(or_live_result* r) {
    free(r->recs);
    free(r->interval);
    free(r->kind);
    memset(r, 0, sizeof *r);
}

/* ---- CSV: src/utils/fluere_csv_exporter.rs:5-81 (csv 1.3, '\n' terminator) */
static const char* CSV_HEADER =
    "source,destination,src_port,dst_port,prot,d_pkts,d_octets,in_pkts,out_pkts,in_bytes,out_bytes,"
    "first,last,min_pkt,max_pkt,min_ttl,max_ttl,fin_cnt,syn_cnt,rst_cnt,psh_cnt,ack_cnt,urg_cnt,"
    "ece_cnt,cwr_cnt,ns_cnt,tos\n";

typedef struct { char* b; uint64_t n, cap; } sbuf;
static void sb_put(sbuf* s, const char* x, uint64_t len) {
    if (s->b && s->n + len <= s->cap) memcpy(s->b + s->n, x, len);
    s->n += len;
}
static void sb_u64(sbuf* s, uint64_t v) {
    char t[24];
    int i = 24;
    do { t[--i] = (char)('0' + v % 10); v /= 10; } while (v);
    sb_put(s, t + i, (uint64_t)(24 - i));
}
static void sb_hex(sbuf* s, unsigned v) {
    char t[8];
    int i = 8;
    do { t[--i] = "0123456789abcdef"[v & 15]; v >>= 4; } while (v);
    sb_put(s, t + i, (uint64_t)(8 - i));
}
/* Rust std Ipv4Addr/Ipv6Addr Display */
static void sb_ip(sbuf* s, const or_ip* ip) {
    if (!ip->v6) {
        for (int i = 0; i < 4; i++) { if (i) sb_put(s, ".", 1); sb_u64(s, ip->b[i]); }
        return;
    }
    uint16_t seg[8];
    for (int i = 0; i < 8; i++) seg[i] = (uint16_t)((ip->b[2 * i] << 8) | ip->b[2 * i + 1]);
    int mapped = 1;
    for (int i = 0; i < 5; i++) if (seg[i]) mapped = 0;
    if (mapped && seg[5] == 0xFFFF) { /* to_ipv4_mapped */
        sb_put(s, "::ffff:", 7);
        for (int i = 12; i < 16; i++) { if (i > 12) sb_put(s, ".", 1); sb_u64(s, ip->b[i]); }
        return;
    }
    int best_s = 0, best_l = 0, cur_s = 0, cur_l = 0;
    for (int i = 0; i < 8; i++) {
        if (seg[i] == 0) {
            if (cur_l == 0) cur_s = i;
            cur_l++;
            if (cur_l > best_l) { best_l = cur_l; best_s = cur_s; }
        } else cur_l = 0;
    }
    if (best_l > 1) {
        for (int i = 0; i < best_s; i++) { if (i) sb_put(s, ":", 1); sb_hex(s, seg[i]); }
        sb_put(s, "::", 2);
        for (int i = best_s + best_l; i < 8; i++) { if (i > best_s + best_l) sb_put(s, ":", 1); sb_hex(s, seg[i]); }
    } else {
        for (int i = 0; i < 8; i++) { if (i) sb_put(s, ":", 1); sb_hex(s, seg[i]); }
    }
}

uint64_t or_format_csv(const or_record* recs, uint64_t n, char* buf, uint64_t cap) {
    sbuf s = {buf, 0, cap};
    sb_put(&s, CSV_HEADER, strlen(CSV_HEADER));
    for (uint64_t i = 0; i < n; i++) {
        const or_record* r = &recs[i];
        uint64_t v[25] = {r->src_port, r->dst_port, r->prot, r->d_pkts, r->d_octets, r->in_pkts, r->out_pkts,
                          r->in_bytes, r->out_bytes, r->first, r->last, r->min_pkt, r->max_pkt, r->min_ttl,
                          r->max_ttl, r->cnt[0], r->cnt[1], r->cnt[2], r->cnt[3], r->cnt[4], r->cnt[5],
                          r->cnt[6], r->cnt[7], r->cnt[8], r->tos};
        sb_ip(&s, &r->source);
        sb_put(&s, ",", 1);
        sb_ip(&s, &r->destination);
        for (int j = 0; j < 25; j++) { sb_put(&s, ",", 1); sb_u64(&s, v[j]); }
        sb_put(&s, "\n", 1);
    }
    return s.n;
}
