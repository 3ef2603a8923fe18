/*
 * fluere_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference CPU path for `fluere offline`
 * (SkuldNorniern/fluere @ /root/reference, fluere 0.7.1-dev).  It is the
 * parity checker for the MI355X path and the CPU baseline ("port") in
 * bench.py.  Nothing in fluere_amd/ links or calls it; only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg do.
 *
 * Parity pinning: the reference is Rust and cannot be built here (no
 * cargo/rustc, no libpcap).  This restatement is pinned by
 * the reference's own byte fixtures (src/net/parser/ipv4.rs:74-106,
 * udp.rs:49-89), by the reference's unit tests of the raw fallback the hot
 * path reaches (raw/mod.rs:353-673, raw/ethertypes/mod.rs:162-346,
 * raw/protocols/openvpn.rs:226-334, raw/protocols/icmp.rs:51-74; transcribed
 * in tests/test_oracle.py) and the known-answer rows derived from the reference
 * source.  Third-party behaviour (pnet 0.35,
 * libpcap via pcap 2.3, csv 1.3, Rust std Display) is restated from
 * their published semantics; see SURVEY.md Appendix C.
 */
#ifndef FLUERE_ORACLE_H
#define FLUERE_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* NetError variants the hot path can produce (src/net/mod.rs:28-36). */
enum {
    OR_OK = 0,
    OR_ERR_EMPTY = 1,        /* NetError::EmptyPacket */
    OR_ERR_INVALID = 2,      /* NetError::InvalidPacket */
    OR_ERR_UNKNOWN_ETHER = 3 /* NetError::UnknownEtherType */
};

/* std::net::IpAddr: v6 = 0 -> V4 in b[0..4] (rest zero), v6 = 1 -> V6. */
typedef struct {
    uint8_t v6;
    uint8_t b[16];
} or_ip;

/* src/net/types/key.rs:5-14 */
typedef struct {
    or_ip src, dst;
    uint16_t sport, dport;
    uint8_t proto;
    uint8_t smac[6], dmac[6];
} or_key;

/* fluereflow/src/types/fluereflow.rs:31-60 (cnt = fin..ns in flags order) */
typedef struct {
    or_ip source, destination;
    uint32_t d_pkts;
    uint64_t d_octets;
    uint64_t first, last;
    uint16_t src_port, dst_port;
    uint32_t min_pkt, max_pkt;
    uint8_t min_ttl, max_ttl;
    uint32_t in_pkts, out_pkts;
    uint64_t in_bytes, out_bytes;
    uint32_t cnt[9];
    uint8_t prot, tos;
} or_record;

/* Per-packet debug view shared (by layout only) with the product's
 * fluere_pkt_meta in include/fluere_gpu.h; 128 bytes. */
typedef struct {
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
    uint16_t flags; /* bit i = flags[i] of parse_flags, i = fin..ns */
    uint8_t raw_used; /* 1 if the raw fallback (src/net/parser/raw) ran */
    uint8_t pad[13];
} or_pkt_meta;

/* parse_keys (src/net/parser/keys.rs:98-343).  Returns OR_OK or an error.
 * *raw_used is set when the raw fallback decided the result. */
int or_parse_keys(const uint8_t* d, uint32_t len, or_key* key, or_key* rev, int* raw_used);

/* parse_fluereflow (src/net/parser/fluereflows.rs:30-199). */
int or_parse_fluereflow(const uint8_t* d, uint32_t len, uint64_t sec, uint64_t usec,
                        uint64_t* doctets, uint8_t flags[9], or_record* rec, int* raw_used);

/* RawProtocolHeader (src/net/parser/raw/mod.rs:9-37): the fields the
 * reference's own unit tests and the hot path read.  Option<T> fields carry
 * a has_ flag; payload is the slice [payload_off, payload_off + payload_len)
 * of the parsed bytes. */
typedef struct {
    uint8_t has_src, has_dst;
    or_ip src, dst;
    uint16_t sport, dport;
    uint8_t proto;
    uint16_t length;
    uint8_t has_flags, flags, has_version, version;
    uint8_t has_ethertype;
    uint16_t ethertype;
    uint8_t has_payload;
    uint32_t payload_off, payload_len;
} or_raw_hdr;

/* The raw fallback's entry points; 1 = Some(header), 0 = None.
 *   or_raw_from_raw_packet   raw/mod.rs:152-328
 *   or_raw_from_ethertype    raw/mod.rs:330-349
 *   or_raw_parse_ethertype   raw/ethertypes/mod.rs:20-61
 *   or_raw_parse_protocol    raw/protocols/mod.rs:48-84
 *   or_raw_openvpn           raw/protocols/openvpn.rs:155-220
 *   or_raw_icmp              raw/protocols/icmp.rs:10-48
 *   or_raw_analyze_structure raw/ethertypes/mod.rs:136-159 */
int or_raw_from_raw_packet(const uint8_t* p, uint32_t n, uint8_t hint, or_raw_hdr* h);
int or_raw_from_ethertype(const uint8_t* p, uint32_t n, uint16_t et, or_raw_hdr* h);
int or_raw_parse_ethertype(const uint8_t* p, uint32_t n, uint16_t et, or_raw_hdr* h);
int or_raw_parse_protocol(const uint8_t* p, uint32_t n, uint8_t proto, or_raw_hdr* h);
int or_raw_openvpn(const uint8_t* p, uint32_t n, or_raw_hdr* h);
int or_raw_icmp(const uint8_t* p, uint32_t n, or_raw_hdr* h);
void or_raw_analyze_structure(const uint8_t* p, uint32_t n, uint32_t* header_size, int* has_payload);

/* Classic pcap record index (libpcap offline semantics). */
typedef struct {
    uint64_t data_off;  /* offset of packet data in the file buffer */
    uint32_t caplen;    /* bytes given to the parser */
    uint32_t ts_sec;
    uint32_t ts_usec;   /* already scaled to microseconds */
} or_pcap_rec;

/* Walks the file buffer like pcap_next_ex until the first error/EOF.
 * Returns number of records, or -1 if the global header is unusable. */
int64_t or_pcap_index(const uint8_t* file, uint64_t nbytes, or_pcap_rec** out);

/* Per-packet parse of every record (the library seam, batch form). */
int or_parse_batch(const uint8_t* file, uint64_t nbytes, or_pkt_meta* out, uint64_t cap,
                   uint64_t* n_out);

typedef struct {
    or_record* recs;
    uint64_t n;        /* total records */
    uint64_t n_ended;  /* recs[0..n_ended) = ended prefix, in reference order */
    uint64_t packets;  /* records read from the pcap */
    uint64_t valid;    /* packets that passed parse_keys and parse_fluereflow */
    uint64_t raw_used; /* packets whose result came through the raw fallback */
    double loop_seconds; /* the reference's "Converted in" window */
    uint64_t cap;        /* internal: allocated records */
} or_result;

/* fluereflow_fileparse state machine (src/net/offline_fluereflows.rs:60-184)
 * over an in-memory pcap.  Active flows are appended in creation order (the
 * reference uses HashMap order; the comparator treats that suffix as a set). */
int or_offline_buffer(const uint8_t* file, uint64_t nbytes, uint64_t timeout_ms, int use_mac,
                      or_result* out);
void or_result_free(or_result* r);

/* live mode (src/net/live_fluereflow.rs:196-376) over a capture cut into
 * batches: packets [batch_end[b-1], batch_end[b]).  The checks the reference
 * runs after a processed packet run once per batch, after its last processed
 * packet (with that packet's time): the interval export when batch_export[b]
 * (idle-timeout scan flow.last < time - timeout, :306-358), and after the last
 * batch the duration scan when duration_end (:361-373).  Then every active
 * flow (:379-383) and the last export.  Records in push order: FIN/RST closes
 * in packet order; scans and the final flush in creation order (the reference
 * iterates a HashMap: unspecified). */
typedef struct {
    or_record* recs;
    uint32_t* interval; /* the export (CSV file) that writes the record */
    uint8_t* kind;      /* 0 FIN/RST close, 1 idle-timeout scan, 2 duration scan, 3 active at the end */
    uint64_t n, cap;
    uint64_t n_exports;
    uint64_t packets;
} or_live_result;
int or_live_buffer(const uint8_t* file, uint64_t nbytes, const uint64_t* batch_end, const uint8_t* batch_export,
                   uint64_t n_batches, uint64_t timeout_ms, int use_mac, int duration_end, or_live_result* out);
void or_live_free(or_live_result* r);
uint64_t or_record_size(void);

/* csv exporter (src/utils/fluere_csv_exporter.rs:5-81).  Returns bytes
 * written into buf (buf may be NULL to size). */
uint64_t or_format_csv(const or_record* recs, uint64_t n, char* buf, uint64_t cap);

#ifdef __cplusplus
}
#endif
#endif
