"""Generates the committed parity fixtures under tests/golden/.

* ``ref_ipv4_frame.pcap``: the 554-byte Ethernet/IPv4/UDP frame held by the
  reference's own unit tests (src/net/parser/ipv4.rs:74-106, same bytes in
  udp.rs:49-81 and etherprotocol.rs:44-76) with the test's timestamp
  (tv_sec 1672986985, tv_usec 100000; ipv4.rs:58-65).  Its expected CSV row
  (``ref_ipv4_frame.expected.csv``) is derived from the reference source
   -- it pins the oracle, it is not produced by it.
* ``ref_raw_vectors.pcap``: every byte vector of the reference's unit tests
  of the raw fallback (tests/raw_vectors.py, transcribed from
  src/net/parser/raw/**) inside frames that reach the call sites of those
  parsers on the hot path: the parse_keys eager chain over an unknown
  ethertype whose low byte is the test's protocol hint (keys.rs:279-296),
  parse_fluereflow's from_ethertype arm (fluereflows.rs:148-195) and
  parse_ports for an unknown IP protocol (ports.rs:47).
* ``edge_pcapng[_swapped].pcap``: the same kind of traffic as pcapng (two
  sections, interfaces at 10^-6 / 10^-9 / 2^-20 s with an if_tsoffset and
  10^-3 s, Enhanced / Simple / obsolete Packet Blocks, blocks a reader skips,
  a truncated last block), both byte orders.  libpcap reads pcapng for
  pcap_open_offline (offline_fluereflows.rs:44); ``pcapng_expected()``
  restates its conversion so tests/test_oracle.py can check the oracle's
  reader against it.
* ``edge_*.pcap``: hand-built captures for every edge the hot path has
  (SURVEY.md Appendix B.3).  Their golden CSVs are produced by the C oracle
  (oracle/fluere_oracle.c) and committed, so the GPU box needs neither the
  reference nor a rebuild of the oracle to check them.

Run from the repo root:  python tests/golden/make_fixtures.py
(reads /root/reference only to extract the byte fixture above).
"""
from __future__ import annotations

import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from pktbuild import (ACK, CWR, ECE, FIN, PSH, RST, SYN, URG, VXLAN, arp, eth, ipv4, ipv6, pcap,  # noqa: E402
                      tcp, udp)

T0 = 1_700_000_000


def ref_frame() -> bytes:
    src = open("/root/reference/src/net/parser/ipv4.rs").read()
    body = src[src.index("data: &[") + len("data: &["):]
    body = body[: body.index("]")]
    data = bytes(int(x) for x in re.findall(r"\d+", body))
    assert len(data) == 554, len(data)
    return data


def U(sec_off, usec, frame):
    return (T0 + sec_off, usec, frame)


def fixtures():
    F = {}
    A, B = "10.0.0.1", "10.0.0.2"
    # UDP basic both directions + ttl/size variety
    F["edge_udp_bidir"] = [
        U(0, 0, eth() + ipv4(A, B, 17, udp(40000, 9000, b"\x01" * 22), ttl=64, dscp=10)),
        U(0, 5, eth("02:00:00:00:00:01", "02:00:00:00:00:02") + ipv4(B, A, 17, udp(9000, 40000, b"\x02" * 100), ttl=50)),
        U(0, 9, eth() + ipv4(A, B, 17, udp(40000, 9000, b"\x03" * 10), ttl=70, dscp=46)),
        U(1, 0, eth() + ipv4(A, "10.0.0.3", 17, udp(40000, 9000, b"\x04" * 30), dscp=1)),
    ]
    # VXLAN in UDP (VNI 100) and in TCP bytes 8..16; bad inner (< 14 bytes)
    inner = eth("02:aa:00:00:00:02", "02:aa:00:00:00:01") + ipv4("192.168.1.1", "192.168.1.2", 17, udp(1111, 2222, b"\x05" * 20))
    tcp_vx = tcp(5000, 6000, 0, seq=1, ack=0x08000000, off=0)[:12] + bytes([0x00, 0x00, 0x64, 0x00])
    F["edge_vxlan"] = [
        U(0, 0, eth() + ipv4(A, B, 17, udp(4789, 4789, VXLAN + inner))),
        U(0, 1, eth() + ipv4(A, B, 17, udp(4789, 4789, VXLAN + inner))),
        U(0, 2, eth() + ipv4(A, B, 6, tcp_vx + inner)),
        U(0, 3, eth() + ipv4(A, B, 17, udp(4789, 4789, VXLAN + b"\x01" * 10))),  # inner < 14: K drops
        U(0, 4, eth() + ipv4(A, B, 17, udp(4789, 4789, VXLAN + inner[:14]))),   # inner header only
    ]
    # empty UDP-view payloads: K drops
    F["edge_empty_payload"] = [
        U(0, 0, eth() + ipv4(A, B, 17, udp(1000, 2000, b""))),
        U(0, 1, eth() + ipv4(A, B, 1, bytes([8, 0, 0, 0, 0, 1, 0, 1]))),      # 8-byte ICMP echo
        U(0, 2, eth() + ipv4(A, B, 1, bytes([8, 0, 0, 0, 0, 1, 0, 1, 9]))),   # 9-byte ICMP echo: kept
        U(0, 3, eth() + ipv4(A, B, 17, udp(1000, 2000, b"x"))),
    ]
    # TCP SYN gate, FIN split, RST, reopen, reverse opener
    F["edge_tcp"] = [
        U(0, 0, eth() + ipv4(A, B, 6, tcp(1234, 80, ACK))),            # no flow, no SYN: dropped
        U(0, 1, eth() + ipv4(A, B, 6, tcp(1234, 80, SYN))),            # creates
        U(0, 2, eth() + ipv4(B, A, 6, tcp(80, 1234, SYN | ACK))),      # reverse
        U(0, 3, eth() + ipv4(A, B, 6, tcp(1234, 80, ACK | PSH, b"hello"))),
        U(0, 4, eth() + ipv4(A, B, 6, tcp(1234, 80, FIN | ACK))),      # closes (record #1)
        U(0, 5, eth() + ipv4(B, A, 6, tcp(80, 1234, ACK))),            # dropped
        U(0, 6, eth() + ipv4(B, A, 6, tcp(80, 1234, FIN | ACK))),      # dropped
        U(0, 7, eth() + ipv4(B, A, 6, tcp(80, 1234, SYN))),            # reopens, reverse orientation
        U(0, 8, eth() + ipv4(A, B, 6, tcp(1234, 80, ACK | URG | ECE | CWR))),
        U(0, 9, eth() + ipv4(A, B, 6, tcp(1234, 80, RST))),            # closes (record #2)
        U(0, 10, eth() + ipv4("10.9.9.9", B, 6, tcp(999, 80, SYN | FIN))),  # opens and closes at once
        U(0, 11, eth() + ipv4("10.9.9.8", B, 6, tcp(998, 80, SYN))),   # stays active
        U(0, 12, eth() + ipv4("10.9.9.8", B, 6, tcp(998, 80, ACK, b"z" * 100))),
        U(0, 13, eth() + ipv4(A, B, 6, tcp(1234, 80, ACK)[:16])),      # truncated TCP: K invalid
    ]
    # DNS special case, DSCP mapping, GRE, proto 0x36 / short unknown protocols
    F["edge_l4_quirks"] = [
        U(0, 0, eth() + ipv4(A, "8.8.8.8", 17, udp(5353, 53, b"\x12" * 30), dscp=46)),
        U(0, 1, eth() + ipv4("8.8.8.8", A, 17, udp(53, 5353, b"\x13" * 60))),
        U(0, 2, eth() + ipv4(A, B, 17, udp(7000, 7001, b"\x14" * 12), dscp=46)),
        U(0, 3, eth() + ipv4(A, B, 17, udp(7000, 7001, b"\x15" * 12), dscp=1)),
        U(0, 4, eth() + ipv4(A, B, 47, bytes([0, 0, 0x08, 0x00]) + b"\x45" * 20)),  # GRE
        U(0, 5, eth() + ipv4(A, B, 0x36, bytes([7, 9, 1, 2, 3]))),    # raw 0x36 pattern
        U(0, 6, eth() + ipv4(A, B, 99, bytes([1, 2, 3, 4, 5]))),      # raw generic ports
        U(0, 7, eth() + ipv4(A, B, 99, bytes([1, 2, 3]))),            # < 4 bytes: (0, 0)
        U(0, 8, eth() + ipv4(A, B, 99, bytes(range(12)))),            # UDP view
        U(0, 9, eth() + ipv4(A, B, 53, bytes([1, 2, 3, 4, 5]))),      # proto 53 short: (53, 53)
        U(0, 10, eth() + ipv4(A, B, 132, bytes(range(40)))),          # SCTP: TCP view ports
        U(0, 11, eth() + ipv4(A, B, 17, udp(1, 2, b"\x01" * 4)[:7])),  # 7-byte UDP: K invalid
    ]
    # IPv4 header oddities
    F["edge_ipv4_hdr"] = [
        U(0, 0, eth() + ipv4(A, B, 17, udp(1, 2, b"\x21" * 16), ihl=6, options=b"\x01\x01\x01\x01")),
        U(0, 1, eth() + ipv4(A, B, 17, udp(1, 2, b"\x22" * 16), tl=10)),     # tl < 20: empty payload
        U(0, 2, eth() + ipv4(A, B, 17, udp(1, 2, b"\x23" * 16), tl=2000)),   # tl > frame: clipped payload
        U(0, 3, eth() + ipv4(A, B, 17, udp(1, 2, b"\x24" * 16), ihl=3)),     # ihl < 5
        U(0, 4, eth() + ipv4(A, B, 17, udp(1, 2, b"\x25" * 16), ihl=15, options=b"\x01" * 40)),
        U(0, 5, eth() + ipv4(A, B, 17, b"")[:30]),                           # short IPv4: K/F fail
        U(0, 6, eth()[:10]),                                                 # < 14 bytes
        U(0, 7, b""),                                                        # empty record
        U(0, 8, (eth() + ipv4(A, B, 17, udp(1, 2, b"\x26" * 20)))[:40]),     # caplen cut
    ]
    # IPv6 UDP / TCP / ICMPv6 / short
    S6, D6 = "2001:db8::1", "2001:db8:0:0:1::2"
    F["edge_ipv6"] = [
        U(0, 0, eth(et=0x86DD) + ipv6(S6, D6, 17, udp(5000, 6000, b"\x31" * 20), tc=46 << 2)),
        U(0, 1, eth(et=0x86DD) + ipv6(D6, S6, 17, udp(6000, 5000, b"\x32" * 40))),
        U(0, 2, eth(et=0x86DD) + ipv6(S6, D6, 58, bytes([128, 0, 0, 0, 0, 1, 0, 1]) + b"\x33" * 8)),
        U(0, 3, eth(et=0x86DD) + ipv6(S6, "::ffff:10.1.2.3", 6, tcp(443, 8443, SYN))),
        U(0, 4, eth(et=0x86DD) + ipv6("::", "::1", 17, udp(1, 2, b"\x34" * 9))),
        U(0, 5, eth(et=0x86DD) + ipv6(S6, D6, 17, udp(5000, 6000, b""))),         # empty UDP payload
        U(0, 6, eth(et=0x86DD) + ipv6(S6, D6, 17, b"\x00" * 4)),                  # 4-byte UDP: invalid
        U(0, 7, (eth(et=0x86DD) + ipv6(S6, D6, 17, udp(1, 2)))[:40]),             # short
        U(0, 8, eth(et=0x86DD) + ipv6("fe80::1:0:0:1", "1:0:0:1::", 17, udp(7, 8, b"\x35" * 9))),
    ]
    # ARP / RARP / VLAN misparse / unknown ethertypes (raw fallback classes)
    F["edge_arp"] = [
        U(0, 0, eth("ff:ff:ff:ff:ff:ff", et=0x0806) + arp(A, B)),
        U(0, 1, eth(et=0x0806) + arp(B, A, op=2)),
        U(0, 2, eth(et=0x0806) + arp(A, B)[:20]),                              # short ARP
    ]
    F["edge_vlan_drop"] = [
        U(0, 0, eth(et=0x8100) + bytes([0, 5, 0x08, 0x00]) + ipv4(A, B, 17, udp(1, 2, b"\x41" * 18))),
        U(0, 1, eth(et=0x8100) + bytes([0, 5, 0x08, 0x00]) + ipv4("10.200.1.1", B, 6, tcp(1, 2, SYN))),
        U(0, 2, eth(et=0x8100) + bytes([0, 5])),                               # VLAN tag cut: K fails
    ]
    F["raw_classes"] = [
        U(0, 0, eth(et=0x8100) + bytes([0, 5, 0x08, 0x00]) + ipv4("8.0.1.1", B, 17, udp(1, 2, b"\x42" * 18))),
        U(0, 1, eth(et=0x88B5) + b"\x45" + b"\x00" * 40),
        U(0, 2, eth(et=0x8035) + arp(A, B)),
        U(0, 3, eth(et=0x88CC) + b"\x01\x02"),                                 # < 4 bytes payload
        U(0, 4, eth(et=0x8847) + bytes([0, 1, 0x41, 64]) + b"\x00" * 30),      # MPLS
    ]
    # every sub-parser of the raw fallback (src/net/parser/raw): VPN, VXLAN,
    # WireGuard and generic ethertype ranges, the eager key chain over an
    # unknown ethertype, OpenVPN shapes, short L4 payloads of unusual protocols
    F["raw_more"] = [
        U(0, 0, eth(et=0x0A08) + bytes([0, 0, 0x12, 0x34]) + ipv4("172.16.0.1", "172.16.0.2", 17, udp(5, 6, b"\x01" * 8))),
        U(0, 1, eth(et=0x4B65) + bytes([0, 0, 0x56, 0x78]) + ipv6("fd00::1", "fd00::2", 17, udp(7, 8, b"\x02" * 8))),
        U(0, 2, eth(et=0x12B5) + VXLAN + b"\x03" * 16),
        U(0, 3, eth(et=0x12B5) + bytes([0x09, 0, 0, 0, 0, 0, 0x64, 0]) + b"\x03" * 16),
        U(0, 4, eth(et=0x88B8) + bytes([1]) + b"\x00" * 147),
        U(0, 5, eth(et=0x88B8) + bytes([2]) + b"\x00" * 50),
        U(0, 6, eth(et=0x88B8) + bytes([4]) + b"\x00" * 31),
        U(0, 7, eth(et=0xB812) + bytes([0x11, 0x22, 0x33, 0x44, 0x55])),
        U(0, 8, eth(et=0x3655) + bytes([0x66, 0x77, 0x88, 0x99])),
        U(0, 9, eth(et=0x88B5) + ipv4("10.9.0.1", "10.9.0.2", 1, b"\x08\x00\x00\x00" + b"\x00" * 12)),
        U(0, 10, eth(et=0x9000) + bytes([0x40]) + b"\x00" * 8 + bytes([10, 1, 1, 1, 10, 1, 1, 2, 0x04, 0xD2, 0x16, 0x2E])
          + b"\x00" * 4),
        U(0, 11, eth(et=0x9000) + bytes([0x06]) + b"\x00" * 8 + ipv4("10.2.2.1", "10.2.2.2", 17, udp(1000, 2000, b"")[:4])),
        U(0, 12, eth() + ipv4("10.0.0.5", "10.0.0.6", 0x36, b"\xAB\xCD\xEF\x01\x02\x03")),
        U(0, 13, eth() + ipv4("10.0.0.5", "10.0.0.6", 171, bytes([6]) + b"\x00" * 5)),
        U(0, 14, eth() + ipv4("10.0.0.5", "10.0.0.6", 99, b"\x12\x34\x56")),
        U(0, 15, eth(et=0x86DD) + ipv6("fd00::5", "fd00::6", 0x36, b"\xAB\xCD\xEF")),
        U(0, 16, eth(et=0x8848) + bytes([0xFF, 0xFF, 0xF3, 0x40]) + b"\x00" * 20),
    ]
    # symmetric key, MAC-keyed flows, timestamp order, expiry
    F["edge_keys"] = [
        U(0, 0, eth() + ipv4(A, A, 17, udp(7, 7, b"\x51" * 10))),               # Key == reverse key
        U(0, 1, eth() + ipv4(A, A, 17, udp(7, 7, b"\x52" * 10))),
        U(0, 2, eth("02:00:00:00:00:09", "02:00:00:00:00:08") + ipv4(A, B, 17, udp(10, 20, b"\x53" * 10))),
        U(0, 3, eth("02:00:00:00:00:07", "02:00:00:00:00:06") + ipv4(A, B, 17, udp(10, 20, b"\x54" * 10))),
        U(0, 4, eth("02:00:00:00:00:06", "02:00:00:00:00:07") + ipv4(B, A, 17, udp(20, 10, b"\x55" * 10))),
        U(-5, 0, eth() + ipv4(A, B, 17, udp(10, 20, b"\x56" * 10))),            # time goes backwards
    ]
    F["edge_expiry"] = [
        U(0, 0, eth() + ipv4(A, B, 17, udp(1, 2, b"\x61" * 10))),
        U(0, 500, eth() + ipv4(A, B, 6, tcp(3, 4, SYN))),
        U(0, 900, eth() + ipv4(A, B, 6, tcp(3, 4, FIN | ACK))),               # closes; stale E entry stays
        U(0, 950, eth() + ipv4(A, B, 6, tcp(3, 4, SYN))),                     # reopened: evicted at 1.5 ms
        U(0, 1400, eth() + ipv4(A, B, 17, udp(1, 2, b"\x62" * 10))),
        U(0, 1600, eth() + ipv4(A, B, 6, tcp(3, 4, ACK))),                    # no flow now: dropped
        U(0, 2100, eth() + ipv4(B, A, 17, udp(2, 1, b"\x63" * 10))),
        U(0, 2100, eth() + ipv4(B, A, 17, udp(2, 1, b"\x64" * 10))),
        U(0, 4000, eth() + ipv4(A, B, 6, tcp(3, 4, SYN))),
    ]
    F["ref_raw_vectors"] = raw_vector_frames()
    return F


def raw_vector_frames():
    import raw_vectors as RV
    out, k = [], 0
    special = {0, 1, 2, 4, 6, 17, 47, 50, 51, 53, 58}
    # from_ethertype reads the whole frame from the destination MAC on: a first
    # byte outside the OpenVPN packet types keeps its heuristic out of the way
    M = "5e:00:00:00:00:02"
    for name, where, fn, data, arg, check in RV.VECTORS:
        frames = []
        if fn in (RV.FROM_RAW_PACKET, RV.PARSE_PROTOCOL, RV.OPENVPN, RV.ICMP):
            hint = arg & 0xFF
            frames.append(eth(M, et=0x9900 | hint) + data)          # eager chain: from_raw_packet(payload, et as u8)
            if hint not in special and len(data) < 8:           # parse_ports -> from_raw_packet(l4, proto)
                frames.append(eth(M) + ipv4("10.7.0.1", "10.7.0.2", hint, data))
        if fn in (RV.FROM_ETHERTYPE, RV.PARSE_ETHERTYPE):
            frames.append(eth(M, et=arg) + data)                 # parse_fluereflow: from_ethertype(frame, et)
        if fn == RV.ICMP:
            frames.append(eth(M) + ipv4("10.7.0.3", "10.7.0.4", 1, data + b"\x00"))
        for f in frames:
            out.append(U(0, k, f))
            k += 1
    for data, size, has in RV.ANALYZE_STRUCTURE:
        out.append(U(0, k, eth(M, et=0x3601) + data))
        k += 1
    return out


def pcapng_items():
    """(pcapng block items, the classic records libpcap yields for them:
    (sec, usec, data, orig_len))."""
    A, B, C = "10.0.0.1", "10.0.0.2", "10.0.0.3"
    f1 = eth() + ipv4(A, B, 17, udp(1000, 2000, b"\x21" * 30))
    f2 = eth() + ipv4(B, A, 17, udp(2000, 1000, b"\x22" * 12))
    f3 = eth() + ipv4(A, C, 6, tcp(3000, 80, SYN))
    f4 = eth() + ipv4(C, A, 6, tcp(80, 3000, SYN | ACK))
    f5 = eth() + ipv4(A, C, 6, tcp(3000, 80, FIN | ACK))
    f6 = eth() + ipv4(C, A, 6, tcp(80, 3000, ACK))
    f7 = eth() + ipv4(A, B, 17, udp(1000, 2000, b"\x23" * 400))
    T = 1_700_000_000
    items = [("shb",),
             ("idb", 0, None, None),                 # interface 0: microseconds, snaplen 0 -> 262144
             ("idb", 65535, 9, None),                # interface 1: nanoseconds
             ("idb", 0, 0x80 | 20, 3600),            # interface 2: 2^-20 s, +1 h offset
             ("epb", 0, T * 10**6 + 5, f1),
             ("nrb",),
             ("epb", 1, T * 10**9 + 7_123_456, f2),
             ("isb", 0),
             ("epb", 2, (T - 3600) * 2**20 + 2**19 + 3, f3),
             ("custom",),
             ("spb", f4),                            # no time: 0.0
             ("opb", 0, T * 10**6 + 999_999, f5),
             ("epb", 1, T * 10**9 + 1_000_000_999, f7),
             ("shb",),                               # a new section forgets the interfaces
             ("idb", 0, 3, None),                    # milliseconds
             ("epb", 0, T * 1000 + 1500, f6),
             ("epb", 0, T * 1000 + 1501, f1)]
    exp = [(T, 5, f1, len(f1)), (T, 7123, f2, len(f2)), (T, 500002, f3, len(f3)), (0, 0, f4, len(f4)),
           (T, 999999, f5, len(f5)), (T + 1, 0, f7, len(f7)), (T + 1, 500000, f6, len(f6)),
           (T + 1, 501000, f1, len(f1))]
    return items, exp


def pcapng_expected():
    return pcap(pcapng_items()[1])


# (timeout_ms, use_mac) combinations checked per fixture
PARAMS = {
    "default": [(600000, False), (600000, True)],
    "edge_expiry": [(600000, False), (1, False), (0, False), (2, False)],
    "edge_udp_bidir": [(600000, False), (0, False), (1000, False)],
    "edge_tcp": [(600000, False), (0, False)],
    "edge_keys": [(600000, False), (600000, True), (1, True)],
}


def main():
    import pyoracle
    pyoracle.build()
    manifest = {}
    frame = ref_frame()
    ref = pcap([(1672986985, 100000, frame)])
    open(os.path.join(HERE, "ref_ipv4_frame.pcap"), "wb").write(ref)
    open(os.path.join(HERE, "ref_ipv4_frame.expected.csv"), "w").write(
        "source,destination,src_port,dst_port,prot,d_pkts,d_octets,in_pkts,out_pkts,in_bytes,out_bytes,"
        "first,last,min_pkt,max_pkt,min_ttl,max_ttl,fin_cnt,syn_cnt,rst_cnt,psh_cnt,ack_cnt,urg_cnt,ece_cnt,"
        "cwr_cnt,ns_cnt,tos\n"
        "192.168.50.241,1.209.175.116,41641,41641,17,1,540,0,1,0,540,1672986985100000,1672986985100000,"
        "540,540,128,128,0,0,0,0,0,0,0,0,0,0\n")
    caps = {}
    for name, pk in fixtures().items():
        caps[name] = pcap(pk)
    caps["edge_udp_bidir_nsec"] = pcap([(s, f * 1000 + 7, d) for s, f, d in fixtures()["edge_udp_bidir"]], nsec=True)
    caps["edge_udp_bidir_swapped"] = pcap(fixtures()["edge_udp_bidir"], swapped=True)
    caps["edge_tcp_snap60"] = pcap(fixtures()["edge_tcp"], snaplen=60)
    caps["ref_ipv4_frame"] = ref
    from pktbuild import pcapng
    items = pcapng_items()[0]
    ng = pcapng(items)
    caps["edge_pcapng"] = ng + ng[12: 12 + 40][:20]  # a truncated block at the end
    caps["edge_pcapng_swapped"] = pcapng(items, swapped=True)
    for name, data in sorted(caps.items()):
        open(os.path.join(HERE, name + ".pcap"), "wb").write(data)
        runs = []
        for timeout, use_mac in PARAMS.get(name.split("_nsec")[0].split("_swapped")[0].split("_snap")[0],
                                          PARAMS["default"]):
            r = pyoracle.offline(data, timeout, use_mac)
            tag = f"{name}.t{timeout}{'.M' if use_mac else ''}"
            open(os.path.join(HERE, tag + ".csv"), "w").write(r["csv"])
            runs.append(dict(timeout_ms=timeout, use_mac=use_mac, csv=tag + ".csv", n_ended=r["n_ended"],
                             records=r["n"], raw_used=r["raw_used"]))
        meta = pyoracle.parse_batch(data)
        manifest[name] = dict(pcap=name + ".pcap", packets=len(meta), raw_packets=int(meta["raw_used"].sum()),
                              runs=runs)
    json.dump(manifest, open(os.path.join(HERE, "manifest.json"), "w"), indent=1, sort_keys=True)
    print(f"wrote {len(manifest)} fixtures")


if __name__ == "__main__":
    main()
