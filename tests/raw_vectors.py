"""The reference's own unit tests of the raw fallback (src/net/parser/raw),
transcribed as data: input bytes, the function called, and the assertions the
reference makes on the returned Option<RawProtocolHeader>.

The hot path reaches this code from parse_ports for IP protocols it does not
know (ports.rs:47), from the eager chain of parse_keys over an unknown
ethertype (keys.rs:279-296) and from parse_fluereflow for every ethertype
other than IPv4 / IPv6 / ARP (fluereflows.rs:148-195).  Each vector is
checked on the oracle (tests/test_oracle.py) and, through the
fluere_debug_raw probe, on the device functions themselves
(tests/test_gpu_parity.py); make_fixtures.py also embeds every vector in
frames that reach those call sites (fixture ``ref_raw_vectors``).

Not transcribed, with the reason:
  raw/mod.rs:357 test_raw_protocol_header_builder and :609
  test_builder_pattern_completeness exercise the Rust builder methods
  (with_flags, with_spi ...), which no parser input reaches;
  raw/ethertypes/mod.rs:313 test_is_known_ethertype tests a logging helper.
The dead protocol parsers (gre, igmp, ah, esp, ipx, sctp, vrrp, ospf, pim:
commented out at raw/protocols/mod.rs:51-63) are not on any path.

A header is a dict with: some, src / dst (bytes of the IpAddr or None),
src_port, dst_port, protocol, length, flags, version, ethertype (None when the
Option is None) and payload (bytes or None).
"""
from __future__ import annotations

FROM_RAW_PACKET, FROM_ETHERTYPE, PARSE_ETHERTYPE, PARSE_PROTOCOL, OPENVPN, ICMP = range(6)

V4 = lambda a, b, c, d: bytes([a, b, c, d])  # noqa: E731  IpAddr::V4(Ipv4Addr::new(..))

_WG_INIT = bytes([0x01, 0x00, 0x00, 0x00]) + bytes(144)
_WG_DATA = bytes([0x04, 0x00, 0x00, 0x00, 0x12, 0x34, 0x56, 0x78, 0x9a, 0xbc, 0xde, 0xf0, 0x11, 0x22, 0x33, 0x44])


def _eq(**want):
    def check(h):
        assert h["some"], "expected Some(header)"
        for k, v in want.items():
            assert h[k] == v, f"{k}: {h[k]!r} != {v!r}"
    return check


def _some(h):
    assert h["some"], "expected Some(header)"


def _none(h):
    assert not h["some"], "expected None"


# (name, reference file:line, function, bytes, argument, check)
VECTORS = [
    # ---- src/net/parser/raw/mod.rs tests (:382-672)
    ("from_raw_packet_valid_ipv4", "raw/mod.rs:382-408", FROM_RAW_PACKET,
     bytes([0x45, 0x00, 0x00, 0x28, 0x12, 0x34, 0x40, 0x00, 0x40, 0x06, 0x00, 0x00, 192, 168, 1, 1, 192, 168, 1, 2,
            0x00, 0x50, 0x01, 0xbb, 0x00, 0x00, 0x00, 0x00]), 6,
     _eq(src=V4(192, 168, 1, 1), dst=V4(192, 168, 1, 2), src_port=80, dst_port=443, protocol=6)),
    ("from_raw_packet_malformed_ipv4", "raw/mod.rs:410-423", FROM_RAW_PACKET,
     bytes([0x44, 0x00, 0x00, 0x14, 0x12, 0x34, 0x40, 0x00, 0x40, 0x06, 0x00, 0x00, 192, 168, 1, 1, 192, 168, 1, 2]), 6,
     _eq(protocol=6)),
    ("from_raw_packet_too_short", "raw/mod.rs:425-431", FROM_RAW_PACKET, bytes([0x45, 0x00]), 6, _none),
    ("from_raw_packet_netflix_vpn_pattern", "raw/mod.rs:433-447", FROM_RAW_PACKET,
     bytes([0x00, 0x50, 0x01, 0xbb, 0xde, 0xad, 0xbe, 0xef]), 0xb9,
     _eq(src_port=80, dst_port=443, protocol=0xb9, payload=bytes([0xde, 0xad, 0xbe, 0xef]))),
    ("from_raw_packet_custom_vpn_pattern", "raw/mod.rs:449-463", FROM_RAW_PACKET,
     bytes([0x50, 0xbb, 0xde, 0xad, 0xbe, 0xef]), 0x36,
     _eq(src_port=0x50, dst_port=0xbb, protocol=0x36, payload=bytes([0xde, 0xad, 0xbe, 0xef]))),
    ("from_raw_packet_generic_fallback", "raw/mod.rs:465-479", FROM_RAW_PACKET,
     bytes([0x12, 0x34, 0x56, 0x78, 0xaa, 0xbb, 0xcc, 0xdd]), 99,
     _eq(src_port=0x1234, dst_port=0x5678, protocol=99, payload=bytes([0x12, 0x34, 0x56, 0x78, 0xaa, 0xbb, 0xcc, 0xdd]))),
    ("from_ethertype_ipv4", "raw/mod.rs:481-504", FROM_ETHERTYPE,
     bytes([0x45, 0x00, 0x00, 0x1c, 0x12, 0x34, 0x40, 0x00, 0x40, 0x11, 0x00, 0x00, 192, 168, 1, 1, 192, 168, 1, 2,
            0x00, 0x35, 0x00, 0x35]), 0x0800,
     _eq(src=V4(192, 168, 1, 1), dst=V4(192, 168, 1, 2), protocol=17)),
    ("from_ethertype_unknown", "raw/mod.rs:506-513", FROM_ETHERTYPE,
     bytes([0x12, 0x34, 0x56, 0x78, 0xaa, 0xbb, 0xcc, 0xdd]), 0x9999, _some),
    ("ipv4_header_with_options", "raw/mod.rs:515-539", FROM_RAW_PACKET,
     bytes([0x46, 0x00, 0x00, 0x20, 0x12, 0x34, 0x40, 0x00, 0x40, 0x06, 0x00, 0x00, 192, 168, 1, 1, 192, 168, 1, 2,
            0x01, 0x02, 0x03, 0x04, 0x00, 0x50, 0x01, 0xbb, 0x00, 0x00, 0x00, 0x00]), 6,
     _eq(src=V4(192, 168, 1, 1), dst=V4(192, 168, 1, 2), src_port=80, dst_port=443)),
    ("ipv6_version_detection", "raw/mod.rs:541-559", FROM_RAW_PACKET,
     bytes([0x60, 0x00, 0x00, 0x00, 0x00, 0x08, 0x11, 0x40,
            0x20, 0x01, 0x0d, 0xb8, 0x85, 0xa3, 0x00, 0x00, 0x00, 0x00, 0x8a, 0x2e, 0x03, 0x70, 0x73, 0x34,
            0x20, 0x01, 0x0d, 0xb8, 0x85, 0xa3, 0x00, 0x00, 0x00, 0x00, 0x8a, 0x2e, 0x03, 0x70, 0x73, 0x35,
            0x00, 0x35, 0x00, 0x35]), 17,
     _eq(protocol=17)),
    ("port_extraction_edge_cases", "raw/mod.rs:561-579", FROM_RAW_PACKET,
     bytes([0x45, 0x00, 0x00, 0x16, 0x12, 0x34, 0x40, 0x00, 0x40, 0x06, 0x00, 0x00, 192, 168, 1, 1, 192, 168, 1, 2,
            0x00, 0x50]), 6,
     _eq(src_port=0, dst_port=0, src=V4(192, 168, 1, 1))),
    ("protocol_preservation", "raw/mod.rs:581-598", FROM_RAW_PACKET,
     bytes([0x45, 0x00, 0x00, 0x1c, 0x12, 0x34, 0x40, 0x00, 0x40, 0x32, 0x00, 0x00, 192, 168, 1, 1, 192, 168, 1, 2,
            0x12, 0x34, 0x56, 0x78]), 99,
     _eq(protocol=50, src=V4(192, 168, 1, 1))),
    ("empty_payload", "raw/mod.rs:600-606", FROM_RAW_PACKET, b"", 6, _none),
    ("invalid_ipv4_total_length", "raw/mod.rs:639-650", FROM_RAW_PACKET,
     bytes([0x45, 0x00, 0xff, 0xff, 0x12, 0x34, 0x40, 0x00, 0x40, 0x06, 0x00, 0x00, 192, 168, 1, 1, 192, 168, 1, 2]), 6,
     _some),
    ("ipv4_fragmented_packet", "raw/mod.rs:652-672", FROM_RAW_PACKET,
     bytes([0x45, 0x00, 0x00, 0x1c, 0x12, 0x34, 0x20, 0x00, 0x40, 0x06, 0x00, 0x00, 192, 168, 1, 1, 192, 168, 1, 2,
            0x00, 0x50, 0x01, 0xbb]), 6,
     _eq(src=V4(192, 168, 1, 1), dst=V4(192, 168, 1, 2), protocol=6)),
    # ---- src/net/parser/raw/ethertypes/mod.rs tests (:166-346)
    ("parse_ethertype_arp", "ethertypes/mod.rs:166-190", PARSE_ETHERTYPE,
     bytes([0x00, 0x01, 0x08, 0x00, 0x06, 0x04, 0x00, 0x01, 0xaa, 0xbb, 0xcc, 0xdd, 0xee, 0xff, 192, 168, 1, 1,
            0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 192, 168, 1, 2]), 0x0806,
     _eq(protocol=0x08, src=V4(192, 168, 1, 1), dst=V4(192, 168, 1, 2))),
    ("parse_ethertype_mpls", "ethertypes/mod.rs:192-204", PARSE_ETHERTYPE,
     bytes([0x00, 0x01, 0x90, 0x3f, 0x45, 0x00, 0x00, 0x1c]), 0x8847, _eq(protocol=137)),
    ("parse_ethertype_vxlan", "ethertypes/mod.rs:206-220", PARSE_ETHERTYPE,
     bytes([0x08, 0x00, 0x00, 0x00, 0x00, 0x00, 0x64, 0x00, 0xaa, 0xbb, 0xcc, 0xdd, 0xee, 0xff]), 0x12B5,
     _eq(protocol=0x12)),
    ("parse_ethertype_wireguard_init", "ethertypes/mod.rs:222-237", PARSE_ETHERTYPE, _WG_INIT, 0x88B8,
     _eq(protocol=1, flags=1, version=1)),
    ("parse_ethertype_wireguard_data", "ethertypes/mod.rs:239-250", PARSE_ETHERTYPE, _WG_DATA, 0x88B8,
     _eq(protocol=4)),
    ("parse_ethertype_vpn_data", "ethertypes/mod.rs:253-265", PARSE_ETHERTYPE,
     bytes([0x05, 0x02, 0x12, 0x34, 0xde, 0xad, 0xbe, 0xef]), 0x0A08, _eq(src_port=2186)),
    ("parse_ethertype_vpn_control", "ethertypes/mod.rs:267-279", PARSE_ETHERTYPE,
     bytes([0x03, 0x01, 0x56, 0x78, 0xca, 0xfe, 0xba, 0xbe]), 0x4B65, _eq(src_port=19301)),
    ("parse_ethertype_experimental", "ethertypes/mod.rs:281-287", PARSE_ETHERTYPE,
     bytes([0xB8, 0x01, 0x02, 0x03, 0x04, 0x05, 0x06, 0x07]), 0xB801, _some),
    ("parse_ethertype_vendor_specific", "ethertypes/mod.rs:289-295", PARSE_ETHERTYPE,
     bytes([0x36, 0x01, 0x02, 0x03, 0x04, 0x05]), 0x3601, _some),
    ("parse_ethertype_unknown", "ethertypes/mod.rs:297-303", PARSE_ETHERTYPE,
     bytes([0x12, 0x34, 0x56, 0x78]), 0xFFFF, _none),
    ("parse_ethertype_too_short", "ethertypes/mod.rs:305-311", PARSE_ETHERTYPE, bytes([0x00]), 0x0806, _none),
    # ---- src/net/parser/raw/protocols/openvpn.rs tests (:226-334)
    ("openvpn_tls_control_packet", "protocols/openvpn.rs:230-284", OPENVPN,
     bytes([0x40, 0x00, 0x01, 0x02, 0x03, 0x04, 0x05, 0x06, 0x07, 192, 168, 1, 1, 192, 168, 1, 2, 0x1F, 0x90, 0x01,
            0xBB, 0x00, 0x01, 0x02, 0x03]), 0x9B,
     _eq(src=V4(192, 168, 1, 1), dst=V4(192, 168, 1, 2), src_port=8080, dst_port=443)),
    ("openvpn_data_packet_with_ipv4", "protocols/openvpn.rs:286-333", OPENVPN,
     bytes([0x06, 0x00, 0x01, 0x02, 0x03, 0x00, 0x00, 0x00, 0x00, 0x45, 0x00, 0x06, 0x00, 192, 168, 1, 1, 192, 168, 1,
            2, 0x1F, 0x90, 0x01, 0xBB]), 0x9B,
     _eq(src=V4(192, 168, 1, 1), dst=V4(192, 168, 1, 2), src_port=8080, dst_port=443)),
    # ---- src/net/parser/raw/protocols/icmp.rs test (:55-73)
    ("icmp_parser", "protocols/icmp.rs:55-73", ICMP,
     bytes([8, 0, 0x00, 0x00, 0x12, 0x34, 0x56, 0x78]), 1,
     _eq(src_port=8, dst_port=0, protocol=1, length=8)),
]

# ethertypes/mod.rs:321-346 test_analyze_packet_structure: (bytes, header_size,
# has_payload).  On the parsers it shows as the payload start of
# parse_custom_protocol (mod.rs:107-134), reached through parse_ethertype with
# an ethertype in 0x3600..=0x36FF.
ANALYZE_STRUCTURE = [
    (bytes([0xB8, 0x01, 0x02, 0x03, 0x04, 0x05, 0x06, 0x07, 0x08, 0x09]), 8, True),
    (bytes([0x36, 0x01, 0x02, 0x03, 0x04, 0x05, 0x06, 0x07]), 6, True),
    (bytes([0x6C, 0x01, 0x02, 0x03, 0x04, 0x05]), 4, True),
    (bytes([0xFF, 0x01, 0x02, 0x03, 0x04, 0x05]), 4, True),
]
