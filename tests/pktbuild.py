"""Tiny packet/pcap builder for the parity fixtures (no third-party deps)."""
from __future__ import annotations

import struct

VXLAN = bytes([0x08, 0, 0, 0, 0, 0, 0x64, 0])


def mac(s: str) -> bytes:
    return bytes(int(x, 16) for x in s.split(":"))


def ip4(s: str) -> bytes:
    return bytes(int(x) for x in s.split("."))


def ip6(s: str) -> bytes:
    import ipaddress
    return ipaddress.IPv6Address(s).packed


def eth(dst="02:00:00:00:00:02", src="02:00:00:00:00:01", et=0x0800) -> bytes:
    return mac(dst) + mac(src) + struct.pack(">H", et)


def ipv4(src, dst, proto, payload: bytes, ttl=64, dscp=0, ihl=5, tl=None, options=b"") -> bytes:
    opts = options.ljust((ihl - 5) * 4, b"\0") if ihl > 5 else b""
    if tl is None:
        tl = 20 + len(opts) + len(payload)
    h = struct.pack(">BBHHHBBH4s4s", (4 << 4) | (ihl & 0xF), dscp << 2, tl, 0x1234, 0x4000, ttl, proto, 0,
                    ip4(src), ip4(dst))
    return h + opts + payload


def ipv6(src, dst, nh, payload: bytes, tc=0, pl=None) -> bytes:
    if pl is None:
        pl = len(payload)
    vtf = (6 << 28) | (tc << 20)
    return struct.pack(">IHBB", vtf, pl, nh, 64) + ip6(src) + ip6(dst) + payload


def udp(sp, dp, payload=b"\x11" * 8, length=None) -> bytes:
    if length is None:
        length = 8 + len(payload)
    return struct.pack(">HHHH", sp, dp, length, 0) + payload


def tcp(sp, dp, flags, payload=b"", seq=1, ack=0, off=5) -> bytes:
    return struct.pack(">HHIIBBHHH", sp, dp, seq, ack, off << 4, flags, 65535, 0, 0) + payload


def arp(sender, target, op=1) -> bytes:
    return struct.pack(">HHBBH", 1, 0x0800, 6, 4, op) + mac("02:00:00:00:00:01") + ip4(sender) + \
        mac("00:00:00:00:00:00") + ip4(target)


FIN, SYN, RST, PSH, ACK, URG, ECE, CWR = 1, 2, 4, 8, 16, 32, 64, 128


def pcap(packets, nsec=False, swapped=False, snaplen=65535) -> bytes:
    """packets: list of (ts_sec, ts_frac, frame bytes[, orig_len])."""
    e = ">" if swapped else "<"
    magic = 0xa1b23c4d if nsec else 0xa1b2c3d4
    out = [struct.pack(e + "IHHiIII", magic, 2, 4, 0, 0, snaplen, 1)]
    for p in packets:
        sec, frac, data = p[0], p[1], p[2]
        orig = p[3] if len(p) > 3 else len(data)
        out.append(struct.pack(e + "IIII", sec, frac, len(data), orig) + data)
    return b"".join(out)
