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


def pcapng(items, swapped=False) -> bytes:
    """A pcapng capture from block items, in order:
      ("shb",)                                  Section Header Block
      ("idb", snaplen, tsresol_byte, tsoffset)  Interface Description Block (None: option absent)
      ("epb", ifid, t, frame[, orig_len])       Enhanced Packet Block (t in the interface's units)
      ("opb", ifid, t, frame)                   obsolete Packet Block (type 2)
      ("spb", frame[, orig_len])                Simple Packet Block
      ("isb", ifid) / ("nrb",) / ("custom",)    blocks a reader skips
    """
    e = ">" if swapped else "<"

    def block(btype, body: bytes) -> bytes:
        body = body + b"\0" * (-len(body) % 4)
        total = 12 + len(body)
        return struct.pack(e + "II", btype, total) + body + struct.pack(e + "I", total)

    def opt(code, value: bytes) -> bytes:
        return struct.pack(e + "HH", code, len(value)) + value + b"\0" * (-len(value) % 4)

    out = []
    for it in items:
        k = it[0]
        if k == "shb":
            out.append(block(0x0A0D0D0A, struct.pack(e + "IHHq", 0x1A2B3C4D, 1, 0, -1)))
        elif k == "idb":
            _, snap, tsres, tsoff = it
            opts = b""
            if tsres is not None:
                opts += opt(9, bytes([tsres]))
            if tsoff is not None:
                opts += opt(14, struct.pack(e + "q", tsoff))
            if opts:
                opts += struct.pack(e + "HH", 0, 0)
            out.append(block(1, struct.pack(e + "HHI", 1, 0, snap) + opts))
        elif k == "epb":
            ifid, t, frame = it[1], it[2], it[3]
            orig = it[4] if len(it) > 4 else len(frame)
            out.append(block(6, struct.pack(e + "IIIII", ifid, t >> 32, t & 0xFFFFFFFF, len(frame), orig) + frame))
        elif k == "opb":
            ifid, t, frame = it[1], it[2], it[3]
            out.append(block(2, struct.pack(e + "HHIIII", ifid, 0, t >> 32, t & 0xFFFFFFFF, len(frame), len(frame))
                             + frame))
        elif k == "spb":
            frame = it[1]
            orig = it[2] if len(it) > 2 else len(frame)
            out.append(block(3, struct.pack(e + "I", orig) + frame))
        elif k == "isb":
            out.append(block(5, struct.pack(e + "III", it[1], 0, 0)))
        elif k == "nrb":
            out.append(block(4, struct.pack(e + "HH", 0, 0)))
        elif k == "custom":
            out.append(block(0x00000BAD, struct.pack(e + "I", 32473) + b"custom"))
    return b"".join(out)
