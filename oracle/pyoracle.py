"""TEST INFRASTRUCTURE: ctypes access to the C restatement of the reference
CPU path (oracle/fluere_oracle.c).  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg import this module."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")
CLI = os.path.join(HERE, "_build", "fluere_oracle")

PKT_META_DTYPE = np.dtype([
    ("k_status", "u1"), ("f_status", "u1"), ("key_v6", "u1"), ("key_proto", "u1"),
    ("key_sport", "<u2"), ("key_dport", "<u2"), ("key_src", "u1", 16), ("key_dst", "u1", 16),
    ("key_smac", "u1", 6), ("key_dmac", "u1", 6), ("rec_v6", "u1"), ("rec_prot", "u1"), ("rec_tos", "u1"),
    ("rec_ttl", "u1"), ("rec_src", "u1", 16), ("rec_dst", "u1", 16), ("rec_sport", "<u2"), ("rec_dport", "<u2"),
    ("rec_pkt", "<u4"), ("doctets", "<u8"), ("time", "<u8"), ("flags", "<u2"), ("raw_used", "u1"),
    ("pad", "u1", 13),
])


class _Result(ctypes.Structure):
    _fields_ = [("recs", ctypes.c_void_p), ("n", ctypes.c_uint64), ("n_ended", ctypes.c_uint64),
                ("packets", ctypes.c_uint64), ("valid", ctypes.c_uint64), ("raw_used", ctypes.c_uint64),
                ("loop_seconds", ctypes.c_double), ("cap", ctypes.c_uint64)]


class _OrIp(ctypes.Structure):
    _fields_ = [("v6", ctypes.c_uint8), ("b", ctypes.c_uint8 * 16)]


class _OrRawHdr(ctypes.Structure):
    _fields_ = [("has_src", ctypes.c_uint8), ("has_dst", ctypes.c_uint8), ("src", _OrIp), ("dst", _OrIp),
                ("sport", ctypes.c_uint16), ("dport", ctypes.c_uint16), ("proto", ctypes.c_uint8),
                ("length", ctypes.c_uint16), ("has_flags", ctypes.c_uint8), ("flags", ctypes.c_uint8),
                ("has_version", ctypes.c_uint8), ("version", ctypes.c_uint8), ("has_ethertype", ctypes.c_uint8),
                ("ethertype", ctypes.c_uint16), ("has_payload", ctypes.c_uint8), ("payload_off", ctypes.c_uint32),
                ("payload_len", ctypes.c_uint32)]


class _LiveResult(ctypes.Structure):
    _fields_ = [("recs", ctypes.c_void_p), ("interval", ctypes.c_void_p), ("kind", ctypes.c_void_p),
                ("n", ctypes.c_uint64), ("cap", ctypes.c_uint64), ("n_exports", ctypes.c_uint64),
                ("packets", ctypes.c_uint64)]


_RAW_FNS = ["or_raw_from_raw_packet", "or_raw_from_ethertype", "or_raw_parse_ethertype", "or_raw_parse_protocol",
            "or_raw_openvpn", "or_raw_icmp"]

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        L.or_offline_buffer.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                                        ctypes.POINTER(_Result)]
        L.or_offline_buffer.restype = ctypes.c_int
        L.or_result_free.argtypes = [ctypes.POINTER(_Result)]
        L.or_format_csv.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64]
        L.or_format_csv.restype = ctypes.c_uint64
        L.or_parse_batch.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                     ctypes.POINTER(ctypes.c_uint64)]
        L.or_parse_batch.restype = ctypes.c_int
        L.or_pcap_index.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p)]
        L.or_pcap_index.restype = ctypes.c_int64
        for i, name in enumerate(_RAW_FNS):
            fn = getattr(L, name)
            fn.restype = ctypes.c_int
            fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32] + ([ctypes.c_uint32] if i < 4 else []) + \
                [ctypes.POINTER(_OrRawHdr)]
        L.or_live_buffer.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                     ctypes.POINTER(_LiveResult)]
        L.or_live_buffer.restype = ctypes.c_int
        L.or_live_free.argtypes = [ctypes.POINTER(_LiveResult)]
        L.or_record_size.restype = ctypes.c_uint64
        L.or_raw_analyze_structure.restype = None
        L.or_raw_analyze_structure.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32),
                                               ctypes.POINTER(ctypes.c_int)]
        _lib = L
    return _lib


def offline(pcap: bytes, timeout_ms: int = 600000, use_mac: bool = False):
    """-> dict(csv=str, n_ended=int, n=int, packets, valid, raw_used, loop_seconds)."""
    L = lib()
    buf = (ctypes.c_uint8 * max(len(pcap), 1)).from_buffer_copy(pcap + b"\0")
    r = _Result()
    if L.or_offline_buffer(buf, len(pcap), timeout_ms, 1 if use_mac else 0, ctypes.byref(r)) != 0:
        raise ValueError("oracle: not a classic pcap")
    try:
        need = L.or_format_csv(r.recs, r.n, None, 0)
        out = ctypes.create_string_buffer(need)
        L.or_format_csv(r.recs, r.n, out, need)
        return dict(csv=out.raw[:need].decode(), n=r.n, n_ended=r.n_ended, packets=r.packets, valid=r.valid,
                    raw_used=r.raw_used, loop_seconds=r.loop_seconds)
    finally:
        L.or_result_free(ctypes.byref(r))


def parse_batch(pcap: bytes) -> np.ndarray:
    L = lib()
    buf = (ctypes.c_uint8 * max(len(pcap), 1)).from_buffer_copy(pcap + b"\0")
    cnt = L.or_pcap_index(buf, len(pcap), ctypes.byref(ctypes.c_void_p()))
    n = max(int(cnt), 0)
    out = np.zeros(max(n, 1), dtype=PKT_META_DTYPE)
    got = ctypes.c_uint64()
    if L.or_parse_batch(buf, len(pcap), out.ctypes.data, n, ctypes.byref(got)) != 0:
        raise ValueError("oracle: not a classic pcap")
    return out[: got.value]


def time_offline_cli(path: str, timeout_ms: int = 600000, use_mac: bool = False, repeat: int = 1, core: int = 0):
    """CPU baseline: the "Converted in" window on one pinned core."""
    import json
    cmd = [CLI, "-f", path, "-t", str(timeout_ms), "--repeat", str(repeat)] + (["-M"] if use_mac else [])
    try:
        os.sched_setaffinity(0, os.sched_getaffinity(0))  # no-op probe
        cmd = ["taskset", "-c", str(core)] + cmd
    except Exception:
        pass
    out = subprocess.run(cmd, check=True, capture_output=True, text=True).stdout
    return json.loads(out.strip().splitlines()[-1])


def _ip(has, ip):
    if not has:
        return None
    return bytes(ip.b) if ip.v6 else bytes(ip.b[:4])


def raw_call(fn: int, data: bytes, arg: int = 0) -> dict:
    """One raw-fallback entry point of the oracle (tests/raw_vectors.py codes)
    -> the RawProtocolHeader as a dict (see tests/raw_vectors.py)."""
    L = lib()
    buf = (ctypes.c_uint8 * max(len(data), 1)).from_buffer_copy(data + b"\0")
    h = _OrRawHdr()
    args = [buf, len(data)] + ([arg] if fn < 4 else []) + [ctypes.byref(h)]
    some = getattr(L, _RAW_FNS[fn])(*args)
    if not some:
        return dict(some=False)
    return dict(some=True, src=_ip(h.has_src, h.src), dst=_ip(h.has_dst, h.dst), src_port=h.sport, dst_port=h.dport,
                protocol=h.proto, length=h.length, flags=h.flags if h.has_flags else None,
                version=h.version if h.has_version else None, ethertype=h.ethertype if h.has_ethertype else None,
                payload=data[h.payload_off:h.payload_off + h.payload_len] if h.has_payload else None)


def analyze_structure(data: bytes):
    L = lib()
    buf = (ctypes.c_uint8 * max(len(data), 1)).from_buffer_copy(data + b"\0")
    hs, hp = ctypes.c_uint32(), ctypes.c_int()
    L.or_raw_analyze_structure(buf, len(data), ctypes.byref(hs), ctypes.byref(hp))
    return hs.value, bool(hp.value)


def live(pcap: bytes, batch_end, batch_export, timeout_ms: int = 600000, use_mac: bool = False,
         duration_end: bool = False):
    """live mode over batches (or_live_buffer) -> list of exports, each
    dict(csv=str, n_ordered=int): the FIN/RST-closed rows first in order, the
    rest in creation order (the reference's HashMap order is unspecified)."""
    L = lib()
    buf = (ctypes.c_uint8 * max(len(pcap), 1)).from_buffer_copy(pcap + b"\0")
    be = np.ascontiguousarray(batch_end, dtype=np.uint64)
    bx = np.ascontiguousarray(batch_export, dtype=np.uint8)
    r = _LiveResult()
    if L.or_live_buffer(buf, len(pcap), be.ctypes.data, bx.ctypes.data, len(be), timeout_ms, 1 if use_mac else 0,
                        1 if duration_end else 0, ctypes.byref(r)) != 0:
        raise ValueError("oracle: not a pcap")
    try:
        rs = int(L.or_record_size())
        raw = ctypes.string_at(r.recs, r.n * rs) if r.n else b""
        interval = np.frombuffer(ctypes.string_at(r.interval, 4 * r.n), dtype=np.uint32) if r.n else np.zeros(0, np.uint32)
        kind = np.frombuffer(ctypes.string_at(r.kind, r.n), dtype=np.uint8) if r.n else np.zeros(0, np.uint8)
        out = []
        for k in range(r.n_exports):
            idx = np.nonzero(interval == k)[0]
            sel = b"".join(raw[int(j) * rs:(int(j) + 1) * rs] for j in idx)
            sb = (ctypes.c_uint8 * max(len(sel), 1)).from_buffer_copy(sel + b"\0")
            need = L.or_format_csv(sb, len(idx), None, 0)
            cb = ctypes.create_string_buffer(need)
            L.or_format_csv(sb, len(idx), cb, need)
            out.append(dict(csv=cb.raw[:need].decode(), n_ordered=int((kind[idx] == 0).sum())))
        return out
    finally:
        L.or_live_free(ctypes.byref(r))
