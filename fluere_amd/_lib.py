"""ctypes binding of the C ABI in include/fluere_gpu.h.

The product path is the in-tree HIP library ``fluere_amd/libfluere_gpu.so``;
there is no CPU fallback: if the library (or a GPU) is missing every compute
call raises.
"""
from __future__ import annotations

import ctypes
import os
import struct

import numpy as np

try:  # bind to torch's HIP runtime when torch is present (one runtime per process)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the C ABI itself
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
# FLUERE_LIB (diagnostics only): an alternative in-tree build of the same
# library, e.g. a kernel variant built by tools/variants.sh
LIB_PATH = os.environ.get("FLUERE_LIB") or os.path.join(_HERE, "libfluere_gpu.so")
CLI_PATH = os.path.join(_HERE, "fluere")

# enum fluere_status
OK = 0
E_ARG, E_IO, E_PCAP, E_HIP, E_NOMEM, E_TABLE_FULL, E_UNSUPPORTED, E_STATE = range(-1, -9, -1)
RETRY = 2  # fluere_merge_gathered_finish: redo the device-agreed step with the host-driven sequence
NEED_SWEEP = 1  # fluere_merge_gathered: complete the merge with the sweep composition (fluere_sweep_*)
_ERR_NAMES = {
    E_ARG: "bad argument", E_IO: "I/O error", E_PCAP: "not a pcap capture", E_HIP: "HIP error / no GPU",
    E_NOMEM: "out of memory", E_TABLE_FULL: "flow table full",
    E_UNSUPPORTED: "no exact result on this path",
    E_STATE: "call order",
}

SYNTH_UDP64, SYNTH_IMIX, SYNTH_VLAN64, SYNTH_MAC64, SYNTH_TCP, SYNTH_SLOW, SYNTH_TCP_BACKTIME = 0, 1, 2, 3, 4, 5, 6


class FluereError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        super().__init__(f"{what}: {_ERR_NAMES.get(code, code)} ({code})")


class Opts(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("stream", ctypes.c_void_p), ("timeout_ms", ctypes.c_uint64),
                ("use_mac", ctypes.c_int), ("max_flows", ctypes.c_uint64)]


class Stats(ctypes.Structure):
    _fields_ = [("packets", ctypes.c_uint64), ("valid", ctypes.c_uint64), ("updates", ctypes.c_uint64),
                ("dropped_parse", ctypes.c_uint64), ("unsupported", ctypes.c_uint64), ("flows", ctypes.c_uint64),
                ("complex_flows", ctypes.c_uint64), ("records", ctypes.c_uint64), ("ended", ctypes.c_uint64),
                ("sequential_mode", ctypes.c_uint32), ("passes", ctypes.c_uint32), ("parse_ms", ctypes.c_double),
                ("total_ms", ctypes.c_double)]

    def as_dict(self):
        # one unpack of the 96 bytes (per-field getattr costs ~3 us, about 1 %
        # of a C2 step)
        return dict(zip(_STATS_NAMES, _STATS_LAYOUT.unpack_from(self)))


_STATS_NAMES = tuple(k for k, _ in Stats._fields_)
_STATS_LAYOUT = struct.Struct("<9Q2I2d")
assert _STATS_LAYOUT.size == ctypes.sizeof(Stats)


class SynthCfg(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint64), ("n_packets", ctypes.c_uint64), ("n_flows", ctypes.c_uint32),
                ("kind", ctypes.c_uint32), ("rev_pct", ctypes.c_uint32), ("pad", ctypes.c_uint32)]


# struct fluere_record (152 bytes)
RECORD_DTYPE = np.dtype([
    ("src_v6", "u1"), ("dst_v6", "u1"), ("prot", "u1"), ("tos", "u1"), ("min_ttl", "u1"), ("max_ttl", "u1"),
    ("src_port", "<u2"), ("dst_port", "<u2"), ("source", "u1", 16), ("destination", "u1", 16), ("pad0", "<u2"),
    ("d_pkts", "<u4"), ("min_pkt", "<u4"), ("max_pkt", "<u4"), ("in_pkts", "<u4"), ("out_pkts", "<u4"),
    ("cnt", "<u4", 9), ("pad1", "<u4"), ("d_octets", "<u8"), ("first", "<u8"), ("last", "<u8"),
    ("in_bytes", "<u8"), ("out_bytes", "<u8"), ("order_key", "<u8"),
])
assert RECORD_DTYPE.itemsize == 152

# struct fluere_pkt_meta (128 bytes); the oracle's or_pkt_meta has the same layout
PKT_META_DTYPE = np.dtype([
    ("k_status", "u1"), ("f_status", "u1"), ("key_v6", "u1"), ("key_proto", "u1"),
    ("key_sport", "<u2"), ("key_dport", "<u2"), ("key_src", "u1", 16), ("key_dst", "u1", 16),
    ("key_smac", "u1", 6), ("key_dmac", "u1", 6), ("rec_v6", "u1"), ("rec_prot", "u1"), ("rec_tos", "u1"),
    ("rec_ttl", "u1"), ("rec_src", "u1", 16), ("rec_dst", "u1", 16), ("rec_sport", "<u2"), ("rec_dport", "<u2"),
    ("rec_pkt", "<u4"), ("doctets", "<u8"), ("time", "<u8"), ("flags", "<u2"), ("raw_used", "u1"),
    ("pad", "u1", 13),
])
assert PKT_META_DTYPE.itemsize == 128

# struct fluere_raw_hdr (64 bytes): fluere_debug_raw output
RAW_HDR_DTYPE = np.dtype([
    ("some", "u1"), ("has_src", "u1"), ("has_dst", "u1"), ("ip_v6", "u1"), ("src", "u1", 16), ("dst", "u1", 16),
    ("src_port", "<u2"), ("dst_port", "<u2"), ("protocol", "u1"), ("has_flags", "u1"), ("flags", "u1"),
    ("has_version", "u1"), ("version", "u1"), ("has_ethertype", "u1"), ("has_payload", "u1"), ("pad0", "u1"),
    ("length", "<u2"), ("ethertype", "<u2"), ("payload_off", "<u4"), ("payload_len", "<u4"), ("pad1", "<u4"),
])
assert RAW_HDR_DTYPE.itemsize == 64

SUMMARY_DTYPE = np.dtype([
    ("key", "<u4", 14), ("pkts", "<u4", 2), ("bytes", "<u8", 2), ("min_pkt", "<u4"), ("max_pkt", "<u4"),
    ("min_ttl", "<u4"), ("max_ttl", "<u4"), ("flag_cnt", "<u4", 8), ("first_all", "<u8"), ("first_create", "<u8"),
    ("finrst_min", "<u8"), ("last", "<u8"), ("first_time", "<u8"), ("last_time", "<u8"), ("first_sport", "<u2"),
    ("first_dport", "<u2"), ("first_dir", "u1"), ("first_prot", "u1"), ("first_tos", "u1"), ("first_v6", "u1"),
    ("first_src", "u1", 16), ("first_dst", "u1", 16), ("annex", "<u4"), ("shard", "<u4"), ("pad", "<u8", 4),
])
PIECE_DTYPE = np.dtype([
    ("pkts", "<u4", 2), ("bytes", "<u8", 2), ("min_pkt", "<u4"), ("max_pkt", "<u4"), ("min_ttl", "<u4"),
    ("max_ttl", "<u4"), ("flag_cnt", "<u4", 8), ("last", "<u8"), ("last_time", "<u8"), ("first", "<u8"),
    ("first_time", "<u8"), ("src", "u1", 16), ("dst", "u1", 16), ("v6", "u1"), ("prot", "u1"), ("tos", "u1"),
    ("dir", "u1"), ("src_port", "<u2"), ("dst_port", "<u2"),
])
ANNEX_DTYPE = np.dtype([("key", "<u4", 14), ("flags", "<u4"), ("pad", "<u4"), ("f0", "<u8"), ("lead", PIECE_DTYPE),
                        ("head", PIECE_DTYPE), ("tail", PIECE_DTYPE), ("mid_last", "<u8")])
SHARD_HEADER_DTYPE = np.dtype([("n_flows", "<u8"), ("n_annex", "<u8"), ("tmin", "<u8"), ("tmax", "<u8"),
                               ("valid", "<u8"), ("dropped", "<u8"), ("err", "<u4"), ("shard", "<u4"),
                               ("n_bare_complex", "<u8")])
SHARD_HEADER_BYTES = 64  # fluere_shard_header
SUMMARY_BYTES = SUMMARY_DTYPE.itemsize  # struct fluere_flow_summary
assert SUMMARY_BYTES == 256 and PIECE_DTYPE.itemsize == 144 and ANNEX_DTYPE.itemsize == 512
assert SHARD_HEADER_DTYPE.itemsize == SHARD_HEADER_BYTES

_lib = None


def available() -> bool:
    return os.path.exists(LIB_PATH)


def lib() -> ctypes.CDLL:
    """Load the HIP library; raises if it was not built (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise FileNotFoundError(f"{LIB_PATH} missing: run __graft_entry__.build() (make -C fluere_amd/csrc)")
    L = ctypes.CDLL(LIB_PATH)
    P, U64, I64, I, U32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int, ctypes.c_uint32
    sig = {
        "fluere_abi_version": (I, []),
        "fluere_open": (I, [ctypes.POINTER(Opts), ctypes.POINTER(P)]),
        "fluere_close": (I, [P]),
        "fluere_reset": (I, [P]),
        "fluere_pcap_index": (I64, [P, U64, P, U64]),
        "fluere_add_device_batch": (I, [P, P, U64, P, U64, ctypes.c_uint32, I, I]),
        "fluere_add_host_pcap": (I, [P, P, U64]),
        "fluere_add_pcap_file": (I, [P, ctypes.c_char_p]),
        "fluere_parse_batch": (I, [P, P, U64]),
        "fluere_run": (I, [P, ctypes.POINTER(Stats)]),
        "fluere_parse_aggregate": (I, [P]),
        "fluere_get_records": (I, [P, ctypes.POINTER(P), ctypes.POINTER(U64), ctypes.POINTER(U64)]),
        "fluere_records_free": (None, [P]),
        "fluere_write_csv": (I, [P, U64, ctypes.c_char_p]),
        "fluere_format_csv": (U64, [P, U64, P, U64]),
        "fluere_offline_file": (I, [ctypes.c_char_p, U64, I, ctypes.c_char_p, ctypes.POINTER(Stats)]),
        "fluere_synth_file_size": (U64, [ctypes.POINTER(SynthCfg)]),
        "fluere_synth_host": (I, [ctypes.POINTER(SynthCfg), P, U64]),
        "fluere_synth_range_bytes": (U64, [ctypes.POINTER(SynthCfg), U64, U64]),
        "fluere_synth_device": (I, [ctypes.POINTER(SynthCfg), U64, U64, P, P, P]),
        "fluere_set_index_base": (I, [P, U64]),
        "fluere_capacity": (U64, [P]),
        "fluere_total_packets": (U64, [P]),
        "fluere_last_kernel_ms": (ctypes.c_double, [P]),
        "fluere_last_hot_kernel": (ctypes.c_char_p, [P]),
        "fluere_last_pass_ms": (ctypes.c_double, [P]),
        "fluere_last_census": (I, [P, P, I]),
        "fluere_debug_dense_ids": (I, [P, P, U64, P]),
        "fluere_debug_raw": (I, [I, P, P, P, P, U64, P, P]),
        "fluere_live_open": (I, [ctypes.POINTER(Opts), ctypes.POINTER(P)]),
        "fluere_live_close": (I, [P]),
        "fluere_live_batch": (I, [P, P, U64, I, ctypes.POINTER(P), ctypes.POINTER(U64), ctypes.POINTER(U64),
                                  ctypes.POINTER(I)]),
        "fluere_live_batch_indexed": (I, [P, P, U64, P, U64, I, ctypes.POINTER(P), ctypes.POINTER(U64),
                                          ctypes.POINTER(U64), ctypes.POINTER(I)]),
        "fluere_live_finish": (I, [P, I, ctypes.POINTER(P), ctypes.POINTER(U64), ctypes.POINTER(U64)]),
        "fluere_shard_block_bytes": (U64, [U64, U64]),
        "fluere_export_device": (I, [P, P, ctypes.c_uint32, ctypes.c_uint32, U64, U64, ctypes.POINTER(U64),
                                     ctypes.POINTER(U64)]),
        "fluere_export_async": (I, [P, P, ctypes.c_uint32, ctypes.c_uint32, U64, U64, P]),
        "fluere_merge_gathered": (I, [P, P, ctypes.c_uint32, U64, U64, ctypes.POINTER(Stats)]),
        "fluere_merge_gathered_async": (I, [P, P, ctypes.c_uint32, U64, U64, P]),
        "fluere_merge_gathered_finish": (I, [P, ctypes.POINTER(Stats)]),
        "fluere_host_waits": (U64, [P]),
        "fluere_wire_bound": (U64, [U64, U64]),
        "fluere_wire_pack": (I, [P, P, U32, U64, U64, P, P]),
        "fluere_wire_unpack": (I, [P, P, U32, P, U64, U64, P]),
        "fluere_wire_pack_slots": (I, [P, P, U32, U64, U64, U64, P]),
        "fluere_wire_unpack_slots": (I, [P, P, U32, U64, U64, U64, P]),
        "fluere_sweep_pack": (I, [P, U32, P, P]),
        "fluere_sweep_load": (I, [P, P, U32, P]),
        "fluere_sweep_index": (I, [P, P, ctypes.POINTER(U64)]),
        "fluere_sweep_queries": (I, [P, U32, U32, P, P, P]),
        "fluere_sweep_answer": (I, [P, P, U64, P]),
        "fluere_sweep_points": (I, [P, P, P]),
        "fluere_sweep_chase": (I, [P, P, P, ctypes.POINTER(I)]),
        "fluere_sweep_seed_requests": (I, [P, U32, P, P, P]),
        "fluere_sweep_seeds": (I, [P, P, U64, P]),
        "fluere_sweep_finish": (I, [P, P, ctypes.POINTER(Stats)]),
        "fluere_get_record_order": (I, [P, P, U64]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def exported_symbols():
    """Names declared in include/fluere_gpu.h that the library must export."""
    hdr = os.path.join(os.path.dirname(_HERE), "include", "fluere_gpu.h")
    import re
    src = open(hdr).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|uint64_t|void|double)\s+(fluere_\w+)\s*\(", src, re.M)))


def check(rc: int, what: str) -> int:
    if rc != OK:
        raise FluereError(rc, what)
    return rc
