"""Host-side mirror of fluere's `live` mode over the MI355X C ABI.

Reference seams mirrored here (SkuldNorniern/fluere):
  * ``packet_capture(args)`` / ``online_packet_capture``  <- src/net/live_fluereflow.rs:48,67-436
  * the plugin hand-off ``PluginManager::process_flow_data(FluereRecord)``
    <- fluere-plugin/src/lib.rs:300-303 (a plugin here is any object with
    ``process_data(list_of_str)``, called with ``FluereRecord.to_vec()`` like
    the Lua ``process_data`` of lib.rs:228-276)

The capture source is a ring of packet batches: each batch is the records a
capture delivered since the previous call, as a classic pcap image.  libpcap
and live devices are not part of this path; the
replay source below cuts a capture file into batches at interval boundaries
of the packets' own timestamps, so a run is deterministic.
"""
from __future__ import annotations

import ctypes
import os
import struct
from typing import Iterable, Iterator, Optional, Tuple

import numpy as np

from . import _lib
from ._lib import RECORD_DTYPE, Opts, check
from .offline import FluereRecord, fluere_exporter


class LiveSession:
    """fluere_live_*: flows stay open across batches."""

    def __init__(self, timeout_ms: int = 600000, use_mac: bool = False, max_flows: int = 1 << 20, device: int = 0):
        L = _lib.lib()
        self._L = L
        o = Opts(device=device, stream=None, timeout_ms=timeout_ms, use_mac=1 if use_mac else 0, max_flows=max_flows)
        h = ctypes.c_void_p()
        check(L.fluere_live_open(ctypes.byref(o), ctypes.byref(h)), "fluere_live_open")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._L.fluere_live_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def _take(p, n):
        try:
            if not n.value:
                return np.zeros(0, dtype=RECORD_DTYPE)
            raw = ctypes.string_at(p, n.value * RECORD_DTYPE.itemsize)
            return np.frombuffer(raw, dtype=RECORD_DTYPE).copy()
        finally:
            _lib.lib().fluere_records_free(p)

    def batch(self, pcap: bytes, export: bool, offsets=None):
        """One batch; (records, n_ordered) when the interval export ran, else
        None.  offsets (optional, uint64): each record's header offset in the
        image, as the capture side delivered them (fluere_live_batch_indexed:
        no host walk over the headers)."""
        if isinstance(pcap, bytes):  # the bytes object's own buffer (no host copy)
            buf = ctypes.cast(ctypes.c_char_p(pcap), ctypes.POINTER(ctypes.c_uint8))
        else:
            buf = (ctypes.c_uint8 * max(len(pcap), 1)).from_buffer_copy(pcap)
        p, n, no, ex = ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()
        if offsets is not None:
            offs = np.ascontiguousarray(offsets, dtype=np.uint64)
            check(self._L.fluere_live_batch_indexed(self._h, buf, len(pcap), offs.ctypes.data_as(ctypes.c_void_p),
                                                    len(offs), 1 if export else 0, ctypes.byref(p), ctypes.byref(n),
                                                    ctypes.byref(no), ctypes.byref(ex)), "fluere_live_batch_indexed")
        else:
            check(self._L.fluere_live_batch(self._h, buf, len(pcap), 1 if export else 0, ctypes.byref(p),
                                            ctypes.byref(n), ctypes.byref(no), ctypes.byref(ex)), "fluere_live_batch")
        recs = self._take(p, n) if p.value else None
        return (recs, no.value) if ex.value else None

    def finish(self, duration_end: bool):
        """The duration scan (when the capture duration was reached) and the
        flush of every active flow: the last export (records, n_ordered)."""
        p, n, no = ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_uint64()
        check(self._L.fluere_live_finish(self._h, 1 if duration_end else 0, ctypes.byref(p), ctypes.byref(n),
                                         ctypes.byref(no)), "fluere_live_finish")
        return self._take(p, n), no.value


def pcap_records(data: bytes) -> Iterator[Tuple[int, int, int]]:
    """(offset, length incl. the 16-byte header, timestamp us) of every record
    of a classic pcap image (libpcap offline: stop at the first bad record)."""
    if len(data) < 24:
        return
    magic = struct.unpack_from("<I", data)[0]
    if magic in (0xa1b2c3d4, 0xa1b23c4d):
        e = "<"
    elif magic in (0xd4c3b2a1, 0x4d3cb2a1):
        e = ">"
    else:
        raise ValueError("not a classic pcap image")
    nsec = magic in (0xa1b23c4d, 0x4d3cb2a1)
    off = 24
    while off + 16 <= len(data):
        sec, frac, incl, _ = struct.unpack_from(e + "IIII", data, off)
        if incl > 262144 or off + 16 + incl > len(data):
            return
        yield off, 16 + incl, sec * 1_000_000 + (frac // 1000 if nsec else frac)
        off += 16 + incl


def _batch_offsets(cur):
    """Header offsets of the records of one batch image (24-byte file header first)."""
    lens = np.fromiter((len(x) for x in cur), dtype=np.uint64, count=len(cur))
    return 24 + np.concatenate([np.zeros(1, np.uint64), np.cumsum(lens)[:-1]]).astype(np.uint64)


def replay_batches(data: bytes, interval_ms: int, batch_packets: int = 0) -> Iterator[Tuple[bytes, bool, np.ndarray]]:
    """A capture file as the batches a ring would deliver: a batch ends with
    the packet whose own clock crosses the next interval boundary (its export
    flag set), or every batch_packets packets without an export in between.
    Yields (classic pcap image, export, record header offsets)."""
    hdr = data[:24]
    cur, start, n = [], None, 0
    for off, ln, t in pcap_records(data):
        if start is None:
            start = t
        cur.append(data[off:off + ln])
        n += 1
        # the interval check follows the packet (live_fluereflow.rs:303-306):
        # the crossing packet belongs to the interval it closes
        if interval_ms and t - start >= interval_ms * 1000:
            yield hdr + b"".join(cur), True, _batch_offsets(cur)
            cur, start, n = [], t, 0
        elif batch_packets and n >= batch_packets:
            yield hdr + b"".join(cur), False, _batch_offsets(cur)
            cur, n = [], 0
    if cur:
        yield hdr + b"".join(cur), False, _batch_offsets(cur)


def packet_capture(args, batches: Iterable[Tuple[bytes, bool]], out_dir: str = "./output", plugins=(),
                   duration_end: bool = False, max_flows: int = 1 << 20):
    """The live mode over a batch source (live_fluereflow.rs:67-436): every
    export writes one CSV file <out_dir>/<csv>_<k>.csv (the reference names
    it by wall time, cur_time_file), and every exported record is handed to
    the plugins in export order.  Returns the list of (path, records,
    n_ordered)."""
    os.makedirs(out_dir, exist_ok=True)
    csv = args.files.csv or "output"
    exports = []

    def write(recs, n_ordered):
        path = os.path.join(out_dir, f"{csv}_{len(exports)}.csv")
        fluere_exporter(recs, path)
        for r in recs:
            rec = FluereRecord.from_row(r)
            for p in plugins:
                p.process_data(rec.to_vec())
        exports.append((path, recs, n_ordered))

    with LiveSession(int(args.parameters.timeout), bool(args.parameters.use_mac), max_flows) as s:
        for item in batches:  # (pcap, export[, record offsets])
            got = s.batch(*item)
            if got is not None:
                write(*got)
        write(*s.finish(duration_end))
    return exports
