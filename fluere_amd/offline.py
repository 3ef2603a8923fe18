"""Host-side mirror of fluere's offline mode over the MI355X C ABI.

Reference seams mirrored here (SkuldNorniern/fluere):
  * ``fluereflow_fileparse(args)``  <- src/net/offline_fluereflows.rs:26-196
  * ``parse_keys`` / ``parse_fluereflow`` (batched) <- src/net/parser/keys.rs:98,
    src/net/parser/fluereflows.rs:30
  * ``fluere_exporter(records, path)`` <- src/utils/fluere_csv_exporter.rs:5-81
  * ``FluereRecord.to_vec()`` <- fluereflow/src/types/fluereflow.rs:122-152
"""
from __future__ import annotations

import ctypes
import dataclasses
import ipaddress
import os
from typing import Optional

import numpy as np

from . import _lib
from ._lib import PKT_META_DTYPE, RECORD_DTYPE, FluereError, Opts, Stats, SynthCfg, check


class FlowContext:
    """One device context: attached packet batches + the flow dictionary."""

    def __init__(self, timeout_ms: int = 600000, use_mac: bool = False, max_flows: int = 0, device: int = 0,
                 stream: Optional[int] = None):
        L = _lib.lib()
        self._L = L
        o = Opts(device=device, stream=stream or None, timeout_ms=timeout_ms, use_mac=1 if use_mac else 0,
                 max_flows=max_flows)
        h = ctypes.c_void_p()
        check(L.fluere_open(ctypes.byref(o), ctypes.byref(h)), "fluere_open")
        self._h = h
        self.stream = stream  # HIP stream handle the context runs on (None: its own)
        self.timeout_ms = int(timeout_ms)
        self.use_mac = bool(use_mac)
        self.index_base = 0  # global index of the first packet (dist.set_index_base)
        self._keep = []  # device buffers the batches point into
        self.n_packets = 0

    def close(self):
        if getattr(self, "_h", None):
            self._L.fluere_close(self._h)
            self._h = None
        self._keep = []

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def reset(self):
        check(self._L.fluere_reset(self._h), "fluere_reset")
        self._keep = []
        self.n_packets = 0

    def add_host_pcap(self, data: bytes):
        buf = (ctypes.c_uint8 * len(data)).from_buffer_copy(data)
        check(self._L.fluere_add_host_pcap(self._h, buf, len(data)), "fluere_add_host_pcap")
        self.n_packets = int(self._L.fluere_total_packets(self._h))

    def add_pcap_file(self, path: str):
        """Stream a capture file to the device (pinned chunks, host-side index)."""
        check(self._L.fluere_add_pcap_file(self._h, os.fsencode(path)), "fluere_add_pcap_file")
        self.n_packets = int(self._L.fluere_total_packets(self._h))

    def add_device_batch(self, d_bytes, nbytes: int, d_offsets, n: int, snaplen: int = 65535, swapped=False,
                         nsec=False, keep=()):
        """Attach device-resident records (pointers or torch tensors)."""
        pb = d_bytes.data_ptr() if hasattr(d_bytes, "data_ptr") else int(d_bytes)
        po = d_offsets.data_ptr() if hasattr(d_offsets, "data_ptr") else int(d_offsets)
        check(self._L.fluere_add_device_batch(self._h, pb, nbytes, po, n, snaplen, int(swapped), int(nsec)),
              "fluere_add_device_batch")
        self._keep.extend([d_bytes, d_offsets, *keep])
        self.n_packets += n

    def run(self) -> dict:
        st = Stats()
        check(self._L.fluere_run(self._h, ctypes.byref(st)), "fluere_run")
        return st.as_dict()

    def parse_aggregate(self):
        check(self._L.fluere_parse_aggregate(self._h), "fluere_parse_aggregate")

    def host_waits(self) -> int:
        """Blocking host waits on the context's stream so far (fluere_host_waits)."""
        return int(self._L.fluere_host_waits(self._h))

    def last_kernel_ms(self) -> float:
        """HIP-event time of the last k_parse_agg launch (the roofline kernel)."""
        return float(self._L.fluere_last_kernel_ms(self._h))

    def last_hot_kernel(self) -> str:
        """Name of the last pass's hot kernel (k_parse_agg or k_parse_spill)."""
        return self._L.fluere_last_hot_kernel(self._h).decode()

    def last_census(self) -> dict:
        """The census of the capture attached last (fluere_last_census)."""
        v = np.zeros(10, dtype=np.uint64)
        runs = self._L.fluere_last_census(self._h, v.ctypes.data, 10)
        keys = ("sampled", "keyed", "slow", "tcp", "distinct", "once", "twice", "tmin", "tmax", "flows_est")
        return {"runs": int(runs), **{k: int(x) for k, x in zip(keys, v)}}

    def last_pass_ms(self) -> float:
        """HIP-event time of the whole last parse+key+aggregate pass."""
        return float(self._L.fluere_last_pass_ms(self._h))

    def records(self):
        """(records ndarray[RECORD_DTYPE], n_ended): ended prefix first, then active."""
        p = ctypes.c_void_p()
        n = ctypes.c_uint64()
        ne = ctypes.c_uint64()
        check(self._L.fluere_get_records(self._h, ctypes.byref(p), ctypes.byref(n), ctypes.byref(ne)),
              "fluere_get_records")
        try:
            raw = ctypes.string_at(p, n.value * RECORD_DTYPE.itemsize) if n.value else b""
        finally:
            self._L.fluere_records_free(p)
        return np.frombuffer(raw, dtype=RECORD_DTYPE).copy(), ne.value

    def record_order(self, n: int) -> np.ndarray:
        """The two order words of each record of records() (n of them; zero
        except after the sharded sweep composition, dist.py)."""
        out = np.zeros((n, 2), dtype=np.uint64)
        check(self._L.fluere_get_record_order(self._h, out.ctypes.data_as(ctypes.c_void_p) if n else None, n),
              "fluere_get_record_order")
        return out

    def parse_batch(self, general_only: bool = False) -> np.ndarray:
        """Per-packet parse_keys / parse_fluereflow view (PKT_META_DTYPE)."""
        import torch
        n = self.n_packets
        out = torch.empty(max(n, 1) * PKT_META_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
        old = os.environ.get("FLUERE_PARSE_MODE")
        os.environ["FLUERE_PARSE_MODE"] = "1" if general_only else "0"
        try:
            check(self._L.fluere_parse_batch(self._h, out.data_ptr(), n), "fluere_parse_batch")
        finally:
            if old is None:
                os.environ.pop("FLUERE_PARSE_MODE", None)
            else:
                os.environ["FLUERE_PARSE_MODE"] = old
        return np.frombuffer(out[: n * PKT_META_DTYPE.itemsize].cpu().numpy().tobytes(), dtype=PKT_META_DTYPE)


def format_csv(recs: np.ndarray) -> str:
    """fluere_exporter's CSV text for records (src/utils/fluere_csv_exporter.rs:5-81)."""
    L = _lib.lib()
    recs = np.ascontiguousarray(recs, dtype=RECORD_DTYPE)
    ptr = recs.ctypes.data if len(recs) else None
    need = L.fluere_format_csv(ptr, len(recs), None, 0)
    buf = ctypes.create_string_buffer(need)
    L.fluere_format_csv(ptr, len(recs), buf, need)
    return buf.raw[:need].decode()


def fluere_exporter(recs: np.ndarray, path: str):
    L = _lib.lib()
    recs = np.ascontiguousarray(recs, dtype=RECORD_DTYPE)
    check(L.fluere_write_csv(recs.ctypes.data if len(recs) else None, len(recs), path.encode()), "fluere_write_csv")


@dataclasses.dataclass
class Files:
    file: Optional[str] = None
    csv: Optional[str] = "output"


@dataclasses.dataclass
class Parameters:
    use_mac: Optional[bool] = False
    timeout: Optional[int] = 600000


@dataclasses.dataclass
class Args:
    """src/types/argument.rs (the fields the offline mode reads)."""
    files: Files = dataclasses.field(default_factory=Files)
    parameters: Parameters = dataclasses.field(default_factory=Parameters)


def fluereflow_fileparse(args: Args, out_dir: str = "./output") -> dict:
    """The offline mode: pcap -> ./output/<stem>_converted.csv (offline_fluereflows.rs:26-196)."""
    if args.files.file is None:
        raise ValueError("pcap file path should be provided")
    L = _lib.lib()
    st = Stats()
    rc = L.fluere_offline_file(args.files.file.encode(), int(args.parameters.timeout), int(bool(args.parameters.use_mac)),
                               out_dir.encode(), ctypes.byref(st))
    check(rc, "fluere_offline_file")
    return st.as_dict()


@dataclasses.dataclass
class FluereRecord:
    """fluereflow::FluereRecord (fluereflow/src/types/fluereflow.rs:31-60)."""
    source: object
    destination: object
    d_pkts: int
    d_octets: int
    first: int
    last: int
    src_port: int
    dst_port: int
    min_pkt: int
    max_pkt: int
    min_ttl: int
    max_ttl: int
    in_pkts: int
    out_pkts: int
    in_bytes: int
    out_bytes: int
    fin_cnt: int
    syn_cnt: int
    rst_cnt: int
    psh_cnt: int
    ack_cnt: int
    urg_cnt: int
    ece_cnt: int
    cwr_cnt: int
    ns_cnt: int
    prot: int
    tos: int

    @staticmethod
    def from_row(r) -> "FluereRecord":
        def ip(v6, b):
            return ipaddress.IPv6Address(bytes(b)) if v6 else ipaddress.IPv4Address(bytes(b[:4]))
        c = [int(x) for x in r["cnt"]]
        return FluereRecord(ip(r["src_v6"], r["source"]), ip(r["dst_v6"], r["destination"]), int(r["d_pkts"]),
                            int(r["d_octets"]), int(r["first"]), int(r["last"]), int(r["src_port"]),
                            int(r["dst_port"]), int(r["min_pkt"]), int(r["max_pkt"]), int(r["min_ttl"]),
                            int(r["max_ttl"]), int(r["in_pkts"]), int(r["out_pkts"]), int(r["in_bytes"]),
                            int(r["out_bytes"]), *c, int(r["prot"]), int(r["tos"]))

    def to_vec(self):
        """fluereflow.rs:122-152 (the order the Lua plugin API sees)."""
        return [str(getattr(self, f.name)) for f in dataclasses.fields(self)]


def synth_cfg(kind: int, n_packets: int, n_flows: int, seed: int, rev_pct: int = 30) -> SynthCfg:
    return SynthCfg(seed=seed, n_packets=n_packets, n_flows=n_flows, kind=kind, rev_pct=rev_pct)


def synth_pcap(cfg: SynthCfg) -> bytes:
    L = _lib.lib()
    n = L.fluere_synth_file_size(ctypes.byref(cfg))
    buf = (ctypes.c_uint8 * n)()
    check(L.fluere_synth_host(ctypes.byref(cfg), buf, n), "fluere_synth_host")
    return bytes(buf)


def synth_device(cfg: SynthCfg, first: int, n: int, stream: Optional[int] = None):
    """Generate packets [first, first+n) directly in HBM -> (bytes, offsets, nbytes) torch tensors."""
    import torch
    L = _lib.lib()
    nbytes = L.fluere_synth_range_bytes(ctypes.byref(cfg), first, n)
    b = torch.empty(nbytes + 256, dtype=torch.uint8, device="cuda")
    b[nbytes:].zero_()
    o = torch.empty(max(n, 1), dtype=torch.int32, device="cuda")
    if stream is None:
        stream = torch.cuda.current_stream().cuda_stream
    check(L.fluere_synth_device(ctypes.byref(cfg), first, n, b.data_ptr(), o.data_ptr(), stream),
          "fluere_synth_device")
    return b, o, nbytes


def synth_device_batches(cfg: SynthCfg, first: int, n: int, max_bytes: int = (1 << 32) - (1 << 20),
                         stream: Optional[int] = None):
    """Packets [first, first+n) generated in HBM as consecutive batches of at
    most max_bytes each (a batch's record offsets are u32, so one batch stays
    below 4 GiB; IMIX shards of C4 are larger) -> [(bytes, offsets, nbytes, n_i)]."""
    L = _lib.lib()
    if max_bytes >= 1 << 32:
        raise ValueError("a batch holds less than 4 GiB")
    out, p, end = [], first, first + n
    while p < end or not out:
        m = end - p
        while m > 1 and L.fluere_synth_range_bytes(ctypes.byref(cfg), p, m) > max_bytes:
            m = (m + 1) // 2
        b, o, nb = synth_device(cfg, p, m, stream)
        out.append((b, o, nb, m))
        p += m
    return out
