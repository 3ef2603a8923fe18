"""C ABI checks that need no GPU: the library loads and exports every symbol
include/fluere_gpu.h declares; host-side egress (CSV) and ingress (pcap
index) agree with the oracle; the synthetic generator produces the captures
SURVEY section 8d specifies (checked through the oracle)."""
import ctypes
import os

import numpy as np
import pyoracle
import pytest
from util import golden_csv, golden_pcap, manifest

import fluere_amd
from fluere_amd import _lib
from fluere_amd._lib import RECORD_DTYPE


def test_library_loads_and_exports_all_symbols():
    L = _lib.lib()
    syms = _lib.exported_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(L, s), f"missing export {s}"
    assert L.fluere_abi_version() == 1


def test_cli_binary_built():
    assert os.access(_lib.CLI_PATH, os.X_OK)


def _rows_to_records(text):
    import ipaddress
    rows = text.splitlines()[1:]
    recs = np.zeros(len(rows), dtype=RECORD_DTYPE)
    for i, row in enumerate(rows):
        f = row.split(",")
        for k, name in ((0, "source"), (1, "destination")):
            a = ipaddress.ip_address(f[k])
            recs[i]["src_v6" if k == 0 else "dst_v6"] = 1 if a.version == 6 else 0
            recs[i][name][: len(a.packed)] = np.frombuffer(a.packed, np.uint8)
        (recs[i]["src_port"], recs[i]["dst_port"], recs[i]["prot"], recs[i]["d_pkts"], recs[i]["d_octets"],
         recs[i]["in_pkts"], recs[i]["out_pkts"], recs[i]["in_bytes"], recs[i]["out_bytes"], recs[i]["first"],
         recs[i]["last"], recs[i]["min_pkt"], recs[i]["max_pkt"], recs[i]["min_ttl"], recs[i]["max_ttl"]) = \
            [int(x) for x in f[2:17]]
        recs[i]["cnt"] = [int(x) for x in f[17:26]]
        recs[i]["tos"] = int(f[26])
    return recs


@pytest.mark.parametrize("name", sorted(manifest()))
def test_csv_writer_matches_golden(name):
    for run in manifest()[name]["runs"]:
        want = golden_csv(run["csv"])
        recs = _rows_to_records(want)
        assert fluere_amd.format_csv(recs) == want


def test_csv_file_writer_blocks(tmp_path):
    """fluere_write_csv formats blocks of rows on threads: the file equals the
    one-pass formatter's text (rows past 2^16, v4 and v6 mixed)."""
    rng = np.random.default_rng(0xC5F)
    n = 70_001
    recs = np.zeros(n, dtype=_lib.RECORD_DTYPE)
    raw = recs.view(np.uint8).reshape(n, -1)
    raw[:] = rng.integers(0, 256, raw.shape, dtype=np.uint8)
    recs["src_v6"] = rng.integers(0, 2, n)
    recs["dst_v6"] = rng.integers(0, 2, n)
    path = tmp_path / "w.csv"
    buf = np.ascontiguousarray(recs)
    assert _lib.lib().fluere_write_csv(buf.ctypes.data, n, str(path).encode()) == 0
    assert path.read_text() == fluere_amd.format_csv(buf)


def test_csv_writer_ipv6_display():
    recs = np.zeros(4, dtype=RECORD_DTYPE)
    cases = ["::", "::ffff:1.2.3.4", "1:0:0:1:0:0:0:1", "2001:db8:0:1:1:1:1:1"]
    import ipaddress
    for i, c in enumerate(cases):
        recs[i]["src_v6"] = recs[i]["dst_v6"] = 1
        recs[i]["source"] = np.frombuffer(ipaddress.IPv6Address(c).packed, np.uint8)
        recs[i]["destination"] = recs[i]["source"]
    rows = fluere_amd.format_csv(recs).splitlines()[1:]
    # Rust Ipv6Addr Display: first longest run (> 1) of zero groups compressed
    assert [r.split(",")[0] for r in rows] == ["::", "::ffff:1.2.3.4", "1:0:0:1::1", "2001:db8:0:1:1:1:1:1"]


@pytest.mark.parametrize("name", sorted(manifest()))
def test_pcap_index_matches_oracle(name):
    data = golden_pcap(name)
    buf = (ctypes.c_uint8 * len(data)).from_buffer_copy(data)
    n = _lib.lib().fluere_pcap_index(buf, len(data), None, 0)
    assert n == len(pyoracle.parse_batch(data)) == manifest()[name]["packets"]


def test_synth_c1_one_tuple():
    # BASELINE configs[0]: 10k x 64 B UDP, one 5-tuple -> one active row
    cfg = fluere_amd.synth_cfg(_lib.SYNTH_UDP64, 10_000, 1, 0xF10E0001, rev_pct=0)
    data = fluere_amd.synth_pcap(cfg)
    assert len(data) == 24 + 10_000 * 80
    r = pyoracle.offline(data)
    rows = r["csv"].splitlines()[1:]
    assert len(rows) == 1 and r["n_ended"] == 0
    f = rows[0].split(",")
    assert f[5:11] == ["10000", "500000", "0", "10000", "0", "500000"]
    assert f[13:15] == ["50", "50"]
    assert int(f[12]) - int(f[11]) == 9999


def test_synth_imix_closers_and_flow_count():
    cfg = fluere_amd.synth_cfg(_lib.SYNTH_IMIX, 20_000, 500, 0xF10E0003)
    r = pyoracle.offline(fluere_amd.synth_pcap(cfg))
    assert r["n"] == 500  # every flow opened in [0, F) and never re-created
    assert 0 < r["n_ended"] < 500  # FIN/RST closers end in the tail region


def test_synth_vlan_header_only_and_mac_keyed():
    v = fluere_amd.synth_cfg(_lib.SYNTH_VLAN64, 5_000, 50, 0xF10E0005)
    assert pyoracle.offline(fluere_amd.synth_pcap(v), use_mac=True)["n"] == 0
    m = fluere_amd.synth_cfg(_lib.SYNTH_MAC64, 5_000, 50, 0xF10E0005)
    assert pyoracle.offline(fluere_amd.synth_pcap(m), use_mac=True)["n"] == 50


def test_synth_slow_classes():
    """FLUERE_SYNTH_SLOW: every packet is valid for the reference parser and
    lands in a general-parser class (IPv6, VXLAN inner IPv4, IPv4 options)."""
    cfg = fluere_amd.synth_cfg(_lib.SYNTH_SLOW, 20_000, 400, 0x51077)
    data = fluere_amd.synth_pcap(cfg)
    r = pyoracle.offline(data)
    assert r["valid"] == 20_000 and r["n"] == 400 and 0 < r["n_ended"] < 400
    rows = [x.split(",") for x in r["csv"].splitlines()[1:]]
    v6 = sum(x[0].startswith("fd00::") for x in rows)
    assert 100 < v6 < 300  # half the flows
    meta = pyoracle.parse_batch(data)
    # VXLAN flows: the outer tunnel endpoints never appear as a key
    assert not any(bytes(m["key_src"][:4]) == bytes([192, 168, 0, 1]) for m in meta[:2000])
    # no packet of this kind fits the hot parser's shape (Ethernet/IPv4 ihl 5/TCP|UDP, not VXLAN)
    import struct
    off, n_hot = 24, 0
    while off + 16 <= len(data):
        incl = struct.unpack_from("<I", data, off + 8)[0]
        f = data[off + 16: off + 16 + incl]
        et, ihl, proto = f[12:14], f[14] & 15, f[23]
        vx = proto == 17 and f[42:50] == bytes([8, 0, 0, 0, 0, 0, 0x64, 0])
        n_hot += et == b"\x08\x00" and ihl == 5 and proto in (6, 17) and not vx
        off += 16 + incl
    assert n_hot == 0


def test_device_batches_split_below_4gib(monkeypatch):
    """bench.py's C4 shard (12.5M IMIX packets, ~4.3 GiB) is attached as
    consecutive batches that each stay below 4 GiB (u32 record offsets) and
    together cover the shard exactly (host-side split; generation stubbed)."""
    from fluere_amd import offline
    cfg = fluere_amd.synth_cfg(_lib.SYNTH_IMIX, 12_500_000, 125_000, 0xF10E0004)
    L = _lib.lib()
    total = L.fluere_synth_range_bytes(ctypes.byref(cfg), 0, 12_500_000)
    assert total >= 1 << 32
    calls = []

    def fake(cfg_, first, n, stream=None):
        nb = L.fluere_synth_range_bytes(ctypes.byref(cfg_), first, n)
        calls.append((first, n, nb))
        return None, None, nb

    monkeypatch.setattr(offline, "synth_device", fake)
    out = offline.synth_device_batches(cfg, 0, 12_500_000)
    assert len(out) >= 2
    assert all(nb < 1 << 32 for _, _, nb, _ in out)
    assert sum(n for _, _, _, n in out) == 12_500_000
    assert [c[0] for c in calls] == [sum(c[1] for c in calls[:i]) for i in range(len(calls))]
    assert sum(c[2] for c in calls) == total
