"""The oracle (C restatement of the reference CPU path) pinned against the
reference's own byte fixture and the committed goldens.  CPU only."""
import pyoracle
import pytest
from util import GOLDEN, assert_csv_equal, golden_csv, golden_pcap, manifest


def test_known_answer_reference_frame():
    # src/net/parser/ipv4.rs:74-106 frame; expected row derived from the
    # reference source, not from the oracle
    r = pyoracle.offline(golden_pcap("ref_ipv4_frame"))
    assert r["csv"] == golden_csv("ref_ipv4_frame.expected.csv")
    assert r["n_ended"] == 0 and r["packets"] == 1


def test_reference_frame_fields():
    # ipv4.rs:108-122 / udp.rs:86-89 assertions on the same bytes
    m = pyoracle.parse_batch(golden_pcap("ref_ipv4_frame"))[0]
    assert m["k_status"] == 0 and m["f_status"] == 0
    assert bytes(m["key_src"][:4]) == bytes([192, 168, 50, 241])
    assert bytes(m["key_dst"][:4]) == bytes([1, 209, 175, 116])
    assert m["key_proto"] == 17 and m["key_sport"] == 41641 and m["key_dport"] == 41641
    assert m["rec_pkt"] == 540 and m["rec_ttl"] == 128 and m["doctets"] == 540


@pytest.mark.parametrize("name", sorted(manifest()))
def test_oracle_matches_committed_golden(name):
    data = golden_pcap(name)
    for run in manifest()[name]["runs"]:
        r = pyoracle.offline(data, run["timeout_ms"], run["use_mac"])
        assert_csv_equal(r["csv"], r["n_ended"], golden_csv(run["csv"]), run["n_ended"], name)


def test_edge_semantics_spot_checks():
    m = manifest()
    # -t 0: every created flow expires in its own iteration (offline_fluereflows.rs:161-175)
    r = [x for x in m["edge_udp_bidir"]["runs"] if x["timeout_ms"] == 0][0]
    assert r["n_ended"] == r["records"] == 4
    # stale expiry entry evicts the re-opened TCP flow
    r = [x for x in m["edge_expiry"]["runs"] if x["timeout_ms"] == 1][0]
    rows = golden_csv(r["csv"]).splitlines()[1:]
    assert rows[2].startswith("10.0.0.1,10.0.0.2,3,4,6,2,80,0,2,0,80,1700000000000950,1700000000001600")
    # VLAN-tagged frames with a 10.x source are dropped by the misparse
    assert all(x["records"] == 0 for x in m["edge_vlan_drop"]["runs"])
    # 8-byte ICMP echo dropped, 9-byte kept (keys.rs:182-184)
    rows = golden_csv("edge_empty_payload.t600000.csv").splitlines()[1:]
    assert len(rows) == 2 and any(",1,1,29," in x for x in rows)


# ---- the reference's unit tests of the raw fallback (tests/raw_vectors.py)
import raw_vectors as RV  # noqa: E402


@pytest.mark.parametrize("vec", RV.VECTORS, ids=[v[0] for v in RV.VECTORS])
def test_reference_raw_vector(vec):
    name, where, fn, data, arg, check = vec
    check(pyoracle.raw_call(fn, data, arg))


@pytest.mark.parametrize("data,size,has", RV.ANALYZE_STRUCTURE)
def test_reference_analyze_packet_structure(data, size, has):
    # ethertypes/mod.rs:321-346, and the payload start parse_custom_protocol takes from it
    assert pyoracle.analyze_structure(data) == (size, has)
    h = pyoracle.raw_call(RV.PARSE_ETHERTYPE, data, 0x3601)
    assert h["some"] and h["payload"] == (data[size:] if has and len(data) > size else None)


@pytest.mark.parametrize("name", ["edge_pcapng", "edge_pcapng_swapped"])
def test_pcapng_reads_like_libpcap(name):
    """The oracle's pcapng reader against make_fixtures.pcapng_expected(): the
    classic records libpcap's conversion (microseconds, per-interface
    resolution and offset, SPB without time) yields for the same blocks."""
    import make_fixtures as mf
    a = pyoracle.offline(golden_pcap(name))
    b = pyoracle.offline(mf.pcapng_expected())
    assert a["packets"] == b["packets"] == 8
    assert a["csv"] == b["csv"] and a["n_ended"] == b["n_ended"]
