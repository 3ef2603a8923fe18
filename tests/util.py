"""Shared test helpers: golden fixtures and the SURVEY section 8c comparator."""
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def manifest():
    return json.load(open(os.path.join(GOLDEN, "manifest.json")))


def golden_pcap(name):
    return open(os.path.join(GOLDEN, name + ".pcap"), "rb").read()


def golden_csv(fname):
    return open(os.path.join(GOLDEN, fname)).read()


def split_csv(text, n_ended):
    lines = text.split("\n")
    assert lines[-1] == "", "CSV must end with the record terminator"
    header, rows = lines[0], lines[1:-1]
    return header, rows[:n_ended], sorted(rows[n_ended:])


def assert_csv_equal(got, got_ended, want, want_ended, what=""):
    """Header byte-equal; ended prefix equal in order; active suffix equal as a multiset
    (the reference emits active flows in HashMap order, offline_fluereflows.rs:182-184)."""
    gh, ge, ga = split_csv(got, got_ended)
    wh, we, wa = split_csv(want, want_ended)
    assert gh == wh, f"{what}: header differs"
    assert got_ended == want_ended, f"{what}: ended count {got_ended} != {want_ended}"
    assert ge == we, f"{what}: ended prefix differs\n got={ge[:5]}\nwant={we[:5]}"
    if ga != wa:
        gs, ws = set(ga), set(wa)
        raise AssertionError(f"{what}: active set differs ({len(ga)} vs {len(wa)} rows)\n"
                             f" only got={sorted(gs - ws)[:5]}\n only want={sorted(ws - gs)[:5]}")
