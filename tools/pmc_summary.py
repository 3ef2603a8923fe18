"""Summarise rocprofv3 outputs written by tools/prof.sh.

  python tools/pmc_summary.py gpurun_out/prof_<tag> [kernel-substring]

Prints per-kernel average duration (kernel trace) and, for each counter pass,
the per-launch counter average for the kernel.  HBM bytes follow
MI355X_MICROARCH.md: FETCH_SIZE is in KB and reports half of the bytes on
gfx950 (x2); WRITE_SIZE in KB.  Writes <dir>/summary.json.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def _rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def kernel_stats(d):
    rows = _rows(os.path.join(d, "trace", "**", "*kernel_stats.csv"))
    return {r["Name"]: {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                        "total_us": float(r["TotalDurationNs"]) / 1e3, "pct": float(r["Percentage"])}
            for r in rows}


def _match(name, kern):
    """kern: a kernel name prefix inside the (demangled) name, matched up to a
    template/argument list -- 'k_parse_agg' matches 'k_parse_agg<0, false>(...)'
    but not 'k_parse_agg_slow(...)'."""
    i = name.find(kern)
    return i >= 0 and (i + len(kern) == len(name) or name[i + len(kern)] in "<(")


def counters(d, sub, kern):
    rows = _rows(os.path.join(d, sub, "**", "*counter_collection.csv"))
    acc = defaultdict(list)
    for r in rows:
        if _match(r["Kernel_Name"], kern):
            # one row per (dispatch, counter); sum over dimension instances happens in rocprofv3
            acc[(r["Counter_Name"], r["Dispatch_Id"])].append(float(r["Counter_Value"]))
    per = defaultdict(list)
    for (name, _), v in acc.items():
        per[name].append(sum(v))
    return {k: sum(v) / len(v) for k, v in per.items()}


def main():
    d = sys.argv[1]
    out = {"kernels": kernel_stats(d), "passes": {}}
    # default: the hot kernel of the run (k_parse_spill for many-flow captures)
    hot = {k: sum(v["total_us"] for n, v in out["kernels"].items() if _match(n, k)) for k in ("k_parse_agg", "k_parse_spill", "k_slow")}
    kern = sys.argv[2] if len(sys.argv) > 2 else max(hot, key=hot.get)
    for sub in sorted(os.listdir(d)):
        if os.path.isdir(os.path.join(d, sub)) and sub != "trace":
            c = counters(d, sub, kern)
            if c:
                out["passes"][sub] = c
    out["kernel"] = kern
    f = out["passes"].get("fetch", {}).get("FETCH_SIZE")
    w = out["passes"].get("write", {}).get("WRITE_SIZE")
    if f is not None:
        out["hbm_read_bytes_per_launch"] = f * 1024 * 2
    if w is not None:
        out["hbm_write_bytes_per_launch"] = w * 1024
    if f is not None and w is not None:
        out["hbm_bytes_per_launch"] = out["hbm_read_bytes_per_launch"] + out["hbm_write_bytes_per_launch"]
    json.dump(out, open(os.path.join(d, "summary.json"), "w"), indent=1)
    for k, v in sorted(out["kernels"].items(), key=lambda kv: -kv[1]["total_us"])[:12]:
        print(f"{v['avg_us']:10.2f} us avg {v['calls']:5d} calls {v['pct']:6.2f}%  {k[:90]}")
    for p, c in out["passes"].items():
        print(p, {k: round(v, 1) for k, v in c.items()})
    for k in ("hbm_read_bytes_per_launch", "hbm_write_bytes_per_launch", "hbm_bytes_per_launch"):
        if k in out:
            print(k, int(out[k]))


if __name__ == "__main__":
    main()
