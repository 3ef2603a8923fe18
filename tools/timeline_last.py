"""Timeline of the last bench step from a rocprofv3 kernel trace CSV:
   python tools/timeline_last.py <run_kernel_trace.csv> [anchor-kernel-substring]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
anchor = sys.argv[2] if len(sys.argv) > 2 else "k_parse_agg"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
for alt in ("k_slow", "k_ex_meta"):  # (a pass without the hot kernel: slow-all starts with k_slow)
    if not idx:
        idx = [i for i, r in enumerate(rows) if alt in r["Kernel_Name"]]
s = idx[-1]
t0 = int(rows[s]["Start_Timestamp"])
prev = t0
tot_gap = 0
for r in rows[max(0, s - 2):]:
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if st - prev > 5_000_000:
        break
    n = r["Kernel_Name"]
    n = n[n.find("k_"):][:48] if "k_" in n else n[:60]
    gap = (st - prev) / 1e3
    if st > t0:
        tot_gap += max(0.0, gap)
    print(f"{(st - t0) / 1e3:8.1f} {(en - st) / 1e3:7.1f} gap {gap:6.1f}  {n}")
    prev = en
print(f"end {(prev - t0) / 1e3:.1f} us, gaps {tot_gap:.1f} us")
