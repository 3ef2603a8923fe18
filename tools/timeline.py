"""Print the kernel timeline of the last few bench steps from a rocprofv3
--kernel-trace CSV (gaps and durations in microseconds).
  python tools/timeline.py gpurun_out/<dir>/run_kernel_trace.csv [n_rows]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 24
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-n:]
t0 = int(rows[0]["Start_Timestamp"])
prev = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    print(f"{(s - t0) / 1e3:9.2f}  gap {gap:7.2f}  dur {(e - s) / 1e3:8.2f}  {r['Kernel_Name'][:80]}")
    prev = e
