"""Print the last N dispatches of a rocprofv3 kernel trace (start offset, duration, name) — the
per-iteration launch sequence and the gaps between launches."""
import csv
import sys

path = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-n:]
t0 = int(rows[0]["Start_Timestamp"])
prev = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1000 if prev is not None else 0.0
    print(f"{(s - t0) / 1000:9.1f} gap {gap:5.1f} dur {(e - s) / 1000:7.1f}  {r['Kernel_Name'][:60]} grid={r['Grid_Size_X']}")
    prev = e
