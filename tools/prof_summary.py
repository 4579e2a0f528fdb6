#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run into profiles/<name>.md
(per-kernel calls / average / min / max / total, sorted by total).

Input: the ``*_kernel_stats.csv`` of ``--output-format csv`` or the rocpd
``*_results.db`` (SQLite) that rocprofv3 writes by default on ROCm 7."""
import csv
import sqlite3
import sys


def rows_from_csv(path):
    out = []
    for r in csv.DictReader(open(path)):
        out.append(dict(name=r["Name"], calls=int(r["Calls"]), avg=float(r["AverageNs"]), mn=float(r["MinNs"]),
                        mx=float(r["MaxNs"]), tot=float(r["TotalDurationNs"])))
    return out


def rows_from_db(path):
    db = sqlite3.connect(path)
    q = ("select name, count(*), avg(end - start), min(end - start), max(end - start), sum(end - start) "
         "from kernels group by name")
    return [dict(name=n, calls=c, avg=a, mn=lo, mx=hi, tot=t) for n, c, a, lo, hi, t in db.execute(q)]


def main(src, out_md, title):
    rows = rows_from_db(src) if src.endswith(".db") else rows_from_csv(src)
    rows.sort(key=lambda r: -r["tot"])
    total = sum(r["tot"] for r in rows) or 1.0
    with open(out_md, "w") as f:
        f.write(f"# {title}\n\nSource: `rocprofv3 --kernel-trace --stats` ({src.split('/')[-1]}).\n\n")
        f.write("| kernel | calls | avg us | min us | max us | total ms | % |\n|---|---|---|---|---|---|---|\n")
        for r in rows:
            name = r["name"].split("(")[0]
            f.write(f"| `{name}` | {r['calls']} | {r['avg'] / 1e3:.2f} | {r['mn'] / 1e3:.2f} | "
                    f"{r['mx'] / 1e3:.2f} | {r['tot'] / 1e6:.3f} | {100.0 * r['tot'] / total:.2f} |\n")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "kernel stats")
