#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run into profiles/<name>.md
(per-kernel calls / average / min / max / total, sorted by total), and, when the
``*_kernel_trace.csv`` sits next to the stats file, the median duration of the
live launches (longer than --live-us; launches that exit at once — iterations
enqueued past the termination, gated camera-side launches — are excluded) with
the VGPR / LDS / scratch figures of each kernel.

Input: the ``*_kernel_stats.csv`` of ``--output-format csv`` or the rocpd
``*_results.db`` (SQLite) that rocprofv3 writes by default on ROCm 7.
Usage: prof_summary.py <stats.csv|results.db> <out.md> [title] [--live-us 6]"""
import csv
import os
import sqlite3
import statistics
import sys


def kname(n):
    """Kernel symbol without its argument list ('(anonymous namespace)::' dropped first)."""
    return n.replace("(anonymous namespace)::", "").split("(")[0]


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


def live_rows(trace, live_us):
    per = {}
    for r in csv.DictReader(open(trace)):
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        k = per.setdefault(r["Kernel_Name"], dict(d=[], vgpr=r["VGPR_Count"], agpr=r["Accum_VGPR_Count"],
                                                  lds=r["LDS_Block_Size"], scratch=r["Scratch_Size"],
                                                  grid=int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1),
                                                  wg=r["Workgroup_Size_X"]))
        if d > live_us:
            k["d"].append(d)
    return per


def main(argv):
    live_us = 6.0
    if "--live-us" in argv:
        i = argv.index("--live-us")
        live_us = float(argv[i + 1])
        argv = argv[:i] + argv[i + 2:]
    src, out_md = argv[1], argv[2]
    title = argv[3] if len(argv) > 3 else "kernel stats"
    rows = rows_from_db(src) if src.endswith(".db") else rows_from_csv(src)
    rows.sort(key=lambda r: -r["tot"])
    total = sum(r["tot"] for r in rows) or 1.0
    with open(out_md, "w") as f:
        f.write(f"# {title}\n\nSource: `rocprofv3 --kernel-trace --stats` ({src.split('/')[-1]}).\n\n")
        f.write("| kernel | calls | avg us | min us | max us | total ms | % |\n|---|---|---|---|---|---|---|\n")
        for r in rows:
            name = kname(r["name"])
            f.write(f"| `{name}` | {r['calls']} | {r['avg'] / 1e3:.2f} | {r['mn'] / 1e3:.2f} | "
                    f"{r['mx'] / 1e3:.2f} | {r['tot'] / 1e6:.3f} | {100.0 * r['tot'] / total:.2f} |\n")
        trace = src.replace("_kernel_stats.csv", "_kernel_trace.csv")
        if trace != src and os.path.exists(trace):
            per = live_rows(trace, live_us)
            f.write(f"\nLive launches only (duration > {live_us:g} us; from {trace.split('/')[-1]}):\n\n")
            f.write("| kernel | live launches | median us | grid (WGs) | WG size | VGPR | AGPR | LDS B | scratch B |\n"
                    "|---|---|---|---|---|---|---|---|---|\n")
            order = sorted(per.items(), key=lambda kv: -sum(kv[1]["d"]))
            for name, k in order:
                if not k["d"] or name.startswith("__amd"):
                    continue
                f.write(f"| `{kname(name)}` | {len(k['d'])} | {statistics.median(k['d']):.2f} | {k['grid']} | "
                        f"{k['wg']} | {k['vgpr']} | {k['agpr']} | {k['lds']} | {k['scratch']} |\n")


if __name__ == "__main__":
    main(sys.argv)
