#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run into profiles/<name>.md
(per-kernel calls / average / total, sorted by total)."""
import csv
import sys


def main(stats_csv, out_md, title):
    rows = list(csv.DictReader(open(stats_csv)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    with open(out_md, "w") as f:
        f.write(f"# {title}\n\nSource: `rocprofv3 --kernel-trace --stats` ({stats_csv.split('/')[-1]}).\n\n")
        f.write("| kernel | calls | avg us | min us | max us | total ms | % |\n|---|---|---|---|---|---|---|\n")
        for r in rows:
            name = r["Name"].split("(")[0]
            f.write(f"| `{name}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.2f} | {float(r['MinNs'])/1e3:.2f} | "
                    f"{float(r['MaxNs'])/1e3:.2f} | {float(r['TotalDurationNs'])/1e6:.3f} | {float(r['Percentage']):.2f} |\n")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "kernel stats")
