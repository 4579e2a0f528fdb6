#!/usr/bin/env python3
"""Per-kernel SQ stall summary from one rocprofv3 --pmc pass of SQ counters (csv output).

usage: sq_summary.py counter_collection.csv "title" [out.md]

Counters (one pass, <= 8 SQ counters): SQ_WAVES, SQ_WAVE_CYCLES, SQ_WAIT_ANY, SQ_WAIT_INST_ANY,
SQ_ACTIVE_INST_ANY, SQ_ACTIVE_INST_VALU, SQ_INSTS_VALU, SQ_IFETCH. Reported per kernel as averages per dispatch
and as fractions of the wave cycles: waiting on anything (SQ_WAIT_ANY), waiting for an instruction to issue
(SQ_WAIT_INST_ANY), issuing any instruction (SQ_ACTIVE_INST_ANY) and issuing VALU (SQ_ACTIVE_INST_VALU).
"""
import csv
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    n = name.split("(")[0].replace("void ", "").replace("miba::", "")
    return n


def main():
    path, title = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else None
    agg = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    rows = []
    for k, d in agg.items():
        if k.startswith("__amd"):
            continue
        avg = {n: sum(v) / len(v) for n, v in d.items()}
        wc = avg.get("SQ_WAVE_CYCLES", 0.0)
        if wc <= 0:
            continue
        n = len(next(iter(d.values())))
        rows.append((wc, k, n, avg))
    rows.sort(reverse=True)
    lines = [f"# SQ stall summary — {title}", "",
             "Fractions of the kernel's wave cycles (SQ_WAVE_CYCLES, summed over its waves): waiting on anything "
             "(SQ_WAIT_ANY), waiting to issue (SQ_WAIT_INST_ANY), issuing any instruction (SQ_ACTIVE_INST_ANY), "
             "issuing VALU (SQ_ACTIVE_INST_VALU). Averages per dispatch.", "",
             "| kernel | dispatches | waves | wave cycles | wait any | wait inst | active any | active VALU |",
             "|---|---|---|---|---|---|---|---|"]
    for wc, k, n, a in rows:
        f = lambda c: f"{100.0 * a.get(c, 0.0) / wc:.1f} %"
        lines.append(f"| `{k}` | {n} | {a.get('SQ_WAVES', 0):.0f} | {wc:.3g} | {f('SQ_WAIT_ANY')} | "
                     f"{f('SQ_WAIT_INST_ANY')} | {f('SQ_ACTIVE_INST_ANY')} | {f('SQ_ACTIVE_INST_VALU')} |")
    text = "\n".join(lines) + "\n"
    print(text)
    if out:
        open(out, "w").write(text)


if __name__ == "__main__":
    main()
