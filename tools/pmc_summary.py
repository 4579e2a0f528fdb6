#!/usr/bin/env python3
"""Per-kernel HBM traffic from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; csv output).

usage: pmc_summary.py FETCH_counter_collection.csv WRITE_counter_collection.csv CONFIG out.json [out.md]

Correction (MI355X_MICROARCH.md §HBM): on gfx950 FETCH_SIZE reports half the bytes of a wide
streaming read (128-B requests tallied at 64 B); WRITE_SIZE is exact. Calibrated on this
run's own D2D parameter reset (__amd_rocclr_copyBuffer of the 100k points = 2,400,000 B):
the calibration rows are printed and stored. hbm_bytes_per_launch = 2 * FETCH + WRITE,
averaged over the dispatches of each kernel (gated-off launches of a converged solve would
read ~0 B; the bench runs with tolerances disabled, so every LM launch does its work).
"""
import csv
import json
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    n = re.sub(r"<.*>", "", n)
    n = n.replace("void ", "").replace("miba::", "")
    return n[2:] if n.startswith("k_") else n


def load(path, counter):
    agg = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024.0)  # KB -> B
    return agg


def main():
    fetch_csv, write_csv, config, out_json = sys.argv[1:5]
    out_md = sys.argv[5] if len(sys.argv) > 5 else None
    fe, wr = load(fetch_csv, "FETCH_SIZE"), load(write_csv, "WRITE_SIZE")
    res = {}
    for k in sorted(set(fe) | set(wr)):
        f = fe.get(k, [])
        w = wr.get(k, [])
        fa = sum(f) / len(f) if f else 0.0
        wa = sum(w) / len(w) if w else 0.0
        res[k] = {"launches": max(len(f), len(w)), "fetch_bytes_raw": fa, "write_bytes": wa,
                  "hbm_bytes_per_launch": 2.0 * fa + wa}
    calib = sorted(v for v in wr.get("__amd_rocclr_copyBuffer", []) if abs(v - 2.4e6) < 2e4)
    fcal = sorted(v for v in fe.get("__amd_rocclr_copyBuffer", []) if 1.1e6 < v < 1.3e6)
    doc = {config: res, "correction": "hbm_bytes = 2 * FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE halves wide reads)",
           "calibration": {"known_copy_bytes": 2400000, "write_size_bytes": calib[:1], "fetch_size_bytes_raw": fcal[:1]}}
    json.dump(doc, open(out_json, "w"), indent=1)
    if out_md:
        with open(out_md, "w") as fmd:
            fmd.write(f"# rocprofv3 --pmc HBM traffic, {config}\n\n{doc['correction']}. Calibration: a known "
                      f"2,400,000 B D2D copy reads FETCH_SIZE {fcal[:1]} B raw, WRITE_SIZE {calib[:1]} B.\n\n")
            fmd.write("| kernel | dispatches | FETCH raw B | x2 | WRITE B | HBM B / launch |\n|---|---|---|---|---|---|\n")
            for k, v in sorted(res.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"] * kv[1]["launches"]):
                fmd.write(f"| `{k}` | {v['launches']} | {v['fetch_bytes_raw']:.0f} | {2 * v['fetch_bytes_raw']:.0f} | "
                          f"{v['write_bytes']:.0f} | {v['hbm_bytes_per_launch']:.0f} |\n")


if __name__ == "__main__":
    main()
