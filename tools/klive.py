"""Median duration (us) of the live launches (> 15 us) of named kernels in rocprofv3 kernel traces:
klive.py DIR... -k name,name"""
import csv
import statistics
import sys

args = sys.argv[1:]
keys = ["lin_point", "schur_tile", "bcr_split", "backsub_chunk"]
if "-k" in args:
    i = args.index("-k")
    keys = args[i + 1].split(",")
    args = args[:i] + args[i + 2:]
for d in args:
    rows = list(csv.DictReader(open(f"{d}/kt_kernel_trace.csv")))
    out = []
    for k in keys:
        v = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in rows if k in r["Kernel_Name"]]
        v = [x for x in v if x > 15]
        if v:
            out.append(f"{k}={statistics.median(v):.1f}(n{len(v)})")
    print(d, " ".join(out))
