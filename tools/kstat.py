"""Average duration (us) of the named kernels in rocprofv3 kernel_stats csv files: kstat.py DIR... -k name,name"""
import csv
import sys

args = sys.argv[1:]
keys = ["lin_point", "schur_tile", "bcr_split", "backsub_chunk", "k_final"]
if "-k" in args:
    i = args.index("-k")
    keys = args[i + 1].split(",")
    args = args[:i] + args[i + 2:]
for d in args:
    rows = list(csv.DictReader(open(f"{d}/kt_kernel_stats.csv")))
    out = []
    for k in keys:
        for r in rows:
            if k in r["Name"]:
                out.append(f"{k}={float(r['AverageNs']) / 1000:.2f}")
                break
    print(d, " ".join(out))
