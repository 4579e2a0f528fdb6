#!/usr/bin/env python3
"""Kernel + memory-copy timeline of the last N events of a rocprofv3 csv run (diagnostic).
usage: timeline.py <dir with *_kernel_trace.csv / *_memory_copy_trace.csv> [N=60]"""
import csv
import glob
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
ev = []
for f in glob.glob(f"{d}/*_memory_copy_trace.csv"):
    for r in csv.DictReader(open(f)):
        ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), 'COPY ' + r['Direction'].replace('MEMORY_COPY_', '')))
for f in glob.glob(f"{d}/*_kernel_trace.csv"):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].replace('miba::', '').replace('(anonymous namespace)::', '')
        ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), 'K ' + k[:48]))
ev.sort()
ev = ev[-n:]
t0 = ev[0][0]
for s, e, name in ev:
    print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} us  {name}")
