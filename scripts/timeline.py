#!/usr/bin/env python3
"""One step's kernel timeline from a rocprofv3 kernel trace (the last run of
decomp_counters_kernel onwards, or the last validate_kernel launch group):
start / end / duration per kernel launch longer than --min ms, with its stream.

  python scripts/timeline.py gpurun_out/<dir>/run_kernel_trace.csv [--min 0.2]
"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--min", type=float, default=0.2)
ap.add_argument("--anchor", default="decomp_counters_kernel")
args = ap.parse_args()
rows = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if args.anchor in r["Kernel_Name"]]
st = idx[-2] if len(idx) >= 2 and args.anchor == "decomp_counters_kernel" else (idx[-1] if idx else 0)
t0 = int(rows[st]["Start_Timestamp"])
for r in rows[st:]:
    s = (int(r["Start_Timestamp"]) - t0) / 1e6
    e = (int(r["End_Timestamp"]) - t0) / 1e6
    if e - s > args.min:
        print(f"{s:8.2f} {e:8.2f} {e - s:8.2f}  stream {r.get('Stream_Id', '')}  {r['Kernel_Name'][:70]}")
