"""Summarise gpurun_out/pmc/p*/ counter CSVs for validate_kernel: mean per
dispatch of each counter (summed over the device), plus per-batch values."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
kern = sys.argv[2] if len(sys.argv) > 2 else "validate_kernel"
nb = float(sys.argv[3]) if len(sys.argv) > 3 else 1048576
vals = defaultdict(lambda: defaultdict(float))
for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for row in csv.DictReader(open(f)):
        if kern not in row.get("Kernel_Name", ""):
            continue
        d = row["Dispatch_Id"]
        vals[row["Counter_Name"]][d] += float(row["Counter_Value"])
for name in sorted(vals):
    per = vals[name]
    m = sum(per.values()) / len(per)
    print(f"{name:32s} {m:16.4g}  per-batch {m / nb:10.4g}  (dispatches {len(per)})")
