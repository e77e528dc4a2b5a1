"""Print one step's kernel timeline (start / end in ms from the step's first
decompression kernel, per stream) from a rocprofv3 rocpd database
(rocprofv3 --kernel-trace -d DIR -o run).  Usage: timeline.py DB [step]"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
step = int(sys.argv[2]) if len(sys.argv) > 2 else -1
rows = list(db.execute("select name, start, end, stream_id, queue_id from kernels order by start"))
starts = [r[1] for r in rows if "decomp_counters_kernel" in r[0]]
# every run launches decomp_counters_kernel twice (plan, then run): take the plan's
plans = starts[0::2]
t0 = plans[step]
t1 = plans[step + 1] if step + 1 < len(plans) and step != -1 else float("inf")
for name, s, e, st, q in rows:
    if t0 <= s < t1:
        short = name.split("(")[0].replace("void ", "").replace("rpgpu::", "")
        if e - s > 0.2e6 or "decomp" in short:
            print(f"{(s - t0) / 1e6:8.2f} {(e - t0) / 1e6:8.2f} {(e - s) / 1e6:7.2f}  s{st} q{q}  {short}")
