"""Critical path of decompress-config bench steps from a rocprofv3 kernel
trace (--kernel-trace, csv).  A step starts at the plan's caps_kernel that
precedes its gzip_bound_kernel (one per step) and ends where the next step
starts.  Per step: wall span, each queue's span and busy time (union of its
kernels' intervals), and each kernel's busy time and span; the queue whose
span ends last is the critical one.  Kernel "time" in rocprof's stats counts
a kernel from dispatch, so a kernel queued behind another stream's persistent
grid looks long there; spans per queue do not have that problem.
Usage: python scripts/decomp_trace.py <kernel_trace.csv> [skip_steps]"""
import csv
import statistics
import sys
from collections import defaultdict


def short(name):
    n = name.split("(")[0]
    return n.replace("rpgpu::", "").replace("void ", "")


def union(iv):
    tot, cs, ce = 0, None, None
    for s, e in sorted(iv):
        if ce is None or s > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + (ce - cs if ce is not None else 0)


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    rows = [r for r in rows if "rpgpu" in r["Kernel_Name"]]
    names = [short(r["Kernel_Name"]) for r in rows]
    starts = []
    for k, nm in enumerate(names):
        if nm == "gzip_bound_kernel":
            j = k
            while j > 0 and names[j] != "caps_kernel":
                j -= 1
            # the plan's caps_kernel is the one before validate_kernel of the input arena
            while j > 0 and names[j - 1] != "summary_kernel" and names[j - 1] != "summary_reduce_kernel" and names[j] != "caps_kernel":
                j -= 1
            # walk back to the first caps_kernel of the step (input validation plan)
            jj = j - 1
            while jj >= 0 and names[jj] not in ("caps_kernel", "summary_kernel", "summary_reduce_kernel"):
                jj -= 1
            starts.append(jj if jj >= 0 and names[jj] == "caps_kernel" else j)
    steps = [rows[a:b] for a, b in zip(starts, starts[1:] + [len(rows)])][skip:]
    walls, crit = [], defaultdict(list)
    for k, st in enumerate(steps):
        t0 = min(int(r["Start_Timestamp"]) for r in st)
        t1 = max(int(r["End_Timestamp"]) for r in st)
        q = defaultdict(list)
        kb = defaultdict(list)
        for r in st:
            iv = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
            q[r["Queue_Id"]].append(iv)
            kb[short(r["Kernel_Name"])].append(iv)
        walls.append((t1 - t0) / 1e6)
        print(f"step {k}: wall {(t1 - t0) / 1e6:.2f} ms")
        for qid, iv in sorted(q.items()):
            s0, s1 = min(a for a, _ in iv), max(b for _, b in iv)
            print(f"  queue {qid}: span {(s0 - t0) / 1e6:8.2f} -> {(s1 - t0) / 1e6:8.2f} ms, busy {union(iv) / 1e6:8.2f} ms")
        for nm, iv in sorted(kb.items(), key=lambda x: -union(x[1])):
            s0, s1 = min(a for a, _ in iv), max(b for _, b in iv)
            crit[nm].append(union(iv) / 1e6)
            print(f"    {nm:28s} x{len(iv):2d} busy {union(iv) / 1e6:8.2f} ms  [{(s0 - t0) / 1e6:8.2f}, {(s1 - t0) / 1e6:8.2f}]")
    if walls:
        print(f"median wall over {len(walls)} steps: {statistics.median(walls):.2f} ms")


if __name__ == "__main__":
    main()
