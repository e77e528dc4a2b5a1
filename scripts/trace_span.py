"""Critical path of bench steps from a rocprofv3 kernel trace (--kernel-trace,
csv): per step (a step starts at each `step_kernel` dispatch), the wall span
from the first dispatch to the last end, the span of the named hot kernels
(first start -> last end), the busy time of each kernel (union of its
intervals) and per-stream busy time.  Usage:
  python scripts/trace_span.py <kernel_trace.csv> [step_kernel] [hot1,hot2,...] [skip_steps]"""
import csv
import sys
from collections import defaultdict


def union(iv):
    iv = sorted(iv)
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def short(name):
    n = name.split("(")[0]
    return n.replace("rpgpu::", "").replace("void ", "")


def main():
    path = sys.argv[1]
    step_k = sys.argv[2] if len(sys.argv) > 2 else "caps_kernel"
    hot = sys.argv[3].split(",") if len(sys.argv) > 3 else ["validate_kernel", "walk_kernel"]
    skip = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if "rpgpu" in r["Kernel_Name"]]
    steps, cur = [], None
    for r in rows:
        if short(r["Kernel_Name"]) == step_k:
            cur = []
            steps.append(cur)
        if cur is not None:
            cur.append(r)
    steps = steps[skip:]
    out = []
    for k, st in enumerate(steps):
        t0 = min(int(r["Start_Timestamp"]) for r in st)
        t1 = max(int(r["End_Timestamp"]) for r in st)
        h = [r for r in st if any(x in r["Kernel_Name"] for x in hot)]
        h0 = min(int(r["Start_Timestamp"]) for r in h) if h else 0
        h1 = max(int(r["End_Timestamp"]) for r in h) if h else 0
        busy = defaultdict(list)
        streams = defaultdict(list)
        for r in st:
            iv = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
            busy[short(r["Kernel_Name"])].append(iv)
            streams[r["Queue_Id"]].append(iv)
        out.append((t1 - t0, h1 - h0, {n: union(v) for n, v in busy.items()},
                    {q: union(v) for q, v in streams.items()}, {n: len(v) for n, v in busy.items()}))
        print(f"step {k}: wall {(t1 - t0) / 1e6:.4f} ms, hot span {(h1 - h0) / 1e6:.4f} ms, "
              + ", ".join(f"{n} {v / 1e6:.4f} ms x{out[-1][4][n]}" for n, v in out[-1][2].items())
              + " | queues " + ", ".join(f"{q}: {v / 1e6:.4f}" for q, v in out[-1][3].items()))
    if out:
        import statistics
        print(f"median over {len(out)} steps: wall {statistics.median(o[0] for o in out) / 1e6:.4f} ms, "
              f"hot span {statistics.median(o[1] for o in out) / 1e6:.4f} ms")


if __name__ == "__main__":
    main()
