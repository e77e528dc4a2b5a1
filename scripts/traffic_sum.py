"""Per-launch HBM traffic of a decompress pipeline from rocprofv3 PMC passes
(scripts/gpu_pmc_traffic.sh with --steps 1 --warmup 0): FETCH_SIZE and
WRITE_SIZE (KB, summed over the device) of every rpgpu:: kernel dispatch of
the one timed step (all walk-overlap chunks included), merged into
profiles/traffic.json under the config.

FETCH_SIZE is reported raw: the decoders' reads are scattered 16-byte
accesses, for which MI355X_MICROARCH.md's 2x streaming-read correction is
uncalibrated; validate_kernel's streaming reads are doubled as the guide
prescribes.  usage: traffic_sum.py <pmc dir> <config> <batches> [payload]
The entry is keyed by config and payload ("c3", "c3:alnum"), as bench.py
looks it up, and carries the first 16 hex digits of librpgpu.so's SHA-256:
bench.py attaches it to roofline.traffic only for that exact library."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root, cfg, nb = sys.argv[1], sys.argv[2], int(sys.argv[3])
payload = sys.argv[4] if len(sys.argv) > 4 else "text"
key = cfg if payload == "text" else f"{cfg}:{payload}"
# one pipeline step: uncompressed configs run only the step (--steps 1 --warmup 0),
# every dispatch counts; a decompress config's bench first runs the validation
# and the decompress plan untimed (to size the output), so its step starts at
# the second-to-last caps_kernel (the step's plan; the last one plans the
# rewritten batches) and every rpgpu:: dispatch from there on counts
plain = cfg in ("c1", "c2")
per = defaultdict(lambda: defaultdict(float))
for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
    rows = [r for r in csv.DictReader(open(f)) if "rpgpu::" in r.get("Kernel_Name", "")]
    start = 0
    if not plain:
        caps = sorted({int(r["Dispatch_Id"]) for r in rows if r["Kernel_Name"].startswith("rpgpu::caps_kernel")})
        start = caps[-2] if len(caps) >= 2 else 0
    for r in rows:
        if plain and not any(k in r["Kernel_Name"] for k in ("validate_kernel", "walk_kernel", "walk_wave_kernel")):
            continue  # the roofline's kernels: the checksums and the walk
        if int(r["Dispatch_Id"]) >= start:
            per[r["Counter_Name"]][r["Kernel_Name"].split("(")[0]] += float(r["Counter_Value"])
fetch = sum(v * (2.0 if "validate_kernel" in k else 1.0) for k, v in per["FETCH_SIZE"].items()) * 1024
write = sum(per["WRITE_SIZE"].values()) * 1024
import hashlib  # noqa: E402

lib = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "redpanda_amd", "librpgpu.so")
lib_hash = hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16] if os.path.exists(lib) else None
out = {"batches": nb, "payload": payload, "lib_sha256_16": lib_hash,
       "kernel": ("validate_kernel + walk_kernel of one step (all chunk dispatches)" if plain
                  else "every rpgpu:: kernel of one pipeline step"),
       "fetch_bytes": int(fetch), "write_bytes": int(write),
       "hbm_bytes_per_launch": int(fetch + write),
       "raw_counters_kb_per_step": {c: dict(v) for c, v in per.items()},
       "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / TCC_HIT_sum TCC_MISS_sum in separate passes "
                 "(scripts/gpu_pmc_traffic.sh, --steps 1 --warmup 0); validate_kernel FETCH doubled "
                 "(16-B/lane streaming reads, MI355X_MICROARCH.md); the decoders' scattered reads raw"}
p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "traffic.json")
doc = json.load(open(p)) if os.path.exists(p) else {}
doc[key] = out
json.dump(doc, open(p, "w"), indent=1)
sums = {c: sum(v.values()) for c, v in per.items()}
print(key, "fetch GB", round(fetch / 1e9, 2), "write GB", round(write / 1e9, 2), {k: f"{v:.3g}" for k, v in sums.items()})
