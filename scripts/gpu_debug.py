import sys, zlib; sys.path.insert(0, '.')
import numpy as np, oracle.oracle as orc
from redpanda_amd import abi, engine
eng = engine.Engine(0)
for rep in range(3):
    for fmt in (0, 1):
        spec = engine.make_spec(seed=zlib.crc32(b"ragged"), format=fmt, body_min=7, body_max=300000, records_per_batch=1)
        data, descs = engine.build_arena(spec, 40)
        res, idx, used = eng.submit(data, descs)
        ores, oidx, oused = orc.validate_arena(data, descs)
        bad = np.nonzero(res != ores)[0]
        print("rep", rep, "fmt", fmt, "bad", bad)
        for b in bad[:3]:
            print(" gpu", res[b]); print(" orc", ores[b]); print(" desc", descs[b])
