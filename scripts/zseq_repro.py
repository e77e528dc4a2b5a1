#!/usr/bin/env python3
"""Repro harness for the round-5 nondeterministic miscompare of the split zstd
decoder's executor: decodes test_many_tiny_zstd_gzip's
arena ITERS times with the library named by RPGPU_DIAG_LIB (split decoder on)
and counts, per iteration, the zstd batches whose rewritten bytes differ from
the oracle's.  For the first few it prints the differing window and a
classification of the wrong bytes:
  stale   -- equal to what the previous decode of the arena left there (the
             slot is not cleared between iterations),
  shifted -- the right bytes moved by a whole number of bits (a register
             computed with a wrong shift amount),
  copy    -- equal to output bytes found elsewhere in the same batch,
  other.

  RPGPU_DIAG_LIB=build/var/librpgpu_X.so python scripts/zseq_repro.py --iters 6
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def classify(g: np.ndarray, h: np.ndarray, prev: np.ndarray | None, whole_h: np.ndarray) -> str:
    if prev is not None and np.array_equal(g, prev):
        return "stale"
    gi = int.from_bytes(g.tobytes(), "little")
    hi = int.from_bytes(h.tobytes(), "little")
    m = (1 << (8 * len(g))) - 1
    for s in range(1, 8 * len(g)):
        if ((hi << s) & m) == gi or (hi >> s) == gi:
            return f"shifted({s} bits)"
    if whole_h.tobytes().find(g.tobytes()) >= 0:
        return "copy"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=150_000)
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--split", default="lds")
    args = ap.parse_args()
    import oracle.oracle as orc
    from redpanda_amd import abi, engine

    print("lib:", os.environ.get("RPGPU_DIAG_LIB", "default"), flush=True)
    spec = engine.make_spec(seed=0x5EED0077, partitions=64, codec_mix=(1 << 4) | (1 << 1), body_min=100,
                            body_max=400, ops=abi.OPS_PRODUCE | abi.OP_DECOMP, payload=abi.PAYLOAD_TEXT,
                            corrupt_ppm=5_000, corrupt_mask=0x3FF)
    data, descs = engine.build_arena(spec, args.n)
    want = None
    prev_out = None
    total = set()
    with engine.Engine(0, zstd_split=args.split if args.split != "off" else False) as e:
        for it in range(args.iters):
            t0 = time.time()
            got = e.decompress_arena(data, descs)
            dres, out = got["dres"], got["out"]
            if want is None:
                wres, _, _ = orc.validate_arena(data, descs, nthreads=8)
                caps = np.where(dres["out_cap"] > 0, dres["out_cap"].astype(np.int64) - 61 - 128, 0).astype(np.uint64)
                want = orc.decompress_arena(data, descs, wres, caps, codecs=(1, 2, 3, 4), nthreads=8)
            assert np.array_equal(dres["verdict"], want["verdicts"]), "verdicts differ"
            ok = np.nonzero((dres["verdict"] == abi.V_OK) & (dres["codec"] == 4))[0]
            bad = []
            for i in ok:
                a = int(dres["out_offset"][i]) + 61
                b = int(want["out_descs"]["offset"][i]) + 61
                m = int(dres["out_len"][i])
                if not np.array_equal(out[a:a + m], want["out"][b:b + m]):
                    bad.append(i)
            print(f"iter {it}: {len(ok)} zstd batches, {len(bad)} differ ({time.time() - t0:.1f} s) {bad[:12]}",
                  flush=True)
            for i in bad[:4]:
                a = int(dres["out_offset"][i]) + 61
                b = int(want["out_descs"]["offset"][i]) + 61
                m = int(dres["out_len"][i])
                g, h = out[a:a + m], want["out"][b:b + m]
                d = np.nonzero(g != h)[0]
                k0, k1 = int(d[0]), int(d[-1]) + 1
                pv = prev_out[a + k0:a + k1] if prev_out is not None and prev_out.size >= a + k1 else None
                print(f"  batch {i}: len {m}, bytes [{k0},{k1}) differ ({d.size}): gpu {g[k0:k1][:16].tolist()} "
                      f"host {h[k0:k1][:16].tolist()} prev {None if pv is None else pv[:16].tolist()} -> "
                      f"{classify(g[k0:k1], h[k0:k1], pv, h)}", flush=True)
            total.update(int(i) for i in bad)
            prev_out = out.copy()
    print(f"distinct batches ever wrong: {len(total)}", flush=True)


if __name__ == "__main__":
    main()
