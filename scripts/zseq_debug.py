#!/usr/bin/env python3
"""Diagnostics for the split zstd decoder on the GPU: decodes an arena, and for
the first batch whose rewritten bytes differ from the oracle's, locates that
batch's literal region and records in the device output buffer (by searching
for what the host build of the same code, tests/native/zseq_host.cpp, makes of
its body) and reports which stage differs: A1 literals, A2 records, or B.

  python scripts/zseq_debug.py [--n 40000]
"""
import argparse
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def host_lib():
    so = "/tmp/zseq_host.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", f"-I{ROOT}/redpanda_amd/csrc", f"-I{ROOT}/include",
                    f"{ROOT}/tests/native/zseq_host.cpp", "-o", so], check=True)
    lib = C.CDLL(so)
    lib.zseq_plan.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                              C.POINTER(C.c_uint32)]
    lib.zseq_decode.restype = C.c_int32
    lib.zseq_decode.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p,
                                C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_void_p, C.c_int]
    return lib


def find(hay: np.ndarray, needle: np.ndarray, start=0):
    b = hay.tobytes()
    return b.find(needle.tobytes(), start)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=40000)
    args = ap.parse_args()
    import oracle.oracle as orc
    from redpanda_amd import abi, engine

    spec = engine.make_spec(seed=0x5EED0077, partitions=64, codec_mix=(1 << 4) | (1 << 1), body_min=100,
                            body_max=400, ops=abi.OPS_PRODUCE | abi.OP_DECOMP, payload=abi.PAYLOAD_TEXT,
                            corrupt_ppm=5_000, corrupt_mask=0x3FF)
    data, descs = engine.build_arena(spec, args.n)
    with engine.Engine(0) as e:
        got = e.decompress_arena(data, descs)
    dres = got["dres"]
    res, _, _ = orc.validate_arena(data, descs)
    caps = np.where(dres["out_cap"] > 0, dres["out_cap"].astype(np.int64) - 61 - 128, 0).astype(np.uint64)
    want = orc.decompress_arena(data, descs, res, caps, codecs=(1, 2, 3, 4))
    ok = (dres["verdict"] == 0) & (want["verdicts"] == 0)
    print("verdicts equal:", bool(np.array_equal(dres["verdict"], want["verdicts"])),
          "lengths equal:", bool(np.array_equal(dres["out_len"][ok], want["out_len"][ok])))
    out = got["out"]
    # each zstd batch again through the host build of the split decoder
    lib = host_lib()
    nbad = 0
    for i in np.nonzero(ok & (dres["codec"] == 4))[0]:
        d = descs[i]
        body = np.ascontiguousarray(data[int(d["offset"]) + 61:int(d["offset"]) + int(d["length"]) + 64])
        n = int(d["length"]) - 61
        lits, recs, nsec = C.c_uint64(), C.c_uint64(), C.c_uint32()
        if not lib.zseq_plan(body.ctypes.data, n, C.byref(lits), C.byref(recs), C.byref(nsec)):
            continue
        cap = int(caps[i])
        lb = np.zeros(lits.value + 64, np.uint8)
        rb = np.zeros(recs.value + 16, np.uint64)
        hb = np.zeros(cap + 128, np.uint8)
        ln, nr = C.c_uint64(), C.c_uint64()
        sec = np.zeros(16, np.uint32)
        v = lib.zseq_decode(body.ctypes.data, n, lb.ctypes.data, lits.value, rb.ctypes.data, recs.value,
                            hb.ctypes.data, cap, C.byref(ln), C.byref(nr), sec.ctypes.data, 1)
        if v != 0:
            continue
        a, m = int(dres["out_offset"][i]) + 61, int(dres["out_len"][i])
        g = out[a:a + m]
        if np.array_equal(g, hb[:m]):
            continue
        nbad += 1
        k = int(np.argmax(g != hb[:m]))
        print(f"batch {i}: body {n} B, decoded {m} B, first diff at {k}: gpu {g[k:k + 8].tolist()} host {hb[k:k + 8].tolist()}")
        if nbad > 3:
            continue
        # A1: the host literal region in the device buffer
        L = int(lits.value)
        if L >= 16:
            at = find(out, lb[:16])
            print(f"  literal region ({L} B): host's first 16 bytes at device offset {at}", end="")
            if at >= 0:
                print(", all equal:", bool(np.array_equal(out[at:at + L], lb[:L])))
            else:
                print()
        # A2: records (skip SETLIT payloads: addresses differ)
        R = int(nr.value)
        recs_h = rb[:R]
        addr = {j + 1 for j in range(R - 1) if (int(recs_h[j]) & ((1 << 28) - 1)) == 0 and int(recs_h[j]) >> 46 == 1}
        seqs = [j for j in range(R) if j not in addr and (int(recs_h[j]) & ((1 << 28) - 1)) != 0]
        if len(seqs) >= 4:
            j0 = seqs[0]
            at = find(out, recs_h[j0:j0 + 3].view(np.uint8))
            print(f"  records ({R}): host's first sequences at device offset {at}")
            if at >= 0:
                base = at - 8 * j0
                gr = out[base:base + 8 * R].view(np.uint64)
                diff = [j for j in range(R) if gr[j] != recs_h[j] and j not in addr]
                print(f"  records differing (excl. addresses): {diff[:10]}")
                for j in diff[:4]:
                    print(f"    rec {j}: gpu {int(gr[j]):#x} host {int(recs_h[j]):#x}")
    print("mismatching zstd batches:", nbad)


if __name__ == "__main__":
    main()
