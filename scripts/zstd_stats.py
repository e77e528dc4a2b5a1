#!/usr/bin/env python3
"""Table modes and shapes of the bench's zstd frames.

Parses the compressed bodies of a sample of a bench configuration's batches
(frame header, block headers, literals section header, Huffman table header
and sequence section header -- RFC 8878 §3.1.1) and prints histograms:
block types, literals types and sizes, Huffman weight counts / header kinds,
sequence counts and the LL / OF / ML table modes (0 predefined, 1 RLE, 2 FSE,
3 repeat) with the FSE accuracy logs.  Pure parsing of the format, no decode.

  python scripts/zstd_stats.py [--config c4] [--n 2048] [--min-bytes 0]
"""
import argparse
import collections
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def le(b, o, n):
    return int.from_bytes(bytes(b[o:o + n]), "little")


def frame_blocks(body):
    """Yields (type, payload bytes, frame header fields) per block of each frame."""
    p = 0
    while p + 5 <= len(body):
        magic = le(body, p, 4)
        if magic & 0xFFFFFFF0 == 0x184D2A50:
            p += 8 + le(body, p + 4, 4)
            continue
        assert magic == 0xFD2FB528, hex(magic)
        fhd = body[p + 4]
        did, ss, fid = fhd & 3, (fhd >> 5) & 1, fhd >> 6
        hs = 5 + (0 if ss else 1) + [0, 1, 2, 4][did] + ([ss, 2, 4, 8][fid])
        q = p + hs
        while True:
            bh = le(body, q, 3)
            t, last, size = (bh >> 1) & 3, bh & 1, bh >> 3
            q += 3
            payload = body[q:q + (1 if t == 1 else size)]
            yield t, payload, dict(fhd=fhd, csum=(fhd >> 2) & 1)
            q += 1 if t == 1 else size
            if last:
                break
        if (fhd >> 2) & 1:
            q += 4
        p = q


def fse_log(b, o):
    return (b[o] & 0xF) + 5


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--n", type=int, default=2048)
    ap.add_argument("--min-bytes", type=int, default=0, help="only bodies of at least this many compressed bytes")
    args = ap.parse_args()
    import bench
    from redpanda_amd import abi, engine

    cfg = bench.CONFIGS[args.config]
    spec = engine.make_spec(seed=0x5EED0000 + int(args.config[1:]), partitions=cfg["partitions"], **cfg["spec"])
    spec.ops = abi.OPS_PRODUCE | abi.OP_DECOMP
    spec.payload = abi.PAYLOAD_TEXT
    data, descs = engine.build_arena(spec, args.n)
    H = collections.defaultdict(collections.Counter)
    sums = collections.Counter()
    for d in descs:
        if d["length"] < 61:
            continue
        b = data[int(d["offset"]):int(d["offset"]) + int(d["length"])]
        if (int.from_bytes(bytes(b[21:23]), "big") & 7) != 4:
            continue
        body = bytes(b[61:])
        if len(body) < args.min_bytes:
            continue
        sums["batches"] += 1
        sums["compressed"] += len(body)
        for t, pl, fh in frame_blocks(body):
            H["block_type"][t] += 1
            if t != 2:
                continue
            lt, lh = pl[0] & 3, (pl[0] >> 2) & 3
            H["lit_type"][lt] += 1
            if lt in (2, 3):
                lhc = le(pl, 0, 5)
                if lh <= 1:
                    hs, size, csize = 3, (lhc >> 4) & 0x3FF, (lhc >> 14) & 0x3FF
                elif lh == 2:
                    hs, size, csize = 4, (lhc >> 4) & 0x3FFF, lhc >> 18 & 0x3FFF
                else:
                    hs, size, csize = 5, (lhc >> 4) & 0x3FFFF, (lhc >> 22) & 0x3FFFF
                H["lit_streams"][1 if lh == 0 else 4] += 1
                sums["lit_bytes"] += size
                sums["lit_cbytes"] += csize
                if lt == 2:
                    hb = pl[hs]
                    H["huf_header"]["direct" if hb >= 128 else "fse"] += 1
                    H["huf_nsym_bucket"][(hb - 127) // 32 * 32 if hb >= 128 else -1] += 1
                q = hs + csize
            else:
                if lh == 1:
                    hs, size = 2, le(pl, 0, 2) >> 4
                elif lh == 3:
                    hs, size = 3, le(pl, 0, 3) >> 4
                else:
                    hs, size = 1, pl[0] >> 3
                sums["lit_bytes"] += size
                q = hs + (size if lt == 0 else 1)
            ns = pl[q]
            q += 1
            if ns > 0x7F:
                if ns == 0xFF:
                    ns = le(pl, q, 2) + 0x7F00
                    q += 2
                else:
                    ns = ((ns - 0x80) << 8) + pl[q]
                    q += 1
            sums["sequences"] += ns
            H["nseq_bucket"][ns // 1000 * 1000] += 1
            if ns == 0:
                continue
            modes = pl[q]
            q += 1
            for name, m in (("LL", modes >> 6), ("OF", (modes >> 4) & 3), ("ML", (modes >> 2) & 3)):
                H[f"{name}_mode"][m] += 1
                if m == 2:
                    H[f"{name}_log"][fse_log(pl, q)] += 1
                    break  # later tables' offsets need the NCount length: only the first FSE table's log
                if m == 1:
                    q += 1
    print(f"{args.config}: {sums['batches']} zstd batches, {sums['compressed'] / max(sums['batches'], 1):.0f} B "
          f"compressed per batch, {sums['sequences'] / max(sums['batches'], 1):.0f} sequences, "
          f"{sums['lit_bytes'] / max(sums['batches'], 1):.0f} literal bytes "
          f"({sums['lit_cbytes'] / max(sums['batches'], 1):.0f} compressed)")
    for k in sorted(H):
        print(f"  {k:16s} {dict(sorted(H[k].items()))}")


if __name__ == "__main__":
    main()
