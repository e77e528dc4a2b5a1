"""Fixture generator (run here, not on the GPU box): crafted zstd frames whose
1 KiB window makes the reference loop's ring buffer wrap every two blocks,
each with one match whose offset reaches into the previous ring segment
(where the current one has or has not overwritten it) or before it
(corruption_detected in libzstd); and (`band_*`) frames whose matches, once
the ring has wrapped, read the previous segment right past the write
position, where libzstd's over-long copies (ZSTD_wildcopy, ZSTD_overlapCopy8,
ZSTD_safecopy near the ring's end) left bytes -- 40 small ones (lane decoder)
and 4 of 400 blocks (wave decoder); and (`span_*`) frames whose second
ring segment opens with a match spanning the previous segment's end into the
current one's start, its second part at a distance that is or is not below
16 (libzstd's ZSTD_overlapCopy8) -- 60 of a grid plus 20 random ones.  Made by
tests/native/zstd_fuzz.cpp --dump-ring / --dump-band / --dump-span (the
engine's own zstd encoder pieces, predefined FSE tables);
the expected outputs come from the oracle (libzstd 1.4.9 through
stream_zstd::do_uncompress) at test time.  Writes tests/golden/zstd_ring.npz."""
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

# (offset, blocks, bad block): small frames for the lane decoder, ~300 KiB ones
# (their bound is 1 KiB per block) for the wave decoder
CASES = [(900, 8, 5), (1500, 8, 5), (2100, 8, 5), (2600, 8, 5), (3000, 8, 5), (3152, 8, 5), (3153, 8, 5),
         (5200, 8, 5), (700, 9, 8), (2500, 12, 11), (2600, 300, 201), (3153, 300, 201)]


def main():
    from test_zstd_fuzz import build_fuzzer

    with tempfile.TemporaryDirectory() as tmp:
        exe = build_fuzzer(Path(tmp))
        frames = []
        for off, nb, bad in CASES:
            subprocess.run([str(exe), "--seed", "11", "--dump-ring", f"{off},{nb},{bad}"], cwd=tmp, check=True)
            frames.append(np.frombuffer((Path(tmp) / "ring.zst").read_bytes(), dtype=np.uint8))
        subprocess.run([str(exe), "--seed", "12", "--dump-band", "40,4"], cwd=tmp, check=True)
        raw = (Path(tmp) / "band.bin").read_bytes()
        band, p = [], 0
        while p < len(raw):
            n = int.from_bytes(raw[p:p + 4], "little")
            band.append(np.frombuffer(raw[p + 4:p + 4 + n], dtype=np.uint8))
            p += 4 + n
        subprocess.run([str(exe), "--seed", "13", "--dump-span", "20"], cwd=tmp, check=True)
        raw = (Path(tmp) / "span.bin").read_bytes()
        span, p = [], 0
        while p < len(raw):
            n = int.from_bytes(raw[p:p + 4], "little")
            span.append(np.frombuffer(raw[p + 4:p + 4 + n], dtype=np.uint8))
            p += 4 + n
    lens = np.array([len(f) for f in frames], dtype=np.int64)
    blens = np.array([len(f) for f in band], dtype=np.int64)
    slens = np.array([len(f) for f in span], dtype=np.int64)
    np.savez_compressed(ROOT / "tests" / "golden" / "zstd_ring.npz", data=np.concatenate(frames), lens=lens,
                        cases=np.array(CASES, dtype=np.int64), band_data=np.concatenate(band), band_lens=blens,
                        span_data=np.concatenate(span), span_lens=slens)
    print("wrote", len(frames), "ring frames,", int(lens.sum()), "bytes;", len(band), "band frames,", int(blens.sum()),
          "bytes;", len(span), "span frames,", int(slens.sum()), "bytes")


if __name__ == "__main__":
    main()
