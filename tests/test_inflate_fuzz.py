"""Differential fuzz of the engine's gzip restatement (redpanda_amd/csrc/
rpgpu_inflate.h, the code the GPU's gzip lanes run, compiled here for the
host) against the oracle: gzip_decompression_codec::inflate_to_iobuf
(compression/internal/gzip_compressor.cc:177-229) over zlib (oracle/codec.c).
Verdicts, decoded lengths and bytes must agree on library-made gzip / zlib
streams and mutated / truncated / concatenated ones, including the wrapper's
chunk rule (output stops at a chunk end once all input is in zlib's bit
buffer) -- tests/native/inflate_fuzz.cpp."""
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CONDA = "/opt/conda"


def build_fuzzer(tmp: Path) -> Path:
    import oracle.oracle as orc

    lib = orc.build()
    exe = tmp / "inflate_fuzz"
    subprocess.run(["g++", "-O2", "-std=c++17", f"-I{ROOT / 'redpanda_amd' / 'csrc'}",
                    f"-I{ROOT / 'include'}", f"-I{CONDA}/include",
                    str(ROOT / "tests" / "native" / "inflate_fuzz.cpp"), "-o", str(exe),
                    f"-L{lib.parent}", "-lrporacle", f"-Wl,-rpath,{lib.parent}",
                    f"{CONDA}/lib/libz.so", f"-Wl,-rpath,{CONDA}/lib"],
                   check=True, capture_output=True, text=True)
    return exe


def test_inflate_restatement_matches_oracle(tmp_path):
    exe = build_fuzzer(tmp_path)
    for seed in (51, 52):
        r = subprocess.run([str(exe), "--cases", "3000", "--seed", str(seed)], cwd=tmp_path,
                           capture_output=True, text=True, timeout=900)
        assert r.returncode == 0, r.stderr[-6000:]
        assert "engine == oracle" in r.stdout
