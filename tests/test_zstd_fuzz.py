"""Differential fuzz of the engine's zstd restatement (redpanda_amd/csrc/
rpgpu_zstd.h, the code the GPU's zstd_kernel runs, compiled here for the host)
against the oracle: the reference's stream_zstd::do_uncompress loop
(compression/stream_zstd.cc:198-223) over libzstd 1.4.9 (oracle/codec.c).
Also pins the restated internals against libzstd's own exported functions
(FSE_readNCount, HUF_selectDecoder, the static-workspace budget).  Verdicts,
decoded lengths and bytes must agree on library-made frames and mutated /
truncated / concatenated ones (tests/native/zstd_fuzz.cpp)."""
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CONDA = "/opt/conda"


def build_fuzzer(tmp: Path) -> Path:
    import oracle.oracle as orc

    lib = orc.build()
    exe = tmp / "zstd_fuzz"
    subprocess.run(["g++", "-O2", "-std=c++17", f"-I{ROOT / 'redpanda_amd' / 'csrc'}",
                    f"-I{ROOT / 'include'}", f"-I{CONDA}/include",
                    str(ROOT / "tests" / "native" / "zstd_fuzz.cpp"), "-o", str(exe),
                    f"-L{lib.parent}", "-lrporacle", f"-Wl,-rpath,{lib.parent}",
                    f"-L{CONDA}/lib", f"-Wl,-rpath,{CONDA}/lib", "-lzstd"],
                   check=True, capture_output=True, text=True)
    return exe


def test_zstd_restatement_matches_oracle(tmp_path):
    exe = build_fuzzer(tmp_path)
    for seed in (21, 22):
        r = subprocess.run([str(exe), "--cases", "1500", "--seed", str(seed)], cwd=tmp_path,
                           capture_output=True, text=True, timeout=900)
        assert r.returncode == 0, r.stderr[-6000:]
        assert "engine == oracle" in r.stdout
