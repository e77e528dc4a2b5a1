"""The engine's decoder restatements (rpgpu_codec.h, rpgpu_zstd.h,
rpgpu_inflate.h: the code the
GPU kernels run) built for the host with AddressSanitizer and
UndefinedBehaviorSanitizer, run over the differential fuzz corpora with the
device's exact buffer geometry (--exact 1: RPGPU_ARENA_TAIL_PAD readable
bytes past each input, an output slot of bound + kSlack).  The decoders copy
in 16/64-byte chunks and rely on kSlack; an access past what the GPU slot
allows would silently corrupt the neighbouring slot on the device, and is a
heap-buffer-overflow here.  (The reference builds its debug configuration
with -fsanitize=address,undefined, cmake/main.cmake:30-41.)"""
import os
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
CONDA = "/opt/conda"
SAN = ["-fsanitize=address,undefined", "-static-libstdc++", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer", "-g", "-O1"]


def build(tmp: Path, name: str, libs: list[str]) -> Path:
    import oracle.oracle as orc

    lib = orc.build()
    exe = tmp / f"{name}_san"
    r = subprocess.run(["g++", "-std=c++17", *SAN, f"-I{ROOT / 'redpanda_amd' / 'csrc'}",
                        f"-I{ROOT / 'include'}", f"-I{CONDA}/include",
                        str(ROOT / "tests" / "native" / f"{name}.cpp"), "-o", str(exe),
                        f"-L{lib.parent}", "-lrporacle", f"-Wl,-rpath,{lib.parent}",
                        f"-Wl,-rpath,{CONDA}/lib", *libs],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    return exe


def run(exe: Path, cases: int, seed: int, cwd: Path):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([str(exe), "--cases", str(cases), "--seed", str(seed), "--exact", "1"], cwd=cwd,
                       capture_output=True, text=True, timeout=1200, env=env)
    assert r.returncode == 0, (r.stdout[-2000:] + r.stderr[-8000:])
    assert "engine == oracle" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-8000:]


@pytest.mark.parametrize("seed", [31])
def test_codec_restatement_asan_ubsan(tmp_path, seed):
    run(build(tmp_path, "codec_fuzz", [f"{CONDA}/lib/liblz4.so", f"{CONDA}/lib/libsnappy.so"]), 4000, seed, tmp_path)


@pytest.mark.parametrize("seed", [41])
def test_zstd_restatement_asan_ubsan(tmp_path, seed):
    run(build(tmp_path, "zstd_fuzz", [f"{CONDA}/lib/libzstd.so"]), 250, seed, tmp_path)


@pytest.mark.parametrize("seed", [61])
def test_inflate_restatement_asan_ubsan(tmp_path, seed):
    run(build(tmp_path, "inflate_fuzz", [f"{CONDA}/lib/libz.so"]), 2000, seed, tmp_path)
