"""Differential fuzz of the engine's codec restatement (redpanda_amd/csrc/
rpgpu_codec.h, the code the GPU decoder runs, compiled here for the host)
against the oracle (the reference's wrapper loops over liblz4 1.9.3 and
snappy 1.1.8, oracle/codec.c): verdicts, decoded lengths and bytes must agree
on library-made frames, hand-built sequences at the decoders' boundaries and
mutated / truncated inputs (tests/native/codec_fuzz.cpp)."""
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CONDA = "/opt/conda"


def build_fuzzer(tmp: Path, defines: tuple = ()) -> Path:
    import oracle.oracle as orc

    lib = orc.build()
    exe = tmp / ("codec_fuzz" + "".join("_" + d.replace("=", "_") for d in defines))
    subprocess.run(["g++", "-O2", "-std=c++17", *[f"-D{d}" for d in defines], f"-I{ROOT / 'redpanda_amd' / 'csrc'}",
                    f"-I{ROOT / 'include'}", f"-I{CONDA}/include",
                    str(ROOT / "tests" / "native" / "codec_fuzz.cpp"), "-o", str(exe),
                    f"-L{lib.parent}", "-lrporacle", f"-Wl,-rpath,{lib.parent}",
                    f"-L{CONDA}/lib", f"-Wl,-rpath,{CONDA}/lib", "-llz4", "-lsnappy"],
                   check=True, capture_output=True, text=True)
    return exe


def test_codec_restatement_matches_oracle(tmp_path):
    exe = build_fuzzer(tmp_path)
    for seed in (11, 12):
        r = subprocess.run([str(exe), "--cases", "15000", "--seed", str(seed)],
                           capture_output=True, text=True, timeout=900)
        assert r.returncode == 0, r.stderr[-6000:]
        assert "engine == oracle" in r.stdout


def test_snappy_lane_decoder_matches_oracle(tmp_path):
    """The opt-in lane-form snappy decoder (RPGPU_SNAPPY_LANE=1, rpgpu_codec.h
    snappy_raw_lane) for lane batches and snappy-java parts: same checks."""
    exe = build_fuzzer(tmp_path, ("RPGPU_SNAPPY_LANE=1",))
    r = subprocess.run([str(exe), "--cases", "15000", "--seed", "13"], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-6000:]
    assert "engine == oracle" in r.stdout
