"""The workgroup LZ4 block decoder's phases (redpanda_amd/csrc/rpgpu_lz4blk.h:
chain entries, range walks, output scan, fast-loop events, LDS copies with
the pending-byte protocol, the serial tail) run on the host thread by thread
(tests/native/lz4blk_sim.cpp) against rpcodec::lz4_block, the serial
restatement of liblz4 1.9.3's block decoder that tests/test_codec_fuzz.py pins
to the library: decoded sizes, error verdicts and bytes must agree on liblz4
blocks, hand-made sequences and mutated / garbage blocks."""
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CONDA = "/opt/conda"


def test_workgroup_block_decoder_matches_serial(tmp_path):
    exe = tmp_path / "lz4blk_sim"
    subprocess.run(["g++", "-O2", "-std=c++17", f"-I{ROOT / 'redpanda_amd' / 'csrc'}", f"-I{ROOT / 'include'}",
                    f"-I{CONDA}/include", str(ROOT / "tests" / "native" / "lz4blk_sim.cpp"), "-o", str(exe),
                    f"-L{CONDA}/lib", f"-Wl,-rpath,{CONDA}/lib", "-llz4"], check=True, capture_output=True, text=True)
    for seed in (1, 2):
        r = subprocess.run([str(exe), "--cases", "600", "--seed", str(seed)], capture_output=True, text=True,
                           timeout=600)
        assert r.returncode == 0, r.stderr[-4000:]
        assert "workgroup == serial" in r.stdout
        decoded = int(r.stdout.split("decoded ")[1].split(",")[0])
        assert decoded > 200, r.stdout
