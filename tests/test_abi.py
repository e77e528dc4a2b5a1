"""The C ABI as a C program sees it (CPU, no GPU needed).

* include/rpgpu.h compiles as C11 with -Wall -Wextra -Werror and links
  against librpgpu.so (tests/native/abi_client.c, the binding a Redpanda
  maintainer would write);
* the library exports exactly the functions the header declares, and
  redpanda_amd.abi.EXPORTED lists the same set;
* the pure entry points work without a device (ABI version, the
  produce-handler error-code map), and rpgpu_open fails cleanly with none;
* the verdict -> Kafka error code map follows produce.cc:440-489 in order.
The same client runs its device half in tests/test_gpu_abi.py."""
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "rpgpu.h"


def declared() -> set[str]:
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return set(re.findall(r"\b(rpgpu_\w+)\s*\(", text))


def exported(lib: Path) -> set[str]:
    out = subprocess.run(["nm", "-D", "--defined-only", str(lib)], capture_output=True, text=True,
                         check=True).stdout
    return {l.split()[-1] for l in out.splitlines() if l.split()[-1].startswith("rpgpu_")}


@pytest.fixture(scope="module")
def client(built, tmp_path_factory):
    from redpanda_amd import _build

    exe = tmp_path_factory.mktemp("abi") / "abi_client"
    r = subprocess.run(["gcc", "-std=c11", "-D_GNU_SOURCE", "-Wall", "-Wextra", "-Werror", "-O1",
                        f"-I{ROOT / 'include'}", str(ROOT / "tests" / "native" / "abi_client.c"),
                        "-o", str(exe), f"-L{_build.PKG}", "-lrpgpu", f"-Wl,-rpath,{_build.PKG}"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


def test_exports_match_header(built):
    from redpanda_amd import _build, abi

    decl = declared()
    exp = exported(_build.LIBRPGPU)
    assert decl <= exp, f"declared but not exported: {sorted(decl - exp)}"
    assert exp - decl == set(), f"exported but not declared: {sorted(exp - decl)}"
    assert set(abi.EXPORTED) == decl, (sorted(set(abi.EXPORTED) ^ decl))


def test_header_compiles_as_cplusplus(tmp_path):
    src = tmp_path / "h.cpp"
    src.write_text('#include "rpgpu.h"\nint main() { return rpgpu_abi_version() > 0 ? 0 : 1; }\n')
    r = subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-fsyntax-only", f"-I{ROOT / 'include'}",
                        str(src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_c_client_without_device(client):
    import torch

    mode = "cpu" if torch.cuda.is_available() else "nodevice"
    r = subprocess.run([str(client), mode], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok" in r.stdout


# produce.cc:440-489 restated: the checks in the handler's order
def reference_code(verdict: int, size_bytes: int, batch_max_bytes: int) -> int:
    from redpanda_amd import abi

    if verdict == abi.V_NULL_RECORDS:                    # !part.records
        return 87
    if verdict in (abi.V_HDR_TRUNC_THROW, abi.V_BAD_CODEC_THROW, abi.V_BODY_TRUNC_THROW):
        return -1                                        # exception escapes decode
    if verdict == abi.V_CRC_MISMATCH:                    # !valid_crc
        return 2
    if verdict in (abi.V_TOO_SMALL, abi.V_BAD_MAGIC):    # !v2_format (flags undefined)
        return 87
    if verdict in (abi.V_REC_ATTR_EOF, abi.V_REC_TRAILING, abi.V_REC_HCOUNT_NEG, abi.V_REC_UNDEFINED):
        return 87                                        # !batch
    if verdict == abi.V_OK:
        return 10 if batch_max_bytes and size_bytes > batch_max_bytes else 0  # produce.cc:317-324
    return -1


def test_kafka_error_code_map(built):
    from redpanda_amd import abi, engine

    r = np.zeros(1, dtype=abi.RESULT_DTYPE)
    for v in sorted(abi.VERDICT_NAMES):
        for size, mx in ((1000, 0), (1000, 999), (1000, 1000), (1 << 20, 1 << 20)):
            r["verdict"], r["size_bytes"] = v, size
            assert engine.Engine.kafka_error_code(r, mx) == reference_code(v, size, mx), (abi.VERDICT_NAMES[v], size, mx)


def test_decomp_scratch_scales_with_the_arena(built):
    """the block-parallel zstd pool is sized for the arena (at most 64
    blocks per frame, one frame per batch), so a one-batch decompress no longer
    reserves the 65,536-block pool (4.4 MB); the scratch grows with n and
    stays below the whole-arena layouts' sum (no device needed)."""
    from redpanda_amd import abi

    f = abi.lib().rpgpu_decomp_scratch_bytes
    assert f(1) < 1 << 20
    sizes = [f(n) for n in (1, 16, 1024, 65536, 131072)]
    assert sizes == sorted(sizes)
    assert f(131072) < 1 << 30
