"""Builds the in-tree native libraries.

librpgpu.so  — HIP kernels + the C ABI (include/rpgpu.h), hipcc for gfx950.
librpgen.so  — the synthetic batch builder (host C++, links the codec libs).

Both land next to this file so a `gpurun` snapshot carries them to the GPU box.
"""
from __future__ import annotations

import os
import subprocess
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
INCLUDE = ROOT / "include"
CONDA = Path(os.environ.get("RPGPU_CODEC_PREFIX", "/opt/conda"))
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")

LIBRPGPU = PKG / "librpgpu.so"
LIBRPGEN = PKG / "librpgen.so"

RPGPU_SRCS = ["rpgpu_kernels.hip", "rpgpu_decomp.hip", "rpgpu_sets.hip", "rpgpu_index.hip", "rpgpu_summary.hip", "rpgpu_compact.hip", "rpgpu_compact_rw.hip", "rpgpu_fetch.hip", "rpgpu_compress.hip", "rpgpu_stamp.hip", "rpgpu_abi.cpp", "rpgpu_tables.cpp"]
RPGPU_HDRS = ["rpgpu_internal.h", "rpgpu_device.h", "rpgpu_walk.h", "rpgpu_codec.h", "rpgpu_zstd.h", "rpgpu_zseq.h", "rpgpu_zblk.h", "rpgpu_wave.h", "rpgpu_inflate.h", "rpgpu_lz4c.h", "rpgpu_snappyc.h", "rpgpu_deflatec.h", "rpgpu_zstdc.h"]
RPGEN_SRCS = ["rpgen.cpp"]
RPGEN_HDRS = ["rpgen.h"]


def _stale(out: Path, srcs: list[Path]) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(s.stat().st_mtime > t for s in srcs)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def build_rpgpu(force: bool = False) -> Path:
    srcs = [CSRC / s for s in RPGPU_SRCS + RPGPU_HDRS] + [INCLUDE / "rpgpu.h"]
    if force or _stale(LIBRPGPU, srcs):
        # one hipcc per translation unit, in parallel, then one link
        from concurrent.futures import ThreadPoolExecutor

        obj = ROOT / "build" / "obj"
        obj.mkdir(parents=True, exist_ok=True)
        flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", f"-I{INCLUDE}", f"-I{CSRC}"]
        objs = [obj / (s + ".o") for s in RPGPU_SRCS]
        jobs = max(1, min(len(objs), os.cpu_count() or 1, 8))
        with ThreadPoolExecutor(jobs) as ex:
            list(ex.map(lambda so: _run(["hipcc", *flags, "-c", str(CSRC / so[0]), "-o", str(so[1])]),
                        zip(RPGPU_SRCS, objs)))
        tmp = LIBRPGPU.with_suffix(".so.tmp")
        _run(["hipcc", f"--offload-arch={ARCH}", "-shared", *[str(o) for o in objs], "-o", str(tmp)])
        os.replace(tmp, LIBRPGPU)
    return LIBRPGPU


def build_rpgen(force: bool = False) -> Path:
    srcs = [CSRC / s for s in RPGEN_SRCS + RPGEN_HDRS] + [INCLUDE / "rpgpu.h"]
    if force or _stale(LIBRPGEN, srcs):
        tmp = LIBRPGEN.with_suffix(".so.tmp")
        _run(["g++", "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread",
              f"-I{INCLUDE}", f"-I{CSRC}", f"-I{CONDA / 'include'}",
              *[str(CSRC / s) for s in RPGEN_SRCS],
              f"-L{CONDA / 'lib'}", f"-Wl,-rpath,{CONDA / 'lib'}",
              "-llz4", "-lzstd", "-lsnappy", "-lz", "-o", str(tmp)])
        os.replace(tmp, LIBRPGEN)
    return LIBRPGEN


def build_all(force: bool = False) -> None:
    build_rpgpu(force)
    build_rpgen(force)


if __name__ == "__main__":
    build_all(force=True)
    print("built", LIBRPGPU, LIBRPGEN)
