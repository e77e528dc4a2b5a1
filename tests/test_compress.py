"""Encode side: storage::internal::compress_batch
(storage/parser_utils.cc:89-128) over compression::compressor::compress.
LZ4 frame and snappy-java are byte-identical to the reference's loops over
liblz4 1.9.3 / snappy 1.1.8: the host build of the engine's restatements
(rpgpu_lz4c.h, rpgpu_snappyc.h) is fuzzed against the oracle
(tests/native/compress_fuzz.cpp; gzip and zstd, rpgpu_deflatec.h /
rpgpu_zstdc.h, are round-tripped there through zlib / libzstd and the
engine's decoders), and the GPU path
(rpgpu_compress_plan_device / _run_device) is compared batch by batch with the
oracle's compress_batch and round-tripped through the GPU decompressor."""
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(__file__))
from kafka_batches import DISK, WIRE, arena, batch, record  # noqa: E402

import oracle.oracle as orc  # noqa: E402
from redpanda_amd import abi  # noqa: E402

ROOT = Path(__file__).resolve().parents[1]
CONDA = "/opt/conda"


def build_fuzzer(tmp: Path, san: bool = False) -> Path:
    lib = orc.build()
    exe = tmp / ("compress_fuzz_san" if san else "compress_fuzz")
    flags = ["-fsanitize=address,undefined", "-static-libstdc++", "-fno-sanitize-recover=undefined", "-g", "-O1"] \
        if san else ["-O2"]
    r = subprocess.run(["g++", "-std=c++17", *flags, f"-I{ROOT / 'redpanda_amd' / 'csrc'}", f"-I{ROOT / 'include'}",
                        f"-I{CONDA}/include", str(ROOT / "tests" / "native" / "compress_fuzz.cpp"), "-o", str(exe),
                        f"-L{lib.parent}", "-lrporacle", f"-Wl,-rpath,{lib.parent}", f"-Wl,-rpath,{CONDA}/lib"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    return exe


@pytest.mark.parametrize("seed", [71, 72])
def test_compress_restatement_matches_oracle(tmp_path, seed):
    exe = build_fuzzer(tmp_path)
    r = subprocess.run([str(exe), "--cases", "250", "--seed", str(seed)], cwd=tmp_path, capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "engine == oracle" in r.stdout


def test_compress_restatement_asan_ubsan(tmp_path):
    exe = build_fuzzer(tmp_path, san=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([str(exe), "--cases", "60", "--seed", "73"], cwd=tmp_path, capture_output=True, text=True,
                       timeout=1200, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-6000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr


def mixed_arena(seed, nb, fmt):
    """Uncompressed batches of varied shape (empty bodies, 1 KiB .. 300 KiB),
    a few already compressed (skipped) and a few corrupted (skipped)."""
    rng = np.random.default_rng(seed)
    words = [b"kafka", b"redpanda", b"offset", b"batch", b"the", b"log", b"segment", b"x"]
    bs = []
    for i in range(nb):
        nrec = int(rng.choice([0, 1, 3, 20, 200, 1500])) if i % 9 else 0
        vlen = int(rng.integers(0, 300))
        recs = []
        for j in range(nrec):
            v = b" ".join(words[k] for k in rng.integers(0, len(words), vlen // 5 + 1))[:vlen] if i % 2 else \
                bytes(rng.integers(0, 256 if i % 3 == 0 else 26, vlen, dtype=np.uint8))
            recs.append(record(b"key%d" % (j % 7), v, ts_delta=j, off_delta=j))
        b = bytearray(batch(recs, fmt=fmt, base_offset=1000 * i, btype=1 + i % 5 if fmt == DISK else 1))
        if i % 17 == 5:
            b = bytearray(batch(orc.compress(3, b"".join(recs)), fmt=fmt, record_count=nrec, attrs=3))
        if i % 23 == 7:
            b[-1] ^= 1
        bs.append(bytes(b))
    return arena(bs, fmt=fmt, ops=abi.OPS_PRODUCE)


def test_oracle_compress_round_trip():
    data, descs = mixed_arena(1, 40, DISK)
    res, _, _ = orc.validate_arena(data, descs)
    for codec in (2, 3):
        comp = orc.compress_batches(data, descs, res, codec)
        for i, c in enumerate(comp):
            if c is None:
                continue
            v, body = orc.uncompress(codec, c[61:], cap=1 << 24)
            o = int(descs["offset"][i])
            assert v == 0 and body == data[o + 61:o + int(res["size_bytes"][i])].tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("codec", [2, 3])
@pytest.mark.parametrize("fmt", [WIRE, DISK])
def test_gpu_compress_matches_oracle(eng, codec, fmt):
    data, descs = mixed_arena(10 + codec, 150, fmt)
    got = eng.compress_arena(data, descs, codec)
    res = got["results"]
    want = orc.compress_batches(data, descs, res, codec)
    cres = got["cres"]
    for i, w in enumerate(want):
        if w is None:
            assert cres["verdict"][i] == abi.V_SKIPPED, i
            continue
        assert cres["verdict"][i] == 0, (i, cres["verdict"][i])
        o, n = int(cres["out_offset"][i]), 61 + int(cres["out_len"][i])
        assert got["out"][o:o + n].tobytes() == w, f"batch {i} differs"
        assert got["out_results"]["verdict"][i] == 0
    # round trip: the compressed batches decompress (on the GPU) to the originals
    ok = np.nonzero(cres["verdict"] == 0)[0]
    od = got["out_descs"][ok].copy()
    od["ops"] = abi.OPS_PRODUCE | abi.OP_DECOMP
    back = eng.decompress_arena(got["out"], od)
    assert (back["dres"]["verdict"] == 0).all()
    for k, i in enumerate(ok):
        a, m = int(back["dres"]["out_offset"][k]), int(back["dres"]["out_len"][k])
        s = int(descs["offset"][i])
        assert back["out"][a + 61:a + 61 + m].tobytes() == data[s + 61:s + int(res["size_bytes"][i])].tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("codec", [2, 3])
def test_gpu_compress_generated(eng, codec):
    """Builder arena: 3000 text batches of 1-64 KiB bodies."""
    from redpanda_amd import engine

    spec = engine.make_spec(seed=0xC0DEC + codec, partitions=8, body_min=1000, body_max=64000, format=DISK,
                            ops=abi.OPS_PRODUCE, payload=abi.PAYLOAD_TEXT)
    data, descs = engine.build_arena(spec, 3000)
    got = eng.compress_arena(data, descs, codec)
    want = orc.compress_batches(data, descs, got["results"], codec)
    cres = got["cres"]
    bad = [i for i, w in enumerate(want)
           if w is not None and got["out"][int(cres["out_offset"][i]):int(cres["out_offset"][i]) + 61 +
                                           int(cres["out_len"][i])].tobytes() != w]
    assert not bad, bad[:8]
    assert (cres["verdict"] == 0).sum() > 2900


@pytest.mark.gpu
@pytest.mark.parametrize("codec", [1, 4])
@pytest.mark.parametrize("fmt", [WIRE, DISK])
def test_gpu_compress_round_trip_gzip_zstd(eng, codec, fmt):
    """gzip / zstd: valid streams (not the libraries' bytes) -- the payload
    decodes to the records bytes with zlib / libzstd through the reference's
    loops and with the GPU decoder; the header fields are compress_batch's."""
    import struct

    data, descs = mixed_arena(20 + codec, 120, fmt)
    got = eng.compress_arena(data, descs, codec)
    res, cres = got["results"], got["cres"]
    want = orc.compress_batches(data, descs, res, 3)  # only for which batches are compressed
    for i, w in enumerate(want):
        if w is None:
            assert cres["verdict"][i] == abi.V_SKIPPED, i
            continue
        assert cres["verdict"][i] == 0, (i, cres["verdict"][i])
        o, m = int(cres["out_offset"][i]), int(cres["out_len"][i])
        b = got["out"][o:o + 61 + m].tobytes()
        s = int(descs["offset"][i])
        body = data[s + 61:s + int(res["size_bytes"][i])].tobytes()
        v, dec = orc.uncompress(codec, b[61:], cap=len(body) + 1024)
        assert v == 0 and dec == body, i
        # every header field but crc / header_crc / size / attrs equals the oracle's (LZ4) rewrite
        hw = np.frombuffer(w[:61], dtype=abi.RP_HEADER_DTYPE)[0]
        hg = np.frombuffer(b[:61], dtype=abi.RP_HEADER_DTYPE)[0]
        assert int(hg["size_bytes"]) == 61 + m and int(hg["attrs"]) == (int(hw["attrs"]) & ~7) | codec
        for f in ("base_offset", "type", "last_offset_delta", "first_timestamp", "max_timestamp", "producer_id",
                  "producer_epoch", "base_sequence", "record_count"):
            assert hg[f] == hw[f], f
        assert int(hg["crc"]) == orc.crc_record_batch(hg, b[61:])
        assert int(hg["header_crc"]) == orc.internal_header_only_crc(hg)
    ok = np.nonzero(cres["verdict"] == 0)[0]
    od = got["out_descs"][ok].copy()
    od["ops"] = abi.OPS_PRODUCE | abi.OP_DECOMP
    back = eng.decompress_arena(got["out"], od)
    assert (back["dres"]["verdict"] == 0).all()
    for k, i in enumerate(ok):
        a, m = int(back["dres"]["out_offset"][k]), int(back["dres"]["out_len"][k])
        s = int(descs["offset"][i])
        assert back["out"][a + 61:a + 61 + m].tobytes() == data[s + 61:s + int(res["size_bytes"][i])].tobytes()
