"""GPU parity of the decompress path (rpgpu_decomp_plan_device /
rpgpu_decomp_run_device and the rpgpu_uncompress scalar mirror) against the
oracle: compression::compressor::uncompress (compression/compression.cc:35-55)
over zlib / liblz4 / snappy / libzstd through the reference's wrapper loops, the batch rewrite
of maybe_decompress_batch_sync (storage/parser_utils.cc:52-68,122-128) and the
record walk of the rewritten batches.  Compared per batch: decompress verdict,
decoded length, the rewritten batch's bytes (header with fresh CRCs + body),
its validation result and its index entries."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(__file__))
from kafka_batches import DISK, WIRE, arena, batch, record  # noqa: E402

import oracle.oracle as orc  # noqa: E402

pytestmark = pytest.mark.gpu

OPS = 1 | 2 | 4 | 8 | 16  # CRC | HDRCRC | PARSE | INDEX | DECOMP


def compare(got, data, descs, nthreads=1):
    from redpanda_amd import abi

    res, dres = got["results"], got["dres"]
    wres, _, _ = orc.validate_arena(data, descs, nthreads=nthreads)
    assert np.array_equal(res.view(np.uint8), wres.view(np.uint8)), "validation results differ"
    caps = np.where(dres["out_cap"] > 0, dres["out_cap"].astype(np.int64) - 61 - 128, 0).astype(np.uint64)
    want = orc.decompress_arena(data, descs, wres, caps, codecs=(1, 2, 3, 4), nthreads=nthreads)
    bad = np.nonzero(dres["verdict"] != want["verdicts"])[0]
    assert bad.size == 0, (f"decompress verdicts differ at {bad[:8]}: gpu {dres['verdict'][bad[:8]]} "
                           f"oracle {want['verdicts'][bad[:8]]}")
    ok = np.nonzero(dres["verdict"] == abi.V_OK)[0]
    assert np.array_equal(dres["out_len"][ok], want["out_len"][ok]), "decoded lengths differ"
    for i in ok:
        a = int(dres["out_offset"][i])
        b = int(want["out_descs"]["offset"][i])
        m = 61 + int(dres["out_len"][i])
        assert np.array_equal(got["out"][a:a + m], want["out"][b:b + m]), f"rewritten batch {i} differs"
    ores, wores = got["out_results"], want["out_results"]
    for f in abi.RESULT_DTYPE.names:
        bad = np.nonzero(ores[f] != wores[f])[0]
        assert bad.size == 0, f"rewritten-batch field {f} differs at {bad[:8]}: {ores[f][bad[:8]]} vs {wores[f][bad[:8]]}"
    assert got["used"] == want["used"]
    assert np.array_equal(got["index"].view(np.uint8), want["index"].view(np.uint8)), "index differs"
    return want


def records(rng, n, key_len, value_len, text):
    out = []
    for j in range(n):
        if text:
            words = [b"kafka", b"redpanda", b"offset", b"batch", b"the", b"log", b"segment", b"x"]
            v = b" ".join(words[k] for k in rng.integers(0, len(words), value_len // 5 + 1))[:value_len]
        else:
            v = bytes(rng.integers(97, 123, value_len, dtype=np.uint8))
        k = bytes(rng.integers(65, 91, key_len, dtype=np.uint8)) if key_len >= 0 else None
        out.append(record(k, v, ts_delta=j, off_delta=j,
                          headers=[(b"h", b"v" * int(rng.integers(0, 5)))] if j % 3 == 0 else []))
    return out


@pytest.mark.parametrize("codec", [1, 2, 3, 4])
@pytest.mark.parametrize("fmt", [WIRE, DISK])
def test_generated_arenas(eng, codec, fmt):
    """Builder arenas (rpgen: the reference's compressor settings), text and alnum payloads."""
    from redpanda_amd import abi, engine

    for payload, shape in ((abi.PAYLOAD_TEXT, (12, 8, 700)), (abi.PAYLOAD_ALNUM, (5, 16, 3000))):
        spec = engine.make_spec(seed=0x5EED0003 + codec, partitions=4, records_per_batch=shape[0],
                                key_len=shape[1], value_len=shape[2], codec=codec, format=fmt,
                                ops=abi.OPS_PRODUCE | abi.OP_DECOMP, payload=payload)
        data, descs = engine.build_arena(spec, 48)
        got = eng.decompress_arena(data, descs)
        compare(got, data, descs)
        assert (got["dres"]["verdict"] == abi.V_OK).all()


def test_mixed_codecs_corrupted(eng):
    """C5-shaped arena: none/gzip/snappy/lz4/zstd, skewed sizes, 1-in-4 corrupted batches."""
    from redpanda_amd import abi, engine

    spec = engine.make_spec(seed=0x5EED0005, partitions=16, codec_mix=0x1F,
                            body_min=7, body_max=300_000, ops=abi.OPS_PRODUCE | abi.OP_DECOMP,
                            payload=abi.PAYLOAD_TEXT, corrupt_ppm=250_000, corrupt_mask=0x3FF)
    data, descs = engine.build_arena(spec, 160)
    got = eng.decompress_arena(data, descs)
    compare(got, data, descs)
    v = got["dres"]["verdict"]
    assert (v == abi.V_DECOMP_UNSUPPORTED).sum() == 0
    assert (v == abi.V_OK).sum() > 10
    codec = got["dres"]["codec"]
    assert ((v == abi.V_OK) & (codec == 4)).sum() > 0
    assert ((v == abi.V_OK) & (codec == 1)).sum() > 0


def mutated_bodies(rng, codec, n):
    """Compressed bodies (whole-frame or chunk level) mutated the ways a bad
    producer or a bit flip would: truncation anywhere / at LZ4 block ends,
    flipped bytes, trailing junk, altered lengths; re-CRC'd by batch()."""
    out = []
    for i in range(n):
        recs = records(rng, int(rng.integers(1, 40)), int(rng.integers(-1, 20)),
                       int(rng.integers(0, 3000)), text=bool(i % 2))
        body = b"".join(recs)
        comp = bytearray(orc.compress(codec, body))
        kind = i % 7
        if kind == 1:
            comp = comp[:int(rng.integers(0, len(comp) + 1))]
        elif kind == 2 and len(comp) > 0:
            for _ in range(int(rng.integers(1, 4))):
                comp[int(rng.integers(0, len(comp)))] ^= int(rng.integers(1, 256))
        elif kind == 3:
            comp += bytes(rng.integers(0, 256, int(rng.integers(1, 9)), dtype=np.uint8))
        elif kind == 4 and codec == 3 and len(comp) > 11:
            comp = comp[:-4]  # no end mark: truncated right after the last block
        elif kind == 4 and codec in (1, 4):
            comp += orc.compress(codec, body[: len(body) // 2])  # a second frame / gzip member
        elif kind == 5 and len(comp) > 20:
            k = int(rng.integers(16, len(comp)))
            comp[k] = 0xFF
        out.append((bytes(comp), len(recs)))
    return out


@pytest.mark.parametrize("codec", [1, 2, 3, 4])
@pytest.mark.parametrize("fmt", [WIRE, DISK])
def test_mutated_payloads(eng, codec, fmt):
    rng = np.random.default_rng(100 + codec * 2 + fmt)
    bs = [batch(c, fmt=fmt, record_count=rc, attrs=codec) for c, rc in mutated_bodies(rng, codec, 70)]
    data, descs = arena(bs, fmt=fmt, ops=OPS)
    compare(eng.decompress_arena(data, descs), data, descs)


def test_large_bodies(eng):
    """~1 MiB bodies: many 64 KiB LZ4 blocks, several 128 KiB snappy-java chunks,
    zstd frames larger than the 64 KiB staging buffer (streamed block by block)."""
    rng = np.random.default_rng(7)
    bs = []
    for codec in (2, 3, 3, 2, 4, 4, 1, 1):
        recs = records(rng, 900, 8, 1100, text=codec == 3)
        bs.append(batch(orc.compress(codec, b"".join(recs)), fmt=WIRE, record_count=len(recs), attrs=codec))
    data, descs = arena(bs, fmt=WIRE, ops=OPS)
    compare(eng.decompress_arena(data, descs), data, descs)


def test_large_bodies_split_fallback(eng):
    """~1 MiB LZ4 frames (independent 64 KiB blocks) and snappy-java bodies
    (128 KiB chunks) decoded one part per lane (rpcodec::lz4f_split /
    snappy_java_split), clean and damaged so that a part fails (a flipped or
    0xFF byte inside a block / chunk: the batch goes back to the serial
    decoder) or no plan is made (cut short, trailing junk): every verdict,
    length and byte as the oracle's."""
    rng = np.random.default_rng(11)
    bs = []
    for codec in (3, 2):
        for kind in range(6):
            recs = records(rng, 900, 8, 1100, text=True)
            comp = bytearray(orc.compress(codec, b"".join(recs)))
            n = len(comp)
            if kind == 1:
                comp[n // 2] ^= 0x5A
            elif kind == 2:
                comp[n - 40] ^= 0x01
            elif kind == 3:
                comp = comp[: int(n * 0.6)]
            elif kind == 4:
                comp += b"\x00junk"
            elif kind == 5:
                comp[n // 3] = 0xFF
            bs.append(batch(bytes(comp), fmt=WIRE, record_count=len(recs), attrs=codec))
    data, descs = arena(bs, fmt=WIRE, ops=OPS)
    compare(eng.decompress_arena(data, descs, runs=3), data, descs)


def test_split_parts_overflow(eng):
    """more split parts than the part list holds ((n + 4096) / 2 per
    codec).  320 ~1 MiB LZ4 bodies of 16 independent 64 KiB blocks each (5,120
    parts) plus damaged and small ones: the bodies whose parts do not fit go
    to the serial decoders; nothing decodes from a stale or unwritten part
    record; every verdict, length and byte as the oracle's, also when the plan
    is run three times."""
    rng = np.random.default_rng(23)
    recs = records(rng, 900, 8, 1100, text=True)
    body = b"".join(recs)
    clean = orc.compress(3, body)
    bs = []
    for i in range(320):
        comp = bytearray(clean)
        if i % 37 == 5:
            comp[len(comp) // 2] ^= 0x5A  # a part fails: serial fallback
        bs.append(batch(bytes(comp), fmt=WIRE, record_count=len(recs), attrs=3, base_offset=i * 1000))
        if i % 16 == 0:  # small batches in between (lane decoders)
            small = records(rng, 4, 4, 200, text=True)
            bs.append(batch(orc.compress(3, b"".join(small)), fmt=WIRE, record_count=4, attrs=3))
    data, descs = arena(bs, fmt=WIRE, ops=OPS)
    compare(eng.decompress_arena(data, descs, runs=3), data, descs)


def test_many_tiny_zstd_gzip(eng):
    """more zstd / gzip batches than the engine runs decoders for
    at once (131,072), ~100-400 B bodies, so decoders are reused across frames;
    1 in 200 batches corrupted.  Every verdict, length, rewritten byte and
    index entry as the oracle's."""
    from redpanda_amd import abi, engine

    spec = engine.make_spec(seed=0x5EED0077, partitions=64, codec_mix=(1 << 4) | (1 << 1), body_min=100,
                            body_max=400, ops=abi.OPS_PRODUCE | abi.OP_DECOMP, payload=abi.PAYLOAD_TEXT,
                            corrupt_ppm=5_000, corrupt_mask=0x3FF)
    data, descs = engine.build_arena(spec, 150_000)
    got = eng.decompress_arena(data, descs)
    compare(got, data, descs)
    v, codec = got["dres"]["verdict"], got["dres"]["codec"]
    assert ((v == abi.V_OK) & (codec == 4)).sum() > 131_072 // 2
    assert ((v == abi.V_OK) & (codec == 1)).sum() > 131_072 // 2


def zstd_workspace_bytes(got):
    """Output bytes past the slots (rounded to 256): the zstd lane workspaces."""
    d = got["dres"]
    end = int((d["out_offset"].astype(np.int64) + d["out_cap"].astype(np.int64))[d["out_cap"] > 0].max(initial=0))
    return got["out_bytes"] - ((end + 255) & ~255) if got["out_bytes"] > end else 0


def test_few_workspace_lanes():
    """rpgpu_opts.decomp_ws_lanes = 256: a mixed arena with 6,000 zstd / gzip
    batches still decodes exactly as the oracle, each of the 256 workspace
    lanes taking ~20 frames in turn; the plan's output bytes hold 256 zstd
    workspaces, the scratch only gzip's (the one-lane zstd decoder: the split
    decoder off)."""
    from redpanda_amd import abi, engine

    spec = engine.make_spec(seed=0x5EED0078, partitions=32, codec_mix=(1 << 4) | (1 << 1) | (1 << 3),
                            body_min=100, body_max=20_000, ops=abi.OPS_PRODUCE | abi.OP_DECOMP,
                            payload=abi.PAYLOAD_TEXT, corrupt_ppm=5_000, corrupt_mask=0x3FF)
    data, descs = engine.build_arena(spec, 9000)
    with engine.Engine(0, decomp_ws_lanes=256) as e:
        n = 200_000
        assert e.decomp_scratch_bytes(n) < abi.lib().rpgpu_decomp_scratch_bytes(n)
        got = e.decompress_arena(data, descs)
    compare(got, data, descs)
    v, codec = got["dres"]["verdict"], got["dres"]["codec"]
    assert ((v == abi.V_OK) & ((codec == 4) | (codec == 1))).sum() > 5000
    ws = zstd_workspace_bytes(got)
    assert ws % 256 == 0 and 8 << 10 < ws // 256 < 32 << 10, ws


def test_zstd_workspaces_follow_the_plan():
    """the zstd lane workspaces sit after the output slots,
    one per zstd lane batch the plan found (up to the cap): an LZ4 / snappy
    arena's output is its slots alone and the scratch holds no zstd workspace;
    k zstd batches add k workspaces; every batch decodes as the oracle (the
    one-lane zstd decoder: the split decoder off)."""
    from redpanda_amd import abi, engine

    eng = engine.Engine(0)

    assert abi.lib().rpgpu_decomp_scratch_bytes(131072) < 1 << 30  # was ~2.6 GB with them
    rng = np.random.default_rng(29)
    per = []
    for codecs, k in (((3, 2), 0), ((3, 4), 9), ((4,), 23)):
        bodies = []
        for j in range(40 if k == 0 else k + 15):
            c = codecs[j % len(codecs)] if k == 0 else (4 if j < k else 3)
            bodies.append((orc.compress(c, b"".join(records(rng, 12, 4, 200, text=True))), c))
        bs = [batch(b, fmt=WIRE, record_count=12, attrs=c) for b, c in bodies]
        data, descs = arena(bs, fmt=WIRE, ops=OPS)
        got = eng.decompress_arena(data, descs)
        compare(got, data, descs)
        assert (got["dres"]["verdict"] == abi.V_OK).all()
        ws = zstd_workspace_bytes(got)
        if k == 0:
            assert ws == 0, ws
        else:
            assert ws % k == 0, (ws, k)
            per.append(ws // k)
    eng.close()
    assert per[0] == per[1] and 8 << 10 < per[0] < 32 << 10, per


def test_ws_lanes_not_a_multiple_of_256():
    """decomp_ws_lanes = 300 (not a whole number of 256-lane
    workgroups) on a mixed zstd / gzip / LZ4 arena with split ~1 MiB LZ4
    bodies and more batches than lanes: no workspace lies past the scratch's
    workspace region (the cap is rounded up to 512 lanes), so the split parts
    and their results beside it stay intact; every verdict, length and byte as
    the oracle's."""
    from redpanda_amd import abi, engine

    spec = engine.make_spec(seed=0x5EED0079, partitions=32, codec_mix=(1 << 4) | (1 << 1) | (1 << 3),
                            body_min=100, body_max=1 << 20, ops=abi.OPS_PRODUCE | abi.OP_DECOMP,
                            payload=abi.PAYLOAD_TEXT, corrupt_ppm=5_000, corrupt_mask=0x3FF)
    data, descs = engine.build_arena(spec, 1400)
    with engine.Engine(0, decomp_ws_lanes=512) as e:
        want_scratch = e.decomp_scratch_bytes(100_000)
    with engine.Engine(0, decomp_ws_lanes=300) as e:
        assert e.decomp_scratch_bytes(100_000) == want_scratch
        got = e.decompress_arena(data, descs, runs=2)
    compare(got, data, descs, nthreads=8)
    v, codec = got["dres"]["verdict"], got["dres"]["codec"]
    assert ((v == abi.V_OK) & ((codec == 4) | (codec == 1))).sum() > 600


def test_decompress_batch_header_room(eng):
    """rpgpu_decompress_batch with less room than the 61-byte
    rewritten header (an empty LZ4 / zstd frame decodes to 0 bytes) reports
    DECOMP_OVERFLOW with the capacity it needs instead of writing the header
    past the caller's buffer."""
    from redpanda_amd import abi

    for codec in (3, 4):
        b = batch(orc.compress(codec, b""), fmt=WIRE, record_count=0, attrs=codec)
        for cap in (0, 1, 60):
            gv, _, glen = eng.decompress_batch(b, WIRE, cap=cap)
            assert gv == abi.V_DECOMP_OVERFLOW and glen == 61, (codec, cap, gv, glen)
        gv, out, glen = eng.decompress_batch(b, WIRE, cap=61)
        assert gv == abi.V_OK and glen == 61 and len(out) == 61


def test_uncompress_scalar_mirror(eng):
    rng = np.random.default_rng(3)
    cases = []
    for codec in (1, 2, 3, 4):
        for c, _ in mutated_bodies(rng, codec, 40):
            cases.append((codec, c))
    gz = orc.compress(1, b"hello gzip " * 50)
    cases += [(1, b""), (1, gz[:10]), (1, gz[:-8]), (1, gz[:-4]), (1, b"\x78\x9c\x03\x00\x00\x00\x00\x01"),
              (1, b"\x78\x9c\x03\x00"), (1, b"\x1f\x8b\x08\x00"), (1, b"\x1f\x8b\x07\x00" + gz[4:])]
    cases += [(3, b""), (2, b""), (4, b""), (0, b"abc"), (3, b"\x04\x22\x4d"), (2, b"\x00"),
              (4, b"\x28\xb5\x2f\xfd"), (4, b"\x28\xb5\x2f\xfd\x00"), (4, b"\x50\x2a\x4d\x18\x00\x00\x00\x00")]
    for codec, c in cases:
        gv, gout = eng.uncompress(codec, c, cap=1 << 21)
        ov, oout = orc.uncompress(codec, c, cap=1 << 21)
        assert gv == ov, (codec, len(c), gv, ov)
        if ov == 0:
            assert gout == oout, (codec, len(c))


def test_zstd_window_limits(eng):
    """Frames past the 8 MiB static workspace (windowLog 24, content size
    unknown: ZSTD_error_memory_allocation) and past ZSTD_MAXWINDOWSIZE_DEFAULT
    (windowLog 28: frameParameter_windowTooLarge) are DECOMP_ERROR like every
    zstd error (stream_zstd.cc:29-36: the bad_alloc branch never matches);
    with a content size the staging buffer holds, the single-pass decode
    takes them.  Scalar mirror and arena path, against the oracle."""
    from redpanda_amd import abi
    from test_zstd_window import window_cases

    cases = list(window_cases())
    for name, frame, want in cases:
        gv, gout = eng.uncompress(4, frame, cap=1 << 20)
        ov, oout = orc.uncompress(4, frame, cap=1 << 20)
        assert ov == want and gv == ov, (name, gv, ov)
        if ov == abi.V_OK:
            assert gout == oout, name
    wanted = {n: w for n, _, w in cases}
    assert wanted["wlog24_nofcs"] == abi.V_DECOMP_ERROR and wanted["wlog28_fcs100k"] == abi.V_DECOMP_ERROR
    # the same frames as record bodies of an arena (payload bytes only: the
    # walk of a decoded OK batch then reports its record verdict)
    bs = [batch(frame, fmt=WIRE, record_count=0, attrs=4) for _, frame, _ in cases]
    data, descs = arena(bs, fmt=WIRE, ops=OPS)
    compare(eng.decompress_arena(data, descs), data, descs)


def rle_frame(blocks: int, content_size: bool) -> bytes:
    """A zstd frame of `blocks` RLE blocks of 128 KiB each (4 bytes apiece on
    the wire): the worst output-per-input-byte a frame can claim."""
    import struct

    bh = struct.pack("<I", (1 << 1) | ((128 << 10) << 3))[:3]  # RLE block, 131072 bytes
    last = struct.pack("<I", 1 | (1 << 1) | ((128 << 10) << 3))[:3]
    body = b"".join(bh + b"x" for _ in range(blocks - 1)) + last + b"y"
    if content_size:
        return b"\x28\xb5\x2f\xfd" + bytes([0x80, (17 - 10) << 3]) + struct.pack("<I", blocks << 17) + body
    return b"\x28\xb5\x2f\xfd" + bytes([0x00, (17 - 10) << 3]) + body


def test_decoded_size_ceiling(built):
    """a batch whose decoded-size bound exceeds the per-batch
    ceiling (opts.max_decoded_batch) gets DECOMP_OVERFLOW and no output slot;
    every other batch of the arena -- before and after it -- decodes as the
    oracle does, and the plan does not grow by the hostile batch's bound."""
    from redpanda_amd import abi, engine

    with engine.Engine(0, max_decoded_batch=4 << 20) as e:
        rng = np.random.default_rng(17)
        good = [(orc.compress(c, b"".join(records(rng, 20, 4, 300, text=True))), c) for c in (3, 4, 2, 4)]
        hostile = rle_frame(64, content_size=False)  # 8 MiB of output from 266 bytes
        bodies = good[:2] + [(hostile, 4)] + good[2:]
        bs = [batch(c, fmt=WIRE, record_count=20, attrs=codec) for c, codec in bodies]
        data, descs = arena(bs, fmt=WIRE, ops=OPS)
        got = e.decompress_arena(data, descs)
        v = got["dres"]["verdict"]
        assert v[2] == abi.V_DECOMP_OVERFLOW and got["dres"]["out_cap"][2] == 0
        assert got["out_bytes"] < 2 << 20
        keep = np.array([0, 1, 3, 4])
        data2, descs2 = arena([bs[i] for i in keep], fmt=WIRE, ops=OPS)
        want = compare(e.decompress_arena(data2, descs2), data2, descs2)
        assert np.array_equal(v[keep], want["verdicts"])
        assert np.array_equal(got["dres"]["out_len"][keep], want["out_len"])
        # the arena reports the capacity a retry needs (the frame's bound)
        need = int(got["dres"]["out_len"][2])
        assert need >= 8 << 20
        # the scalar mirror applies the same ceiling to a caller buffer below the bound ...
        gv, _ = e.uncompress(4, hostile, cap=1 << 20)
        assert gv == abi.V_DECOMP_OVERFLOW and e.last_out_len == need
        # ... and decodes when the caller supplies the capacity (the retry)
        gv, gout = e.uncompress(4, hostile, cap=need)
        ov, oout = orc.uncompress(4, hostile, cap=16 << 20)
        assert gv == ov == abi.V_OK and gout == oout
    # under the default ceiling the same frame decodes, as the oracle does
    gv, gout = eng_default_uncompress(hostile)
    assert gv == ov == abi.V_OK and gout == oout


def test_overflow_retry_80mib(eng):
    """DECOMP_OVERFLOW is a retry signal, not a rejection.  A valid
    zstd frame decoding to 80 MiB (above the default 64 MiB per-batch ceiling)
    gets no slot in the arena pass and reports the capacity it needs;
    rpgpu_decompress_batch then rewrites it exactly as the oracle's
    maybe_decompress_batch_sync does (rewritten header with fresh CRCs + body)."""
    from redpanda_amd import abi

    rng = np.random.default_rng(80)
    words = [b"kafka ", b"redpanda ", b"offset ", b"batch ", b"segment ", b"raft ", b"log ", b"term "]
    chunk = b"".join(words[k] for k in rng.integers(0, len(words), 40_000))
    body = (chunk * (80 * (1 << 20) // len(chunk) + 1))[:80 << 20]
    big = batch(orc.compress(4, body), fmt=WIRE, record_count=0, attrs=4, base_offset=77)
    small = [batch(orc.compress(c, b"".join(records(rng, 10, 4, 300, text=True))), fmt=WIRE, record_count=10,
                   attrs=c) for c in (3, 4)]
    bs = [small[0], big, small[1]]
    data, descs = arena(bs, fmt=WIRE, ops=OPS)
    got = eng.decompress_arena(data, descs)
    v = got["dres"]["verdict"]
    assert v[1] == abi.V_DECOMP_OVERFLOW and got["dres"]["out_cap"][1] == 0
    assert v[0] == v[2] == abi.V_OK
    need = int(got["dres"]["out_len"][1])
    assert need >= 80 << 20
    gv, gout, glen = eng.decompress_batch(big, WIRE, cap=61 + need)
    assert gv == abi.V_OK and glen == 61 + (80 << 20)
    # the oracle's rewrite of the same batch, given the room
    d1 = descs[1:2].copy()
    d1["offset"] = 0
    one = np.frombuffer(big + bytes(64), dtype=np.uint8).copy()
    wres, _, _ = orc.validate_arena(one, d1)
    want = orc.decompress_arena(one, d1, wres, np.array([need], dtype=np.uint64))
    assert want["verdicts"][0] == abi.V_OK
    o = int(want["out_descs"]["offset"][0])
    assert gout == want["out"][o:o + glen].tobytes()
    # a buffer too small: the retry reports the capacity again
    gv, _, glen = eng.decompress_batch(big, WIRE, cap=1 << 20)
    assert gv == abi.V_DECOMP_OVERFLOW and glen >= 61 + (80 << 20)


def eng_default_uncompress(frame):
    from redpanda_amd import engine

    with engine.Engine(0) as e:
        return e.uncompress(4, frame, cap=16 << 20)


@pytest.mark.parametrize("codec", [1, 2, 3, 4])
def test_mutated_payloads_many(eng, codec):
    """Differential fuzz of the wave-cooperative device decoders (rpgpu_wave.h)
    against the oracle: 600 library frames per codec, most of them mutated
    (truncation, flipped bytes, junk, second frames, 0xFF bytes), in one arena."""
    rng = np.random.default_rng(900 + codec)
    bs = [batch(c, fmt=WIRE, record_count=rc, attrs=codec) for c, rc in mutated_bodies(rng, codec, 600)]
    data, descs = arena(bs, fmt=WIRE, ops=OPS)
    compare(eng.decompress_arena(data, descs), data, descs)


def test_zstd_ring_extdict_frames(eng):
    """Crafted zstd frames (tests/golden/make_zstd_ring.py) whose 1 KiB window
    makes the reference loop's ring buffer wrap every two blocks, each with one
    match reaching into the previous ring segment -- where the current segment
    has or has not overwritten it -- or before it (libzstd: corruption_detected):
    8 KiB frames on the lane decoder, ~300 KiB ones on the wave decoder.  Every
    verdict, length and byte as the oracle's (libzstd 1.4.9 through
    stream_zstd::do_uncompress)."""
    from redpanda_amd import abi

    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "zstd_ring.npz"))
    ends = np.cumsum(g["lens"])
    frames = [g["data"][e - n:e].tobytes() for e, n in zip(ends, g["lens"])]
    bs = [batch(f, fmt=WIRE, record_count=1, attrs=4) for f in frames]
    data, descs = arena(bs, fmt=WIRE, ops=OPS)
    got = eng.decompress_arena(data, descs)
    want = compare(got, data, descs)
    v = want["verdicts"]
    assert (v == abi.V_OK).sum() >= 6 and (v == abi.V_DECOMP_ERROR).sum() >= 2, v


def test_zstd_wildcopy_band_frames(eng):
    """crafted zstd frames (tests/golden/make_zstd_ring.py
    `band_*`) with a 1 KiB window whose matches, once the ring has wrapped,
    read the previous segment right past the write position -- where libzstd
    1.4.9's over-long copies (ZSTD_copy16 / ZSTD_wildcopy of literals and
    matches, ZSTD_overlapCopy8, ZSTD_safecopy near the ring's end) left bytes
    that the match then copies.  40 small frames on the lane decoder's ring
    pass, 4 of 400 blocks on the wave decoder: every verdict, length and byte
    as the oracle's (the restatement: rpgpu_zstd.h ring_seq; host differential
    fuzz: tests/native/zstd_fuzz.cpp check_band)."""
    from redpanda_amd import abi

    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "zstd_ring.npz"))
    ends = np.cumsum(g["band_lens"])
    frames = [g["band_data"][e - n:e].tobytes() for e, n in zip(ends, g["band_lens"])]
    bs = [batch(f, fmt=WIRE, record_count=1, attrs=4) for f in frames]
    data, descs = arena(bs, fmt=WIRE, ops=OPS)
    got = eng.decompress_arena(data, descs)
    want = compare(got, data, descs)
    v = want["verdicts"]
    assert (v == abi.V_OK).sum() >= 20, v
    assert (got["dres"]["out_cap"][-4:] > 61 + (256 << 10)).all()  # slots for the wave decoder


def test_zstd_segment_span_frames(eng):
    """crafted zstd frames (tests/golden/make_zstd_ring.py
    `span_*`, tests/native/zstd_fuzz.cpp span_frame) with a 1 KiB window whose
    second ring segment opens with a match that starts in the extDict (the
    previous segment's last bytes) and continues from the current segment's
    start, at a distance below 16 or not (libzstd 1.4.9: ZSTD_execSequence's
    two-part copy, then ZSTD_overlapCopy8 / ZSTD_wildcopy).  The lane
    decoder's ring pass (rpgpu_zstd.h ring_seq) gives every verdict, length and
    byte as the oracle does (host: 1,397 such frames == libzstd in the fuzz)."""
    from redpanda_amd import abi

    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "zstd_ring.npz"))
    ends = np.cumsum(g["span_lens"])
    frames = [g["span_data"][e - n:e].tobytes() for e, n in zip(ends, g["span_lens"])]
    bs = [batch(f, fmt=WIRE, record_count=1, attrs=4) for f in frames]
    data, descs = arena(bs, fmt=WIRE, ops=OPS)
    got = eng.decompress_arena(data, descs)
    want = compare(got, data, descs)
    v = want["verdicts"]
    assert (v == abi.V_OK).sum() >= 60, v


def test_split_fallback_below_wave_size(eng):
    """A corrupt LZ4 frame from C5's arena (batch 126,469 of the bench's seed,
    tests/golden/lz4_split_fallback.npz: 45,806 bytes, two 64 KiB blocks, the
    first decoding to 65,534 bytes) is split (slot above the 80 KiB split
    threshold), its parts do not bear the plan out, and the serial fallback --
    the LZ wave decoder, for a batch below the wave size -- gives the serial
    verdict (DECOMP_ERROR), as the oracle does.  Round 4's first 80 KiB build
    left such batches undecoded."""
    from redpanda_amd import abi

    body = np.load(os.path.join(os.path.dirname(__file__), "golden", "lz4_split_fallback.npz"))["body"].tobytes()
    rng = np.random.default_rng(3)
    good = orc.compress(3, b"".join(records(rng, 40, 4, 3000, text=True)))
    bs = [batch(body, fmt=WIRE, record_count=64, attrs=3), batch(good, fmt=WIRE, record_count=40, attrs=3)]
    data, descs = arena(bs, fmt=WIRE, ops=OPS)
    got = eng.decompress_arena(data, descs)
    want = compare(got, data, descs)
    assert want["verdicts"][0] == abi.V_DECOMP_ERROR and want["verdicts"][1] == abi.V_OK


def lz4_frame(blocks, content=None):
    """An LZ4 frame (independent 64 KiB blocks, no checksums) around the given
    compressed blocks, with or without a content size."""
    import struct

    import xxhash

    desc = bytes([0x60 | (0x08 if content is not None else 0), 0x40])
    desc += struct.pack("<Q", content) if content is not None else b""
    f = struct.pack("<I", 0x184D2204) + desc + bytes([(xxhash.xxh32(desc, seed=0).intdigest() >> 8) & 0xFF])
    for b in blocks:
        f += struct.pack("<I", len(b)) + b
    return f + b"\0\0\0\0"


def lz4_run_block(n, c=b"a", tail=b"12345"):
    """An LZ4 block decoding to n bytes: c, a run of it (offset 1), then tail."""
    import struct

    def ext(r):
        return b"\xff" * (r // 255) + bytes([r % 255])

    return bytes([0x1F]) + c + struct.pack("<H", 1) + ext(n - 1 - len(tail) - 4 - 15) + bytes([len(tail) << 4]) + tail


def test_split_short_block_frames(eng):
    """LZ4 frames whose first (non-final) block decodes to 65,534 bytes: the
    serial decoder places the next block there, not at 64 KiB.  Without a
    content size, or with one the blocks add up to, the split plan's parts
    are misplaced and the LZ wave decoder re-decodes the frame serially (OK,
    161,070 bytes); with a content size they contradict, the parts alone give
    the serial verdict (frameSize_wrong -> DECOMP_ERROR) -- C5's split
    fallbacks, decided in split_finish_kernel since round 6."""
    from redpanda_amd import abi

    rng = np.random.default_rng(5)
    tail = bytes(rng.integers(97, 123, 30000, dtype=np.uint8))
    bl = [lz4_run_block(65534), lz4_run_block(65536, b"b"), bytes([0xF0]) + b"\xff" * 117 + bytes([30000 - 15 - 117 * 255]) + tail]
    frames = [lz4_frame(bl), lz4_frame(bl, 65534 + 65536 + 30000), lz4_frame(bl, 2 * 65536 + 30000)]
    rng = np.random.default_rng(3)
    good = orc.compress(3, b"".join(records(rng, 40, 4, 3000, text=True)))
    bs = [batch(f, fmt=WIRE, record_count=1, attrs=3) for f in frames] + [batch(good, fmt=WIRE, record_count=40, attrs=3)]
    data, descs = arena(bs, fmt=WIRE, ops=OPS)
    got = eng.decompress_arena(data, descs)
    want = compare(got, data, descs)
    assert list(want["verdicts"]) == [abi.V_OK, abi.V_OK, abi.V_DECOMP_ERROR, abi.V_OK]
    assert list(want["out_len"][:2]) == [161070, 161070]


@pytest.mark.parametrize("case", ["tiny", "mixed", "c4", "mutated"])
def test_zstd_lane_decoder_cases(eng, case):
    """The one-lane zstd decoder with its write-combined sequences
    (rpgpu_zstd.h wc_seq) against the oracle: many tiny bodies (more batches
    than the lane kernel's lanes), mixed sizes up to the lane / wave boundary
    with 1 % corruption, the C4 shape (64 x 1 KiB text records at level 3), and
    mutated payloads (verdicts on corrupt frames) -- the cases round 5 ran
    through the split decoder this round removed."""
    from redpanda_amd import abi, engine

    kw = dict(ops=abi.OPS_PRODUCE | abi.OP_DECOMP, payload=abi.PAYLOAD_TEXT)
    if case == "tiny":
        spec = engine.make_spec(seed=0x5EED0A01, partitions=64, codec_mix=1 << 4, body_min=60, body_max=500,
                                corrupt_ppm=10_000, corrupt_mask=0x3FF, **kw)
        n = 120_000
    elif case == "mixed":
        spec = engine.make_spec(seed=0x5EED0A02, partitions=64, codec_mix=(1 << 4) | (1 << 3), body_min=7,
                                body_max=300_000, corrupt_ppm=10_000, corrupt_mask=0x3FF, **kw)
        n = 6000
    elif case == "c4":
        spec = engine.make_spec(seed=0x5EED0A03, partitions=4096, records_per_batch=64, key_len=16, value_len=999,
                                codec=4, **kw)
        n = 4096
    else:
        spec = engine.make_spec(seed=0x5EED0A04, partitions=64, codec_mix=1 << 4, body_min=100, body_max=60_000,
                                corrupt_ppm=200_000, corrupt_mask=0x200, **kw)
        n = 6000
    data, descs = engine.build_arena(spec, n)
    got = eng.decompress_arena(data, descs)
    compare(got, data, descs, nthreads=8)
    v, codec = got["dres"]["verdict"], got["dres"]["codec"]
    assert ((v == abi.V_OK) & (codec == 4)).sum() > n // 4
    if case == "mutated":
        assert ((v != abi.V_OK) & (codec == 4)).sum() > 20


def large_mutated_zstd(rng, n):
    """Multi-block zstd frames (200 KiB - 1 MiB of records) mutated as
    mutated_bodies does: flipped bytes, truncation, junk, a second frame, 0xFF."""
    out = []
    for i in range(n):
        recs = records(rng, int(rng.integers(180, 900)), 8, 1100, text=bool(i % 3))
        comp = bytearray(orc.compress(4, b"".join(recs)))
        kind = i % 6
        if kind == 1:
            for _ in range(int(rng.integers(1, 4))):
                comp[int(rng.integers(0, len(comp)))] ^= int(rng.integers(1, 256))
        elif kind == 2:
            comp = comp[:int(rng.integers(len(comp) // 2, len(comp) + 1))]
        elif kind == 3:
            comp += bytes(rng.integers(0, 256, int(rng.integers(1, 9)), dtype=np.uint8))
        elif kind == 4:
            comp[int(rng.integers(16, len(comp)))] = 0xFF
        out.append((bytes(comp), len(recs)))
    return out


def drop_content_size(frame: bytes) -> bytes:
    """The same zstd frame without its content size (as the Java client's
    streaming compressor writes them): a window descriptor of 2^ceil(log2 fcs)
    instead of single-segment mode; the blocks unchanged."""
    fhd = frame[4]
    did, ss, fid = fhd & 3, (fhd >> 5) & 1, fhd >> 6
    dsz = [0, 1, 2, 4][did]
    fsz = [ss, 2, 4, 8][fid]
    pos = 5 + (0 if ss else 1)
    wd = bytes([frame[5]]) if not ss else b""
    dict_id = frame[pos:pos + dsz]
    fcs = int.from_bytes(frame[pos + dsz:pos + dsz + fsz], "little") + (256 if fid == 1 else 0)
    if ss:
        e = max(10, (fcs - 1).bit_length())
        wd = bytes([(e - 10) << 3])
    return frame[:4] + bytes([fhd & 0x1F & ~0x20]) + wd + dict_id + frame[pos + dsz + fsz:]


@pytest.mark.parametrize("case", ["large", "mutated", "no_content_size"])
def test_zstd_block_parallel(case):
    """Large zstd frames decoded block-parallel (rpgpu_zblk.h: the blocks'
    literals and sequences by separate lanes, repeat offsets resolved by a wave
    scan, one wave executing each frame) against the oracle, and byte for byte
    against the one-wave decoder (RPGPU_OPT_ZSTD_WAVE_ONLY) on the same arena:
    verdicts, lengths, rewritten batches, index.  Cases: C5-shaped bodies of
    200 KiB - 1 MiB with 1 % corrupted batches, library frames of 2-8 blocks
    mutated (errors found by any stage in any block), and frames without a
    content size (the Java client's kind: the ring's room instead).  The
    plan's output holds the block decoder's literal and record regions."""
    from redpanda_amd import abi, engine

    if case == "large":
        spec = engine.make_spec(seed=0x5EED0B01, partitions=64, codec_mix=1 << 4, body_min=200_000,
                                body_max=1 << 20, ops=abi.OPS_PRODUCE | abi.OP_DECOMP, payload=abi.PAYLOAD_TEXT,
                                corrupt_ppm=10_000, corrupt_mask=0x3FF)
        data, descs = engine.build_arena(spec, 400)
    elif case == "mutated":
        rng = np.random.default_rng(0xB02)
        bs = [batch(c, fmt=WIRE, record_count=rc, attrs=4) for c, rc in large_mutated_zstd(rng, 120)]
        data, descs = arena(bs, fmt=WIRE, ops=OPS)
    else:
        rng = np.random.default_rng(0xB03)
        bs = []
        for i in range(60):
            recs = records(rng, int(rng.integers(250, 900)), 8, 1100, text=bool(i % 3))
            bs.append(batch(drop_content_size(orc.compress(4, b"".join(recs))), fmt=WIRE, record_count=len(recs),
                            attrs=4))
        data, descs = arena(bs, fmt=WIRE, ops=OPS)
    with engine.Engine(0) as e:
        got = e.decompress_arena(data, descs)
    with engine.Engine(0, zstd_blocks=False) as e:
        one = e.decompress_arena(data, descs)
    for f in ("dres", "out_descs", "out_results"):
        assert np.array_equal(got[f].view(np.uint8), one[f].view(np.uint8)), f
    ok = np.nonzero(got["dres"]["verdict"] == abi.V_OK)[0]
    for i in ok:
        a = int(got["dres"]["out_offset"][i])
        m = 61 + int(got["dres"]["out_len"][i])
        assert np.array_equal(got["out"][a:a + m], one["out"][a:a + m]), f"batch {i}"
    want = compare(got, data, descs, nthreads=8)
    assert got["out_bytes"] > one["out_bytes"], "no frame took the block-parallel path"
    v = want["verdicts"]
    assert (v == abi.V_OK).sum() > (len(v) // 2 if case == "mutated" else len(v) * 9 // 10)
    if case == "mutated":
        assert (v == abi.V_DECOMP_ERROR).sum() > 10


@pytest.mark.parametrize("ungated", [False, True])
def test_c5_shaped_arena_gated_and_ungated(eng, ungated):
    """A C5-shaped arena (none / LZ4 / zstd / snappy-java bodies log-uniform in
    [7 B, 1 MiB], 1 % corruption) against the oracle, with the run reading the
    plan's counts on the host (the broker's flow: only the decoders with work
    are launched) and enqueued right behind a fresh plan (every decoder
    launched, the counts read on the device): the split parts, the listed LZ
    lanes, the zstd lanes, the block-parallel zstd stages with their HBM
    workspaces and the wave decoders, on the context's three streams."""
    from redpanda_amd import abi, engine

    mix = (1 << 0) | (1 << 2) | (1 << 3) | (1 << 4)
    spec = engine.make_spec(seed=0x5EED0C55, partitions=64, records_per_batch=1, key_len=0, value_len=0,
                            codec_mix=mix, body_min=7, body_max=1 << 20, corrupt_ppm=10_000, corrupt_mask=0x3FF,
                            ops=abi.OPS_PRODUCE | abi.OP_DECOMP, payload=abi.PAYLOAD_TEXT)
    data, descs = engine.build_arena(spec, 1500, nthreads=8)
    got = eng.decompress_arena(data, descs, runs=2, ungated=ungated)
    want = compare(got, data, descs, nthreads=8)
    v = want["verdicts"]
    assert (v == abi.V_OK).sum() > 1000
