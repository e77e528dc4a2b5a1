"""zstd window / workspace limits against the oracle (CPU, no GPU).

The reference decodes through a static DCtx over ZSTD_estimateDStreamSize(8
MiB) (stream_zstd.cc:44-87).  A frame whose window needs more ring buffer
than that fails with ZSTD_error_memory_allocation, a window above 2^27 with
frameParameter_windowTooLarge -- and both reach the caller as
std::runtime_error: throw_zstd_err (stream_zstd.cc:29-36) compares the raw
size_t return with the enum value, so its bad_alloc branch never fires.
These tests pin the oracle to that reading (DECOMP_ERROR, never a separate
bad_alloc verdict); tests/test_gpu_decomp.py runs the same frames on the GPU.
"""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(__file__))
from kafka_batches import zstd_reheader  # noqa: E402

import oracle.oracle as orc  # noqa: E402

V_OK, V_ERROR = 0, 30


def payload(n: int) -> bytes:
    words = [b"kafka ", b"redpanda ", b"offset ", b"batch ", b"log ", b"segment "]
    out = bytearray()
    i = 0
    while len(out) < n:
        out += words[(i * 7 + i // 3) % len(words)]
        i += 1
    return bytes(out[:n])


def window_cases():
    """(name, frame, expected oracle verdict)."""
    body = payload(64 << 10)
    big = payload(100 << 10)
    f64, f100 = orc.compress(4, body), orc.compress(4, big)
    yield "as_compressed", f64, V_OK
    for wl in (17, 20, 23):
        yield f"wlog{wl}_nofcs", zstd_reheader(f64, wl, None), V_OK
    # 2^24 window, content size unknown: ring 16 MiB + 128 KiB + 64 > the 8 MiB workspace
    yield "wlog24_nofcs", zstd_reheader(f64, 24, None), V_ERROR
    yield "wlog23_m7_nofcs", zstd_reheader(f64, 23, None, mantissa=7), V_ERROR
    # content size known and <= the 64 KiB staging buffer: single-pass decode,
    # no ring buffer, no window check
    yield "wlog24_fcs64k", zstd_reheader(f64, 24, "keep"), V_OK
    yield "wlog28_fcs64k", zstd_reheader(f64, 28, "keep"), V_OK
    # content size 100 KiB > staging: streamed; ring = min(fcs, window ring)
    yield "wlog24_fcs100k", zstd_reheader(f100, 24, "keep"), V_OK
    yield "wlog27_fcs100k", zstd_reheader(f100, 27, "keep"), V_OK
    # window > ZSTD_MAXWINDOWSIZE_DEFAULT (2^27): frameParameter_windowTooLarge
    yield "wlog28_fcs100k", zstd_reheader(f100, 28, "keep"), V_ERROR
    yield "wlog28_nofcs", zstd_reheader(f64, 28, None), V_ERROR
    yield "wlog31_nofcs", zstd_reheader(f64, 31, None), V_ERROR
    # window smaller than the matches reach: corrupt offsets
    yield "wlog10_nofcs", zstd_reheader(f64, 10, None), V_ERROR
    yield "single_segment", zstd_reheader(f64, None, "keep"), V_OK


@pytest.mark.parametrize("name,frame,want", list(window_cases()), ids=lambda x: x if isinstance(x, str) else "")
def test_oracle_window_verdicts(name, frame, want):
    v, out = orc.uncompress(4, frame, cap=1 << 20)
    assert v == want, (name, v)
    if v == V_OK:
        assert len(out) in (64 << 10, 100 << 10)
