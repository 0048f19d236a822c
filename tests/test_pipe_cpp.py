"""f4: the loopback transport feeding checksum batches.
tests/cpp/test_pipe.cpp mirrors the reference's transport conformance suite
(transport/test/conn.go) against nsx/pipe.hpp (a restatement of
transport/pipe/pipe.go); the config-1 harness (network-stack_amd/tools/
loopback.cpp) sends 64 x 1500 B TCP segments through it and verifies every
checksum on arrival — per segment on the host (CPU) or as one GPU batch (gpu)."""
import json
import os
import subprocess

import pytest

import nsx
from conftest import ROOT

INC = os.path.join(ROOT, "network-stack_amd", "include")
LOOPBACK = os.path.join(ROOT, "network-stack_amd", "build", "nsx_loopback")


def _build_pipe_test(tmp_path, extra=()):
    exe = tmp_path / "test_pipe"
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-Wall", "-Wextra", "-Werror", "-pthread", *extra,
                           os.path.join(ROOT, "tests", "cpp", "test_pipe.cpp"), "-I", INC, "-o", str(exe)])
    return exe


def test_pipe_conformance(tmp_path):
    out = subprocess.run([str(_build_pipe_test(tmp_path))], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.split("\n")[:3] == ["pipe: 12 tests x 20 OK", "buffered: 14 tests x 20 OK", "OK"]


def test_pipe_conformance_tsan(tmp_path):
    """The race tests (conn.go TestWriteRace/TestReadRace) under ThreadSanitizer."""
    try:
        exe = _build_pipe_test(tmp_path, ("-fsanitize=thread",))
    except subprocess.CalledProcessError:
        pytest.skip("ThreadSanitizer unavailable")
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and "WARNING: ThreadSanitizer" not in out.stderr, out.stderr


def _loopback(*args):
    if not os.path.exists(LOOPBACK):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "network-stack_amd")])
    out = subprocess.run([LOOPBACK, *args], capture_output=True, text=True, timeout=300)
    return out.returncode, json.loads(out.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("mode", ["host", "ring-host"])
def test_loopback_config1_host_verifies_every_segment(mode):
    rc, r = _loopback("--mode", mode, "--reps", "20")
    assert rc == 0 and r["bad"] == 0 and r["reps"] == 20


@pytest.mark.parametrize("mode", ["host", "ring-host"])
def test_loopback_detects_corruption_host(mode):
    rc, r = _loopback("--mode", mode, "--reps", "3", "--corrupt", "17")
    assert rc == 0 and r["bad"] == 3


@pytest.mark.parametrize("mode", ["host", "ring-host"])
def test_loopback_odd_lengths_host(mode):
    for L in ("20", "21", "1501", "9001"):
        rc, r = _loopback("--mode", mode, "--reps", "2", "--seg-len", L, "--segments", "9")
        assert rc == 0 and r["bad"] == 0, L


@pytest.mark.parametrize("mode", ["batch", "ring-gpu"])
def test_loopback_gpu_modes_refuse_without_gpu(mode):
    if nsx.device_count() > 0:
        pytest.skip("GPU present")
    rc, r = _loopback("--mode", mode, "--reps", "1")
    assert rc == 1 and "error" in r


def _raw_sums_vs_oracle(tmp_path, mode, seg_len=1500, segments=64, corrupt=None):
    """Every raw sum the receiver computed (nsx_loopback --dump) equals the oracle's computeChecksum
    (tcp.go:72-95, Go-faithful C loop) over the same pseudo-header and the bytes that were sent."""
    import numpy as np
    from oracle import csum_oracle as O
    path = tmp_path / f"dump_{mode}_{seg_len}.bin"
    args = ["--mode", mode, "--reps", "3", "--seg-len", str(seg_len), "--segments", str(segments), "--dump", str(path)]
    if corrupt is not None:
        args += ["--corrupt", str(corrupt)]
    rc, r = _loopback(*args)
    assert rc == 0, r
    blob = path.read_bytes()
    rec = 12 + seg_len + 2
    assert len(blob) == segments * rec
    for i in range(segments):
        b = blob[i * rec:(i + 1) * rec]
        pseudo, wire, raw = b[:12], b[12:12 + seg_len], int.from_bytes(b[-2:], "little")
        assert raw == O.c_go_checksum(pseudo, wire), (mode, seg_len, i)
        assert O.verify(raw) == (i != corrupt), (mode, i)
    return r


@pytest.mark.parametrize("mode", ["host", "ring-host"])
def test_loopback_host_raw_sums_vs_oracle(tmp_path, mode):
    for L, corrupt in ((1500, None), (1500, 17), (21, None), (9001, None)):
        _raw_sums_vs_oracle(tmp_path, mode, L, 64 if L == 1500 else 9, corrupt)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["batch", "ring-gpu"])
def test_loopback_config1_gpu_batch(mode, tmp_path):
    """Config 1's GPU modes: the raw sums of the GPU batch (what arrived through the pipe, one host batch call)
    against the oracle on every segment, intact and with a segment damaged in transit; odd lengths."""
    rc, r = _loopback("--mode", mode, "--reps", "50")
    assert rc == 0 and r["bad"] == 0
    r = _raw_sums_vs_oracle(tmp_path, mode)
    assert r["bad"] == 0
    r = _raw_sums_vs_oracle(tmp_path, mode, corrupt=63)
    assert r["bad"] == 3
    for L in (21, 1501, 9001):
        r = _raw_sums_vs_oracle(tmp_path, mode, seg_len=L, segments=9)
        assert r["bad"] == 0, L

