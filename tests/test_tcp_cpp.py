"""C++ host mirror (network-stack_amd/include/nsx/tcp.hpp) of transport/tcp:
builds tests/cpp/test_tcp.cpp with g++ against libnsx_csum.so, runs the
tcp_test.go mirror, and checks its golden segment lines against
tests/golden/segments.json (CPU only: the single-segment path never touches
the GPU)."""
import json
import os
import subprocess

import nsx
from conftest import GOLDEN, ROOT


def test_cpp_tcp_mirror(tmp_path):
    exe = tmp_path / "test_tcp"
    libdir = os.path.dirname(nsx.LIB_PATH)
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-Werror",
                           os.path.join(ROOT, "tests", "cpp", "test_tcp.cpp"),
                           "-I", os.path.join(ROOT, "network-stack_amd", "include"),
                           "-L", libdir, "-lnsx_csum", f"-Wl,-rpath,{libdir}", "-o", str(exe)])
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    lines = out.stdout.strip().splitlines()
    assert lines[-1] == "OK"
    want = {c["name"]: c for c in json.load(open(os.path.join(GOLDEN, "segments.json")))}
    got = {}
    for ln in lines[:-1]:
        name, off, hx, raw, rawp = ln.split()
        got[name] = (int(off), hx, int(raw), int(rawp))
    assert set(got) == set(want)
    for name, c in want.items():
        assert got[name] == (c["offset"], c["bytes"], c["raw"], c["raw_with_pseudo"]), name


def test_cpp_parse_segment_matches_python_oracle_on_golden_segments(tmp_path):
    """The two restatements of parseSegment (tcp.go:130-185) — the C++ mirror's parse_segment and the Python
    oracle's parse_segment, which made tests/golden/parse.json — agree on every golden segment: fields, data
    offset, option count and status (errors, and the cases where the reference would panic or loop)."""
    exe = tmp_path / "parse_dump"
    libdir = os.path.dirname(nsx.LIB_PATH)
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-Werror",
                           os.path.join(ROOT, "tests", "cpp", "parse_dump.cpp"),
                           "-I", os.path.join(ROOT, "network-stack_amd", "include"),
                           "-L", libdir, "-lnsx_csum", f"-Wl,-rpath,{libdir}", "-o", str(exe)])
    meta = json.load(open(os.path.join(GOLDEN, "parse.json")))
    offs = tmp_path / "offs.txt"
    offs.write_text("\n".join(str(x) for x in meta["offsets"]))
    out = subprocess.run([str(exe), os.path.join(GOLDEN, "parse.bin"), str(offs)], capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    cols = ("status", "src_port", "dst_port", "seq_num", "ack_num", "offset", "control", "window", "checksum",
            "urgent_ptr", "data_off", "n_options")
    lines = out.stdout.strip().splitlines()
    assert len(lines) == len(meta["status"])
    for i, ln in enumerate(lines):
        got = [int(x) for x in ln.split()]
        assert got == [meta[c][i] for c in cols], (i, got)


def _build_san(tmp_path, src, name):
    exe = tmp_path / name
    libdir = os.path.dirname(nsx.LIB_PATH)
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-g", "-Wall", "-Wextra", "-Werror",
                           "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer",
                           os.path.join(ROOT, "tests", "cpp", src),
                           "-I", os.path.join(ROOT, "network-stack_amd", "include"),
                           "-L", libdir, "-lnsx_csum", f"-Wl,-rpath,{libdir}", "-o", str(exe)])
    return exe


# The uninstrumented product library is loaded beside the sanitized test; its own allocations are not checked.
_SAN_ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")


def test_cpp_mirror_under_asan_ubsan(tmp_path):
    """The host mirror's serialisation and checksum path (bytes(), computeChecksum, the cgo-facing nsx_csum16)
    under AddressSanitizer + UBSan: no out-of-bounds access, leak or undefined behaviour."""
    exe = _build_san(tmp_path, "test_tcp.cpp", "test_tcp_san")
    out = subprocess.run([str(exe)], capture_output=True, text=True, env=_SAN_ENV)
    assert out.returncode == 0, out.stderr[-4000:]
    assert out.stdout.strip().splitlines()[-1] == "OK"


def test_cpp_parse_segment_random_bytes_under_asan_ubsan(tmp_path):
    """parseSegment's restatement over untrusted bytes (tcp.go:130-185 reads past the end or loops on some
    inputs; the mirror must report those as errors): 3000 random segments of 0-120 bytes — random offset nibbles,
    option kinds and lengths, truncated options — plus the golden ones, parsed under AddressSanitizer + UBSan,
    every result equal to the Python oracle's."""
    import numpy as np
    exe = _build_san(tmp_path, "parse_dump.cpp", "parse_dump_san")
    rng = np.random.default_rng(0x7C9)
    segs = []
    for _ in range(3000):
        n = int(rng.integers(0, 121))
        b = rng.integers(0, 256, n).astype(np.uint8)
        if n > 12:
            b[12] = rng.integers(0, 16)  # low-nibble data offset (the reference's convention): often in range
        if n > 20 and rng.random() < 0.7:  # option area of known kinds with random lengths
            k = 20
            while k < n:
                b[k] = rng.choice([0, 1, 2, 3, 4, 8, 254])
                if k + 1 < n:
                    b[k + 1] = rng.integers(0, 12)
                k += int(rng.integers(1, 6))
        segs.append(b.tobytes())
    blob = b"".join(segs)
    offs = np.concatenate([[0], np.cumsum([len(x) for x in segs])])
    (tmp_path / "blob.bin").write_bytes(blob)
    (tmp_path / "offs.txt").write_text("\n".join(str(int(x)) for x in offs))
    out = subprocess.run([str(exe), str(tmp_path / "blob.bin"), str(tmp_path / "offs.txt")], capture_output=True,
                         text=True, env=_SAN_ENV, timeout=120)
    assert out.returncode == 0, out.stderr[-4000:]
    lines = out.stdout.strip().splitlines()
    assert len(lines) == len(segs)
    status = [int(x.split()[0]) for x in lines]
    assert set(status) <= {0, 1, 2, 3, 4}
    assert 0 in status and len(set(status)) >= 3  # the draw reaches valid segments and several error kinds
    # and the C++ mirror agrees with the Python oracle's parse_segment on every random segment
    import _parse
    want = _parse.expected(np.frombuffer(blob, np.uint8), offs.astype(np.uint64))
    cols = ("status", "src_port", "dst_port", "seq_num", "ack_num", "offset", "control", "window", "checksum",
            "urgent_ptr", "data_off", "n_options")
    for i, ln in enumerate(lines):
        got = [int(x) for x in ln.split()]
        assert got == [int(want[c][i]) for c in cols], (i, got)
    meta = json.load(open(os.path.join(GOLDEN, "parse.json")))
    offs_g = tmp_path / "offs_g.txt"
    offs_g.write_text("\n".join(str(x) for x in meta["offsets"]))
    out = subprocess.run([str(exe), os.path.join(GOLDEN, "parse.bin"), str(offs_g)], capture_output=True, text=True,
                         env=_SAN_ENV, timeout=120)
    assert out.returncode == 0, out.stderr[-4000:]


def test_host_csum16_and_shard_plan_under_asan_ubsan(tmp_path):
    """host_csum16 (the cgo-facing single-segment computeChecksum, tcp.go:72-95) built from its source with
    AddressSanitizer + UBSan: 600 random cases (lengths 0-3000, odd and even prefixes, segment starts at every
    offset 0-15, each segment ending exactly at its allocation's end) equal the oracle's Go-faithful checksum,
    and shard_plan's byte-balanced bounds over random ragged offsets are monotone and cover the batch."""
    import struct
    import numpy as np
    import oracle.csum_oracle as O
    exe = tmp_path / "host_csum_san"
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-g", "-Wall", "-Wextra", "-Werror",
                           "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer",
                           os.path.join(ROOT, "tests", "cpp", "host_csum_dump.cpp"),
                           os.path.join(ROOT, "network-stack_amd", "csrc", "host_csum.cpp"), "-o", str(exe)])
    rng = np.random.default_rng(0x1071)
    cases, blob = [], bytearray()
    for i in range(600):
        pl = int(rng.choice([0, 12, 40, int(rng.integers(0, 64))]))
        sl = int(rng.integers(0, 3001)) if i % 4 else int(rng.integers(0, 20))
        al = int(rng.integers(0, 16))
        pre = rng.integers(0, 256, pl).astype(np.uint8).tobytes()
        seg = (b"\xff" * sl) if i % 50 == 0 else rng.integers(0, 256, sl).astype(np.uint8).tobytes()
        cases.append((pre, seg))
        blob += struct.pack("<III", pl, sl, al) + pre + seg
    (tmp_path / "cases.bin").write_bytes(bytes(blob))
    n, parts = 5000, 7
    lens = rng.integers(0, 9001, n).astype(np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    (tmp_path / "plan.bin").write_bytes(struct.pack("<QI", n, parts) + offs.tobytes())
    out = subprocess.run([str(exe), str(tmp_path / "cases.bin"), str(tmp_path / "plan.bin")], capture_output=True,
                         text=True, env=_SAN_ENV, timeout=120)
    assert out.returncode == 0, out.stderr[-4000:]
    lines = out.stdout.split("\n")
    sums = [int(x) for x in lines[:len(cases)]]
    for (pre, seg), got in zip(cases, sums):
        assert got == O.go_checksum(pre, seg)
    bounds = [int(x.split()[1]) for x in lines[len(cases):] if x.startswith("b ")]
    assert len(bounds) == parts + 1 and bounds[0] == 0 and bounds[-1] == n
    assert all(a <= b for a, b in zip(bounds, bounds[1:]))
