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
