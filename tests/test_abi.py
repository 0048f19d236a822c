"""C-ABI boundary tests that need no GPU: the library loads, exports every
function include/nsx_csum.h (the drop-in boundary) and include/nsx_tune.h (per-call
bench/test overrides) declare, the single-segment host entry point
(computeChecksum, tcp.go:72-95) matches the oracle, host logic (shard plan, layout)
behaves, and device entry points refuse loudly without a GPU."""
import ctypes
import json
import os
import re
import subprocess

import numpy as np
import pytest

import nsx
from conftest import GOLDEN, ROOT
from oracle import csum_oracle as O

HEADER = os.path.join(ROOT, "include", "nsx_csum.h")
TUNE_HEADER = os.path.join(ROOT, "include", "nsx_tune.h")


def declared_functions(header=HEADER):
    src = open(header).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(nsx_[a-z_0-9]+)\s*\(", src, flags=re.M)
    inline = set(re.findall(r"static inline [a-z_0-9]+ (nsx_[a-z_0-9]+)\(", src))
    return sorted(set(names) - inline)


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("nsx_csum16", "nsx_csum_fixed_dev", "nsx_csum_ragged_dev", "nsx_csum_fixed_host",
                 "nsx_csum_ragged_host", "nsx_verify_ragged_dev", "nsx_pseudo_ipv4_partial_dev"):
        assert must in names


def test_library_exports_every_declared_symbol():
    L = nsx.lib()
    declared = declared_functions() + declared_functions(TUNE_HEADER)
    assert len(declared_functions(TUNE_HEADER)) == 16
    missing = [n for n in declared if not hasattr(L, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", nsx.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (nsx_\w+)", out))
    assert set(declared) <= exported


def test_no_process_wide_tuning_state_in_the_boundary():
    """ADVICE/VERDICT r1: the product header holds no global knobs; overrides travel per call."""
    src = open(HEADER).read()
    assert "NSX_PARAM_" not in src and "set_param" not in src
    out = subprocess.run(["nm", "-D", "--defined-only", nsx.LIB_PATH], capture_output=True, text=True).stdout
    assert "nsx_set_param" not in out and "nsx_get_param" not in out


def test_tune_struct_layout_matches_header():
    """nsx_tune as the C compiler lays it out (what a cgo or C caller sees) == the ctypes mirror."""
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "t.c")
        open(src, "w").write(r'''
#include <stddef.h>
#include <stdio.h>
#include "nsx_tune.h"
int main(void) {
    printf("%zu %zu %zu %zu %zu %zu\n", sizeof(nsx_tune), offsetof(nsx_tune, window_bytes),
           offsetof(nsx_tune, kernel), offsetof(nsx_tune, shards_per_device), offsetof(nsx_tune, deal),
           offsetof(nsx_tune, reserved));
    return 0;
}
''')
        exe = os.path.join(td, "t")
        subprocess.check_call(["gcc", "-std=c11", "-Wall", "-Werror", src, "-I", os.path.join(ROOT, "include"), "-o", exe])
        got = [int(x) for x in subprocess.run([exe], capture_output=True, text=True).stdout.split()]
    T = nsx.Tune
    assert got == [ctypes.sizeof(T), T.window_bytes.offset, T.kernel.offset, T.shards_per_device.offset,
                   T.deal.offset, T.reserved.offset]
    with pytest.raises(ValueError):
        nsx._tune(dict(no_such_knob=1))


def test_library_has_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/bin/roc-obj-ls", nsx.LIB_PATH], capture_output=True, text=True)
    if out.returncode == 0:
        assert "gfx950" in out.stdout
    else:  # no roc-obj-ls: the offload bundle names its target triple in the clear
        assert b"amdgcn-amd-amdhsa--gfx950" in open(nsx.LIB_PATH, "rb").read()


def test_abi_version():
    assert nsx.abi_version() == 2


@pytest.mark.parametrize("case", json.load(open(os.path.join(GOLDEN, "kat.json"))), ids=lambda c: c["name"])
def test_csum16_kat(case):
    assert nsx.csum16(bytes.fromhex(case["prefix"]), bytes.fromhex(case["segment"])) == case["raw"]


def test_csum16_golden_vectors():
    idx = json.load(open(os.path.join(GOLDEN, "vectors.json")))
    blob = np.fromfile(os.path.join(GOLDEN, "vectors.bin"), np.uint8)
    for c in idx:
        seg = blob[c["offset"]:c["offset"] + c["length"]].tobytes()
        assert nsx.csum16(bytes.fromhex(c["prefix"]), seg) == c["raw"], c


def test_csum16_reference_TestSegmentComputeChecksum():
    """tcp_test.go:26-32 through the C ABI."""
    s = O.Segment(data=b"hello")
    s.checksum = nsx.field(nsx.csum16(b"", s.bytes()))
    assert nsx.verify(nsx.csum16(b"", s.bytes()))


def test_csum16_random_vs_oracle():
    rng = np.random.default_rng(11)
    for _ in range(1500):
        n = int(rng.integers(0, 3000))
        pl = int(rng.integers(0, 45))
        seg = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        if rng.integers(0, 8) == 0:
            seg = b"\xff" * n
        pre = rng.integers(0, 256, pl, dtype=np.uint8).tobytes()
        assert nsx.csum16(pre, seg) == O.c_go_checksum(pre, seg), (n, pl)


def test_csum16_unaligned_views():
    """Misaligned host pointers (computeChecksum takes any []byte)."""
    buf = O.c_splitmix64(0x1071, 70000)
    for start in range(8):
        for n in (0, 1, 2, 7, 8, 9, 1499, 1500, 65536):
            seg = buf[start:start + n]
            out = ctypes.c_uint16()
            rc = nsx.lib().nsx_csum16(None, 0, seg.ctypes.data_as(ctypes.c_void_p), n, ctypes.byref(out))
            assert rc == 0 and out.value == O.c_go_checksum(b"", seg.tobytes())


def test_csum16_errors():
    L = nsx.lib()
    out = ctypes.c_uint16()
    assert L.nsx_csum16(None, 4, None, 0, ctypes.byref(out)) == nsx.NSX_EINVAL
    assert L.nsx_csum16(None, 0, None, 3, ctypes.byref(out)) == nsx.NSX_EINVAL
    assert L.nsx_csum16(None, 0, None, 0, None) == nsx.NSX_EINVAL
    assert L.nsx_csum16(None, 0, None, 0, ctypes.byref(out)) == 0 and out.value == 0


def test_shard_plan_fixed():
    for n, parts in ((0, 1), (10, 3), (1 << 20, 8), (5, 8)):
        b = nsx.shard_plan(n, parts)
        assert b[0] == 0 and b[-1] == n and np.all(np.diff(b.astype(np.int64)) >= 0)
        sizes = np.diff(b.astype(np.int64))
        assert sizes.max() - sizes.min() <= 1


def test_shard_plan_ragged_byte_balanced():
    rng = np.random.default_rng(0x1072)
    lens = rng.integers(64, 9001, 100000).astype(np.uint64)
    offs = np.zeros(lens.size + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    b = nsx.shard_plan(lens.size, 8, offs)
    assert b[0] == 0 and b[-1] == lens.size
    per = [int(offs[b[g + 1]] - offs[b[g]]) for g in range(8)]
    assert max(per) - min(per) <= 2 * 9000
    assert sum(per) == int(offs[-1])


def test_device_calls_fail_loudly_without_gpu():
    """No CPU fallback: on a GPU-less host every device/batch entry point reports
    NSX_ENODEV (never a silently computed result)."""
    if nsx.device_count() > 0:
        pytest.skip("GPU present")
    L = nsx.lib()
    fake = ctypes.c_void_p(0x1000)
    assert L.nsx_csum_fixed_dev(fake, 1500, 1500, 4, None, fake, None) == nsx.NSX_ENODEV
    assert L.nsx_csum_ragged_dev(fake, fake, 4, None, fake, None) == nsx.NSX_ENODEV
    assert L.nsx_verify_ragged_dev(fake, fake, 4, None, fake, None, None) == nsx.NSX_ENODEV
    assert L.nsx_pseudo_ipv4_partial_dev(fake, fake, fake, 6, 4, fake, None) == nsx.NSX_ENODEV
    assert L.nsx_pseudo_ipv6_partial_dev(fake, fake, fake, 6, 4, fake, None) == nsx.NSX_ENODEV
    assert L.nsx_verify_mask_dev(fake, 4, fake, None) == nsx.NSX_ENODEV
    assert L.nsx_fill_splitmix64_dev(fake, 0, 16, 1, None) == nsx.NSX_ENODEV
    assert L.nsx_ipv4_hdr_csum_dev(fake, 64, 0, 4, 0, fake, None) == nsx.NSX_ENODEV
    assert L.nsx_ipv4_hdr_verify_mask_dev(fake, 20, 0, 4, fake, None) == nsx.NSX_ENODEV
    soa = nsx.TcpHdrSoA(*([0x1000] * 8))
    assert L.nsx_tcp_build_dev(ctypes.byref(soa), None, None, fake, fake, 16, None, 4, fake, fake, None,
                               None) == nsx.NSX_ENODEV
    tune = ctypes.byref(nsx.Tune(blocks_per_cu=2))
    assert L.nsx_csum_fixed_dev_tuned(fake, 1500, 1500, 4, None, fake, None, tune) == nsx.NSX_ENODEV
    assert L.nsx_csum_ragged_dev_tuned(fake, fake, 4, None, fake, None, tune) == nsx.NSX_ENODEV
    assert L.nsx_verify_ragged_dev_tuned(fake, fake, 4, None, fake, None, None, tune) == nsx.NSX_ENODEV
    assert L.nsx_ipv4_hdr_csum_dev_tuned(fake, 64, 0, 4, 0, fake, None, tune) == nsx.NSX_ENODEV
    assert L.nsx_ipv4_hdr_verify_mask_dev_tuned(fake, 20, 0, 4, fake, None, tune) == nsx.NSX_ENODEV
    assert L.nsx_tcp_build_dev_tuned(ctypes.byref(soa), None, None, fake, fake, 16, None, 4, fake, fake, None,
                                     None, tune) == nsx.NSX_ENODEV
    cnt = ctypes.c_uint64(7)
    assert L.nsx_fixed_launch_count(1500, 1500, 4, None, ctypes.byref(cnt)) == nsx.NSX_ENODEV
    assert L.nsx_ipv4_hdr_launch_count(fake, 20, 0, 4, None, ctypes.byref(cnt)) == nsx.NSX_ENODEV
    buf = np.zeros(3000, np.uint8)
    with pytest.raises(nsx.NsxError) as e:
        nsx.fixed_host(buf, 1500, 1500, 2)
    assert e.value.code == nsx.NSX_ENODEV
    with pytest.raises(nsx.NsxError):
        nsx.ragged_host(buf, np.array([0, 10, 3000], np.uint64))
    with pytest.raises(nsx.NsxError) as e:
        nsx.fixed_host(buf, 1500, 1500, 2, tune=dict(shards_per_device=3))
    assert e.value.code == nsx.NSX_ENODEV
    assert L.nsx_rx_ipv4_tcp_verify_dev(fake, fake, 4, fake, None, None, None) == nsx.NSX_ENODEV
    assert L.nsx_rx_ipv6_tcp_verify_dev(fake, fake, 4, fake, None, None) == nsx.NSX_ENODEV
    parsed = nsx.TcpParsedSoA()
    assert L.nsx_tcp_parse_dev(fake, fake, 4, ctypes.byref(parsed), None) == nsx.NSX_ENODEV
    assert L.nsx_tcp_parse_dev(fake, fake, 4, None, None) == nsx.NSX_EINVAL
    assert L.nsx_rx_ipv6_tcp_verify_dev_tuned(fake, fake, 4, fake, None, None, tune) == nsx.NSX_ENODEV
    for v in (4, 6):
        with pytest.raises(nsx.NsxError) as e:
            nsx.rx_ipv4_tcp_verify_host(buf, np.array([0, 100, 3000], np.uint64), ipver=v)
        assert e.value.code == nsx.NSX_ENODEV
    p = ctypes.c_void_p()
    assert L.nsx_alloc_pinned(64, ctypes.byref(p)) == nsx.NSX_ENODEV
    assert L.nsx_host_cache_release() == 0  # nothing cached, nothing to do


def test_device_calls_validate_before_device():
    L = nsx.lib()
    fake = ctypes.c_void_p(0x1000)
    assert L.nsx_csum_fixed_dev(fake, 1500, 1500, 0, None, None, None) == 0   # n == 0 is a no-op
    assert L.nsx_csum_fixed_dev(None, 1500, 1500, 4, None, fake, None) == nsx.NSX_EINVAL
    assert L.nsx_csum_fixed_dev(fake, 1500, 1500, 4, None, None, None) == nsx.NSX_EINVAL
    assert L.nsx_csum_ragged_dev(fake, None, 4, None, fake, None) == nsx.NSX_EINVAL
    assert L.nsx_verify_mask_dev(None, 4, fake, None) == nsx.NSX_EINVAL
    assert L.nsx_ipv4_hdr_verify_mask_dev(None, 20, 0, 4, fake, None) == nsx.NSX_EINVAL
    assert L.nsx_ipv4_hdr_verify_mask_dev(fake, 20, 0, 4, None, None) == nsx.NSX_EINVAL
    assert L.nsx_ipv4_hdr_verify_mask_dev(fake, 0, 0, 4, fake, None) == nsx.NSX_EINVAL
    assert L.nsx_verify_mask_dev(fake, 0, None, None) == 0
    assert L.nsx_pseudo_ipv6_partial_dev(fake, None, fake, 6, 4, fake, None) == nsx.NSX_EINVAL
    bad = np.array([0, 10, 5], np.uint64)
    assert L.nsx_csum_ragged_host(np.zeros(16, np.uint8).ctypes.data_as(ctypes.c_void_p),
                                  bad.ctypes.data_as(ctypes.c_void_p), 2, None,
                                  np.zeros(2, np.uint16).ctypes.data_as(ctypes.c_void_p), 0) == nsx.NSX_EINVAL


def test_binding_checks_extents_before_the_c_call():
    """the C ABI cannot see a tensor's extent, so the Python wrappers refuse undersized,
    wrongly typed, non-contiguous or host tensors with ValueError before any C call (CPU tensors here: every
    check runs before the device check, and a well-formed CPU tensor is refused as not on a device)."""
    import torch
    u8 = lambda k: torch.zeros(k, dtype=torch.uint8)  # noqa: E731
    i16 = lambda k: torch.zeros(k, dtype=torch.int16)  # noqa: E731
    offs = torch.tensor([0, 10, 20, 30], dtype=torch.int64)
    cases = [
        (lambda: nsx.fixed_dev(u8(2999), 1500, 1500, 2, out=i16(2)), "3000 B needed"),
        (lambda: nsx.fixed_dev(u8(3000), 1500, 1500, 2, out=i16(1)), "fixed_dev out"),
        (lambda: nsx.fixed_dev(u8(3000), 1500, 1500, 2, out=torch.zeros(2, dtype=torch.int32)), "2-byte elements"),
        (lambda: nsx.fixed_dev(u8(3000), 1500, 1500, 2, out=i16(4)[::2]), "contiguous"),
        (lambda: nsx.fixed_dev(u8(3000), 1500, 1500, 2, partial=torch.zeros(1, dtype=torch.int32), out=i16(2)),
         "fixed_dev partial"),
        (lambda: nsx.fixed_dev(u8(3000), 1500, 1500, 2, out=i16(2)), "device"),
        (lambda: nsx.ragged_dev(u8(30), offs.to(torch.int32)), "8-byte elements"),
        (lambda: nsx.ragged_dev(u8(30), offs, out=i16(2)), "ragged_dev out"),
        (lambda: nsx.ragged_dev(u8(30), offs, partial=torch.zeros(2, dtype=torch.int32), out=i16(3)),
         "ragged_dev partial"),
        (lambda: nsx.verify_mask_dev(i16(65), out=torch.zeros(1, dtype=torch.int64)), "verify_mask_dev out"),
        (lambda: nsx.ipv4_hdr_csum_dev(u8(20 * 9 + 19), 20, 10, out=i16(10)), "200 B needed"),
        (lambda: nsx.ipv4_hdr_verify_mask_dev(u8(20 * 65), 20, 65, mask=torch.zeros(1, dtype=torch.int64)), "mask"),
        (lambda: nsx.rx_ipv4_tcp_verify_dev(u8(30), offs, mask=torch.zeros(1, dtype=torch.int64), ip_raw=i16(2)),
         "ip_raw"),
        (lambda: nsx.rx_ipv6_tcp_verify_dev(u8(30), offs, mask=torch.zeros(0, dtype=torch.int64)), "mask"),
        (lambda: nsx.tcp_parse_dev(u8(30), offs, fields={"seq_num": torch.zeros(3, dtype=torch.int16)}),
         "seq_num"),
        (lambda: nsx.pseudo_ipv4_partial_dev(u8(7), u8(8), torch.zeros(2, dtype=torch.int32)), "src"),
        (lambda: nsx.fixed_host(np.zeros(2999, np.uint8), 1500, 1500, 2), "3000 B needed"),
        (lambda: nsx.ragged_host(np.zeros(29, np.uint8), np.array([0, 10, 30], np.uint64)), "end at 30"),
    ]
    n = 3
    fields = {k: torch.zeros(n, dtype={1: torch.uint8, 2: torch.int16, 4: torch.int32}[s]) for k, s in nsx.BUILD_FIELDS}
    build = dict(data=u8(30), data_off=offs, out=u8(200), out_off=offs)
    cases += [
        (lambda: nsx.tcp_build_dev(dict(fields, window=torch.zeros(2, dtype=torch.int16)), **build), "window"),
        (lambda: nsx.tcp_build_dev(dict(fields, seq_num=None), **build), "'seq_num' missing"),
        (lambda: nsx.tcp_build_dev(fields, **dict(build, out_off=offs[:3])), "out_off"),
        (lambda: nsx.tcp_build_dev(fields, **build, raw=i16(2)), "raw"),
        (lambda: nsx.tcp_build_dev(fields, **build, opt_off=offs), "opt_off given without opts"),
    ]
    for fn, msg in cases:
        with pytest.raises(ValueError) as e:
            fn()
        assert msg in str(e.value), (msg, str(e.value))


def test_c_caller_compiles_and_links(tmp_path):
    """A plain C program (what cgo compiles) includes the header and links the library."""
    src = tmp_path / "caller.c"
    src.write_text(r'''
#include <stdio.h>
#include <string.h>
#include "nsx_csum.h"
int main(void) {
    unsigned char seg[25] = {0};
    memcpy(seg + 20, "hello", 5);
    uint16_t raw = 0;
    if (nsx_csum16(NULL, 0, seg, sizeof seg, &raw) != NSX_OK) return 2;
    uint16_t f = nsx_field(raw);
    seg[16] = f >> 8; seg[17] = f & 0xFF;           /* tcp.go:110 */
    uint16_t again = 0;
    nsx_csum16(NULL, 0, seg, sizeof seg, &again);
    printf("%04x %04x %d\n", raw, again, nsx_verify(again));
    return nsx_verify(again) ? 0 : 1;
}
''')
    exe = tmp_path / "caller"
    libdir = os.path.dirname(nsx.LIB_PATH)
    subprocess.check_call(["gcc", "-std=c11", "-Wall", "-Werror", str(src), "-I", os.path.join(ROOT, "include"),
                           "-L", libdir, "-lnsx_csum", f"-Wl,-rpath,{libdir}", "-o", str(exe)])
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.split() == ["43d2", "ffff", "1"]


def test_tcp_wire_len_and_layout_match_reference_bytes():
    """nsx_tcp_wire_len / nsx_tcp_layout_host agree with len(segment.bytes()) (tcp.go:98-128)."""
    rng = np.random.default_rng(21)
    opt_sets = [[], [O.Option(kind=1)], [O.Option(kind=2, length=4, data=b"\x05\xb4\0\0")],
                [O.Option(kind=1), O.Option(kind=1), O.Option(kind=0)],
                [O.Option(kind=2, length=4, data=b"abcd"), O.Option(kind=1)]]
    segs = []
    for i in range(200):
        opts = opt_sets[i % len(opt_sets)]
        segs.append(O.Segment(options=opts, data=bytes(int(rng.integers(0, 300)))))
    for s in segs:
        ol = sum(len(o.bytes()) for o in s.options)
        assert nsx.tcp_wire_len(ol, len(s.data)) == len(s.bytes())
    opt_off = np.zeros(len(segs) + 1, np.uint64)
    opt_off[1:] = np.cumsum([sum(len(o.bytes()) for o in s.options) for s in segs])
    data_off = np.zeros(len(segs) + 1, np.uint64)
    data_off[1:] = np.cumsum([len(s.data) for s in segs])
    out_off = nsx.tcp_layout_host(data_off, opt_off)
    want = np.zeros(len(segs) + 1, np.uint64)
    want[1:] = np.cumsum([(len(s.bytes()) + 3) & ~3 for s in segs])
    assert np.array_equal(out_off, want)


def test_ragged_segs_per_wave_outside_its_forms_is_einval():
    """Ragged checksum tunes: segs_per_wave 0 / 1 / 2 / 3 / 5 name its forms; 4 (runs of four sets, removed in round
    4) and any other value are refused with NSX_EINVAL before a device is touched (host entry
    point), instead of silently running the automatic form."""
    offs = np.array([0, 40, 100], np.uint64)
    buf = np.zeros(100, np.uint8)
    for bad in (4, 6, 8, -1):
        with pytest.raises(nsx.NsxError) as e:
            nsx.ragged_host(buf, offs, tune=dict(segs_per_wave=bad))
        assert e.value.code == nsx.NSX_EINVAL, bad


def test_receive_grid_modes_off_the_default_grid_are_einval():
    """segs_per_wave 5 / 6 / 7 force a mode of the receive pass's default grid; with rows 4-16 or
    blocks_per_cu set they name no shape and are refused (NSX_EINVAL) instead of silently running the auto shape.
    The host entry points check before touching a device, so this runs on any host."""
    offs = np.array([0, 40], np.uint64)
    buf = np.zeros(40, np.uint8)
    for mode in (5, 6, 7, 8, 9):
        for bad in (dict(blocks_per_cu=2), dict(rows=4), dict(rows=16, blocks_per_cu=1)):
            for fn in (nsx.rx_ipv4_tcp_verify_host, nsx.rx_ipv6_tcp_verify_host):
                with pytest.raises(nsx.NsxError) as e:
                    fn(buf, offs, tune=dict(bad, segs_per_wave=mode))
                assert e.value.code == nsx.NSX_EINVAL, (mode, bad)
    # values that name no receive form at all are refused on every grid, not run as the auto shape
    for bad in (3, 4, 10, -1):
        for extra in ({}, dict(rows=4), dict(blocks_per_cu=2)):
            for fn in (nsx.rx_ipv4_tcp_verify_host, nsx.rx_ipv6_tcp_verify_host):
                with pytest.raises(nsx.NsxError) as e:
                    fn(buf, offs, tune=dict(extra, segs_per_wave=bad))
                assert e.value.code == nsx.NSX_EINVAL, (bad, extra)


def _build_host_case(n=3, pay=10):
    fields = {k: np.arange(n).astype({1: np.uint8, 2: np.uint16, 4: np.uint32}[s]) for k, s in nsx.BUILD_FIELDS}
    data_off = np.arange(n + 1, dtype=np.uint64) * np.uint64(pay)
    return fields, np.zeros(n * pay, np.uint8), data_off


def test_tcp_build_host_validates_before_any_device():
    """nsx_tcp_build_host (the sender pass over host memory) checks every span it will copy before
    touching a device — on a GPU-less host a well-formed call is NSX_ENODEV and a malformed one NSX_EINVAL: offsets
    that decrease, image slots that are not 4-aligned or too short for image + padding (nsx_tcp_layout_host's rule),
    opt_off without opts, a missing header field."""
    fields, data, data_off = _build_host_case()
    if nsx.device_count() == 0:
        with pytest.raises(nsx.NsxError) as e:
            nsx.tcp_build_host(fields, data, data_off)
        assert e.value.code == nsx.NSX_ENODEV
    lay = nsx.tcp_layout_host(data_off)  # 32 B slots: 30 B images + 2 B padding
    bad_layouts = [lay + np.uint64(2),                                            # not 4-aligned
                   np.array([0, 32, 60, 96], np.uint64),                          # slot 1 too short
                   np.array([0, 32, 64, 64], np.uint64)]                          # last slot empty
    for oo in bad_layouts:
        with pytest.raises(nsx.NsxError) as e:
            nsx.tcp_build_host(fields, data, data_off, out_off=oo, out=np.zeros(200, np.uint8))
        assert e.value.code == nsx.NSX_EINVAL, oo
    with pytest.raises(nsx.NsxError) as e:  # decreasing data offsets
        nsx.tcp_build_host(fields, data, np.array([0, 10, 5, 30], np.uint64), out_off=lay, out=np.zeros(200, np.uint8))
    assert e.value.code == nsx.NSX_EINVAL
    L = nsx.lib()
    soa = nsx.TcpHdrSoA(*[None if k == "window" else c.ctypes.data for k, c in
                          ((k, fields[k]) for k, _ in nsx.BUILD_FIELDS)])
    out = np.zeros(200, np.uint8)
    ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    assert L.nsx_tcp_build_host(ctypes.byref(soa), None, None, ptr(data), ptr(data_off), None, 3, ptr(out), ptr(lay),
                                None, 0) == nsx.NSX_EINVAL  # window missing
    soa.window = fields["window"].ctypes.data
    assert L.nsx_tcp_build_host(ctypes.byref(soa), None, ptr(data_off), ptr(data), ptr(data_off), None, 3, ptr(out),
                                ptr(lay), None, 0) == nsx.NSX_EINVAL  # opt_off without opts
    assert L.nsx_tcp_build_host(ctypes.byref(soa), None, None, ptr(data), ptr(data_off), None, 0, ptr(out), ptr(lay),
                                None, 0) == 0  # n == 0: nothing to do
    # binding extent checks (ValueError before the C call)
    for kw, msg in ((dict(data=np.zeros(29, np.uint8)), "data_off ends at 30"),
                    (dict(out=np.zeros(95, np.uint8)), "out_off ends at 96"),
                    (dict(partial=np.zeros(2, np.uint32)), "partial"),
                    (dict(opt_off=np.zeros(4, np.uint64)), "opt_off given without opts"),
                    # the images are written contiguously from out's first byte
                    (dict(out=np.zeros(400, np.uint8)[::2]), "C-contiguous uint8"),
                    (dict(out=np.zeros(100, np.uint16)), "C-contiguous uint8")):
        args = dict(fields=fields, data=data, data_off=data_off)
        args.update(kw)
        with pytest.raises(ValueError) as e:
            nsx.tcp_build_host(**args)
        assert msg in str(e.value), (msg, str(e.value))
    with pytest.raises(ValueError):
        nsx.tcp_build_host(dict(fields, seq_num=None), data, data_off)
