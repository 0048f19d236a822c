"""Randomised GPU parity (seeded, bounded to a few seconds): every device entry
point on batches whose sizes, alignments, lengths and kernel knobs are drawn at
random, against the CPU oracle. Complements the hand-picked edge cases of
test_gpu_parity.py with combinations nobody wrote down, and collects after it (and
after the BASELINE configs of test_gpu_00_baseline.py) so that under -x a fuzz failure
never hides those. NSX_FUZZ_SCALE=k runs k times as many cases (new seeds; the default
set is the first of them). Launch overrides (include/nsx_tune.h) are drawn per case."""
import os

import numpy as np
import pytest

from oracle import csum_oracle as O

pytestmark = pytest.mark.gpu
SCALE = max(1, int(os.environ.get("NSX_FUZZ_SCALE", "1")))

torch = pytest.importorskip("torch")

import nsx  # noqa: E402

FIXED_KNOBS = [dict(), dict(segs_per_wave=4, blocks_per_cu=2), dict(segs_per_wave=1), dict(segs_per_wave=2),
               dict(blocks_per_cu=8), dict(blocks_per_cu=1, segs_per_wave=8), dict(xcd_chunk=-1), dict(xcd_chunk=3),
               dict(block_mode=2), dict(block_mode=1), dict(window_bytes=1_000_000), dict(window_bytes=7_777)]
RAGGED_KNOBS = [dict(), dict(rows=4), dict(rows=8), dict(run_segs=1), dict(run_segs=17, blocks_per_cu=1),
                dict(blocks_per_cu=8), dict(block_mode=2), dict(block_mode=1), dict(kernel=nsx.KERNEL_SCAN_PLAIN),
                dict(kernel=nsx.KERNEL_SCAN_PLAIN, rows=16, run_segs=5), dict(segs_per_wave=1),
                dict(segs_per_wave=1, run_segs=7), dict(segs_per_wave=2), dict(segs_per_wave=2, run_segs=9), dict(segs_per_wave=3),
                dict(segs_per_wave=3, run_segs=5),
                dict(segs_per_wave=5, blocks_per_cu=1), dict(segs_per_wave=5),
                dict(segs_per_wave=5, run_segs=11, blocks_per_cu=2)]


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _u16(t):
    return t.cpu().numpy().view(np.uint16)


@pytest.mark.parametrize("case", range(120 * SCALE))
def test_fuzz_fixed(case):
    rng = np.random.default_rng(1000 + case)
    seg_len = int(rng.choice([int(rng.integers(0, 64)), int(rng.integers(64, 4200)), int(rng.integers(4200, 70000))]))
    stride = seg_len + int(rng.choice([0, 0, int(rng.integers(0, 9)), int(rng.integers(0, 300))]))
    stride = max(stride, 1)
    n = int(rng.integers(1, max(2, min(60000, (24 << 20) // stride))))
    lead = int(rng.integers(0, 8))
    buf = rng.integers(0, 256, lead + (n - 1) * stride + seg_len, dtype=np.uint8)
    if case % 7 == 0:
        buf[:] = 0xFF
    part = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32) if case % 3 == 0 else None
    knobs = FIXED_KNOBS[case % len(FIXED_KNOBS)]
    d = _dev(buf)[lead:]
    want = O.c_batch(buf[lead:], n, stride=stride, seg_len=seg_len, partial=part)
    got = _u16(nsx.fixed_dev(d, stride, seg_len, n, partial=None if part is None else _dev(part.view(np.int32)),
                             tune=knobs))
    assert np.array_equal(got, want), (case, knobs, seg_len, stride, n, lead)


@pytest.mark.parametrize("case", range(90 * SCALE))
def test_fuzz_ragged(case):
    rng = np.random.default_rng(2000 + case)
    n = int(rng.integers(1, 30000))
    hi = int(rng.choice([8, 100, 2000, 9000, 40000]))
    lens = rng.integers(0, hi + 1, n).astype(np.uint64)
    if case % 5 == 0:
        lens[rng.integers(0, n, max(1, n // 10))] = 0
    offs = np.zeros(n + 1, np.uint64)
    np.cumsum(lens, out=offs[1:])
    lead = int(rng.integers(0, 8))
    offs += np.uint64(lead)
    buf = rng.integers(0, 256, int(offs[-1]) + int(rng.integers(0, 5)), dtype=np.uint8)
    part = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32) if case % 2 else None
    knobs = RAGGED_KNOBS[case % len(RAGGED_KNOBS)]
    want = O.c_batch(buf, n, offsets=offs, partial=part)
    d, o = _dev(buf), _dev(offs.view(np.int64))
    p = None if part is None else _dev(part.view(np.int32))
    got = _u16(nsx.ragged_dev(d, o, partial=p, tune=knobs))
    assert np.array_equal(got, want), (case, knobs, n, hi, lead)
    okv = nsx.verify_ragged_dev(d, o, partial=p, tune=knobs).cpu().numpy().astype(bool)
    assert np.array_equal(okv, want == 0xFFFF), (case, knobs)


@pytest.mark.parametrize("case", range(60 * SCALE))
def test_fuzz_ipv4_headers(case):
    rng = np.random.default_rng(3000 + case)
    stride = int(rng.choice([20, 20, 24, 28, 40, 60, 64, int(rng.integers(20, 200)), 1514]))
    hdr_off = 0 if stride == 20 and case % 2 else int(rng.integers(0, min(16, stride - 19)))
    n = int(rng.integers(1, max(2, min(200000, (16 << 20) // stride))))
    buf = rng.integers(0, 256, n * stride + 64, dtype=np.uint8)
    ihl = rng.integers(5, 16, n)
    ihl[rng.random(n) < 0.6] = 5
    ihl[::53] = rng.integers(0, 5, len(ihl[::53]))
    buf[hdr_off:n * stride:stride] = (0x40 | ihl).astype(np.uint8)
    tune = dict(kernel=int(rng.choice([0, 0, nsx.KERNEL_HDR_THREAD, nsx.KERNEL_HDR_DENSE])))
    got = _u16(nsx.ipv4_hdr_csum_dev(_dev(buf), stride, n, hdr_off=hdr_off, mode=0, tune=tune))
    for i in list(range(0, n, max(1, n // 500))) + [n - 1]:
        L = int(ihl[i]) * 4
        ok = L >= 20 and hdr_off + L <= stride
        b0 = i * stride + hdr_off
        assert got[i] == (O.c_fold_checksum(b"", buf[b0:b0 + L].tobytes()) if ok else 0), (case, stride, hdr_off, i)


@pytest.mark.parametrize("case", range(40 * SCALE))
def test_fuzz_tcp_build(case):
    rng = np.random.default_rng(4000 + case)
    n = int(rng.integers(1, 3000))
    P = int(rng.choice([int(rng.integers(0, 40)), 1480, int(rng.integers(0, 3000)), int(rng.integers(0, 9000))]))
    uniform = case % 2 == 0
    lens = np.full(n, P & ~3 if uniform else P, np.uint64) if uniform else rng.integers(0, P + 1, n).astype(np.uint64)
    lead = int(rng.choice([0, 1, 20, 24, 33]))
    data_off = np.zeros(n + 1, np.uint64)
    np.cumsum(lens, out=data_off[1:])
    data_off += np.uint64(lead)
    data = rng.integers(0, 256, int(data_off[-1]) + 8, dtype=np.uint8)
    out_off = nsx.tcp_layout_host(data_off - np.uint64(lead))
    fields = {"src_port": rng.integers(0, 1 << 16, n).astype(np.uint16),
              "dst_port": rng.integers(0, 1 << 16, n).astype(np.uint16),
              "seq_num": rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32),
              "ack_num": rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32),
              "offset": np.full(n, 5, np.uint8), "control": rng.integers(0, 256, n).astype(np.uint8),
              "window": rng.integers(0, 1 << 16, n).astype(np.uint16),
              "urgent_ptr": rng.integers(0, 1 << 16, n).astype(np.uint16)}
    tune = dict(kernel=int(rng.choice([0, nsx.KERNEL_BUILD_PLAIN, nsx.KERNEL_BUILD_GENERAL])),
                blocks_per_cu=int(rng.choice([0, 1, 8])))
    want, wraw = O.c_go_tcp_build(fields, data, data_off, out_off, None)
    dt = {np.uint16: np.int16, np.uint32: np.int32, np.uint8: np.uint8}
    f = {k: _dev(v.view(dt[v.dtype.type])) for k, v in fields.items()}
    out = torch.full((int(out_off[-1]),), 0xAB, dtype=torch.uint8, device="cuda")
    raw = torch.empty(n, dtype=torch.int16, device="cuda")
    nsx.tcp_build_dev(f, _dev(data), _dev(data_off.view(np.int64)), out, _dev(out_off.view(np.int64)), raw=raw,
                      tune=tune)
    assert np.array_equal(_u16(raw), wraw), (case, n, P, lead)
    assert np.array_equal(out.cpu().numpy(), want), (case, n, P, lead)


@pytest.mark.parametrize("case", range(30 * SCALE))
def test_fuzz_tcp_build_options(case):
    """Random option lists per segment (1-byte kinds and kind-2 options with random
    lengths, tcp.go:225-231), mostly ≤ 40 bytes (group-staged in the kernel), some
    longer; option and payload arrays at random alignments; random kernel knobs.
    Expected images from the Python oracle's Segment.bytes() / computeChecksum."""
    rng = np.random.default_rng(5000 + case)
    n = int(rng.integers(1, 400))
    P = int(rng.choice([int(rng.integers(0, 40)), 1468, int(rng.integers(0, 3000))]))
    uniform = case % 2 == 0
    rb = lambda k: rng.integers(0, 256, k, dtype=np.uint8).tobytes()
    long_p = 0.0 if case % 3 else 0.05

    def opts():
        if rng.random() < 0.15:
            return []
        out, left = [], int(rng.integers(1, 41)) if rng.random() >= long_p else int(rng.integers(41, 130))
        while left > 0:
            if left >= 3 and rng.random() < 0.5:
                k = int(rng.integers(1, left - 1))  # kind 2: 2 + k bytes
                out.append(O.Option(kind=2, length=int(rng.integers(0, 256)), data=rb(k)))
                left -= 2 + k
            else:
                out.append(O.Option(kind=int(rng.choice([0, 1, 3, 4, 8]))))
                left -= 1
        return out

    segs, pseudos = [], []
    for i in range(n):
        L = P & ~3 if uniform else int(rng.integers(0, P + 1))
        sg = O.Segment(src_port=int(rng.integers(1 << 16)), dst_port=int(rng.integers(1 << 16)),
                       seq_num=int(rng.integers(1 << 32)), ack_num=int(rng.integers(1 << 32)),
                       control=O.Ctl.from_byte(int(rng.integers(256))), window=int(rng.integers(1 << 16)),
                       urgent_ptr=int(rng.integers(1 << 16)), options=opts(), data=rb(L))
        sg.offset = sg.compute_offset() & 0xFF
        segs.append(sg)
        pseudos.append(O.ipv4_pseudo_header(rb(4), rb(4), 6, len(sg.bytes())))
    want_raw, want = np.empty(n, np.uint16), []
    for i, sg in enumerate(segs):
        sg.checksum = 0
        want_raw[i] = O.c_go_checksum(pseudos[i], sg.bytes())
        sg.checksum = O.field_value(int(want_raw[i]))
        want.append(sg.bytes())
    ob = [b"".join(o.bytes() for o in sg.options) for sg in segs]
    olead, dlead = int(rng.integers(0, 8)), int(rng.choice([0, 3, 60, 64, 130]))
    optarr = np.frombuffer(bytes(olead) + b"".join(ob) + bytes(4), np.uint8)
    opt_off = np.zeros(n + 1, np.uint64)
    opt_off[1:] = np.cumsum([len(b) for b in ob])
    opt_off += np.uint64(olead)
    data = np.frombuffer(rb(dlead) + b"".join(sg.data for sg in segs) + rb(8), np.uint8)
    data_off = np.zeros(n + 1, np.uint64)
    data_off[1:] = np.cumsum([len(sg.data) for sg in segs])
    data_off += np.uint64(dlead)
    out_off = nsx.tcp_layout_host(data_off, opt_off)
    tune = dict(kernel=int(rng.choice([0, nsx.KERNEL_BUILD_PLAIN, nsx.KERNEL_BUILD_GENERAL])),
                blocks_per_cu=int(rng.choice([0, 1, 8])))
    col = lambda k, dt: _dev(np.array([getattr(sg, k) for sg in segs], dt).view(
        {np.uint16: np.int16, np.uint32: np.int32, np.uint8: np.uint8}[dt]))
    f = {"src_port": col("src_port", np.uint16), "dst_port": col("dst_port", np.uint16),
         "seq_num": col("seq_num", np.uint32), "ack_num": col("ack_num", np.uint32),
         "offset": col("offset", np.uint8),
         "control": _dev(np.array([sg.control.byte() for sg in segs], np.uint8)),
         "window": col("window", np.uint16), "urgent_ptr": col("urgent_ptr", np.uint16)}
    part = _dev(np.array([O.be_word_sum(p) for p in pseudos], np.uint32).view(np.int32))
    out = torch.full((int(out_off[-1]),), 0xAB, dtype=torch.uint8, device="cuda")
    raw = torch.empty(n, dtype=torch.int16, device="cuda")
    nsx.tcp_build_dev(f, _dev(data), _dev(data_off.view(np.int64)), out, _dev(out_off.view(np.int64)),
                      opts=_dev(optarr), opt_off=_dev(opt_off.view(np.int64)), partial=part, raw=raw, tune=tune)
    got = out.cpu().numpy()
    assert np.array_equal(_u16(raw), want_raw), (case, n, P)
    for i in range(n):
        o = int(out_off[i])
        assert got[o:o + len(want[i])].tobytes() == want[i], (case, i)
        assert not got[o + len(want[i]):int(out_off[i + 1])].any(), (case, i)


def rx_fuzz_tune(rng) -> dict:
    """A random receive-pass launch shape: one of the default grid's modes (segs_per_wave 0 auto, 5 small-frame,
    6 two-wave prefix, 7 hybrid, 8 streamed, 9 small-frame through the LDS-DMA ring; rows 0 or 2, no blocks_per_cu), or one of the older shapes rows / blocks_per_cu
    select (segs_per_wave 0 auto, 1 streamed, 2 LDS) — never a mode on a grid it does not exist on."""
    if rng.random() < 0.5:
        return dict(rows=int(rng.choice([0, 2])), segs_per_wave=int(rng.choice([0, 5, 6, 7, 8, 9])))
    return dict(rows=int(rng.choice([0, 2, 4, 8, 16])), blocks_per_cu=int(rng.choice([1, 2, 4, 8])),
                segs_per_wave=int(rng.choice([0, 1, 2])))


@pytest.mark.parametrize("case", range(40 * SCALE))
def test_fuzz_rx(case):
    """Random received-datagram batches (every frame kind of tests/_rx.py in random proportions, random start
    alignment, sizes from tiny to a few thousand frames, random launch shape) through the fused receive pass,
    device and host entry points, against oracle_go_rx_ipv4_tcp."""
    import _rx
    rng = np.random.default_rng(6000 + case)
    n = int(rng.choice([int(rng.integers(1, 70)), int(rng.integers(60, 700)), int(rng.integers(500, 3000))]))
    w = rng.random(len(_rx.KINDS)) ** 3
    buf, offs, _ = _rx.batch(rng, n, weights=w / w.sum(), lead=int(rng.integers(0, 8)),
                             max_payload=int(rng.choice([64, 600, 1460, 9000])))
    want_m, want_i, want_t = O.c_rx_ipv4_tcp(buf, offs)
    tune = rx_fuzz_tune(rng)
    mask = torch.empty((n + 63) // 64, dtype=torch.int64, device="cuda")
    ipr, tcpr = torch.empty(n, dtype=torch.int16, device="cuda"), torch.empty(n, dtype=torch.int16, device="cuda")
    nsx.rx_ipv4_tcp_verify_dev(_dev(buf), _dev(offs.view(np.int64)), mask=mask, ip_raw=ipr, tcp_raw=tcpr, tune=tune)
    assert np.array_equal(mask.cpu().numpy().view(np.uint64), want_m), (case, n, tune)
    assert np.array_equal(_u16(ipr), want_i) and np.array_equal(_u16(tcpr), want_t), (case, n, tune)
    if case % 4 == 0:
        assert np.array_equal(nsx.rx_ipv4_tcp_verify_host(buf, offs, tune=dict(shards_per_device=1 + case % 3)),
                              want_m), case


@pytest.mark.parametrize("case", range(30 * SCALE))
def test_fuzz_rx6(case):
    """The IPv6 receive pass over random packet batches (every kind of tests/_rx.py's KINDS6 in random
    proportions, random alignment, sizes and launch shapes), device and host entry points, against
    oracle_go_rx_ipv6_tcp."""
    import _rx
    rng = np.random.default_rng(7000 + case)
    n = int(rng.choice([int(rng.integers(1, 70)), int(rng.integers(60, 700)), int(rng.integers(500, 3000))]))
    w = rng.random(len(_rx.KINDS6)) ** 3
    buf, offs, _ = _rx.batch(rng, n, kinds=_rx.KINDS6, weights=w / w.sum(), lead=int(rng.integers(0, 8)),
                             max_payload=int(rng.choice([64, 600, 1440, 9000])), ip=6)
    want_m, want_t = O.c_rx_ipv6_tcp(buf, offs)
    tune = rx_fuzz_tune(rng)
    mask = torch.empty((n + 63) // 64, dtype=torch.int64, device="cuda")
    tcpr = torch.empty(n, dtype=torch.int16, device="cuda")
    nsx.rx_ipv6_tcp_verify_dev(_dev(buf), _dev(offs.view(np.int64)), mask=mask, tcp_raw=tcpr, tune=tune)
    assert np.array_equal(mask.cpu().numpy().view(np.uint64), want_m), (case, n, tune)
    assert np.array_equal(_u16(tcpr), want_t), (case, n, tune)
    if case % 4 == 0:
        assert np.array_equal(nsx.rx_ipv6_tcp_verify_host(buf, offs, tune=dict(shards_per_device=1 + case % 3)),
                              want_m), case


@pytest.mark.parametrize("case", range(30 * SCALE))
def test_fuzz_parse(case):
    """Random segment batches for the receive-side parse (every kind of tests/_parse.py in random proportions,
    random alignment and sizes) against the oracle's parseSegment (tcp.go:130-185)."""
    import _parse
    rng = np.random.default_rng(8000 + case)
    n = int(rng.choice([int(rng.integers(1, 70)), int(rng.integers(60, 700)), int(rng.integers(500, 4000))]))
    w = rng.random(len(_parse.KINDS)) ** 3
    buf, offs, _ = _parse.batch(rng, n, weights=w / w.sum(), lead=int(rng.integers(0, 8)),
                                max_payload=int(rng.choice([0, 40, 600, 1460])))
    exp = _parse.expected(buf, offs)
    got = nsx.tcp_parse_dev(_dev(buf), _dev(offs.view(np.int64)))
    for k, v in got.items():
        assert np.array_equal(v.cpu().numpy().view(exp[k].dtype), exp[k]), (case, k)
