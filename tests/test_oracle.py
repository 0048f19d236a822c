"""Oracle pinning (CPU): the restatement against the reference's own test, RFC
1071 and the committed golden fixtures; the four formulations against each
other. Mirrors transport/tcp/tcp_test.go for the segment model."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import csum_oracle as O


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


# --- transport/tcp/tcp_test.go, restated against the oracle segment model ---

def test_reference_TestSegmentComputeChecksum():
    """tcp_test.go:26-32: field = ^sum; the re-sum over the same segment is 0xFFFF."""
    s = O.Segment(data=b"hello")
    s.checksum = (~s.compute_checksum(b"")) & 0xFFFF
    assert s.compute_checksum(b"") == 0xFFFF, f"{s.checksum:b}"
    # and with the C restatements
    assert O.c_go_checksum(b"", s.bytes()) == 0xFFFF
    assert O.c_fold_checksum(b"", s.bytes()) == 0xFFFF


def test_reference_TestSegmentComputeOffset():
    """tcp_test.go:11-24."""
    s = O.Segment()
    assert s.compute_offset() == 20 // 4
    s.options.append(O.Option())
    assert s.compute_offset() == 20 // 4 + 1


def test_reference_TestSegmentCodec_bytes():
    """tcp_test.go:34-55 builds this segment; its bytes() layout (tcp.go:98-128)."""
    s = O.Segment(src_port=1, dst_port=2, seq_num=3, ack_num=4, offset=5, window=6, checksum=7,
                  urgent_ptr=8, data=bytes([9]))
    s.offset = s.compute_offset()
    assert s.bytes().hex() == "00010002" "00000003" "00000004" "05" "00" "0006" "0007" "0008" "09"


def test_reference_TestCTLCodec():
    """tcp_test.go:57-67."""
    c = O.Ctl(urg=True, rst=True)
    assert O.Ctl.from_byte(c.byte()) == c
    assert c.byte() == 0b00100100


# --- KATs and formulation agreement ---

@pytest.mark.parametrize("case", load("kat.json"), ids=lambda c: c["name"])
def test_kat(case):
    p, s = bytes.fromhex(case["prefix"]), bytes.fromhex(case["segment"])
    for f in (O.go_checksum, O.fold_checksum, O.c_go_checksum, O.c_fold_checksum):
        assert f(p, s) == case["raw"], f.__name__
    assert case["field"] == (~case["raw"]) & 0xFFFF


def test_kat_sender_receiver_roundtrip():
    """Storing field=^raw at bytes 16-17 (tcp.go:110) makes the receiver's sum 0xFFFF."""
    rng = np.random.default_rng(7)
    for n in (0, 1, 5, 100, 1480):
        seg = O.Segment(src_port=int(rng.integers(65536)), dst_port=443, seq_num=int(rng.integers(1 << 32)),
                        data=rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        seg.offset = seg.compute_offset()
        pseudo = O.ipv4_pseudo_header(b"\x0a\x00\x00\x01", b"\x0a\x00\x00\x02", 6, len(seg.bytes()))
        seg.checksum = O.field_value(seg.compute_checksum(pseudo))
        assert O.verify(seg.compute_checksum(pseudo))


def test_random_agreement_all_formulations():
    rng = np.random.default_rng(0xC0FFEE)
    for _ in range(400):
        n = int(rng.integers(0, 700))
        pl = int(rng.integers(0, 45))
        kind = rng.integers(0, 4)
        if kind == 0:
            seg = bytes(n)
        elif kind == 1:
            seg = b"\xff" * n
        else:
            seg = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        pre = rng.integers(0, 256, pl, dtype=np.uint8).tobytes()
        want = O.go_checksum(pre, seg)
        assert O.fold_checksum(pre, seg) == want
        assert O.c_go_checksum(pre, seg) == want
        assert O.c_fold_checksum(pre, seg) == want


def test_zero_only_for_all_zero_input():
    rng = np.random.default_rng(3)
    for _ in range(200):
        n = int(rng.integers(1, 64))
        seg = bytearray(n)
        seg[int(rng.integers(n))] = int(rng.integers(1, 256))
        assert O.c_go_checksum(b"", bytes(seg)) != 0


# --- golden fixtures ---

def test_golden_vectors():
    idx = load("vectors.json")
    blob = np.fromfile(os.path.join(GOLDEN, "vectors.bin"), np.uint8)
    for c in idx:
        seg = blob[c["offset"]:c["offset"] + c["length"]].tobytes()
        pre = bytes.fromhex(c["prefix"])
        assert O.c_go_checksum(pre, seg) == c["raw"]
        assert O.c_fold_checksum(b"", seg) == c["raw_no_prefix"]
        assert O.fold(O.be_word_sum(seg) + c["prefix_partial"]) == c["raw"]


def test_golden_ragged():
    meta = load("ragged.json")
    blob = np.fromfile(os.path.join(GOLDEN, "ragged.bin"), np.uint8)
    offs = np.array(meta["offsets"], np.uint64)
    part = np.array(meta["partial"], np.uint32)
    assert O.c_batch(blob, offs.size - 1, offsets=offs).tolist() == meta["raw"]
    assert O.c_batch(blob, offs.size - 1, offsets=offs, partial=part).tolist() == meta["raw_with_partial"]
    assert O.batch_ragged(blob, offs).tolist() == meta["raw"]


def test_golden_segments():
    for c in load("segments.json"):
        b = bytes.fromhex(c["bytes"])
        assert O.go_checksum(b"", b) == c["raw"]
        assert O.go_checksum(bytes.fromhex(c["pseudo_ipv4"]), b) == c["raw_with_pseudo"]


def test_reference_option_padding_quirk():
    """tcp.go:118-121 pads `remainder` zero bytes, not 4-remainder: 20 B + MSS(6)
    = 26 → remainder 2 → 28 B (aligned by luck); NOOP: 21 → +1 → 22 (not 24)."""
    s = O.Segment(options=[O.Option(kind=1)])
    assert len(s.bytes()) == 22
    s = O.Segment(options=[O.Option(kind=2, length=4, data=b"\x05\xb4\x00\x00")])
    assert len(s.bytes()) == 28


# --- synthetic data generator ---

def test_splitmix64_py_vs_c():
    for off, n in ((0, 64), (3, 61), (8, 1000), (12345, 777)):
        assert np.array_equal(O.splitmix64_bytes(0x1071, off, n), O.c_splitmix64(0x1071, n, off))


def test_batch_fixed_numpy_vs_c():
    buf = O.c_splitmix64(0x1071, 1500 * 64)
    a = O.batch_fixed(buf, 1500, 1500, 64)
    b = O.c_batch(buf, 64, stride=1500, seg_len=1500)
    assert np.array_equal(a, b)
    for i in (0, 17, 63):
        assert a[i] == O.go_checksum(b"", buf[i * 1500:(i + 1) * 1500].tobytes())


def test_c_go_tcp_build_matches_segment_model():
    """The C Go-faithful sender loop (bench cpu_baseline / checker for workload 6)
    agrees with the Python Segment model (tcp.go:98-128 + :68-71) byte for byte."""
    rng = np.random.default_rng(606)
    n = 200
    lens = rng.integers(0, 1600, n).astype(np.uint64)
    lens[:3] = [0, 1, 1480]
    data = rng.integers(0, 256, int(lens.sum()) + 1, dtype=np.uint8)
    data_off = np.zeros(n + 1, np.uint64)
    data_off[1:] = np.cumsum(lens)
    fields = {k: rng.integers(0, np.iinfo(dt).max + 1, n, dtype=np.uint64).astype(dt)
              for k, dt in zip(O.TCP_FIELDS, O.TCP_FIELD_DTYPES)}
    pseudo = rng.integers(0, 256, (n, 12), dtype=np.uint8)
    out_off = np.zeros(n + 1, np.uint64)
    out_off[1:] = np.cumsum(lens + np.uint64(20))
    wire, raw = O.c_go_tcp_build(fields, data, data_off, out_off, pseudo)
    for i in range(n):
        s = O.Segment(src_port=int(fields["src_port"][i]), dst_port=int(fields["dst_port"][i]),
                      seq_num=int(fields["seq_num"][i]), ack_num=int(fields["ack_num"][i]),
                      offset=int(fields["offset"][i]), control=O.Ctl.from_byte(int(fields["control"][i])),
                      window=int(fields["window"][i]), urgent_ptr=int(fields["urgent_ptr"][i]),
                      data=data[int(data_off[i]):int(data_off[i + 1])].tobytes())
        r = s.compute_checksum(pseudo[i].tobytes())
        assert raw[i] == r
        s.checksum = O.field_value(r)
        assert wire[int(out_off[i]):int(out_off[i + 1])].tobytes() == s.bytes()
    # the threaded form (full-size GPU checks of workloads 6 and 12) is the same loop over index shards
    for t in (1, 3, 16):
        w2, r2 = O.c_go_tcp_build_mt(fields, data, data_off, out_off, pseudo, threads=t)
        assert np.array_equal(w2, wire) and np.array_equal(r2, raw), t


def test_c_go_tcp_build_opts_matches_segment_model():
    """The C sender loop for segments with options (bench cpu_baseline / checker for
    workload 8) agrees with the Python Segment model, including the reference's
    `remainder` option padding (tcp.go:118-121), for option lists of every kind."""
    rng = np.random.default_rng(607)
    n = 200
    rb = lambda k: rng.integers(0, 256, k, dtype=np.uint8).tobytes()
    sets = [lambda: [], lambda: [O.Option(kind=1)], lambda: [O.Option(kind=1)] * 3,
            lambda: [O.Option(kind=1), O.Option(kind=1), O.Option(kind=2, length=10, data=rb(8))],
            lambda: [O.Option(kind=2, length=4, data=rb(2)), O.Option(kind=0)],
            lambda: [O.Option(kind=2, length=200, data=rb(int(rng.integers(0, 60))))]]
    segs = []
    for i in range(n):
        sg = O.Segment(src_port=int(rng.integers(1 << 16)), dst_port=int(rng.integers(1 << 16)),
                       seq_num=int(rng.integers(1 << 32)), ack_num=int(rng.integers(1 << 32)),
                       control=O.Ctl.from_byte(int(rng.integers(256))), window=int(rng.integers(1 << 16)),
                       urgent_ptr=int(rng.integers(1 << 16)), options=sets[i % len(sets)](),
                       data=rb(int(rng.integers(0, 1600))))
        sg.offset = sg.compute_offset() & 0xFF
        segs.append(sg)
    ob = [b"".join(o.bytes() for o in sg.options) for sg in segs]
    opts = np.frombuffer(b"".join(ob), np.uint8)
    opt_off = np.zeros(n + 1, np.uint64)
    opt_off[1:] = np.cumsum([len(b) for b in ob])
    data = np.frombuffer(b"".join(sg.data for sg in segs) + b"\0", np.uint8)
    data_off = np.zeros(n + 1, np.uint64)
    data_off[1:] = np.cumsum([len(sg.data) for sg in segs])
    out_off = np.zeros(n + 1, np.uint64)
    out_off[1:] = np.cumsum([len(sg.bytes()) for sg in segs])
    pseudo = rng.integers(0, 256, (n, 12), dtype=np.uint8)
    fields = {"src_port": np.array([sg.src_port for sg in segs], np.uint16),
              "dst_port": np.array([sg.dst_port for sg in segs], np.uint16),
              "seq_num": np.array([sg.seq_num for sg in segs], np.uint32),
              "ack_num": np.array([sg.ack_num for sg in segs], np.uint32),
              "offset": np.array([sg.offset for sg in segs], np.uint8),
              "control": np.array([sg.control.byte() for sg in segs], np.uint8),
              "window": np.array([sg.window for sg in segs], np.uint16),
              "urgent_ptr": np.array([sg.urgent_ptr for sg in segs], np.uint16)}
    wire, raw = O.c_go_tcp_build_opts(fields, opts, opt_off, data, data_off, out_off, pseudo)
    for i, sg in enumerate(segs):
        r = sg.compute_checksum(pseudo[i].tobytes())
        assert raw[i] == r, i
        sg.checksum = O.field_value(r)
        assert wire[int(out_off[i]):int(out_off[i + 1])].tobytes() == sg.bytes(), i
    for t in (1, 7):  # the threaded form (full-size GPU check of workload 8)
        w2, r2 = O.c_go_tcp_build_mt(fields, data, data_off, out_off, pseudo, opts=opts, opt_off=opt_off, threads=t)
        assert np.array_equal(w2, wire) and np.array_equal(r2, raw), t


def test_cpu_fast_line_matches_go_checksum():
    """The best-CPU reference line (bench extras) computes the reference's sums."""
    rng = np.random.default_rng(707)
    for L in (0, 1, 2, 3, 31, 32, 33, 63, 1500, 1501, 9000):
        n = 37
        buf = rng.integers(0, 256, n * (L + 3) + 1, dtype=np.uint8)
        buf[: L + 3] = 0xFF
        out = np.empty(n, np.uint16)
        O.c_fast().cpu_fast_batch_fixed(buf[1:].ctypes.data, L + 3, L, n, None, out.ctypes.data, 4)
        for i in range(n):
            seg = buf[1 + i * (L + 3):1 + i * (L + 3) + L].tobytes()
            assert out[i] == O.c_go_checksum(b"", seg), (L, i)
        # with per-segment IPv4 pseudo-headers given as partials (config 2's headline form)
        ph = rng.integers(0, 256, (n, 12), dtype=np.uint8)
        part = np.array([O.be_word_sum(p.tobytes()) for p in ph], np.uint32)
        O.c_fast().cpu_fast_batch_fixed(buf[1:].ctypes.data, L + 3, L, n, part.ctypes.data, out.ctypes.data, 4)
        go = np.empty(n, np.uint16)
        O.c_oracle().oracle_go_batch_fixed_pseudo(buf[1:].ctypes.data, L + 3, L, n, ph.ctypes.data, 12,
                                                  go.ctypes.data)
        for i in range(n):
            seg = buf[1 + i * (L + 3):1 + i * (L + 3) + L].tobytes()
            assert out[i] == go[i] == O.go_checksum(ph[i].tobytes(), seg), (L, i)


# --- fused receive check (SURVEY.md §8 f2 + f3): Python vs C restatement, fixtures, per-kind rules ---

def test_rx_golden_fixture_both_restatements():
    meta = load("rx.json")
    blob = np.fromfile(os.path.join(GOLDEN, "rx.bin"), np.uint8)
    offs = np.array(meta["offsets"], np.uint64)
    mask, ipr, tcpr = O.c_rx_ipv4_tcp(blob, offs)
    assert mask.tolist() == meta["mask"] and ipr.tolist() == meta["ip_raw"] and tcpr.tolist() == meta["tcp_raw"]
    for i in range(offs.size - 1):
        f = blob[int(offs[i]):int(offs[i + 1])].tobytes()
        assert O.rx_ipv4_tcp(f) == (meta["ip_raw"][i], meta["tcp_raw"][i], meta["valid"][i]), i
    assert 0 < sum(meta["valid"]) < len(meta["valid"])


def test_rx_rules_per_kind():
    """Every kind of frame tests/_rx.py builds lands on the side of the check it should: the valid kinds
    pass (and their TCP segments re-verify through computeChecksum with the pseudo-header, tcp.go:70), every
    broken or malformed kind fails, with the raw sums zeroed exactly where the rules say."""
    import _rx
    rng = np.random.default_rng(0x78)
    for kind in _rx.KINDS:
        for _ in range(20):
            f = _rx.frame(rng, kind, max_payload=200)
            ipr, tcpr, ok = O.rx_ipv4_tcp(f)
            assert ok == (kind in ("valid", "valid_options", "header_only", "odd_payload")), (kind, f.hex())
            if kind in ("short", "empty", "ihl_lt5", "ihl_past_end"):
                assert ipr == 0 and tcpr == 0, kind
            if kind in ("udp", "fragment_mf", "fragment_off", "version6", "total_mismatch", "tcp_lt20"):
                assert tcpr == 0 and (kind == "total_mismatch" or ipr == 0xFFFF), kind


def test_rx_rfc791_header_is_not_tcp():
    h = bytearray.fromhex("45000073000040004011b861c0a80001c0a800c7")  # RFC 791 §3.1 example: UDP
    f = bytes(h) + bytes(0x73 - 20)
    assert O.rx_ipv4_tcp(f) == (0xFFFF, 0, False)
    h[9] = 6  # as TCP the header sum breaks
    assert O.rx_ipv4_tcp(bytes(h) + bytes(0x73 - 20))[2] is False


def test_rx6_golden_fixture_both_restatements():
    meta = load("rx6.json")
    blob = np.fromfile(os.path.join(GOLDEN, "rx6.bin"), np.uint8)
    offs = np.array(meta["offsets"], np.uint64)
    mask, tcpr = O.c_rx_ipv6_tcp(blob, offs)
    assert mask.tolist() == meta["mask"] and tcpr.tolist() == meta["tcp_raw"]
    for i in range(offs.size - 1):
        f = blob[int(offs[i]):int(offs[i + 1])].tobytes()
        assert O.rx_ipv6_tcp(f) == (meta["tcp_raw"][i], meta["valid"][i]), i
    assert 0 < sum(meta["valid"]) < len(meta["valid"])


def test_rx6_rules_per_kind():
    """Every IPv6 kind lands on the side of the check it should; a valid packet's TCP sum re-verifies through
    the wide-form sum over the RFC 8200 §8.1 pseudo-header built by hand (independent of rx_ipv6_tcp's slicing),
    and malformed packets report tcp_raw 0."""
    import _rx
    rng = np.random.default_rng(0x7A)
    for kind in _rx.KINDS6:
        for _ in range(20):
            f = _rx.frame6(rng, kind, max_payload=200)
            tcpr, ok = O.rx_ipv6_tcp(f)
            assert ok == (kind in _rx.VALID6), (kind, f.hex())
            if kind in _rx.VALID6:
                pseudo = f[8:40] + (len(f) - 40).to_bytes(4, "big") + b"\0\0\0\x06"
                assert O.fold_checksum(pseudo, f[40:]) == 0xFFFF
            if kind in ("short", "empty", "udp", "ext_header", "len_short", "len_long", "version4", "tcp_lt20",
                        "jumbo"):
                assert tcpr == 0, kind
            if kind in ("bad_tcp_sum", "bad_addr"):
                assert tcpr not in (0, 0xFFFF), kind


def test_rx6_c_matches_python_random_batches():
    import _rx
    rng = np.random.default_rng(0x7B)
    for lead in (0, 1, 2, 3):
        buf, offs, kinds = _rx.batch(rng, 300, kinds=_rx.KINDS6, lead=lead, max_payload=400, ip=6)
        mask, tcpr = O.c_rx_ipv6_tcp(buf, offs)
        bits = np.unpackbits(mask.view(np.uint8), bitorder="little")[:300]
        for i in range(300):
            a, v = O.rx_ipv6_tcp(buf[int(offs[i]):int(offs[i + 1])].tobytes())
            assert (tcpr[i], bool(bits[i])) == (a, v), (i, kinds[i])


def test_parse_segment_restates_reference_cases():
    """parseSegment (tcp.go:130-185) on the reference's own case (tcp_test.go:26-32: segment{data:"hello"},
    offset 0, so dataAt 0 and the data is the whole segment), round trips of bytes() with the options the
    reference serialises faithfully (NOP, MSS of length 4), and every error and would-panic/loop case."""
    s, st = O.parse_segment(bytes(20) + b"hello")
    assert st == O.PARSE_OK and s.offset == 0 and s.data == bytes(20) + b"hello" and s.options == []
    t = O.Segment(src_port=1, dst_port=2, seq_num=3, ack_num=4, control=O.Ctl.from_byte(0x12), window=5,
                  checksum=6, urgent_ptr=7, options=[O.Option(kind=1), O.Option(kind=2, length=4, data=b"abcd")],
                  data=b"payload")
    t.offset = t.compute_offset()
    # 7 option bytes: bytes() pads 27 → 30 with `remainder` = 3 zeros (tcp.go:118-121) while offset = 7 puts
    # dataAt at 28, so the parsed data starts with the last 2 padding bytes
    s, st = O.parse_segment(t.bytes())
    assert st == O.PARSE_OK and s.options == t.options and s.data == b"\0\0payload"
    t.options.insert(0, O.Option(kind=1))  # 8 option bytes: no padding, an exact round trip
    t.offset = t.compute_offset()
    s, st = O.parse_segment(t.bytes())
    assert st == O.PARSE_OK and s == t
    assert O.parse_segment(bytes(19))[1] == O.PARSE_SHORT
    b = bytearray(t.bytes())
    b[12] = 200
    assert O.parse_segment(bytes(b)) == (O.Segment(), O.PARSE_OFFSET)
    b = bytearray(t.bytes())
    b[23] = 60  # MSS length past the end (options NOP NOP MSS: the length byte is 23)
    assert O.parse_segment(bytes(b))[1] == O.PARSE_OPTION_RANGE
    b = bytearray(t.bytes())
    b[20] = 9  # unknown kind
    assert O.parse_segment(bytes(b))[1] == O.PARSE_OPTION_KIND


def test_parse_golden_fixture_is_the_oracle():
    import _parse
    meta = load("parse.json")
    blob = np.fromfile(os.path.join(GOLDEN, "parse.bin"), np.uint8)
    exp = _parse.expected(blob, np.array(meta["offsets"], np.uint64))
    for k, v in exp.items():
        assert v.tolist() == meta[k], k
    assert set(meta["status"]) == {0, 1, 2, 3, 4}


def test_rx_c_matches_python_random_batches():
    import _rx
    rng = np.random.default_rng(0x79)
    for lead in (0, 1, 2, 3):
        buf, offs, kinds = _rx.batch(rng, 300, lead=lead, max_payload=400)
        mask, ipr, tcpr = O.c_rx_ipv4_tcp(buf, offs)
        bits = np.unpackbits(mask.view(np.uint8), bitorder="little")[:300]
        for i in range(300):
            a, b, v = O.rx_ipv4_tcp(buf[int(offs[i]):int(offs[i + 1])].tobytes())
            assert (ipr[i], tcpr[i], bool(bits[i])) == (a, b, v), (i, kinds[i])
