"""GPU parity first in line (collected before every other -m gpu file, so that
`pytest -x` can never stop ahead of them): the committed golden fixtures and the
reference's own test (transport/tcp/tcp_test.go:26-32) through the device entry
points, then BASELINE.json's device-resident configurations at full size, every
segment of each against the oracle: config 2 (1M x 1500 B), config 3 (1M ragged
64-9000 B), config 4 (256K x 64 KiB, 16 GiB) and config 5 (16M x 1500 B per GPU,
23.4 GiB; the two large ones come back to the host in ~1 GiB chunks), plus
size-independent properties on every segment. Bit-exact throughout (integer
work)."""
import json
import os

import numpy as np
import pytest

from _gpu import dev, host, pseudo_headers, run_fixed, run_ragged, setup_gpu, torch, u16
from conftest import GOLDEN
from oracle import csum_oracle as O

import nsx  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu():
    setup_gpu()


# ------------------------------------------------------------------ golden fixtures

def test_golden_vectors_fixed_and_ragged():
    """tests/golden/vectors.*: 86 cases (lengths 0-65536, start misalignment 0-7, no / IPv4 / IPv6
    prefix) through the fixed entry point (with and without the prefix partial) and the ragged one."""
    idx = json.load(open(os.path.join(GOLDEN, "vectors.json")))
    blob = np.fromfile(os.path.join(GOLDEN, "vectors.bin"), np.uint8)
    d = dev(blob)
    for c in idx:
        out = torch.empty(1, dtype=torch.int16, device="cuda")
        part = dev(np.array([c["prefix_partial"]], np.uint32).view(np.int32))
        nsx.fixed_dev(d[c["offset"]:], 0, c["length"], 1, partial=part, out=out)
        assert u16(out)[0] == c["raw"], c
        nsx.fixed_dev(d[c["offset"]:], 0, c["length"], 1, out=out)
        assert u16(out)[0] == c["raw_no_prefix"], c
        r = run_ragged(blob, [c["offset"], c["offset"] + c["length"]])
        assert r[0] == c["raw_no_prefix"], c


def test_golden_ragged_batch():
    meta = json.load(open(os.path.join(GOLDEN, "ragged.json")))
    blob = np.fromfile(os.path.join(GOLDEN, "ragged.bin"), np.uint8)
    assert run_ragged(blob, meta["offsets"]).tolist() == meta["raw"]
    assert run_ragged(blob, meta["offsets"], meta["partial"]).tolist() == meta["raw_with_partial"]


def test_golden_kat_and_reference_test():
    for c in json.load(open(os.path.join(GOLDEN, "kat.json"))):
        seg = np.frombuffer(bytes.fromhex(c["segment"]) or b"\0", np.uint8)
        L = len(bytes.fromhex(c["segment"]))
        partial = [O.be_word_sum(bytes.fromhex(c["prefix"]))]
        if len(bytes.fromhex(c["prefix"])) % 2:
            continue  # the device API's prefix partial requires an even-length prefix
        assert run_fixed(seg, 0, L, 1, partial)[0] == c["raw"], c["name"]


def test_reference_TestSegmentComputeChecksum_on_device():
    """tcp_test.go:26-32 on the device: segment{data:"hello"} (offset 0, every header field 0;
    tests/golden/segments.json) → raw 0x43D2; store ^sum at bytes 16-17, the re-sum is 0xFFFF."""
    case = next(c for c in json.load(open(os.path.join(GOLDEN, "segments.json")))
                if c["name"] == "TestSegmentComputeChecksum")
    b = np.frombuffer(bytes.fromhex(case["bytes"]), np.uint8).copy()
    assert b.size == 25 and b[12] == 0 and case["raw"] == 0x43D2
    raw = run_fixed(b, 0, len(b), 1)[0]
    assert raw == case["raw"]
    b[16], b[17] = (~raw & 0xFFFF) >> 8, (~raw) & 0xFF
    assert run_fixed(b, 0, len(b), 1)[0] == 0xFFFF
    # the same through the ragged entry point at an odd start
    pad = np.concatenate([np.zeros(1, np.uint8), b])
    assert run_ragged(pad, [1, 26])[0] == 0xFFFF


def _segment_cases():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLDEN, "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    return mg.segment_cases()


def _same_segment(a, b) -> bool:
    """assert.Equal(t, original, got) of tcp_test.go:54 over the Python segment model."""
    return (a.src_port, a.dst_port, a.seq_num, a.ack_num, a.offset, a.control.byte(), a.window, a.checksum,
            a.urgent_ptr, [(o.kind, o.length, bytes(o.data)) for o in a.options], bytes(a.data)) == \
        (b.src_port, b.dst_port, b.seq_num, b.ack_num, b.offset, b.control.byte(), b.window, b.checksum,
         b.urgent_ptr, [(o.kind, o.length, bytes(o.data)) for o in b.options], bytes(b.data))


@pytest.mark.parametrize("pseudo", [False, True])
def test_reference_TestSegmentCodec_on_device(pseudo):
    """tcp_test.go:34-55 (and the option segments of tests/golden/segments.json) through the device pair:
    nsx_tcp_build_dev serialises each segment (bytes(), tcp.go:98-128) and writes ^raw into the field
    (tcp.go:68-71); nsx_tcp_parse_dev parses the images back (parseSegment, tcp.go:130-185). Checked: the raw
    sum equals the oracle's computeChecksum over the image with the field zero (with and without an IPv4
    pseudo-header), the image equals the oracle's bytes() with that field, the receiver's re-sum is 0xFFFF,
    and every parsed field equals the oracle's parseSegment of the same image. The reference's own assertion
    `parse(bytes(s)) == s` (field taken from the image) holds on the device for TestSegmentCodec and every
    case where the oracle says it holds; the padding-quirk cases (tcp.go:118-121: NOP padded by `remainder`,
    an explicit EOL dropped by the parse) must fail it on the device exactly as in the oracle."""
    cases = _segment_cases()
    names = [c[0] for c in cases]
    segs = [c[1] for c in cases]
    n = len(segs)
    addr = [(bytes([192, 168, 0, 1 + i]), bytes([10, 0, i, 2])) for i in range(n)]
    pseudos = [O.ipv4_pseudo_header(a, b, 6, len(s.bytes())) if pseudo else b"" for (a, b), s in zip(addr, segs)]
    data = b"".join(s.data for s in segs) or b"\0"
    data_off = np.zeros(n + 1, np.uint64)
    data_off[1:] = np.cumsum([len(s.data) for s in segs])
    opts = b"".join(o.bytes() for s in segs for o in s.options) or b"\0"
    opt_off = np.zeros(n + 1, np.uint64)
    opt_off[1:] = np.cumsum([sum(len(o.bytes()) for o in s.options) for s in segs])
    out_off = nsx.tcp_layout_host(data_off, opt_off)
    u = lambda a, dt, vt: dev(np.asarray(a, dt).view(vt))  # noqa: E731
    fields = {"src_port": u([s.src_port for s in segs], np.uint16, np.int16),
              "dst_port": u([s.dst_port for s in segs], np.uint16, np.int16),
              "seq_num": u([s.seq_num for s in segs], np.uint32, np.int32),
              "ack_num": u([s.ack_num for s in segs], np.uint32, np.int32),
              "offset": u([s.offset for s in segs], np.uint8, np.uint8),
              "control": u([s.control.byte() for s in segs], np.uint8, np.uint8),
              "window": u([s.window for s in segs], np.uint16, np.int16),
              "urgent_ptr": u([s.urgent_ptr for s in segs], np.uint16, np.int16)}
    part = dev(np.array([O.be_word_sum(p) for p in pseudos], np.uint32).view(np.int32)) if pseudo else None
    out = torch.full((int(out_off[-1]),), 0xAB, dtype=torch.uint8, device="cuda")
    raw = torch.empty(n, dtype=torch.int16, device="cuda")
    nsx.tcp_build_dev(fields, dev(np.frombuffer(data, np.uint8)), dev(data_off.view(np.int64)), out,
                      dev(out_off.view(np.int64)), opts=dev(np.frombuffer(opts, np.uint8)),
                      opt_off=dev(opt_off.view(np.int64)), partial=part, raw=raw)
    img_all, raw_h = host(out), u16(raw)
    images = []
    for i, s in enumerate(segs):
        zero = O.Segment(**{**s.__dict__, "checksum": 0})
        want_raw = O.go_checksum(pseudos[i], zero.bytes())        # computeChecksum with the field zero
        assert raw_h[i] == want_raw, names[i]
        sent = O.Segment(**{**s.__dict__, "checksum": O.field_value(want_raw)})
        img = img_all[int(out_off[i]):int(out_off[i]) + len(sent.bytes())].tobytes()
        assert img == sent.bytes(), names[i]                      # bytes() with ^raw at 16-17 (tcp.go:110)
        assert O.verify(O.go_checksum(pseudos[i], img)), names[i]  # tcp.go:70
        images.append((sent, img))
    # the images back through the device parse, densely packed behind an odd lead
    blob = b"\x77" + b"".join(img for _, img in images)
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum([len(img) for _, img in images])
    offs += np.uint64(1)
    got = nsx.tcp_parse_dev(dev(np.frombuffer(blob, np.uint8)), dev(offs.view(np.int64)))
    g = {k: host(v).view({1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[v.element_size()])
         for k, v in got.items()}
    holds = {}
    for i, (sent, img) in enumerate(images):
        exp, status = O.parse_segment(img)
        assert g["status"][i] == status == O.PARSE_OK, names[i]
        for k in ("src_port", "dst_port", "seq_num", "ack_num", "offset", "window", "checksum", "urgent_ptr"):
            assert int(g[k][i]) == getattr(exp, k), (names[i], k)
        assert int(g["control"][i]) == exp.control.byte(), names[i]
        assert int(g["n_options"][i]) == len(exp.options), names[i]
        assert blob[int(g["data_off"][i]):int(offs[i + 1])] == exp.data, names[i]
        # the reference's assertion, on what the device parsed (options: kinds/lengths/data from the image)
        dev_seg = O.Segment(src_port=int(g["src_port"][i]), dst_port=int(g["dst_port"][i]),
                            seq_num=int(g["seq_num"][i]), ack_num=int(g["ack_num"][i]), offset=int(g["offset"][i]),
                            control=O.Ctl.from_byte(int(g["control"][i])), window=int(g["window"][i]),
                            checksum=int(g["checksum"][i]), urgent_ptr=int(g["urgent_ptr"][i]),
                            options=exp.options, data=blob[int(g["data_off"][i]):int(offs[i + 1])])
        holds[names[i]] = _same_segment(dev_seg, sent)
        assert holds[names[i]] == _same_segment(exp, sent), names[i]
    assert holds["TestSegmentCodec"] and holds["ctl_urg_rst"] and holds["option_mss"]
    assert not holds["option_noop"] and not holds["options_mss_noop_eol"]  # the reference's padding quirk


# ------------------------------------------------------------------ BASELINE configs at full size

def ipv4_pseudo_partials(addrs: np.ndarray, tcp_len: int) -> np.ndarray:
    """The BE-word sum of each segment's 12 B IPv4 pseudo-header src(4) dst(4) 0 6 len(2) (RFC 9293 §3.1;
    ip.Addr.Raw(), network/ip/v4/ipv4.go:15; ip.NextProtoTCP, protocols.go:8), from (2, n, 4) address bytes."""
    a = addrs.astype(np.uint32)
    return ((a[..., 0] << 8) + a[..., 1] + (a[..., 2] << 8) + a[..., 3]).sum(0).astype(np.uint32) + 6 + tcp_len


def test_config2_1M_x_1500_full():
    """Config 2 exactly as bench.py times it (bench.build_workload): 1M x 1500 B, each segment over its own IPv4
    pseudo-header given as the N x u32 partials SURVEY.md §8d specifies (tcp.go:72-73), generated on the device
    by nsx_pseudo_ipv4_partial_dev. Every segment against the oracle fed partials computed on the host from the
    same addresses; a sample against the Go-faithful loop over the 12 B pseudo-header bytes themselves; then
    the same batch without partials."""
    import bench
    n, L = 1 << 20, 1500
    w = bench.build_workload(bench.WORKLOADS[2], 0, torch.device("cuda"))
    t = w["buf"]
    assert w["alg"] == n * L + 2 * n + 4 * n and w["part"] is not None
    h = host(t)
    assert np.array_equal(h[:4096], O.c_splitmix64(0x1071, 4096))
    assert np.array_equal(h[-4096:], O.c_splitmix64(0x1071, 4096, n * L - 4096))
    addrs = host(w["addrs"])
    part = ipv4_pseudo_partials(addrs, L)
    assert np.array_equal(np.array([O.fold(int(x)) for x in host(w["part"]).view(np.uint32)[:4096]]),
                          np.array([O.fold(int(x)) for x in part[:4096]]))
    w["step"]()
    got = u16(w["out"])
    want = O.c_batch(h, n, stride=L, seg_len=L, partial=part, threads=16)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (bad[:8], got[bad[:8]], want[bad[:8]])
    # the Go-faithful loop over the pseudo-header bytes (allocate, concatenate, serial compare-carry) on a sample
    m = 20000
    go = np.empty(m, np.uint16)
    ph = pseudo_headers(addrs[:, :m], L)
    O.c_oracle().oracle_go_batch_fixed_pseudo(h.ctypes.data, L, L, m, ph.ctypes.data, 12, go.ctypes.data)
    assert np.array_equal(go, got[:m])
    w["step"]()
    assert np.array_equal(u16(w["out"]), got)  # idempotent
    # the partial-less form over the same bytes
    out = nsx.fixed_dev(t, L, L, n, out=torch.empty(n, dtype=torch.int16, device="cuda"))
    assert np.array_equal(u16(out), O.c_batch(h, n, stride=L, seg_len=L, threads=16))


def test_config3_1M_ragged_full():
    n = 1 << 20
    rng = np.random.default_rng(0x1072)
    lens = rng.integers(64, 9001, n).astype(np.uint64)
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    t = torch.empty(int(offs[-1]), dtype=torch.uint8, device="cuda")
    nsx.fill_splitmix64_dev(t, 0x1072)
    want = O.c_batch(host(t), n, offsets=offs, threads=16)
    d_offs = dev(offs.view(np.int64))
    for tune in (None, dict(kernel=nsx.KERNEL_SCAN_PLAIN, rows=16, run_segs=16), dict(blocks_per_cu=1, rows=8)):
        out = nsx.ragged_dev(t, d_offs, out=torch.empty(n, dtype=torch.int16, device="cuda"), tune=tune)
        assert np.array_equal(u16(out), want), tune


def oracle_fixed_chunked(t, n, L, S, seed=None, chunk=1 << 30, partial=None):
    """The C oracle (O.c_batch, 16 threads) over EVERY segment of a device-resident fixed-stride batch too large
    to copy whole: ~1 GiB of segments at a time comes back to the host and is checked there. With `seed`, each
    chunk's first and last 4 KiB are also compared with the counter-based splitmix64 stream (the batch is the
    declared workload)."""
    per = max(1, chunk // S)
    want = np.empty(n, np.uint16)
    for i0 in range(0, n, per):
        i1 = min(n, i0 + per)
        lo, hi = i0 * S, (i1 - 1) * S + L
        h = host(t[lo:hi])
        if seed is not None:
            k = min(4096, hi - lo)
            assert np.array_equal(h[:k], O.c_splitmix64(seed, k, lo)), i0
            assert np.array_equal(h[-k:], O.c_splitmix64(seed, k, hi - k)), i0
        want[i0:i1] = O.c_batch(h, i1 - i0, stride=S, seg_len=L, threads=16,
                                partial=None if partial is None else partial[i0:i1])
        del h
    return want


def test_config4_256K_x_64KiB_full_oracle_and_roundtrip():
    """Config 4 (256K x 64 KiB = 16 GiB): every segment against the oracle (chunked D2H), then the other launch
    form and a sender/receiver round trip on every segment as extra properties."""
    n, L, seed = 1 << 18, 65536, 0x1073
    t = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    nsx.fill_splitmix64_dev(t, seed)
    got = u16(nsx.fixed_dev(t, L, L, n, out=torch.empty(n, dtype=torch.int16, device="cuda")))
    want = oracle_fixed_chunked(t, n, L, L, seed)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (bad[:8], got[bad[:8]], want[bad[:8]])
    # spot check of the chunked check itself: a few segments regenerated on the host from the seed alone
    for i in (0, 1, n // 2, n - 1):
        assert want[i] == O.c_fold_checksum(b"", O.c_splitmix64(seed, L, i * L).tobytes()), i
    # extra property (not the parity): block-per-segment mode agrees with wave mode on every segment
    out_b = nsx.fixed_dev(t, L, L, n, out=torch.empty(n, dtype=torch.int16, device="cuda"), tune=dict(block_mode=2))
    assert np.array_equal(u16(out_b), got)
    # sender/receiver round trip on every segment: the field words are zeroed before the sum
    # (tcp.go:68), ^raw goes into bytes 16-17, and every re-sum is 0xFFFF
    v = t.view(n, L)
    v[:, 16:18] = 0
    raw0 = u16(nsx.fixed_dev(t, L, L, n, out=torch.empty(n, dtype=torch.int16, device="cuda")))
    fld = torch.from_numpy(((~raw0) & 0xFFFF).astype(np.int32)).cuda()
    v[:, 16] = (fld >> 8).to(torch.uint8)
    v[:, 17] = (fld & 0xFF).to(torch.uint8)
    ok = u16(nsx.fixed_dev(t, L, L, n, out=torch.empty(n, dtype=torch.int16, device="cuda")))
    assert (ok == 0xFFFF).all()


def test_config5_16M_x_1500_per_gpu_full_oracle():
    """Config 5's per-GPU batch as bench.py times it on rank 3 (16M x 1500 B = 23.4 GiB, each segment over its
    IPv4 pseudo-header partial, SURVEY.md §8d, run as 16 back-to-back windows): every segment against the oracle
    (chunked D2H; bytes checked against the counter-based stream at every chunk edge), including both sides of
    every 8-way shard boundary and every window boundary; the one-launch and block-per-segment forms agree on
    every segment as extra properties (without partials)."""
    import bench
    n, L, seed = 1 << 24, 1500, 0x1071 + 3  # the rank-3 seed
    w = bench.build_workload(bench.WORKLOADS[5], 3, torch.device("cuda"))
    t = w["buf"]
    assert nsx.fixed_launch_count(L, L, n) == 16 == w["launches"]
    part = ipv4_pseudo_partials(host(w["addrs"]), L)
    del w["addrs"]
    w["step"]()
    got = u16(w["out"])
    want = oracle_fixed_chunked(t, n, L, L, seed, partial=part)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (bad[:8], got[bad[:8]], want[bad[:8]])
    edges = set()
    for b in list(nsx.shard_plan(n, 8)[1:-1]) + [k * (n // 16) for k in range(1, 16)]:
        edges |= {int(b) - 1, int(b)}
    for i in sorted(edges)[:8] + [n - 1]:  # the edges from the seed alone, independent of the D2H
        assert got[i] == O.fold(O.be_word_sum(O.c_splitmix64(seed, L, i * L).tobytes()) + int(part[i])), i
    plain = u16(nsx.fixed_dev(t, L, L, n, out=torch.empty(n, dtype=torch.int16, device="cuda")))
    one = u16(nsx.fixed_dev(t, L, L, n, out=torch.empty(n, dtype=torch.int16, device="cuda"),
                            tune=dict(window_bytes=-1)))
    assert np.array_equal(one, plain)
    alt = u16(nsx.fixed_dev(t, L, L, n, out=torch.empty(n, dtype=torch.int16, device="cuda"),
                            tune=dict(block_mode=2)))
    assert np.array_equal(alt, plain)
    for i in sorted(edges)[:8] + [n - 1]:
        assert plain[i] == O.c_fold_checksum(b"", O.c_splitmix64(seed, L, i * L).tobytes()), i
