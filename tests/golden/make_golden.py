"""Generate the committed golden fixtures under tests/golden/.

The reference (Go) cannot be built or run in this container or on the GPU box
(no Go toolchain), so every expected value here comes from the
oracle restatement (oracle/csum_oracle.py, oracle/csum_oracle.c) and is written
only if the four formulations agree: pure-Python serial loop (tcp.go:80-92
statement for statement), numpy wide fold, C serial loop, C wide fold. The
restatement itself is pinned by tests/test_oracle.py against the reference's own
test (transport/tcp/tcp_test.go:26-32) and the RFC 1071 §3 example (kat.json).

Run from the repo root:  python tests/golden/make_golden.py
Outputs (small, committed): kat.json, vectors.json + vectors.bin,
ragged.json + ragged.bin, segments.json, rx.json + rx.bin (received IPv4/TCP
frames for the fused receive pass: expected bitmask and raw sums, written only if
the Python and C restatements of the receive check agree).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import csum_oracle as O  # noqa: E402


def agreed(prefix: bytes, seg: bytes, serial: bool = True) -> int:
    vals = {O.fold_checksum(prefix, seg), O.c_go_checksum(prefix, seg), O.c_fold_checksum(prefix, seg)}
    if serial:
        vals.add(O.go_checksum(prefix, seg))
    assert len(vals) == 1, (prefix.hex(), len(seg), vals)
    return vals.pop()


def kat() -> list:
    """Known answers. Sources: tcp_test.go:26-32 (hello), RFC 1071 §3 (example
    words 0001 f203 f4f5 f6f7 → sum ddf2), and the 0/0xFFFF edge rules."""
    cases = [
        ("tcp_test_hello_segment", "", (bytes(20) + b"hello").hex(), 0x43D2,
         "transport/tcp/tcp_test.go:27: segment{data:\"hello\"}.bytes(): 20 zero header bytes + hello"),
        ("rfc1071_sec3_example", "", "0001f203f4f5f6f7", 0xDDF2, "RFC 1071 §3 numerical example"),
        ("all_ones_word", "", "ffff", 0xFFFF, "single 0xFFFF word"),
        ("nonzero_multiple_of_ffff", "", "0001fffe", 0xFFFF, "nonzero input ≡ 0 mod 0xFFFF → 0xFFFF, never 0"),
        ("empty", "", "", 0x0000, "no words → 0"),
        ("all_zero_odd", "", "00" * 7, 0x0000, "all-zero → 0 (only case giving 0)"),
        ("single_byte", "", "ab", 0xAB00, "odd length: pad 0x00 after (tcp.go:74-77)"),
        ("carry_wrap", "", "ffff0001", 0x0001, "0xFFFF + 1 → end-around carry → 1"),
        ("prefix_odd_shifts_pairing", "aa", "bbcc", 0xAABB + 0xCC00 - 0xFFFF, "odd prefix: segment pairs shift"),
        ("hello_with_ipv4_pseudo", O.ipv4_pseudo_header(bytes([10, 0, 0, 1]), bytes([10, 0, 0, 2]), 6, 25).hex(),
         (bytes(20) + b"hello").hex(), None, "IPv4 pseudo-header (RFC 9293 §3.1) + hello segment"),
        ("ipv4_header_valid", "", "45000073000040004011b861c0a80001c0a800c7", 0xFFFF,
         "IPv4 header with its checksum field b861 (RFC 791 §3.1; widely published example): re-sum 0xFFFF"),
        ("ipv4_header_field_zeroed", "", "450000730000400040110000c0a80001c0a800c7", 0x479E,
         "same header, field zeroed: raw 0x479e, field = ~raw = 0xb861"),
    ]
    out = []
    for name, p, s, expect, src in cases:
        prefix, seg = bytes.fromhex(p), bytes.fromhex(s)
        got = agreed(prefix, seg)
        if expect is not None:
            assert got == expect, (name, hex(got), hex(expect))
        out.append({"name": name, "prefix": p, "segment": s, "raw": got, "field": O.field_value(got),
                    "source": src})
    return out


def vectors(rng: np.random.Generator):
    """Seeded random segments at the SURVEY.md §8c lengths, every start
    misalignment 0-7, with no prefix / an IPv4 / an IPv6 pseudo-header."""
    lengths = [0, 1, 2, 3, 63, 64, 65, 1499, 1500, 1501, 9000, 65536]
    blob = bytearray()
    index = []
    for L in lengths:
        for mis in range(8):
            if L >= 9000 and mis not in (0, 1, 3):
                continue
            kind = ["none", "ipv4", "ipv6"][(L + mis) % 3]
            data = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
            if mis == 5 and L > 4:   # an all-0xFF and an all-0x00 variant
                data = b"\xff" * L
            if mis == 6 and L > 4:
                data = bytes(L)
            if kind == "ipv4":
                prefix = O.ipv4_pseudo_header(rng.integers(0, 256, 4, dtype=np.uint8).tobytes(),
                                              rng.integers(0, 256, 4, dtype=np.uint8).tobytes(), 6, L)
            elif kind == "ipv6":
                prefix = O.ipv6_pseudo_header(rng.integers(0, 256, 16, dtype=np.uint8).tobytes(),
                                              rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), 6, L)
            else:
                prefix = b""
            # place so that (offset % 8) == mis inside the blob
            while len(blob) % 8 != mis:
                blob.append(0x5A)
            off = len(blob)
            blob += data
            raw = agreed(prefix, data, serial=L <= 9000)
            raw_noprefix = agreed(b"", data, serial=L <= 9000)
            index.append({"offset": off, "length": L, "misalign": mis, "prefix": prefix.hex(),
                          "prefix_kind": kind, "raw": raw, "raw_no_prefix": raw_noprefix,
                          "prefix_partial": O.be_word_sum(prefix)})
    return bytes(blob), index


def ragged(rng: np.random.Generator):
    """A densely packed ragged batch (odd starts, zero-length segments, one
    long segment) with expected raw sums with and without prefix partials."""
    lens = rng.integers(0, 300, 400).astype(np.uint64)
    lens[[5, 17, 99]] = 0
    lens[200] = 5000
    offs = np.zeros(lens.size + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    offs += np.uint64(3)  # the batch itself starts at an odd offset of the blob
    blob = rng.integers(0, 256, int(offs[-1]) + 5, dtype=np.uint8)
    partial = rng.integers(0, 1 << 20, lens.size, dtype=np.uint32)
    raw = [agreed(b"", blob[int(offs[i]):int(offs[i + 1])].tobytes()) for i in range(lens.size)]
    raw_p = [int(O.fold(int(partial[i]) + O.be_word_sum(blob[int(offs[i]):int(offs[i + 1])].tobytes())))
             for i in range(lens.size)]
    # cross-check with the C batch oracle
    c = O.c_batch(blob, lens.size, offsets=offs)
    cp = O.c_batch(blob, lens.size, offsets=offs, partial=partial)
    assert c.tolist() == raw and cp.tolist() == raw_p
    return blob.tobytes(), {"offsets": [int(x) for x in offs], "partial": [int(x) for x in partial],
                            "raw": raw, "raw_with_partial": raw_p}


def segment_cases() -> list:
    """(name, O.Segment) for the struct-level cases: the exact segments of transport/tcp/tcp_test.go plus
    option-bearing ones exercising the reference's padding (tcp.go:118-121), offset set as each test sets it
    (also used by tests/test_gpu_00_baseline.py to drive the device build + parse)."""
    cases = [
        ("TestSegmentComputeChecksum", O.Segment(data=b"hello")),
        ("TestSegmentCodec", O.Segment(src_port=1, dst_port=2, seq_num=3, ack_num=4, offset=5, window=6,
                                       checksum=7, urgent_ptr=8, data=bytes([9]))),
        ("ctl_urg_rst", O.Segment(src_port=80, dst_port=443, control=O.Ctl(urg=True, rst=True), data=b"x" * 11)),
        ("option_noop", O.Segment(src_port=1, options=[O.Option(kind=1)], data=b"abc")),
        ("option_mss", O.Segment(src_port=1234, dst_port=80, seq_num=0xDEADBEEF, ack_num=0x01020304,
                                 control=O.Ctl(syn=True, ack=True), window=65535,
                                 options=[O.Option(kind=2, length=4, data=bytes([0x05, 0xB4, 0, 0]))],
                                 data=b"payload!")),
        ("options_mss_noop_eol", O.Segment(src_port=7, options=[O.Option(kind=2, length=4, data=bytes([1, 2, 3, 4])),
                                                                O.Option(kind=1), O.Option(kind=0)],
                                           data=bytes(range(37)))),
    ]
    for name, s in cases:
        # tcp_test.go:27 never sets offset (it stays 0, so byte 12 is 0x00); tcp_test.go:47 and every other
        # case set it with computeOffset (tcp.go:59-66)
        if name != "TestSegmentComputeChecksum":
            s.offset = s.compute_offset()
    return cases


def segments() -> list:
    out = []
    for name, s in segment_cases():
        b = s.bytes()
        pseudo = O.ipv4_pseudo_header(bytes([192, 168, 0, 1]), bytes([192, 168, 0, 2]), 6, len(b))
        raw = agreed(b"", b)
        raw_p = agreed(pseudo, b)
        out.append({"name": name, "offset": s.offset, "control": s.control.byte(), "bytes": b.hex(),
                    "raw": raw, "pseudo_ipv4": pseudo.hex(), "raw_with_pseudo": raw_p})
    return out


def rx(rng):
    """Received IPv4/TCP frames of every kind tests/_rx.py builds (valid, broken sums, malformed, fragments,
    non-TCP, short), plus the RFC 791 example header as a frame of its own (a UDP datagram: header valid,
    not TCP), packed behind an odd lead. Expected per-frame (ip_raw, tcp_raw, valid) from O.rx_ipv4_tcp,
    checked against the C restatement."""
    sys.path.insert(0, os.path.join(os.path.dirname(HERE)))
    import _rx
    frames = []
    for k in _rx.KINDS:
        frames += [_rx.frame(rng, k, max_payload=300) for _ in range(12)]
    rfc = bytes.fromhex("450000730000400040110000c0a80001c0a800c7")
    rfc = rfc[:10] + O.field_value(O.go_checksum(b"", rfc)).to_bytes(2, "big") + rfc[12:]
    frames.append(rfc + bytes(0x73 - 20))  # RFC 791-style header; total length 0x73 = the frame
    order = rng.permutation(len(frames))
    frames = [frames[i] for i in order]
    lead = 3
    offs = np.zeros(len(frames) + 1, np.uint64)
    offs[1:] = np.cumsum([len(f) for f in frames])
    offs += np.uint64(lead)
    blob = bytes(range(lead)) + b"".join(frames)
    res = [O.rx_ipv4_tcp(f) for f in frames]
    mask, ipr, tcpr = O.c_rx_ipv4_tcp(np.frombuffer(blob, np.uint8), offs)
    valid = np.array([v for _, _, v in res])
    pad = np.zeros((len(frames) + 63) // 64 * 64, np.uint8)
    pad[:len(frames)] = valid
    assert np.array_equal(mask, np.packbits(pad, bitorder="little").view(np.uint64))
    assert ipr.tolist() == [a for a, _, _ in res] and tcpr.tolist() == [b for _, b, _ in res]
    return blob, {"offsets": [int(x) for x in offs], "ip_raw": ipr.tolist(), "tcp_raw": tcpr.tolist(),
                  "valid": [bool(v) for v in valid], "mask": [int(x) for x in mask]}


def rx6(rng):
    """Received IPv6/TCP packets of every kind tests/_rx.py builds (KINDS6), packed behind an odd lead.
    Expected per-packet (tcp_raw, valid) from O.rx_ipv6_tcp, checked against the C restatement."""
    sys.path.insert(0, os.path.join(os.path.dirname(HERE)))
    import _rx
    frames = []
    for k in _rx.KINDS6:
        frames += [_rx.frame6(rng, k, max_payload=300) for _ in range(12)]
    frames = [frames[i] for i in rng.permutation(len(frames))]
    lead = 5
    offs = np.zeros(len(frames) + 1, np.uint64)
    offs[1:] = np.cumsum([len(f) for f in frames])
    offs += np.uint64(lead)
    blob = bytes(range(lead)) + b"".join(frames)
    res = [O.rx_ipv6_tcp(f) for f in frames]
    mask, tcpr = O.c_rx_ipv6_tcp(np.frombuffer(blob, np.uint8), offs)
    valid = np.array([v for _, v in res])
    pad = np.zeros((len(frames) + 63) // 64 * 64, np.uint8)
    pad[:len(frames)] = valid
    assert np.array_equal(mask, np.packbits(pad, bitorder="little").view(np.uint64))
    assert tcpr.tolist() == [a for a, _ in res]
    return blob, {"offsets": [int(x) for x in offs], "tcp_raw": tcpr.tolist(), "valid": [bool(v) for v in valid],
                  "mask": [int(x) for x in mask]}


def parse(rng):
    """TCP segments of every kind tests/_parse.py builds (valid with and without options, and every case
    parseSegment rejects or cannot handle), packed behind an odd lead; expected per-segment fields, data
    offset, option count and status from O.parse_segment (tcp.go:130-185)."""
    sys.path.insert(0, os.path.join(os.path.dirname(HERE)))
    import _parse
    segs = []
    for k in _parse.KINDS:
        segs += [_parse.segment(rng, k, max_payload=200) for _ in range(8)]
    segs = [segs[i] for i in rng.permutation(len(segs))]
    lead = 7
    offs = np.zeros(len(segs) + 1, np.uint64)
    offs[1:] = np.cumsum([len(s) for s in segs])
    offs += np.uint64(lead)
    blob = bytes(range(lead)) + b"".join(segs)
    exp = _parse.expected(np.frombuffer(blob, np.uint8), offs)
    meta = {"offsets": [int(x) for x in offs]}
    meta.update({k: [int(x) for x in v] for k, v in exp.items()})
    return blob, meta


def main():
    rng = np.random.default_rng(0x1071)
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kat(), f, indent=1)
    blob, idx = vectors(rng)
    with open(os.path.join(HERE, "vectors.bin"), "wb") as f:
        f.write(blob)
    with open(os.path.join(HERE, "vectors.json"), "w") as f:
        json.dump(idx, f, indent=0)
    rblob, rmeta = ragged(rng)
    with open(os.path.join(HERE, "ragged.bin"), "wb") as f:
        f.write(rblob)
    with open(os.path.join(HERE, "ragged.json"), "w") as f:
        json.dump(rmeta, f)
    with open(os.path.join(HERE, "segments.json"), "w") as f:
        json.dump(segments(), f, indent=1)
    xblob, xmeta = rx(np.random.default_rng(0x1078))
    with open(os.path.join(HERE, "rx.bin"), "wb") as f:
        f.write(xblob)
    with open(os.path.join(HERE, "rx.json"), "w") as f:
        json.dump(xmeta, f)
    x6blob, x6meta = rx6(np.random.default_rng(0x1079))
    with open(os.path.join(HERE, "rx6.bin"), "wb") as f:
        f.write(x6blob)
    with open(os.path.join(HERE, "rx6.json"), "w") as f:
        json.dump(x6meta, f)
    pblob, pmeta = parse(np.random.default_rng(0x107C))
    with open(os.path.join(HERE, "parse.bin"), "wb") as f:
        f.write(pblob)
    with open(os.path.join(HERE, "parse.json"), "w") as f:
        json.dump(pmeta, f)
    print(f"parse: {len(pmeta['status'])} segments, statuses {sorted(set(pmeta['status']))}")
    print(f"rx6: {len(x6meta['valid'])} packets ({sum(x6meta['valid'])} valid), {len(x6blob)} B")
    print(f"vectors: {len(idx)} cases, {len(blob)} B; ragged: {len(rmeta['raw'])} segments, {len(rblob)} B; "
          f"rx: {len(xmeta['valid'])} frames ({sum(xmeta['valid'])} valid), {len(xblob)} B")


if __name__ == "__main__":
    main()
