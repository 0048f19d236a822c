"""TCP segments for the receive-side parse (nsx_tcp_parse_dev, parseSegment tcp.go:130-185): valid segments
with and without options, and every case the reference rejects or cannot handle. Shared by the CPU oracle tests,
the golden fixture generator and the GPU parity tests."""
import numpy as np

from oracle import csum_oracle as O

KINDS = ("plain", "nop_mss", "mss_eol", "nops", "eol_first", "header_only", "offset_zero", "offset_small",
         "short", "empty", "offset_long", "mss_range", "unknown_kind", "mss_odd_len", "padding_bug")


def _seg(rng, options, payload: int, offset=None) -> O.Segment:
    s = O.Segment(src_port=int(rng.integers(1 << 16)), dst_port=int(rng.integers(1 << 16)),
                  seq_num=int(rng.integers(1 << 32)), ack_num=int(rng.integers(1 << 32)),
                  control=O.Ctl.from_byte(int(rng.integers(256))), window=int(rng.integers(1 << 16)),
                  checksum=int(rng.integers(1 << 16)), urgent_ptr=int(rng.integers(1 << 16)), options=options,
                  data=rng.integers(0, 256, payload, dtype=np.uint8).tobytes())
    s.offset = s.compute_offset() if offset is None else offset
    return s


def segment(rng, kind: str, max_payload: int = 1460) -> bytes:
    """One segment's bytes (serialised by Segment.bytes(), tcp.go:98-128, then bent for the broken kinds)."""
    payload = int(rng.integers(0, max_payload + 1))
    mss = lambda: O.Option(kind=2, length=4, data=rng.integers(0, 256, 4, dtype=np.uint8).tobytes())
    if kind == "plain":
        return _seg(rng, [], payload).bytes()
    if kind == "nop_mss":
        return _seg(rng, [O.Option(kind=1), O.Option(kind=1), mss()], payload).bytes()
    if kind == "mss_eol":  # MSS then EOL: the walk stops at the EOL
        return _seg(rng, [mss(), O.Option(kind=0), O.Option(kind=0)], payload).bytes()
    if kind == "nops":
        return _seg(rng, [O.Option(kind=1)] * int(rng.integers(1, 13)), payload).bytes()
    if kind == "eol_first":
        return _seg(rng, [O.Option(kind=0), O.Option(kind=1), O.Option(kind=1), O.Option(kind=1)], payload).bytes()
    if kind == "header_only":
        return _seg(rng, [], 0).bytes()
    if kind == "offset_zero":  # tcp_test.go:27 builds this one: dataAt 0, the data is the whole segment
        return _seg(rng, [], payload, offset=0).bytes()
    if kind == "offset_small":
        return _seg(rng, [], payload, offset=int(rng.integers(1, 5))).bytes()
    if kind == "short":
        return rng.integers(0, 256, int(rng.integers(1, 20)), dtype=np.uint8).tobytes()
    if kind == "empty":
        return b""
    if kind == "offset_long":  # offset*4 past the end
        b = bytearray(_seg(rng, [], int(rng.integers(0, 40))).bytes())
        b[12] = int(rng.integers((len(b) + 3) // 4 + 1, 256))
        return bytes(b)
    if kind == "mss_range":  # an MSS option whose length runs past the segment
        b = bytearray(_seg(rng, [O.Option(kind=1), O.Option(kind=1), mss()], 0).bytes())
        b[23] = int(rng.integers(len(b) - 23, 256))
        return bytes(b)
    if kind == "unknown_kind":
        b = bytearray(_seg(rng, [O.Option(kind=1)] * 4, payload).bytes())
        b[20 + int(rng.integers(0, 4))] = int(rng.integers(3, 256))
        return bytes(b)
    if kind == "mss_odd_len":  # a kind-2 option of length 2 (RFC style): the walk still advances 6 (tcp.go:175)
        return _seg(rng, [O.Option(kind=2, length=2, data=b""), O.Option(kind=1)] * 3, payload).bytes()
    if kind == "padding_bug":  # 3 option bytes: bytes() pads `remainder` = 3 zeros (tcp.go:118-121)
        return _seg(rng, [O.Option(kind=1)] * 3, payload).bytes()
    raise ValueError(kind)


def batch(rng, n: int, kinds=KINDS, weights=None, lead: int = 0, max_payload: int = 1460):
    """(buf uint8, offsets uint64[n+1], kinds): n segments packed back to back behind `lead` bytes."""
    ks = list(rng.choice(kinds, n, p=weights)) if n else []
    segs = [segment(rng, k, max_payload) for k in ks]
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum([len(s) for s in segs]) if n else []
    offs += np.uint64(lead)
    buf = np.frombuffer(rng.integers(0, 256, lead, dtype=np.uint8).tobytes() + b"".join(segs) +
                        rng.integers(0, 256, 3, dtype=np.uint8).tobytes(), np.uint8).copy()
    return buf, offs, ks


def expected(buf: np.ndarray, offs: np.ndarray) -> dict:
    """The oracle's parse of every segment as the arrays nsx_tcp_parse_dev writes."""
    n = offs.size - 1
    cols = {k: [] for k in ("src_port", "dst_port", "seq_num", "ack_num", "offset", "control", "window",
                            "checksum", "urgent_ptr", "data_off", "n_options", "status")}
    for i in range(n):
        lo, hi = int(offs[i]), int(offs[i + 1])
        s, st = O.parse_segment(buf[lo:hi].tobytes())
        for k in ("src_port", "dst_port", "seq_num", "ack_num", "offset", "window", "checksum", "urgent_ptr"):
            cols[k].append(getattr(s, k))
        cols["control"].append(s.control.byte())
        cols["data_off"].append(lo + s.offset * 4 if st == O.PARSE_OK else 0)
        cols["n_options"].append(len(s.options))
        cols["status"].append(st)
    dts = {"src_port": np.uint16, "dst_port": np.uint16, "seq_num": np.uint32, "ack_num": np.uint32,
           "offset": np.uint8, "control": np.uint8, "window": np.uint16, "checksum": np.uint16,
           "urgent_ptr": np.uint16, "data_off": np.uint64, "n_options": np.uint8, "status": np.uint8}
    return {k: np.array(v, dts[k]) for k, v in cols.items()}
