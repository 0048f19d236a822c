"""TEST INFRASTRUCTURE ONLY — not part of the product.

Python/numpy restatement of the reference's Internet checksum, used to generate
and check the committed golden fixtures (tests/golden/) and as a second,
independent formulation beside oracle/csum_oracle.c. Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.

Reference (pure Go; cannot be built or run here):
  transport/tcp/tcp.go:72-95   computeChecksum — concat prefix‖segment, zero-pad an
                               odd total, 16-bit BE words, compare-carry end-around
                               add, return the RAW sum (not complemented)
  transport/tcp/tcp.go:98-128  segment.bytes — BE header, options, (buggy) padding, data
  transport/tcp/tcp.go:59-66   computeOffset
  transport/tcp/tcp.go:188-216 ctl.byte / ctlFromByte
Pinned by transport/tcp/tcp_test.go:26-32 and RFC 1071 §3 (see tests/test_oracle.py).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass, field

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libnsx_oracle.so")


# ---------------------------------------------------------------------------
# Pure-Python restatements (small inputs only)
# ---------------------------------------------------------------------------
def go_checksum(prefix: bytes, seg: bytes) -> int:
    """Literal restatement of tcp.go:72-95 (serial compare-carry loop)."""
    data = bytearray(prefix) + bytearray(seg)          # tcp.go:73
    if len(data) % 2 == 1:                              # tcp.go:74-77
        data.append(0)
    s = 0
    for idx in range(0, len(data), 2):                  # tcp.go:80-92
        v = ((data[idx] << 8) + data[idx + 1]) & 0xFFFF
        v = (v + s) & 0xFFFF
        if s > v:
            v += 1
        s = v
    return s                                            # tcp.go:94


def fold(s: int) -> int:
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s


def be_word_sum(b: bytes, pos: int = 0) -> int:
    """Integer sum of BE 16-bit words for bytes starting at stream position pos."""
    a = np.frombuffer(bytes(b), dtype=np.uint8).astype(np.uint64)
    if a.size == 0:
        return 0
    w = np.where((np.arange(a.size) + pos) % 2 == 0, a << np.uint64(8), a)
    return int(w.sum(dtype=np.uint64))


def fold_checksum(prefix: bytes, seg: bytes) -> int:
    """Wide formulation: integer BE-word sum of the virtual concatenation, folded."""
    return fold(be_word_sum(prefix, 0) + be_word_sum(seg, len(prefix)))


def field_value(raw: int) -> int:
    """What the sender stores in the checksum field (tcp_test.go:28)."""
    return (~raw) & 0xFFFF


def verify(raw: int) -> bool:
    """Receiver acceptance rule (tcp.go:70)."""
    return raw == 0xFFFF


# ---------------------------------------------------------------------------
# numpy batch forms (fixture generation, full-size spot checks)
# ---------------------------------------------------------------------------
def batch_fixed(buf: np.ndarray, stride: int, seg_len: int, n: int,
                partial: np.ndarray | None = None) -> np.ndarray:
    buf = np.asarray(buf, dtype=np.uint8)
    out = np.empty(n, dtype=np.uint16)
    if n == 0:
        return out
    idx = (np.arange(n, dtype=np.int64) * stride)[:, None] + np.arange(seg_len, dtype=np.int64)[None, :]
    seg = buf[idx].astype(np.uint64) if seg_len else np.zeros((n, 0), np.uint64)
    wts = np.where(np.arange(seg_len) % 2 == 0, 256, 1).astype(np.uint64)
    s = (seg * wts[None, :]).sum(axis=1, dtype=np.uint64)
    if partial is not None:
        s = s + np.asarray(partial, dtype=np.uint64)
    for _ in range(4):
        s = (s & np.uint64(0xFFFF)) + (s >> np.uint64(16))
    out[:] = s.astype(np.uint16)
    return out


def batch_ragged(buf: np.ndarray, offsets: np.ndarray, partial: np.ndarray | None = None) -> np.ndarray:
    buf = np.asarray(buf, dtype=np.uint8)
    offsets = np.asarray(offsets, dtype=np.uint64)
    n = offsets.size - 1
    out = np.empty(n, dtype=np.uint16)
    for i in range(n):
        lo, hi = int(offsets[i]), int(offsets[i + 1])
        s = be_word_sum(buf[lo:hi].tobytes(), 0)
        if partial is not None:
            s += int(partial[i])
        out[i] = fold(s)
    return out


def splitmix64_bytes(seed: int, byte_off: int, nbytes: int) -> np.ndarray:
    """Byte j of the stream = byte j%8 of LE word j//8, word i = splitmix64(seed, i)."""
    w0 = byte_off // 8
    w1 = (byte_off + nbytes + 7) // 8
    i = np.arange(w0, w1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (i + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    b = z.astype("<u8").view(np.uint8)
    s = byte_off - w0 * 8
    return b[s:s + nbytes].copy()


# ---------------------------------------------------------------------------
# tcp.go segment model (struct-level parity)
# ---------------------------------------------------------------------------
@dataclass
class Ctl:
    """tcp.go:188-216 — flags in order cwr, ece, urg, ack, psh, rst, syn, fin (MSB first)."""
    cwr: bool = False
    ece: bool = False
    urg: bool = False
    ack: bool = False
    psh: bool = False
    rst: bool = False
    syn: bool = False
    fin: bool = False

    def byte(self) -> int:
        flags = [self.cwr, self.ece, self.urg, self.ack, self.psh, self.rst, self.syn, self.fin]
        b = 0
        for idx, f in enumerate(flags):
            if f:
                b |= 1 << (7 - idx)
        return b

    @staticmethod
    def from_byte(b: int) -> "Ctl":
        names = ["cwr", "ece", "urg", "ack", "psh", "rst", "syn", "fin"]
        return Ctl(**{n: bool(b & (1 << (7 - i))) for i, n in enumerate(names)})


@dataclass
class Option:
    kind: int = 0
    length: int = 0
    data: bytes = b""

    def bytes(self) -> bytes:  # tcp.go:225-231
        if self.kind == 2:
            return bytes([self.kind, self.length]) + self.data
        return bytes([self.kind])


@dataclass
class Segment:
    src_port: int = 0
    dst_port: int = 0
    seq_num: int = 0
    ack_num: int = 0
    offset: int = 0
    control: Ctl = field(default_factory=Ctl)
    window: int = 0
    checksum: int = 0
    urgent_ptr: int = 0
    options: list = field(default_factory=list)
    data: bytes = b""

    def compute_offset(self) -> int:  # tcp.go:59-66
        off = 20 + sum(len(o.bytes()) for o in self.options)
        return (off + 3) // 4

    def bytes(self) -> bytes:  # tcp.go:98-128
        b = bytearray()
        b += self.src_port.to_bytes(2, "big") + self.dst_port.to_bytes(2, "big")
        b += self.seq_num.to_bytes(4, "big") + self.ack_num.to_bytes(4, "big")
        b += bytes([self.offset & 0xFF, self.control.byte()])
        b += self.window.to_bytes(2, "big")
        b += self.checksum.to_bytes(2, "big") + self.urgent_ptr.to_bytes(2, "big")
        if self.options:
            for o in self.options:
                b += o.bytes()
            rem = len(b) % 4
            if rem > 0:
                b += bytes(rem)  # reference pads `remainder`, not 4-remainder (tcp.go:118-121)
        b += self.data
        return bytes(b)

    def compute_checksum(self, pseudo: bytes = b"") -> int:  # tcp.go:72-95
        return go_checksum(pseudo, self.bytes())


PARSE_OK, PARSE_SHORT, PARSE_OFFSET, PARSE_OPTION_RANGE, PARSE_OPTION_KIND = 0, 1, 2, 3, 4


def parse_segment(raw: bytes):
    """parseSegment (tcp.go:130-185), statement by statement: (Segment, status). On a reference error the
    segment is Segment() (Go's segment{}) with status SHORT (:131-133) or OFFSET (:152-154). Where the reference's
    MSS slice runs past the segment (:173-174: the length byte past the end panics; a data slice past len(raw)
    panics, or reads the caller's bytes beyond the segment when the slice has spare capacity, which the bytes
    alone cannot tell) or it would loop forever on another option kind (:160-179, optIdx never advances) the
    status is OPTION_RANGE / OPTION_KIND and the segment is Segment()."""
    raw = bytes(raw)
    if len(raw) < 20:
        return Segment(), PARSE_SHORT
    s = Segment(src_port=int.from_bytes(raw[0:2], "big"), dst_port=int.from_bytes(raw[2:4], "big"),
                seq_num=int.from_bytes(raw[4:8], "big"), ack_num=int.from_bytes(raw[8:12], "big"),
                offset=raw[12], control=Ctl.from_byte(raw[13]), window=int.from_bytes(raw[14:16], "big"),
                checksum=int.from_bytes(raw[16:18], "big"), urgent_ptr=int.from_bytes(raw[18:20], "big"))
    data_at = s.offset * 4
    if data_at > len(raw):
        return Segment(), PARSE_OFFSET
    if s.offset > 20 // 4:
        idx = 20
        while idx < data_at:
            kind = raw[idx]
            if kind == 0:  # EOL: the rest is padding
                break
            opt = Option(kind=kind)
            if kind == 1:
                idx += 1
            elif kind == 2:
                if idx + 2 > len(raw) or idx + 2 + raw[idx + 1] > len(raw):
                    return Segment(), PARSE_OPTION_RANGE
                opt.length = raw[idx + 1]
                opt.data = raw[idx + 2:idx + 2 + opt.length]
                idx += 6  # 1(kind) + 1(length) + 4(data)
            else:
                return Segment(), PARSE_OPTION_KIND
            s.options.append(opt)
    s.data = raw[data_at:]
    return s, PARSE_OK


def ipv4_pseudo_header(src: bytes, dst: bytes, proto: int, length: int) -> bytes:
    """RFC 9293 §3.1 IPv4 pseudo-header: src(4) dst(4) zero(1) proto(1) len(2).
    Inputs as ip.Addr.Raw() (ipv4.go:15) and ip.NextProtoTCP = 6 (protocols.go:8)."""
    return bytes(src) + bytes(dst) + bytes([0, proto & 0xFF]) + (length & 0xFFFF).to_bytes(2, "big")


def ipv6_pseudo_header(src: bytes, dst: bytes, next_header: int, length: int) -> bytes:
    """RFC 8200 §8.1 IPv6 pseudo-header: src(16) dst(16) len(4) zero(3) nh(1)."""
    return bytes(src) + bytes(dst) + (length & 0xFFFFFFFF).to_bytes(4, "big") + bytes(3) + bytes([next_header & 0xFF])


def rx_ipv4_tcp(frame: bytes) -> tuple:
    """One received frame through the fused receive check (nsx_rx_ipv4_tcp_verify_dev), pure Python:
    (ip_raw, tcp_raw, valid). Every sum is go_checksum (tcp.go:72-95); the pseudo-header is built from the
    frame's own addresses (ipv4.go:15 Raw) and ip.NextProtoTCP = 6 (protocols.go:8); a segment is at least
    minSegmentLength = 20 bytes (tcp.go:131); the receiver accepts iff the sum is 0xFFFF (tcp.go:70)."""
    f = bytes(frame)
    if len(f) < 20:
        return 0, 0, False
    ihl = f[0] & 15
    hlen = ihl * 4
    if ihl < 5 or hlen > len(f):
        return 0, 0, False
    ipr = go_checksum(b"", f[:hlen])
    total = int.from_bytes(f[2:4], "big")
    frag = int.from_bytes(f[6:8], "big") & 0x3FFF
    if f[0] >> 4 != 4 or total != len(f) or frag or f[9] != 6 or total - hlen < 20:
        return ipr, 0, False
    tcpr = go_checksum(ipv4_pseudo_header(f[12:16], f[16:20], 6, total - hlen), f[hlen:total])
    return ipr, tcpr, ipr == 0xFFFF and tcpr == 0xFFFF


def ipv4_tcp_frame(seg: bytes, src: bytes, dst: bytes, ident: int = 0, ttl: int = 64, options: bytes = b"",
                   fix_tcp: bool = True) -> bytes:
    """An IPv4 datagram carrying the TCP segment `seg` (RFC 791 header, IHL = 5 + len(options)/4, DF set,
    protocol 6), with a valid header checksum and — when fix_tcp — the segment's checksum field (bytes 16-17)
    set to ^computeChecksum(pseudo) over the segment with the field zeroed (tcp.go:68-71, :110)."""
    assert len(options) % 4 == 0 and len(options) <= 40
    seg = bytearray(seg)
    if fix_tcp and len(seg) >= 18:
        seg[16:18] = b"\0\0"
        raw = go_checksum(ipv4_pseudo_header(src, dst, 6, len(seg)), bytes(seg))
        seg[16:18] = field_value(raw).to_bytes(2, "big")
    hlen = 20 + len(options)
    h = bytearray([0x40 | (hlen // 4), 0]) + (hlen + len(seg)).to_bytes(2, "big") + ident.to_bytes(2, "big") + \
        b"\x40\x00" + bytes([ttl, 6]) + b"\0\0" + bytes(src) + bytes(dst) + bytes(options)
    h[10:12] = field_value(go_checksum(b"", bytes(h))).to_bytes(2, "big")
    return bytes(h) + bytes(seg)


def rx_ipv6_tcp(frame: bytes) -> tuple:
    """One received IPv6 packet through nsx_rx_ipv6_tcp_verify_dev's checks, pure Python: (tcp_raw, valid).
    RFC 8200 §3 fixed header, Next Header 6 directly (no extension headers walked); the pseudo-header (RFC 8200
    §8.1) from the packet's own addresses (ipv6.go:16 Raw) and ip.NextProtoTCP = 6 (protocols.go:8); a segment
    is at least 20 bytes (tcp.go:131); the receiver accepts iff the sum is 0xFFFF (tcp.go:70)."""
    f = bytes(frame)
    if len(f) < 40:
        return 0, False
    plen = int.from_bytes(f[4:6], "big")
    if f[0] >> 4 != 6 or 40 + plen != len(f) or f[6] != 6 or plen < 20:
        return 0, False
    tcpr = go_checksum(ipv6_pseudo_header(f[8:24], f[24:40], 6, plen), f[40:])
    return tcpr, tcpr == 0xFFFF


def ipv6_tcp_frame(seg: bytes, src: bytes, dst: bytes, hop: int = 64, flow: int = 0, tclass: int = 0,
                   fix_tcp: bool = True) -> bytes:
    """An IPv6 packet carrying the TCP segment `seg` (RFC 8200 §3 header, Next Header 6), with — when fix_tcp —
    the segment's checksum field (bytes 16-17) set to ^computeChecksum(pseudo) over the segment with the field
    zeroed (tcp.go:68-71, :110)."""
    assert len(src) == 16 and len(dst) == 16 and len(seg) < 1 << 16
    seg = bytearray(seg)
    if fix_tcp and len(seg) >= 18:
        seg[16:18] = b"\0\0"
        raw = go_checksum(ipv6_pseudo_header(src, dst, 6, len(seg)), bytes(seg))
        seg[16:18] = field_value(raw).to_bytes(2, "big")
    h = ((6 << 28) | ((tclass & 0xFF) << 20) | (flow & 0xFFFFF)).to_bytes(4, "big") + len(seg).to_bytes(2, "big") + \
        bytes([6, hop & 0xFF]) + bytes(src) + bytes(dst)
    return h + bytes(seg)


# ---------------------------------------------------------------------------
# C restatement (oracle/csum_oracle.c) via ctypes
# ---------------------------------------------------------------------------
def build_c_oracle(force: bool = False) -> str:
    src = os.path.join(HERE, "csum_oracle.c")
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


_c = None


def c_oracle():
    global _c
    if _c is None:
        if not os.path.exists(LIB_PATH):
            build_c_oracle()
        lib = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.c_void_p
        lib.oracle_go_checksum.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t]
        lib.oracle_go_checksum.restype = ctypes.c_uint32
        lib.oracle_fold_checksum.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t]
        lib.oracle_fold_checksum.restype = ctypes.c_uint32
        lib.oracle_batch_fixed.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, u8p, u8p]
        lib.oracle_batch_ragged.argtypes = [u8p, u8p, ctypes.c_uint64, u8p, u8p]
        lib.oracle_batch_mt.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint32, u8p, ctypes.c_uint64,
                                        u8p, u8p, ctypes.c_int]
        lib.oracle_go_batch_fixed.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                              u8p, ctypes.c_size_t, u8p]
        lib.oracle_go_batch_fixed_pseudo.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                                     u8p, ctypes.c_size_t, u8p]
        lib.oracle_go_batch_ragged.argtypes = [u8p, u8p, ctypes.c_uint64, u8p, ctypes.c_size_t, u8p]
        lib.oracle_go_rx_ipv4_tcp.argtypes = [u8p, u8p, ctypes.c_uint64, u8p, u8p, u8p]
        lib.oracle_go_rx_ipv6_tcp.argtypes = [u8p, u8p, ctypes.c_uint64, u8p, u8p]
        lib.oracle_splitmix64_fill.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
        lib.oracle_go_tcp_build_batch.argtypes = [u8p] * 10 + [u8p, ctypes.c_size_t, ctypes.c_uint64, u8p, u8p, u8p]
        lib.oracle_go_tcp_build_batch.restype = ctypes.c_int
        lib.oracle_go_tcp_build_batch_opts.argtypes = ([u8p] * 12 + [u8p, ctypes.c_size_t, ctypes.c_uint64, u8p, u8p,
                                                                    u8p])
        lib.oracle_go_tcp_build_batch_opts.restype = ctypes.c_int
        _c = lib
    return _c


_fast = None
FAST_PATH = os.path.join(os.path.dirname(LIB_PATH), "libnsx_cpu_fast.so")


def c_fast():
    """Vectorised multi-threaded CPU checksum (oracle/csum_cpu_fast.c): the
    best-CPU reference line for bench.py, not a checker."""
    global _fast
    if _fast is None:
        if not os.path.exists(FAST_PATH):
            build_c_oracle(force=True)
        lib = ctypes.CDLL(FAST_PATH)
        lib.cpu_fast_batch_fixed.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        lib.cpu_fast_batch_fixed.restype = None
        _fast = lib
    return _fast


def _ptr(a):
    if a is None:
        return None
    return a.ctypes.data_as(ctypes.c_void_p)


TCP_FIELDS = ("src_port", "dst_port", "seq_num", "ack_num", "offset", "control", "window", "urgent_ptr")
TCP_FIELD_DTYPES = (np.uint16, np.uint16, np.uint32, np.uint32, np.uint8, np.uint8, np.uint16, np.uint16)


def c_go_tcp_build(fields: dict, data: np.ndarray, data_off: np.ndarray, out_off: np.ndarray,
                   pseudo: np.ndarray | None = None):
    """Go-faithful sender loop (oracle_go_tcp_build_batch): option-less segments
    serialised (tcp.go:98-128), checksummed over pseudo_i ‖ bytes (tcp.go:72-95),
    ^sum stored at 16-17. pseudo: (n, k) uint8 or None. Returns (wire, raw)."""
    n = data_off.size - 1
    cols = [np.ascontiguousarray(fields[k], dt) for k, dt in zip(TCP_FIELDS, TCP_FIELD_DTYPES)]
    data = np.ascontiguousarray(data, np.uint8)
    data_off = np.ascontiguousarray(data_off, np.uint64)
    out_off = np.ascontiguousarray(out_off, np.uint64)
    out = np.zeros(int(out_off[-1]), np.uint8)
    raw = np.empty(n, np.uint16)
    pl = 0 if pseudo is None else pseudo.shape[1]
    ps = None if pseudo is None else np.ascontiguousarray(pseudo, np.uint8)
    rc = c_oracle().oracle_go_tcp_build_batch(*[_ptr(c) for c in cols], _ptr(data), _ptr(data_off), _ptr(ps), pl, n,
                                              _ptr(out), _ptr(out_off), _ptr(raw))
    assert rc == 0
    return out, raw


def c_go_tcp_build_opts(fields: dict, opts: np.ndarray, opt_off: np.ndarray, data: np.ndarray,
                        data_off: np.ndarray, out_off: np.ndarray, pseudo: np.ndarray | None = None):
    """c_go_tcp_build for segments with options given as their serialisation
    (oracle_go_tcp_build_batch_opts). Returns (wire, raw)."""
    n = data_off.size - 1
    cols = [np.ascontiguousarray(fields[k], dt) for k, dt in zip(TCP_FIELDS, TCP_FIELD_DTYPES)]
    opts = np.ascontiguousarray(opts, np.uint8) if len(opts) else np.zeros(1, np.uint8)
    opt_off = np.ascontiguousarray(opt_off, np.uint64)
    data = np.ascontiguousarray(data, np.uint8)
    data_off = np.ascontiguousarray(data_off, np.uint64)
    out_off = np.ascontiguousarray(out_off, np.uint64)
    out = np.zeros(int(out_off[-1]), np.uint8)
    raw = np.empty(n, np.uint16)
    pl = 0 if pseudo is None else pseudo.shape[1]
    ps = None if pseudo is None else np.ascontiguousarray(pseudo, np.uint8)
    rc = c_oracle().oracle_go_tcp_build_batch_opts(*[_ptr(c) for c in cols], _ptr(opts), _ptr(opt_off), _ptr(data),
                                                   _ptr(data_off), _ptr(ps), pl, n, _ptr(out), _ptr(out_off),
                                                   _ptr(raw))
    assert rc == 0
    return out, raw


def c_go_tcp_build_mt(fields: dict, data: np.ndarray, data_off: np.ndarray, out_off: np.ndarray,
                      pseudo: np.ndarray | None = None, opts: np.ndarray | None = None,
                      opt_off: np.ndarray | None = None, threads: int = 16):
    """c_go_tcp_build (opts None) or c_go_tcp_build_opts over contiguous index shards, one thread each (ctypes
    releases the GIL), so that every segment of a full-size batch goes through the Go-faithful sender loop
    (tcp.go:98-128, :72-95, :68-71) in seconds. Offsets are absolute into `data` / `opts` / the returned wire
    buffer, as in the single-threaded forms. Returns (wire, raw)."""
    from concurrent.futures import ThreadPoolExecutor
    n = data_off.size - 1
    cols = [np.ascontiguousarray(fields[k], dt) for k, dt in zip(TCP_FIELDS, TCP_FIELD_DTYPES)]
    data = np.ascontiguousarray(data, np.uint8)
    data_off = np.ascontiguousarray(data_off, np.uint64)
    out_off = np.ascontiguousarray(out_off, np.uint64)
    out = np.zeros(int(out_off[-1]), np.uint8)
    raw = np.empty(n, np.uint16)
    pl = 0 if pseudo is None else pseudo.shape[1]
    ps = None if pseudo is None else np.ascontiguousarray(pseudo, np.uint8)
    if opts is not None:
        opts = np.ascontiguousarray(opts, np.uint8) if len(opts) else np.zeros(1, np.uint8)
        opt_off = np.ascontiguousarray(opt_off, np.uint64)
    lib = c_oracle()

    def at(a, i, k=1):  # pointer to element i (row i of a k-byte-per-row array)
        return None if a is None else ctypes.c_void_p(a.ctypes.data + i * a.itemsize * k)

    def run(lo, hi):
        head = [at(c, lo) for c in cols]
        if opts is None:
            return lib.oracle_go_tcp_build_batch(*head, _ptr(data), at(data_off, lo), at(ps, lo, pl), pl, hi - lo,
                                                 _ptr(out), at(out_off, lo), at(raw, lo))
        return lib.oracle_go_tcp_build_batch_opts(*head, _ptr(opts), at(opt_off, lo), _ptr(data), at(data_off, lo),
                                                  at(ps, lo, pl), pl, hi - lo, _ptr(out), at(out_off, lo),
                                                  at(raw, lo))
    T = max(1, min(threads, n))
    b = [n * t // T for t in range(T + 1)]
    with ThreadPoolExecutor(T) as ex:
        rcs = list(ex.map(lambda t: run(b[t], b[t + 1]), range(T)))
    assert all(rc == 0 for rc in rcs), rcs
    return out, raw


def c_go_checksum(prefix: bytes, seg: bytes) -> int:
    p = np.frombuffer(bytes(prefix), np.uint8) if prefix else None
    s = np.frombuffer(bytes(seg), np.uint8) if seg else None
    return c_oracle().oracle_go_checksum(_ptr(p), len(prefix), _ptr(s), len(seg))


def c_fold_checksum(prefix: bytes, seg: bytes) -> int:
    p = np.frombuffer(bytes(prefix), np.uint8) if prefix else None
    s = np.frombuffer(bytes(seg), np.uint8) if seg else None
    return c_oracle().oracle_fold_checksum(_ptr(p), len(prefix), _ptr(s), len(seg))


def c_batch(buf: np.ndarray, n: int, stride: int = 0, seg_len: int = 0, offsets: np.ndarray | None = None,
            partial: np.ndarray | None = None, threads: int = 8) -> np.ndarray:
    """Multi-threaded C oracle over a fixed-stride (offsets None) or ragged batch."""
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    out = np.empty(n, dtype=np.uint16)
    if offsets is not None:
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    if partial is not None:
        partial = np.ascontiguousarray(partial, dtype=np.uint32)
    c_oracle().oracle_batch_mt(_ptr(buf), stride, seg_len, _ptr(offsets), n, _ptr(partial), _ptr(out), threads)
    return out


def c_rx_ipv4_tcp(buf: np.ndarray, offsets: np.ndarray):
    """oracle_go_rx_ipv4_tcp over a packed frame batch: (mask u64[ceil(n/64)], ip_raw u16[n], tcp_raw u16[n])."""
    buf = np.ascontiguousarray(buf, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    n = offsets.size - 1
    mask = np.zeros((n + 63) // 64, np.uint64)
    ipr, tcpr = np.empty(n, np.uint16), np.empty(n, np.uint16)
    c_oracle().oracle_go_rx_ipv4_tcp(_ptr(buf if buf.size else np.zeros(1, np.uint8)), _ptr(offsets), n, _ptr(mask),
                                     _ptr(ipr), _ptr(tcpr))
    return mask, ipr, tcpr


def c_rx_ipv6_tcp(buf: np.ndarray, offsets: np.ndarray):
    """oracle_go_rx_ipv6_tcp over a packed packet batch: (mask u64[ceil(n/64)], tcp_raw u16[n])."""
    buf = np.ascontiguousarray(buf, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    n = offsets.size - 1
    mask = np.zeros((n + 63) // 64, np.uint64)
    tcpr = np.empty(n, np.uint16)
    c_oracle().oracle_go_rx_ipv6_tcp(_ptr(buf if buf.size else np.zeros(1, np.uint8)), _ptr(offsets), n, _ptr(mask),
                                     _ptr(tcpr))
    return mask, tcpr


def c_splitmix64(seed: int, nbytes: int, byte_off: int = 0) -> np.ndarray:
    out = np.empty(nbytes, dtype=np.uint8)
    c_oracle().oracle_splitmix64_fill(_ptr(out), byte_off, nbytes, seed)
    return out
