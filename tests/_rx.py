"""Received-frame batches for the fused receive pass (nsx_rx_ipv4_tcp_verify_dev): IPv4 datagrams carrying
TCP segments serialised by the oracle's Segment.bytes() (tcp.go:98-128), valid or broken in every way the
check distinguishes. Shared by the CPU oracle tests, the golden fixture generator and the GPU parity tests."""
import numpy as np

from oracle import csum_oracle as O

KINDS = ("valid", "valid_options", "bad_ip_sum", "bad_tcp_sum", "udp", "fragment_mf", "fragment_off",
         "total_mismatch", "ihl_lt5", "version6", "short", "tcp_lt20", "empty", "ihl_past_end", "header_only",
         "odd_payload")


def _segment(rng, payload: int) -> bytes:
    s = O.Segment(src_port=int(rng.integers(1 << 16)), dst_port=int(rng.integers(1 << 16)),
                  seq_num=int(rng.integers(1 << 32)), ack_num=int(rng.integers(1 << 32)),
                  control=O.Ctl.from_byte(int(rng.integers(256))), window=int(rng.integers(1 << 16)),
                  urgent_ptr=int(rng.integers(1 << 16)), data=rng.integers(0, 256, payload, dtype=np.uint8).tobytes())
    s.offset = s.compute_offset()
    return s.bytes()


def _refix_ip(f: bytearray) -> bytearray:
    hlen = (f[0] & 15) * 4
    f[10:12] = b"\0\0"
    f[10:12] = O.field_value(O.go_checksum(b"", bytes(f[:hlen]))).to_bytes(2, "big")
    return f


def frame(rng, kind: str, max_payload: int = 1460) -> bytes:
    src, dst = rng.integers(0, 256, 4, dtype=np.uint8).tobytes(), rng.integers(0, 256, 4, dtype=np.uint8).tobytes()
    payload = int(rng.integers(0, max_payload + 1))
    if kind == "odd_payload":
        payload |= 1
    if kind == "header_only":
        payload = 0
    opts = b""
    if kind == "valid_options":
        opts = rng.integers(0, 256, 4 * int(rng.integers(1, 11)), dtype=np.uint8).tobytes()
    if kind == "short":
        return rng.integers(0, 256, int(rng.integers(1, 20)), dtype=np.uint8).tobytes()
    if kind == "empty":
        return b""
    if kind == "tcp_lt20":
        seg = rng.integers(0, 256, int(rng.integers(0, 20)), dtype=np.uint8).tobytes()
        return O.ipv4_tcp_frame(seg, src, dst, ident=int(rng.integers(1 << 16)))
    f = bytearray(O.ipv4_tcp_frame(_segment(rng, payload), src, dst, ident=int(rng.integers(1 << 16)),
                                   ttl=int(rng.integers(1, 256)), options=opts))
    hlen = (f[0] & 15) * 4
    if kind == "bad_ip_sum":
        f[int(rng.choice([1, 4, 5, 8, 12, 19]))] ^= 1 << int(rng.integers(8))
    elif kind == "bad_tcp_sum":
        f[hlen + int(rng.integers(0, len(f) - hlen))] ^= 1 << int(rng.integers(8))
    elif kind == "udp":
        f[9] = 17
        _refix_ip(f)
    elif kind == "fragment_mf":
        f[6] |= 0x20
        _refix_ip(f)
    elif kind == "fragment_off":
        f[7] = int(rng.integers(1, 256))
        _refix_ip(f)
    elif kind == "total_mismatch":
        f += bytes([int(rng.integers(256))])  # the frame holds one byte more than its total length
    elif kind == "ihl_lt5":
        f[0] = 0x40 | int(rng.integers(0, 5))
    elif kind == "version6":
        f[0] = 0x60 | (f[0] & 15)
        _refix_ip(f)
    elif kind == "ihl_past_end":
        f = bytearray(f[:int(rng.integers(20, 60))])
        f[0] = 0x4F
    return bytes(f)


KINDS6 = ("valid", "bad_tcp_sum", "bad_addr", "udp", "ext_header", "len_short", "len_long", "version4", "short",
          "tcp_lt20", "empty", "header_only", "odd_payload", "jumbo")
VALID6 = ("valid", "header_only", "odd_payload")


def frame6(rng, kind: str, max_payload: int = 1440) -> bytes:
    """An IPv6 packet (RFC 8200 §3) carrying a TCP segment serialised by Segment.bytes(), valid or broken in
    every way nsx_rx_ipv6_tcp_verify_dev distinguishes."""
    src, dst = rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
    payload = int(rng.integers(0, max_payload + 1))
    if kind == "odd_payload":
        payload |= 1
    if kind == "header_only":
        payload = 0
    if kind == "short":
        return rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8).tobytes()
    if kind == "empty":
        return b""
    if kind == "tcp_lt20":
        seg = rng.integers(0, 256, int(rng.integers(0, 20)), dtype=np.uint8).tobytes()
        return O.ipv6_tcp_frame(seg, src, dst)
    f = bytearray(O.ipv6_tcp_frame(_segment(rng, payload), src, dst, hop=int(rng.integers(256)),
                                   flow=int(rng.integers(1 << 20)), tclass=int(rng.integers(256))))
    if kind == "bad_tcp_sum":
        f[40 + int(rng.integers(0, len(f) - 40))] ^= 1 << int(rng.integers(8))
    elif kind == "bad_addr":  # a flipped address bit breaks the pseudo-header sum
        f[8 + int(rng.integers(0, 32))] ^= 1 << int(rng.integers(8))
    elif kind == "udp":
        f[6] = 17
    elif kind == "ext_header":  # hop-by-hop options header: not walked, so not accepted
        f[6] = 0
    elif kind == "len_short":  # the frame holds more than 40 + payload length
        f += bytes([int(rng.integers(256))])
    elif kind == "len_long":
        f = f[:-1] if len(f) > 40 else f + b"\0"
    elif kind == "version4":
        f[0] = 0x40 | (f[0] & 15)
    elif kind == "jumbo":  # payload length 0 (RFC 2675 jumbogram form) with a real payload behind it
        f[4:6] = b"\0\0"
    return bytes(f)


def batch(rng, n: int, kinds=KINDS, weights=None, lead: int = 0, max_payload: int = 1460, ip: int = 4):
    """(buf uint8, offsets uint64[n+1], kinds list): n frames (IPv4, or IPv6 with ip=6 and kinds=KINDS6) packed
    back to back behind `lead` bytes."""
    ks = list(rng.choice(kinds, n, p=weights)) if n else []
    make = frame6 if ip == 6 else frame
    frames = [make(rng, k, max_payload) for k in ks]
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum([len(f) for f in frames]) if n else []
    offs += np.uint64(lead)
    buf = np.frombuffer(rng.integers(0, 256, lead, dtype=np.uint8).tobytes() + b"".join(frames) +
                        rng.integers(0, 256, 3, dtype=np.uint8).tobytes(), np.uint8).copy()
    return buf, offs, ks
