"""nsx — Python binding of libnsx_csum.so (include/nsx_csum.h) for tests and bench.

The product is the C ABI + gfx950 kernels in ../csrc; this module is plumbing:
ctypes calls with torch tensors as device buffers. There is no fallback of any
kind: if the library is missing, importing a device call raises, and on a host
without a GPU the device calls return NSX_ENODEV, raised here as NsxError.

Reference interface mirrored (transport/tcp/tcp.go:72-95):
    computeChecksum(ipPseudoHeader []byte) uint16  → csum16(prefix, seg) -> int
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "lib", "libnsx_csum.so")
HEADER_PATH = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "nsx_csum.h")

NSX_OK, NSX_EIO, NSX_ENOMEM, NSX_ENODEV, NSX_EINVAL = 0, -5, -12, -19, -22
# nsx_tune.kernel (include/nsx_tune.h)
KERNEL_HDR_THREAD, KERNEL_HDR_DENSE, KERNEL_BUILD_PLAIN, KERNEL_BUILD_GENERAL, KERNEL_SCAN_PLAIN = 1, 2, 2, 3, 2


class Tune(ctypes.Structure):
    """include/nsx_tune.h: per-call launch overrides (0 = default). Benchmarks and tests only."""
    _fields_ = [("blocks_per_cu", ctypes.c_int32), ("segs_per_wave", ctypes.c_int32),
                ("block_mode", ctypes.c_int32), ("rows", ctypes.c_int32), ("run_segs", ctypes.c_int32),
                ("xcd_chunk", ctypes.c_int32), ("window_bytes", ctypes.c_int64), ("kernel", ctypes.c_int32),
                ("shards_per_device", ctypes.c_int32), ("deal", ctypes.c_int32),
                ("reserved", ctypes.c_int32 * 5)]


TUNE_FIELDS = tuple(f for f, _ in Tune._fields_ if f != "reserved")


def _tune(tune):
    """dict (or Tune, or None) → ctypes pointer argument (None = defaults)."""
    if tune is None or isinstance(tune, Tune):
        return None if tune is None else ctypes.byref(tune)
    bad = set(tune) - set(TUNE_FIELDS)
    if bad:
        raise ValueError(f"unknown nsx_tune field(s): {sorted(bad)}")
    return ctypes.byref(Tune(**{k: int(v) for k, v in tune.items()}))


class NsxError(RuntimeError):
    def __init__(self, code: int, what: str):
        self.code = code
        super().__init__(f"{what}: {lib().nsx_strerror(code).decode()} ({code})")


_lib = None


def lib() -> ctypes.CDLL:
    """Load the in-tree product library; fail loudly if it was not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"libnsx_csum.so not built at {LIB_PATH}: run `make -C network-stack_amd` "
                              "or __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        vp, sz, u64, u32, i32, u8 = (ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint32,
                                     ctypes.c_int, ctypes.c_uint8)
        sig = {
            "nsx_csum16": [vp, sz, vp, sz, vp],
            "nsx_csum_fixed_dev": [vp, u64, u32, u64, vp, vp, vp],
            "nsx_csum_ragged_dev": [vp, vp, u64, vp, vp, vp],
            "nsx_verify_ragged_dev": [vp, vp, u64, vp, vp, vp, vp],
            "nsx_pseudo_ipv4_partial_dev": [vp, vp, vp, u8, u64, vp, vp],
            "nsx_pseudo_ipv6_partial_dev": [vp, vp, vp, u8, u64, vp, vp],
            "nsx_verify_mask_dev": [vp, u64, vp, vp],
            "nsx_host_cache_release": [],
            "nsx_stream_release": [vp],
            "nsx_deal_sets_in_use": [ctypes.POINTER(u32)],
            "nsx_csum_fixed_host": [vp, u64, u32, u64, vp, vp, i32],
            "nsx_csum_ragged_host": [vp, vp, u64, vp, vp, i32],
            "nsx_alloc_pinned": [sz, ctypes.POINTER(vp)],
            "nsx_free_pinned": [vp],
            "nsx_shard_plan": [vp, u64, i32, vp],
            "nsx_fill_splitmix64_dev": [vp, u64, u64, u64, vp],
            "nsx_ipv4_hdr_csum_dev": [vp, u64, u32, u64, i32, vp, vp],
            "nsx_ipv4_hdr_verify_mask_dev": [vp, u64, u32, u64, vp, vp],
            "nsx_rx_ipv4_tcp_verify_dev": [vp, vp, u64, vp, vp, vp, vp],
            "nsx_rx_ipv4_tcp_verify_dev_tuned": [vp, vp, u64, vp, vp, vp, vp, vp],
            "nsx_rx_ipv4_tcp_verify_host": [vp, vp, u64, vp, i32],
            "nsx_rx_ipv4_tcp_verify_host_tuned": [vp, vp, u64, vp, i32, vp],
            "nsx_tcp_parse_dev": [vp, vp, u64, vp, vp],
            "nsx_rx_ipv6_tcp_verify_dev": [vp, vp, u64, vp, vp, vp],
            "nsx_rx_ipv6_tcp_verify_dev_tuned": [vp, vp, u64, vp, vp, vp, vp],
            "nsx_rx_ipv6_tcp_verify_host": [vp, vp, u64, vp, i32],
            "nsx_rx_ipv6_tcp_verify_host_tuned": [vp, vp, u64, vp, i32, vp],
            "nsx_tcp_build_dev": [vp, vp, vp, vp, vp, u64, vp, u64, vp, vp, vp, vp],
            "nsx_tcp_layout_host": [vp, vp, u64, vp],
            "nsx_abi_version": [],
            "nsx_device_count": [ctypes.POINTER(i32)],
            # include/nsx_tune.h (per-call overrides)
            "nsx_csum_fixed_dev_tuned": [vp, u64, u32, u64, vp, vp, vp, vp],
            "nsx_csum_ragged_dev_tuned": [vp, vp, u64, vp, vp, vp, vp],
            "nsx_verify_ragged_dev_tuned": [vp, vp, u64, vp, vp, vp, vp, vp],
            "nsx_tcp_build_dev_tuned": [vp, vp, vp, vp, vp, u64, vp, u64, vp, vp, vp, vp, vp],
            "nsx_ipv4_hdr_csum_dev_tuned": [vp, u64, u32, u64, i32, vp, vp, vp],
            "nsx_ipv4_hdr_verify_mask_dev_tuned": [vp, u64, u32, u64, vp, vp, vp],
            "nsx_csum_fixed_host_tuned": [vp, u64, u32, u64, vp, vp, i32, vp],
            "nsx_csum_ragged_host_tuned": [vp, vp, u64, vp, vp, i32, vp],
            "nsx_tcp_build_host": [vp, vp, vp, vp, vp, vp, u64, vp, vp, vp, i32],
            "nsx_tcp_build_host_tuned": [vp, vp, vp, vp, vp, vp, u64, vp, vp, vp, i32, vp],
            "nsx_fixed_launch_count": [u64, u32, u64, vp, ctypes.POINTER(u64)],
            "nsx_ipv4_hdr_launch_count": [vp, u64, u32, u64, vp, ctypes.POINTER(u64)],
        }
        # present since ABI round 6; an older library (same-box A/B against a previous build) lacks them
        optional = {"nsx_stream_release", "nsx_deal_sets_in_use"}
        for name, args in sig.items():
            if name in optional and not hasattr(L, name):
                continue
            f = getattr(L, name)
            f.argtypes = args
            f.restype = ctypes.c_int
        L.nsx_tcp_wire_len.argtypes = [u64, u64]
        L.nsx_tcp_wire_len.restype = ctypes.c_uint64
        L.nsx_strerror.argtypes = [i32]
        L.nsx_strerror.restype = ctypes.c_char_p
        _lib = L
    return _lib


def _check(rc: int, what: str) -> None:
    if rc != NSX_OK:
        raise NsxError(rc, what)


def _np_ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _dev_ptr(t):
    """A device tensor's address for the C call (a host tensor is refused: the device entry points take HBM
    pointers). Called after every _span check of the wrapper, so extent errors are reported first."""
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError(f"must be a device (HIP) tensor, got one on {t.device}")
    return ctypes.c_void_p(t.data_ptr())


def _span(t, nbytes: int, what: str, elem: int | None = None):
    """The C ABI takes bare device pointers and cannot see extents, so every device wrapper checks its tensors
    here, before the C call: contiguous, `elem`-byte elements (when given), at least `nbytes` bytes (_dev_ptr then
    refuses host tensors). An undersized tensor would otherwise be an out-of-bounds device access. (Data-dependent extents — a ragged
    batch's last offset — live in device memory and are not read here: that would synchronise the stream.)"""
    if t is None:
        return
    if not t.is_contiguous():
        raise ValueError(f"{what}: tensor must be contiguous")
    if elem is not None and t.element_size() != elem:
        raise ValueError(f"{what}: needs {elem}-byte elements, got {t.dtype}")
    have = t.numel() * t.element_size()
    if have < nbytes:
        raise ValueError(f"{what}: {have} B given, {nbytes} B needed")


def _count(offsets, what: str) -> int:
    """n from an (n+1)-entry offsets tensor of 8-byte elements."""
    _span(offsets, 8, what, elem=8)
    return offsets.numel() - 1


def _stream(stream):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


# ---------------------------------------------------------------------------
# host-side API
# ---------------------------------------------------------------------------
def abi_version() -> int:
    return lib().nsx_abi_version()


def device_count() -> int:
    c = ctypes.c_int(0)
    _check(lib().nsx_device_count(ctypes.byref(c)), "nsx_device_count")
    return c.value


def csum16(prefix: bytes, seg: bytes) -> int:
    """computeChecksum (tcp.go:72-95): raw one's-complement sum over prefix ‖ seg."""
    p = np.frombuffer(bytes(prefix), np.uint8) if prefix else None
    s = np.frombuffer(bytes(seg), np.uint8) if seg else None
    out = ctypes.c_uint16(0)
    _check(lib().nsx_csum16(_np_ptr(p), len(prefix), _np_ptr(s), len(seg), ctypes.byref(out)), "nsx_csum16")
    return out.value


def field(raw: int) -> int:
    return (~raw) & 0xFFFF


def verify(raw: int) -> bool:
    return raw == 0xFFFF


def shard_plan(n: int, parts: int, offsets: np.ndarray | None = None) -> np.ndarray:
    b = np.zeros(parts + 1, np.uint64)
    off = None if offsets is None else np.ascontiguousarray(offsets, np.uint64)
    _check(lib().nsx_shard_plan(_np_ptr(off), n, parts, _np_ptr(b)), "nsx_shard_plan")
    return b


def stream_release(stream) -> None:
    """nsx_stream_release: return a stream's deal counters (call after it has drained, before destroying it).
    `stream`: a torch stream, or a raw handle value (int)."""
    h = stream if isinstance(stream, int) else stream.cuda_stream
    _check(lib().nsx_stream_release(ctypes.c_void_p(h)), "nsx_stream_release")


def deal_sets_in_use() -> int:
    """Per-stream deal counter sets given out on the current device (nsx_deal_sets_in_use)."""
    c = ctypes.c_uint32(0)
    _check(lib().nsx_deal_sets_in_use(ctypes.byref(c)), "nsx_deal_sets_in_use")
    return c.value


def ipv4_hdr_launch_count(buf, stride: int, n: int, hdr_off: int = 0, tune=None) -> int:
    """Kernel launches one IPv4 header call makes for this batch on the current device."""
    c = ctypes.c_uint64(0)
    _check(lib().nsx_ipv4_hdr_launch_count(ctypes.c_void_p(buf.data_ptr()), stride, hdr_off, n, _tune(tune),
                                           ctypes.byref(c)), "nsx_ipv4_hdr_launch_count")
    return c.value


def fixed_launch_count(stride: int, seg_len: int, n: int, tune=None) -> int:
    """Kernel launches one fixed_dev call makes for this batch on the current device."""
    c = ctypes.c_uint64(0)
    _check(lib().nsx_fixed_launch_count(stride, seg_len, n, _tune(tune), ctypes.byref(c)), "nsx_fixed_launch_count")
    return c.value


def fixed_host(buf: np.ndarray, stride: int, seg_len: int, n: int, partial: np.ndarray | None = None,
               num_gpus: int = 0, tune=None) -> np.ndarray:
    buf = np.ascontiguousarray(buf, np.uint8)
    out = np.empty(n, np.uint16)
    part = None if partial is None else np.ascontiguousarray(partial, np.uint32)
    if n > 0 and buf.size < (n - 1) * stride + seg_len:
        raise ValueError(f"fixed_host buf: {buf.size} B given, {(n - 1) * stride + seg_len} B needed")
    if part is not None and part.size < n:
        raise ValueError(f"fixed_host partial: {part.size} entries for {n} segments")
    _check(lib().nsx_csum_fixed_host_tuned(_np_ptr(buf), stride, seg_len, n, _np_ptr(part), _np_ptr(out), num_gpus,
                                           _tune(tune)), "nsx_csum_fixed_host")
    return out


def ragged_host(buf: np.ndarray, offsets: np.ndarray, partial: np.ndarray | None = None,
                num_gpus: int = 0, tune=None) -> np.ndarray:
    buf = np.ascontiguousarray(buf, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    n = offsets.size - 1
    out = np.empty(max(n, 0), np.uint16)
    part = None if partial is None else np.ascontiguousarray(partial, np.uint32)
    if n > 0 and buf.size < int(offsets[-1]):
        raise ValueError(f"ragged_host buf: {buf.size} B given, offsets end at {int(offsets[-1])}")
    if part is not None and part.size < n:
        raise ValueError(f"ragged_host partial: {part.size} entries for {n} segments")
    _check(lib().nsx_csum_ragged_host_tuned(_np_ptr(buf), _np_ptr(offsets), n, _np_ptr(part), _np_ptr(out), num_gpus,
                                            _tune(tune)), "nsx_csum_ragged_host")
    return out


def rx_ipv4_tcp_verify_host(buf: np.ndarray, offsets: np.ndarray, num_gpus: int = 0, tune=None,
                            ipver: int = 4) -> np.ndarray:
    """Fused receive pass over host-resident datagrams (IPv4, or IPv6 with ipver=6): the validity bitmask
    (uint64[ceil(n/64)])."""
    buf = np.ascontiguousarray(buf, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    n = offsets.size - 1
    mask = np.zeros((max(n, 0) + 63) // 64, np.uint64)
    if n > 0 and buf.size < int(offsets[-1]):
        raise ValueError(f"rx host buf: {buf.size} B given, offsets end at {int(offsets[-1])}")
    name = "nsx_rx_ipv6_tcp_verify_host" if ipver == 6 else "nsx_rx_ipv4_tcp_verify_host"
    _check(getattr(lib(), name + "_tuned")(_np_ptr(buf), _np_ptr(offsets), n, _np_ptr(mask), num_gpus, _tune(tune)),
           name)
    return mask


def rx_ipv6_tcp_verify_host(buf: np.ndarray, offsets: np.ndarray, num_gpus: int = 0, tune=None) -> np.ndarray:
    return rx_ipv4_tcp_verify_host(buf, offsets, num_gpus, tune, ipver=6)


class PinnedBuffer:
    """nsx_alloc_pinned-backed numpy view (DMA-registered host memory)."""

    def __init__(self, nbytes: int):
        p = ctypes.c_void_p()
        _check(lib().nsx_alloc_pinned(nbytes, ctypes.byref(p)), "nsx_alloc_pinned")
        self._p = p
        self.nbytes = nbytes
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p.value)) if nbytes else \
            np.zeros(0, np.uint8)

    def free(self):
        if self._p:
            _check(lib().nsx_free_pinned(self._p), "nsx_free_pinned")
            self._p = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


# ---------------------------------------------------------------------------
# device-side API (torch tensors as HBM buffers)
# ---------------------------------------------------------------------------
def fixed_dev(buf, stride: int, seg_len: int, n: int, partial=None, out=None, stream=None, tune=None):
    import torch
    if out is None:
        out = torch.empty(n, dtype=torch.int16, device=buf.device)  # u16 bits
    _span(buf, (n - 1) * stride + seg_len if n > 0 else 0, "fixed_dev buf")
    _span(partial, 4 * n, "fixed_dev partial", elem=4)
    _span(out, 2 * n, "fixed_dev out", elem=2)
    _check(lib().nsx_csum_fixed_dev_tuned(_dev_ptr(buf), stride, seg_len, n, _dev_ptr(partial), _dev_ptr(out),
                                          _stream(stream), _tune(tune)), "nsx_csum_fixed_dev")
    return out


def ragged_dev(buf, offsets, partial=None, out=None, stream=None, tune=None):
    import torch
    n = _count(offsets, "ragged_dev offsets")
    if out is None:
        out = torch.empty(max(n, 0), dtype=torch.int16, device=offsets.device)  # u16 bits
    _span(buf, 0, "ragged_dev buf")
    _span(partial, 4 * n, "ragged_dev partial", elem=4)
    _span(out, 2 * n, "ragged_dev out", elem=2)
    _check(lib().nsx_csum_ragged_dev_tuned(_dev_ptr(buf), _dev_ptr(offsets), n, _dev_ptr(partial), _dev_ptr(out),
                                           _stream(stream), _tune(tune)), "nsx_csum_ragged_dev")
    return out


def verify_ragged_dev(buf, offsets, partial=None, raw=None, stream=None, tune=None, ok=None):
    import torch
    n = _count(offsets, "verify_ragged_dev offsets")
    if ok is None:
        ok = torch.empty(max(n, 0), dtype=torch.uint8, device=offsets.device)
    _span(ok, n, "verify_ragged_dev ok")
    _span(buf, 0, "verify_ragged_dev buf")
    _span(partial, 4 * n, "verify_ragged_dev partial", elem=4)
    _span(raw, 2 * n, "verify_ragged_dev raw", elem=2)
    _check(lib().nsx_verify_ragged_dev_tuned(_dev_ptr(buf), _dev_ptr(offsets), n, _dev_ptr(partial), _dev_ptr(ok),
                                             _dev_ptr(raw), _stream(stream), _tune(tune)), "nsx_verify_ragged_dev")
    return ok


def pseudo_ipv4_partial_dev(src, dst, length, proto: int = 6, out=None, stream=None):
    import torch
    n = length.numel()
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=length.device)  # u32 bits
    _span(length, 4 * n, "pseudo_ipv4_partial_dev length", elem=4)
    _span(src, 4 * n, "pseudo_ipv4_partial_dev src")
    _span(dst, 4 * n, "pseudo_ipv4_partial_dev dst")
    _span(out, 4 * n, "pseudo_ipv4_partial_dev out", elem=4)
    _check(lib().nsx_pseudo_ipv4_partial_dev(_dev_ptr(src), _dev_ptr(dst), _dev_ptr(length), proto, n,
                                             _dev_ptr(out), _stream(stream)), "nsx_pseudo_ipv4_partial_dev")
    return out


def pseudo_ipv6_partial_dev(src, dst, length, next_header: int = 6, out=None, stream=None):
    import torch
    n = length.numel()
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=length.device)  # u32 bits
    _span(length, 4 * n, "pseudo_ipv6_partial_dev length", elem=4)
    _span(src, 16 * n, "pseudo_ipv6_partial_dev src")
    _span(dst, 16 * n, "pseudo_ipv6_partial_dev dst")
    _span(out, 4 * n, "pseudo_ipv6_partial_dev out", elem=4)
    _check(lib().nsx_pseudo_ipv6_partial_dev(_dev_ptr(src), _dev_ptr(dst), _dev_ptr(length), next_header, n,
                                             _dev_ptr(out), _stream(stream)), "nsx_pseudo_ipv6_partial_dev")
    return out


def verify_mask_dev(raw, out=None, stream=None):
    """Bitmask of raw == 0xFFFF (tcp.go:70): int64 tensor of ceil(n/64) words."""
    import torch
    n = raw.numel()
    if out is None:
        out = torch.empty((n + 63) // 64, dtype=torch.int64, device=raw.device)  # u64 bits
    _span(raw, 2 * n, "verify_mask_dev raw", elem=2)
    _span(out, 8 * ((n + 63) // 64), "verify_mask_dev out", elem=8)
    _check(lib().nsx_verify_mask_dev(_dev_ptr(raw), n, _dev_ptr(out), _stream(stream)), "nsx_verify_mask_dev")
    return out


def ipv4_hdr_csum_dev(buf, stride: int, n: int, hdr_off: int = 0, mode: int = 0, out=None, stream=None, tune=None):
    """RFC 791 header checksums of n packets at a fixed stride (mode 0 verify, 1 fill in place)."""
    import torch
    if out is None and mode == 0:
        out = torch.empty(n, dtype=torch.int16, device=buf.device)  # u16 bits
    _span(buf, (n - 1) * stride + hdr_off + 20 if n > 0 else 0, "ipv4_hdr_csum_dev buf")
    _span(out, 2 * n, "ipv4_hdr_csum_dev out", elem=2)
    _check(lib().nsx_ipv4_hdr_csum_dev_tuned(_dev_ptr(buf), stride, hdr_off, n, mode, _dev_ptr(out), _stream(stream),
                                             _tune(tune)), "nsx_ipv4_hdr_csum_dev")
    return out


def ipv4_hdr_verify_mask_dev(buf, stride: int, n: int, hdr_off: int = 0, mask=None, stream=None, tune=None):
    """Fused IPv4 header verify into a bitmask: bit i%64 of mask[i//64] iff header i is valid."""
    import torch
    if mask is None:
        mask = torch.empty((n + 63) // 64, dtype=torch.int64, device=buf.device)  # u64 bits
    _span(buf, (n - 1) * stride + hdr_off + 20 if n > 0 else 0, "ipv4_hdr_verify_mask_dev buf")
    _span(mask, 8 * ((n + 63) // 64), "ipv4_hdr_verify_mask_dev mask", elem=8)
    _check(lib().nsx_ipv4_hdr_verify_mask_dev_tuned(_dev_ptr(buf), stride, hdr_off, n, _dev_ptr(mask),
                                                    _stream(stream), _tune(tune)), "nsx_ipv4_hdr_verify_mask_dev")
    return mask


def rx_ipv4_tcp_verify_dev(buf, offsets, mask=None, ip_raw=None, tcp_raw=None, stream=None, tune=None):
    """Fused receive pass over packed IPv4/TCP frames: validity bitmask (+ optional raw sums)."""
    import torch
    n = _count(offsets, "rx_ipv4_tcp_verify_dev offsets")
    if mask is None:
        mask = torch.empty((max(n, 0) + 63) // 64, dtype=torch.int64, device=offsets.device)  # u64 bits
    _span(buf, 0, "rx_ipv4_tcp_verify_dev buf")
    _span(mask, 8 * ((n + 63) // 64), "rx_ipv4_tcp_verify_dev mask", elem=8)
    _span(ip_raw, 2 * n, "rx_ipv4_tcp_verify_dev ip_raw", elem=2)
    _span(tcp_raw, 2 * n, "rx_ipv4_tcp_verify_dev tcp_raw", elem=2)
    _check(lib().nsx_rx_ipv4_tcp_verify_dev_tuned(_dev_ptr(buf), _dev_ptr(offsets), n, _dev_ptr(mask),
                                                  _dev_ptr(ip_raw), _dev_ptr(tcp_raw), _stream(stream), _tune(tune)),
           "nsx_rx_ipv4_tcp_verify_dev")
    return mask


def rx_ipv6_tcp_verify_dev(buf, offsets, mask=None, tcp_raw=None, stream=None, tune=None):
    """Fused receive pass over packed IPv6/TCP packets: validity bitmask (+ optional raw TCP sums)."""
    import torch
    n = _count(offsets, "rx_ipv6_tcp_verify_dev offsets")
    if mask is None:
        mask = torch.empty((max(n, 0) + 63) // 64, dtype=torch.int64, device=offsets.device)  # u64 bits
    _span(buf, 0, "rx_ipv6_tcp_verify_dev buf")
    _span(mask, 8 * ((n + 63) // 64), "rx_ipv6_tcp_verify_dev mask", elem=8)
    _span(tcp_raw, 2 * n, "rx_ipv6_tcp_verify_dev tcp_raw", elem=2)
    _check(lib().nsx_rx_ipv6_tcp_verify_dev_tuned(_dev_ptr(buf), _dev_ptr(offsets), n, _dev_ptr(mask),
                                                  _dev_ptr(tcp_raw), _stream(stream), _tune(tune)),
           "nsx_rx_ipv6_tcp_verify_dev")
    return mask


BUILD_FIELDS = (("src_port", 2), ("dst_port", 2), ("seq_num", 4), ("ack_num", 4), ("offset", 1), ("control", 1),
                ("window", 2), ("urgent_ptr", 2))  # nsx_tcp_hdr_soa members and their element sizes


class TcpHdrSoA(ctypes.Structure):
    _fields_ = [(name, ctypes.c_void_p) for name, _ in BUILD_FIELDS]


PARSE_FIELDS = (("src_port", "int16"), ("dst_port", "int16"), ("seq_num", "int32"), ("ack_num", "int32"),
                ("offset", "uint8"), ("control", "uint8"), ("window", "int16"), ("checksum", "int16"),
                ("urgent_ptr", "int16"), ("data_off", "int64"), ("n_options", "uint8"), ("status", "uint8"))
PARSE_OK, PARSE_SHORT, PARSE_OFFSET, PARSE_OPTION_RANGE, PARSE_OPTION_KIND = 0, 1, 2, 3, 4


class TcpParsedSoA(ctypes.Structure):
    _fields_ = [(name, ctypes.c_void_p) for name, _ in PARSE_FIELDS]


def tcp_parse_dev(buf, offsets, fields=None, want=None, stream=None) -> dict:
    """parseSegment (tcp.go:130-185) over the segments buf[offsets[i], offsets[i+1]) into device tensors (dict
    by field; `want` = the field names to produce, default all; `fields` = caller tensors to fill)."""
    import torch
    n = _count(offsets, "tcp_parse_dev offsets")
    names = [k for k, _ in PARSE_FIELDS] if want is None else list(want)
    out = dict(fields or {})
    for k, dt in PARSE_FIELDS:
        if k in names and k not in out:
            out[k] = torch.empty(max(n, 0), dtype=getattr(torch, dt), device=offsets.device)
    _span(buf, 0, "tcp_parse_dev buf")
    for k, dt in PARSE_FIELDS:
        size = np.dtype(dt).itemsize
        _span(out.get(k), size * n, f"tcp_parse_dev {k}", elem=size)
    soa =TcpParsedSoA(*[_dev_ptr(out.get(k)) for k, _ in PARSE_FIELDS])
    _check(lib().nsx_tcp_parse_dev(_dev_ptr(buf), _dev_ptr(offsets), n, ctypes.byref(soa), _stream(stream)),
           "nsx_tcp_parse_dev")
    return out


def tcp_wire_len(opt_len: int, data_len: int) -> int:
    return lib().nsx_tcp_wire_len(opt_len, data_len)


def tcp_layout_host(data_off: np.ndarray, opt_off: np.ndarray | None = None) -> np.ndarray:
    data_off = np.ascontiguousarray(data_off, np.uint64)
    n = data_off.size - 1
    out = np.zeros(n + 1, np.uint64)
    oo = None if opt_off is None else np.ascontiguousarray(opt_off, np.uint64)
    _check(lib().nsx_tcp_layout_host(_np_ptr(oo), _np_ptr(data_off), n, _np_ptr(out)), "nsx_tcp_layout_host")
    return out


def tcp_build_dev(fields: dict, data, data_off, out, out_off, opts=None, opt_off=None, partial=None, raw=None,
                  stream=None, tune=None):
    """Fused segment.bytes() + checksum + field write (fields: dict of device tensors; a missing or None
    "offset" computes byte 12 on the device as computeOffset() does, tcp.go:59-66)."""
    n = _count(data_off, "tcp_build_dev data_off")
    for k, size in BUILD_FIELDS:
        if fields.get(k) is None and k != "offset":  # only byte 12 may be computed on the device
            raise ValueError(f"tcp_build_dev: header field {k!r} missing")
        _span(fields.get(k), size * n, f"tcp_build_dev {k}", elem=size)
    _span(data, 0, "tcp_build_dev data")
    _span(out_off, 8 * (n + 1), "tcp_build_dev out_off", elem=8)
    _span(out, 0, "tcp_build_dev out")
    _span(opt_off, 8 * (n + 1), "tcp_build_dev opt_off", elem=8)
    if opt_off is not None and opts is None:
        raise ValueError("tcp_build_dev: opt_off given without opts")
    _span(opts, 0, "tcp_build_dev opts")
    _span(partial, 4 * n, "tcp_build_dev partial", elem=4)
    _span(raw, 2 * n, "tcp_build_dev raw", elem=2)
    soa = TcpHdrSoA(*[_dev_ptr(fields.get(k)) for k, _ in BUILD_FIELDS])
    _check(lib().nsx_tcp_build_dev_tuned(ctypes.byref(soa), _dev_ptr(opts), _dev_ptr(opt_off), _dev_ptr(data),
                                         _dev_ptr(data_off), data.numel(), _dev_ptr(partial), n, _dev_ptr(out),
                                         _dev_ptr(out_off), _dev_ptr(raw), _stream(stream), _tune(tune)),
           "nsx_tcp_build_dev")
    return out


_BUILD_NP = {"src_port": np.uint16, "dst_port": np.uint16, "seq_num": np.uint32, "ack_num": np.uint32,
             "offset": np.uint8, "control": np.uint8, "window": np.uint16, "urgent_ptr": np.uint16}


def tcp_build_host(fields: dict, data: np.ndarray, data_off: np.ndarray, out_off: np.ndarray | None = None,
                   opts: np.ndarray | None = None, opt_off: np.ndarray | None = None,
                   partial: np.ndarray | None = None, out: np.ndarray | None = None, want_raw: bool = True,
                   num_gpus: int = 0, tune=None):
    """The fused sender pass over host-resident segments (nsx_tcp_build_host): fields = dict of host arrays (a
    missing or None "offset" is computed on the device, tcp.go:59-66); out_off defaults to nsx_tcp_layout_host;
    out (host uint8, e.g. a PinnedBuffer's array) is allocated when not given. Returns (out, raw or None)."""
    data = np.ascontiguousarray(data, np.uint8)
    data_off = np.ascontiguousarray(data_off, np.uint64)
    n = data_off.size - 1
    cols = {}
    for k, _ in BUILD_FIELDS:
        v = fields.get(k)
        if v is None:
            if k != "offset":
                raise ValueError(f"tcp_build_host: header field {k!r} missing")
            continue
        v = np.ascontiguousarray(v).view(_BUILD_NP[k]) if np.asarray(v).dtype.itemsize == np.dtype(_BUILD_NP[k]).itemsize \
            else np.ascontiguousarray(v, _BUILD_NP[k])
        if v.size < n:
            raise ValueError(f"tcp_build_host {k}: {v.size} entries for {n} segments")
        cols[k] = v
    oo = None if opt_off is None else np.ascontiguousarray(opt_off, np.uint64)
    if oo is not None and opts is None:
        raise ValueError("tcp_build_host: opt_off given without opts")
    ob = None if opts is None else (np.ascontiguousarray(opts, np.uint8) if len(opts) else np.zeros(1, np.uint8))
    if out_off is None:
        out_off = tcp_layout_host(data_off, oo)
    out_off = np.ascontiguousarray(out_off, np.uint64)
    if n > 0 and data.size < int(data_off[-1]):
        raise ValueError(f"tcp_build_host data: {data.size} B given, data_off ends at {int(data_off[-1])}")
    if oo is not None and n > 0 and ob.size < int(oo[-1]):
        raise ValueError(f"tcp_build_host opts: {ob.size} B given, opt_off ends at {int(oo[-1])}")
    if out is None:
        out = np.zeros(int(out_off[-1]) if n > 0 else 0, np.uint8)
    # the C call writes the images contiguously from out's first byte: a strided view, or a view of wider elements,
    # would be written past
    if not isinstance(out, np.ndarray) or out.dtype != np.uint8 or not out.flags.c_contiguous:
        raise ValueError("tcp_build_host out: needs a C-contiguous uint8 array")
    if n > 0 and out.size < int(out_off[-1]):
        raise ValueError(f"tcp_build_host out: {out.size} B given, out_off ends at {int(out_off[-1])}")
    part = None if partial is None else np.ascontiguousarray(partial, np.uint32)
    if part is not None and part.size < n:
        raise ValueError(f"tcp_build_host partial: {part.size} entries for {n} segments")
    raw = np.empty(max(n, 0), np.uint16) if want_raw else None
    soa = TcpHdrSoA(*[_np_ptr(cols.get(k)) for k, _ in BUILD_FIELDS])
    _check(lib().nsx_tcp_build_host_tuned(ctypes.byref(soa), _np_ptr(ob), _np_ptr(oo), _np_ptr(data),
                                          _np_ptr(data_off), _np_ptr(part), n, _np_ptr(out), _np_ptr(out_off),
                                          _np_ptr(raw), num_gpus, _tune(tune)), "nsx_tcp_build_host")
    return out, raw


def fill_splitmix64_dev(buf, seed: int, byte_off: int = 0, stream=None):
    _span(buf, 0, "fill_splitmix64_dev buf")
    _check(lib().nsx_fill_splitmix64_dev(_dev_ptr(buf), byte_off, buf.numel() * buf.element_size(), seed,
                                         _stream(stream)), "nsx_fill_splitmix64_dev")
    return buf
