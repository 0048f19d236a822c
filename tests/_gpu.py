"""Shared helpers of the -m gpu tests: numpy <-> device tensors and the two batch
entry points with numpy inputs (the results come back as uint16 arrays)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
import nsx  # noqa: E402


def setup_gpu():
    assert torch.cuda.is_available(), "GPU tests need an MI355X; the HIP path has no CPU fallback"
    assert nsx.device_count() > 0
    torch.cuda.set_device(0)


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def u16(t):
    return host(t.view(torch.int16)).view(np.uint16)


def run_fixed(buf_np, stride, seg_len, n, partial=None, start=0, tune=None):
    d = dev(buf_np)
    p = None if partial is None else dev(np.asarray(partial, np.uint32).view(np.int32))
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    nsx.fixed_dev(d[start:], stride, seg_len, n, partial=p, out=out, tune=tune)
    return u16(out)


def run_ragged(buf_np, offsets, partial=None, tune=None):
    d = dev(buf_np)
    o = dev(np.asarray(offsets, np.uint64).view(np.int64))
    p = None if partial is None else dev(np.asarray(partial, np.uint32).view(np.int32))
    n = len(offsets) - 1
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    nsx.ragged_dev(d, o, partial=p, out=out, tune=tune)
    return u16(out)


def mask_words(valid):
    pad = np.zeros((valid.size + 63) // 64 * 64, np.uint8)
    pad[:valid.size] = valid
    return np.packbits(pad, bitorder="little").view(np.uint64)


def pseudo_headers(addrs, tcp_len):
    """(n, 12) IPv4 pseudo-header bytes src(4) dst(4) 0 6 len(2) (RFC 9293 §3.1; ip.Addr.Raw(),
    network/ip/v4/ipv4.go:15; ip.NextProtoTCP, protocols.go:8) from (2, n, 4) address bytes, as a Go caller
    would pass ipPseudoHeader (tcp.go:72-73)."""
    n = addrs.shape[1]
    return np.ascontiguousarray(np.concatenate(
        [addrs[0], addrs[1], np.tile(np.array([0, 6, tcp_len >> 8, tcp_len & 0xFF], np.uint8), (n, 1))], 1))
