#!/usr/bin/env python3
"""End-to-end host-memory rate of the checksum path (north_star: segments come
from and return to the transport's host buffers). Times nsx_csum_fixed_host /
nsx_csum_ragged_host — pinned H2D → kernel → D2H, double-buffered over two
streams per GPU — on config 2 (1M x 1500 B) and config 3 (1M ragged) batches
held in pinned memory (nsx_alloc_pinned) and in pageable numpy memory, and the
fused receive pass from host memory (nsx_rx_ipv4_tcp_verify_host) over ~770 MB of
received datagrams (a mixed batch of tests/_rx.py tiled 200 times), and the fused
sender pass from host memory (nsx_tcp_build_host) on bench workload 6's shape.
Results are spot-checked against the oracle (tools are test infrastructure).

    python tools/e2e_host.py [--reps 5] [--gpus 0]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "network-stack_amd"))

import numpy as np  # noqa: E402

import nsx  # noqa: E402
from oracle import csum_oracle as O  # noqa: E402


def timed(fn, reps):
    fn()  # warm (allocations, first touch)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts), out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--gpus", type=int, default=0)
    a = ap.parse_args()
    res = {"gpus_visible": nsx.device_count()}
    n, L = 1 << 20, 1500
    nbytes = n * L
    page = O.c_splitmix64(0x1071, nbytes)
    pin = nsx.PinnedBuffer(nbytes)
    pin.array[:] = page
    for name, arr in (("fixed_pinned", pin.array), ("fixed_pageable", page)):
        t, out = timed(lambda: nsx.fixed_host(arr, L, L, n, num_gpus=a.gpus), a.reps)
        idx = np.arange(0, n, 4099)
        want = O.batch_fixed(page[: (idx[-1] + 1) * L], L, L, int(idx[-1]) + 1)[idx]
        assert np.array_equal(out[idx], want), name
        res[name] = {"seconds": t, "GB_per_s": nbytes / t / 1e9, "GiB_per_s": nbytes / t / (1 << 30)}
        print(name, json.dumps(res[name]), flush=True)
    pin.free()
    rng = np.random.default_rng(0x1072)
    lens = rng.integers(64, 9001, n).astype(np.uint64)
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    total = int(offs[-1])
    rpage = O.c_splitmix64(0x1072, total)
    rpin = nsx.PinnedBuffer(total)
    rpin.array[:] = rpage
    for name, arr in (("ragged_pinned", rpin.array), ("ragged_pageable", rpage)):
        t, out = timed(lambda: nsx.ragged_host(arr, offs, num_gpus=a.gpus), a.reps)
        sel = np.arange(0, n, 4099)
        for i in sel[:64]:
            assert out[i] == O.c_fold_checksum(b"", rpage[int(offs[i]):int(offs[i + 1])].tobytes()), (name, i)
        res[name] = {"seconds": t, "GB_per_s": total / t / 1e9, "GiB_per_s": total / t / (1 << 30)}
        print(name, json.dumps(res[name]), flush=True)
    rpin.free()
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _rx
    buf0, offs0, _ = _rx.batch(np.random.default_rng(0x1079), 4992, max_payload=1460)
    span, reps = int(offs0[-1]), 200
    xbuf = np.concatenate([buf0[:span]] * reps)
    xoffs = np.concatenate([offs0[:-1] + np.uint64(k * span) for k in range(reps)] +
                           [np.array([reps * span], np.uint64)])
    want = O.c_rx_ipv4_tcp(buf0, offs0)[0]
    xpin = nsx.PinnedBuffer(xbuf.nbytes)
    xpin.array[:] = xbuf
    for name, arr in (("rx_pinned", xpin.array), ("rx_pageable", xbuf)):
        t, out = timed(lambda: nsx.rx_ipv4_tcp_verify_host(arr, xoffs, num_gpus=a.gpus), a.reps)
        assert np.array_equal(out.reshape(reps, -1), np.tile(want, (reps, 1))), name  # 4992 frames = 78 words a tile
        res[name] = {"seconds": t, "GB_per_s": xbuf.nbytes / t / 1e9, "GiB_per_s": xbuf.nbytes / t / (1 << 30),
                     "frames": int(xoffs.size - 1)}
        print(name, json.dumps(res[name]), flush=True)
    xpin.free()
    buf6, offs6, _ = _rx.batch(np.random.default_rng(0x107A), 4992, kinds=_rx.KINDS6, max_payload=1440, ip=6)
    span6 = int(offs6[-1])
    ybuf = np.concatenate([buf6[:span6]] * reps)
    yoffs = np.concatenate([offs6[:-1] + np.uint64(k * span6) for k in range(reps)] +
                           [np.array([reps * span6], np.uint64)])
    want6 = O.c_rx_ipv6_tcp(buf6, offs6)[0]
    ypin = nsx.PinnedBuffer(ybuf.nbytes)
    ypin.array[:] = ybuf
    for name, arr in (("rx6_pinned", ypin.array), ("rx6_pageable", ybuf)):
        t, out = timed(lambda: nsx.rx_ipv6_tcp_verify_host(arr, yoffs, num_gpus=a.gpus), a.reps)
        assert np.array_equal(out.reshape(reps, -1), np.tile(want6, (reps, 1))), name
        res[name] = {"seconds": t, "GB_per_s": ybuf.nbytes / t / 1e9, "GiB_per_s": ybuf.nbytes / t / (1 << 30),
                     "frames": int(yoffs.size - 1)}
        print(name, json.dumps(res[name]), flush=True)
    ypin.free()
    # the sender pass from host memory (nsx_tcp_build_host): bench workload 6's shape — 1M option-less segments,
    # 1480 B payloads, IPv4 pseudo-header partials — fields, payloads and partials in host memory, the 1500 B wire
    # images and raw sums back into host memory. Rate by wire bytes; PCIe bytes = H2D (payload + 18 B fields + 16 B
    # offsets + 4 B partial) + D2H (image + 2 B raw) per segment.
    P, W = 1480, 1500
    brng = np.random.default_rng(0x1074)
    fields = {k: brng.integers(0, 1 << (8 * np.dtype(dt).itemsize), n, dtype=np.uint64).astype(dt)
              for k, dt in zip(O.TCP_FIELDS, O.TCP_FIELD_DTYPES)}
    fields["offset"][:] = 5
    pseudo = np.concatenate([brng.integers(0, 256, (n, 8), dtype=np.uint8),
                             np.tile(np.array([0, 6, W >> 8, W & 0xFF], np.uint8), (n, 1))], 1)
    pw = pseudo.reshape(n, 6, 2).astype(np.uint32)
    part = ((pw[..., 0] << 8) | pw[..., 1]).sum(1).astype(np.uint32)
    data_off = np.arange(n + 1, dtype=np.uint64) * np.uint64(P)
    out_off = nsx.tcp_layout_host(data_off)
    dpage = O.c_splitmix64(0x1074, n * P)
    dpin, opin = nsx.PinnedBuffer(n * P), nsx.PinnedBuffer(n * W)
    dpin.array[:] = dpage
    opage = np.zeros(n * W, np.uint8)
    sel = np.arange(0, n, 4099)
    sfields = {k: v[sel] for k, v in fields.items()}
    sdata = np.concatenate([dpage[i * P:(i + 1) * P] for i in sel])
    want, wraw = O.c_go_tcp_build(sfields, sdata, np.arange(sel.size + 1, dtype=np.uint64) * np.uint64(P),
                                  np.arange(sel.size + 1, dtype=np.uint64) * np.uint64(W), pseudo[sel])
    pcie = n * (P + 18 + 16 + 4) + n * (W + 2)
    for name, d, o in (("build_pinned", dpin.array, opin.array), ("build_pageable", dpage, opage)):
        t, (img, raw) = timed(lambda: nsx.tcp_build_host(fields, d, data_off, out_off=out_off, partial=part, out=o,
                                                         num_gpus=a.gpus), a.reps)
        assert np.array_equal(raw[sel], wraw), name
        assert np.array_equal(np.concatenate([img[i * W:(i + 1) * W] for i in sel]), want), name
        res[name] = {"seconds": t, "GB_per_s": n * W / t / 1e9, "GiB_per_s": n * W / t / (1 << 30),
                     "pcie_GB_per_s_both_directions": pcie / t / 1e9, "segments": n}
        print(name, json.dumps(res[name]), flush=True)
    dpin.free()
    opin.free()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "e2e_host.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
