#!/usr/bin/env python3
"""Cost per call of the C-call sequences the Go shim makes (network-stack_amd/go/transport/tcp/*_nsx.go), timed
from ctypes (no Go toolchain exists in this pool): the one-shot forms, which pin a block per call,
against the reuse forms a transport keeps across batches.

    one-shot (ChecksumSegments, VerifyDatagrams, BuildSegments):  nsx_alloc_pinned → fill → call → nsx_free_pinned
    reuse    (PinnedBatch.Checksum / .Verify, Sender.Build):        fill → call  (the block pinned once, before)

"fill" is the shim's copy of the batch into the pinned block (Append's copy per segment, or build()'s field, offset,
partial and payload stores), done here as one bulk copy per array — the Go loop's own per-segment overhead is not
what is measured; "call" is the library call the shim makes with the same arguments (offsets, partials and outputs
in ordinary host memory where the shim passes Go memory; for the build, everything in the block as build() lays it
out). Sizes: config 1's 64 × 1500 B (the reference's loopback batch, transport/pipe/pipe.go:92-124) and 1M × 1500 B.
Each stage is timed on its own (perf_counter), median over the reps; every result is spot-checked against the oracle.

    python tools/go_call_cost.py [--reps-small 300] [--reps-large 3]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "network-stack_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402

import nsx  # noqa: E402
from oracle import csum_oracle as O  # noqa: E402

L = nsx.lib()
vp = ctypes.c_void_p


def ptr(a, off=0):
    return vp(a.ctypes.data + off)


class Pinned:
    """nsx_alloc_pinned / nsx_free_pinned, timed."""

    def __init__(self, nbytes):
        p = vp()
        t0 = time.perf_counter()
        assert L.nsx_alloc_pinned(nbytes, ctypes.byref(p)) == 0
        self.t_alloc = time.perf_counter() - t0
        self.p, self.n = p, nbytes
        self.arr = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p.value))

    def free(self):
        t0 = time.perf_counter()
        assert L.nsx_free_pinned(self.p) == 0
        return time.perf_counter() - t0


def seq_checksum(n, seg, reps, kind):
    """ChecksumSegments (one-shot) / PinnedBatch.Reset+Append+Checksum (reuse) over n segments of `seg` bytes,
    each over its IPv4 pseudo-header partial; VerifyDatagrams / PinnedBatch.Verify with kind='verify'."""
    rng = np.random.default_rng(n + seg)
    data = rng.integers(0, 256, n * seg, dtype=np.uint8)
    offs = np.arange(n + 1, dtype=np.uint64) * np.uint64(seg)
    part = rng.integers(0, 1 << 20, n, dtype=np.uint32)
    out = np.empty(n, np.uint16)
    mask = np.empty((n + 63) // 64, np.uint64)
    total = n * seg + 1

    def call(block):
        t0 = time.perf_counter()
        if kind == "verify":
            rc = L.nsx_rx_ipv4_tcp_verify_host(block.p, ptr(offs), n, ptr(mask), 0)
        else:
            rc = L.nsx_csum_ragged_host(block.p, ptr(offs), n, ptr(part), ptr(out), 0)
        assert rc == 0, rc
        return time.perf_counter() - t0

    def fill(block):
        t0 = time.perf_counter()
        ctypes.memmove(block.p.value, data.ctypes.data, n * seg)
        return time.perf_counter() - t0

    res = {"one_shot": [], "reuse": []}
    kept = Pinned(total)  # the reuse form's block, pinned once
    for r in range(reps + 1):
        b = Pinned(total)
        tf = fill(b)
        tc = call(b)
        tfree = b.free()
        if r:
            res["one_shot"].append((b.t_alloc, tf, tc, tfree))
        tf = fill(kept)
        tc = call(kept)
        if r:
            res["reuse"].append((0.0, tf, tc, 0.0))
    kept.free()
    if kind == "verify":
        assert np.array_equal(mask, O.c_rx_ipv4_tcp(data, offs)[0])
    else:
        assert np.array_equal(out, O.c_batch(data, n, offsets=offs, partial=part, threads=16))
    return res


def seq_build(n, payload, reps):
    """BuildSegments (one-shot) / Sender.Build (reuse): build_nsx.go's block — 8 field arrays, data/opt/out offsets,
    partials, options, payloads, images, raw sums — filled, then nsx_tcp_build_host over it."""
    rng = np.random.default_rng(n + payload)
    fields = {k: rng.integers(0, 1 << (8 * np.dtype(dt).itemsize), n, dtype=np.uint64).astype(dt)
              for k, dt in zip(O.TCP_FIELDS, O.TCP_FIELD_DTYPES)}
    fields["offset"][:] = 5
    data = rng.integers(0, 256, n * payload, dtype=np.uint8)
    data_off = np.arange(n + 1, dtype=np.uint64) * np.uint64(payload)
    out_off = nsx.tcp_layout_host(data_off)
    pseudo = np.concatenate([rng.integers(0, 256, (n, 8), dtype=np.uint8),
                             np.tile(np.array([0, 6, (payload + 20) >> 8, (payload + 20) & 0xFF], np.uint8), (n, 1))], 1)
    pw = pseudo.reshape(n, 6, 2).astype(np.uint32)
    part = ((pw[..., 0] << 8) | pw[..., 1]).sum(1).astype(np.uint32)  # build_nsx.go pseudoPartial
    n_out = int(out_off[-1])
    order = ["src_port", "dst_port", "seq_num", "ack_num", "offset", "control", "window", "urgent_ptr"]
    arrays = [np.ascontiguousarray(fields[k]) for k in order] + [data_off, np.zeros(n + 1, np.uint64), out_off, part]
    sizes = [a.nbytes for a in arrays] + [1, n * payload + 1, n_out, 2 * n]
    at = [0]
    for sz in sizes:
        at.append((at[-1] + sz + 63) // 64 * 64)
    total = at[-1]

    def fill(b):
        t0 = time.perf_counter()
        for k, a in enumerate(arrays):
            ctypes.memmove(b.p.value + at[k], a.ctypes.data, a.nbytes)
        ctypes.memmove(b.p.value + at[13], data.ctypes.data, data.nbytes)
        return time.perf_counter() - t0

    def call(b):
        soa = nsx.TcpHdrSoA(*[b.p.value + at[k] for k in range(8)])
        t0 = time.perf_counter()
        rc = L.nsx_tcp_build_host(ctypes.byref(soa), vp(b.p.value + at[12]), None, vp(b.p.value + at[13]),
                                  vp(b.p.value + at[8]), vp(b.p.value + at[11]), n, vp(b.p.value + at[14]),
                                  vp(b.p.value + at[10]), vp(b.p.value + at[15]), 0)
        assert rc == 0, rc
        return time.perf_counter() - t0

    res = {"one_shot": [], "reuse": []}
    kept = Pinned(total)
    for r in range(reps + 1):
        b = Pinned(total)
        tf = fill(b)
        tc = call(b)
        tfree = b.free()
        if r:
            res["one_shot"].append((b.t_alloc, tf, tc, tfree))
        tf = fill(kept)
        tc = call(kept)
        if r:
            res["reuse"].append((0.0, tf, tc, 0.0))
    # spot check the kept block's last build against the Go-faithful sender loop
    sel = np.arange(0, n, max(1, n // 16))
    img = kept.arr[at[14]:at[14] + n_out]
    raw = kept.arr[at[15]:at[15] + 2 * n].view(np.uint16)
    sdata = np.concatenate([data[i * payload:(i + 1) * payload] for i in sel])
    sfields = {k: v[sel] for k, v in fields.items()}
    want, wraw = O.c_go_tcp_build(sfields, sdata, np.arange(sel.size + 1, dtype=np.uint64) * np.uint64(payload),
                                  nsx.tcp_layout_host(np.arange(sel.size + 1, dtype=np.uint64) * np.uint64(payload)),
                                  pseudo[sel])
    w = int(out_off[1])
    assert np.array_equal(raw[sel], wraw)
    assert np.array_equal(np.concatenate([img[i * w:(i + 1) * w] for i in sel]), want)
    kept.free()
    return res


def summarise(name, n, seg, res):
    line = {"sequence": name, "segments": n, "bytes_per_segment": seg}
    for form, rows in res.items():
        a = np.array(rows) * 1e6
        med = {s: float(np.median(a[:, k])) for k, s in enumerate(("alloc_pinned", "fill", "call", "free_pinned"))}
        med["total"] = float(np.median(a.sum(1)))
        line[form] = {k: round(v, 1) for k, v in med.items()}
        line[form]["reps"] = len(rows)
    print(json.dumps(line), flush=True)
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps-small", type=int, default=300)
    ap.add_argument("--reps-large", type=int, default=3)
    a = ap.parse_args()
    lines = []
    for n, reps in ((64, a.reps_small), (1 << 20, a.reps_large)):
        lines.append(summarise("checksum: ChecksumSegments | PinnedBatch.Checksum", n, 1500,
                               seq_checksum(n, 1500, reps, "checksum")))
        lines.append(summarise("verify: VerifyDatagrams | PinnedBatch.Verify(4)", n, 1500,
                               seq_checksum(n, 1500, reps, "verify")))
        lines.append(summarise("build: BuildSegments | Sender.Build", n, 1480, seq_build(n, 1480, reps)))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "go_call_cost.json"), "w") as f:
        json.dump(lines, f, indent=1)


if __name__ == "__main__":
    main()
