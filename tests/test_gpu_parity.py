"""GPU parity: the gfx950 kernels (through the C ABI) against the oracle on the
same inputs — bit-exact, as integer work must be. Edge cases the reference's
arithmetic has (odd lengths, zero/0xFFFF sums, odd starts, empty segments,
end-of-allocation tails), every launch shape the per-call overrides of
include/nsx_tune.h allow, the SURVEY §8 f-rows (verify, pseudo-headers, TCP build,
IPv4 headers), the host batch path and re-entrancy. The golden fixtures and the
BASELINE configs at full size run first, in test_gpu_00_baseline.py."""
import numpy as np
import pytest

from _gpu import dev, host, mask_words, pseudo_headers, run_fixed, run_ragged, setup_gpu, torch, u16
from oracle import csum_oracle as O

import nsx  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu():
    setup_gpu()


# ------------------------------------------------------------------ edges

@pytest.mark.parametrize("seg_len", [0, 1, 2, 3, 4, 5, 15, 16, 17, 63, 64, 65, 1020, 1021, 1023, 1024, 1025,
                                     1499, 1500, 1501, 2044, 2045, 2047, 2048, 2049, 4093, 4096, 4097, 9000])
def test_fixed_lengths_strides_starts(seg_len):
    rng = np.random.default_rng(seg_len)
    for stride in sorted({seg_len, seg_len + 1, seg_len + 3, seg_len + 4, max(seg_len, 1) * 2 + 1}):
        for start in (0, 1, 2, 3, 5):
            n = int(rng.integers(1, 70))
            buf = rng.integers(0, 256, start + stride * n + seg_len + 8, dtype=np.uint8)
            partial = rng.integers(0, 1 << 20, n, dtype=np.uint32) if start % 2 else None
            got = run_fixed(buf, stride, seg_len, n, partial, start)
            want = O.c_batch(buf[start:], n, stride=stride, seg_len=seg_len, partial=partial)
            assert np.array_equal(got, want), (stride, start, n)


def test_special_sums():
    # all-zero → 0; all-0xFF → 0xFFFF; nonzero multiples of 0xFFFF → 0xFFFF
    L = 1500
    z = np.zeros(L * 4, np.uint8)
    assert run_fixed(z, L, L, 4).tolist() == [0] * 4
    f = np.full(L * 4, 0xFF, np.uint8)
    assert run_fixed(f, L, L, 4).tolist() == [0xFFFF] * 4
    m = np.zeros(L * 2, np.uint8)
    m[[0, 1, 2, 3]] = [0x00, 0x01, 0xFF, 0xFE]
    m[L + 700:L + 702] = 0xFF
    assert run_fixed(m, L, L, 2).tolist() == [0xFFFF, 0xFFFF]


def test_tail_at_end_of_allocation():
    """The batch's last byte is the tensor's last byte (no slack for 16-B loads)."""
    for total in (2 * 1024 * 1024, 4 * 1024 * 1024 + 4096, 6 * 1024 * 1024):
        for seg_len in (1497, 1498, 1499, 1500, 65535):
            n = total // seg_len
            t = torch.empty(total, dtype=torch.uint8, device="cuda")
            nsx.fill_splitmix64_dev(t, 0x1071)
            start = total - n * seg_len
            out = torch.empty(n, dtype=torch.int16, device="cuda")
            nsx.fixed_dev(t[start:], seg_len, seg_len, n, out=out)
            want = O.c_batch(host(t)[start:], n, stride=seg_len, seg_len=seg_len)
            assert np.array_equal(u16(out), want)
            offs = dev((np.arange(n + 1, dtype=np.uint64) * seg_len + start).view(np.int64))
            rout = torch.empty(n, dtype=torch.int16, device="cuda")
            nsx.ragged_dev(t, offs, out=rout)
            assert np.array_equal(u16(rout), want)


def test_ragged_dense_odd_starts_and_empties():
    rng = np.random.default_rng(99)
    lens = rng.integers(0, 5000, 3000).astype(np.uint64)
    lens[rng.integers(0, 3000, 100)] = 0
    lens[rng.integers(0, 3000, 20)] = rng.integers(60000, 70000, 20)
    for base_off in (0, 1, 3, 6):
        offs = np.zeros(lens.size + 1, np.uint64)
        offs[1:] = np.cumsum(lens)
        offs += np.uint64(base_off)
        buf = rng.integers(0, 256, int(offs[-1]), dtype=np.uint8)
        part = rng.integers(0, 1 << 31, lens.size, dtype=np.uint32)
        assert np.array_equal(run_ragged(buf, offs), O.c_batch(buf, lens.size, offsets=offs))
        assert np.array_equal(run_ragged(buf, offs, part), O.c_batch(buf, lens.size, offsets=offs, partial=part))


def test_zero_segments_is_noop():
    out = torch.full((4,), 7, dtype=torch.int16, device="cuda")
    nsx.fixed_dev(torch.zeros(16, dtype=torch.uint8, device="cuda"), 16, 16, 0, out=out)
    assert host(out).tolist() == [7] * 4


# ------------------------------------------------------------------ variants

FIXED_TUNES = [dict(segs_per_wave=s, blocks_per_cu=b, xcd_chunk=c) for s in (0, 1, 2, 4, 8) for b in (0, 1, 3, 8)
               for c in (0, -1, 3)]


def test_all_launch_shapes_bit_exact():
    """Every segments-per-task / grid / XCD-deal shape, each in auto, wave and block mode, over
    aligned short (config 2's pipelined kernel), unaligned short (edge-masked buffer kernel) and
    long (wave kernel) batches."""
    buf = O.c_splitmix64(0x1071, 1500 * 50001 + 64)
    d = dev(buf)
    want = {}
    for L, stride, n in ((1500, 1500, 50001), (1400, 1500, 50001), (700, 700, 9999), (1499, 1501, 30001),
                         (3000, 3001, 20000), (9000, 9000, 5000), (65536, 65536, 500)):
        want[(L, stride, n)] = O.c_batch(buf, n, stride=stride, seg_len=L)
    for t in FIXED_TUNES:
        for bm in (0, 1, 2):
            if bm == 2 and t["segs_per_wave"] not in (0, 8):
                continue  # block mode ignores the task shape
            tune = dict(t, block_mode=bm)
            for (L, stride, n), w in want.items():
                out = torch.empty(n, dtype=torch.int16, device="cuda")
                nsx.fixed_dev(d, stride, L, n, out=out, tune=tune)
                assert np.array_equal(u16(out), w), (tune, L, stride, n)


# Launch shapes of the ragged checksum: pipelined (rows 2/4/8) and plain (4/8/16) row batches; one boundary set
# per lane; runs of two sets forced (blocks_per_cu 8 allocates no LDS: results stored directly, else parked); the
# LDS forms (2 = the small-segment mode with parked results, 3 = four waves per block).
RAGGED_TUNES = [dict(kernel=k, rows=r, run_segs=rs, blocks_per_cu=b)
                for k, rows in ((0, (0, 4, 8)), (nsx.KERNEL_SCAN_PLAIN, (0, 4, 16))) for r in rows
                for rs in (0, 1, 16, 63) for b in (0, 1, 8)] + \
               [dict(segs_per_wave=1, run_segs=rs, blocks_per_cu=b) for rs in (0, 1, 16, 63) for b in (0, 1, 8)] + \
               [dict(segs_per_wave=5, run_segs=rs, blocks_per_cu=b) for rs in (0, 1, 16, 63) for b in (0, 1, 8)] + \
               [dict(segs_per_wave=sp, run_segs=rs, blocks_per_cu=b, kernel=k)
                for sp in (2, 3) for rs in (0, 1, 16, 63) for b in (0, 1, 8) for k in (0, nsx.KERNEL_SCAN_PLAIN)]


def test_ragged_small_segment_bench_workload_full_size():
    """Bench workload 15 at full size (8M ragged segments of 64-128 B, equal-count wave ranges, the LDS form): every
    raw sum equals the C oracle's (16 threads): the default small-segment mode (runs of 64 parked and written 8 KiB
    at a time), the four-wave LDS form, the streamed runs, and the default with partials."""
    import bench
    cfg = bench.WORKLOADS[15]
    w = bench.build_workload(cfg, 0, torch.device("cuda", 0))
    want = O.c_batch(host(w["buf"]), cfg["n"], offsets=w["offsets"], threads=16)
    for tune in (None, dict(segs_per_wave=3), dict(segs_per_wave=5), dict(segs_per_wave=1)):
        w["out"].zero_()
        w["step_for"](tune)()
        assert np.array_equal(u16(w["out"]), want), tune
    part = torch.randint(0, 1 << 31, (cfg["n"],), dtype=torch.int64, device="cuda").to(torch.int32)
    want_p = O.c_batch(host(w["buf"]), cfg["n"], offsets=w["offsets"], partial=host(part).view(np.uint32), threads=16)
    out = nsx.ragged_dev(w["buf"], w["d_offs"], partial=part, out=torch.empty_like(w["out"]))
    assert np.array_equal(u16(out), want_p)


def test_fixed_dealt_tasks_back_to_back_and_on_many_streams():
    """The aligned fixed-stride kernel deals its last eighth of tasks through each block's LDS ring (a fifth, dealer
    wave per block pulling from the stream's heads): the three default shapes (8 segments × 1
    row, 8 × 2, 4 × 4), batch sizes from just over the dealing threshold (64 tasks per block) to 1M segments, with
    and without partials, outputs 2 B past a 16 B boundary, launched back to back on one stream with no sync between
    them — interleaved with the static split (deal -1) and with receive-pass launches that deal from the same heads —
    then on 70 streams at once; every raw sum equals the oracle."""
    import ctypes
    import _rx
    rng = np.random.default_rng(0x8D)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    cases = []
    for L, n in ((1500, 1 << 20), (1500, 64 * 8 * cus + 7), (1000, 300_001), (3000, 200_003), (1500, 64 * 8 * cus - 8),
                 (3996, 150_001)):
        buf = O.c_splitmix64(0x8D + n + L, n * L + 4)
        part = rng.integers(0, 1 << 31, n, dtype=np.uint32)
        cases.append((dev(buf), L, n, dev(part.view(np.int32)), O.c_batch(buf, n, stride=L, seg_len=L, threads=16),
                      O.c_batch(buf, n, stride=L, seg_len=L, partial=part, threads=16)))
    rbuf, roffs, _ = _rx.batch(rng, 20_000, max_payload=1460)
    rx = (dev(rbuf), dev(roffs.view(np.int64)), O.c_rx_ipv4_tcp(rbuf, roffs)[0])

    def launch(k, tune=None, stream=None):
        d, L, n, p, _, _ = cases[k % len(cases)]
        with torch.cuda.stream(stream or torch.cuda.current_stream()):
            out = torch.empty(n + 1, dtype=torch.int16, device="cuda")[1:]
            nsx.fixed_dev(d, L, L, n, partial=p if k & 1 else None, out=out, tune=tune)
            mask = nsx.rx_ipv4_tcp_verify_dev(rx[0], rx[1])
        return k, out, mask

    def check(results):
        torch.cuda.synchronize()
        for k, out, mask in results:
            c = cases[k % len(cases)]
            assert np.array_equal(u16(out), c[5] if k & 1 else c[4]), k
            assert np.array_equal(host(mask).view(np.uint64), rx[2]), k

    check([launch(k, dict(deal=-1) if r == 1 else None) for r in range(3) for k in range(2 * len(cases))])
    torch.cuda.synchronize()
    hip = ctypes.CDLL("libamdhip64.so")
    handles = []
    for _ in range(70):
        h = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(h)) == 0
        handles.append(h)
    try:
        streams = [torch.cuda.ExternalStream(h.value) for h in handles]
        check([launch(i + r, None, streams[i]) for r in range(2) for i in range(len(streams))])
    finally:
        torch.cuda.synchronize()
        for h in handles:
            nsx.stream_release(h.value)
            hip.hipStreamDestroy(h)


def test_ragged_dealt_runs_back_to_back_and_on_many_streams():
    """The small-segment mode deals each launch's last runs from the stream's counters, shared with the receive pass
    and left at zero by every launch: checksum and batch-verify launches of 3 to 300k
    segments, with and without partials, back to back on one stream with no sync between them and interleaved with
    receive launches on the same counters (and packed-header launches), then on 70 HIP streams at once (past the 64
    counter sets a device gives out), all equal the oracle; a dealt run that does not follow the parked ones flushes
    them (outputs at odd offsets)."""
    import ctypes
    import _rx
    rng = np.random.default_rng(0x8B)
    cases = []
    for n in (300_001, 3, 64 * 700, 129, 100_000):
        lens = rng.integers(0, 160, n).astype(np.uint64)
        offs = np.zeros(n + 1, np.uint64)
        offs[1:] = np.cumsum(lens)
        offs += np.uint64(int(rng.integers(4)))
        buf = O.c_splitmix64(0x8B + n, int(offs[-1]) + 3)
        part = rng.integers(0, 1 << 31, n, dtype=np.uint32)
        cases.append((dev(buf), dev(offs.view(np.int64)), dev(part.view(np.int32)),
                      O.c_batch(buf, n, offsets=offs, threads=16), O.c_batch(buf, n, offsets=offs, partial=part, threads=16)))
    rbuf, roffs, _ = _rx.batch(rng, 50_000, max_payload=40)
    rx = (dev(rbuf), dev(roffs.view(np.int64)), O.c_rx_ipv4_tcp(rbuf, roffs)[0])
    # packed 20 B headers between them (IHL 5 everywhere, so every raw sum is the plain sum of the 20 bytes)
    nh = 300_001
    hbuf = rng.integers(0, 256, nh * 20 + 4, dtype=np.uint8)
    hbuf[0:nh * 20:20] = 0x45
    hdr = (dev(hbuf), O.c_batch(hbuf, nh, stride=20, seg_len=20, threads=16))

    def launch(k, stream=None):
        d, o, p, want, want_p = cases[k % len(cases)]
        n = o.numel() - 1
        with torch.cuda.stream(stream or torch.cuda.current_stream()):
            out = torch.empty(n + 1, dtype=torch.int16, device="cuda")[1:]  # 2 B past a 16 B boundary
            nsx.ragged_dev(d, o, partial=p if k & 1 else None, out=out)
            raw = torch.empty(n, dtype=torch.int16, device="cuda")
            ok = nsx.verify_ragged_dev(d, o, partial=p if k & 1 else None, raw=raw)
            mask = torch.empty((rx[1].numel() + 62) // 64, dtype=torch.int64, device="cuda")
            nsx.rx_ipv4_tcp_verify_dev(rx[0], rx[1], mask=mask)
            hraw = nsx.ipv4_hdr_csum_dev(hdr[0], 20, nh, mode=0)
        return k, out, raw, ok, mask, hraw

    def check(results):
        torch.cuda.synchronize()
        for k, out, raw, ok, mask, hraw in results:
            assert np.array_equal(u16(hraw), hdr[1]), k
            want = cases[k % len(cases)][4 if k & 1 else 3]
            assert np.array_equal(u16(out), want), k
            assert np.array_equal(u16(raw), want), k
            assert np.array_equal(host(ok).astype(bool), want == 0xFFFF), k
            assert np.array_equal(host(mask).view(np.uint64), rx[2]), k

    check([launch(k) for k in range(3 * len(cases))])
    torch.cuda.synchronize()
    hip = ctypes.CDLL("libamdhip64.so")
    handles = []
    for _ in range(70):
        h = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(h)) == 0
        handles.append(h)
    used0 = nsx.deal_sets_in_use()
    try:
        streams = [torch.cuda.ExternalStream(h.value) for h in handles]
        check([launch(i + r, streams[i]) for r in range(2) for i in range(len(streams))])
    finally:
        torch.cuda.synchronize()
        for h in handles:
            nsx.stream_release(h.value)  # the sets go back before the stream is destroyed
            hip.hipStreamDestroy(h)
    assert nsx.deal_sets_in_use() <= used0
    # a released set is given to the next new stream, not a fresh one: creating and destroying streams in a loop
    # does not use the 64 sets up
    for r in range(80):
        h = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(h)) == 0
        try:
            res = [launch(r, torch.cuda.ExternalStream(h.value))]
            check(res)
            assert nsx.deal_sets_in_use() <= used0 + 1
        finally:
            torch.cuda.synchronize()
            nsx.stream_release(h.value)
            hip.hipStreamDestroy(h)


def test_dealt_runs_on_hipStreamPerThread_from_concurrent_threads():
    """hipStreamPerThread (handle 2) is ONE handle value that names a different stream on every host thread, so
    launches from several threads on it run at the same time: sharing one deal-counter set between them would
    interleave their tickets. The library gives that handle no set (equal static
    shares, deal_heads in csum_kernels.hip). Four host threads each make 20 launches of the ragged checksum's
    small-segment mode and of the IPv4 receive pass's small-frame mode through the C ABI on hipStreamPerThread,
    concurrently, into their own outputs; every output equals the oracle, no set was given out for them, and fresh
    launches on the null stream and on a new stream afterwards equal the oracle too (no counter left non-zero)."""
    import ctypes
    import threading
    import _rx
    L = nsx.lib()
    hip = ctypes.CDLL("libamdhip64.so")
    per_thread = ctypes.c_void_p(2)  # hipStreamPerThread (hip_runtime_api.h)
    rng = np.random.default_rng(0x5A7)
    n = 200_001
    lens = rng.integers(0, 160, n).astype(np.uint64)  # mean < 128 B: the small-segment mode (dealt runs)
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    buf = O.c_splitmix64(0x5A7, int(offs[-1]) + 3)
    want = O.c_batch(buf, n, offsets=offs, threads=16)
    rbuf, roffs, _ = _rx.batch(rng, 120_000, max_payload=40)  # small frames: the two-wave LDS mode (dealt runs)
    rwant = O.c_rx_ipv4_tcp(rbuf, roffs)[0]
    d, o, rd, ro = dev(buf), dev(offs.view(np.int64)), dev(rbuf), dev(roffs.view(np.int64))
    nr = roffs.size - 1
    T, K = 4, 20
    outs = [[torch.full((n,), -1, dtype=torch.int16, device="cuda") for _ in range(K)] for _ in range(T)]
    masks = [[torch.full(((nr + 63) // 64,), -1, dtype=torch.int64, device="cuda") for _ in range(K)] for _ in range(T)]
    torch.cuda.synchronize()
    used0 = nsx.deal_sets_in_use()
    errs = []
    go = threading.Barrier(T)

    def worker(t):
        try:
            assert hip.hipSetDevice(0) == 0
            go.wait()
            for k in range(K):
                rc = L.nsx_csum_ragged_dev(ctypes.c_void_p(d.data_ptr()), ctypes.c_void_p(o.data_ptr()), n, None,
                                           ctypes.c_void_p(outs[t][k].data_ptr()), per_thread)
                assert rc == 0, rc
                rc = L.nsx_rx_ipv4_tcp_verify_dev(ctypes.c_void_p(rd.data_ptr()), ctypes.c_void_p(ro.data_ptr()), nr,
                                                  ctypes.c_void_p(masks[t][k].data_ptr()), None, None, per_thread)
                assert rc == 0, rc
            assert hip.hipStreamSynchronize(per_thread) == 0
        except BaseException as e:  # noqa: BLE001 — reported below
            errs.append((t, e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    torch.cuda.synchronize()
    assert not errs, errs
    assert nsx.deal_sets_in_use() == used0  # hipStreamPerThread took no set
    for t in range(T):
        for k in range(K):
            assert np.array_equal(u16(outs[t][k]), want), (t, k)
            assert np.array_equal(host(masks[t][k]).view(np.uint64), rwant), (t, k)
    # afterwards: the null stream and a new stream (each with its own set) still get exact results
    null = torch.cuda.default_stream()
    s = torch.cuda.Stream()
    for st in (null, s, null):
        out = nsx.ragged_dev(d, o, out=torch.empty(n, dtype=torch.int16, device="cuda"), stream=st)
        mask = nsx.rx_ipv4_tcp_verify_dev(rd, ro, stream=st)
        st.synchronize()
        assert np.array_equal(u16(out), want)
        assert np.array_equal(host(mask).view(np.uint64), rwant)
    # and the A/B switch: equal static shares on a stream that has a set
    out = nsx.ragged_dev(d, o, tune=dict(deal=-1))
    assert np.array_equal(u16(out), want)
    assert np.array_equal(host(nsx.rx_ipv4_tcp_verify_dev(rd, ro, tune=dict(deal=-1))).view(np.uint64), rwant)


@pytest.mark.parametrize("n", [1, 126, 252, 253, 30_001, 400_003])
def test_ragged_small_segments_every_form(n):
    """Segments of 0-200 B (mean ~100): the small-segment mode (2), the four-wave LDS form (3), the streamed runs
    of one and of two 63-segment sets (1, 5) and the automatic choice equal the oracle, with
    and without partials.
    block_mode=1 keeps even the smallest batches on the scan kernel, and short runs (run_segs 1, 16) at one block
    per CU make every wave stream many runs, so both sets, partial last sets and set-to-set frame ends run
    (ADVICE r2)."""
    rng = np.random.default_rng(n + 42)
    lens = rng.integers(0, 201, n).astype(np.uint64)
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    offs += np.uint64(3)
    buf = O.c_splitmix64(0x42, int(offs[-1]) + 3)
    part = rng.integers(0, 1 << 31, n, dtype=np.uint32)
    want = O.c_batch(buf, n, offsets=offs, threads=16)
    want_p = O.c_batch(buf, n, offsets=offs, partial=part, threads=16)
    d, o, p = dev(buf), dev(offs.view(np.int64)), dev(part.view(np.int32))
    tunes = [None, dict(segs_per_wave=1), dict(segs_per_wave=5), dict(segs_per_wave=2), dict(segs_per_wave=3)]
    tunes += [dict(block_mode=1, blocks_per_cu=1, run_segs=rs, **sp)
              for rs in (0, 1, 16) for sp in ({}, dict(segs_per_wave=1), dict(segs_per_wave=5), dict(segs_per_wave=2),
                                              dict(segs_per_wave=3))]
    for tune in tunes:
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        nsx.ragged_dev(d, o, out=out, tune=tune)
        assert np.array_equal(u16(out), want), tune
        nsx.ragged_dev(d, o, partial=p, out=out, tune=tune)
        assert np.array_equal(u16(out), want_p), tune


@pytest.mark.parametrize("shift", [0, 1, 3, 7])
@pytest.mark.parametrize("mix", ["small", "mid", "wide_runs"])
def test_ragged_parked_results_any_output_alignment(mix, shift):
    """Parked results (ResultPark) go out in 16 B blocks aligned to the output buffer, with
    the partial blocks at either end of a flush written result by result: outputs starting 0-7 results past a
    16 B boundary, inside a sentinel-filled buffer, receive exactly the oracle's sums and nothing outside them is
    written. Mixes: 64-128 B (the small-segment mode), 0-400 B (streamed runs of one and two sets), and segments of
    0-200 B with scattered 20-60 KB ones (LDS runs interrupted by streamed ones: flushes mid-range)."""
    rng = np.random.default_rng(900 + shift)
    n = 300_003
    lens = {"small": rng.integers(64, 129, n), "mid": rng.integers(0, 401, n),
            "wide_runs": rng.integers(0, 201, n)}[mix].astype(np.uint64)
    if mix == "wide_runs":
        lens[rng.integers(0, n, 400)] = rng.integers(20_000, 60_000, 400).astype(np.uint64)
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    offs += np.uint64(1)
    buf = O.c_splitmix64(0x5A + shift, int(offs[-1]) + 3)
    part = rng.integers(0, 1 << 31, n, dtype=np.uint32)
    want = O.c_batch(buf, n, offsets=offs, threads=16)
    want_p = O.c_batch(buf, n, offsets=offs, partial=part, threads=16)
    d, o, p = dev(buf), dev(offs.view(np.int64)), dev(part.view(np.int32))
    big = torch.empty(n + 64, dtype=torch.int16, device="cuda")
    assert big.data_ptr() % 16 == 0
    for tune in (None, dict(segs_per_wave=2), dict(segs_per_wave=3), dict(segs_per_wave=5),
                 dict(segs_per_wave=1), dict(segs_per_wave=5, blocks_per_cu=3), dict(segs_per_wave=5, run_segs=16)):
        for pt, w in ((None, want), (p, want_p)):
            big.fill_(0x5A5A)
            nsx.ragged_dev(d, o, partial=pt, out=big[shift:shift + n], tune=tune)
            got = u16(big)
            assert np.array_equal(got[shift:shift + n], w), (tune, pt is None)
            assert (got[:shift] == 0x5A5A).all() and (got[shift + n:] == 0x5A5A).all(), tune
    # the batch verify parks its 1-byte verdicts (16 per block): ok outputs 0-15 bytes past a 16 B boundary, with
    # and without raw sums beside them
    # partials that make about half the segments verify (the sum plus 0xFFFF - raw is 0xFFFF), so both verdicts occur
    part_v = np.where(rng.random(n) < 0.5, (0xFFFF - want.astype(np.uint32)), part).astype(np.uint32)
    want_v = O.c_batch(buf, n, offsets=offs, partial=part_v, threads=16)
    assert 0.3 < (want_v == 0xFFFF).mean() < 0.7
    pv = dev(part_v.view(np.int32))
    okb = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    for tune in (None, dict(segs_per_wave=2), dict(segs_per_wave=3), dict(segs_per_wave=5), dict(segs_per_wave=1)):
        for oshift in (0, shift, 9, 15):
            for with_raw in (False, True):
                okb.fill_(0xA5)
                big.fill_(0x5A5A)
                nsx.verify_ragged_dev(d, o, partial=pv, raw=big[shift:shift + n] if with_raw else None, tune=tune,
                                      ok=okb[oshift:oshift + n])
                gok = host(okb)
                assert np.array_equal(gok[oshift:oshift + n].astype(bool), want_v == 0xFFFF), (tune, oshift)
                assert set(np.unique(gok[oshift:oshift + n])) <= {0, 1}, (tune, oshift)
                assert (gok[:oshift] == 0xA5).all() and (gok[oshift + n:] == 0xA5).all(), (tune, oshift)
                if with_raw:
                    assert np.array_equal(u16(big)[shift:shift + n], want_v), (tune, oshift)


def test_ragged_launch_shapes_bit_exact():
    rng = np.random.default_rng(1234)
    lens = rng.integers(0, 9001, 20000).astype(np.uint64)
    lens[rng.integers(0, 20000, 300)] = 0
    lens[rng.integers(0, 20000, 40)] = rng.integers(1, 4, 40)
    lens[rng.integers(0, 20000, 10)] = rng.integers(100000, 300000, 10)
    offs = np.zeros(lens.size + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    offs += np.uint64(5)
    buf = O.c_splitmix64(0x1072, int(offs[-1]) + 3)
    part = rng.integers(0, 1 << 31, lens.size, dtype=np.uint32)
    want = O.c_batch(buf, lens.size, offsets=offs)
    want_p = O.c_batch(buf, lens.size, offsets=offs, partial=part)
    d, o, p = dev(buf), dev(offs.view(np.int64)), dev(part.view(np.int32))
    for t in RAGGED_TUNES + [dict(block_mode=2)]:
        tune = dict(t, block_mode=t.get("block_mode", 1))
        out = torch.empty(lens.size, dtype=torch.int16, device="cuda")
        nsx.ragged_dev(d, o, out=out, tune=tune)
        assert np.array_equal(u16(out), want), tune
        nsx.ragged_dev(d, o, partial=p, out=out, tune=tune)
        assert np.array_equal(u16(out), want_p), tune
        okv = host(nsx.verify_ragged_dev(d, o, partial=p, tune=tune))
        assert np.array_equal(okv.astype(bool), want_p == 0xFFFF), tune


def test_ragged_byte_balanced_partition_edges():
    """Byte-balanced wave ranges (found by an in-kernel 64-ary search over the offsets):
    skewed, sorted, all-empty and tiny batches, more waves than segments."""
    rng = np.random.default_rng(77)
    cases = {
        "sorted": np.sort(rng.integers(0, 20000, 6000)).astype(np.uint64),
        "one_giant": np.concatenate([np.full(3000, 3, np.uint64), [2_000_000], np.full(3000, 70, np.uint64)]),
        "empties_at_ends": np.concatenate([np.zeros(1500, np.uint64), rng.integers(1, 3000, 2000).astype(np.uint64),
                                           np.zeros(1500, np.uint64)]),
        "all_empty": np.zeros(4000, np.uint64),
        "few": rng.integers(0, 5000, 1030).astype(np.uint64),
        # large skewed batches on the default grid (round 5): every wave's byte slice far from its equal-count
        # share, and a dealt pool of large units behind a long run of empties
        "sorted_big": np.sort(rng.integers(0, 3000, 300_000)).astype(np.uint64),
        "empties_then_big": np.concatenate([np.zeros(200_000, np.uint64),
                                            rng.integers(500, 9000, 60_000).astype(np.uint64)]),
    }
    for name, lens in cases.items():
        offs = np.zeros(lens.size + 1, np.uint64)
        offs[1:] = np.cumsum(lens)
        offs += np.uint64(3)
        buf = O.c_splitmix64(0x1099, int(offs[-1]) + 8)
        want = O.c_batch(buf, lens.size, offsets=offs, threads=16)
        d, o = dev(buf), dev(offs.view(np.int64))
        for tune in [None] + [dict(blocks_per_cu=b, run_segs=rs, block_mode=1) for b in (1, 8) for rs in (1, 16, 63)]:
            out = torch.empty(lens.size, dtype=torch.int16, device="cuda")
            nsx.ragged_dev(d, o, out=out, tune=tune)
            assert np.array_equal(u16(out), want), (name, tune)


# ------------------------------------------------------------------ verify / pseudo-header

def test_pseudo_ipv4_partial_and_verify_roundtrip():
    rng = np.random.default_rng(5)
    n = 4000
    lens = rng.integers(20, 1500, n).astype(np.uint64)
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    buf = rng.integers(0, 256, int(offs[-1]), dtype=np.uint8)
    for i in range(n):  # zero each segment's checksum field (tcp.go:68 sender rule)
        buf[int(offs[i]) + 16:int(offs[i]) + 18] = 0
    src = rng.integers(0, 256, 4 * n, dtype=np.uint8)
    dst = rng.integers(0, 256, 4 * n, dtype=np.uint8)
    part = nsx.pseudo_ipv4_partial_dev(dev(src), dev(dst), dev(lens.astype(np.uint32).view(np.int32)), 6)
    part_h = host(part.view(torch.int32)).view(np.uint32)
    for i in range(0, n, 97):
        ph = O.ipv4_pseudo_header(src[4 * i:4 * i + 4].tobytes(), dst[4 * i:4 * i + 4].tobytes(), 6, int(lens[i]))
        assert O.fold(int(part_h[i])) == O.fold(O.be_word_sum(ph))
    d_buf, d_off = dev(buf), dev(offs.view(np.int64))
    raw = torch.empty(n, dtype=torch.int16, device="cuda")
    nsx.ragged_dev(d_buf, d_off, partial=part, out=raw)
    raw_h = u16(raw)
    for i in range(0, n, 89):
        ph = O.ipv4_pseudo_header(src[4 * i:4 * i + 4].tobytes(), dst[4 * i:4 * i + 4].tobytes(), 6, int(lens[i]))
        assert raw_h[i] == O.go_checksum(ph, buf[int(offs[i]):int(offs[i + 1])].tobytes())
    # sender: store ^raw at bytes 16-17 (tcp.go:110); receiver: verify == 0xFFFF (tcp.go:70)
    fld = (~raw_h) & 0xFFFF
    for i in range(n):
        buf[int(offs[i]) + 16] = fld[i] >> 8
        buf[int(offs[i]) + 17] = fld[i] & 0xFF
    d_buf = dev(buf)
    ok = nsx.verify_ragged_dev(d_buf, d_off, partial=part)
    assert host(ok).all()
    buf[int(offs[7]) + 30] ^= 0x01
    ok = nsx.verify_ragged_dev(dev(buf), d_off, partial=part)
    okh = host(ok)
    assert not okh[7] and okh.sum() == n - 1


def test_pseudo_ipv6_partial_matches_oracle():
    rng = np.random.default_rng(6)
    n = 5000
    src = rng.integers(0, 256, 16 * n + 1, dtype=np.uint8)
    dst = rng.integers(0, 256, 16 * n + 1, dtype=np.uint8)
    src[:32] = 0xFF  # saturating words
    lens = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    lens[:3] = [0, 0xFFFFFFFF, 65536]
    d_len = dev(lens.view(np.int32))
    for off in (0, 1):  # 4-aligned (dwordx4 path) and misaligned address arrays (byte path)
        d_src, d_dst = dev(src)[off:off + 16 * n], dev(dst)[off:off + 16 * n]
        part = host(nsx.pseudo_ipv6_partial_dev(d_src, d_dst, d_len, 6)).view(np.uint32)
        for i in list(range(0, n, 41)) + [0, 1, 2, n - 1]:
            ph = O.ipv6_pseudo_header(src[off + 16 * i:off + 16 * i + 16].tobytes(),
                                      dst[off + 16 * i:off + 16 * i + 16].tobytes(), 6, int(lens[i]))
            assert int(part[i]) == O.be_word_sum(ph), (off, i)


def test_ipv6_pseudo_partial_drives_fixed_checksum():
    """IPv6 pseudo-header partials into the fixed-stride path == oracle over pseudo ‖ segment."""
    rng = np.random.default_rng(61)
    n, L = 3000, 1500
    buf = rng.integers(0, 256, n * L, dtype=np.uint8)
    src = rng.integers(0, 256, 16 * n, dtype=np.uint8)
    dst = rng.integers(0, 256, 16 * n, dtype=np.uint8)
    lens = np.full(n, L, np.uint32)
    part = nsx.pseudo_ipv6_partial_dev(dev(src), dev(dst), dev(lens.view(np.int32)), 6)
    raw = u16(nsx.fixed_dev(dev(buf), L, L, n, partial=part))
    for i in range(0, n, 37):
        ph = O.ipv6_pseudo_header(src[16 * i:16 * i + 16].tobytes(), dst[16 * i:16 * i + 16].tobytes(), 6, L)
        assert raw[i] == O.go_checksum(ph, buf[i * L:(i + 1) * L].tobytes()), i


@pytest.mark.parametrize("n", [1, 63, 64, 65, 1000, 100_003])
def test_verify_mask_matches_raw(n):
    rng = np.random.default_rng(n)
    raw = rng.integers(0, 1 << 16, n, dtype=np.uint64).astype(np.uint16)
    raw[rng.random(n) < 0.5] = 0xFFFF
    raw[0] = 0xFFFF
    mask = host(nsx.verify_mask_dev(dev(raw.view(np.int16)))).view(np.uint64)
    assert mask.size == (n + 63) // 64
    bits = np.unpackbits(mask.view(np.uint8), bitorder="little")
    want = np.zeros(mask.size * 64, np.uint8)
    want[:n] = raw == 0xFFFF
    assert np.array_equal(bits, want)


# ------------------------------------------------------------------ host batch path

def test_host_batch_cache_grows_and_releases():
    """Host batch calls reuse per-device buffers: growing, shrinking and mixed
    fixed/ragged/partial calls stay exact, also after nsx_host_cache_release."""
    rng = np.random.default_rng(81)
    L = 1500
    for rel in (False, True, False):
        for n in (64, 1, 5000, 64, 100_000, 3):
            buf = rng.integers(0, 256, n * L, dtype=np.uint8)
            part = rng.integers(0, 1 << 20, n, dtype=np.uint64).astype(np.uint32)
            got = nsx.fixed_host(buf, L, L, n, partial=part)
            want = O.c_batch(buf, n, stride=L, seg_len=L, partial=part)
            assert np.array_equal(got, want), n
            lens = rng.integers(0, 3000, n).astype(np.uint64)
            offs = np.zeros(n + 1, np.uint64)
            offs[1:] = np.cumsum(lens)
            rb = rng.integers(0, 256, int(offs[-1]) + 1, dtype=np.uint8)
            assert np.array_equal(nsx.ragged_host(rb, offs), O.c_batch(rb, n, offsets=offs)), n
        if rel:
            assert nsx.lib().nsx_host_cache_release() == 0


def test_host_batch_paths_pageable_and_pinned():
    rng = np.random.default_rng(8)
    n, L = 100_003, 1500
    buf = O.c_splitmix64(0x1071, n * L)
    part = rng.integers(0, 1 << 20, n, dtype=np.uint32)
    want = O.c_batch(buf, n, stride=L, seg_len=L, partial=part)
    assert np.array_equal(nsx.fixed_host(buf, L, L, n, part), want)
    pin = nsx.PinnedBuffer(buf.nbytes)
    pin.array[:] = buf
    assert np.array_equal(nsx.fixed_host(pin.array, L, L, n, part), want)
    lens = rng.integers(64, 9001, 20000).astype(np.uint64)
    offs = np.zeros(lens.size + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    rbuf = O.c_splitmix64(0x1072, int(offs[-1]))
    assert np.array_equal(nsx.ragged_host(rbuf, offs), O.c_batch(rbuf, lens.size, offsets=offs))
    pin.free()


@pytest.mark.parametrize("shards", [2, 3, 8])
def test_host_batch_sharded_threads_on_one_device(shards):
    """The multi-GPU host path's shard-and-stitch logic (run_sharded: contiguous shards, byte-balanced
    for ragged batches, one host thread + its own streams and staging per shard) on the one GPU:
    nsx_tune.shards_per_device = K splits the batch into K shards on device 0. Fixed and ragged
    host batches, pageable and with partials, against the oracle; more shards than segments too.
    (The host path starts in transport buffers: transport/pipe/pipe.go:73-124.)"""
    rng = np.random.default_rng(0x5A + shards)
    tune = dict(shards_per_device=shards)
    L = 1500
    for n in (1, shards - 1 or 1, 5000, 70_001):
        buf = rng.integers(0, 256, n * L + 3, dtype=np.uint8)
        part = rng.integers(0, 1 << 20, n, dtype=np.uint64).astype(np.uint32)
        got = nsx.fixed_host(buf[3:], L, L, n, partial=part, tune=tune)
        assert np.array_equal(got, O.c_batch(buf[3:], n, stride=L, seg_len=L, partial=part)), (shards, n)
        lens = rng.integers(0, 9001, n).astype(np.uint64)
        offs = np.zeros(n + 1, np.uint64)
        offs[1:] = np.cumsum(lens)
        offs += np.uint64(1)
        rb = rng.integers(0, 256, int(offs[-1]) + 2, dtype=np.uint8)
        assert np.array_equal(nsx.ragged_host(rb, offs, partial=part, tune=tune),
                              O.c_batch(rb, n, offsets=offs, partial=part)), (shards, n)


def test_host_batch_more_gpus_than_present_is_enodev():
    """num_gpus > device count: NSX_ENODEV, nothing computed, the caller's current device unchanged."""
    before = torch.cuda.current_device()
    buf = np.zeros(3000, np.uint8)
    with pytest.raises(nsx.NsxError) as e:
        nsx.fixed_host(buf, 1500, 1500, 2, num_gpus=nsx.device_count() + 1)
    assert e.value.code == nsx.NSX_ENODEV
    with pytest.raises(nsx.NsxError) as e:
        nsx.ragged_host(buf, np.array([0, 1000, 3000], np.uint64), num_gpus=nsx.device_count() + 1)
    assert e.value.code == nsx.NSX_ENODEV
    assert torch.cuda.current_device() == before
    assert np.array_equal(nsx.fixed_host(buf, 1500, 1500, 2, num_gpus=nsx.device_count()), [0, 0])


def _host_build_case(rng, n, with_opts, lead=7):
    """Host-resident sender batch: payloads of 0-1600 B (every 97th a 8940 B jumbo payload) packed behind `lead`
    bytes, random header fields, every third segment (with_opts) carrying one of _OPT_SETS' option lists, and each
    segment's own IPv4 pseudo-header (TCP length = its wire length). Returns (fields, data, data_off, opts,
    opt_off, pseudo, partials)."""
    lens = rng.integers(0, 1601, n).astype(np.uint64)
    lens[::97] = 8940
    lens[:3] = [0, 1, 1480][:n]
    data = rng.integers(0, 256, lead + int(lens.sum()) + 8, dtype=np.uint8)
    data_off = np.zeros(n + 1, np.uint64)
    data_off[1:] = np.cumsum(lens)
    data_off += np.uint64(lead)
    fields = {k: rng.integers(0, 1 << (8 * np.dtype(dt).itemsize), n, dtype=np.uint64).astype(dt)
              for k, dt in zip(O.TCP_FIELDS, O.TCP_FIELD_DTYPES)}
    opts = opt_off = None
    olen = np.zeros(n, np.uint64)
    if with_opts:
        keys = sorted(_OPT_SETS)
        rb = lambda k: rng.integers(0, 256, k, dtype=np.uint8).tobytes()  # noqa: E731
        ob = [b"".join(o.bytes() for o in _OPT_SETS[keys[i % len(keys)]](rb)) if i % 3 == 1 else b""
              for i in range(n)]
        olen = np.array([len(b) for b in ob], np.uint64)
        opts = np.frombuffer(b"\x77" + b"".join(ob) + b"\x77", np.uint8)
        opt_off = np.zeros(n + 1, np.uint64)
        opt_off[1:] = np.cumsum(olen)
        opt_off += np.uint64(1)
    fields["offset"] = ((20 + olen + 3) // 4).astype(np.uint8)  # computeOffset (tcp.go:59-66)
    wire = 20 + olen + np.where(olen > 0, (20 + olen) % 4, 0) + lens
    pseudo = np.concatenate([rng.integers(0, 256, (n, 8), dtype=np.uint8), np.zeros((n, 1), np.uint8),
                             np.full((n, 1), 6, np.uint8), (wire >> np.uint64(8)).astype(np.uint8)[:, None] & 0xFF,
                             (wire & np.uint64(0xFF)).astype(np.uint8)[:, None]], 1)
    pw = pseudo.reshape(n, 6, 2).astype(np.uint32)
    part = ((pw[..., 0] << 8) | pw[..., 1]).sum(1).astype(np.uint32)
    return fields, data, data_off, opts, opt_off, pseudo, part


@pytest.mark.parametrize("opts", [False, True])
@pytest.mark.parametrize("mem", ["pageable", "pinned"])
@pytest.mark.parametrize("shards", [1, 2, 3])
def test_tcp_build_host_every_segment(shards, mem, opts):
    """nsx_tcp_build_host (the sender pass from and to host memory, as a Go transport's send loop
    would call it — tcp.go:98-128, :110, :68-71 — before writing the images into its pipe, transport/pipe/
    pipe.go:92-124): 100K mixed-size segments (~86 MB of images: two 64 MiB chunks on one shard), with and without
    options, each over its own IPv4 pseudo-header partial, payloads and images in pageable or pinned memory, K = 1, 2
    or 3 shards (host threads, streams, staging) on the device. Every image byte and every raw sum against the
    Go-faithful sender loop (O.c_go_tcp_build_mt); the padding bytes after each image are zero."""
    rng = np.random.default_rng(0xB0 + shards * 4 + (mem == "pinned") * 2 + opts)
    n = 100_003
    fields, data, data_off, ob, oo, pseudo, part = _host_build_case(rng, n, opts)
    out_off = nsx.tcp_layout_host(data_off, oo)
    want, wraw = O.c_go_tcp_build_mt(fields, data, data_off, out_off, pseudo, opts=ob, opt_off=oo)
    tune = dict(shards_per_device=shards)
    if mem == "pinned":
        dp, op = nsx.PinnedBuffer(data.nbytes), nsx.PinnedBuffer(int(out_off[-1]))
        dp.array[:] = data
        op.array[:] = 0xAB
        got, raw = nsx.tcp_build_host(fields, dp.array, data_off, out_off=out_off, opts=ob, opt_off=oo, partial=part,
                                      out=op.array, tune=tune)
        got = got.copy()
        dp.free()
        op.free()
    else:
        got, raw = nsx.tcp_build_host(fields, data, data_off, out_off=out_off, opts=ob, opt_off=oo, partial=part,
                                      out=np.full(int(out_off[-1]), 0xAB, np.uint8), tune=tune)
    bad = np.nonzero(raw != wraw)[0]
    assert bad.size == 0, (bad[:8], raw[bad[:8]], wraw[bad[:8]])
    if not np.array_equal(got, want):
        d = np.nonzero(got != want)[0]
        seg = int(np.searchsorted(out_off, d[0], side="right")) - 1
        raise AssertionError(f"{d.size} bytes differ, first at {d[0]} (segment {seg}, byte {d[0] - int(out_off[seg])})")


def test_tcp_build_host_gaps_offset_none_no_raw_and_the_device_call():
    """Image slots longer than image + padding: the caller's bytes between them stay as they were (the device call's
    rule, test_tcp_build_output_bases_and_gaps); `offset` NULL computes byte 12 on the device (computeOffset,
    tcp.go:59-66); h_raw NULL writes no sums; and the host call's images and sums equal nsx_tcp_build_dev's over the
    same inputs in HBM, in one chunk and over many (segments past 64 MiB of images, shards 2)."""
    rng = np.random.default_rng(0xB7)
    n = 30_011
    fields, data, data_off, ob, oo, pseudo, part = _host_build_case(rng, n, True, lead=0)
    lay = nsx.tcp_layout_host(data_off, oo)
    gap = 4 * rng.integers(0, 9, n).astype(np.uint64) * (rng.random(n) < 0.3)
    out_off = np.zeros(n + 1, np.uint64)
    out_off[1:] = np.cumsum(np.diff(lay) + gap)
    want, wraw = O.c_go_tcp_build_mt(fields, data, data_off, out_off, pseudo, opts=ob, opt_off=oo)
    sentinel = np.full(int(out_off[-1]), 0xAB, np.uint8)
    exp = sentinel.copy()
    slot = np.diff(lay)
    for i in range(n):
        o = int(out_off[i])
        exp[o:o + int(slot[i])] = want[o:o + int(slot[i])]
    got, raw = nsx.tcp_build_host(dict(fields, offset=None), data, data_off, out_off=out_off, opts=ob, opt_off=oo,
                                  partial=part, out=sentinel.copy(), want_raw=True)
    assert np.array_equal(raw, wraw)
    assert np.array_equal(got, exp)
    got2, raw2 = nsx.tcp_build_host(fields, data, data_off, out_off=out_off, opts=ob, opt_off=oo, partial=part,
                                    out=sentinel.copy(), want_raw=False)
    assert raw2 is None and np.array_equal(got2, exp)
    # the device call over the same inputs in HBM (packed layout, no gaps)
    img_h, raw_h = nsx.tcp_build_host(fields, data, data_off, opts=ob, opt_off=oo, partial=part,
                                      tune=dict(shards_per_device=2))
    dt = {np.uint16: np.int16, np.uint32: np.int32, np.uint8: np.uint8}
    f = {k: dev(v.view(dt[v.dtype.type])) for k, v in fields.items()}
    out = torch.zeros(int(lay[-1]), dtype=torch.uint8, device="cuda")
    rawd = torch.empty(n, dtype=torch.int16, device="cuda")
    nsx.tcp_build_dev(f, dev(data), dev(data_off.view(np.int64)), out, dev(lay.view(np.int64)), opts=dev(ob),
                      opt_off=dev(oo.view(np.int64)), partial=dev(part.view(np.int32)), raw=rawd)
    assert np.array_equal(host(out), img_h) and np.array_equal(u16(rawd), raw_h)
    # many chunks: 60K workload-6-shaped segments (~90 MB of images), two shards
    m, P, W = 60_000, 1480, 1500
    fw = {k: rng.integers(0, 1 << (8 * np.dtype(dt).itemsize), m, dtype=np.uint64).astype(dt)
          for k, dt in zip(O.TCP_FIELDS, O.TCP_FIELD_DTYPES)}
    fw["offset"] = np.full(m, 5, np.uint8)
    dw = O.c_splitmix64(0x1074, m * P)
    doff = np.arange(m + 1, dtype=np.uint64) * np.uint64(P)
    ps = np.concatenate([rng.integers(0, 256, (m, 8), dtype=np.uint8),
                         np.tile(np.array([0, 6, W >> 8, W & 0xFF], np.uint8), (m, 1))], 1)
    pw = ps.reshape(m, 6, 2).astype(np.uint32)
    pp = ((pw[..., 0] << 8) | pw[..., 1]).sum(1).astype(np.uint32)
    wwant, wwraw = O.c_go_tcp_build_mt(fw, dw, doff, np.arange(m + 1, dtype=np.uint64) * np.uint64(W), ps)
    gw, rw = nsx.tcp_build_host(fw, dw, doff, partial=pp, tune=dict(shards_per_device=2))
    assert np.array_equal(rw, wwraw) and np.array_equal(gw, wwant)


def test_tcp_build_host_more_gpus_than_present_is_enodev():
    """num_gpus > device count: NSX_ENODEV before anything is copied, the caller's device unchanged."""
    before = torch.cuda.current_device()
    rng = np.random.default_rng(3)
    fields, data, data_off, _, _, _, _ = _host_build_case(rng, 5, False)
    with pytest.raises(nsx.NsxError) as e:
        nsx.tcp_build_host(fields, data, data_off, num_gpus=nsx.device_count() + 1)
    assert e.value.code == nsx.NSX_ENODEV
    assert torch.cuda.current_device() == before


# ------------------------------------------------------------------ large batches

@pytest.mark.parametrize("L", [1500, 1501])
@pytest.mark.parametrize("window", [1_000_003, 3000, 1500, 1])
def test_fixed_back_to_back_windows(window, L):
    """nsx_tune.window_bytes splits the fixed short-segment path into back-to-back launches
    (DESIGN.md §7 step 21): window sizes that cut the batch unevenly, down to one segment
    per launch, aligned and odd strides, with per-segment partials, against the oracle; the
    library's launch count says how many launches that is."""
    rng = np.random.default_rng(0x21 + window)
    n = 2048 if window <= 3000 else 6001
    buf = rng.integers(0, 256, n * L, dtype=np.uint8)
    part = rng.integers(0, 1 << 20, n, dtype=np.uint32)
    want = O.c_batch(buf, n, stride=L, seg_len=L, partial=part)
    tune = dict(window_bytes=window)
    assert np.array_equal(run_fixed(buf, L, L, n, part, tune=tune), want)
    assert nsx.fixed_launch_count(L, L, n, tune) == -(-n // max(1, window // L))


@pytest.mark.parametrize("window", [0, 1, 3000, -1])
def test_fixed_stride_zero_aliases_first_segment(window):
    """stride 0 (every segment aliases the first — allowed by nsx_csum_fixed_dev) with and without
    windows: one launch, every result equal (window_bytes / stride divided by zero)."""
    rng = np.random.default_rng(7)
    for L in (1500, 1497, 64, 8):
        buf = rng.integers(0, 256, L + 8, dtype=np.uint8)
        n = 5000
        got = run_fixed(buf, 0, L, n, tune=dict(window_bytes=window))
        assert (got == O.c_go_checksum(b"", buf[:L].tobytes())).all(), (L, window)
        assert nsx.fixed_launch_count(0, L, n, dict(window_bytes=window)) == 1


def test_fixed_batch_past_the_launch_chunk():
    """n > 2^28 segments: nsx_csum_fixed_dev splits the batch into launches of 2^28
    (buffer descriptors address < 2^31 bytes of results); segments either side of the
    split, a stride sample and the last one against the oracle, and all of them
    against a grid-stride launch of the same kernel."""
    n, L, seed = (1 << 28) + 4099, 4, 0x28
    t = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    nsx.fill_splitmix64_dev(t, seed)
    got = u16(nsx.fixed_dev(t, L, L, n, out=torch.empty(n, dtype=torch.int16, device="cuda")))
    idx = sorted(set(range(0, n, 1_000_003)) | set(range((1 << 28) - 5, (1 << 28) + 5)) | {n - 1})
    for i in idx:
        assert got[i] == O.c_fold_checksum(b"", O.c_splitmix64(seed, L, i * L).tobytes()), i
    alt = u16(nsx.fixed_dev(t, L, L, n, out=torch.empty(n, dtype=torch.int16, device="cuda"),
                            tune=dict(xcd_chunk=-1, segs_per_wave=2, blocks_per_cu=8)))
    assert np.array_equal(alt, got)


def test_ragged_batch_past_the_launch_chunk():
    """n > 2^27 ragged segments (0-16 B, odd starts): nsx_csum_ragged_dev splits the
    batch into launches of 2^27; segments either side of the split and a sample
    against the oracle."""
    n, seed = (1 << 27) + 999, 0x27
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 17, n).astype(np.uint64)
    offs = np.zeros(n + 1, np.uint64)
    np.cumsum(lens, out=offs[1:])
    t = torch.empty(int(offs[-1]) + 4, dtype=torch.uint8, device="cuda")
    nsx.fill_splitmix64_dev(t, seed)
    got = u16(nsx.ragged_dev(t, dev(offs.view(np.int64)), out=torch.empty(n, dtype=torch.int16, device="cuda")))
    idx = sorted(set(range(0, n, 999_983)) | set(range((1 << 27) - 5, (1 << 27) + 5)) | {n - 1})
    for i in idx:
        o, ln = int(offs[i]), int(lens[i])
        assert got[i] == O.c_fold_checksum(b"", O.c_splitmix64(seed, ln, o).tobytes() if ln else b""), i


def test_ipv4_packed_headers_past_the_launch_chunk():
    """n > 2^28 packed 20 B headers (5.4 GB): the header kernel splits the batch into
    launches of 2^28; fill then verify gives 0xFFFF everywhere, and fields either side
    of the split match the oracle."""
    n, H, seed = (1 << 28) + 77, 20, 0x29
    t = torch.empty(n * H, dtype=torch.uint8, device="cuda")
    nsx.fill_splitmix64_dev(t, seed)
    t.view(n, H)[:, 0] = 0x45
    near = list(range((1 << 28) - 3, (1 << 28) + 3)) + [n - 1]
    before = {i: host(t[i * H:(i + 1) * H]) for i in near}
    nsx.ipv4_hdr_csum_dev(t, H, n, mode=1)
    raw = u16(nsx.ipv4_hdr_csum_dev(t, H, n, mode=0))
    assert (raw == 0xFFFF).all()
    for i in near:
        h = bytearray(before[i].tobytes())
        h[10:12] = b"\0\0"
        f = O.field_value(O.go_checksum(b"", bytes(h)))
        after = host(t[i * H:(i + 1) * H])
        assert after[10] == f >> 8 and after[11] == f & 0xFF, i
    mask = host(nsx.ipv4_hdr_verify_mask_dev(t, H, n)).view(np.uint64)  # mask words either side of the split
    assert (mask[:-1] == np.uint64(0xFFFFFFFFFFFFFFFF)).all() and mask[-1] == np.uint64((1 << (n % 64)) - 1)


def test_ipv4_packed_headers_auto_windows():
    """2^26 + 300 packed headers (1.34 GB) go out as three back-to-back windows of whole 256-header tasks
    (kHdrAutoWindow): raw sums and the validity bitmask equal one launch over the whole batch, and headers either
    side of every window edge match the oracle."""
    n, H, seed = (1 << 26) + 300, 20, 0x2A
    t = torch.empty(n * H, dtype=torch.uint8, device="cuda")
    nsx.fill_splitmix64_dev(t, seed)
    t.view(n, H)[:, 0] = 0x45
    t.view(n, H)[::7, 10] ^= 0x5A  # some headers invalid
    one = dict(window_bytes=-1)
    assert nsx.ipv4_hdr_launch_count(t, H, n) == 3 and nsx.ipv4_hdr_launch_count(t, H, n, tune=one) == 1
    assert nsx.ipv4_hdr_launch_count(t, H, (1 << 26) - 1) == 1
    win = -(-(-(-n // 3)) // 256) * 256
    raw = u16(nsx.ipv4_hdr_csum_dev(t, H, n, mode=0))
    assert np.array_equal(raw, u16(nsx.ipv4_hdr_csum_dev(t, H, n, mode=0, tune=one)))
    mask = host(nsx.ipv4_hdr_verify_mask_dev(t, H, n)).view(np.uint64)
    assert np.array_equal(mask, host(nsx.ipv4_hdr_verify_mask_dev(t, H, n, tune=one)).view(np.uint64))
    for e in (win, 2 * win, n):
        lo = e - 70
        hb = host(t[lo * H:min(e + 70, n) * H])
        m = hb.size // H
        want = O.c_batch(hb, m, stride=20, seg_len=20)
        assert np.array_equal(raw[lo:lo + m], want), e
        bits = np.array([(int(mask[i // 64]) >> (i % 64)) & 1 for i in range(lo, lo + m)])
        assert np.array_equal(bits, (want == 0xFFFF).astype(int)), e
    assert mask[-1] >> np.uint64(n % 64) == 0


def _oracle_build_workload(w, cfg):
    """The Go-faithful sender loop over EVERY segment of a bench f1 workload, from the device batch's own header
    fields, payloads, options, offsets and pseudo-header addresses: per segment bytes() (tcp.go:98-128, with
    tcp.go:118-121's padding), computeChecksum over its own 12 B IPv4 pseudo-header (tcp.go:72-95), ^sum stored at
    bytes 16-17 (tcp.go:68-71), the image copied to its out_off slot; 16 threads over index shards
    (O.c_go_tcp_build_mt). Returns (wire, raw)."""
    P, OL = cfg["payload"], cfg.get("opt", 0)
    W = P + 20 + OL
    fields = {k: host(w["fields"][k]).view(dt) for k, dt in zip(O.TCP_FIELDS, O.TCP_FIELD_DTYPES)}
    kw = {}
    if OL:
        kw = dict(opts=host(w["opts"]), opt_off=host(w["opt_off"]).view(np.uint64))
    return O.c_go_tcp_build_mt(fields, host(w["data"]), host(w["data_off"]).view(np.uint64),
                               host(w["out_off"]).view(np.uint64), pseudo_headers(host(w["addrs"]), W), **kw)


@pytest.mark.parametrize("wl", [6, 8, 12])
def test_f1_bench_workload_full_size_every_segment(wl):
    """The bench's f1 workloads exactly as bench.py builds and times them (bench.build_workload): 6 (1M x 1500 B
    images), 8 (1M images with a 12 B NOP NOP kind-2 option block) and 12 (256K x 8960 B jumbo images). EVERY wire
    image byte for byte and EVERY raw sum against the Go-faithful sender loop run over the same inputs
    (_oracle_build_workload); the outputs are poisoned first, so nothing stale can pass. Extra properties, not the
    parity: every image passes the receiver check on the device (sum over pseudo ‖ image == 0xFFFF, tcp.go:70), the
    raw sums equal the fixed-stride kernel's re-sum of the images with the field zeroed, and a second step writes
    the same bytes."""
    import bench
    cfg = bench.WORKLOADS[wl]
    w = bench.build_workload(cfg, 0, torch.device("cuda", 0))
    n, W = cfg["n"], cfg["payload"] + 20 + cfg.get("opt", 0)
    w["wire"].fill_(0xA5)
    w["out"].fill_(0x5A5A)
    w["step"]()
    img, raw = host(w["wire"]), u16(w["out"])
    want, wraw = _oracle_build_workload(w, cfg)
    bad = np.nonzero(raw != wraw)[0]
    assert bad.size == 0, (bad.size, bad[:8], raw[bad[:8]], wraw[bad[:8]])
    assert img.size == want.size == n * W
    if not np.array_equal(img, want):
        d = np.nonzero(img != want)[0]
        raise AssertionError(f"{d.size} image bytes differ in {np.unique(d // W).size} segments, first at byte "
                             f"{d[0]} (segment {d[0] // W}, offset {d[0] % W})")
    del want
    # extra properties on the device
    part = nsx.pseudo_ipv4_partial_dev(w["addrs"][0].reshape(-1), w["addrs"][1].reshape(-1),
                                       torch.full((n,), W, dtype=torch.int32, device="cuda"), 6)
    assert (u16(nsx.fixed_dev(w["wire"], W, W, n, partial=part)) == 0xFFFF).all()
    w["step"]()
    assert np.array_equal(host(w["wire"]), img) and np.array_equal(u16(w["out"]), raw)
    w["wire"].view(n, W)[:, 16:18] = 0
    assert np.array_equal(u16(nsx.fixed_dev(w["wire"], W, W, n, partial=part)), raw)


def test_f3_bench_workload7_full_size_every_header():
    """The bench's workload 7 at full size (64M packed 20 B headers): the setup fill (mode 1) and the timed verify
    (mode 0), every header against the oracle. Fill: each header's raw sum over its 20 bytes with the field zeroed
    (RFC 791 §3.1 with tcp.go:72-95's sum, O.c_batch) and its field = ^sum, every other byte untouched; verify:
    every header's raw sum over the filled bytes, all 0xFFFF. The buffer is the one bench.build_workload makes
    (splitmix64 bytes, version/IHL 0x45), checked equal to it after the fill."""
    import bench
    cfg = bench.WORKLOADS[7]
    n, H, seed = cfg["n"], cfg["hdr"], cfg["seed"]
    t = torch.empty(n * H, dtype=torch.uint8, device="cuda")
    nsx.fill_splitmix64_dev(t, seed)
    t.view(n, H)[:, 0] = 0x45
    before = host(t).reshape(n, H)
    head = O.c_splitmix64(seed, 4096 * H).reshape(-1, H)
    head[:, 0] = 0x45
    assert np.array_equal(before[:4096], head)
    fill = torch.full((n,), 0x5A5A, dtype=torch.int16, device="cuda")
    nsx.ipv4_hdr_csum_dev(t, H, n, mode=1, out=fill)
    z = before.copy()
    z[:, 10:12] = 0
    want_fill = O.c_batch(z.reshape(-1), n, stride=H, seg_len=H, threads=16)
    del z
    got_fill = u16(fill)
    bad = np.nonzero(got_fill != want_fill)[0]
    assert bad.size == 0, (bad.size, bad[:8])
    expect = before
    f = (~want_fill).astype(np.uint16)
    expect[:, 10] = (f >> 8).astype(np.uint8)
    expect[:, 11] = (f & 0xFF).astype(np.uint8)
    after = host(t).reshape(n, H)
    assert np.array_equal(after, expect)
    del expect, before
    w = bench.build_workload(cfg, 0, torch.device("cuda", 0))
    assert torch.equal(w["buf"], t)
    del w
    out = torch.full((n,), 0x5A5A, dtype=torch.int16, device="cuda")
    nsx.ipv4_hdr_csum_dev(t, H, n, mode=0, out=out)  # the bench step
    want = O.c_batch(after.reshape(-1), n, stride=H, seg_len=H, threads=16)
    assert np.array_equal(u16(out), want)
    assert (want == 0xFFFF).all()


# ------------------------------------------------------------------ IPv4 header checksum

def _ipv4_headers(rng, n, stride, hdr_off):
    buf = rng.integers(0, 256, n * stride + 8, dtype=np.uint8)
    ihl = rng.integers(5, 16, n)
    if stride == 20:  # packed ring: option-less headers, some with options that overrun the stride
        ihl[:] = 5
        ihl[::89] = rng.integers(6, 16, len(ihl[::89]))
    ihl[::97] = rng.integers(0, 5, len(ihl[::97]))  # some malformed
    for i in range(n):
        b0 = i * stride + hdr_off
        buf[b0] = 0x40 | int(ihl[i])
    return buf, ihl


@pytest.mark.parametrize("kernel", [0, 1, 2])  # 0: by layout (packed 20 B flat, LDS-dense for stride <= 64), 1: per-thread, 2: LDS-dense
@pytest.mark.parametrize("stride,hdr_off", [(64, 0), (61, 1), (1514, 14), (1500, 0), (60, 0), (40, 3), (20, 0)])
def test_ipv4_header_checksum_verify_and_fill(stride, hdr_off, kernel):
    tune = dict(kernel=kernel)
    rng = np.random.default_rng(stride * 31 + hdr_off)
    n = 3000
    buf, ihl = _ipv4_headers(rng, n, stride, hdr_off)
    d = dev(buf)
    raw = u16(nsx.ipv4_hdr_csum_dev(d, stride, n, hdr_off=hdr_off, mode=0, tune=tune))
    for i in range(n):
        L = int(ihl[i]) * 4
        ok = L >= 20 and hdr_off + L <= stride
        h = buf[i * stride + hdr_off:i * stride + hdr_off + L].tobytes()
        assert raw[i] == (O.go_checksum(b"", h) if ok else 0), i
    # fill mode: field written in place, then every valid header verifies
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    nsx.ipv4_hdr_csum_dev(d, stride, n, hdr_off=hdr_off, mode=1, out=out, tune=tune)
    filled = host(d)
    raw_fill = u16(out)
    for i in range(0, n, 7):
        L = int(ihl[i]) * 4
        b0 = i * stride + hdr_off
        if L >= 20 and hdr_off + L <= stride:
            h = bytearray(buf[b0:b0 + L].tobytes())
            h[10:12] = b"\0\0"
            assert raw_fill[i] == O.go_checksum(b"", bytes(h))
            assert (int(filled[b0 + 10]) << 8 | int(filled[b0 + 11])) == (~raw_fill[i]) & 0xFFFF
        else:
            assert np.array_equal(filled[b0:b0 + 12], buf[b0:b0 + 12])  # malformed: untouched
    again = u16(nsx.ipv4_hdr_csum_dev(d, stride, n, hdr_off=hdr_off, mode=0, tune=tune))
    valid = np.array([int(ihl[i]) * 4 >= 20 and hdr_off + int(ihl[i]) * 4 <= stride for i in range(n)])
    assert (again[valid] == 0xFFFF).all()


@pytest.mark.parametrize("kernel", [0, 1, 2])
@pytest.mark.parametrize("stride,hdr_off", [(20, 0), (22, 2), (60, 0), (61, 1), (1514, 14)])
@pytest.mark.parametrize("n", [1, 63, 64, 65, 255, 256, 257, 3001])
def test_ipv4_header_verify_mask(n, stride, hdr_off, kernel):
    """nsx_ipv4_hdr_verify_mask_dev: bit i set iff header i is well-formed and sums to
    0xFFFF — the oracle's go_checksum over the header (RFC 791 §3.1 with tcp.go:72-95's
    sum) on about half the headers made valid, the rest corrupted or malformed; every
    mask word written (garbage before), bits past n zero; all three kernels."""
    tune = dict(kernel=kernel)
    rng = np.random.default_rng(n * 7 + stride)
    buf, ihl = _ipv4_headers(rng, n, stride, hdr_off)
    valid = np.zeros(n, bool)
    for i in range(n):
        L, b0 = int(ihl[i]) * 4, i * stride + hdr_off
        if not (L >= 20 and hdr_off + L <= stride):
            continue
        if rng.random() < 0.6:  # give it a correct checksum field
            h = bytearray(buf[b0:b0 + L].tobytes())
            h[10:12] = b"\0\0"
            f = O.field_value(O.go_checksum(b"", bytes(h)))
            buf[b0 + 10], buf[b0 + 11] = f >> 8, f & 0xFF
        valid[i] = O.go_checksum(b"", buf[b0:b0 + L].tobytes()) == 0xFFFF
    mask = torch.full(((n + 63) // 64,), 0x5A5A5A5A5A5A5A5A, dtype=torch.int64, device="cuda")
    nsx.ipv4_hdr_verify_mask_dev(dev(buf), stride, n, hdr_off=hdr_off, mask=mask, tune=tune)
    got = host(mask).view(np.uint64)
    assert np.array_equal(got, mask_words(valid)), (n, stride, kernel)
    # the same answer as verify-into-raw-sums followed by the f2 mask kernel
    raw = nsx.ipv4_hdr_csum_dev(dev(buf), stride, n, hdr_off=hdr_off, mode=0, tune=tune)
    assert np.array_equal(host(nsx.verify_mask_dev(raw)).view(np.uint64), got)


@pytest.mark.parametrize("kernel", [0, 1, 2])
@pytest.mark.parametrize("stride,hdr_off", [(20, 0), (22, 2), (23, 3)])
def test_ipv4_dense_headers_end_at_allocation_end(stride, hdr_off, kernel):
    """Packed IHL=5 headers (header-split ring), the last one ending exactly at
    the allocation's last byte: no read past a header's own 20 bytes."""
    tune = dict(kernel=kernel)
    rng = np.random.default_rng(stride)
    n = 70_001
    buf = rng.integers(0, 256, n * stride, dtype=np.uint8)
    buf[hdr_off::stride] = 0x45
    d = dev(buf[: (n - 1) * stride + hdr_off + 20])
    nsx.ipv4_hdr_csum_dev(d, stride, n, hdr_off=hdr_off, mode=1, tune=tune)
    got = host(d)
    want = buf[: (n - 1) * stride + hdr_off + 20].copy()
    for i in list(range(0, n, 1013)) + [n - 1]:
        b0 = i * stride + hdr_off
        h = bytearray(want[b0:b0 + 20].tobytes())
        h[10:12] = b"\0\0"
        f = O.field_value(O.go_checksum(b"", bytes(h)))
        assert got[b0 + 10] == f >> 8 and got[b0 + 11] == f & 0xFF, i
    raw = u16(nsx.ipv4_hdr_csum_dev(d, stride, n, hdr_off=hdr_off, mode=0, tune=tune))
    assert (raw == 0xFFFF).all()


def test_xcd_deal_variants_agree_build_and_headers():
    """The XCD deal (auto interleaved chunks, fixed small chunks, contiguous eighths)
    changes only which wave takes which task: TCP build images and IPv4 header sums
    are identical under every deal."""
    rng = np.random.default_rng(31)
    n, P = 64 * 700 + 13, 1480
    fields, data, data_off, out_off, ps = _uniform_build_case(rng, n, P, 20)
    ref_img, ref_raw = O.c_go_tcp_build(fields, data, data_off, out_off, ps)
    nh = 256 * 900 + 77
    hb = rng.integers(0, 256, nh * 20, dtype=np.uint8)
    hb[::20] = 0x45
    want_h = O.c_batch(hb, nh, stride=20, seg_len=20)
    for chunk in (0, 2, 4, -1):
        tune = dict(xcd_chunk=chunk)
        img, raw = _run_build(fields, data, data_off, out_off, ps, tune=tune)
        assert np.array_equal(raw, ref_raw) and np.array_equal(img, ref_img), chunk
        got = u16(nsx.ipv4_hdr_csum_dev(dev(hb), 20, nh, mode=0, tune=tune))
        assert np.array_equal(got, want_h), chunk


def test_ipv4_header_kat():
    h = np.frombuffer(bytes.fromhex("450000730000400040110000c0a80001c0a800c7"), np.uint8).copy()
    d = dev(h)
    out = torch.empty(1, dtype=torch.int16, device="cuda")
    nsx.ipv4_hdr_csum_dev(d, 20, 1, mode=1, out=out)
    assert u16(out)[0] == 0x479E
    assert host(d)[10:12].tobytes() == bytes.fromhex("b861")
    assert u16(nsx.ipv4_hdr_csum_dev(d, 20, 1, mode=0))[0] == 0xFFFF


# ------------------------------------------------------------------ fused serialize + checksum

def _uniform_build_case(rng, n, P, lead, pseudo=True):
    """n option-less segments, payload P each, payloads back to back behind `lead`
    bytes, images back to back: the kernel's uniform-group (flat) layout."""
    fields = {"src_port": rng.integers(0, 1 << 16, n).astype(np.uint16),
              "dst_port": rng.integers(0, 1 << 16, n).astype(np.uint16),
              "seq_num": rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32),
              "ack_num": rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32),
              "offset": np.full(n, 5, np.uint8), "control": rng.integers(0, 256, n).astype(np.uint8),
              "window": rng.integers(0, 1 << 16, n).astype(np.uint16),
              "urgent_ptr": rng.integers(0, 1 << 16, n).astype(np.uint16)}
    data = rng.integers(0, 256, lead + n * P + 8, dtype=np.uint8)
    data_off = (np.arange(n + 1, dtype=np.uint64) * np.uint64(P)) + np.uint64(lead)
    out_off = nsx.tcp_layout_host(data_off - np.uint64(lead))
    ps = None
    if pseudo:
        ps = np.concatenate([rng.integers(0, 256, (n, 8), dtype=np.uint8),
                             np.tile(np.array([0, 6, (20 + P) >> 8 & 0xFF, (20 + P) & 0xFF], np.uint8), (n, 1))], 1)
    return fields, data, data_off, out_off, ps


def _run_build(fields, data, data_off, out_off, ps, tune=None):
    n = data_off.size - 1
    dt = {np.uint16: np.int16, np.uint32: np.int32, np.uint8: np.uint8}
    f = {k: dev(v.view(dt[v.dtype.type])) for k, v in fields.items()}
    part = None if ps is None else dev(np.array([O.be_word_sum(p.tobytes()) for p in ps], np.uint32).view(np.int32))
    out = torch.full((int(out_off[-1]),), 0xAB, dtype=torch.uint8, device="cuda")
    raw = torch.empty(n, dtype=torch.int16, device="cuda")
    nsx.tcp_build_dev(f, dev(data), dev(data_off.view(np.int64)), out, dev(out_off.view(np.int64)), partial=part,
                      raw=raw, tune=tune)
    return host(out), u16(raw)


@pytest.mark.parametrize("P", [0, 4, 8, 12, 16, 100, 1004, 1480, 4096, 8996, 65536])
@pytest.mark.parametrize("n", [1, 63, 64, 65, 300])
def test_tcp_build_uniform_batches(P, n):
    """Packed option-less batches (same payload length, payloads and images back to
    back — the bench's f1 layout): images and raw sums equal the Go-faithful oracle's
    for tiny, row-sized and 64 KiB payloads, with the pipelined fast-group path
    (kernel 0, images ≤ 2 KiB), the general pipelined composition (kernel 3) and the
    unpipelined path (kernel 2)."""
    if n * (P + 20) > 40 << 20:
        n = 65
    rng = np.random.default_rng(P * 1000 + n)
    for lead in (20, 28, 0):  # lead 0: segment 0 has no 20 bytes before its payload (general path)
        fields, data, data_off, out_off, ps = _uniform_build_case(rng, n, P, lead)
        want, wraw = O.c_go_tcp_build(fields, data, data_off, out_off, ps)
        for kern in (0, nsx.KERNEL_BUILD_GENERAL, nsx.KERNEL_BUILD_PLAIN):
            got, raw = _run_build(fields, data, data_off, out_off, ps, tune=dict(kernel=kern))
            assert np.array_equal(raw, wraw), (P, n, lead, kern)
            assert np.array_equal(got, want), (P, n, lead, kern)


@pytest.mark.parametrize("P", [0, 4, 12, 1004, 1480, 2012, 2016, 2028])
@pytest.mark.parametrize("out_base", [0, 4, 8, 12])
@pytest.mark.parametrize("gaps", ["none", "some", "all"])
def test_tcp_build_output_bases_and_gaps(P, out_base, gaps):
    """The fast path's descriptor-clipped stores: output arrays at every 4 B offset from a 16 B boundary, images
    back to back or with gaps of 4-60 bytes between some or all of them, group edges (n = 211, 16-segment
    groups) and images at the 2-row limit (P 2012-2028: 2032-2048 B images). Every image equals the oracle's,
    and no byte outside the images (gaps, the array's lead and tail) changes."""
    rng = np.random.default_rng(P * 31 + out_base * 7 + len(gaps))
    n = 211
    fields, data, data_off, out_off, ps = _uniform_build_case(rng, n, P, 20)
    wire = 20 + P
    gap = {"none": np.zeros(n, np.uint64), "all": 4 * rng.integers(1, 16, n).astype(np.uint64),
           "some": 4 * rng.integers(1, 16, n).astype(np.uint64) * (rng.random(n) < 0.2)}[gaps]
    out_off = np.zeros(n + 1, np.uint64)
    out_off[1:] = np.cumsum(np.uint64((wire + 3) & ~3) + gap)
    want, wraw = O.c_go_tcp_build(fields, data, data_off, out_off, ps)
    dt = {np.uint16: np.int16, np.uint32: np.int32, np.uint8: np.uint8}
    f = {k: dev(v.view(dt[v.dtype.type])) for k, v in fields.items()}
    part = dev(np.array([O.be_word_sum(p.tobytes()) for p in ps], np.uint32).view(np.int32))
    full = torch.full((out_base + int(out_off[-1]) + 32,), 0xAB, dtype=torch.uint8, device="cuda")
    out = full[out_base:]
    raw = torch.empty(n, dtype=torch.int16, device="cuda")
    nsx.tcp_build_dev(f, dev(data), dev(data_off.view(np.int64)), out, dev(out_off.view(np.int64)), partial=part,
                      raw=raw)
    got = host(full)
    exp = np.full(got.size, 0xAB, np.uint8)
    for i in range(n):
        o = int(out_off[i])
        exp[out_base + o:out_base + o + ((wire + 3) & ~3)] = want[o:o + ((wire + 3) & ~3)]
    assert np.array_equal(u16(raw), wraw)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, (bad[:8], got[bad[:8]], exp[bad[:8]])


_OPT_SETS = {  # option lists as the reference serialises them (tcp.go:225-231: kind 2 carries length + data)
    "nop_nop_k2len10": lambda r: [O.Option(kind=1), O.Option(kind=1), O.Option(kind=2, length=10, data=r(8))],
    "mss": lambda r: [O.Option(kind=2, length=4, data=r(2))],
    "nop_nop": lambda r: [O.Option(kind=1)] * 2,           # 22 B header: 2 pad bytes, still 4-aligned
    "nop": lambda r: [O.Option(kind=1)],                   # 21 B + 1 pad: a 22 B header (general path)
    "nop3": lambda r: [O.Option(kind=1)] * 3,              # 23 B + 3 pad: 26 B
    "k2len40": lambda r: [O.Option(kind=2, length=40, data=r(38))],  # 60 B header, the TCP maximum
    # longer than TCP allows (the data offset field wraps; the ABI still builds the bytes): > 40 option bytes
    # take the per-segment option loads instead of the group-staged ones
    "k2len41": lambda r: [O.Option(kind=2, length=41, data=r(39))],  # 61 B + 1 pad: 62 B header
    "k2len100": lambda r: [O.Option(kind=2, length=100, data=r(98))],  # 120 B header, 4-aligned
}


@pytest.mark.parametrize("P", [0, 12, 1468, 3000])
@pytest.mark.parametrize("opt", sorted(_OPT_SETS))
def test_tcp_build_uniform_batches_with_options(opt, P):
    """Packed batches whose every segment carries the same option list (the bench's
    config 8 layout): images and raw sums equal the Python oracle's Segment.bytes() /
    computeChecksum (tcp.go:98-128, :72-95) with the options at image byte 20, the
    reference's padding rule, option arrays at every byte alignment, payloads with and
    without hdr_end bytes before them, pipelined and unpipelined."""
    rng = np.random.default_rng(P * 7 + len(opt))
    n = 130
    rb = lambda k: rng.integers(0, 256, k, dtype=np.uint8).tobytes()
    segs, pseudos = [], []
    for i in range(n):
        sg = O.Segment(src_port=int(rng.integers(1 << 16)), dst_port=int(rng.integers(1 << 16)),
                       seq_num=int(rng.integers(1 << 32)), ack_num=int(rng.integers(1 << 32)),
                       control=O.Ctl.from_byte(int(rng.integers(256))), window=int(rng.integers(1 << 16)),
                       urgent_ptr=int(rng.integers(1 << 16)), options=_OPT_SETS[opt](rb), data=rb(P))
        sg.offset = sg.compute_offset()
        segs.append(sg)
        pseudos.append(O.ipv4_pseudo_header(rb(4), rb(4), 6, len(sg.bytes())))
    want_raw = np.empty(n, np.uint16)
    want_wire = []
    for i, sg in enumerate(segs):
        sg.checksum = 0
        want_raw[i] = O.c_go_checksum(pseudos[i], sg.bytes())
        sg.checksum = O.field_value(int(want_raw[i]))
        want_wire.append(sg.bytes())
    ob = [b"".join(o.bytes() for o in sg.options) for sg in segs]
    u = lambda a, dt: dev(np.asarray(a, dt).view({np.uint16: np.int16, np.uint32: np.int32, np.uint8: np.uint8}[dt]))
    fields = {"src_port": u([sg.src_port for sg in segs], np.uint16),
              "dst_port": u([sg.dst_port for sg in segs], np.uint16),
              "seq_num": u([sg.seq_num for sg in segs], np.uint32), "ack_num": u([sg.ack_num for sg in segs], np.uint32),
              "offset": u([sg.offset for sg in segs], np.uint8),
              "control": u([sg.control.byte() for sg in segs], np.uint8),
              "window": u([sg.window for sg in segs], np.uint16),
              "urgent_ptr": u([sg.urgent_ptr for sg in segs], np.uint16)}
    part = dev(np.array([O.be_word_sum(p) for p in pseudos], np.uint32).view(np.int32))
    for opt_lead, data_lead in ((0, 60), (2, 32), (3, 0), (1, 64)):
        opts = np.frombuffer(b"\x77" * opt_lead + b"".join(ob) + b"\x77" * 3, np.uint8)
        opt_off = np.zeros(n + 1, np.uint64)
        opt_off[1:] = np.cumsum([len(b) for b in ob])
        opt_off += np.uint64(opt_lead)
        data = np.frombuffer(b"\x99" * data_lead + b"".join(sg.data for sg in segs) + b"\x99" * 8, np.uint8)
        data_off = np.arange(n + 1, dtype=np.uint64) * np.uint64(P) + np.uint64(data_lead)
        out_off = nsx.tcp_layout_host(data_off, opt_off)
        assert all(int(out_off[i + 1] - out_off[i]) >= len(want_wire[i]) for i in range(n))
        # offset=None: byte 12 computed on the device (computeOffset, tcp.go:59-66) from the option bytes
        for kern, comp in ((0, False), (nsx.KERNEL_BUILD_GENERAL, False), (nsx.KERNEL_BUILD_PLAIN, False),
                           (0, True), (nsx.KERNEL_BUILD_PLAIN, True)):
            out = torch.full((int(out_off[-1]),), 0xAB, dtype=torch.uint8, device="cuda")
            raw = torch.empty(n, dtype=torch.int16, device="cuda")
            nsx.tcp_build_dev(dict(fields, offset=None) if comp else fields, dev(data), dev(data_off.view(np.int64)),
                              out, dev(out_off.view(np.int64)), opts=dev(opts), opt_off=dev(opt_off.view(np.int64)),
                              partial=part, raw=raw, tune=dict(kernel=kern))
            got, raw_h = host(out), u16(raw)
            key = (opt, P, opt_lead, data_lead, kern, comp)
            assert np.array_equal(raw_h, want_raw), key
            for i in range(n):
                o = int(out_off[i])
                assert got[o:o + len(want_wire[i])].tobytes() == want_wire[i], key + (i,)
                assert not got[o + len(want_wire[i]):int(out_off[i + 1])].any(), key + (i,)


def test_tcp_build_whole_dword_and_ragged_payloads_interleaved():
    """Whole-dword payloads (the kernel's no-shift fast path) next to a 1476 B payload
    in every other group of 64, which shifts every later payload's alignment."""
    rng = np.random.default_rng(9)
    n, P = 64 * 12, 1480
    lens = np.full(n, P, np.uint64)
    lens[64 * np.arange(0, 12, 2) + 17] = 1476  # every other group is not uniform
    data = rng.integers(0, 256, 24 + int(lens.sum()) + 8, dtype=np.uint8)
    data_off = np.zeros(n + 1, np.uint64)
    data_off[1:] = np.cumsum(lens)
    data_off += np.uint64(24)
    out_off = nsx.tcp_layout_host(data_off - np.uint64(24))
    fields = _uniform_build_case(rng, n, P, 24, pseudo=False)[0]
    got, raw = _run_build(fields, data, data_off, out_off, None)
    want, wraw = O.c_go_tcp_build(fields, data, data_off, out_off, None)
    assert np.array_equal(raw, wraw)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("lead,align4", [(1, False), (0, True), (20, True)])
def test_tcp_build_matches_reference_bytes_and_checksum(lead, align4):
    """lead = bytes before the first payload; align4 = most payloads are whole dwords at
    4-aligned offsets (the kernel's no-shift/no-mask fast path, interleaved with the
    general path for segments with options or ragged payloads)."""
    rng = np.random.default_rng(77 + lead)
    n = 3000
    opt_sets = [[], [O.Option(kind=1)], [O.Option(kind=2, length=4, data=b"\x05\xb4\0\0")],
                [O.Option(kind=1), O.Option(kind=1), O.Option(kind=0)],
                [O.Option(kind=2, length=4, data=b"wxyz"), O.Option(kind=1)], [O.Option(kind=1)] * 3]
    segs, pseudos = [], []
    for i in range(n):
        L = int(rng.integers(0, 3000)) if i % 10 else int(rng.integers(0, 8))
        if align4 and i % 7:
            L &= ~3
        s = O.Segment(src_port=int(rng.integers(1 << 16)), dst_port=int(rng.integers(1 << 16)),
                      seq_num=int(rng.integers(1 << 32)), ack_num=int(rng.integers(1 << 32)),
                      control=O.Ctl.from_byte(int(rng.integers(256))), window=int(rng.integers(1 << 16)),
                      urgent_ptr=int(rng.integers(1 << 16)),
                      options=list(opt_sets[i % len(opt_sets)]) if not align4 or i % 3 == 0 else [],
                      data=rng.integers(0, 256, L, dtype=np.uint8).tobytes())
        s.offset = s.compute_offset()
        segs.append(s)
        pseudos.append(O.ipv4_pseudo_header(rng.integers(0, 256, 4, dtype=np.uint8).tobytes(),
                                            rng.integers(0, 256, 4, dtype=np.uint8).tobytes(), 6,
                                            len(s.bytes())))
    # payloads densely packed behind a `lead`-byte lead (lead 1: odd source alignment)
    data = b"\x99" * lead + b"".join(s.data for s in segs)
    data_off = np.zeros(n + 1, np.uint64)
    data_off[1:] = np.cumsum([len(s.data) for s in segs])
    data_off += np.uint64(lead)
    opts = b"".join(o.bytes() for s in segs for o in s.options) or b"\0"
    opt_off = np.zeros(n + 1, np.uint64)
    opt_off[1:] = np.cumsum([sum(len(o.bytes()) for o in s.options) for s in segs])
    out_off = nsx.tcp_layout_host(data_off - np.uint64(lead), opt_off)
    u = lambda a, dt: dev(np.asarray(a, dt).view({np.uint16: np.int16, np.uint32: np.int32, np.uint8: np.uint8}[dt]))
    fields = {"src_port": u([s.src_port for s in segs], np.uint16), "dst_port": u([s.dst_port for s in segs], np.uint16),
              "seq_num": u([s.seq_num for s in segs], np.uint32), "ack_num": u([s.ack_num for s in segs], np.uint32),
              "offset": u([s.offset for s in segs], np.uint8), "control": u([s.control.byte() for s in segs], np.uint8),
              "window": u([s.window for s in segs], np.uint16), "urgent_ptr": u([s.urgent_ptr for s in segs], np.uint16)}
    part = np.array([O.be_word_sum(p) for p in pseudos], np.uint32)
    outs = []
    for f in (fields, dict(fields, offset=None)):  # the caller's byte 12, then computeOffset on the device
        out = torch.full((int(out_off[-1]),), 0xAB, dtype=torch.uint8, device="cuda")
        raw = torch.empty(n, dtype=torch.int16, device="cuda")
        nsx.tcp_build_dev(f, dev(np.frombuffer(data, np.uint8)), dev(data_off.view(np.int64)), out,
                          dev(out_off.view(np.int64)), opts=dev(np.frombuffer(opts, np.uint8)),
                          opt_off=dev(opt_off.view(np.int64)), partial=dev(part.view(np.int32)), raw=raw)
        outs.append((host(out), u16(raw)))
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
    got, raw_h = outs[0]
    for i, s in enumerate(segs):
        s.checksum = 0
        r = s.compute_checksum(pseudos[i])
        assert raw_h[i] == r, i
        s.checksum = O.field_value(r)
        wire = s.bytes()
        o = int(out_off[i])
        assert got[o:o + len(wire)].tobytes() == wire, i
        assert not got[o + len(wire):int(out_off[i + 1])].any()   # slack zero-filled
        assert O.verify(O.go_checksum(pseudos[i], wire))          # receiver accepts (tcp.go:70)


# ------------------------------------------------------------------ re-entrancy (include/nsx_csum.h "Threading")

def test_concurrent_calls_from_threads_on_separate_streams():
    """Four host threads, each on its own HIP stream, call different device entry points
    (fixed, ragged, TCP build with options, IPv4 verify-into-mask) 25 times each while two
    more threads run host-resident batches; ctypes drops the GIL for every C call, so the
    library runs them concurrently. Every result equals its single-threaded reference."""
    import threading
    rng = np.random.default_rng(0xC0C0)
    # fixed
    nf, L = 20000, 1500
    fb = dev(rng.integers(0, 256, nf * L, dtype=np.uint8))
    ref_f = u16(nsx.fixed_dev(fb, L, L, nf))
    # ragged
    lens = rng.integers(0, 9000, 5000).astype(np.uint64)
    offs = np.zeros(lens.size + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    rbh = rng.integers(0, 256, int(offs[-1]) + 1, dtype=np.uint8)
    rb, ro = dev(rbh), dev(offs.view(np.int64))
    ref_r = u16(nsx.ragged_dev(rb, ro))
    # TCP build with 12 B options
    n, P, OL = 3000, 1468, 12
    fields, data, data_off, out_off, _ = _uniform_build_case(rng, n, P, 64, pseudo=False)
    fields["offset"][:] = 8
    opts = rng.integers(0, 256, n * OL, dtype=np.uint8)
    opt_off = np.arange(n + 1, dtype=np.uint64) * np.uint64(OL)
    out_off = nsx.tcp_layout_host(data_off, opt_off)
    dt = {np.uint16: np.int16, np.uint32: np.int32, np.uint8: np.uint8}
    fd = {k: dev(v.view(dt[v.dtype.type])) for k, v in fields.items()}
    dd, do, oo, od, oof = dev(data), dev(data_off.view(np.int64)), dev(out_off.view(np.int64)), dev(opts), \
        dev(opt_off.view(np.int64))

    def build(stream=None):
        out = torch.zeros(int(out_off[-1]), dtype=torch.uint8, device="cuda")
        raw = torch.empty(n, dtype=torch.int16, device="cuda")
        nsx.tcp_build_dev(fd, dd, do, out, oo, opts=od, opt_off=oof, raw=raw, stream=stream)
        return out, raw
    ref_b = [host(t) for t in build()]
    # IPv4 headers into a mask
    nh = 100_000
    hb = rng.integers(0, 256, nh * 20, dtype=np.uint8)
    hb[::20] = 0x45
    hd = dev(hb)
    nsx.ipv4_hdr_csum_dev(hd, 20, nh, mode=1)
    hd.view(nh, 20)[::7, 9] ^= 1
    ref_m = host(nsx.ipv4_hdr_verify_mask_dev(hd, 20, nh))
    # host-resident fixed batch
    hh = rng.integers(0, 256, 4000 * L, dtype=np.uint8)
    ref_h = O.c_batch(hh, 4000, stride=L, seg_len=L)

    errors = []

    def worker(kind):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                for _ in range(25):
                    if kind == "fixed":
                        got = nsx.fixed_dev(fb, L, L, nf, stream=s)
                        s.synchronize()
                        assert np.array_equal(host(got).view(np.uint16), ref_f)
                    elif kind == "ragged":
                        got = nsx.ragged_dev(rb, ro, stream=s)
                        s.synchronize()
                        assert np.array_equal(host(got).view(np.uint16), ref_r)
                    elif kind == "build":
                        out, raw = build(stream=s)
                        s.synchronize()
                        assert np.array_equal(host(out), ref_b[0]) and np.array_equal(host(raw), ref_b[1])
                    elif kind == "mask":
                        got = nsx.ipv4_hdr_verify_mask_dev(hd, 20, nh, stream=s)
                        s.synchronize()
                        assert np.array_equal(host(got), ref_m)
                    else:
                        assert np.array_equal(nsx.fixed_host(hh, L, L, 4000), ref_h)
        except Exception as e:  # surfaced below
            errors.append((kind, repr(e)))

    ts = [threading.Thread(target=worker, args=(k,)) for k in ("fixed", "ragged", "build", "mask", "host", "host")]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in ts)
    assert not errors, errors


def test_entry_points_capture_into_a_hip_graph():
    """The device entry points are plain stream-ordered launches, so a transport can
    capture a receive/send step into a HIP graph (torch.cuda.CUDAGraph) and replay it:
    replays over new bytes in the same buffers give the oracle's results."""
    rng = np.random.default_rng(0x6A)
    n, L = 4096, 1500
    buf = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    lens = rng.integers(0, 4000, 1000).astype(np.uint64)
    offs = np.zeros(lens.size + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    rb = torch.empty(int(offs[-1]), dtype=torch.uint8, device="cuda")
    ro = dev(offs.view(np.int64))
    nh = 50_000
    hb = torch.empty(nh * 20, dtype=torch.uint8, device="cuda")
    out_f = torch.empty(n, dtype=torch.int16, device="cuda")
    out_r = torch.empty(lens.size, dtype=torch.int16, device="cuda")
    mask = torch.empty((nh + 63) // 64, dtype=torch.int64, device="cuda")
    nsx.fixed_dev(buf, L, L, n, out=out_f)  # first calls outside capture (library and device-info setup)
    nsx.ragged_dev(rb, ro, out=out_r)
    nsx.ipv4_hdr_verify_mask_dev(hb, 20, nh, mask=mask)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        nsx.fixed_dev(buf, L, L, n, out=out_f)
        nsx.ragged_dev(rb, ro, out=out_r)
        nsx.ipv4_hdr_verify_mask_dev(hb, 20, nh, mask=mask)
    for rep in range(3):
        fb = rng.integers(0, 256, n * L, dtype=np.uint8)
        rbh = rng.integers(0, 256, int(offs[-1]), dtype=np.uint8)
        hh = rng.integers(0, 256, nh * 20, dtype=np.uint8)
        hh[::20] = 0x45
        buf.copy_(torch.from_numpy(fb))
        rb.copy_(torch.from_numpy(rbh))
        hb.copy_(torch.from_numpy(hh))
        nsx.ipv4_hdr_csum_dev(hb, 20, nh, mode=1)  # valid checksums, then break every 5th header
        hb.view(nh, 20)[::5, 8] ^= 0x10
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(u16(out_f), O.c_batch(fb, n, stride=L, seg_len=L)), rep
        assert np.array_equal(u16(out_r), O.c_batch(rbh, lens.size, offsets=offs)), rep
        valid = np.ones(nh, bool)
        valid[::5] = False
        assert np.array_equal(host(mask).view(np.uint64), mask_words(valid)), rep


def test_f3_mask_bench_workload9_full_size_every_header():
    """The bench's workload 9 exactly as bench.py builds and times it (64M headers filled, then every 1000th
    header's TTL flipped): the mask against the oracle's verdict on EVERY header — bit i set iff the header is
    well-formed (IHL*4 >= 20 and within its 20 B stride) and its sum over the header (RFC 791 §3.1 with
    tcp.go:72-95's loop, O.c_batch) is 0xFFFF — all mask words written (poisoned first), bits past n zero.
    Extra property: exactly the flipped headers fail."""
    import bench
    cfg = bench.WORKLOADS[9]
    w = bench.build_workload(cfg, 0, torch.device("cuda", 0))
    n, H = cfg["n"], cfg["hdr"]
    w["out"].fill_(0x5A5A5A5A5A5A5A5A)
    w["step"]()
    got = host(w["out"]).view(np.uint64)
    hb = host(w["buf"])
    sums = O.c_batch(hb, n, stride=H, seg_len=H, threads=16)
    ihl4 = (hb.reshape(n, H)[:, 0] & 15).astype(np.int64) * 4
    valid = (ihl4 >= 20) & (ihl4 <= H) & (sums == 0xFFFF)
    assert np.array_equal(got, mask_words(valid))
    flipped = np.zeros(n, bool)
    flipped[::1000] = True
    assert np.array_equal(valid, ~flipped)
