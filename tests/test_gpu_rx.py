"""GPU parity of the fused receive pass (nsx_rx_ipv4_tcp_verify_dev, SURVEY.md §8 f2 + f3 in one launch):
validity bitmask and both raw sums per frame against the oracle (oracle_go_rx_ipv4_tcp: every sum through
the reference's computeChecksum loop, tcp.go:72-95; pseudo-header from the frame's own addresses,
ipv4.go:15, protocol 6, protocols.go:8; receiver rule tcp.go:70) — the committed golden frames, every kind
of valid / broken / malformed frame at every start alignment and batch size around the 64-frame mask
words, every launch shape, maximum-size datagrams, and the bench's workload 10 at full size."""
import json
import os

import numpy as np
import pytest

import _rx
from _gpu import dev, host, setup_gpu, torch, u16
from conftest import GOLDEN
from oracle import csum_oracle as O

import nsx  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu():
    setup_gpu()


def run_rx(buf, offs, tune=None):
    n = offs.size - 1
    mask = torch.full(((n + 63) // 64,), 0x5A5A5A5A5A5A5A5A, dtype=torch.int64, device="cuda")  # garbage before
    ipr = torch.empty(n, dtype=torch.int16, device="cuda")
    tcpr = torch.empty(n, dtype=torch.int16, device="cuda")
    nsx.rx_ipv4_tcp_verify_dev(dev(buf), dev(offs.view(np.int64)), mask=mask, ip_raw=ipr, tcp_raw=tcpr, tune=tune)
    return host(mask).view(np.uint64), u16(ipr), u16(tcpr)


def test_rx_golden_frames():
    meta = json.load(open(os.path.join(GOLDEN, "rx.json")))
    blob = np.fromfile(os.path.join(GOLDEN, "rx.bin"), np.uint8)
    mask, ipr, tcpr = run_rx(blob, np.array(meta["offsets"], np.uint64))
    assert mask.tolist() == meta["mask"]
    assert ipr.tolist() == meta["ip_raw"] and tcpr.tolist() == meta["tcp_raw"]


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 127, 128, 129, 1000, 4099])
@pytest.mark.parametrize("lead", [0, 1, 2, 3])
def test_rx_mixed_batches(n, lead):
    rng = np.random.default_rng(n * 4 + lead)
    buf, offs, kinds = _rx.batch(rng, n, lead=lead, max_payload=1460)
    want = O.c_rx_ipv4_tcp(buf, offs)
    for tune in [None] + PFX:
        got = run_rx(buf, offs, tune)
        for w, g, what in zip(want, got, ("mask", "ip_raw", "tcp_raw")):
            assert np.array_equal(w, g), (what, n, lead, tune)


TUNES = [dict(rows=2), dict(rows=4), dict(rows=16), dict(blocks_per_cu=1), dict(blocks_per_cu=8), dict(rows=16, blocks_per_cu=1),
         dict(segs_per_wave=1), dict(segs_per_wave=1, rows=4), dict(segs_per_wave=1, blocks_per_cu=4),  # streamed runs
         dict(segs_per_wave=2), dict(segs_per_wave=2, blocks_per_cu=1), dict(segs_per_wave=2, blocks_per_cu=4),
         dict(segs_per_wave=2, blocks_per_cu=8), dict(blocks_per_cu=4),  # LDS form; 4 blocks/CU = the capped kernel
         dict(segs_per_wave=5), dict(segs_per_wave=6), dict(segs_per_wave=7), dict(segs_per_wave=8),
         dict(segs_per_wave=9)]  # the default grid's modes
# the default grid's modes forced (5 the LDS loop handing over to the hybrid loop, 7 the hybrid loop throughout, both
# on two waves per block; 6 the 15-row prefix form on two waves per block; 9 the LDS loop fed by LDS-DMA through a ring,
# handing over to the hybrid loop like 5)
PFX = [dict(segs_per_wave=5), dict(segs_per_wave=6), dict(segs_per_wave=7), dict(segs_per_wave=8), dict(segs_per_wave=9)]


@pytest.mark.parametrize("n", [1, 255, 256, 257, 1000, 30_001])
@pytest.mark.parametrize("lead", [0, 3])
def test_rx_small_frames_runs_of_four_sets(n, lead):
    """Frames of at most 40 B of payload: waves whose frames average under 128 B take the LDS form (DESIGN.md §7
    step 43); it, and the streamed runs of 64-frame sets, equal the oracle at every run boundary and partial last
    run, at the default 4-blocks/CU grid and at 3."""
    rng = np.random.default_rng(n * 2 + lead)
    buf, offs, _ = _rx.batch(rng, n, lead=lead, max_payload=40)
    want = O.c_rx_ipv4_tcp(buf, offs)
    for tune in [None, dict(segs_per_wave=1), dict(segs_per_wave=2), dict(blocks_per_cu=3)] + PFX:
        got = run_rx(buf, offs, tune)
        for w, g, what in zip(want, got, ("mask", "ip_raw", "tcp_raw")):
            assert np.array_equal(w, g), (what, n, lead, tune)


def _device_frames(cfg, seed):
    """Frames built on the device (bench.build_rx_frames: valid IPv4 / IPv6 datagrams, every 1000th corrupted),
    then broken further so the large small-frame batches hold every outcome: bit flips in the TCP bytes of ~3% of
    the frames, and in the IPv4 case the protocol set to UDP in ~1% and the total length off by one in ~1%."""
    import bench
    w = bench.build_rx_frames(cfg, seed, torch.device("cuda", 0))
    buf, d_offs = w["buf"], w["d_offs"]
    st = d_offs[:-1]
    ln = d_offs[1:] - st
    g = torch.Generator(device="cuda").manual_seed(seed)
    n = cfg["n"]
    pick = torch.randint(0, n, (n // 33,), generator=g, device="cuda")
    hl = 40 if cfg.get("ipver") == 6 else 20
    pos = st[pick] + hl + torch.remainder(torch.randint(0, 1 << 30, pick.shape, generator=g, device="cuda"), ln[pick] - hl)
    buf[pos] ^= (1 << torch.randint(0, 8, pick.shape, generator=g, device="cuda")).to(torch.uint8)
    if cfg.get("ipver") != 6:
        udp = torch.randint(0, n, (n // 100,), generator=g, device="cuda")
        buf[st[udp] + 9] = 17
        bad_len = torch.randint(0, n, (n // 100,), generator=g, device="cuda")
        buf[st[bad_len] + 3] ^= 1
    torch.cuda.synchronize()
    return w


@pytest.mark.parametrize("ipver", [4, 6])
def test_rx_small_frames_300K_every_set_form_vs_oracle(ipver):
    """~300K ACK-sized frames (40-100 B IPv4 / 60-120 B IPv6), enough that every wave walks
    many runs of its form (the LDS form's run-to-run pipeline, its fallback-free loop, partial last runs). The
    automatic choice and the forced streamed and LDS forms, at the default grid and at 1, 3 and 4 blocks per CU,
    against the oracle's mask and raw sums on every frame."""
    cfg = dict(n=300_007, lo=40, hi=100, seed=0x5A11) if ipver == 4 else \
        dict(ipver=6, n=300_007, lo=60, hi=120, seed=0x5A16)
    w = _device_frames(cfg, cfg["seed"])
    buf_h = host(w["buf"])
    offs = w["offsets"]
    n = cfg["n"]
    want = O.c_rx_ipv4_tcp(buf_h, offs) if ipver == 4 else O.c_rx_ipv6_tcp(buf_h, offs)
    bits = np.unpackbits(want[0].view(np.uint8), bitorder="little")[:n]
    assert 0.85 * n < bits.sum() < 0.985 * n  # mostly valid, every kind of failure present
    for tune in (None, dict(segs_per_wave=1), dict(segs_per_wave=2), dict(blocks_per_cu=1), dict(blocks_per_cu=3),
                 dict(blocks_per_cu=1, segs_per_wave=1), dict(blocks_per_cu=1, segs_per_wave=2),
                 dict(blocks_per_cu=4, segs_per_wave=1), *PFX):
        got = run_rx(buf_h, offs, tune) if ipver == 4 else run_rx6(buf_h, offs, tune)
        for wv, g, what in zip(want, got, ("mask", "ip_raw", "tcp_raw") if ipver == 4 else ("mask", "tcp_raw")):
            bad = np.nonzero(wv != g)[0]
            assert bad.size == 0, (what, tune, bad[:5])


@pytest.mark.parametrize("config", [13, 14, 16, 17, 18])
def test_rx_small_frame_bench_workloads_full_size(config):
    """The bench's small-frame receive workloads at full size (13: 8M IPv4 frames of 40-100 B; 14: 2M frames, half
    40-66 B ACKs and half 1500 B; 16: 8M IPv6 packets of 60-120 B; 17: 8M frames, 95% ACKs and 5% 1500 B — equal-count
    wave ranges with runs too wide for the LDS slot among LDS runs): the device mask equals the oracle's on every
    frame, and exactly the corrupted frames fail."""
    import bench
    cfg = bench.WORKLOADS[config]
    w = bench.build_workload(cfg, 0, torch.device("cuda", 0))
    w["step"]()
    got = host(w["out"]).view(np.uint64)
    rx = O.c_rx_ipv6_tcp if cfg.get("ipver") == 6 else O.c_rx_ipv4_tcp
    want = rx(host(w["buf"]), w["offsets"])[0]
    assert np.array_equal(got, want)
    n = cfg["n"]
    valid = np.ones(n, bool)
    valid[::1000] = False
    pad = np.zeros((n + 63) // 64 * 64, np.uint8)
    pad[:n] = valid
    assert np.array_equal(got, np.packbits(pad, bitorder="little").view(np.uint64))


@pytest.mark.parametrize("config", [10, 13, 14, 16, 17, 18])
def test_rx_prefix_form_bench_workloads_full_size(config):
    """The default grid's forms forced on the bench's receive workloads at full size:
    the hybrid loop (direct runs and 7-row prefix pieces) and the 15-row prefix form on two waves per block —
    pieces cut at every multiple of 8 frames, whole runs, the streamed fallback; mask and raw sums against the
    oracle on every frame."""
    import bench
    cfg = bench.WORKLOADS[config]
    w = bench.build_workload(cfg, 0, torch.device("cuda", 0))
    buf_h = host(w["buf"])
    v6 = cfg.get("ipver") == 6
    want = (O.c_rx_ipv6_tcp if v6 else O.c_rx_ipv4_tcp)(buf_h, w["offsets"])
    for tune in PFX:
        got = run_rx6(buf_h, w["offsets"], tune) if v6 else run_rx(buf_h, w["offsets"], tune)
        for wv, g, what in zip(want, got, ("mask", "tcp_raw") if v6 else ("mask", "ip_raw", "tcp_raw")):
            bad = np.nonzero(wv != g)[0]
            assert bad.size == 0, (what, config, tune, bad[:5])


def test_rx_batch_past_the_launch_chunk():
    """n > 2^27 ACK-sized frames (7.1 GB): the receive pass splits the batch into launches of 2^27 frames, each
    starting on a mask word and choosing its form by its own mean frame. The mask is the expected pattern on every
    frame (exactly the corrupted ones fail), the last word's bits past n are 0, and the raw sums of the frames either
    side of the split and at the end equal the oracle's."""
    import bench
    cfg = dict(kind="rx", n=(1 << 27) + 999, lo=40, hi=66, seed=0x27)
    w = bench.build_rx_frames(cfg, cfg["seed"], torch.device("cuda", 0))
    n, offs = cfg["n"], w["offsets"]
    mask = torch.full(((n + 63) // 64,), 0x5A5A5A5A5A5A5A5A, dtype=torch.int64, device="cuda")
    ipr = torch.empty(n, dtype=torch.int16, device="cuda")
    tcpr = torch.empty(n, dtype=torch.int16, device="cuda")
    nsx.rx_ipv4_tcp_verify_dev(w["buf"], w["d_offs"], mask=mask, ip_raw=ipr, tcp_raw=tcpr)
    got = host(mask).view(np.uint64)
    valid = np.ones(n, bool)
    valid[::1000] = False
    pad = np.zeros((n + 63) // 64 * 64, np.uint8)
    pad[:n] = valid
    assert np.array_equal(got, np.packbits(pad, bitorder="little").view(np.uint64))
    for lo, hi in (((1 << 27) - 70, (1 << 27) + 70), (n - 100, n)):
        o0 = int(offs[lo])
        sub = host(w["buf"][o0:int(offs[hi])])
        _, want_i, want_t = O.c_rx_ipv4_tcp(sub, offs[lo:hi + 1] - np.uint64(o0))
        assert np.array_equal(u16(ipr[lo:hi]), want_i) and np.array_equal(u16(tcpr[lo:hi]), want_t), (lo, hi)


@pytest.mark.parametrize("tune", TUNES, ids=lambda t: ",".join(f"{k}={v}" for k, v in t.items()))
def test_rx_launch_shapes(tune):
    rng = np.random.default_rng(0x7E)
    buf, offs, _ = _rx.batch(rng, 20_000, lead=1, max_payload=1460)
    want = O.c_rx_ipv4_tcp(buf, offs)
    got = run_rx(buf, offs, tune)
    for w, g in zip(want, got):
        assert np.array_equal(w, g), tune


def test_rx_mostly_valid_large_frames_and_junk():
    """Maximum-size datagrams (total length 65535 − header), jumbo-ish frames, runs of empty frames, and a
    4 MB junk frame (not IPv4, longer than any datagram) in the middle: its neighbours still verify."""
    rng = np.random.default_rng(0x7F)
    frames = []
    for i in range(700):
        r = i % 7
        if r == 0:
            seg_len = 65535 - 20 - 20 * (i % 3)
            frames.append(O.ipv4_tcp_frame(_rx._segment(rng, seg_len - 20), rng.bytes(4), rng.bytes(4)))
        elif r == 1:
            frames.append(b"")
        else:
            frames.append(_rx.frame(rng, "valid", max_payload=9000))
    frames.insert(350, rng.integers(0, 256, 4 << 20, dtype=np.uint8).tobytes())
    offs = np.zeros(len(frames) + 1, np.uint64)
    offs[1:] = np.cumsum([len(f) for f in frames])
    buf = np.frombuffer(b"".join(frames) + bytes(3), np.uint8)
    want = O.c_rx_ipv4_tcp(buf, offs)
    for tune in [None] + PFX:  # the prefix form streams the pieces whose first 8 frames exceed its slot
        got = run_rx(buf, offs, tune)
        for w, g in zip(want, got):
            assert np.array_equal(w, g), tune
    bits = np.unpackbits(want[0].view(np.uint8), bitorder="little")
    assert bits[:len(frames)].sum() == sum(1 for i, f in enumerate(frames) if len(f) and i != 350)


def test_rx_bench_workload_full_size():
    """The bench's workload 10 at full size (1M frames of 40-1500 B, 1 in 1000 corrupted after the fill):
    the device mask equals the oracle's on every frame, and exactly the corrupted frames fail."""
    import bench
    cfg = bench.WORKLOADS[10]
    w = bench.build_workload(cfg, 0, torch.device("cuda", 0))
    w["step"]()
    got = host(w["out"]).view(np.uint64)
    want, _, _ = O.c_rx_ipv4_tcp(host(w["buf"]), w["offsets"])
    assert np.array_equal(got, want)
    n = cfg["n"]
    valid = np.ones(n, bool)
    valid[::1000] = False
    pad = np.zeros((n + 63) // 64 * 64, np.uint8)
    pad[:n] = valid
    assert np.array_equal(got, np.packbits(pad, bitorder="little").view(np.uint64))


def test_rx_skewed_batches_every_mode():
    """Skewed batches — 100k ACK-size frames then 20k large ones, and the reverse — where equal-count and byte-balanced
    wave ranges differ most and the dealt pool holds only large (or only small) frames, in
    the automatic mode and every forced two-wave and streamed mode, equal the oracle."""
    rng = np.random.default_rng(0x8C)
    small, so, _ = _rx.batch(rng, 100_000, max_payload=40)
    big, bo, _ = _rx.batch(rng, 20_000, max_payload=1460)
    for first, fo, second, sec_o in ((small, so, big, bo), (big, bo, small, so)):
        cut = int(fo[-1])
        buf = np.concatenate([first[:cut], second])
        offs = np.concatenate([fo[:-1], sec_o + np.uint64(cut)])
        want = O.c_rx_ipv4_tcp(buf, offs)
        for tune in [None, dict(segs_per_wave=1)] + PFX:
            got = run_rx(buf, offs, tune)
            for w, g, what in zip(want, got, ("mask", "ip_raw", "tcp_raw")):
                assert np.array_equal(w, g), (what, tune)


def test_rx_dealt_runs_back_to_back_and_on_many_streams():
    """The two-wave modes deal each launch's last runs from counters of the launch's stream, which the launch leaves
    at zero for the next: launches back to back on one stream with no sync between them —
    batches of different sizes (3 frames to 200k) and modes (auto, 5, 6, 7) — and launches on 70 HIP streams at once,
    more than the 64 counter sets a device gives out (the rest run equal static shares), all equal the oracle."""
    import ctypes
    rng = np.random.default_rng(0x8A)
    cases = []
    for n, mp in ((200_000, 40), (150_001, 120), (3, 40), (70_000, 1460), (129, 40), (64 * 1000, 80)):
        buf, offs, _ = _rx.batch(rng, n, lead=int(rng.integers(4)), max_payload=mp)
        cases.append((dev(buf), dev(offs.view(np.int64)), O.c_rx_ipv4_tcp(buf, offs)))
    modes = [None, dict(segs_per_wave=5), dict(segs_per_wave=6), dict(segs_per_wave=7)]

    def launch(k, tune, stream=None):
        dbuf, doffs, _ = cases[k]
        n = doffs.numel() - 1
        with torch.cuda.stream(stream or torch.cuda.current_stream()):  # the outputs' fill ordered before the launch
            mask = torch.full(((n + 63) // 64,), 0x5A5A5A5A5A5A5A5A, dtype=torch.int64, device="cuda")
            ipr = torch.empty(n, dtype=torch.int16, device="cuda")
            tcpr = torch.empty(n, dtype=torch.int16, device="cuda")
            nsx.rx_ipv4_tcp_verify_dev(dbuf, doffs, mask=mask, ip_raw=ipr, tcp_raw=tcpr, tune=tune)
        return k, tune, (mask, ipr, tcpr)

    def check(results):
        torch.cuda.synchronize()
        for k, tune, (mask, ipr, tcpr) in results:
            got = (host(mask).view(np.uint64), u16(ipr), u16(tcpr))
            for w, g, what in zip(cases[k][2], got, ("mask", "ip_raw", "tcp_raw")):
                assert np.array_equal(w, g), (what, k, tune)

    check([launch(k, modes[(r + k) % 4]) for r in range(4) for k in range(len(cases))])
    torch.cuda.synchronize()
    hip = ctypes.CDLL("libamdhip64.so")
    handles = []
    for _ in range(70):
        h = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(h)) == 0
        handles.append(h)
    try:
        streams = [torch.cuda.ExternalStream(h.value) for h in handles]
        check([launch((i + r) % len(cases), modes[i % 4], streams[i]) for r in range(2) for i in range(len(streams))])
    finally:
        torch.cuda.synchronize()
        for h in handles:
            nsx.stream_release(h.value)  # later tests' streams get these sets again
            hip.hipStreamDestroy(h)


def test_rx_streamed_dealt_pieces_back_to_back_and_on_many_streams():
    """The streamed modes deal the batch's last eighth in 16-frame pieces through each block's LDS ring: waves 0-2
    stream, wave 3 pulls tickets from the stream's heads for the pieces they claim, and the last dealer of a head
    resets it. IPv4 and IPv6 batches of 1 to 250k frames of full-size payloads (the streamed
    choice), launched back to back on one stream with no sync between them — auto, forced mode 8, the static split
    (deal -1) — interleaved with small-frame launches (mode 5, DealtRuns on the same heads), raw outputs 2 B past a
    16 B boundary; then on 70 streams at once; every mask bit and raw sum equals the oracle."""
    import ctypes
    rng = np.random.default_rng(0x8C)
    cases = []
    for n, mp, ip in ((250_001, 1460, 4), (1, 1460, 4), (3, 1400, 6), (129, 1460, 4), (1000, 1460, 6),
                      (70_001, 1460, 4), (64 * 700, 1440, 6), (50_000, 40, 4)):
        kinds = _rx.KINDS6 if ip == 6 else _rx.KINDS
        buf, offs, _ = _rx.batch(rng, n, kinds=kinds, lead=int(rng.integers(4)), max_payload=mp, ip=ip)
        want = O.c_rx_ipv6_tcp(buf, offs) if ip == 6 else O.c_rx_ipv4_tcp(buf, offs)
        cases.append((dev(buf), dev(offs.view(np.int64)), ip, want))
    modes = [None, dict(segs_per_wave=8), dict(deal=-1), dict(segs_per_wave=5)]

    def launch(k, tune, stream=None):
        dbuf, doffs, ip, _ = cases[k]
        n = doffs.numel() - 1
        with torch.cuda.stream(stream or torch.cuda.current_stream()):
            mask = torch.full(((n + 63) // 64,), 0x5A5A5A5A5A5A5A5A, dtype=torch.int64, device="cuda")
            ipr = torch.empty(n + 1, dtype=torch.int16, device="cuda")[1:]
            tcpr = torch.empty(n + 1, dtype=torch.int16, device="cuda")[1:]
            if ip == 6:
                nsx.rx_ipv6_tcp_verify_dev(dbuf, doffs, mask=mask, tcp_raw=tcpr, tune=tune)
            else:
                nsx.rx_ipv4_tcp_verify_dev(dbuf, doffs, mask=mask, ip_raw=ipr, tcp_raw=tcpr, tune=tune)
        return k, tune, (mask, ipr, tcpr)

    def check(results):
        torch.cuda.synchronize()
        for k, tune, (mask, ipr, tcpr) in results:
            ip, want = cases[k][2], cases[k][3]
            assert np.array_equal(host(mask).view(np.uint64), want[0]), ("mask", k, tune)
            if ip == 6:
                assert np.array_equal(u16(tcpr), want[1]), ("tcp_raw", k, tune)
            else:
                assert np.array_equal(u16(ipr), want[1]), ("ip_raw", k, tune)
                assert np.array_equal(u16(tcpr), want[2]), ("tcp_raw", k, tune)

    check([launch(k, modes[(r + k) % 4]) for r in range(6) for k in range(len(cases))])
    # the mask alone (no raw outputs: the bench's call) on the default stream, back to back
    for k in range(len(cases)):
        dbuf, doffs, ip, want = cases[k]
        f = nsx.rx_ipv6_tcp_verify_dev if ip == 6 else nsx.rx_ipv4_tcp_verify_dev
        masks = [f(dbuf, doffs) for _ in range(3)]
        for m in masks:
            assert np.array_equal(host(m).view(np.uint64), want[0]), k
    hip = ctypes.CDLL("libamdhip64.so")
    handles = []
    for _ in range(70):
        h = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(h)) == 0
        handles.append(h)
    try:
        streams = [torch.cuda.ExternalStream(h.value) for h in handles]
        check([launch((i + r) % len(cases), modes[(i + r) % 2], streams[i]) for r in range(2)
               for i in range(len(streams))])
    finally:
        torch.cuda.synchronize()
        for h in handles:
            nsx.stream_release(h.value)
            hip.hipStreamDestroy(h)


@pytest.mark.parametrize("shards", [1, 2, 3, 8])
def test_rx_host_batches_sharded(shards):
    """nsx_rx_ipv4_tcp_verify_host: the receive pass from host memory (pinned staging, H2D → kernel → D2H of
    mask words), the batch split into `shards` shards on the one device and into 64 MiB chunks, every shard and
    chunk starting on a 64-frame mask word; ~200 MB of frames (a tiled mixed batch), pageable input."""
    rng = np.random.default_rng(0x80 + shards)
    buf0, offs0, _ = _rx.batch(rng, 4999, lead=0, max_payload=1460)
    reps = 40
    span = int(offs0[-1])
    buf = np.concatenate([buf0[:span]] * reps + [np.zeros(3, np.uint8)])
    offs = np.concatenate([offs0[:-1] + np.uint64(k * span) for k in range(reps)] + [np.array([reps * span], np.uint64)])
    want, _, _ = O.c_rx_ipv4_tcp(buf, offs)
    got = nsx.rx_ipv4_tcp_verify_host(buf, offs, tune=dict(shards_per_device=shards))
    assert np.array_equal(got, want), shards
    small = nsx.rx_ipv4_tcp_verify_host(buf0, offs0, tune=dict(shards_per_device=shards))
    assert np.array_equal(small, O.c_rx_ipv4_tcp(buf0, offs0)[0])


# ------------------------------------------------------------------ IPv6 (nsx_rx_ipv6_tcp_verify_dev)

def run_rx6(buf, offs, tune=None):
    n = offs.size - 1
    mask = torch.full(((n + 63) // 64,), 0x5A5A5A5A5A5A5A5A, dtype=torch.int64, device="cuda")
    tcpr = torch.empty(n, dtype=torch.int16, device="cuda")
    nsx.rx_ipv6_tcp_verify_dev(dev(buf), dev(offs.view(np.int64)), mask=mask, tcp_raw=tcpr, tune=tune)
    return host(mask).view(np.uint64), u16(tcpr)


def test_rx6_golden_packets():
    meta = json.load(open(os.path.join(GOLDEN, "rx6.json")))
    blob = np.fromfile(os.path.join(GOLDEN, "rx6.bin"), np.uint8)
    mask, tcpr = run_rx6(blob, np.array(meta["offsets"], np.uint64))
    assert mask.tolist() == meta["mask"]
    assert tcpr.tolist() == meta["tcp_raw"]


@pytest.mark.parametrize("n", [1, 63, 64, 65, 129, 1000, 4099])
@pytest.mark.parametrize("lead", [0, 1, 2, 3])
def test_rx6_mixed_batches(n, lead):
    rng = np.random.default_rng(n * 8 + lead + 1)
    buf, offs, kinds = _rx.batch(rng, n, kinds=_rx.KINDS6, lead=lead, max_payload=1440, ip=6)
    want = O.c_rx_ipv6_tcp(buf, offs)
    for tune in [None] + PFX:
        got = run_rx6(buf, offs, tune)
        for w, g, what in zip(want, got, ("mask", "tcp_raw")):
            assert np.array_equal(w, g), (what, n, lead, tune)


@pytest.mark.parametrize("tune", TUNES, ids=lambda t: ",".join(f"{k}={v}" for k, v in t.items()))
def test_rx6_launch_shapes(tune):
    rng = np.random.default_rng(0x7E6)
    buf, offs, _ = _rx.batch(rng, 20_000, kinds=_rx.KINDS6, lead=3, max_payload=1440, ip=6)
    want = O.c_rx_ipv6_tcp(buf, offs)
    got = run_rx6(buf, offs, tune)
    for w, g in zip(want, got):
        assert np.array_equal(w, g), tune


def test_rx6_maximum_packets_and_junk():
    """Packets at the 16-bit payload length limit (65535 B of TCP), runs of empty frames, and a 4 MB junk
    frame in the middle: its neighbours still verify."""
    rng = np.random.default_rng(0x7F6)
    frames = []
    for i in range(500):
        r = i % 5
        if r == 0:
            frames.append(O.ipv6_tcp_frame(_rx._segment(rng, 65535 - 20 - (i % 3)), rng.bytes(16), rng.bytes(16)))
        elif r == 1:
            frames.append(b"")
        else:
            frames.append(_rx.frame6(rng, "valid", max_payload=9000))
    frames.insert(250, rng.integers(0, 256, 4 << 20, dtype=np.uint8).tobytes())
    offs = np.zeros(len(frames) + 1, np.uint64)
    offs[1:] = np.cumsum([len(f) for f in frames])
    buf = np.frombuffer(b"".join(frames) + bytes(3), np.uint8)
    want = O.c_rx_ipv6_tcp(buf, offs)
    for tune in [None] + PFX:
        got = run_rx6(buf, offs, tune)
        for w, g in zip(want, got):
            assert np.array_equal(w, g), tune
    bits = np.unpackbits(want[0].view(np.uint8), bitorder="little")
    assert bits[:len(frames)].sum() == sum(1 for i, f in enumerate(frames) if len(f) and i != 250)


def test_rx6_bench_workload_full_size():
    """The bench's workload 11 at full size: the device mask equals the oracle's, and exactly the corrupted
    packets fail."""
    import bench
    cfg = bench.WORKLOADS[11]
    w = bench.build_workload(cfg, 0, torch.device("cuda", 0))
    w["step"]()
    got = host(w["out"]).view(np.uint64)
    want, _ = O.c_rx_ipv6_tcp(host(w["buf"]), w["offsets"])
    assert np.array_equal(got, want)
    n = cfg["n"]
    valid = np.ones(n, bool)
    valid[::1000] = False
    pad = np.zeros((n + 63) // 64 * 64, np.uint8)
    pad[:n] = valid
    assert np.array_equal(got, np.packbits(pad, bitorder="little").view(np.uint64))


@pytest.mark.parametrize("shards", [1, 3])
def test_rx6_host_batches_sharded(shards):
    rng = np.random.default_rng(0x90 + shards)
    buf0, offs0, _ = _rx.batch(rng, 4999, kinds=_rx.KINDS6, lead=0, max_payload=1440, ip=6)
    reps = 30
    span = int(offs0[-1])
    buf = np.concatenate([buf0[:span]] * reps + [np.zeros(3, np.uint8)])
    offs = np.concatenate([offs0[:-1] + np.uint64(k * span) for k in range(reps)] + [np.array([reps * span], np.uint64)])
    want, _ = O.c_rx_ipv6_tcp(buf, offs)
    got = nsx.rx_ipv6_tcp_verify_host(buf, offs, tune=dict(shards_per_device=shards))
    assert np.array_equal(got, want), shards


@pytest.mark.parametrize("ipver", [4, 6])
def test_rx_parked_raw_sums_any_output_alignment(ipver):
    """The streamed form parks its raw sums in the wave's LDS slot and writes them in 16 B
    blocks aligned to each output: raw outputs 0-7 sums past a 16 B boundary inside sentinel-filled buffers, either
    one alone or both, get exactly the oracle's sums and nothing outside them is written; the mask is unaffected.
    40-1500 B frames (mean ~770 B: the default takes streamed runs) and the forced streamed mode 8."""
    rng = np.random.default_rng(0x67 + ipver)
    n = 120_003
    kinds = _rx.KINDS6 if ipver == 6 else _rx.KINDS
    buf, offs, _ = _rx.batch(rng, n, kinds=kinds, lead=3, max_payload=1460, ip=ipver)
    want = (O.c_rx_ipv6_tcp if ipver == 6 else O.c_rx_ipv4_tcp)(buf, offs)
    want_m, want_t = want[0], want[-1]
    want_i = want[1] if ipver == 4 else None
    d, o = dev(buf), dev(offs.view(np.int64))
    fn = nsx.rx_ipv6_tcp_verify_dev if ipver == 6 else nsx.rx_ipv4_tcp_verify_dev
    ib = torch.empty(n + 32, dtype=torch.int16, device="cuda")
    tb = torch.empty(n + 32, dtype=torch.int16, device="cuda")
    for tune in (None, dict(segs_per_wave=8)):
        for si, st in ((0, 0), (1, 7), (5, 3), (7, 0)):
            for which in (("t",) if ipver == 6 else ("i", "t", "it")):
                ib.fill_(0x5A5A)
                tb.fill_(0x5A5A)
                kw = {}
                if "t" in which:
                    kw["tcp_raw"] = tb[st:st + n]
                if "i" in which:
                    kw["ip_raw"] = ib[si:si + n]
                mask = fn(d, o, tune=tune, **kw)
                assert np.array_equal(host(mask).view(np.uint64), want_m), (tune, which)
                if "t" in which:
                    g = u16(tb)
                    assert np.array_equal(g[st:st + n], want_t), (tune, which, st)
                    assert (g[:st] == 0x5A5A).all() and (g[st + n:] == 0x5A5A).all(), (tune, which, st)
                if "i" in which:
                    g = u16(ib)
                    assert np.array_equal(g[si:si + n], want_i), (tune, which, si)
                    assert (g[:si] == 0x5A5A).all() and (g[si + n:] == 0x5A5A).all(), (tune, which, si)
