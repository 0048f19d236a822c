"""GPU parity of the receive-side parse (nsx_tcp_parse_dev, parseSegment transport/tcp/tcp.go:130-185): every
field, the data offset, the option count and the status against the oracle's parse_segment (itself checked
against the C++ mirror on the golden segments, tests/test_tcp_cpp.py) — the committed golden segments, every
kind of valid / rejected / would-panic / would-loop segment at every start alignment and batch size, partial
output sets, and a large batch."""
import json
import os

import numpy as np
import pytest

import _parse
from _gpu import dev, host, setup_gpu, torch
from conftest import GOLDEN

import nsx  # noqa: E402

pytestmark = pytest.mark.gpu

VIEW = {"src_port": np.uint16, "dst_port": np.uint16, "seq_num": np.uint32, "ack_num": np.uint32, "offset": np.uint8,
        "control": np.uint8, "window": np.uint16, "checksum": np.uint16, "urgent_ptr": np.uint16,
        "data_off": np.uint64, "n_options": np.uint8, "status": np.uint8}


@pytest.fixture(scope="module", autouse=True)
def gpu():
    setup_gpu()


def run_parse(buf, offs, want=None):
    got = nsx.tcp_parse_dev(dev(buf), dev(offs.view(np.int64)), want=want)
    return {k: host(v).view(VIEW[k]) for k, v in got.items()}


def check(got, exp, key):
    for k, v in got.items():
        assert np.array_equal(v, exp[k]), (k, key, np.nonzero(v != exp[k])[0][:5])


def test_parse_golden_segments():
    meta = json.load(open(os.path.join(GOLDEN, "parse.json")))
    blob = np.fromfile(os.path.join(GOLDEN, "parse.bin"), np.uint8)
    got = run_parse(blob, np.array(meta["offsets"], np.uint64))
    for k in VIEW:
        assert got[k].tolist() == meta[k], k


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 257, 1000, 5003])
@pytest.mark.parametrize("lead", [0, 1, 2, 3])
def test_parse_mixed_batches(n, lead):
    rng = np.random.default_rng(n * 4 + lead + 0x500)
    buf, offs, _ = _parse.batch(rng, n, lead=lead, max_payload=600)
    check(run_parse(buf, offs), _parse.expected(buf, offs), (n, lead))


@pytest.mark.parametrize("want", [("status",), ("data_off", "n_options"), ("seq_num", "ack_num", "checksum")])
def test_parse_partial_outputs(want):
    """Any member of nsx_tcp_parsed_soa may be null: only the requested arrays are written."""
    rng = np.random.default_rng(0x51)
    buf, offs, _ = _parse.batch(rng, 3000, lead=1, max_payload=300)
    got = run_parse(buf, offs, want=want)
    assert set(got) == set(want)
    check(got, _parse.expected(buf, offs), want)


def test_parse_large_batch_of_valid_segments():
    """200K segments of the common kinds (plain, NOP/MSS options, header-only) with 1460 B payloads."""
    rng = np.random.default_rng(0x52)
    kinds = ("plain", "nop_mss", "mss_eol", "header_only", "padding_bug")
    buf, offs, _ = _parse.batch(rng, 200_000, kinds=kinds, lead=2, max_payload=1460)
    got = run_parse(buf, offs)
    exp = _parse.expected(buf, offs)
    check(got, exp, "large")
    assert (got["status"] == 0).all()
