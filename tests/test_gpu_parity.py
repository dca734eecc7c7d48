"""GPU parity: every batch entry point, through the C ABI, bit-exact against
the oracle (integer work: no tolerance).  Run on the MI355X box:
    python -m pytest tests -m gpu -x -q
Covers the golden fixtures, the edge lengths (0..3 bytes, row boundaries at
128, the init-spill case L = 1..3 mod 128, MTUs, 65507-byte datagrams), odd
strides and alignments, datagrams at the very start of the buffer (windows
that would begin before d_base), empty datagrams and all-empty batches,
partial last batches, non-default streams, the verify (inbound) mode with
corrupted datagrams, the host streaming path, and the full 2^20 x 1400 B
configuration.
"""
import os

import numpy as np
import pytest

import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def P():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import litenetlibpp_amd as pkg
    pkg.lib()  # raises if the in-tree library is missing: no fallback
    return pkg


# Large CSR / verify batches (>= 16 Ki datagrams) take the product's large-batch
# path (crc32c_api.cpp, launch_csr); the shapes below were written against the
# experiment kernels too (pairs, segments, uniform batches: tools/kvariants.py)
# and stay as edge cases for whichever kernel is the product's.


def u32(t):
    return t.cpu().numpy().view(np.uint32)


def dev(a, dtype=torch.uint8):
    return torch.from_numpy(np.ascontiguousarray(a)).to(device="cuda", dtype=dtype)


def test_golden_fixed(P):
    data = np.fromfile(os.path.join(GOLD, "fixed_bytes.bin"), dtype=np.uint8)
    exp = np.fromfile(os.path.join(GOLD, "fixed_crc.u32"), dtype=np.uint32)
    got = u32(P.batch_fixed(dev(data), 1400, 1400, 64))
    assert np.array_equal(got, exp)


def test_golden_csr(P):
    data = np.fromfile(os.path.join(GOLD, "csr_bytes.bin"), dtype=np.uint8)
    off = np.fromfile(os.path.join(GOLD, "csr_offsets.u64"), dtype=np.uint64)
    exp = np.fromfile(os.path.join(GOLD, "csr_crc.u32"), dtype=np.uint32)
    got = u32(P.batch_csr(dev(data), dev(off.view(np.int64), torch.int64)))
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first at {bad[:5]}"


LENGTHS = [1, 2, 3, 4, 5, 8, 31, 100, 127, 128, 129, 130, 131, 255, 256, 257, 384, 1000, 1399,
           1400, 1401, 1427, 1428, 1431, 1432, 4096, 9000]


@pytest.mark.parametrize("length", LENGTHS)
def test_fixed_lengths(P, length):
    rng = np.random.default_rng(length)
    for stride, n in ((length, 1), (length, 63), (length + 3, 64), (length + 13, 130),
                      (max(length, 2048), 1000)):
        data = rng.integers(0, 256, (n - 1) * stride + length, dtype=np.uint8)
        exp = oracle.batch_fixed(data, stride, length, n)
        got = u32(P.batch_fixed(dev(data), stride, length, n))
        assert np.array_equal(got, exp), (length, stride, n)


# (stride, len): the lane-run plan (crc32c_run.hip, runs of K = 4) covers whole
# superblocks of 64 * max(4, 128 / gcd(stride, 128)) datagrams; the rest goes to
# the batch kernel.  Odd strides (superblock 8192), strides that are multiples of 128,
# gaps between datagrams (including gaps of whole rows), len = 129.
RUN_CASES = [(1400, 1400), (1401, 1401), (1432, 1432), (1408, 1408), (130, 129), (129, 129),
             (200, 129), (1500, 1400), (1600, 1400), (4096, 4000), (2048, 1400), (1404, 1400)]


@pytest.mark.parametrize("stride,length", RUN_CASES)
def test_fixed_lane_runs(P, stride, length):
    low = stride & -stride
    q = max(4, 1 if low >= 128 else 128 // low)
    sb = 64 * q
    rng = np.random.default_rng(stride * 7 + length)
    for m, extra, shift in ((1, 0, 0), (2, 5, 3), (3, sb - 1, 127), (1, 100, 64)):
        n = m * sb + extra
        data = rng.integers(0, 256, shift + (n - 1) * stride + length, dtype=np.uint8)
        d = dev(data)[shift:]
        exp = oracle.batch_fixed(data[shift:], stride, length, n)
        got = u32(P.batch_fixed(d, stride, length, n))
        bad = np.nonzero(got != exp)[0]
        assert bad.size == 0, (stride, length, n, shift, bad.size, bad[:5])


def test_fixed_lane_runs_persistent_waves(P):
    """More wave-batches than resident waves (6,144 against 2,048, and a
    leftover for the batch kernel): one batch per wave, the later workgroups
    started by the dispatcher as the first finish (round 5's uncapped grid;
    the experiments build's capped grid loops its waves over the batches)."""
    n = 3 * (1 << 19) + 777
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    d = torch.randint(0, 256, (n * 1400 + 1,), dtype=torch.uint8, device="cuda", generator=g)[1:]
    got = u32(P.batch_fixed(d, 1400, 1400, n))
    data = d.cpu().numpy()
    exp = oracle.batch_fixed(data, 1400, 1400, n)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, (bad.size, bad[:5])


def test_fixed_zero_length_and_empty_batch(P):
    data = torch.zeros(64, dtype=torch.uint8, device="cuda")
    out = torch.full((10,), -1, dtype=torch.int32, device="cuda")
    P.batch_fixed(data, 0, 0, 10, out=out)
    assert np.all(u32(out) == 0)
    assert P.batch_fixed(data, 16, 16, 0).numel() == 0


def random_csr(rng, n, max_len):
    """n datagrams of 0..max_len bytes, starting `lead` bytes into the buffer
    (off[0] != 0) with a few trailing bytes after the last one."""
    lens = rng.integers(0, max_len + 1, n)
    lead = int(rng.integers(0, 64))
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64) + np.uint64(lead)
    data = rng.integers(0, 256, int(off[-1]) + int(rng.integers(0, 17)), dtype=np.uint8)
    return data, off


@pytest.mark.parametrize("seed", range(6))
def test_csr_random(P, seed):
    rng = np.random.default_rng(100 + seed)
    n = [1, 64, 65, 1000, 5000, 20000][seed]
    data, off = random_csr(rng, n, [50, 300, 1500, 1500, 1432, 1400][seed])
    exp = oracle.batch_csr(data, off)
    got = u32(P.batch_csr(dev(data), dev(off.view(np.int64), torch.int64)))
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first at {bad[:5]}"


def test_csr_mixed_length_config3_shape(P):
    # BASELINE config 3 shape (64..1400 B uniform) at 2^16 datagrams
    rng = np.random.default_rng(43)
    lens = 64 + rng.integers(0, 1337, 1 << 16)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
    exp = oracle.batch_csr(data, off)
    got = u32(P.batch_csr(dev(data), dev(off.view(np.int64), torch.int64)))
    assert np.array_equal(got, exp)


def test_csr_bucketed_mix(P):
    """Batches large enough for the line-count bucketing pre-pass
    (crc32c_bucket.hip): empty, 1..3-byte, line-crossing and very long
    datagrams (line-count bucket 63) mixed, buffer not line-aligned."""
    rng = np.random.default_rng(21)
    n = 40000
    lens = rng.integers(0, 1433, n)
    lens[rng.integers(0, n, 3000)] = 0
    lens[rng.integers(0, n, 3000)] = rng.integers(1, 4, 3000)
    lens[rng.integers(0, n, 20)] = rng.integers(8000, 70000, 20)
    lead = 77
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64) + np.uint64(lead)
    data = rng.integers(0, 256, int(off[-1]) + 9, dtype=np.uint8)
    exp = oracle.batch_csr(data, off)
    d = dev(np.concatenate([np.zeros(5, np.uint8), data]))[5:]
    got = u32(P.batch_csr(d, dev(off.view(np.int64), torch.int64)))
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first at {bad[:5]}"


@pytest.mark.parametrize("case", ["odd_n", "tiny", "line_multiples", "overflow_heavy"])
def test_csr_span_shared_lines(P, case):
    """CSR batches through the product path (the span kernel and its overflow
    batch kernel; shapes first written for round 1's pair kernel): an odd
    count, runs of tiny datagrams sharing one line (several boundaries per lane
    and row), lengths ending exactly on line boundaries, and one datagram in
    eight long enough to cross three segments (the overflow list)."""
    rng = np.random.default_rng(["odd_n", "tiny", "line_multiples", "overflow_heavy"].index(case) + 300)
    n = {"odd_n": 30001, "tiny": 50000, "line_multiples": 20000, "overflow_heavy": 20000}[case]
    if case == "tiny":
        lens = rng.integers(0, 12, n)
    elif case == "line_multiples":
        lens = 128 * rng.integers(0, 12, n) + rng.choice([0, 0, 0, 1, 127], n)
    elif case == "overflow_heavy":
        lens = rng.integers(0, 1433, n)
        lens[rng.integers(0, n, n // 8)] = rng.integers(1900, 4000, n // 8)
    else:
        lens = rng.integers(0, 1433, n)
    lead = int(rng.integers(0, 128))
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64) + np.uint64(lead)
    data = rng.integers(0, 256, int(off[-1]) + 3, dtype=np.uint8)
    exp = oracle.batch_csr(data, off)
    got = u32(P.batch_csr(dev(data), dev(off.view(np.int64), torch.int64)))
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"{case}: {bad.size} mismatches, first at {bad[:5]}"


@pytest.mark.parametrize("case", ["segment_multiples", "line_multiples", "lead_and_tail", "tiny_excess"])
def test_csr_span_segment_edges(P, case):
    """CSR batches through the product path (the span kernel), at its segment
    edges: datagram ends on segment boundaries (lengths of 2 KiB multiples,
    the segment size of batches this small), on line boundaries, a batch that
    starts and ends mid-line, and segments with more than 16 ends (queue
    refills)."""
    rng = np.random.default_rng(["segment_multiples", "line_multiples", "lead_and_tail", "tiny_excess"].index(case) + 500)
    n = 40000
    if case == "segment_multiples":
        lens = 2048 * rng.integers(1, 4, n) - rng.choice([0, 0, 1], n)
    elif case == "line_multiples":
        lens = 128 * rng.integers(0, 13, n)
    elif case == "tiny_excess":
        lens = np.where(rng.random(n) < 0.7, rng.integers(0, 20, n), rng.integers(20, 1433, n))
    else:
        lens = rng.integers(0, 1433, n)
    lead = 0 if case == "segment_multiples" else int(rng.integers(1, 128))
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64) + np.uint64(lead)
    data = rng.integers(0, 256, int(off[-1]) + 77, dtype=np.uint8)
    exp = oracle.batch_csr(data, off)
    got = u32(P.batch_csr(dev(data), dev(off.view(np.int64), torch.int64)))
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"{case}: {bad.size} mismatches, first at {bad[:5]}"


def test_csr_span_several_wave_batches_per_wave(P):
    """A batch larger than one segment per lane at the largest segment size
    (> 2 GiB on 256 CUs): waves take several wave-batches."""
    rng = np.random.default_rng(600)
    n = 1_700_000
    lens = rng.integers(1200, 1433, n)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    g = torch.Generator(device="cuda")
    g.manual_seed(601)
    d = torch.randint(0, 256, (int(off[-1]),), dtype=torch.uint8, device="cuda", generator=g)
    got = u32(P.batch_csr(d, dev(off.view(np.int64), torch.int64)))
    exp = oracle.batch_csr(d.cpu().numpy(), off)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first at {bad[:5]}"


def test_csr_span_dense_small_datagrams(P):
    """1.2 M datagrams of 0-39 bytes (~24 MB): dense wave-batches whose offset
    window does not reach their end (global-memory searches for those lanes),
    many boundaries per row."""
    rng = np.random.default_rng(404)
    n = 1_200_000
    lens = rng.integers(0, 40, n)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = rng.integers(0, 256, int(off[-1]) + 1, dtype=np.uint8)
    exp = oracle.batch_csr(data, off)
    got = u32(P.batch_csr(dev(data), dev(off.view(np.int64), torch.int64)))
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first at {bad[:5]}"


@pytest.mark.parametrize("order", ["small_first", "large_first"])
def test_csr_span_skewed_density(P, order):
    """A batch whose datagram density changes half way (tiny datagrams, then
    MTU-sized ones, or the reverse): an index interpolated from a byte position
    misses by hundreds of thousands of datagrams, so the setup's windows are
    found by the fallback searches (probe, 64-ary search), not the first guess."""
    rng = np.random.default_rng(["small_first", "large_first"].index(order) + 410)
    n_small, n_large = 700_000, 500_000
    small = rng.integers(0, 40, n_small)
    large = rng.integers(1000, 1433, n_large)
    lens = np.concatenate([small, large] if order == "small_first" else [large, small])
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64) + np.uint64(17)
    g = torch.Generator(device="cuda")
    g.manual_seed(411)
    d = torch.randint(0, 256, (int(off[-1]) + 5,), dtype=torch.uint8, device="cuda", generator=g)
    got = u32(P.batch_csr(d, dev(off.view(np.int64), torch.int64)))
    exp = oracle.batch_csr(d.cpu().numpy(), off)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"{order}: {bad.size} mismatches, first at {bad[:5]}"


def test_verify_mode_bucketed(P):
    rng = np.random.default_rng(22)
    n = 30000
    lens = rng.integers(0, 1433, n)
    lens[::13] = rng.integers(0, 5, lens[::13].size)   # runts
    body_off = np.concatenate([[0], np.cumsum(lens + 4)])[:-1].astype(np.uint64)
    wire = np.empty(int(np.sum(lens + 4)), np.uint8)
    bodies = rng.integers(0, 256, int(np.sum(lens)), dtype=np.uint8)
    boff = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    crcs = oracle.batch_csr(bodies, boff)
    for i in range(n):
        o, L = int(body_off[i]), int(lens[i])
        wire[o:o + L] = bodies[int(boff[i]):int(boff[i]) + L]
        wire[o + L:o + L + 4] = np.frombuffer(int(crcs[i]).to_bytes(4, "little"), np.uint8)
    corrupt = rng.integers(0, n, 500)
    for i in corrupt:
        o, L = int(body_off[i]), int(lens[i]) + 4
        wire[o + int(rng.integers(0, L))] ^= np.uint8(1 << int(rng.integers(0, 8)))
    off = np.concatenate([body_off, [wire.size]]).astype(np.uint64)
    want = np.zeros(n, bool)
    want_crc = np.zeros(n, np.uint32)
    tot = lens + 4
    for i in range(n):
        o, T = int(off[i]), int(tot[i])
        if T >= 5:
            want_crc[i] = oracle.crc(wire[o:o + T - 4])
            want[i] = int(want_crc[i]) == int.from_bytes(wire[o + T - 4:o + T].tobytes(), "little")
    ok, crc = P.verify_csr(dev(wire), dev(off.view(np.int64), torch.int64), want_crc=True)
    assert np.array_equal(ok.cpu().numpy().astype(bool), want)
    big = tot >= 5
    assert np.array_equal(u32(crc)[big], want_crc[big])


def _wire_batch(rng, n, corrupt_frac=0.2):
    """n wire datagrams (body || LE32 CRC) with random header bytes and short
    bodies around every verify() threshold (empty bodies give 4-byte runts),
    some corrupted."""
    lens = np.where(rng.random(n) < 0.5, rng.integers(0, 30, n), rng.integers(0, 1429, n))
    bodies = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    wire = np.empty(int(lens.sum()) + 4 * n, np.uint8)
    off = np.zeros(n + 1, np.uint64)
    pos = bpos = 0
    for i, L in enumerate(lens):
        body = bodies[bpos:bpos + L]
        bpos += L
        wire[pos:pos + L] = body
        wire[pos + L:pos + L + 4] = np.frombuffer(np.uint32(oracle.crc(body)).tobytes(), np.uint8)
        if rng.random() < corrupt_frac:
            wire[pos + int(rng.integers(0, L + 4))] ^= np.uint8(1 << int(rng.integers(0, 8)))
        pos += L + 4
        off[i + 1] = pos
    return wire, off


@pytest.mark.parametrize("n", [1000, 40000])
def test_inbound_filter(P, n):
    """lnl_inbound_filter_csr_dev: CRC layer, then net_packet::verify() of the
    stripped packet (reference-pinned restatement, tests/test_packet_verify.py),
    per datagram, on every CSR path (n = 1000 takes the unbucketed kernel)."""
    rng = np.random.default_rng(77 + n)
    wire, off = _wire_batch(rng, n)
    exp = np.array([oracle.inbound_status(wire[int(off[i]):int(off[i + 1])]) for i in range(n)], np.uint8)
    got = P.inbound_filter(dev(wire), dev(off.view(np.int64), torch.int64)).cpu().numpy()
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first at {bad[:5]}: got {got[bad[:5]]} exp {exp[bad[:5]]}"
    assert set(np.unique(exp)) == {0, 1, 2}


def test_full_config3_bit_exact(P):
    # BASELINE config 3 at full size: 2^20 datagrams of 64..1400 B, CSR
    rng = np.random.default_rng(43)
    lens = 64 + rng.integers(0, 1337, 1 << 20)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    g = torch.Generator(device="cuda")
    g.manual_seed(44)
    d = torch.randint(0, 256, (int(off[-1]),), dtype=torch.uint8, device="cuda", generator=g)
    got = u32(P.batch_csr(d, dev(off.view(np.int64), torch.int64)))
    exp = oracle.batch_csr(d.cpu().numpy(), off)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first at {bad[:5]}"


def test_csr_empty_datagrams_and_all_empty_batches(P):
    rng = np.random.default_rng(7)
    lens = np.zeros(300, np.int64)
    lens[200:] = rng.integers(0, 300, 100)   # batches 0..2 all empty, then mixed
    lens[150] = 5
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = rng.integers(0, 256, max(int(off[-1]), 1), dtype=np.uint8)
    exp = oracle.batch_csr(data, off)
    got = u32(P.batch_csr(dev(data), dev(off.view(np.int64), torch.int64)))
    assert np.array_equal(got, exp)


def test_csr_large_datagrams(P):
    rng = np.random.default_rng(8)
    lens = np.array([65507, 0, 1, 65535, 100000, 7, 128 * 300 + 1], np.int64)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
    exp = oracle.batch_csr(data, off, bitwise=True)
    got = u32(P.batch_csr(dev(data), dev(off.view(np.int64), torch.int64)))
    assert np.array_equal(got, exp)


def test_near_base_datagrams(P):
    # many short datagrams inside the first 128 bytes of the buffer: their first
    # row window starts before d_base and is filled lane-by-lane
    rng = np.random.default_rng(9)
    lens = rng.integers(0, 40, 200)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
    exp = oracle.batch_csr(data, off)
    got = u32(P.batch_csr(dev(data), dev(off.view(np.int64), torch.int64)))
    assert np.array_equal(got, exp)
    # and the fixed-stride form with stride < 128
    for stride, length in ((16, 16), (40, 33), (127, 100)):
        n = 300
        d = rng.integers(0, 256, (n - 1) * stride + length, dtype=np.uint8)
        assert np.array_equal(u32(P.batch_fixed(dev(d), stride, length, n)),
                              oracle.batch_fixed(d, stride, length, n))


def test_non_default_stream_and_async(P):
    rng = np.random.default_rng(10)
    data = dev(rng.integers(0, 256, 4096 * 1400, dtype=np.uint8))
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        out = P.batch_fixed(data, 1400, 1400, 4096, stream=s)
    s.synchronize()
    exp = oracle.batch_fixed(data.cpu().numpy(), 1400, 1400, 4096)
    assert np.array_equal(u32(out), exp)


def test_verify_mode(P):
    rng = np.random.default_rng(11)
    n = 3000
    blobs, want = [], []
    for i in range(n):
        L = int(rng.integers(0, 1433))
        body = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        wire = P.Crc32cLayer().process_outbound(body)
        if i % 7 == 3 and L > 0:
            b = bytearray(wire)
            b[int(rng.integers(0, len(b)))] ^= 1 << int(rng.integers(0, 8))
            wire = bytes(b)
        if i % 11 == 5:
            wire = wire[: int(rng.integers(0, 5))]   # runt datagram
        blobs.append(wire)
        want.append(P.Crc32cLayer().process_inbound(wire) is not None)
    lens = np.array([len(b) for b in blobs], np.int64)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = np.frombuffer(b"".join(blobs), dtype=np.uint8)
    ok, crc = P.verify_csr(dev(data), dev(off.view(np.int64), torch.int64), want_crc=True)
    assert np.array_equal(ok.cpu().numpy().astype(bool), np.array(want))
    body_off = off[:-1]
    body_len = np.maximum(lens - 4, 0)
    long_enough = lens >= 5
    exp = np.array([oracle.crc(data[int(o):int(o) + int(L)]) for o, L in zip(body_off, body_len)],
                   np.uint32)
    assert np.array_equal(u32(crc)[long_enough], exp[long_enough])


def test_host_streaming_path(P):
    rng = np.random.default_rng(12)
    lens = rng.integers(0, 1433, 200_000)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64) + np.uint64(5)
    data = rng.integers(0, 256, int(off[-1]) + 3, dtype=np.uint8)
    exp = oracle.batch_csr(data, off)
    assert np.array_equal(P.batch_host(data, off, 0), exp)
    pinned = torch.from_numpy(data).pin_memory()
    assert np.array_equal(P.batch_host(pinned.numpy(), off, 0), exp)


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_host_multi_device_path(P, devices):
    """lnl_crc32c_batch_host_multi: contiguous ranges of ceil(n / ndev), one
    host thread each (one GPU on the test box: the same device listed several
    times), nonzero first offset, n not a multiple of ndev."""
    rng = np.random.default_rng(31 + len(devices))
    n = 70001
    lens = rng.integers(0, 1433, n)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64) + np.uint64(13)
    data = rng.integers(0, 256, int(off[-1]) + 5, dtype=np.uint8)
    pinned = torch.from_numpy(data).pin_memory().numpy()
    got = P.batch_host_multi(pinned, off, devices)
    assert np.array_equal(got, oracle.batch_csr(data, off))


@pytest.mark.parametrize("receivers,egress", [(1, 0), (3, 0), (1, 1), (2, 1)])
def test_socket_example_receivers(P, receivers, egress):
    """examples/socket_path (built by build()): R SO_REUSEPORT receive sockets,
    one thread and pinned burst buffer each, GPU filter per burst; every GPU
    status equals lnl_inbound_status on the CPU (exit code 3 otherwise).  With
    --egress 1 the senders run the product's send side per burst
    (lnl_crc32c_append_host, then lnl_egress_send_batch)."""
    import json
    import subprocess
    exe = os.path.join(ROOT, "examples", "socket_path")
    if not os.path.exists(exe):
        pytest.fail("examples/socket_path not built (run __graft_entry__.build())")
    r = subprocess.run([exe, "--count", "30000", "--burst", "1024", "--receivers", str(receivers),
                        "--egress", str(egress)], capture_output=True, text=True, timeout=90)
    assert r.returncode == 0, r.stderr
    j = json.loads(r.stdout.strip().splitlines()[-1])
    assert j["gpu_cpu_mismatch"] == 0 and j["receivers"] == receivers
    assert j["received"] >= 0.5 * j["sent"] and j["accept"] > 0 and j["drop_crc"] > 0
    if egress:
        assert j["egress"] and j["tx_payload_bytes"] > 0 and j["append_host_gbps"] > 0


def test_socket_path_end_to_end(P):
    """Config 5 over real sockets: wire datagrams sent over UDP loopback,
    received in recvmmsg bursts into a pinned buffer (lnl_ingress_recv_batch),
    filtered on the GPU (lnl_inbound_filter_host) -- statuses equal the
    oracle's per datagram."""
    import socket
    rng = np.random.default_rng(55)
    rx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rx.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 1 << 23)
    rx.bind(("127.0.0.1", 0))
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    tx.connect(rx.getsockname())
    layer = P.Crc32cLayer()
    sent = []
    for i in range(3000):
        body = rng.integers(0, 256, int(rng.integers(0, 1428)), dtype=np.uint8)
        if body.size:
            body[0] = rng.choice([0x00, 0x01, 0x81, 0x05, 0x1F])
        w = bytearray(layer.process_outbound(body.tobytes()))
        if i % 17 == 0:
            w[int(rng.integers(0, len(w)))] ^= 0x10
        sent.append(bytes(w))
        tx.send(bytes(w))
    burst = 256
    buf = torch.empty(burst * P.INGRESS_SLOT, dtype=torch.uint8).pin_memory().numpy()
    got_status, got_wire = [], []
    while len(got_wire) < len(sent):
        n, off = P.ingress_recv_batch(rx.fileno(), buf, burst, wait_ms=2000)
        assert n > 0, f"timed out after {len(got_wire)}"
        got_status += list(P.inbound_filter_host(buf, off, 0))
        got_wire += [bytes(buf[int(off[i]):int(off[i + 1])]) for i in range(n)]
    rx.close()
    tx.close()
    assert got_wire == sent
    exp = [oracle.inbound_status(np.frombuffer(w, np.uint8)) for w in sent]
    assert got_status == exp and set(exp) == {0, 1, 2}


@pytest.mark.parametrize("n,shift", [(1, 0), (777, 3), (200_000, 11)])
def test_append_host_matches_layer_outbound(P, n, shift):
    """lnl_crc32c_append_host (pinned payload burst -> H2D -> CRC + append ->
    D2H, chunks over the default 4 streams; 200,000 datagrams take several chunks): every
    wire byte equals lnl_crc32c_layer_outbound of its payload, back to back, and
    the CRCs equal the oracle's.  Nonzero first offset."""
    rng = np.random.default_rng(400 + n)
    lens = rng.integers(0, 1429, n)
    lens[: min(n, 4)] = [0, 1, 1428, 64][: min(n, 4)]
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64) + np.uint64(shift)
    data = rng.integers(0, 256, int(off[-1]) + 7, dtype=np.uint8)
    pinned = torch.from_numpy(data).pin_memory().numpy()
    wire, woff, crc = P.append_host(pinned, off, 0, want_crc=True)
    exp = oracle.batch_csr(data, off)
    assert np.array_equal(crc, exp)
    assert wire.size == int(off[-1] - off[0]) + 4 * n
    assert np.array_equal(np.diff(woff.astype(np.int64)), lens + 4)
    crcpos = woff[1:].astype(np.int64) - 4
    keep = np.ones(wire.size, dtype=bool)
    for j in range(4):
        keep[crcpos + j] = False
    assert np.array_equal(wire[keep], data[int(off[0]):int(off[-1])])
    assert np.array_equal(wire[crcpos[:, None] + np.arange(4)[None, :]].reshape(-1), exp.astype("<u4").view(np.uint8))
    layer = P.Crc32cLayer()
    for i in list(range(min(n, 50))) + [n - 1]:
        w = bytes(wire[int(woff[i]):int(woff[i + 1])])
        assert w == layer.process_outbound(data[int(off[i]):int(off[i + 1])].tobytes())


def test_append_host_egress_loopback(P):
    """The send half of the socket path end to end:
    payload bursts in pinned memory -> lnl_crc32c_append_host -> one
    lnl_egress_send_batch (sendmmsg) per burst over UDP loopback ->
    lnl_ingress_recv_batch on the receiver.  Every received datagram equals
    lnl_crc32c_layer_outbound of its payload and passes lnl_inbound_status (and
    the GPU filter)."""
    import socket
    rng = np.random.default_rng(808)
    rx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rx.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 1 << 23)
    rx.bind(("127.0.0.1", 0))
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    layer = P.Crc32cLayer()
    burst, bursts = 48, 25
    rbuf = torch.empty(burst * P.INGRESS_SLOT, dtype=torch.uint8).pin_memory().numpy()
    sent_payloads, got = [], []
    for b in range(bursts):
        lens = rng.integers(16, 1429, burst)  # >= every header the chosen bytes need
        off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        data = torch.from_numpy(rng.integers(0, 256, int(off[-1]), dtype=np.uint8)).pin_memory().numpy()
        data[off[:-1].astype(np.int64)] = rng.choice([0x00, 0x01, 0x81], burst)  # header bytes verify() accepts
        wire, woff = P.append_host(data, off, 0)
        r, st = P.egress_send_batch(tx.fileno(), wire, woff, addrs=rx.getsockname())
        assert r == burst and bool((st == lens + 4).all())
        sent_payloads += [data[int(off[i]):int(off[i + 1])].tobytes() for i in range(burst)]
        k = 0
        while k < burst:
            n, roff = P.ingress_recv_batch(rx.fileno(), rbuf, burst, wait_ms=2000)
            assert n > 0, f"timed out in burst {b} after {k}"
            st_gpu = P.inbound_filter_host(rbuf, roff, 0)
            assert bool((st_gpu == P.INBOUND_ACCEPT).all())
            got += [bytes(rbuf[int(roff[i]):int(roff[i + 1])]) for i in range(n)]
            k += n
    rx.close()
    tx.close()
    assert len(got) == len(sent_payloads)
    for p, w in zip(sent_payloads, got):
        assert w == layer.process_outbound(p)
        assert P.inbound_status(w) == P.INBOUND_ACCEPT


@pytest.mark.parametrize("replicas,fused", [(1, False), (1, True), (150, False), (150, True)])
@pytest.mark.parametrize("tail", ["datagram", "zero", "layer"])
def test_dispatch_reference_fixture(P, replicas, fused, tail):
    """The MERGED cut against the REFERENCE's own process_packet
    (tests/golden/dispatch_ref*.json, made by running the reference's
    net_manager: tests/golden/make_dispatch_ref.py): every container of the
    fixture, as a wire datagram with its CRC, through lnl_inbound_filter_csr_dev
    + lnl_dispatch_csr_dev_ex or the fused lnl_inbound_filter_dispatch_csr_dev_ex;
    the packets each container gives (their in-burst bytes, then the zero fill
    of d_pkt_avail), handed to the caller's process_packet (oracle.deliver),
    must be exactly what the reference delivered:
      zero   every delivery of the plain reference (dispatch_ref.json), the
             zero-padded packets included (LNL_DISPATCH_TAIL_ZERO)
      layer  every delivery of the reference with INTEGRATION.md's layer
             compiled in (dispatch_ref_layer.json: the CRC field, then zeros;
             LNL_DISPATCH_TAIL_LAYER)
      datagram  the default rule: the deliveries before the first read past
             the datagram, and all of them for every other container.
    150 replicas (17,250 datagrams, shuffled) take the span path."""
    from test_dispatch_ref import expected, load_fixture, packet_bytes, reference_deliveries, with_crc
    mode = {"datagram": P.DISPATCH_TAIL_DATAGRAM, "zero": P.DISPATCH_TAIL_ZERO, "layer": P.DISPATCH_TAIL_LAYER}[tail]
    cont, conn, recs = load_fixture("layer" if tail == "layer" else "plain")
    rng = np.random.default_rng(60 + replicas)
    order = np.concatenate([rng.permutation(len(cont)) for _ in range(replicas)])
    wires = [with_crc(cont[k]) for k in order]
    lead = int(rng.integers(0, 64))
    off = np.concatenate([[0], np.cumsum([len(w) for w in wires])]).astype(np.uint64) + np.uint64(lead)
    data = np.frombuffer(bytes(lead) + b"".join(wires) + bytes(5), dtype=np.uint8)
    d, o = dev(data), dev(off.view(np.int64), torch.int64)
    if fused:
        status, start, length, parent, avail = P.filter_dispatch(d, o, tail=mode, avail=True)
    else:
        status = P.inbound_filter(d, o)
        start, length, parent, avail = P.dispatch(d, o, status, tail=mode, avail=True)
    assert bool((status == P.INBOUND_ACCEPT).all())
    got = [[] for _ in wires]
    padded = 0
    for s0, L, i, av in zip(start.cpu().numpy(), length.cpu().numpy(), parent.cpu().numpy(), avail.cpu().numpy()):
        assert 0 <= av <= L
        padded += int(av < L)
        got[int(i)] += oracle.deliver(packet_bytes(data, int(s0), int(L), int(av)), conn, ref_tail=mode != 0)
    want = [reference_deliveries(recs[k]) if mode else expected(recs[k]) for k in order]
    bad = [j for j in range(len(wires)) if got[j] != want[j]]
    assert not bad, [(j, int(order[j])) for j in bad[:8]]
    assert (padded > 0) == (mode != 0)


def _merged(rng, parts, mode):
    """A MERGED container (header 0x0C) of sub-packets as net_peer::send_merged
    lays them out ([u16 LE size][packet]...), optionally damaged."""
    out = bytearray([0x0C])
    for body in parts:
        out += len(body).to_bytes(2, "little") + body
    if mode == "truncated" and len(out) > 4:
        out = out[: int(rng.integers(2, len(out)))]
    elif mode == "bad_sub" and parts:
        k = 1 + 2                                      # first sub-packet's header byte
        out[k] = 0x1F                                  # unknown property: verify() fails
    elif mode == "zero_len":
        out += (0).to_bytes(2, "little") + bytes([0x00, 0x01])
    return bytes(out)


@pytest.mark.parametrize("n", [500, 30000])
def test_dispatch_merged_containers(P, n):
    """lnl_dispatch_csr_dev after lnl_inbound_filter_csr_dev: accepted
    datagrams and the packets of MERGED containers (well-formed, truncated,
    with a rejected sub-packet, a zero-length entry, nested), in datagram
    order, against oracle.dispatch (net_peer.cpp:164-187 restated)."""
    rng = np.random.default_rng(900 + n)
    layer = P.Crc32cLayer()
    wires = []
    for i in range(n):
        r = rng.random()
        if r < 0.5:
            parts = [bytes([int(rng.choice([0x00, 0x01, 0x03]))]) +
                     rng.integers(0, 256, int(rng.integers(3, 60)), dtype=np.uint8).tobytes()
                     for _ in range(int(rng.integers(0, 12)))]
            mode = rng.choice(["ok", "ok", "ok", "truncated", "bad_sub", "zero_len"])
            body = _merged(rng, parts, mode)
            if rng.random() < 0.05:                        # nested container: delivered whole
                body = _merged(rng, [body], "ok")
        else:
            body = bytes([int(rng.choice([0x00, 0x01, 0x1F]))]) + \
                rng.integers(0, 256, int(rng.integers(0, 200)), dtype=np.uint8).tobytes()
        w = bytearray(layer.process_outbound(body))
        if rng.random() < 0.03:
            w[int(rng.integers(0, len(w)))] ^= 0x04
        wires.append(bytes(w))
    off = np.concatenate([[0], np.cumsum([len(w) for w in wires])]).astype(np.uint64)
    blob = np.frombuffer(b"".join(wires), np.uint8)
    d, o = dev(blob), dev(off.view(np.int64), torch.int64)
    status = P.inbound_filter(d, o)
    start, length, parent = P.dispatch(d, o, status)
    st = status.cpu().numpy()
    exp = oracle.dispatch([np.frombuffer(w, np.uint8) for w in wires], st)
    got = list(zip(parent.cpu().numpy().tolist(),
                   (start.cpu().numpy() - off[parent.cpu().numpy()].astype(np.int64)).tolist(),
                   length.cpu().numpy().tolist()))
    assert got == exp
    assert any(L for (_, pos, L) in exp if pos > 0)        # some container packets delivered
    # a capped call writes the first `cap` packets and still reports the total
    s2, l2, p2 = P.dispatch(d, o, status, cap=7)
    assert p2.cpu().numpy().tolist() == [e[0] for e in exp[:7]]


def _tail_wires(P, rng, n):
    """Containers whose walk runs past the datagram in every way the tail
    rules see: truncated entries, a size field in the last byte, a last
    entry longer than what is left, entries reaching past the 2048-byte
    capacity, more than 8 entries before the cut, nested containers, plain
    datagrams and corrupted CRCs."""
    layer = P.Crc32cLayer()
    sub = lambda m: bytes([int(rng.choice([0x00, 0x01, 0x03]))]) + \
        rng.integers(0, 256, max(m - 1, 0), dtype=np.uint8).tobytes()
    wires = []
    for _ in range(n):
        r = rng.random()
        if r < 0.7:
            parts = [sub(int(rng.integers(1, 90))) for _ in range(int(rng.integers(0, 12)))]
            body = bytearray(_merged(rng, parts, "ok"))
            kind = rng.integers(0, 6)
            if kind == 0 and len(body) > 2:
                body = body[:int(rng.integers(2, len(body)))]            # truncated anywhere
            elif kind == 1:
                body += bytes([int(rng.integers(0, 256))])              # size field in the last byte
            elif kind == 2:
                body += int(rng.integers(1, 3000)).to_bytes(2, "little") + sub(int(rng.integers(0, 5)))
            elif kind == 3:
                body += int(rng.integers(1, 8)).to_bytes(2, "little")   # a size field, nothing after it
            body = bytes(body)
            if rng.random() < 0.05:
                body = _merged(rng, [body], "ok")
        else:
            body = sub(int(rng.integers(0, 300)))
        w = bytearray(layer.process_outbound(body))
        if rng.random() < 0.02:
            w[int(rng.integers(0, len(w)))] ^= 0x10
        wires.append(bytes(w))
    return wires


@pytest.mark.parametrize("tail", ["zero", "layer"])
@pytest.mark.parametrize("n", [500, 30000])
def test_dispatch_tail_rules(P, n, tail):
    """lnl_dispatch_csr_dev_ex and lnl_inbound_filter_dispatch_csr_dev_ex under
    the reference's tail rules (the walk bounded by the zero-filled 2048-byte
    buffer, net_peer.cpp:167-183): every packet's start, length and in-burst
    bytes equal oracle.dispatch_ex's, and the datagram rule still gives
    oracle.dispatch's packets on the same burst."""
    mode = P.DISPATCH_TAIL_ZERO if tail == "zero" else P.DISPATCH_TAIL_LAYER
    rng = np.random.default_rng(3100 + n + mode)
    wires = _tail_wires(P, rng, n)
    off = np.concatenate([[0], np.cumsum([len(w) for w in wires])]).astype(np.uint64)
    # the bytes after the batch read as a container: a tail walk must never take them
    trail = bytes([0x0C]) + b"".join(bytes([1, 0, 0]) for _ in range(40))
    blob = np.frombuffer(b"".join(wires) + trail, np.uint8)
    d, o = dev(blob), dev(off.view(np.int64), torch.int64)
    status = P.inbound_filter(d, o)
    st = status.cpu().numpy()
    exp = oracle.dispatch_ex([np.frombuffer(w, np.uint8) for w in wires], st, mode)
    assert sum(1 for e in exp if e[3] < e[2]) > n // 100          # zero-padded packets occur
    for fused in (False, True):
        if fused:
            st2, start, length, parent, avail = P.filter_dispatch(d, o, tail=mode, avail=True)
            assert torch.equal(st2, status)
        else:
            start, length, parent, avail = P.dispatch(d, o, status, tail=mode, avail=True)
        got = [e + (int(a),) for e, a in zip(_packets(off, start, length, parent), avail.cpu().numpy())]
        assert got == exp, next(((k, g, e) for k, (g, e) in enumerate(zip(got, exp)) if g != e), None)
    # the default rule on the same burst: the datagram-bounded cut, avail == len
    s3, l3, p3, a3 = P.filter_dispatch(d, o, avail=True)[1:]
    assert _packets(off, s3, l3, p3) == oracle.dispatch([np.frombuffer(w, np.uint8) for w in wires], st)
    assert torch.equal(a3, l3)
    with pytest.raises(ValueError):
        P.dispatch(d, o, status, tail=7)


def test_dispatch_records_and_rewalk(P):
    """The emit pass's two sources: containers of <= 8 packets come from the
    counting walk's records, longer ones and datagrams of >= 64 KiB (16-bit
    record positions) are walked again; all in datagram order."""
    rng = np.random.default_rng(77)
    layer = P.Crc32cLayer()
    sub = lambda m: bytes([0x00]) + rng.integers(0, 256, m - 1, dtype=np.uint8).tobytes()
    bodies = [_merged(rng, [sub(30000) for _ in range(3)], "ok"),      # 90 KB, 3 packets
              _merged(rng, [sub(20) for _ in range(8)], "ok"),         # exactly 8 records
              _merged(rng, [sub(20) for _ in range(9)], "ok"),         # one more: re-walk
              _merged(rng, [sub(7) for _ in range(400)], "ok"),
              bytes([0x01]) + sub(70000)]                              # plain, >= 64 KiB
    wires = [bytes(layer.process_outbound(b)) for b in bodies] * 50
    off = np.concatenate([[0], np.cumsum([len(w) for w in wires])]).astype(np.uint64)
    blob = np.frombuffer(b"".join(wires), np.uint8)
    d, o = dev(blob), dev(off.view(np.int64), torch.int64)
    status = P.inbound_filter(d, o)
    start, length, parent = P.dispatch(d, o, status)
    exp = oracle.dispatch([np.frombuffer(w, np.uint8) for w in wires], status.cpu().numpy())
    got = list(zip(parent.cpu().numpy().tolist(),
                   (start.cpu().numpy() - off[parent.cpu().numpy()].astype(np.int64)).tolist(),
                   length.cpu().numpy().tolist()))
    assert got == exp and len(exp) == 50 * (3 + 8 + 9 + 400 + 1)


def _packets(off, start, length, parent):
    par = parent.cpu().numpy()
    return list(zip(par.tolist(), (start.cpu().numpy() - off[par].astype(np.int64)).tolist(),
                    length.cpu().numpy().tolist()))


def _fused_vs_two_calls(P, wires, cap_check=True):
    """lnl_inbound_filter_dispatch_csr_dev against lnl_inbound_filter_csr_dev +
    lnl_dispatch_csr_dev and against oracle.inbound_status / oracle.dispatch."""
    off = np.concatenate([[0], np.cumsum([len(w) for w in wires])]).astype(np.uint64)
    # bytes after the batch that read as a MERGED container: nothing may walk them
    trail = bytes([0x0C]) + b"".join(bytes([1, 0, 0]) for _ in range(40))
    blob = np.frombuffer(b"".join(wires) + trail, np.uint8)
    d, o = dev(blob), dev(off.view(np.int64), torch.int64)
    status, start, length, parent = P.filter_dispatch(d, o)
    st2 = P.inbound_filter(d, o)
    s2, l2, p2 = P.dispatch(d, o, st2)
    st = status.cpu().numpy()
    assert np.array_equal(st, st2.cpu().numpy())
    exp_st = np.array([oracle.inbound_status(np.frombuffer(w, np.uint8)) for w in wires], np.uint8)
    bad = np.nonzero(st != exp_st)[0]
    assert bad.size == 0, f"{bad.size} status mismatches, first at {bad[:5]}"
    got = _packets(off, start, length, parent)
    assert got == _packets(off, s2, l2, p2)
    exp = oracle.dispatch([np.frombuffer(w, np.uint8) for w in wires], st)
    assert got == exp
    if cap_check:
        _, _, _, p3 = P.filter_dispatch(d, o, cap=11)
        assert p3.cpu().numpy().tolist() == [e[0] for e in exp[:11]]
    return exp


@pytest.mark.parametrize("n", [20000, 120000])
def test_filter_dispatch_fused(P, n):
    """Filter + dispatch in one pass (the span kernel walks each MERGED
    container while its bytes are in LDS): same statuses and packets as the two
    calls, and as the oracle, for well-formed, truncated, rejected-entry,
    zero-length-entry and nested containers, plain datagrams, runts and
    corrupted CRCs; containers long enough to cross segments (and, at n =
    20000, three or more of them: 2 KiB segments) and entries that straddle rows."""
    rng = np.random.default_rng(4242 + n)
    layer = P.Crc32cLayer()
    wires = []
    for i in range(n):
        r = rng.random()
        if r < 0.55:
            big = rng.random() < 0.1
            parts = [bytes([int(rng.choice([0x00, 0x01, 0x03]))]) +
                     rng.integers(0, 256, int(rng.integers(3, 700 if big else 60)), dtype=np.uint8).tobytes()
                     for _ in range(int(rng.integers(0, 12)))]
            mode = rng.choice(["ok", "ok", "ok", "truncated", "bad_sub", "zero_len"])
            body = _merged(rng, parts, mode)
            if rng.random() < 0.05:
                body = _merged(rng, [body], "ok")
        elif r < 0.6:
            body = bytes(int(rng.integers(0, 4)))                                   # runts
        else:
            body = bytes([int(rng.choice([0x00, 0x01, 0x1F, 0x8C]))]) + \
                rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8).tobytes()
        w = bytearray(layer.process_outbound(body))
        if rng.random() < 0.03:
            w[int(rng.integers(0, len(w)))] ^= 0x04
        wires.append(bytes(w))
    exp = _fused_vs_two_calls(P, wires)
    assert sum(1 for (_, pos, _) in exp if pos > 0) > n // 10


def test_filter_dispatch_fused_edges(P):
    """Fused call at the edges: no datagrams (total 0), a small batch (the two
    calls underneath), and a large one whose offsets start mid-buffer with the
    buffer itself at an odd address."""
    layer = P.Crc32cLayer()
    rng = np.random.default_rng(5151)
    d0 = torch.zeros(16, dtype=torch.uint8, device="cuda")
    st, s0, l0, p0 = P.filter_dispatch(d0, torch.zeros(1, dtype=torch.int64, device="cuda"))
    assert st.numel() == 0 and s0.numel() == 0
    sub = lambda m: bytes([0x00]) + rng.integers(0, 256, m - 1, dtype=np.uint8).tobytes()
    for n, lead, shift in ((300, 0, 0), (30000, 77, 3)):
        wires = [bytes(layer.process_outbound(_merged(rng, [sub(int(rng.integers(1, 300)))
                                                            for _ in range(int(rng.integers(0, 7)))], "ok")))
                 for _ in range(n)]
        off = np.concatenate([[0], np.cumsum([len(w) for w in wires])]).astype(np.uint64) + np.uint64(lead)
        blob = np.frombuffer(bytes(shift + lead) + b"".join(wires) + bytes(9), np.uint8)
        d = dev(blob)[shift:]
        o = dev(off.view(np.int64), torch.int64)
        status, start, length, parent = P.filter_dispatch(d, o)
        st2 = P.inbound_filter(d, o)
        s2, l2, p2 = P.dispatch(d, o, st2)
        assert torch.equal(status, st2)
        assert torch.equal(start, s2) and torch.equal(length, l2) and torch.equal(parent, p2)
        assert int((status == 1).sum()) == n


def test_dispatch_totals_and_scan_paths_agree(P):
    """Batches of up to kDispatchPrefixWgs x 256 = 2 Mi datagrams find their
    output slots from per-workgroup totals (the emit pass adds up its
    predecessors'); larger ones run a hipCUB scan between the passes.  A
    2.2 M-datagram batch (scan) delivers exactly its two halves' packets
    (totals), for the standalone and the fused call."""
    rng = np.random.default_rng(99)
    n = 2_200_000
    ent = lambda k: b"".join(bytes([3, 0, 0, 0x40 + k, 0x41]) for _ in range(k))  # [u16 3][UNRELIABLE, 2 B]
    templates = [bytes([0x0C]) + ent(k) for k in range(5)] + [bytes([0x00]) + bytes(m) for m in (0, 3, 17)]
    pick = rng.integers(0, len(templates), n)
    payload = np.frombuffer(b"".join(templates[j] for j in pick) + bytes(8), np.uint8)
    lens = np.array([len(t) for t in templates], np.int64)[pick]
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    wire = P.append_csr(dev(payload), dev(off, torch.int64))
    woff = dev(off + 4 * np.arange(n + 1, dtype=np.int64), torch.int64)
    status = P.inbound_filter(wire, woff)
    assert int((status == 1).sum()) == n
    full = P.dispatch(wire, woff, status)
    h = n // 2
    a = P.dispatch(wire, woff[:h + 1], status[:h])
    b = P.dispatch(wire, woff[h:], status[h:])
    assert torch.equal(full[0], torch.cat([a[0], b[0]]))
    assert torch.equal(full[1], torch.cat([a[1], b[1]]))
    assert torch.equal(full[2], torch.cat([a[2], b[2] + h]))
    assert full[0].numel() == int(np.array([0, 1, 2, 3, 4, 1, 1, 1])[pick].sum())
    fst, fs, fl, fp = P.filter_dispatch(wire, woff)
    assert torch.equal(fst, status)
    assert torch.equal(fs, full[0]) and torch.equal(fl, full[1]) and torch.equal(fp, full[2])


def test_filter_dispatch_fused_several_batches_per_wave(P):
    """Fused call over ~2.3 GB of 1300-byte containers (five 256-byte packets
    each, some plain datagrams, some corrupted): waves take several
    wave-batches; statuses and packets equal the two calls'."""
    n = 1_750_000
    S = 1 + 5 * 259 + 4
    g = torch.Generator(device="cuda")
    g.manual_seed(2024)
    data = torch.randint(0, 256, (n * S,), dtype=torch.uint8, device="cuda", generator=g)
    d2 = data.view(n, S)
    plain = torch.rand(n, device="cuda", generator=g) < 0.1
    d2[:, 0] = torch.where(plain, torch.tensor(0x01, dtype=torch.uint8, device="cuda"),
                           torch.tensor(0x0C, dtype=torch.uint8, device="cuda"))
    for j in range(5):
        b = 1 + 259 * j
        d2[:, b] = 1
        d2[:, b + 1] = 1
        d2[:, b + 2] = 0
    crc = P.batch_fixed(data, S, S - 4, n)
    d2[:, S - 4:] = crc.view(torch.uint8).view(n, 4)
    bad_rows = torch.nonzero(torch.rand(n, device="cuda", generator=g) < 0.02).flatten()
    d2[bad_rows, 7] ^= 0x10
    off = torch.arange(0, (n + 1) * S, S, dtype=torch.int64, device="cuda")
    status, start, length, parent = P.filter_dispatch(data, off)
    st2 = P.inbound_filter(data, off)
    s2, l2, p2 = P.dispatch(data, off, st2)
    assert torch.equal(status, st2)
    assert int((status == 1).sum()) == n - bad_rows.numel()
    assert torch.equal(parent, p2) and torch.equal(start, s2) and torch.equal(length, l2)
    del data, d2


def test_filter_dispatch_fused_shapes(P):
    """Fused path, container shapes at the walk's edges: > 8 entries (emit
    walks again), datagrams >= 64 KiB (16-bit records), many 1..3-byte
    entries (several per row, entries straddling rows), and the bench's 5 x
    256-B shape, in a batch large enough for the span path."""
    rng = np.random.default_rng(99)
    layer = P.Crc32cLayer()
    sub = lambda m: bytes([0x00]) + rng.integers(0, 256, m - 1, dtype=np.uint8).tobytes()
    bodies = [_merged(rng, [sub(30000) for _ in range(3)], "ok"),
              _merged(rng, [sub(20) for _ in range(9)], "ok"),
              _merged(rng, [sub(int(rng.integers(1, 4))) for _ in range(500)], "ok"),
              bytes([0x01]) + sub(70000)]
    wires = [bytes(layer.process_outbound(b)) for b in bodies] * 12
    wires += [bytes(layer.process_outbound(_merged(rng, [sub(256) for _ in range(5)], "ok")))
              for _ in range(20000)]
    order = rng.permutation(len(wires))
    _fused_vs_two_calls(P, [wires[i] for i in order])


@pytest.mark.parametrize("klen", [1, 3, 16, 37, 256])
def test_xor_layer_csr(P, klen):
    """XorEncryptLayer over a device CSR batch, in place: every datagram equals
    the restatement (phase restarts per datagram); neighbouring datagrams that
    share a 16-byte piece keep each other's bytes; twice = identity."""
    rng = np.random.default_rng(1000 + klen)
    key = rng.integers(0, 256, klen, dtype=np.uint8).tobytes()
    n = 20000
    lens = rng.integers(0, 1433, n)
    lens[rng.integers(0, n, 3000)] = rng.integers(0, 20, 3000)      # many datagrams inside one piece
    lead = int(rng.integers(0, 16))
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64) + np.uint64(lead)
    data = rng.integers(0, 256, int(off[-1]) + 21, dtype=np.uint8)
    d = dev(data)
    o = dev(off.view(np.int64), torch.int64)
    P.xor_layer_csr(d, o, key)
    got = d.cpu().numpy()
    exp = data.copy()
    for i in range(n):
        a, b = int(off[i]), int(off[i + 1])
        exp[a:b] = oracle.xor_layer(data[a:b], key)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:5]}"
    P.xor_layer_csr(d, o, key)
    assert np.array_equal(d.cpu().numpy(), data)


@pytest.mark.parametrize("shift", [0, 5])
def test_xor_layer_csr_dense_and_misaligned(P, shift):
    """The flat CSR kernel's other cases: runs of tiny and empty datagrams
    (chunks holding 64 or more datagram starts: the global-memory path), a
    buffer at an odd address, a batch ending mid-piece, and a batch whose
    first chunk starts before its first byte."""
    rng = np.random.default_rng(77 + shift)
    key = rng.integers(0, 256, 23, dtype=np.uint8).tobytes()
    n = 30000
    lens = rng.integers(0, 1433, n)
    lens[5000:6000] = rng.integers(0, 12, 1000)    # ~6 KB of starts every few bytes
    lens[20000:20300] = 0                          # a run of empty datagrams
    lead = 9
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64) + np.uint64(lead)
    data = rng.integers(0, 256, shift + int(off[-1]) + 7, dtype=np.uint8)
    d = dev(data)[shift:]
    o = dev(off.view(np.int64), torch.int64)
    P.xor_layer_csr(d, o, key)
    got = d.cpu().numpy()
    src = data[shift:]
    exp = src.copy()
    for i in range(n):
        a, b = int(off[i]), int(off[i + 1])
        exp[a:b] = oracle.xor_layer(src[a:b], key)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:5]}"


def test_xor_layer_csr_runs_of_chunks(P):
    """A batch of ~220 MB: every wave of the flat CSR kernel takes a run of
    chunks (the next chunk's datagram carried from the count of starts, or
    searched again after a dense chunk), checked byte for byte against the
    restatement, vectorised."""
    rng = np.random.default_rng(4321)
    key = rng.integers(0, 256, 22, dtype=np.uint8)
    n = 300000
    lens = rng.integers(64, 1401, n)
    for s0 in (1000, 150000, 297000):               # dense stretches inside the runs
        lens[s0:s0 + 2000] = rng.integers(0, 24, 2000)
    lead = 3
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64) + lead
    total = int(off[-1]) + 5
    g = torch.Generator(device="cuda")
    g.manual_seed(17)
    d = torch.randint(0, 256, (total,), dtype=torch.uint8, device="cuda", generator=g)
    src = d.cpu().numpy()
    o = dev(off.view(np.int64), torch.int64)
    P.xor_layer_csr(d, o, key.tobytes())
    got = d.cpu().numpy()
    phase = np.arange(int(off[-1]) - lead, dtype=np.int64) - np.repeat(off[:-1] - lead, lens)
    exp = src.copy()
    exp[lead:int(off[-1])] ^= key[phase % key.size]
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:5]}"


@pytest.mark.parametrize("shape", ["mixed", "one", "clustered"])
def test_xor_layer_csr_large_datagrams(P, shape):
    """Batches averaging far over 2 KiB per datagram: the CSR kernel's chunk
    map (one word per datagram + 1) coarsens to blocks of 2^k chunks, so a
    chunk's map word names a datagram at or before it -- checked with mixed
    sizes, one datagram of several MB, and runs of tiny datagrams between huge
    ones (a window of 64 starts that ends before the chunk)."""
    rng = np.random.default_rng({"mixed": 5, "one": 6, "clustered": 7}[shape])
    key = rng.integers(0, 256, 29, dtype=np.uint8)
    if shape == "mixed":
        lens = rng.integers(0, 200000, 400)
    elif shape == "one":
        lens = np.array([5_000_003])
    else:
        parts = []
        for _ in range(40):
            parts.append(rng.integers(100000, 300000, 1))
            parts.append(rng.integers(0, 40, int(rng.integers(1, 300))))
        lens = np.concatenate(parts)
    n = lens.size
    lead = 11
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64) + lead
    total = int(off[-1]) + 9
    g = torch.Generator(device="cuda")
    g.manual_seed(23)
    d = torch.randint(0, 256, (total,), dtype=torch.uint8, device="cuda", generator=g)
    src = d.cpu().numpy()
    o = dev(off.view(np.int64), torch.int64)
    P.xor_layer_csr(d, o, key.tobytes())
    got = d.cpu().numpy()
    phase = np.arange(int(off[-1]) - lead, dtype=np.int64) - np.repeat(off[:-1] - lead, lens)
    exp = src.copy()
    exp[lead:int(off[-1])] ^= key[phase % key.size]
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"{n} datagrams: {bad.size} bytes differ, first at {bad[:5]}"


@pytest.mark.parametrize("stride,length,klen,shift", [
    (1400, 1400, 10, 0), (1408, 1400, 10, 0), (64, 17, 10, 0), (1432, 1, 10, 0),
    (16, 16, 3, 0), (17, 17, 256, 0), (17, 5, 1, 0), (33, 32, 37, 0), (1400, 1400, 22, 0),
    (15, 15, 4, 0), (1400, 1400, 22, 3), (100, 64, 16, 1)])
def test_xor_layer_fixed(P, stride, length, klen, shift):
    """Fixed-stride XOR layer in place: the flat kernel (stride >= 16, 16-byte
    aligned base; pieces that straddle two datagrams, gaps between them, a last
    piece past the batch) and the per-datagram kernel (stride < 16, unaligned
    base: shift > 0) against the restatement; gap bytes stay untouched."""
    rng = np.random.default_rng(stride + length + klen)
    key = rng.integers(0, 256, klen, dtype=np.uint8).tobytes()
    n = 5000
    data = rng.integers(0, 256, n * stride + 16 + shift, dtype=np.uint8)
    full = dev(data)
    d = full[shift:]
    P.xor_layer_fixed(d, stride, length, n, key)
    exp = data.copy()
    for i in range(n):
        a = shift + i * stride
        exp[a:a + length] = oracle.xor_layer(data[a:a + length], key)
    assert np.array_equal(full.cpu().numpy(), exp)


def test_xor_layer_fixed_full_config2(P):
    """The bench workload at full size (2^20 x 1400 B, 22-byte key): every byte
    against a vectorised restatement (key stream per datagram, tiled)."""
    n, L = 1 << 20, 1400
    key = b"LiteNetLibPP-bench-key"
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    d = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
    data = d.cpu().numpy()
    P.xor_layer_fixed(d, L, L, n, key)
    ks = np.frombuffer(key, np.uint8)[np.arange(L) % len(key)]
    exp = (data.reshape(n, L) ^ ks[None, :]).reshape(-1)
    assert np.array_equal(d.cpu().numpy(), exp)


def test_full_config2_bit_exact(P):
    # BASELINE config 2 at full size: 2^20 x 1400 B, every CRC compared
    n, L = 1 << 20, 1400
    g = torch.Generator(device="cuda")
    g.manual_seed(42)
    data = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
    got = u32(P.batch_fixed(data, L, L, n))
    exp = oracle.batch_fixed(data.cpu().numpy(), L, L, n)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first at {bad[:5]}"
    # size-independent property: checksum of checksums is stable across launches
    again = u32(P.batch_fixed(data, L, L, n))
    assert np.array_equal(got, again)


def test_full_config2_survey_input(P):
    # SURVEY.md 8(d) recipe: mt19937_64(42) bytes; pinned out[0] = 0xD26C5CFE
    n, L = 1 << 20, 1400
    host = oracle.mt19937_64_bytes(42, n * L)
    got = u32(P.batch_fixed(dev(host), L, L, n))
    assert got[0] == 0xD26C5CFE
    import json
    with open(os.path.join(GOLD, "kat.json")) as f:
        pin = {k["recipe"]: k for k in json.load(f) if "recipe" in k}["config2"]
    assert int(np.bitwise_xor.reduce(got)) == pin["xor_all"]   # checksum of checksums
    exp = oracle.batch_fixed(host, L, L, n)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first at {bad[:5]}"


def test_error_paths_raise(P):
    data = torch.zeros(100, dtype=torch.uint8, device="cuda")
    with pytest.raises(ValueError):
        P.batch_fixed(data, 100, 100, 2)
    with pytest.raises(TypeError):
        P.batch_fixed(data.cpu(), 10, 10, 1)


def test_full_config3_survey_recipe(P):
    """SURVEY.md 8(d) config 3 recipe at full size: L_i = 64 + (u_i mod 1337),
    u = mt19937_64(43), bytes mt19937_64(44), packed CSR; out[0] and the XOR of
    all CRCs equal the pins in tests/golden/kat.json (make_recipe_pins.py), and
    every CRC equals the oracle's."""
    import ctypes
    import json
    with open(os.path.join(GOLD, "kat.json")) as f:
        pin = {k["recipe"]: k for k in json.load(f) if "recipe" in k}["config3"]
    n = 1 << 20
    u = np.empty(n, np.uint64)
    L = oracle.load()
    L.oracle_fill_mt19937_64.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_size_t]
    L.oracle_fill_mt19937_64(43, u.ctypes.data, n)
    off = np.concatenate([[0], np.cumsum(np.uint64(64) + u % np.uint64(1337))]).astype(np.uint64)
    host = oracle.mt19937_64_bytes(44, int(off[-1]))
    got = u32(P.batch_csr(dev(host), dev(off.view(np.int64), torch.int64)))
    assert int(got[0]) == pin["out0"]
    assert int(np.bitwise_xor.reduce(got)) == pin["xor_all"]
    exp = oracle.batch_csr(host, off)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first at {bad[:5]}"


# ---- outbound layer over a device burst (lnl_crc32c_append_csr_dev) ----------
APPEND_CASES = ["mixed", "tiny_and_empty", "long", "long_mix", "line_starts"]


@pytest.mark.parametrize("align", ["dword", "odd"])
@pytest.mark.parametrize("case", APPEND_CASES)
def test_append_csr_matches_layer_outbound(P, case, align):
    """Every byte of the wire burst equals lnl_crc32c_layer_outbound (the CPU
    layer, called per datagram through the C ABI) of each payload, back to
    back; the CRCs equal the oracle's; nothing outside the burst is written
    (guard bytes around the destination).  align: the destination a whole
    number of dwords from the first payload byte, or not (every source / wire
    phase the append kernel's shifted loads meet).  long_mix: overflow
    datagrams (three or more span segments) inside a span batch; line_starts:
    boundaries on 16-byte piece and 128-byte line starts, several per line,
    runs of empty datagrams."""
    rng = np.random.default_rng(APPEND_CASES.index(case) + 900 + (align == "odd") * 50)
    n = {"mixed": 20000, "tiny_and_empty": 30000, "long": 600, "long_mix": 20000, "line_starts": 40000}[case]
    if case == "mixed":
        lens = rng.integers(0, 1501, n)
    elif case == "tiny_and_empty":
        lens = np.where(rng.random(n) < 0.3, 0, rng.integers(1, 40, n))
    elif case == "long":
        lens = rng.integers(2000, 40000, n)
    elif case == "long_mix":
        lens = np.where(rng.random(n) < 0.02, rng.integers(5000, 60000, n), rng.integers(0, 300, n))
    else:
        lens = rng.choice(np.array([0, 0, 1, 15, 16, 17, 112, 128, 128, 256, 384, 1024]), n)
    lead = int(rng.integers(0, 128))
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64) + np.uint64(lead)
    data = rng.integers(0, 256, int(off[-1]) + 5, dtype=np.uint8)
    size = int(off[-1] - off[0]) + 4 * n
    # torch allocations are 256-byte aligned: (dst - first byte) % 4 = (shift - lead) % 4
    shift = int(rng.integers(1, 16))
    if align == "dword":
        shift = 16 + (lead % 4) if (shift - lead) % 4 else shift
    elif (shift - lead) % 4 == 0:
        shift += 1
    buf = torch.full((size + 64,), 0xA5, dtype=torch.uint8, device="cuda")
    wire, crc = P.append_csr(dev(data), dev(off.view(np.int64), torch.int64), out=buf[shift:shift + size],
                             want_crc=True)
    assert np.array_equal(u32(crc), oracle.batch_csr(data, off))
    got = buf.cpu().numpy()
    assert (got[:shift] == 0xA5).all() and (got[shift + size:] == 0xA5).all(), "wrote outside the burst"
    layer = P.Crc32cLayer()
    exp = b"".join(layer.process_outbound(data, int(off[i]), int(lens[i])) for i in range(n))
    assert got[shift:shift + size].tobytes() == exp


def test_append_csr_config3_full(P):
    """2^20 config-3 payloads (SURVEY recipe shape): CRCs bit-exact, every CRC
    field holds its CRC and every payload byte sits at its shift."""
    rng = np.random.default_rng(77)
    n = 1 << 20
    lens = rng.integers(64, 1401, n)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    g = torch.Generator(device="cuda")
    g.manual_seed(78)
    d = torch.randint(0, 256, (int(off[-1]),), dtype=torch.uint8, device="cuda", generator=g)
    wire, crc = P.append_csr(d, dev(off.view(np.int64), torch.int64), want_crc=True)
    data = d.cpu().numpy()
    exp_crc = oracle.batch_csr(data, off)
    assert np.array_equal(u32(crc), exp_crc)
    w = wire.cpu().numpy()
    assert w.size == int(off[-1]) + 4 * n
    crcpos = off[1:].astype(np.int64) + 4 * np.arange(n)
    fields = w[crcpos[:, None] + np.arange(4)[None, :]].reshape(-1).view("<u4")
    assert np.array_equal(fields, exp_crc)
    # every payload byte, in chunks of datagrams: byte x of datagram i at x + 4 i
    for a in range(0, n, 1 << 16):
        b = min(n, a + (1 << 16))
        x = np.arange(int(off[a]), int(off[b]), dtype=np.int64)
        x += 4 * np.repeat(np.arange(a, b, dtype=np.int64), lens[a:b])
        assert np.array_equal(w[x], data[int(off[a]):int(off[b])]), f"payload bytes of datagrams {a}..{b}"
