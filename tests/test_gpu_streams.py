"""GPU tests of the host pipelines' stream count (lnl_host_opts, BASELINE
config 5's "2 HIP streams"), the per-stream scratch the CSR span path keeps
(hipStreamPerThread keys, the LRU bound, lnl_stream_release) and the span
kernel's epoch-paired wave-batch exchange (stale arrival words never pair).
Everything is checked bit-exact against the oracle."""
import ctypes
import threading

import numpy as np
import pytest

import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

HIP_STREAM_PER_THREAD = 2  # hipStreamPerThread, /opt/rocm/include/hip/hip_runtime_api.h


@pytest.fixture(scope="module")
def P():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import litenetlibpp_amd as pkg
    pkg.lib()
    return pkg


def u32(t):
    return t.cpu().numpy().view(np.uint32)


def dev(a, dtype=torch.uint8):
    return torch.from_numpy(np.ascontiguousarray(a)).to(device="cuda", dtype=dtype)


def csr_batch(seed, n, lo=0, hi=1433, shift=0):
    rng = np.random.default_rng(seed)
    lens = rng.integers(lo, hi, n)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64) + np.uint64(shift)
    data = rng.integers(0, 256, int(off[-1]) + 9, dtype=np.uint8)
    return data, off


def wire_batch(P, seed, n):
    """Wire datagrams: two in three carry their right CRC, the rest random
    bytes (drops); some runts and empties."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 1433, n)
    lens[rng.integers(0, n, n // 50)] = rng.integers(0, 5, n // 50)
    blobs = []
    for i, L in enumerate(lens):
        b = rng.integers(0, 256, int(L), dtype=np.uint8).tobytes()
        if L >= 5 and i % 3:
            b = b[:-4] + P.crc32c(b[:-4]).to_bytes(4, "little")
        blobs.append(b)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = np.frombuffer(b"".join(blobs) + bytes(7), dtype=np.uint8).copy()
    exp = np.array([oracle.inbound_status(data[int(off[i]):int(off[i + 1])]) for i in range(n)], np.uint8)
    return data, off, exp


@pytest.mark.parametrize("streams", [1, 2, 4, 8])
def test_host_crc_stream_counts(P, streams):
    """lnl_crc32c_batch_host_ex at every stream count, chunks small enough
    (8 Ki datagrams) that every stream takes several; nonzero first offset."""
    data, off = csr_batch(500 + streams, 100_003, shift=3)
    pinned = torch.from_numpy(data).pin_memory().numpy()
    got = P.batch_host(pinned, off, 0, streams=streams, chunk_datagrams=8192)
    assert np.array_equal(got, oracle.batch_csr(data, off))
    # the default chunks too (64 Ki datagrams: two chunks here)
    assert np.array_equal(P.batch_host(pinned, off, 0, streams=streams), oracle.batch_csr(data, off))


def test_host_outputs_pinned_and_pageable(P):
    """The host pipeline's small results (CRCs, statuses) go straight into a
    page-locked output array and through the slots' pinned staging into a
    pageable one (copied out as each slot is reused and at the end): both
    equal the oracle, several chunks per stream."""
    import ctypes
    data, off = csr_batch(901, 70_001, shift=1)
    pinned = torch.from_numpy(data).pin_memory().numpy()
    exp = oracle.batch_csr(data, off)
    opts = P.HostOpts.make(streams=2, chunk_datagrams=4096)
    n = off.size - 1
    for out in (np.zeros(n, np.uint32), torch.zeros(n, dtype=torch.int32).pin_memory().numpy().view(np.uint32)):
        rc = P.lib().lnl_crc32c_batch_host_ex(pinned.ctypes.data, off.ctypes.data, n, out.ctypes.data, 0,
                                              ctypes.pointer(opts))
        assert rc == 0, P.lib().lnl_crc32c_last_error()
        assert np.array_equal(out, exp)
    wd, woff, wexp = wire_batch(P, 902, 30_000)
    wpinned = torch.from_numpy(wd).pin_memory().numpy()
    for st in (np.full(woff.size - 1, 9, np.uint8), torch.full((woff.size - 1,), 9, dtype=torch.uint8).pin_memory().numpy()):
        rc = P.lib().lnl_inbound_filter_host_ex(wpinned.ctypes.data, woff.ctypes.data, woff.size - 1, st.ctypes.data,
                                                0, ctypes.pointer(opts))
        assert rc == 0, P.lib().lnl_crc32c_last_error()
        assert np.array_equal(st, wexp)


@pytest.mark.parametrize("streams", [2, 4])
def test_host_filter_stream_counts(P, streams):
    data, off, exp = wire_batch(P, 600 + streams, 40_000)
    pinned = torch.from_numpy(data).pin_memory().numpy()
    got = P.inbound_filter_host(pinned, off, 0, streams=streams, chunk_datagrams=4096)
    assert np.array_equal(got, exp) and set(np.unique(exp)) >= {0, 1}


@pytest.mark.parametrize("streams", [2, 4])
def test_host_append_stream_counts(P, streams):
    """lnl_crc32c_append_host_ex at 2 and 4 streams: the wire burst (payload ||
    LE32(CRC) back to back) and the CRCs, several chunks per stream."""
    data, off = csr_batch(700 + streams, 60_001, shift=5)
    pinned = torch.from_numpy(data).pin_memory().numpy()
    wire, woff, crc = P.append_host(pinned, off, 0, want_crc=True, streams=streams, chunk_datagrams=4096)
    exp = oracle.batch_csr(data, off)
    assert np.array_equal(crc, exp)
    lens = np.diff(off.astype(np.int64))
    crcpos = woff[1:].astype(np.int64) - 4
    keep = np.ones(wire.size, dtype=bool)
    for j in range(4):
        keep[crcpos + j] = False
    assert np.array_equal(wire[keep], data[int(off[0]):int(off[-1])])
    assert np.array_equal(wire[crcpos[:, None] + np.arange(4)[None, :]].reshape(-1), exp.astype("<u4").view(np.uint8))
    assert np.array_equal(np.diff(woff.astype(np.int64)), lens + 4)


def test_host_opts_rejected(P):
    L = P.lib()
    data = np.zeros(64, np.uint8)
    off = np.array([0, 16, 64], np.uint64)
    out = np.zeros(2, np.uint32)
    bad = [P.HostOpts.make(streams=9), P.HostOpts(4, 2, 0, 0, 0), P.HostOpts(ctypes.sizeof(P.HostOpts), 2, 0, 1, 0)]
    for o in bad:
        rc = L.lnl_crc32c_batch_host_ex(data.ctypes.data, off.ctypes.data, 2, out.ctypes.data, 0, ctypes.pointer(o))
        assert rc == -22, rc
    with pytest.raises(ValueError):
        P.batch_host(data, off, 0, streams=9)


def test_span_stale_arrival_words_never_pair(P):
    """The span kernel's wave-batch exchange pairs by the call's epoch: arrival
    words filled with whatever an aborted call might leave -- either side, any
    epoch up to the calls made so far (the old protocol needed them at 0
    between calls) -- change nothing in the next calls; a value with a later
    epoch is refused (it could pair with a future call's own arrival)."""
    data, off = csr_batch(800, 200_000)
    d, o = dev(data), dev(off.view(np.int64), torch.int64)
    exp = oracle.batch_csr(data, off)
    s = torch.cuda.Stream()  # (its own scratch: the epoch count starts here)
    torch.cuda.synchronize()
    first = P.batch_csr(d, o, stream=s)
    s.synchronize()
    assert np.array_equal(u32(first), exp)
    calls = 1
    for value in (1, 2, 3, 5, 6, 7, (2 << 2) | 1, (3 << 2) | 2, (7 << 2) | 1, (9 << 2) | 2):
        rc = P.lib().lnl_diag_fill_span_arrivals(s.cuda_stream, value)
        if (value >> 2) > calls:  # an epoch no earlier call reached: refused, nothing written
            assert rc == -22, rc
        else:
            assert rc == 0, P.lib().lnl_crc32c_last_error()
        calls += 2
        for _ in range(2):
            out = torch.full((off.size - 1,), -1, dtype=torch.int32, device="cuda")
            torch.cuda.synchronize()
            got = P.batch_csr(d, o, out=out, stream=s)
            s.synchronize()
            assert np.array_equal(u32(got), exp), hex(value)
    # and the status path (verify mode on the same scratch)
    wd, woff, wexp = wire_batch(P, 801, 30_000)
    assert P.lib().lnl_diag_fill_span_arrivals(s.cuda_stream, 1) == 0
    wd_d, woff_d = dev(wd), dev(woff.view(np.int64), torch.int64)
    torch.cuda.synchronize()
    got = P.inbound_filter(wd_d, woff_d, stream=s)
    s.synchronize()
    assert np.array_equal(got.cpu().numpy(), wexp)
    P.stream_release(s)


def test_span_scratch_per_thread_streams(P):
    """Two threads call lnl_crc32c_batch_csr_dev concurrently on
    hipStreamPerThread: each thread's launches go to its own stream, so the
    library must not hand both the same control and exchange blocks."""
    L = P.lib()
    batches = [csr_batch(900 + t, 120_000) for t in range(2)]
    dev_in = [(dev(d), dev(o.view(np.int64), torch.int64)) for d, o in batches]
    exp = [oracle.batch_csr(d, o) for d, o in batches]
    outs = [[torch.full((o.size - 1,), -1, dtype=torch.int32, device="cuda") for _ in range(6)]
            for _, o in batches]
    torch.cuda.synchronize()
    errors = []

    def run(t):
        d, o = dev_in[t]
        n = o.numel() - 1
        for out in outs[t]:
            rc = L.lnl_crc32c_batch_csr_dev(d.data_ptr(), o.data_ptr(), n, out.data_ptr(), HIP_STREAM_PER_THREAD)
            if rc:
                errors.append((t, rc, L.lnl_crc32c_last_error()))
        torch.cuda.synchronize()

    th = [threading.Thread(target=run, args=(t,)) for t in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    torch.cuda.synchronize()
    assert not errors, errors
    for t in range(2):
        for out in outs[t]:
            assert np.array_equal(u32(out), exp[t])


def test_stream_release_and_cache_bound(P):
    """lnl_stream_release frees a stream's scratch (the next call on it starts
    afresh), and more distinct streams than LNL_STREAM_CACHE (32) stay correct
    while the least recently used scratch is evicted."""
    data, off = csr_batch(950, 40_000)
    d, o = dev(data), dev(off.view(np.int64), torch.int64)
    exp = oracle.batch_csr(data, off)
    streams = [torch.cuda.Stream() for _ in range(40)]
    for rep in range(2):
        for s in streams:
            with torch.cuda.stream(s):
                out = P.batch_csr(d, o, stream=s)
            s.synchronize()
            assert np.array_equal(u32(out), exp)
    for s in streams[:5]:
        P.stream_release(s)
        with torch.cuda.stream(s):
            out = P.batch_csr(d, o, stream=s)
        s.synchronize()
        assert np.array_equal(u32(out), exp)
        P.stream_release(s)
    # releasing a stream the library never saw is a no-op
    assert P.lib().lnl_stream_release(torch.cuda.Stream().cuda_stream) == 0


def test_cache_bound_with_calls_in_flight(P):
    """Evictions while the victims' calls are still queued: 40 streams, three
    rounds of calls with no host synchronise between them.  Past half the bound
    each call records its last-use event and an eviction frees behind it on the
    library stream; earlier entries are freed after a device synchronise."""
    data, off = csr_batch(951, 60_000)
    d, o = dev(data), dev(off.view(np.int64), torch.int64)
    exp = oracle.batch_csr(data, off)
    streams = [torch.cuda.Stream() for _ in range(40)]
    outs = []
    for rep in range(3):
        for s in streams:
            with torch.cuda.stream(s):
                outs.append(P.batch_csr(d, o, stream=s))
    torch.cuda.synchronize()
    for out in outs:
        assert np.array_equal(u32(out), exp)
    for s in streams:
        P.stream_release(s)
    torch.cuda.synchronize()
