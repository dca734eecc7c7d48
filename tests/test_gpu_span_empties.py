"""Empty datagrams on the CSR span path (crc32c_span.hip), placed where the
kernel's two empty-datagram branches meet: at the batch's first byte, as a
run at the very end of the batch, exactly on segment boundaries, exactly on
wave-batch boundaries (64 segments), and in a batch with several
wave-batches per wave.  Every mode the span kernel serves -- CRC, verify and
the inbound filter -- writes into outputs poisoned beforehand, so a datagram
whose result is never stored shows up.  The geometry restates
crc32c_span.h span_geometry (R lines per segment)."""
import numpy as np
import pytest

import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

K_RMIN, K_RMAX = 16, 127


@pytest.fixture(scope="module")
def P():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import litenetlibpp_amd as pkg
    pkg.lib()
    return pkg


def span_R(first_addr, end_addr, waves):
    s0 = first_addr & ~127
    lines = (end_addr - s0 + 127) >> 7
    per = 64 * waves
    return min(max((lines + per - 1) // per, K_RMIN), K_RMAX), s0


def place_empties(lens, positions, run, rng):
    """Split the datagram holding each byte position p (from the batch's first
    byte) at p and put `run` empty datagrams there."""
    off = np.concatenate([[0], np.cumsum(lens)])
    out = list(lens)
    for p in sorted(set(int(x) for x in positions), reverse=True):
        i = int(np.searchsorted(off, p, side="right")) - 1
        if i >= len(lens):
            continue
        a = p - int(off[i])
        if a == 0:
            out[i:i] = [0] * run
        else:
            out[i:i + 1] = [a] + [0] * run + [int(lens[i]) - a]
    return np.array(out, np.int64)


def build(P, seed, n, waves, rounds_hint=1, wire=False, mean=700):
    rng = np.random.default_rng(seed)
    lens = rng.integers(1, 2 * mean, n)
    total = int(lens.sum())
    # the geometry as the kernel will see it (the buffer is 512-byte aligned)
    R, _ = span_R(0, total, waves)
    Sb = 128 * R
    segs = total // Sb
    pos = [0]
    pos += [g * Sb for g in range(1, segs, 7)]                 # segment boundaries
    pos += [w * 64 * Sb for w in range(1, segs // 64 + 1)]     # wave-batch boundaries
    pos += [g * Sb + 1 for g in range(3, segs, 97)]            # one byte past a boundary
    lens = place_empties(lens, pos, 3, rng)
    lens = np.concatenate([lens, np.zeros(5, np.int64)])        # a trailing run
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    if not wire:
        data = rng.integers(0, 256, int(off[-1]) + 7, dtype=np.uint8)
        return data, off, R
    blobs = []
    for i, L in enumerate(lens):
        b = rng.integers(0, 256, int(L), dtype=np.uint8).tobytes()
        if L >= 5 and i % 2:
            b = b[:-4] + P.crc32c(b[:-4]).to_bytes(4, "little")
        blobs.append(b)
    data = np.frombuffer(b"".join(blobs) + bytes(7), dtype=np.uint8).copy()
    return data, off, R


def waves_of_device():
    return torch.cuda.get_device_properties(0).multi_processor_count * 8


@pytest.mark.parametrize("seed,n", [(1, 40_000), (2, 70_001)])
def test_span_crc_empties_at_edges(P, seed, n):
    data, off, R = build(P, seed, n, waves_of_device())
    d = torch.from_numpy(data).cuda()
    assert d.data_ptr() % 512 == 0
    o = torch.from_numpy(off.view(np.int64)).cuda()
    out = torch.full((off.size - 1,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    got = P.batch_csr(d, o, out=out).cpu().numpy().view(np.uint32)
    exp = oracle.batch_csr(data, off)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, (R, bad[:8], np.diff(off.astype(np.int64))[bad[:8]])
    assert int((np.diff(off.astype(np.int64)) == 0).sum()) > 20


@pytest.mark.parametrize("mode", ["verify", "filter"])
def test_span_status_empties_at_edges(P, mode):
    data, off, R = build(P, 3, 50_000, waves_of_device(), wire=True)
    d = torch.from_numpy(data).cuda()
    o = torch.from_numpy(off.view(np.int64)).cuda()
    n = off.size - 1
    st = torch.full((n,), 0x77, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    L = P.lib()
    if mode == "verify":
        rc = L.lnl_crc32c_verify_csr_dev(d.data_ptr(), o.data_ptr(), n, st.data_ptr(), None, s)
    else:
        rc = L.lnl_inbound_filter_csr_dev(d.data_ptr(), o.data_ptr(), n, st.data_ptr(), s)
    assert rc == 0, L.lnl_crc32c_last_error()
    got = st.cpu().numpy()
    exp = np.array([oracle.inbound_status(data[int(off[i]):int(off[i + 1])]) for i in range(n)], np.uint8)
    if mode == "verify":
        exp = (exp != 0).astype(np.uint8)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, (R, bad[:8])


def test_span_empties_several_wave_batches_per_wave(P):
    """A batch larger than one round of every resident wave at the largest
    segment (R = 127: > 2 GiB on 256 CUs), so waves take several
    wave-batches; empties on its segment and wave-batch boundaries and at its
    end.  Bytes generated on the device."""
    waves = waves_of_device()
    rng = np.random.default_rng(610)
    lens = rng.integers(1200, 1433, 1_700_000)
    total = int(lens.sum())
    R, _ = span_R(0, total, waves)
    Sb = 128 * R
    segs = total // Sb
    assert R == K_RMAX and segs > 64 * waves
    pos = [0] + [g * Sb for g in range(1, segs, 331)] + [w * 64 * Sb for w in range(1, segs // 64 + 1, 3)]
    lens = np.concatenate([place_empties(lens, pos, 2, rng), np.zeros(3, np.int64)])
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    g = torch.Generator(device="cuda")
    g.manual_seed(611)
    d = torch.randint(0, 256, (int(off[-1]) + 1,), dtype=torch.uint8, device="cuda", generator=g)
    o = torch.from_numpy(off.view(np.int64)).cuda()
    out = torch.full((off.size - 1,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    got = P.batch_csr(d, o, out=out).cpu().numpy().view(np.uint32)
    exp = oracle.batch_csr(d.cpu().numpy(), off)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, (bad.size, bad[:8])
