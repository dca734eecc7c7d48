"""The outbound layer (lnl_crc32c_append_csr_dev: the CSR CRC pass, then
lnl_append.hip's copy kernel) on the GPU: every shape of head chunk, whole
chunks and tail (payload remainder + CRC) the copy distinguishes, at every
destination alignment, with and without the CRC output; the wire burst checked
byte for byte against lnl_crc32c_layer_outbound (the CPU layer) and the CRCs
against the oracle.  (tests/test_gpu_parity.py holds the round-3 append cases
and the full config-3 burst.)"""
import numpy as np
import pytest

import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def P():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import litenetlibpp_amd as pkg
    pkg.lib()
    return pkg


def run_burst(P, lens, shift, lead, seed, want_crc=True):
    rng = np.random.default_rng(seed)
    lens = np.asarray(lens, np.int64)
    n = lens.size
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64) + np.uint64(lead)
    data = rng.integers(0, 256, int(off[-1]) + 9, dtype=np.uint8)
    size = int(off[-1] - off[0]) + 4 * n
    buf = torch.full((size + 64,), 0xA5, dtype=torch.uint8, device="cuda")
    d = torch.from_numpy(data).cuda()
    o = torch.from_numpy(off.view(np.int64)).cuda()
    res = P.append_csr(d, o, out=buf[shift:shift + size], want_crc=want_crc)
    got = buf.cpu().numpy()
    assert (got[:shift] == 0xA5).all() and (got[shift + size:] == 0xA5).all(), "wrote outside the burst"
    layer = P.Crc32cLayer()
    exp = b"".join(layer.process_outbound(data, int(off[i]), int(lens[i])) for i in range(n))
    bad = np.nonzero(got[shift:shift + size] != np.frombuffer(exp, np.uint8))[0]
    assert bad.size == 0, (shift, lead, bad[:10])
    if want_crc:
        assert np.array_equal(res[1].cpu().numpy().view(np.uint32), oracle.batch_csr(data, off))


@pytest.mark.parametrize("shift", range(16))
def test_append_small_lengths_every_alignment(P, shift):
    """Lengths 0..80 in runs and next to 1400-byte neighbours: the 12-byte
    threshold below which a chunk holds two CRC fields (byte stores), the
    head chunk shared with a short predecessor, empty datagrams at every
    phase."""
    lens = []
    for L in range(81):
        lens += [L, 1400 - L, 3, L]
    run_burst(P, lens, shift, lead=(shift * 7) % 16, seed=shift)


@pytest.mark.parametrize("want_crc", [True, False])
def test_append_random_bursts(P, want_crc):
    rng = np.random.default_rng(3 + want_crc)
    for it in range(12):
        n = int(rng.integers(1, 3000))
        k = rng.integers(0, 10, n)
        lens = np.where(k < 3, rng.integers(0, 24, n),
                        np.where(k < 8, rng.integers(64, 1401, n), rng.integers(1400, 9000, n)))
        run_burst(P, lens, int(rng.integers(0, 16)), int(rng.integers(0, 128)), 100 + it, want_crc)


def test_append_huge_datagrams_and_edges(P):
    """65,507-byte datagrams (many 1,536-byte load groups per team), a burst
    of one datagram, and single-byte bursts at the buffer's edges."""
    run_burst(P, [65507, 0, 1, 65535, 12, 11, 13], 7, 5, 1)
    for L in (0, 1, 11, 12, 13, 16, 17, 1432):
        for shift in (0, 15):
            run_burst(P, [L], shift, 0, L)
