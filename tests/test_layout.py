"""Descriptor placement of the window pre-pass (crc32c_bucket.hip,
bucket_window_kernel), restated: window w of W datagrams goes to slot
s = (w mod M) * (G / M) + w / M (full windows, K = G / M > 1), and with the XCD
option the window's batch q to 256 (s / 8) + 32 (q / 4) + 4 (s mod 8) + q mod 4.
The kernel's parity runs on the GPU; this checks on the CPU that the index map
is a permutation of [0, n) for batch sizes around the edges (partial last
window, fewer than 8 or M full windows), so no descriptor is lost or doubled."""
import numpy as np
import pytest


def placement(n, W, M, xcd):
    gf = n // W
    K = gf // M if M else 0
    pos = np.empty(n, dtype=np.int64)
    for w in range((n + W - 1) // W):
        d0 = w * W
        if K > 1 and w < K * M:
            d0 = ((w % M) * K + w // M) * W
        slot = d0 // W
        r = np.arange(min(W, n - w * W))
        q = r >> 6
        xmap = xcd and W // 64 == 32 and slot < gf // 8 * 8
        if xmap:
            p = 64 * (256 * (slot >> 3) + 32 * (q >> 2) + 4 * (slot & 7) + (q & 3)) + (r & 63)
        else:
            p = d0 + r
        pos[w * W: w * W + r.size] = p
    return pos


@pytest.mark.parametrize("n", [1, 2047, 2048, 16384, 16385, 5 * 2048 + 7, 1 << 20, (1 << 20) + 999])
@pytest.mark.parametrize("W,M,xcd", [(2048, 4, False), (2048, 4, True), (2048, 0, True),
                                     (1024, 4, False), (8192, 8, False), (2048, 3, True)])
def test_window_placement_is_a_permutation(n, W, M, xcd):
    pos = placement(n, W, M, xcd)
    assert pos.min() >= 0 and pos.max() < n
    assert np.unique(pos).size == n


def test_spread_places_neighbouring_windows_apart():
    # the windows the chip works on at once (consecutive slots) lie M windows apart
    n, W, M = 1 << 20, 2048, 4
    pos = placement(n, W, M, False)
    slot_of_window = pos[::W] // W
    window_at_slot = np.argsort(slot_of_window)
    assert np.all(np.diff(window_at_slot[: (n // W) // M]) == M)
