"""Batched socket ingress (lnl_ingress_recv_batch):
recvmmsg bursts over UDP loopback compacted into the CSR layout the batch
entry points take.  CPU only (the GPU end of the socket path is
tests/test_gpu_parity.py::test_socket_path_end_to_end)."""
import socket

import numpy as np
import pytest


@pytest.fixture(scope="module")
def pkg():
    import litenetlibpp_amd as P
    P.lib()
    return P


def loopback_pair():
    rx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rx.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 1 << 22)
    rx.bind(("127.0.0.1", 0))
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    tx.connect(rx.getsockname())
    return rx, tx


def drain(pkg, rx, buf, max_n, want):
    got = []
    while len(got) < want:
        n, off = pkg.ingress_recv_batch(rx.fileno(), buf, max_n, wait_ms=2000)
        assert n > 0, f"timed out after {len(got)} of {want}"
        assert off[0] == 0 and np.all(np.diff(off.astype(np.int64)) >= 0)
        got += [bytes(buf[int(off[i]):int(off[i + 1])]) for i in range(n)]
    return got


def test_bursts_are_csr_and_byte_exact(pkg):
    rx, tx = loopback_pair()
    rng = np.random.default_rng(9)
    sent = [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes()
            for L in np.concatenate([[0, 1, 1431, 1432], rng.integers(0, 1433, 600)])]
    for d in sent:
        tx.send(d)
    buf = np.zeros(64 * pkg.INGRESS_SLOT, dtype=np.uint8)   # bursts of <= 64
    assert drain(pkg, rx, buf, 64, len(sent)) == sent       # UDP loopback keeps order
    rx.close()
    tx.close()


def test_long_datagram_truncated_like_recvfrom(pkg):
    rx, tx = loopback_pair()
    tx.send(bytes(range(256)) * 8)                          # 2048 B > the 1432-byte slot
    buf = np.zeros(4 * pkg.INGRESS_SLOT, dtype=np.uint8)
    got = drain(pkg, rx, buf, 4, 1)
    assert got == [(bytes(range(256)) * 8)[:pkg.INGRESS_SLOT]]
    rx.close()
    tx.close()


def test_nothing_ready_and_bad_arguments(pkg):
    rx, tx = loopback_pair()
    buf = np.zeros(2 * pkg.INGRESS_SLOT, dtype=np.uint8)
    n, off = pkg.ingress_recv_batch(rx.fileno(), buf, 2, wait_ms=0)
    assert n == 0 and list(off) == [0]
    small = np.zeros(100, dtype=np.uint8)                  # not even one slot
    with pytest.raises(pkg.Crc32cError):
        pkg.ingress_recv_batch(rx.fileno(), small, 1)
    with pytest.raises(pkg.Crc32cError):
        pkg.ingress_recv_batch(-1, buf, 1)
    rx.close()
    tx.close()
