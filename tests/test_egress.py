"""Batched socket egress (lnl_egress_send_batch, SURVEY.md 8(f) item 2, the
send half): one sendmmsg burst of a CSR wire burst over UDP loopback, each
datagram to its own endpoint, one endpoint for all, or a connected socket,
received with the ingress path (lnl_ingress_recv_batch) byte for byte.  The
reference sends one datagram per sendto (/root/reference/src/lnl/net_manager.cpp:
515-523) and keeps going after a per-datagram error (:525-567).  CPU only; the
GPU outbound layer in front of it is tests/test_gpu_parity.py::
test_append_host_egress_loopback."""
import socket

import numpy as np
import pytest


@pytest.fixture(scope="module")
def pkg():
    import litenetlibpp_amd as P
    P.lib()
    return P


def rx_socket():
    rx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rx.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 1 << 22)
    rx.bind(("127.0.0.1", 0))
    return rx


def csr(datagrams):
    off = np.zeros(len(datagrams) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(d) for d in datagrams])
    wire = np.frombuffer(b"".join(datagrams), dtype=np.uint8).copy() if datagrams else np.zeros(0, np.uint8)
    return wire, off


def drain(pkg, rx, want, max_n=64):
    buf = np.zeros(max_n * pkg.INGRESS_SLOT, dtype=np.uint8)
    got = []
    while len(got) < want:
        n, off = pkg.ingress_recv_batch(rx.fileno(), buf, max_n, wait_ms=2000)
        assert n > 0, f"timed out after {len(got)} of {want}"
        got += [bytes(buf[int(off[i]):int(off[i + 1])]) for i in range(n)]
    return got


def test_one_endpoint_byte_exact_in_order(pkg):
    rx = rx_socket()
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rng = np.random.default_rng(3)
    sent = [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes()
            for L in np.concatenate([[0, 1, 5, 1431, 1432], rng.integers(0, 1433, 150)])]
    got = []
    for b in range(0, len(sent), 40):  # bursts the loopback receive buffer holds
        wire, off = csr(sent[b:b + 40])
        r, st = pkg.egress_send_batch(tx.fileno(), wire, off, addrs=rx.getsockname())
        assert r == len(sent[b:b + 40])
        assert list(st) == [len(d) for d in sent[b:b + 40]]
        got += drain(pkg, rx, r)
    assert got == sent  # UDP loopback keeps order
    rx.close()
    tx.close()


def test_per_datagram_endpoints(pkg):
    rxs = [rx_socket() for _ in range(3)]
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    sent = [bytes([i]) * (10 + i) for i in range(45)]
    dests = [rxs[i % 3].getsockname() for i in range(45)]
    wire, off = csr(sent)
    r, st = pkg.egress_send_batch(tx.fileno(), wire, off, addrs=dests)
    assert r == 45 and all(st[i] == 10 + i for i in range(45))
    for k, rx in enumerate(rxs):
        assert drain(pkg, rx, 15) == sent[k::3]
        rx.close()
    tx.close()


def test_connected_socket_and_more_than_one_sendmmsg_call(pkg):
    """No addresses on a connected socket; 1500 datagrams take two sendmmsg
    calls (1024 per call)."""
    rx = rx_socket()
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    tx.connect(rx.getsockname())
    sent = [i.to_bytes(4, "little") for i in range(1500)]
    wire, off = csr(sent)
    r, st = pkg.egress_send_batch(tx.fileno(), wire, off)
    assert r == 1500 and bool((st == 4).all())
    assert drain(pkg, rx, 1500, max_n=512) == sent
    rx.close()
    tx.close()


def test_per_datagram_error_does_not_stop_the_burst(pkg):
    """A datagram the kernel refuses (here: longer than a UDP datagram can be,
    EMSGSIZE) gets its negative errno and the burst goes on, as send_raw's
    error case does for one datagram."""
    import errno
    rx = rx_socket()
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    sent = [b"a" * 10, b"b" * 70000, b"c" * 20]
    wire, off = csr(sent)
    r, st = pkg.egress_send_batch(tx.fileno(), wire, off, addrs=rx.getsockname())
    assert r == 3
    assert st[0] == 10 and st[1] == -errno.EMSGSIZE and st[2] == 20
    assert drain(pkg, rx, 2) == [sent[0], sent[2]]
    rx.close()
    tx.close()


def test_bad_calls(pkg):
    wire, off = csr([b"xy", b"z"])
    with pytest.raises(pkg.Crc32cError):
        pkg.egress_send_batch(-1, wire, off, addrs=("127.0.0.1", 9))
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    with pytest.raises(ValueError):  # two endpoints for three datagrams
        pkg.egress_send_batch(tx.fileno(), *csr([b"a", b"b", b"c"]), addrs=[("127.0.0.1", 9)] * 2)
    r, st = pkg.egress_send_batch(tx.fileno(), np.zeros(0, np.uint8), np.zeros(1, np.uint64))
    assert r == 0 and st.size == 0
    tx.close()
