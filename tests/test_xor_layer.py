"""Upstream LiteNetLib's XOR-encryption layer on the
CPU entry point, against the restatement in tests/oracle.py (parity unpinned:
the reference has no layer and the C# upstream is not available offline)."""
import numpy as np
import pytest

import oracle


@pytest.fixture(scope="module")
def pkg():
    import litenetlibpp_amd as P
    P.lib()
    return P


@pytest.mark.parametrize("klen", [1, 3, 16, 17, 255, 256])
def test_cpu_layer_matches_restatement_and_roundtrips(pkg, klen):
    rng = np.random.default_rng(klen)
    key = rng.integers(0, 256, klen, dtype=np.uint8).tobytes()
    for n in (0, 1, 15, 16, 17, 1400, 1432):
        d = rng.integers(0, 256, n, dtype=np.uint8)
        x = d.copy()
        pkg.xor_layer(x, key)
        assert np.array_equal(x, oracle.xor_layer(d, key))
        pkg.xor_layer(x, key)                      # the same map both ways
        assert np.array_equal(x, d)


def test_string_key_is_utf8_and_bad_keys_refused(pkg):
    d = np.arange(10, dtype=np.uint8)
    x = d.copy()
    pkg.xor_layer(x, "kéy")
    assert np.array_equal(x, oracle.xor_layer(d, "kéy".encode("utf-8")))
    with pytest.raises(ValueError):
        pkg.xor_layer(x, b"")
    with pytest.raises(ValueError):
        pkg.xor_layer(x, bytes(257))
    L = pkg.lib()
    assert L.lnl_xor_layer(x.ctypes.data, 10, None, 0) == -22
