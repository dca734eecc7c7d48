"""Debug helper (GPU box): fused filter + dispatch vs the two calls on the
shapes batch of tests/test_gpu_parity.py::test_filter_dispatch_fused_shapes;
prints the mismatching datagrams with their place in the span geometry."""
import os
import sys
from collections import defaultdict

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import litenetlibpp_amd as P  # noqa: E402
from test_gpu_parity import _merged  # noqa: E402

rng = np.random.default_rng(99)
layer = P.Crc32cLayer()
sub = lambda m: bytes([0x00]) + rng.integers(0, 256, m - 1, dtype=np.uint8).tobytes()
which = sys.argv[1] if len(sys.argv) > 1 else "all"
bodies = [_merged(rng, [sub(30000) for _ in range(3)], "ok"),
          _merged(rng, [sub(20) for _ in range(9)], "ok"),
          _merged(rng, [sub(int(rng.integers(1, 4))) for _ in range(500)], "ok"),
          bytes([0x01]) + sub(70000)]
wires = [bytes(layer.process_outbound(b)) for b in bodies] * 12
wires += [bytes(layer.process_outbound(_merged(rng, [sub(256) for _ in range(5)], "ok"))) for _ in range(20000)]
order = rng.permutation(len(wires))
wires = [wires[i] for i in order]
if which == "plain":
    wires = wires[:]  # same
off = np.concatenate([[0], np.cumsum([len(w) for w in wires])]).astype(np.uint64)
blob = np.frombuffer(b"".join(wires), np.uint8)
d = torch.from_numpy(blob.copy()).cuda()
o = torch.from_numpy(off.view(np.int64).copy()).cuda()
st, s1, l1, p1 = P.filter_dispatch(d, o)
st2 = P.inbound_filter(d, o)
s2, l2, p2 = P.dispatch(d, o, st2)
print("status equal", torch.equal(st, st2), "packets", s1.numel(), s2.numel())


def per(s, l, p):
    r = defaultdict(list)
    for a, b, c in zip(s.cpu().numpy().tolist(), l.cpu().numpy().tolist(), p.cpu().numpy().tolist()):
        r[c].append((a - int(off[c]), b))
    return r


A, B = per(s1, l1, p1), per(s2, l2, p2)
n = len(wires)
lines = (int(off[-1]) + 127) // 128
R = max(16, min(127, -(-lines // (64 * 2048))))
Sb = 128 * R
bad = [i for i in range(n) if A.get(i) != B.get(i)]
print("n", n, "R", R, "Sb", Sb, "bad datagrams", len(bad))
for i in bad[:25]:
    s0, s1_ = int(off[i]), int(off[i + 1])
    print(f"i={i} len={s1_ - s0} start={s0} seg={s0 // Sb} cs={s0 % Sb} endseg={(s1_ - 1) // Sb} "
          f"lane={(s0 // Sb) % 64} fused={A.get(i, [])[:6]} two={B.get(i, [])[:6]} nf={len(A.get(i, []))} nt={len(B.get(i, []))}")
