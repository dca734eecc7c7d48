#!/usr/bin/env python3
"""Generate litenetlibpp_amd/csrc/crc32c_networks.inc.

Each emitted function applies a constant GF(2) matrix -- a CRC-32C advance
operator expressed in the transpose-free stream basis (gf2.py: A = L^-1
step^1024 L for one 128-byte row, B^d = L^-1 step^d L for the fold) -- to 32
bit-sliced registers:

    out[i] = XOR_{k : N[i][k] = 1} in[k]  ^  x[i]

where bit j of register r is lane-stream j.  The XOR program comes from
xornet.synthesize (Paar CSE + 3-input XOR packing) and is emitted as
straight-line code using LNL_XOR3 / LNL_XOR2 macros (gfx950 v_bitop3_b32 0x96
on the device, plain ^ on the host build used by the CPU tests).

Usage: python gen_networks.py [--check]   (--check: verify the file is current)
"""
from __future__ import annotations

import argparse
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gf2 import apply, rows_of, stream_basis_matrix  # noqa: E402
from xornet import evaluate, synthesize  # noqa: E402

OUT = os.path.join(HERE, "..", "csrc", "crc32c_networks.inc")

# (function name, message bits the operator advances, with_x)
NETWORKS = [
    ("lnl_net_row_x", 1024, True),   # Horner row step: V <- A V ^ X (X = the row's words)
    # fold tree, level l: V <- B^d V ^ (V >> d), d = 2^(l-1): the x term of
    # output i is s[i] >> d, computed at its use (no 32-register shift array)
    ("lnl_net_fold1", 1, "shr"),
    ("lnl_net_fold2", 2, "shr"),
    ("lnl_net_fold4", 4, "shr"),
    ("lnl_net_fold8", 8, "shr"),
    ("lnl_net_fold16", 16, "shr"),
]


def verify(net, nbits, with_x, trials=64):
    cols = stream_basis_matrix(nbits)
    rng = random.Random(12345)
    for _ in range(trials):
        v = [rng.getrandbits(32) for _ in range(64 if with_x else 32)]
        out = evaluate(net, v)
        for j in range(32):
            c = sum(((v[k] >> j) & 1) << k for k in range(32))
            e = apply(cols, c)
            if with_x:
                e ^= sum(((v[32 + i] >> j) & 1) << i for i in range(32))
            got = sum(((out[i] >> j) & 1) << i for i in range(32))
            if got != e:
                raise AssertionError(f"network {nbits} wrong at bit {j}")


def _peak_live(order, net, n_in=64):
    """Peak number of simultaneously live values (inputs until their last use,
    temporaries, produced outputs) when the ops run in `order`."""
    last = {}
    outs = set(o for o in net.outputs if o is not None)
    for i, (_, srcs) in enumerate(order):
        for x in srcs:
            last[x] = i
    live = set(k for k in range(n_in) if k in last)
    peak = len(live)
    for i, (d, srcs) in enumerate(order):
        for x in srcs:
            if last[x] == i and x not in outs:
                live.discard(x)
        live.add(d)
        peak = max(peak, len(live))
    return peak


def _schedule(net, rng, n_in=64):
    """List-schedule the ops to keep few values live: among the ready ops take
    the one that frees the most operands (random tie-break)."""
    ops = list(net.ops)
    users = {}
    for i, (_, srcs) in enumerate(ops):
        for x in srcs:
            users.setdefault(x, []).append(i)
    outs = set(o for o in net.outputs if o is not None)
    remaining = {x: len(u) for x, u in users.items()}
    avail = set(range(n_in))
    done = [False] * len(ops)
    ready = {i for i, (_, srcs) in enumerate(ops) if all(x in avail for x in srcs)}
    order = []
    while ready:
        best, bs = None, None
        for i in sorted(ready):
            _, srcs = ops[i]
            freed = sum(1 for x in set(srcs) if remaining[x] == srcs.count(x) and x not in outs)
            score = freed + rng.random() * 0.5
            if bs is None or score > bs:
                best, bs = i, score
        ready.discard(best)
        done[best] = True
        d, srcs = ops[best]
        order.append(ops[best])
        for x in srcs:
            remaining[x] -= 1
        avail.add(d)
        for j in users.get(d, []):
            if not done[j] and all(x in avail for x in ops[j][1]):
                ready.add(j)
    assert len(order) == len(ops)
    return order


def low_pressure_order(net, tries=40):
    best = list(net.ops)
    bp = _peak_live(best, net)
    for r in range(tries):
        o = _schedule(net, random.Random(r))
        p = _peak_live(o, net)
        if p < bp:
            best, bp = o, p
    return best, bp


def emit(name, nbits, with_x, net):
    lines = []
    shr = with_x == "shr"
    sig = "const uint32_t* __restrict__ s, const uint32_t* __restrict__ x, uint32_t* __restrict__ o" \
        if with_x is True else "const uint32_t* __restrict__ s, uint32_t* __restrict__ o"
    what = f"o = (L^-1 step^{nbits} L)(s)" + (f" ^ (s >> {nbits})" if shr else " ^ x" if with_x else "")
    order, peak = low_pressure_order(net)
    lines.append(f"// {what}   [{net.cost()} ops, "
                 f"{sum(1 for _, src in net.ops if len(src) == 3)} of them 3-input; "
                 f"ordered for <= {peak} live values]")
    lines.append(f"LNL_HD LNL_INLINE void {name}({sig}) {{")

    def ref(sig_id):
        if sig_id < 32:
            return f"s[{sig_id}]"
        if sig_id < 64:
            return f"(s[{sig_id - 32}] >> {nbits})" if shr else f"x[{sig_id - 32}]"
        return f"t{sig_id - (1 << 20)}"

    for d, srcs in order:
        if len(srcs) == 3:
            lines.append(f"  const uint32_t {ref(d)} = LNL_XOR3({ref(srcs[0])}, {ref(srcs[1])}, {ref(srcs[2])});")
        else:
            lines.append(f"  const uint32_t {ref(d)} = LNL_XOR2({ref(srcs[0])}, {ref(srcs[1])});")
    for i, o in enumerate(net.outputs):
        lines.append(f"  o[{i}] = {'0u' if o is None else ref(o)};")
    lines.append("}")
    return "\n".join(lines)


def generate(restarts: int) -> str:
    parts = [
        "// GENERATED by litenetlibpp_amd/tools/gen_networks.py -- do not edit.",
        "// Bit-sliced CRC-32C operators in the transpose-free stream basis",
        "// (reflected poly 0x82F63B78; see crc32c_bitslice.h and tools/gf2.py).",
        "// Register r bit j = coordinate r of lane-stream j.",
        "#pragma once",
        "",
    ]
    for name, nbits, with_x in NETWORKS:
        rows = rows_of(stream_basis_matrix(nbits))
        extra = [32 + i for i in range(32)] if with_x else None
        net = synthesize(rows, 32, extra_terms=extra, restarts=restarts, greedy3_restarts=60)
        verify(net, nbits, bool(with_x))
        parts.append(emit(name, nbits, with_x, net))
        parts.append("")
    return "\n".join(parts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--restarts", type=int, default=48)
    a = ap.parse_args()
    text = generate(a.restarts)
    if a.check:
        cur = open(OUT).read() if os.path.exists(OUT) else ""
        if cur != text:
            print("crc32c_networks.inc is stale", file=sys.stderr)
            sys.exit(1)
        return
    with open(OUT, "w") as f:
        f.write(text)
    print(f"wrote {OUT}")


if __name__ == "__main__":
    main()
