"""Straight-line XOR-network synthesis for constant GF(2) matrices.

A bit-sliced CRC step computes out[i] = XOR_{k in row_i} in[k] for 32 outputs
(plus optional extra per-output terms).  This module finds a short program
for that with common-subexpression elimination (Paar's greedy pair
extraction, randomised tie-breaking, best of several restarts) and then
packs the XOR2 program into 3-input XORs (gfx950 ``v_bitop3_b32`` with
truth table 0x96) by fusing single-use intermediates into their consumer.

Build-time only.
"""
from __future__ import annotations

import random
from collections import Counter
from dataclasses import dataclass, field


DERIVED_BASE = 1 << 16   # ids of Paar-derived signals
EMIT_BASE = 1 << 20      # ids of emitted op results


@dataclass
class Net:
    n_inputs: int
    # op list: (dst_signal, [src_signals]) with 2 or 3 sources, XOR
    ops: list = field(default_factory=list)
    # output i -> signal id (or None if the output is identically zero)
    outputs: list = field(default_factory=list)

    def cost(self) -> int:
        return len(self.ops)


def _paar(rows: list[set], n_inputs: int, rng: random.Random | None):
    rows = [set(r) for r in rows]
    defs = {}  # new signal -> (a, b)
    nxt = DERIVED_BASE
    while True:
        cnt = Counter()
        for r in rows:
            rl = sorted(r)
            for i in range(len(rl)):
                for j in range(i + 1, len(rl)):
                    cnt[(rl[i], rl[j])] += 1
        if not cnt:
            break
        best = max(cnt.values())
        if best < 2:
            break
        cands = [p for p, c in cnt.items() if c == best]
        a, b = rng.choice(cands) if rng else cands[0]
        s = nxt
        nxt += 1
        defs[s] = (a, b)
        for r in rows:
            if a in r and b in r:
                r.discard(a)
                r.discard(b)
                r.add(s)
    return rows, defs, nxt


def _greedy3(rows: list[set], rng: random.Random, pair_weight: float):
    """Greedy CSE that extracts 3-input common subexpressions as well as pairs.

    A triple shared by c rows costs one XOR3 and saves about c ops downstream
    (each row's XOR3 chain gets one term-pair shorter); a pair shared by c rows
    saves about c/2.  Pick the best by that estimate (pair_weight tunes the
    pair estimate; ties broken at random)."""
    from itertools import combinations
    rows = [set(r) for r in rows]
    defs = {}
    nxt = DERIVED_BASE
    while True:
        c3 = Counter()
        c2 = Counter()
        for r in rows:
            rl = sorted(r)
            c2.update(combinations(rl, 2))
            if len(rl) >= 3:
                c3.update(combinations(rl, 3))
        b3 = max(c3.values()) if c3 else 0
        b2 = max(c2.values()) if c2 else 0
        g3 = b3 - 1 if b3 >= 2 else -1
        g2 = (b2 * pair_weight - 1) if b2 >= 2 else -1
        if g3 < 0 and g2 < 0:
            break
        if g3 >= g2:
            t = rng.choice([k for k, v in c3.items() if v == b3])
        else:
            t = rng.choice([k for k, v in c2.items() if v == b2])
        st = set(t)
        sig = nxt
        nxt += 1
        defs[sig] = tuple(t)
        for r in rows:
            if st <= r:
                r -= st
                r.add(sig)
    return rows, defs, nxt


def synthesize(rows_bits: list[int], n_inputs: int, extra_terms: list | None = None,
               restarts: int = 40, seed: int = 1, greedy3_restarts: int = 0) -> Net:
    """rows_bits[i]: bitmask over inputs 0..n_inputs-1 for output i.
    extra_terms[i]: optional extra input id (>= n_inputs) xored into output i
    (each used once, e.g. the data word in a Horner step)."""
    base_rows = []
    for i, rb in enumerate(rows_bits):
        r = {k for k in range(n_inputs) if (rb >> k) & 1}
        base_rows.append(r)
    n_total_inputs = n_inputs + (len(rows_bits) if extra_terms is not None else 0)
    best = None
    for attempt in range(restarts):
        rng = random.Random(seed * 1000 + attempt) if attempt else None
        rows, defs, nxt = _paar(base_rows, n_inputs, rng)
        net = _pack(rows, defs, n_inputs, extra_terms, DERIVED_BASE, n_total_inputs)
        if best is None or net.cost() < best.cost():
            best = net
    for attempt in range(greedy3_restarts):
        rng = random.Random(seed * 7919 + attempt)
        pw = (0.5, 0.6, 0.75)[attempt % 3]
        rows, defs, nxt = _greedy3(base_rows, rng, pw)
        net = _pack(rows, defs, n_inputs, extra_terms, DERIVED_BASE, n_total_inputs)
        if net.cost() < best.cost():
            best = net
    return best


def _pack(rows, defs, n_inputs, extra_terms, first_new, n_total_inputs):
    """Turn Paar output into an XOR2/XOR3 op list with fusion of single-use
    intermediates."""
    # expression tree: each derived signal = multiset of operands
    expr = {s: list(v) for s, v in defs.items()}
    out_terms = []
    for i, r in enumerate(rows):
        t = sorted(r)
        if extra_terms is not None and extra_terms[i] is not None:
            t.append(extra_terms[i])
        out_terms.append(t)
    # use counts of derived signals
    uses = Counter()
    for s, ops in expr.items():
        for o in ops:
            uses[o] += 1
    for t in out_terms:
        for o in t:
            uses[o] += 1
    # fuse: a derived signal used exactly once gets inlined into its consumer
    # when that lets the consumer use a 3-input op.  We do it by flattening
    # operand lists, then emitting each list as a chain of XOR3s.
    def flatten(ops):
        res = []
        for o in ops:
            if o >= first_new and o in expr and uses[o] == 1 and len(expr[o]) == 2:
                res.extend(flatten(expr[o]))
            else:
                res.append(o)
        return res

    net = Net(n_inputs=n_total_inputs)
    emitted = {}
    sig_counter = [EMIT_BASE]

    def newsig():
        sig_counter[0] += 1
        return sig_counter[0]

    # topological emission
    order = sorted(expr.keys())

    def emit_list(ops):
        ops = list(ops)
        # reduce with 3-input xors first, one 2-input at the end if needed
        while len(ops) > 1:
            if len(ops) >= 3:
                a, b, c = ops[0], ops[1], ops[2]
                d = newsig()
                net.ops.append((d, [a, b, c]))
                ops = [d] + ops[3:]
            else:
                a, b = ops
                d = newsig()
                net.ops.append((d, [a, b]))
                ops = [d]
        return ops[0] if ops else None

    remap = {}

    def resolve(o):
        return remap.get(o, o)

    for s in order:
        if uses[s] == 1 and len(expr[s]) == 2:
            continue  # inlined into its consumer
        flat = [resolve(o) for o in flatten(expr[s])]
        remap[s] = emit_list(flat)
    for i, t in enumerate(out_terms):
        flat = [resolve(o) for o in flatten(t)]
        if not flat:
            net.outputs.append(None)
        elif len(flat) == 1:
            # pure copy: no op needed
            net.outputs.append(flat[0])
        else:
            net.outputs.append(emit_list(flat))
    return net


def evaluate(net: Net, inputs: list[int]) -> list[int]:
    val = dict(enumerate(inputs))
    for d, srcs in net.ops:
        v = 0
        for s in srcs:
            v ^= val[s]
        val[d] = v
    return [0 if o is None else val[o] for o in net.outputs]
