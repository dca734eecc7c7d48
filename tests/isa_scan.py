"""Static check of gfx950 kernels for VGPRs touched while a vector-memory load
into them is still in flight (test infrastructure; CPU only).

Why.  The CRC kernels issue their row loads as inline asm
(crc32c_span.hip row_load / off_load, crc32c_run.hip's table loads) and wait
for them with hand-counted `s_waitcnt vmcnt(N)` statements.  The compiler
treats such an asm statement's "=v" outputs as defined when the statement
ends, although the hardware writes them when the load returns: if it reads,
copies (v_mov, v_accvgpr_write) or reuses one of those registers before the
covering wait, the kernel computes with stale data or -- once the register
holds something else, e.g. an address -- the late load overwrites it.  The
three-row span experiment of round 4 faulted that way
(profiles/bench_r04b/r04ad_span_rows3_fault.log).  gfx9 has no
hardware interlock on VMEM results; the compiler's own loads are always
covered by waits it inserts, so every hazard this scan finds comes from an
asm load.

How.  The disassembly (llvm-objdump -d) of each kernel is split into basic
blocks (branch targets, fall-through after branches).  The state of a path is
(a) the registers that may have a load in flight, each with the fewest
vector-memory instructions issued after that load (vmcnt counts loads and
stores in issue order on gfx9), and (b) what is known of the scalar state:
SGPRs holding immediates or lane masks that are Boolean formulas over scalar
comparisons (s_cmp -> s_cselect -1/0 -> s_and / s_or / s_andn2 ...), SCC and
VCC as such formulas, and the comparisons the path has branched on.  A
vector-memory instruction ages every entry by one and adds its destination
registers at age 0 (LDS-DMA forms have none); `s_waitcnt vmcnt(N)` retires
every entry of age >= N (63 younger ones: retired, the counter holds 63).  A
branch on a formula the facts decide takes one edge; an undecided one forks
on its first open comparison.  An edge taken only when exec is zero
(s_cbranch_execnz's fall-through, s_cbranch_execz's target) drops the loads
issued since exec was last written: they ran with no lane.  States are kept
per block by their scalar part (up to a budget, beyond which the facts and
then the scalar knowledge are dropped) and joined to a fixpoint in the
pending part (a register pending on any path is pending).  Every instruction
that names a pending register -- as source or destination; a later load
into the same register is allowed, loads return in order -- is a hazard,
reported once at its first touch.  Exact on straight-line code; no
arithmetic on loop counters (tests/test_kernel_resources.py says where that
leaves reports in the product).
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess
import tempfile
from dataclasses import dataclass, field

LLVM = "/opt/rocm/lib/llvm/bin"
VMCNT_MAX = 63

_INSN = re.compile(r"^\s+([a-z_0-9.]+)(.*?)\s*//\s*([0-9A-Fa-f]+):")
_SYM = re.compile(r"^([0-9a-f]+) <(.+)>:$")
_TARGET = re.compile(r"<([^>+]+)\+0x([0-9a-f]+)>")
_REG_RANGE = re.compile(r"\b([va])\[(\d+):(\d+)\]")
_REG_ONE = re.compile(r"\b([va])(\d+)\b")
_VMCNT = re.compile(r"vmcnt\((\d+)\)")
_VMEM_PREFIX = ("global_", "buffer_", "flat_", "scratch_", "image_", "tbuffer_")


@dataclass
class Insn:
    addr: int
    op: str
    args: str
    regs: list = field(default_factory=list)   # every VGPR / AGPR named, e.g. ("v", 5)
    target: int | None = None


@dataclass
class Hazard:
    kernel: str
    addr: int
    text: str
    regs: list

    def __str__(self):
        return f"{self.kernel} +0x{self.addr:x}: {self.text}  (in flight: {', '.join(f'{k}{i}' for k, i in self.regs)})"


def _regs(args: str):
    out = []
    for k, lo, hi in _REG_RANGE.findall(args):
        out += [(k, i) for i in range(int(lo), int(hi) + 1)]
    stripped = _REG_RANGE.sub(" ", args)
    out += [(k, int(i)) for k, i in _REG_ONE.findall(stripped)]
    return out


def _first_operand_regs(args: str):
    first = args.strip().split(",")[0]
    return _regs(first)


def is_vmem(op: str) -> bool:
    return op.startswith(_VMEM_PREFIX) and not op.startswith(("buffer_wbinvl1", "buffer_inv", "buffer_wbl2"))


def vmem_dest(insn: Insn):
    """Registers a vector-memory instruction writes when it completes."""
    op, args = insn.op, insn.args
    if "_load_lds_" in op or re.search(r"\blds\b", args):
        return []                                   # LDS-DMA: no VGPR destination
    if "_load" in op:
        return _first_operand_regs(args)
    if "atomic" in op and re.search(r"\b(sc0|glc)\b", args):
        return _first_operand_regs(args)            # returning atomic
    return []


def parse(text: str):
    """{kernel symbol: [Insn]} from llvm-objdump -d --no-show-raw-insn output."""
    kernels, cur, name, base = {}, None, None, {}
    for line in text.splitlines():
        m = _SYM.match(line)
        if m:
            name = m.group(2)
            base[name] = int(m.group(1), 16)
            cur = kernels.setdefault(name, [])
            continue
        if cur is None:
            continue
        m = _INSN.match(line)
        if not m:
            continue
        op, args, addr = m.group(1), m.group(2), int(m.group(3), 16)
        insn = Insn(addr, op, args.strip(), _regs(args))
        t = _TARGET.search(line)
        if op.startswith(("s_branch", "s_cbranch")) and t and t.group(1) in base:
            insn.target = base[t.group(1)] + int(t.group(2), 16)
        cur.append(insn)
    return kernels


def _blocks(insns):
    addrs = {x.addr: k for k, x in enumerate(insns)}
    leaders = {0}
    for k, x in enumerate(insns):
        if x.op.startswith(("s_branch", "s_cbranch")):
            if x.target in addrs:
                leaders.add(addrs[x.target])
            if k + 1 < len(insns):
                leaders.add(k + 1)
        elif x.op in ("s_endpgm", "s_setpc_b64", "s_swappc_b64") and k + 1 < len(insns):
            leaders.add(k + 1)
    starts = sorted(leaders)
    blocks = [(s, (starts[j + 1] if j + 1 < len(starts) else len(insns))) for j, s in enumerate(starts)]
    index = {s: j for j, (s, _) in enumerate(blocks)}
    succ = []
    for s, e in blocks:
        last = insns[e - 1]
        nxt = []
        if last.op.startswith("s_branch"):
            nxt = [index[addrs[last.target]]] if last.target in addrs else []
        elif last.op.startswith("s_cbranch"):
            nxt = ([index[addrs[last.target]]] if last.target in addrs else []) + ([index[e]] if e in index else [])
        elif last.op in ("s_endpgm", "s_setpc_b64"):
            nxt = []
        elif e in index:
            nxt = [index[e]]
        succ.append(nxt)
    return blocks, succ


_VREG_ONE = re.compile(r"v(\d+)")
_VREG_RANGE = re.compile(r"\bv\[(\d+):(\d+)\]")


def _vregs(text: str):
    out = set()
    for lo, hi in _VREG_RANGE.findall(text):
        out |= set(range(int(lo), int(hi) + 1))
    out |= {int(i) for i in re.findall(r"\bv(\d+)\b", _VREG_RANGE.sub(" ", text))}
    return out


_SREG_RANGE = re.compile(r"\bs\[(\d+):(\d+)\]")
_SREG_ONE = re.compile(r"\bs(\d+)\b")
# scalar instructions without a scalar destination operand
_NO_SDST = ("s_cmp", "s_bitcmp", "s_cbranch", "s_branch", "s_waitcnt", "s_barrier", "s_setprio", "s_nop",
            "s_sleep", "s_endpgm", "s_store", "s_dcache", "s_sendmsg", "s_trap", "s_setreg", "s_icache",
            "s_ttrace", "s_set_gpr_idx", "s_setpc")
# scalar instructions that leave SCC alone
_KEEP_SCC = ("s_mov", "s_cmov", "s_cselect", "s_cbranch", "s_branch", "s_waitcnt", "s_nop", "s_barrier",
             "s_setprio", "s_sleep", "s_load", "s_buffer_load", "s_store", "s_dcache", "s_getpc", "s_setpc",
             "s_sendmsg", "s_memtime", "s_memrealtime", "s_icache", "s_ttrace", "s_endpgm", "s_trap")
_CMP = re.compile(r"^s_cmp_(eq|lg|gt|ge|lt|le)_(u32|i32|u64)$")


def _sregs(text: str):
    out = set()
    for lo, hi in _SREG_RANGE.findall(text):
        out |= set(range(int(lo), int(hi) + 1))
    out |= {int(i) for i in _SREG_ONE.findall(_SREG_RANGE.sub(" ", text))}
    return out


def _imm(text: str):
    try:
        return int(text.strip(), 0)
    except ValueError:
        return None


def _cmp_ints(c: str, t: str, a: int, b: int) -> bool:
    """s_cmp_<c>_<t> of two known values."""
    bits = 64 if t.endswith("64") else 32
    mask = (1 << bits) - 1
    a, b = a & mask, b & mask
    if t.startswith("i"):
        a = a - (1 << bits) if a >> (bits - 1) else a
        b = b - (1 << bits) if b >> (bits - 1) else b
    return {"lt": a < b, "le": a <= b, "gt": a > b, "ge": a >= b, "eq": a == b, "lg": a != b}[c]


def _cmp_expr(op: str, a: str, b: str):
    """s_cmp_<c>_<t> a, b as (canonical comparison, truth): lt / eq only."""
    c, t = _CMP.match(op).groups()
    if c == "lt":
        return ("lt", t, a, b), True
    if c == "ge":
        return ("lt", t, a, b), False
    if c == "gt":
        return ("lt", t, b, a), True
    if c == "le":
        return ("lt", t, b, a), False
    x, y = sorted((a, b))
    return ("eq", t, x, y), c == "eq"


# Boolean formulas over comparisons (the scalar model's lane masks, SCC and
# VCC): ("cond", expr) -- the comparison holds; ("not", f); ("and", f, g);
# ("or", f, g); True / False.  A mask holding formula f is -1 where f holds
# and 0 elsewhere (exec is taken nonzero: kernel-level uniform branches).


def _not(f):
    if f is True or f is False:
        return not f
    if f[0] == "not":
        return f[1]
    return ("not", f)


def _and(f, g):
    if f is False or g is False:
        return False
    if f is True:
        return g
    if g is True:
        return f
    return ("and", f, g) if f != g else f


def _or(f, g):
    if f is True or g is True:
        return True
    if f is False:
        return g
    if g is False:
        return f
    return ("or", f, g) if f != g else f


def _atoms(f, out):
    if f is True or f is False:
        return out
    if f[0] == "cond":
        out.add(f[1])
    else:
        for g in f[1:]:
            _atoms(g, out)
    return out


def _eval(f, facts):
    """True / False under the facts, or None when an atom is undecided."""
    if f is True or f is False:
        return f
    k = f[0]
    if k == "cond":
        return facts.get(f[1])
    if k == "not":
        v = _eval(f[1], facts)
        return None if v is None else not v
    a, b = _eval(f[1], facts), _eval(f[2], facts)
    if k == "and":
        return False if (a is False or b is False) else (True if (a and b) else None)
    return True if (a is True or b is True) else (False if (a is False and b is False) else None)


def _subst(f, facts):
    """f with its decided atoms replaced by their truth."""
    if f is True or f is False:
        return f
    k = f[0]
    if k == "cond":
        return facts[f[1]] if f[1] in facts else f
    if k == "not":
        return _not(_subst(f[1], facts))
    a, b = _subst(f[1], facts), _subst(f[2], facts)
    return _and(a, b) if k == "and" else _or(a, b)


def _expr_regs(e):
    return _sregs(e[2]) | _sregs(e[3])


class Scalar:
    """What the scan knows about the scalar state on one path: SGPRs holding
    immediates or lane masks that are Boolean formulas over comparisons (key:
    the operand text), SCC and VCC as such formulas, and the comparisons this
    path has branched on (facts).  Enough to follow the structurizer's flag
    patterns -- s_cselect_b64 s[a:b], -1, 0 after an s_cmp, masks combined
    with s_and / s_or / s_andn2, s_and(n2)_b64 vcc, exec, s[a:b] and
    s_cbranch_vcc(n)z / _scc0/1 on the same comparisons later -- so that the
    scan does not walk paths the kernel can never take."""
    __slots__ = ("vals", "scc", "vcc", "facts", "vv")

    def __init__(self, vals=None, scc=None, vcc=None, facts=None, vv=None):
        self.vals = vals or {}      # sgpr operand text -> int | formula
        self.scc = scc              # formula or None
        self.vcc = vcc              # formula or None
        self.facts = facts or {}    # comparison -> bool
        self.vv = vv or {}          # vgpr -> formula: 1 in every lane where it holds, else 0
                                    # (v_cndmask_b32 v, 0, 1, mask -- uni() of a flag)

    def key(self):
        return (frozenset(self.vals.items()), self.scc, self.vcc, frozenset(self.facts.items()),
                frozenset(self.vv.items()))

    def copy(self):
        return Scalar(dict(self.vals), self.scc, self.vcc, dict(self.facts), dict(self.vv))

    def formula(self, operand):
        """The operand as a mask formula, or None (a 32-bit half of a 64-bit
        mask is all-ones or zero as the mask is: the same formula)."""
        if operand == "exec":
            return True
        v = self.vals.get(operand, _imm(operand) if _imm(operand) is not None else None)
        if v is None:
            m = _SREG_ONE.fullmatch(operand)
            if m:
                r = int(m.group(1))
                for pair in (f"s[{r}:{r + 1}]", f"s[{r - 1}:{r}]"):
                    w = self.vals.get(pair)
                    if w is not None and not isinstance(w, int):
                        return w
        if v is None:
            return None
        if isinstance(v, int):
            if v == 0:
                return False
            return True if (v & 0xFFFFFFFFFFFFFFFF) == 0xFFFFFFFFFFFFFFFF else None
        return v

    def clobber(self, regs: set):
        """SGPRs regs were written: drop what names them (formulas keep the
        truth of the comparisons this path has decided)."""
        if not regs:
            return
        for k in [k for k in self.vals if _sregs(k) & regs]:
            del self.vals[k]

        def fix(f):
            if f is None or f is True or f is False or isinstance(f, int):
                return f
            g = _subst(f, self.facts)
            if g is True or g is False:
                return g
            return None if any(_expr_regs(e) & regs for e in _atoms(g, set())) else g

        for k, v in list(self.vals.items()):
            if not isinstance(v, int):
                g = fix(v)
                if g is None:
                    del self.vals[k]
                elif g is True or g is False:
                    self.vals[k] = -1 if g else 0
                else:
                    self.vals[k] = g
        self.scc, self.vcc = fix(self.scc), fix(self.vcc)
        for r, v in list(self.vv.items()):
            g = fix(v)
            if g is None:
                del self.vv[r]
            else:
                self.vv[r] = g
        for e in [e for e in self.facts if _expr_regs(e) & regs]:
            del self.facts[e]


def _scalar_step(sc: Scalar, x: Insn):
    """The scalar state after x (a select between two immediates on an
    unknown condition forks)."""
    ops = [o.strip() for o in x.args.split(",")] if x.args else []
    c = sc.copy()
    op = x.op
    if op.startswith("s_"):
        m = _CMP.match(op)
        if m and len(ops) == 2:
            known = [sc.vals.get(o) if isinstance(sc.vals.get(o), int) else _imm(o) for o in ops]
            if known[0] is not None and known[1] is not None:  # two known values: the result
                c.scc = _cmp_ints(m.group(1), m.group(2), known[0], known[1])
                return [c]
            if m.group(1) in ("eq", "lg") and 0 in known:  # a mask (or a copy of one) against zero
                f = sc.formula(ops[1] if known[0] == 0 else ops[0])
                if f is not None:
                    c.scc = _not(f) if m.group(1) == "eq" else f
                    return [c]
            e, truth = _cmp_expr(op, ops[0], ops[1])
            c.scc = ("cond", e) if truth else ("not", ("cond", e))
            return [c]
        if op.startswith(_NO_SDST) or not ops:
            if not op.startswith(_KEEP_SCC):
                c.scc = None
            return [c]
        dst, src = ops[0], ops[1:]
        res = None  # the written mask's formula, for the logic ops
        if op in ("s_and_b32", "s_or_b32") and len(src) == 2:
            # 32-bit logic on masks (or their halves): a nonzero immediate
            # keeps the mask's truth (all-ones & imm != 0 exactly when it holds)
            f, g = sc.formula(src[0]), sc.formula(src[1])
            if f is None and g is not None and _imm(src[0]) not in (None, 0):
                f = True
            if g is None and f is not None and _imm(src[1]) not in (None, 0):
                g = True
            if f is not None and g is not None:
                res = _and(f, g) if op == "s_and_b32" else _or(f, g)
        elif op in ("s_and_b64", "s_or_b64", "s_andn2_b64", "s_orn2_b64", "s_xor_b64") and len(src) == 2:
            f, g = sc.formula(src[0]), sc.formula(src[1])
            if f is not None and g is not None:
                if op == "s_and_b64":
                    res = _and(f, g)
                elif op == "s_or_b64":
                    res = _or(f, g)
                elif op == "s_andn2_b64":
                    res = _and(f, _not(g))
                elif op == "s_orn2_b64":
                    res = _or(f, _not(g))
                elif f is True or g is True:
                    res = _not(g if f is True else f)
        elif op == "s_not_b64" and len(src) == 1:
            f = sc.formula(src[0])
            res = None if f is None else _not(f)
        if not op.startswith(_KEEP_SCC):
            c.scc = res  # (SCC = result != 0 for the logic ops; unknown otherwise)
        if dst == "vcc":
            c.vcc = res
            return [c]
        if dst == "exec" or dst.startswith(("ttmp", "m0", "flat_scratch", "xnack")):
            return [c]
        scc_in = sc.scc  # (s_cselect reads SCC before the write)
        c.clobber(_sregs(dst))
        if res is not None:
            c.vals[dst] = -1 if res is True else (0 if res is False else res)
        elif op in ("s_mov_b64", "s_mov_b32") and len(src) == 1 and _imm(src[0]) is not None:
            c.vals[dst] = _imm(src[0])
        elif op.startswith("s_mov") and len(src) == 1 and src[0] in sc.vals:
            c.vals[dst] = sc.vals[src[0]]
        elif op == "s_mov_b32" and len(src) == 1 and sc.formula(src[0]) not in (None, True, False):
            c.vals[dst] = sc.formula(src[0])  # a half of a mask
        elif op in ("s_cselect_b64", "s_cselect_b32") and len(src) == 2 \
                and _imm(src[0]) is not None and _imm(src[1]) is not None:
            a, b = _imm(src[0]), _imm(src[1])
            if scc_in is not None and (a, b) in ((-1, 0), (0, -1)):
                f = scc_in if a == -1 else _not(scc_in)
                c.vals[dst] = -1 if f is True else (0 if f is False else f)
            elif scc_in is not None and _eval(scc_in, sc.facts) is not None:
                c.vals[dst] = a if _eval(scc_in, sc.facts) else b
            else:
                out = []
                for val in (a, b):
                    f = c.copy()
                    f.vals[dst] = val
                    out.append(f)
                return out
        return [c]
    # VGPR flags: v_cndmask_b32 v, 0, 1, mask (the uniform 0 / 1 of a mask),
    # read back by v_readfirstlane_b32 s, v; any other write of v forgets it
    vdst = ops[0] if ops and op.startswith("v_") and not op.startswith(("v_cmp", "v_readlane", "v_readfirstlane")) \
        else None
    if vdst is not None:
        for r in _vregs(vdst):
            c.vv.pop(r, None)
    elif ops and is_vmem(op) or op.startswith("ds_read"):
        for r in (vmem_dest(x) if is_vmem(op) else _vregs(ops[0])):
            c.vv.pop(r, None)
    if op.startswith("v_cndmask_b32") and len(ops) == 4 and _imm(ops[1]) == 0 and _imm(ops[2]) == 1:
        f = sc.formula(ops[3])
        if f is not None and _VREG_ONE.fullmatch(ops[0]):
            c.vv[int(ops[0][1:])] = f
    if "vcc" in x.args and not op.startswith("s_cbranch"):
        c.vcc = None  # (a VALU compare / carry writes it; reads do not matter)
    if op.startswith(("v_cmp", "v_readlane", "v_readfirstlane")) and ops:
        c.clobber(_sregs(ops[0]))
        m = _VREG_ONE.fullmatch(ops[1]) if op.startswith("v_readfirstlane_b32") and len(ops) == 2 else None
        if m and int(m.group(1)) in c.vv and _SREG_ONE.fullmatch(ops[0]):
            c.vals[ops[0]] = c.vv[int(m.group(1))]
    return [c]


def _decide(sc: Scalar, f):
    """[(truth of f, state)] over the cases the facts leave open."""
    v = _eval(f, sc.facts)
    if v is not None:
        return [(v, sc)]
    atom = sorted(_atoms(_subst(f, sc.facts), set()))[0]
    out = []
    for val in (True, False):
        g = sc.copy()
        g.facts[atom] = val
        out += _decide(g, f)
    return out


def _branch(sc: Scalar, last: Insn, taken_t: int, fall_t):
    """The feasible successors of a conditional branch, each with its state."""
    f = None  # formula that makes the branch taken
    if last.op in ("s_cbranch_scc1", "s_cbranch_scc0") and sc.scc is not None:
        f = sc.scc if last.op == "s_cbranch_scc1" else _not(sc.scc)
    elif last.op in ("s_cbranch_vccz", "s_cbranch_vccnz") and sc.vcc is not None:
        f = sc.vcc if last.op == "s_cbranch_vccnz" else _not(sc.vcc)
    if f is None:
        return [(t, sc) for t in (taken_t, fall_t) if t is not None]
    out = []
    for taken, g in _decide(sc, f):
        t = taken_t if taken else fall_t
        if t is not None:
            out.append((t, g))
    return out


def _writes_exec(x: Insn) -> bool:
    if x.op.startswith("v_cmpx"):
        return True
    return x.op.startswith("s_") and x.args.split(",")[0].strip() == "exec" or "saveexec" in x.op


def _step(state: dict, x: Insn, report=None):
    """Apply one instruction to the pending-register state: reg -> (age,
    fresh), fresh = issued since the last write of exec on every path."""
    if x.op == "s_waitcnt":
        m = _VMCNT.search(x.args)
        if m:
            n = int(m.group(1))
            for r in [r for r, (a, _) in state.items() if a >= n]:
                del state[r]
        return
    if is_vmem(x.op):
        dest = vmem_dest(x)
        if report is not None:
            src = [r for r in x.regs if r in state and r not in dest]
            if src:
                report(x, src)
                for r in set(src):
                    del state[r]
        for r in list(state):
            a, f = state[r]
            if a + 1 >= VMCNT_MAX:
                del state[r]
            else:
                state[r] = (a + 1, f)
        for r in dest:
            state[r] = (0, True)
        return
    if report is not None:
        hit = [r for r in x.regs if r in state]
        if hit:
            report(x, hit)
            for r in set(hit):  # reported once, at its first touch: no cascade
                del state[r]
    if _writes_exec(x):
        for r in state:
            state[r] = (state[r][0], False)


def _exec_zero(state: dict) -> dict:
    """The state on an edge taken only when exec is zero: the loads issued
    since exec was last written ran with no lane and write nothing."""
    return {r: v for r, v in state.items() if not v[1]}


def _merge(a: dict, b: dict) -> dict:
    out = dict(a)
    for r, (age, f) in b.items():
        if r in out:
            out[r] = (min(age, out[r][0]), f and out[r][1])
        else:
            out[r] = (age, f)
    return out


MAX_CONSTS = 64  # distinct scalar states kept per block before they are dropped


def scan_kernel(name: str, insns, max_consts: int = None) -> list:
    """Path-sensitive in the scalar state (one pending-register state per
    distinct Scalar reaching a block, at most MAX_CONSTS, beyond which the
    scalar knowledge is dropped), a may-analysis joined to a fixpoint in the
    pending registers."""
    if not insns:
        return []
    cap = max_consts or MAX_CONSTS
    blocks, succ_all = _blocks(insns)
    addrs = {x.addr: k for k, x in enumerate(insns)}
    start_of = {s: j for j, (s, _) in enumerate(blocks)}
    seen = [dict() for _ in blocks]   # Scalar key -> (Scalar, pending)
    work = []
    hazards = {}

    def add(j, pend, sc):
        key = sc.key()
        if key not in seen[j] and len(seen[j]) >= cap:
            # widen: first the branch facts, then everything scalar
            sc = Scalar(dict(sc.vals), sc.scc, sc.vcc, None, dict(sc.vv))
            key = sc.key()
            if key not in seen[j] and len(seen[j]) >= 8 * cap:
                sc = Scalar()
                key = sc.key()
        old = seen[j].get(key)
        new = pend if old is None else _merge(old[1], pend)
        if old is not None and new == old[1]:
            return
        seen[j][key] = (sc, new)
        work.append((j, key))

    def note(x, regs):
        hazards.setdefault(x.addr, Hazard(name, x.addr, f"{x.op} {x.args}", sorted(set(regs))))

    add(0, {}, Scalar())
    while work:
        j, key = work.pop()
        sc0, pend = seen[j][key]
        st, scs = dict(pend), [sc0]
        s, e = blocks[j]
        for x in insns[s:e]:
            _step(st, x, note)
            nxt, keys = [], set()
            for sc in scs:
                for f in _scalar_step(sc, x):
                    k = f.key()
                    if k not in keys:
                        keys.add(k)
                        nxt.append(f)
            scs = nxt
        last = insns[e - 1]
        for sc in scs:
            if last.op.startswith("s_cbranch") and last.target in addrs:
                tj = start_of[addrs[last.target]]
                fall = start_of.get(e)
                for t, f in _branch(sc, last, tj, fall):
                    zero = (last.op == "s_cbranch_execnz" and t == fall and t != tj) or \
                           (last.op == "s_cbranch_execz" and t == tj and t != fall)
                    add(t, _exec_zero(st) if zero else st, f)
            else:
                for t in succ_all[j]:
                    add(t, st, sc)
    return sorted(hazards.values(), key=lambda h: h.addr)


def disassemble_code_objects(paths) -> str:
    return "".join(subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", p],
                                  check=True, capture_output=True, text=True).stdout for p in paths)


def library_code_objects(lib: str, workdir: str):
    """The gfx950 code objects bundled in a host shared library."""
    dst = os.path.join(workdir, "lib.so")
    shutil.copy(lib, dst)
    subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", dst], cwd=workdir, check=True,
                   capture_output=True)
    return [os.path.join(workdir, f) for f in sorted(os.listdir(workdir)) if f.endswith("gfx950")]


def scan_library(lib: str, only: str = "", caps: dict | None = None) -> dict:
    """{kernel: [Hazard]} for every kernel in a built library whose name
    contains `only`; caps: {name substring: max_consts} for kernels scanned
    with a smaller path budget."""
    with tempfile.TemporaryDirectory() as d:
        text = disassemble_code_objects(library_code_objects(lib, d))
    out = {}
    for k, v in parse(text).items():
        if only in k:
            cap = next((c for sub, c in (caps or {}).items() if sub in k), None)
            out[k] = scan_kernel(k, v, cap)
    return out


def kernel_notes(code_objects) -> dict:
    """{kernel: {field: int}} from the code objects' metadata notes (one
    record per '- .' list entry: fields such as .agpr_count sort before .name)."""
    out = {}
    for co in code_objects:
        txt = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True, capture_output=True,
                             text=True).stdout
        rec = {}
        for line in txt.splitlines() + ["  - .end"]:
            if re.match(r"^  - \.", line) and rec:  # a kernel entry (args entries are deeper)
                if "name" in rec:
                    out[rec.pop("name")] = rec
                rec = {}
            m = re.match(r"^  (?:- |  )\.(\w+):\s+(\S+)", line)
            if m:
                k, v = m.group(1), m.group(2)
                if k == "name":
                    rec["name"] = v
                elif v.isdigit():
                    rec.setdefault(k, int(v))
    return out


def scan_code_object(path: str) -> dict:
    return {k: scan_kernel(k, v) for k, v in parse(disassemble_code_objects([path])).items()}


if __name__ == "__main__":
    import sys
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "litenetlibpp_amd", "liblnl_crc32c.so")
    res = scan_code_object(lib) if lib.endswith((".co", ".hsaco")) else scan_library(lib)
    bad = 0
    for k, hz in sorted(res.items()):
        print(f"{len(hz):5d}  {k[:110]}")
        for h in hz[:5]:
            print("       ", h)
        bad += len(hz)
    sys.exit(1 if bad else 0)
