#!/usr/bin/env python3
"""In-flight load hazard check on the gfx950 ISA of the built kernels (r06).

The wave-specialised kernels issue their window loads from inline asm (`buffer_load_dwordx4 ... offen`,
ws_common.h / fir_cf_mfma.hip) and wait for them with hand-counted `s_waitcnt vmcnt(N)`. The compiler
does not know those loads are in flight: it treats the asm outputs as written when the asm statement
issues, so once a window's value is dead (the loop's last, out-of-range loads for tiles past the end)
it may hand the destination VGPRs to other values while the loads are still landing. A late load then
overwrites a live register - an address, a loop bound, a partial sum. That is the r05 multi-rank C5
fault (hipErrorIllegalAddress under contention): nothing in the index math, everything in
the timing of the loads' return.

This tool proves the absence of that hazard on the machine code. For every kernel in a code object it
builds the control-flow graph from the disassembly and runs a forward dataflow over the pending
vector-memory loads: each load's destination registers stay pending until an `s_waitcnt vmcnt(N)`
that retires it on EVERY path (N smaller than the number of vector-memory operations - loads, stores,
atomics; gfx9 counts them all in vmcnt - issued after it on every path). Any instruction that reads or
writes a pending destination register is reported. Compiler-generated loads pass (the compiler waits
before it touches them); a hand-counted wait that is too loose, or a register reused under an
in-flight asm load, fails.

Usage: isa_vmcnt_check.py <object or .so or disassembly> [--kernel SUBSTR] [-v]
Exit status 0 when no kernel has a hazard. tests/test_isa_hazards.py runs it on the library's objects.
"""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys
import tempfile

LLVM = os.environ.get("ROCM_LLVM", "/opt/rocm/lib/llvm/bin")
_FUNC = re.compile(r"^([0-9a-f]+) <([^>]+)>:$")
_INST = re.compile(r"^\s+(\S+)(.*?)//\s*([0-9A-F]+):")
_TARGET = re.compile(r"<([^>+]+)\+0x([0-9a-f]+)>")
_VR = re.compile(r"\b([va])\[(\d+):(\d+)\]|\b([va])(\d+)\b")


def disassemble(path: str) -> str:
    """llvm-objdump text of the gfx950 code object inside `path` (a host object / shared library with a
    .hip_fatbin section, or a raw code object); a .dis / .txt file is read as is."""
    if path.endswith((".dis", ".txt")):
        return open(path).read()
    with tempfile.TemporaryDirectory() as td:
        co = path
        fb = os.path.join(td, "fb.bin")
        r = subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", path, fb],
                           capture_output=True)
        if r.returncode == 0 and os.path.getsize(fb) > 0:
            co = os.path.join(td, "k.co")
            subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fb}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        out = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", co],
                             capture_output=True, text=True, check=True)
        return out.stdout


def kernel_metadata(path: str) -> dict:
    """{kernel symbol: {vgpr_count, agpr_count, vgpr_spill_count, sgpr_spill_count, private_segment_fixed_size}}
    from the code object's notes (llvm-readelf --notes). r06: a register spill inside a hot loop (the C5
    kernel's K loop reloaded a tap fragment from scratch every tile) costs more than any tuning gains."""
    with tempfile.TemporaryDirectory() as td:
        co = path
        fb = os.path.join(td, "fb.bin")
        r = subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", path, fb], capture_output=True)
        if r.returncode == 0 and os.path.getsize(fb) > 0:
            co = os.path.join(td, "k.co")
            subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fb}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], capture_output=True, text=True,
                               check=True).stdout
    out = {}
    keys = ("vgpr_count", "agpr_count", "vgpr_spill_count", "sgpr_spill_count", "private_segment_fixed_size")
    for blk in notes.split(".name:")[1:]:
        name = blk.split("\n")[0].strip()
        if name.endswith(".kd"):
            continue
        meta = {}
        for k in keys:
            m = re.search(r"\." + k + r":\s+(\d+)", blk)
            meta[k] = int(m.group(1)) if m else 0
        out[name] = meta
    return out


def regs(text: str) -> set:
    s = set()
    for m in _VR.finditer(text):
        if m.group(1):
            s |= {(m.group(1), r) for r in range(int(m.group(2)), int(m.group(3)) + 1)}
        else:
            s.add((m.group(4), int(m.group(5))))
    return s


class Inst:
    __slots__ = ("addr", "op", "args", "target", "vmem", "dest", "uses", "vmwait")

    def __init__(self, addr, op, args, target):
        self.addr, self.op, self.args, self.target = addr, op, args, target
        self.vmem = op.startswith(("buffer_", "global_", "flat_", "scratch_")) and "wbinvl1" not in op \
            and not op.endswith(("_wbl2", "_inv", "_wb"))
        load = self.vmem and ("_load" in op or ("atomic" in op and re.search(r"\b(sc0|glc)\b", args)))
        lds_dma = self.vmem and (op.startswith("global_load_lds") or re.search(r"\blds\b", args))
        first, _, rest = args.partition(",")
        self.dest = regs(first) if load and not lds_dma else set()
        self.uses = regs(rest) if self.dest else regs(args)
        m = re.search(r"vmcnt\((\d+)\)", args) if op == "s_waitcnt" else None
        self.vmwait = int(m.group(1)) if m else (0 if op == "s_waitcnt" and args.strip() in ("0", "") else None)


def parse(dis: str, want=lambda name: True):
    """{kernel symbol: [Inst]} for the kernels `want` accepts (the others are skipped unparsed)."""
    funcs, cur = {}, None
    for line in dis.splitlines():
        if line and line[0] != "\t" and line[0] != " ":
            m = _FUNC.match(line)
            if m:
                cur = m.group(2) if want(m.group(2)) else None
                if cur is not None:
                    funcs[cur] = []
            continue
        if cur is None:
            continue
        m = _INST.match(line)
        if not m:
            continue
        op, args, addr = m.group(1), m.group(2).strip(), int(m.group(3), 16)
        target = None
        if op.startswith(("s_branch", "s_cbranch")):
            t = _TARGET.search(line)
            if t:
                target = (t.group(1), int(t.group(2), 16))
        funcs[cur].append(Inst(addr, op, args, target))
    return funcs


_SR = re.compile(r"\bs\[(\d+):(\d+)\]|\bs(\d+)\b")

# ---- exec masks as boolean functions of the lane predicates (enough to tell uniform code) ----------
# A mask is a DNF: a frozenset of terms, a term a frozenset of (predicate, bit) literals; FULL = {{}}.
# Predicates are opaque lane conditions named by the instruction that produced them (a v_cmp, a merge
# of two paths that disagree). s_cbranch_execz cannot branch - and s_cbranch_execnz cannot fall
# through - while exec is FULL: those edges are infeasible in uniform code, where the compiler still
# emits them around regions it cannot prove uniform.
FULL = frozenset([frozenset()])
EMPTY = frozenset()


def _simplify(m):
    terms = set(m)
    changed = True
    while changed and len(terms) > 1:
        changed = False
        tl = list(terms)
        for x in range(len(tl)):
            for y in range(x + 1, len(tl)):
                t, u = tl[x], tl[y]
                if len(t) != len(u):
                    continue
                d = t ^ u
                if len(d) == 2:
                    (p1, b1), (p2, b2) = sorted(d)
                    if p1 == p2 and b1 != b2:
                        terms.discard(t)
                        terms.discard(u)
                        terms.add(t & u)
                        changed = True
                        break
            if changed:
                break
        # absorption: a term that contains another is redundant
        for t in list(terms):
            if any(u < t for u in terms):
                terms.discard(t)
    if len(terms) > 16:  # give up precision, keep soundness: an opaque non-full mask
        return frozenset([frozenset([("'big'", 1)])])
    return frozenset(terms)


def m_and(m, n):
    out = set()
    for t in m:
        for u in n:
            lits = dict(t)
            ok = True
            for p, bit in u:
                if lits.get(p, bit) != bit:
                    ok = False
                    break
                lits[p] = bit
            if ok:
                out.add(frozenset(lits.items()))
    return _simplify(out)


def m_or(m, n):
    return _simplify(set(m) | set(n))


def m_not(m):
    out = FULL
    for t in m:  # not(t1 or t2 ...) = and over terms of (or over the term's negated literals)
        out = m_and(out, frozenset(frozenset([(p, 1 - bit)]) for p, bit in t) if t else EMPTY)
    return out


def m_pred(name):
    return frozenset([frozenset([(repr(name), 1)])])


class ExecState:
    """exec and the SGPR pairs / vcc that hold masks."""
    __slots__ = ("exec", "sreg")

    def __init__(self, ex=FULL, sreg=None):
        self.exec = ex
        self.sreg = sreg or {}

    def key(self):
        return (self.exec, frozenset(self.sreg.items()))


def _loc(tok):
    tok = tok.strip()
    if tok in ("exec", "vcc"):
        return tok
    m = re.fullmatch(r"s\[(\d+):(\d+)\]", tok)
    if m:
        return ("s", int(m.group(1)), int(m.group(2)))
    m = re.fullmatch(r"s(\d+)", tok)
    return ("s", int(m.group(1)), int(m.group(1))) if m else None


def _clobber(st, loc):
    if loc is None or loc == "exec":
        return
    if loc == "vcc":
        st.sreg.pop("vcc", None)
        return
    for k in list(st.sreg):
        if k != "vcc" and not (k[2] < loc[1] or k[1] > loc[2]):
            del st.sreg[k]


def exec_step(i, st, addr):
    """The exec / mask state after instruction i (a new ExecState)."""
    ops = [t.strip() for t in re.split(r",(?![^\[]*\])", i.args)] if i.args else []
    ops = [o.split()[0] if o else o for o in ops]
    n = ExecState(st.exec, dict(st.sreg))

    def val(tok):
        l = _loc(tok)
        if tok == "exec":
            return n.exec
        if tok == "-1":
            return FULL
        if tok == "0":
            return EMPTY
        if l is not None and l in n.sreg:
            return n.sreg[l]
        return m_pred(("v", addr, tok))  # an opaque lane condition

    op = i.op
    if op.endswith("_saveexec_b64") and len(ops) >= 2:
        old = n.exec
        src = val(ops[1])
        kind = op[2:op.index("_saveexec")]
        new = {"and": m_and(src, old), "or": m_or(src, old), "andn2": m_and(src, m_not(old)),
               "orn2": m_or(src, m_not(old)), "xor": None}.get(kind)
        d = _loc(ops[0])
        _clobber(n, d)
        if d is not None:
            n.sreg[d] = old
        n.exec = new if new is not None else m_pred(("x", addr))
        return n
    if op in ("s_and_b64", "s_or_b64", "s_andn2_b64", "s_orn2_b64", "s_xor_b64", "s_mov_b64", "s_not_b64") and ops:
        d = _loc(ops[0])
        if op == "s_mov_b64":
            v = val(ops[1]) if len(ops) > 1 else None
        elif op == "s_not_b64":
            v = m_not(val(ops[1])) if len(ops) > 1 else None
        elif len(ops) >= 3:
            x, y = val(ops[1]), val(ops[2])
            v = {"s_and_b64": lambda: m_and(x, y), "s_or_b64": lambda: m_or(x, y),
                 "s_andn2_b64": lambda: m_and(x, m_not(y)), "s_orn2_b64": lambda: m_or(x, m_not(y)),
                 "s_xor_b64": lambda: m_or(m_and(x, m_not(y)), m_and(m_not(x), y))}[op]()
        else:
            v = None
        if d == "exec":
            # a divergent loop's latch (s_andn2_b64 exec, exec, acc; s_cbranch_execnz): when it falls
            # through, no lane of the old exec is outside acc - the exit restore (s_or_b64 exec, exec, acc)
            # brings back exactly the lanes that entered
            if op == "s_andn2_b64" and len(ops) >= 3 and ops[1] == "exec" and _loc(ops[2]) not in (None, "exec"):
                l2 = _loc(ops[2])
                if l2 != "vcc":
                    n.sreg[("e",) + l2[1:]] = st.exec
            n.exec = v if v is not None else m_pred(("x", addr))
        else:
            _clobber(n, d)
            if d is not None and v is not None:
                n.sreg[d] = v
        return n
    if op.startswith("v_cmpx"):
        n.exec = m_and(n.exec, m_pred(("c", addr)))
        return n
    if op.startswith("v_cmp") and ops:
        d = _loc(ops[0])
        _clobber(n, d)
        if d is not None:
            n.sreg[d] = m_pred(("c", addr))
        return n
    if ops and (op.startswith(("s_", "v_readfirstlane", "v_readlane", "v_div_scale")) or "_e64" in op or
                op.startswith(("v_add_co", "v_sub_co", "v_addc", "v_subb", "v_cndmask"))):
        # any other write of an SGPR / vcc (v_*_co_* and _e64 carry-outs write vcc or an SGPR pair)
        for tok in (ops[0], ops[1] if len(ops) > 1 and op.startswith(("v_add_co", "v_sub_co", "v_addc", "v_subb",
                                                                        "v_div_scale", "v_mad_u64", "v_mad_i64"))
                    else ""):
            if tok and not op.startswith(("s_cmp", "s_bitcmp", "s_waitcnt", "s_branch", "s_cbranch", "s_nop",
                                          "s_sleep", "s_setprio", "s_barrier", "s_endpgm", "s_store",
                                          "s_atomic", "s_buffer_store", "s_sendmsg", "s_dcache", "s_setreg")):
                _clobber(n, _loc(tok))
    if re.search(r"\bvcc\b", i.args) and op.startswith("v_") and ("_e32" in op or op.startswith(
            ("v_add_co", "v_sub_co", "v_addc", "v_subb", "v_cmp"))):
        n.sreg.pop("vcc", None)
    return n


def _merge_pending(into, pend):
    changed = False
    for lk, (n, dr) in pend.items():
        if lk not in into or n < into[lk][0]:
            into[lk] = (n, dr)
            changed = True
    return changed


def check(name, insts, verbose=False):
    """Hazards in one kernel: [(addr, op, args, the load's addr, regs)]. Forward dataflow over the CFG:
    per instruction one state - the pending loads {load index: (min VMEM ops issued after it on any
    path, dest regs)} and what is known of exec and the mask registers; joins take the union of pending
    loads (the fewest VMEM ops since each) and of exec. Path-insensitive across uniform scalar branches:
    a loop whose break is tested on an SCC / boolean the compiler carries in an SGPR can be reported on a
    path its conditions exclude."""
    if not insts:
        return []
    base = insts[0].addr
    index = {i.addr: k for k, i in enumerate(insts)}
    succ = []
    for k, i in enumerate(insts):
        s = []
        if i.target is not None:
            ta = base + i.target[1]
            if i.target[0] == name and ta in index:
                s.append(("t", index[ta]))
        if i.op not in ("s_branch", "s_endpgm", "s_setpc_b64") and k + 1 < len(insts):
            s.append(("f", k + 1))
        succ.append(s)
    state_in = [None] * len(insts)
    state_in[0] = ({}, ExecState())
    work = [0]
    visits = [0] * len(insts)
    hazards = {}
    while work:
        k = work.pop()
        visits[k] += 1
        pend, es = state_in[k]
        st = dict(pend)
        i = insts[k]
        # a later load into a pending register is ordered behind it (loads return in issue order):
        # only its address / data operands count; any other instruction counts with everything it names
        touched = i.uses if i.dest else i.uses | regs(i.args)
        if touched:
            for lk, (_, dr) in st.items():
                hit = dr & touched
                if hit and lk != k:
                    hazards[(i.addr, insts[lk].addr)] = (i, insts[lk], hit)
        if i.vmwait is not None:
            st = {lk: v for lk, v in st.items() if v[0] < i.vmwait}
        if i.vmem:
            st = {lk: (n + 1, dr) for lk, (n, dr) in st.items()}
            if i.dest:
                st[k] = (0, i.dest)
        nes = exec_step(i, es, i.addr - base)
        full = es.exec == FULL
        for kind, s in succ[k]:
            if full and ((i.op == "s_cbranch_execz" and kind == "t") or (i.op == "s_cbranch_execnz" and kind == "f")):
                continue  # infeasible while every lane is active
            if es.exec == EMPTY and ((i.op == "s_cbranch_execz" and kind == "f") or
                                     (i.op == "s_cbranch_execnz" and kind == "t")):
                continue
            vcc = es.sreg.get("vcc")  # a mask test of vcc (s_and_b64 vcc, exec, saved; s_cbranch_vccnz)
            if vcc is not None and i.op in ("s_cbranch_vccz", "s_cbranch_vccnz"):
                nz = {FULL: True, EMPTY: False}.get(vcc)
                if nz is not None and (kind == "t") != (nz == (i.op == "s_cbranch_vccnz")):
                    continue
            ees = nes
            if (i.op == "s_cbranch_execz" and kind == "t") or (i.op == "s_cbranch_execnz" and kind == "f"):
                ees = ExecState(EMPTY, dict(nes.sreg))  # taken only when no lane is active
                if i.op == "s_cbranch_execnz":
                    for kk in [kk for kk in ees.sreg if kk != "vcc" and kk[0] == "e"]:
                        ees.sreg[("s",) + kk[1:]] = ees.sreg.pop(kk)
            old = state_in[s]
            if old is None:
                state_in[s] = (st, ees)
                work.append(s)
                continue
            merged = dict(old[0])
            changed = _merge_pending(merged, st)
            oes = old[1]
            if oes.key() != ees.key():
                # exec at a join is one of the two paths' masks; their union is what the restore after it
                # (s_or_b64 exec, exec, saved) sees either way (an EMPTY mask from a skip edge adds nothing)
                mex = m_or(oes.exec, ees.exec) if visits[s] < 64 else m_pred(("merge", s))
                msreg = {kk: v for kk, v in oes.sreg.items() if ees.sreg.get(kk) == v}
                mes = ExecState(mex, msreg)
                if mes.key() != oes.key():
                    changed = True
            else:
                mes = oes
            if changed:
                state_in[s] = (merged, mes)
                work.append(s)
    out = []
    for (a, la), (i, li, hit) in sorted(hazards.items()):
        out.append((i.addr - base, i.op, i.args, li.addr - base, li.op, sorted(hit)))
    return out


def memory_hazards(hz):
    """The hazards that can fault: a pending register used by a vector-memory instruction (an address,
    an offset or store data) - the r05 C5 fault's class."""
    return [h for h in hz if h[1].startswith(("buffer_", "global_", "flat_", "scratch_"))]


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("inputs", nargs="+")
    ap.add_argument("--kernel", default="", help="only kernels whose symbol contains this")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    bad = 0
    total = 0
    for path in a.inputs:
        funcs = parse(disassemble(path), lambda n: a.kernel in n)
        for name, insts in funcs.items():
            total += 1
            hz = check(name, insts, a.verbose)
            if hz:
                bad += 1
                print(f"{os.path.basename(path)}: {name}: {len(hz)} hazard(s)")
                for off, op, args, loff, lop, hit in hz[: (None if a.verbose else 6)]:
                    print(f"  +0x{off:x} {op} {args[:60]}  <- in flight from +0x{loff:x} {lop} {hit[:4]}")
    print(f"{total} kernel(s) checked, {bad} with in-flight load hazards")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
