"""In-flight load hazards in the gfx950 machine code (r06; tools/isa_vmcnt_check.py).

The r05 multi-rank C5 fault (hipErrorIllegalAddress) was a register the compiler reused while
an inline-asm window load was still landing in it: after the producer loop the last loads (tiles past the
block's range) are in flight, and the compiler - which does not see them - gave their registers to the
audio tail, including an output store's address. The checker runs a dataflow over each kernel's control
flow graph and reports every instruction that touches a register of a load not yet retired by an
`s_waitcnt vmcnt`. Here: the analysis on hand-made programs, then the built kernels: no wave-specialised
kernel has a hazard on a vector-memory instruction (an address or store operand: the fault's class; the
r05 build of the C5 kernel had four, profiles/r06/isa_hazards_c5_kernel_r05_build.txt). The checker is
path-insensitive across uniform scalar branches, so it also lists window conversions on paths the producer
loop's break conditions exclude; those are not asserted on."""
import glob
import os

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(REPO, "cuda-sdr_amd", "build", "kernels")


@pytest.fixture(scope="module")
def chk():
    import sys
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import isa_vmcnt_check
    return isa_vmcnt_check


def _prog(lines):
    """A kernel in llvm-objdump's format: one instruction per 4 bytes, branch targets as <k+0x..>."""
    out = ["0000000000001000 <k>:"]
    for n, text in enumerate(lines):
        addr = 0x1000 + 4 * n
        if "->" in text:  # "s_branch ->3": target instruction 3
            op, tgt = text.split("->")
            text = f"{op.strip()} 0 // {addr:012X}: 00000000 <k+0x{4 * int(tgt):x}>"
            out.append("\t" + text)
        else:
            out.append(f"\t{text} // {addr:012X}: 00000000")
    return "\n".join(out) + "\n"


def _hz(chk, lines):
    f = chk.parse(_prog(lines))
    return chk.check("k", f["k"])


def test_reuse_under_a_landing_load_is_found(chk):
    bad = ["buffer_load_dwordx4 v[4:7], v1, s[0:3], 0 offen",
           "v_mov_b32_e32 v5, 0",  # the compiler reuses v5 while the load still lands there
           "global_store_dword v[4:5], v2, off",
           "s_waitcnt vmcnt(0)",
           "s_endpgm"]
    hz = _hz(chk, bad)
    assert {h[1] for h in hz} == {"v_mov_b32_e32", "global_store_dword"}
    assert [h[1] for h in chk.memory_hazards(hz)] == ["global_store_dword"]
    good = ["buffer_load_dwordx4 v[4:7], v1, s[0:3], 0 offen", "s_waitcnt vmcnt(0)"] + bad[1:3] + ["s_endpgm"]
    assert _hz(chk, good) == []


def test_counted_waits_and_loops(chk):
    # two windows in flight, the counted wait retires the older one only (vmcnt counts stores too)
    prog = ["buffer_load_dwordx4 v[4:7], v1, s[0:3], 0 offen",      # 0 window A
            "buffer_load_dwordx4 v[8:11], v1, s[0:3], 0 offen",     # 1 window B
            "s_waitcnt vmcnt(1)",                                    # 2 A landed
            "v_xor_b32_e32 v4, 1, v4",                               # 3 A: fine
            "buffer_load_dwordx4 v[4:7], v1, s[0:3], 0 offen",      # 4 A again
            "s_waitcnt vmcnt(1)",                                    # 5 B landed
            "v_xor_b32_e32 v8, 1, v8",                               # 6 B: fine
            "buffer_load_dwordx4 v[8:11], v1, s[0:3], 0 offen",     # 7 B again
            "s_cbranch_scc1 ->2",                                    # 8 loop
            "s_waitcnt vmcnt(0)",                                    # 9 drain
            "v_mov_b32_e32 v9, 0",                                   # 10 reuse after the drain: fine
            "s_endpgm"]
    assert _hz(chk, prog) == []
    # without the drain the reuse lands under the last B load; with a wait one count too loose, A is read
    assert [h[0] for h in _hz(chk, prog[:9] + prog[10:])] == [4 * 9]
    loose = list(prog)
    loose[2] = "s_waitcnt vmcnt(2)"
    assert any(h[0] == 4 * 3 for h in _hz(chk, loose))


def test_uniform_exec_skip_edges(chk):
    # an execz skip in uniform code (exec full) cannot branch: the load issued inside is always counted
    prog = ["buffer_load_dword v4, v1, s[0:3], 0 offen",     # 0
            "s_cbranch_execz ->3",                           # 1 (never taken: exec full)
            "buffer_store_dword v2, v1, s[0:3], 0 offen",    # 2 one more VMEM op
            "s_waitcnt vmcnt(1)",                            # 3 retires load 0 (store 2 is newer)
            "v_add_u32_e32 v4, 1, v4",                       # 4
            "s_endpgm"]
    assert _hz(chk, prog) == []
    # under a partial exec (a divergent if) the skip is possible and the wait no longer covers the load
    div = ["v_cmp_gt_i32_e32 vcc, 5, v0", "s_and_saveexec_b64 s[4:5], vcc"] + prog[:4] + \
          ["s_or_b64 exec, exec, s[4:5]"] + prog[4:]
    div[3] = "s_cbranch_execz ->5"
    assert any(h[1] == "v_add_u32_e32" for h in _hz(chk, div))


def _objects():
    objs = {n: os.path.join(BUILD, n) for n in ("fir_i8_ws4.o", "fir_cf_mfma.o")}
    if not all(os.path.exists(p) for p in objs.values()):
        pytest.skip("kernel objects not built (make -C cuda-sdr_amd)")
    return objs


@pytest.fixture(scope="module")
def ws_kernels(chk):
    """{symbol: hazards} of every wave-specialised kernel in the built objects."""
    objs = _objects()
    out = {}
    for path, fam in ((objs["fir_i8_ws4.o"], "firI8Ws4Kernel"), (objs["fir_cf_mfma.o"], "firI8WsKernel"),
                      (objs["fir_cf_mfma.o"], "firCfWsKernel")):
        for name, insts in chk.parse(chk.disassemble(path), lambda n, fam=fam: fam in n).items():
            out[name] = chk.check(name, insts)
    return out


def test_no_memory_instruction_under_a_landing_load(chk, ws_kernels):
    """Every wave-specialised kernel: no vector-memory instruction uses a register a load is still
    landing in (what remains is reported on paths the loops' uniform break conditions exclude - window
    conversions after their wait)."""
    assert len(ws_kernels) >= 200
    bad = {n: chk.memory_hazards(h)[:3] for n, h in ws_kernels.items() if chk.memory_hazards(h)}
    assert not bad, bad


def test_product_kernels_do_not_spill(chk):
    """No register spill in the kernels the bench lines and the default paths run (r06: the zero-window
    guard's direct form inside the 4-way kernel's consumer loop pushed its tap fragments to scratch - a
    reload every tile, C5 0.160 -> 0.202 ms per step; the guard's work moved to the producer waves). C5's
    fused and plain 4-way kernels (KS = 21, G = 3), every 8-way int8 kernel, every cf32 wave-specialised
    kernel, C2's int8 kernel. (The 4-way K = 1408 instantiations, KS = 22, spill and are not asserted.)"""
    objs = _objects()
    objs["fir_i8_mfma.o"] = os.path.join(BUILD, "fir_i8_mfma.o")
    meta = {}
    for path in objs.values():
        meta.update(chk.kernel_metadata(path))
    want = [n for n in meta if ("firI8Ws4KernelILi21ELi3E" in n or "firI8WsKernel" in n or "firCfWsKernel" in n
                                or "firI8MfmaKernelILi5ELi2E" in n)]
    assert len(want) >= 100, len(want)
    spilled = {n: meta[n] for n in want if meta[n]["vgpr_spill_count"] or meta[n]["sgpr_spill_count"]}
    assert not spilled, spilled


def test_no_bit_cast_of_a_vector_element():
    """This compiler reads element 0 for `__builtin_bit_cast(T, v.y)` when `v` is an ext vector (r06: the cf32
    WS kernels' statistics saw every other sample). No kernel source may use the pattern."""
    import re
    pat = re.compile(r"__builtin_bit_cast\(\s*[\w:]+\s*,\s*[^(),]*\.[xyzw]\s*\)")
    src = os.path.join(REPO, "cuda-sdr_amd", "csrc", "kernels")
    hits = []
    for path in sorted(glob.glob(os.path.join(src, "*.hip")) + glob.glob(os.path.join(src, "*.h"))):
        for n, line in enumerate(open(path), 1):
            if pat.search(line):
                hits.append(f"{os.path.basename(path)}:{n}: {line.strip()}")
    assert not hits, hits
