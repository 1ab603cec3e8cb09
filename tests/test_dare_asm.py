"""The row DARE kernel's inline-asm DPP FMAs (csrc/qt_dare.hip, fmac_row /
fmac_col) against gfx950's DPP hazards, on the device assembly built with the
library's own flags (Makefile `dare-asm`; CPU only, hipcc cross-compiles).

The compiler's hazard recognizer does not look inside inline asm, so the
kernel states its rule and this test checks it on every DPP instruction of
the row kernels (the asm FMAs and moves, and the compiler's own DPP, whose
sources inline asm may have written):
  * no VALU instruction writing the DPP source (src0) VGPRs within the 2 wait
    states before it;
  * no VALU write of EXEC (v_cmpx) within the 5 wait states before it (the
    hazard LLVM's recognizer models; scalar EXEC writes are not one);
  * along every path into the instruction (fall-through and branches to the
    labels in that window).
Each instruction is one wait state, `s_nop N` is N + 1."""

import os
import re
import subprocess

import pytest

from conftest import ROOT

PKG = os.path.join(ROOT, "lqr-quadcopter-test_amd")
OBJ = os.path.join(ROOT, "build", "dare_asm")


@pytest.fixture(scope="module")
def asm():
    if subprocess.run(["which", "hipcc"], capture_output=True).returncode != 0 and not os.path.exists(
            "/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc not available")
    r = subprocess.run(["make", "-s", "-C", PKG, "dare-asm", f"OBJ={OBJ}"], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return open(os.path.join(OBJ, "qt_dare.s")).read()


def _vregs(op):
    """VGPR numbers an operand names (v7, v[4:5]), else an empty set."""
    m = re.fullmatch(r"v(\d+)", op)
    if m:
        return {int(m.group(1))}
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", op)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    return set()


def _ops(text):
    parts = text.split(None, 1)
    if len(parts) < 2:
        return parts[0], []
    return parts[0], [o.strip() for o in parts[1].split(",")]


def _hazards(lines):
    """(line index, reason) of every DPP instruction that breaks the rule.
    Walking back across a label follows every way into it: the fall-through
    (unless an unconditional branch ends the block above) and every branch to
    it."""
    branches = {}
    for j, t in enumerate(lines):
        m = re.match(r"s_(?:c?branch\w*)\s+(\.LBB\S+)", t)
        if m:
            branches.setdefault(m.group(1) + ":", []).append(j)

    def walk(j, ws, src0, seen):
        """Hazard reason walking back from line j with ws wait states behind, or None."""
        while j >= 0 and ws < 5:
            prev = lines[j]
            if prev.endswith(":"):  # a label: every way in
                if (j, ws) in seen:
                    return None
                seen.add((j, ws))
                for bj in branches.get(prev, []):
                    why = walk(bj, ws, src0, seen)
                    if why:
                        return why
                if j > 0 and lines[j - 1].startswith("s_branch"):
                    return None
                j -= 1
                continue
            op, pops = _ops(prev)
            if op.startswith("v_cmpx") or (op.startswith("v_") and pops and pops[0].startswith("exec")):
                return f"EXEC write `{prev}` {ws} wait states before"
            if op.startswith("v_") and not op.startswith(("v_cmp", "v_readlane", "v_readfirstlane")) and pops:
                if _vregs(pops[0]) & src0 and ws < 2:
                    return f"VALU write of the DPP source `{prev}` {ws} wait states before"
            ws += int(pops[0]) + 1 if op == "s_nop" else 1
            j -= 1
        if j < 0 and ws < 5:
            return "kernel entry within the window"
        return None

    bad = []
    for i, text in enumerate(lines):
        if not re.match(r"v_\w+_dpp\b", text):
            continue
        _, ops = _ops(re.split(r" (?:row_|quad_perm)", text)[0])
        why = walk(i - 1, 0, _vregs(ops[1]), set())
        if why:
            bad.append((i, why))
    return bad


def _kernels(s):
    for m in re.finditer(r"^(_Z\S*dare_row_kernel\S*):[ \t]*(?:;.*)?$", s, re.M):
        body = s[m.end():s.index(".Lfunc_end", m.end())]
        lines = []
        for ln in body.splitlines():
            t = ln.split(";")[0].strip()
            if t and not t.startswith((".", "//")) or re.match(r"^\.LBB\S*:$", t):
                lines.append(t)
        yield m.group(1), lines


def test_dpp_fma_hazards(asm):
    n_fmac = 0
    for name, lines in _kernels(asm):
        n_fmac += sum(t.startswith("v_fmac_f64_dpp") for t in lines)
        bad = _hazards(lines)
        assert not bad, (name, [(lines[i], why) for i, why in bad[:5]])
    assert n_fmac > 0


def test_checker_catches_hazards():
    ok = ["s_nop 4", "v_fmac_f64_dpp v[0:1], v[2:3], v[4:5] row_newbcast:0 row_mask:0xf bank_mask:0xf"]
    assert _hazards(ok) == []
    write = ["s_nop 4", "v_mov_b64_e32 v[2:3], v[8:9]", ok[1]]
    assert _hazards(write) and "VALU write" in _hazards(write)[0][1]
    exe = ["v_cmpx_lt_f64_e32 vcc, 0, v[6:7]", "v_mov_b32_e32 v9, 0", ok[1]]
    assert _hazards(exe) and "EXEC" in _hazards(exe)[0][1]
    # a branch into the block from a point 1 wait state after writing the source
    lab = ["s_nop 4", "v_mov_b64_e32 v[2:3], v[8:9]", "s_cbranch_vccz .LBB0_3", "s_nop 4", ".LBB0_3:", ok[1]]
    assert _hazards(lab) and "VALU write" in _hazards(lab)[0][1]
    # the same with a long fall-through path only: clean
    assert _hazards(["s_nop 4", "v_mov_b64_e32 v[2:3], v[8:9]", "s_nop 4", ".LBB0_3:", "v_mov_b32_e32 v9, 0",
                     ok[1]]) == []
