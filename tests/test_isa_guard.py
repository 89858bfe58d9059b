"""ISA guard for the fused_v2 kernels (CPU, needs hipcc): the kernels issue global loads the
compiler does not track (inline asm, exact s_waitcnt vmcnt(N) by hand), so no
instruction may touch a load's destination VGPRs before a wait retires it.  Compiles
the device code to assembly and runs scripts/check_async_loads.py's dataflow check on
every compiled k_ehx_ws / k_vr_ws instance; a compiler change that copies or re-uses an in-flight
register fails here, before any GPU run."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def _hipcc():
    for c in ("/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    return None


@pytest.mark.skipif(_hipcc() is None, reason="hipcc not available")
@pytest.mark.parametrize("diag", [False, True], ids=["product", "diag"])
def test_untracked_loads_never_touched_in_flight(tmp_path, diag):
    """Both builds: the product library's instances and the diagnostics build's
    experimental ones."""
    import check_async_loads as cal

    # every translation unit that instantiates fused_v2.hpp's kernels, compiled in parallel
    units = ["fused_v2.hip", "fused_v2_gen.hip", "fused_v2_get.hip", "fused_v2_get_gen.hip"] + (
        ["fused_v2_diag.hip"] if diag else [])
    procs = []
    for u in units:
        asm = tmp_path / (u + ".s")
        procs.append((asm, subprocess.Popen(
            [_hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S"]
            + (["-DZS3_DIAG=1"] if diag else []) +
            ["-o", str(asm), os.path.join(ROOT, "zs3server_amd", "csrc", u), "-I", os.path.join(ROOT, "include")],
            stderr=subprocess.DEVNULL)))
    text = []
    for asm, p in procs:
        assert p.wait() == 0, asm
        text += asm.read_text().split("\n")
    funcs, cur = [], None
    for i, line in enumerate(text, 1):
        if line.startswith("_Z") and line.rstrip().endswith(":") or (line.startswith("_Z") and ":" in line and "@" in line):
            name = line.split(":")[0]
            cur = (name, [])
            funcs.append(cur)
            continue
        if cur is not None:
            # a kernel may hold several s_endpgm (k_ehx_ws: the hash role returns early);
            # the function ends at its .Lfunc_end label
            if line.startswith(".Lfunc_end"):
                cur = None
                continue
            cur[1].append((i, line))
    kernels = [(n, b) for n, b in funcs if "k_ehx" in n or "k_vr_ws" in n or "k_vr_quad" in n]
    assert kernels, "no k_ehx instance found in the assembly"
    bad = {n: cal.check(b, n) + cal.sgpr_hazards(b, n) for n, b in kernels}
    assert all(v == 0 for v in bad.values()), bad


def _body(src):
    return [(i, line) for i, line in enumerate(src.strip("\n").split("\n"), 1)]


LOOP_FLAG = """
	s_cbranch_scc0 .LBB0_5
	;;#ASMSTART
	global_load_dwordx2 v[10:11], v[2:3], off
	;;#ASMEND
	s_mov_b64 s[0:1], 0
	s_branch .LBB0_6
.LBB0_5:
	s_waitcnt vmcnt(0)
	s_mov_b64 s[0:1], -1
.LBB0_6:
	s_and_b64 vcc, exec, s[0:1]
	s_cbranch_vccz .LBB0_8
	v_mov_b64_e32 v[10:11], v[20:21]
.LBB0_8:
	s_waitcnt vmcnt(0)
	v_mov_b64_e32 v[30:31], v[10:11]
"""


def test_guard_specializes_loop_entered_flag():
    """The join block's fall-through (the mov into v[10:11]) is reachable only from the
    predecessor that set s[0:1] = -1, where nothing is in flight: no violation.  With
    the flag constants swapped the load path reaches the mov: reported."""
    import check_async_loads as cal
    assert cal.check(_body(LOOP_FLAG), "ok") == 0
    swapped = LOOP_FLAG.replace("s_mov_b64 s[0:1], 0", "s_mov_b64 s[0:1], @").replace(
        "s_mov_b64 s[0:1], -1", "s_mov_b64 s[0:1], 0").replace("s_mov_b64 s[0:1], @", "s_mov_b64 s[0:1], -1")
    assert cal.check(_body(swapped), "bad") == 1
    unknown = LOOP_FLAG.replace("s_mov_b64 s[0:1], 0", "s_mov_b64 s[0:1], s[4:5]")
    assert cal.check(_body(unknown), "unknown") == 1


HAZARD = """
	v_readfirstlane_b32 s6, v4
	;;#ASMSTART
	buffer_load_dword v19, v2, s[28:31], s6 offen
	;;#ASMEND
"""


def test_guard_flags_valu_sgpr_write_before_asm_vmem():
    """A VALU write of an SGPR (v_readfirstlane / v_readlane spill restore) read by an
    inline-asm buffer load needs 5 wait states (gfx9 hazard the compiler does not guard
    for asm): reported without them, accepted after s_nop 4 or 5 other instructions, and
    a compiler-emitted (non-asm) load is not the guard's business."""
    import check_async_loads as cal
    assert cal.sgpr_hazards(_body(HAZARD), "bad", report=False) == 1
    nop = HAZARD.replace("\t;;#ASMSTART", "\ts_nop 4\n\t;;#ASMSTART")
    assert cal.sgpr_hazards(_body(nop), "nop", report=False) == 0
    other = HAZARD.replace("\t;;#ASMSTART", "\ts_add_u32 s0, s1, s2\n" * 5 + "\t;;#ASMSTART")
    assert cal.sgpr_hazards(_body(other), "five", report=False) == 0
    plain = HAZARD.replace("\t;;#ASMSTART\n", "").replace("\t;;#ASMEND\n", "")
    assert cal.sgpr_hazards(_body(plain), "plain", report=False) == 0
