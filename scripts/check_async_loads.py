#!/usr/bin/env python3
"""Static guard for the untracked (inline-asm) global loads of fused_v2.hip.

The compiler does not know those loads are in flight, so nothing may read or write a
load's destination VGPRs before an `s_waitcnt vmcnt(N)` has retired the load.  This
runs a forward dataflow over each kernel's basic blocks: the state maps every pending
asm-load destination to its age (vector-memory ops issued after it: every global_,
buffer_, scratch_ and flat_ op counts on vmcnt), merged by minimum age at control-flow
joins; `s_waitcnt vmcnt(N)` retires entries of age >= N.  Any instruction other than
another asm load touching a pending destination is reported.  Join blocks that branch
on a flag every predecessor sets to a constant are split per predecessor (specialize).

  hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S -o v2.s fused_v2.hip
  python scripts/check_async_loads.py v2.s [kernel-substring]
Exit status 1 on any violation (or when no kernel matched).
"""
import re
import sys

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
VMEM = ("global_", "buffer_", "scratch_", "flat_")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return frozenset(out)


def parse_blocks(body):
    """body: [(lineno, text)] -> ordered blocks [(label, [(ln, insn, is_asm)], succs)]."""
    blocks, cur_label, cur, in_asm = [], "entry", [], False
    order = []

    def close(label, insns):
        blocks.append([label, insns, []])

    for ln, raw in body:
        s = raw.strip()
        if s.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if s.startswith(";;#ASMEND"):
            in_asm = False
            continue
        m = re.match(r"^(\.LBB\S+):", s)
        if m:
            close(cur_label, cur)
            cur_label, cur = m.group(1), []
            continue
        code = s.split(";")[0].strip()
        if not code or code.startswith("."):
            continue
        cur.append((ln, code, in_asm))
        op = code.split()[0]
        if op.startswith("s_cbranch") or op == "s_branch" or op == "s_setpc_b64":
            close(cur_label, cur)
            cur_label, cur = f"__after{ln}", []
    close(cur_label, cur)
    idx = {b[0]: i for i, b in enumerate(blocks)}
    for i, b in enumerate(blocks):
        last = b[1][-1][1] if b[1] else ""
        op = last.split()[0] if last else ""
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = last.split()[1]
            if tgt in idx:
                b[2].append(idx[tgt])
            if op != "s_branch" and i + 1 < len(blocks):
                b[2].append(i + 1)
        elif i + 1 < len(blocks):
            b[2].append(i + 1)
    return blocks


SREG = re.compile(r"\bs\[(\d+):(\d+)\]|\bs(\d+)\b")


def sregs(text):
    out = set()
    for m in SREG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def dest(code):
    parts = code.split(None, 1)
    return parts[1].split(",")[0].strip() if len(parts) > 1 else ""


def const_of(insns, pair):
    """Value the block leaves in the SGPR pair (s_mov_b64 <pair>, imm as its last write)."""
    val = None
    for _, code, _ in insns:
        if pair & sregs(dest(code)):
            m = re.match(r"s_mov_b64\s+s\[(\d+):(\d+)\],\s*(-?\d+)$", code)
            val = int(m.group(3)) if m and set(range(int(m.group(1)), int(m.group(2)) + 1)) == pair else None
    return val


def specialize(blocks):
    """Clone a join block that ends `s_and_b64 vcc, exec, s[a:b]` + `s_cbranch_vcc(n)z`
    once per predecessor when every predecessor leaves a known constant (0 or -1) in
    s[a:b]: each clone keeps only the successor that constant selects.  The compiler
    emits this for 'was the loop entered' flags; without it the dataflow merges the
    loop-exit state into a path that only the skipped-loop predecessor can take."""
    i = 0
    while i < len(blocks):
        label, insns, succs = blocks[i]
        last = insns[-1][1] if insns else ""
        op = last.split()[0] if last else ""
        if op in ("s_cbranch_vccz", "s_cbranch_vccnz") and len(insns) >= 2:
            pair = None
            for j in range(len(insns) - 2, -1, -1):
                code = insns[j][1]
                m = re.match(r"s_and_b64\s+vcc,\s*exec,\s*s\[(\d+):(\d+)\]$", code)
                if m:
                    pair = set(range(int(m.group(1)), int(m.group(2)) + 1))
                    before = insns[:j]
                    break
                if "vcc" in dest(code) or code.startswith(("s_cbranch", "s_branch")):
                    break
            preds = [p for p, b in enumerate(blocks) if i in b[2]]
            if pair and len(preds) > 1 and "@" not in label and not any(pair & sregs(dest(c)) for _, c, _ in before):
                vals = [const_of(blocks[p][1], pair) for p in preds]
                if all(v in (0, -1) for v in vals):
                    tgt = last.split()[1]
                    taken = [t for t in succs if blocks[t][0] == tgt]
                    fall = [t for t in succs if blocks[t][0] != tgt]
                    for p, v in zip(preds, vals):
                        zero = v == 0  # vcc = exec & v; exec is non-zero on a uniform branch
                        go = taken if (zero == (op == "s_cbranch_vccz")) else fall
                        blocks.append([f"{label}@{p}", insns, list(go)])
                        blocks[p][2] = [len(blocks) - 1 if t == i else t for t in blocks[p][2]]
        i += 1
    return blocks


def transfer(state, insns, report, name):
    st = dict(state)
    bad = 0
    for ln, code, is_asm in insns:
        op = code.split()[0]
        args = code[len(op):]
        m = re.search(r"vmcnt\((\d+)\)", code) if op.startswith("s_waitcnt") else None
        if m:
            n = int(m.group(1))
            st = {r: a for r, a in st.items() if a < n}
            continue
        if op == "s_waitcnt" and args.strip() == "0":
            st = {}
            continue
        touched = regs(args)
        is_vmem = op.startswith(VMEM)
        # an LDS-DMA load (global_load_lds_*, buffer_load ... lds) has no VGPR destination:
        # its first operand is the address; it only ages the other loads
        is_asm_load = is_vmem and is_asm and "load" in op and "_lds" not in op and not args.rstrip().endswith(" lds")
        if not is_asm_load:
            hit = [r for r in st if r & touched]
            if hit and report:
                print(f"{name}:{ln}: touches in-flight load destination {sorted(set().union(*hit) & touched)}: {code}")
            bad += len(hit) > 0
        if is_vmem:
            st = {r: a + 1 for r, a in st.items()}
            if is_asm_load:
                dst = regs(args.split(",")[0])
                st = {r: a for r, a in st.items() if not (r & dst)}
                st[dst] = 0
    return st, bad


def check(body, name):
    blocks = specialize(parse_blocks(body))
    ins = [None] * len(blocks)
    ins[0] = {}
    work = [0]
    while work:
        i = work.pop()
        out, _ = transfer(ins[i], blocks[i][1], False, name)
        for s in blocks[i][2]:
            if ins[s] is None:
                new = dict(out)
            else:
                new = dict(ins[s])
                for r, a in out.items():
                    new[r] = min(a, new.get(r, a))
            if new != ins[s]:
                ins[s] = new
                work.append(s)
    bad = 0
    for i, b in enumerate(blocks):
        if ins[i] is not None:
            bad += transfer(ins[i], b[1], True, name)[1]
    return bad


def valu_sgpr_dests(code):
    """SGPRs a VALU instruction writes: its first operand when that is an SGPR
    (v_readlane / v_readfirstlane / v_cmp_*_e64 / v_*_co_* carry-out in VOP3b form take
    the SGPR as destination), plus the carry-out of v_*_co_* / v_div_scale."""
    op = code.split()[0]
    if not op.startswith("v_"):
        return set()
    ops = [x.strip() for x in code[len(op):].split(",")]
    out = set()
    if ops and ops[0].startswith(("s", "vcc")):
        out |= sregs(ops[0]) if ops[0].startswith("s") else {-1}
    if ("_co_" in op or op.startswith("v_div_scale")) and len(ops) > 1:
        if ops[1].startswith("s"):
            out |= sregs(ops[1])
        elif ops[1].startswith("vcc"):
            out.add(-1)
    return out


def sgpr_hazards(body, name, report=True):
    """gfx9 hazard the compiler does not guard for inline asm: a VALU write of an SGPR
    read by a vector-memory instruction needs 5 wait states in between (the asm loads'
    buffer resource / soffset / saddr).  Scans back over the linear instruction stream
    (over-approximating across labels); s_nop N counts N + 1 states."""
    insns = []
    in_asm = False
    for ln, raw in body:
        t = raw.strip()
        if t.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if t.startswith(";;#ASMEND"):
            in_asm = False
            continue
        code = t.split(";")[0].strip()
        if not code or code.startswith(".") or code.endswith(":"):
            continue
        insns.append((ln, code, in_asm))
    bad = 0
    for i, (ln, code, is_asm) in enumerate(insns):
        op = code.split()[0]
        if not (is_asm and op.startswith(VMEM)):
            continue
        used = sregs(code[len(op):])
        if not used:
            continue
        states, j = 0, i - 1
        while j >= 0 and states < 5:
            pc = insns[j][1]
            pop = pc.split()[0]
            w = valu_sgpr_dests(pc) & used
            if w:
                bad += 1
                if report:
                    print(f"{name}:{ln}: VALU SGPR write {sorted(w)} {states} wait states before asm VMEM: "
                          f"{pc} -> {code}")
                break
            m = re.match(r"s_nop\s+(\d+)", pc)
            states += int(m.group(1)) + 1 if m else 1
            j -= 1
    return bad


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else "k_ehx"
    text = open(path).read().split("\n")
    funcs, cur = [], None
    for i, l in enumerate(text, 1):
        m = re.match(r"^(_Z\S+):", l)
        if m:
            cur = (m.group(1), [])
            funcs.append(cur)
            continue
        if cur is not None:
            # a kernel may hold several s_endpgm (warp-specialised roles return early);
            # the function ends at its .Lfunc_end label
            if l.startswith(".Lfunc_end"):
                cur = None
                continue
            cur[1].append((i, l))
    total, n = 0, 0
    for name, body in funcs:
        if want in name:
            n += 1
            b = check(body, name[:70]) + sgpr_hazards(body, name[:70])
            total += b
            print(f"{name[:70]}: {b} violations")
    print(f"checked {n} kernels, {total} violations")
    sys.exit(1 if total or n == 0 else 0)


if __name__ == "__main__":
    main()
