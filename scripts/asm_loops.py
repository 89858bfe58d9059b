#!/usr/bin/env python3
"""Static instruction mix of a kernel's loops from device assembly.

  hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S -o k.s kernels.hip
  python scripts/asm_loops.py k.s 'k_encode_hashILi8ELi4ELi4ELi384ELi1ELi192ELi8ELi1ELb0ELb0ELi4ELb0ELi0E'

For every backward branch (a loop) prints the instruction count of the body by class
(VALU / SALU / LDS / VMEM / other) and the most frequent VALU opcodes, plus the
kernel's VGPR/SGPR/LDS usage from the metadata.
"""
import re
import sys
from collections import Counter


def klass(op: str) -> str:
    if op.startswith("v_"):
        return "VALU"
    if op.startswith("s_") and not op.startswith(("s_waitcnt", "s_barrier", "s_cbranch", "s_branch", "s_nop",
                                                   "s_load", "s_buffer", "s_setprio", "s_sleep")):
        return "SALU"
    if op.startswith("s_load") or op.startswith("s_buffer"):
        return "SMEM"
    if op.startswith("ds_"):
        return "LDS"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "VMEM"
    return "other"


def main() -> None:
    path, pat = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        if re.match(r"^_Z\S*" + re.escape(pat) + r"\S*:", l):
            start = i
            break
    if start is None:
        sys.exit(f"no function matching {pat}")
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    body = lines[start:end]
    labels = {}
    insts = []  # (line_index_in_body, opcode, text)
    for i, l in enumerate(body):
        s = l.strip()
        if re.match(r"^\.LBB\S+:", s):
            labels[s[:-1].split()[0].rstrip(":")] = len(insts)
            continue
        if not s or s.startswith((";", ".", "_Z")):
            continue
        op = s.split()[0]
        insts.append((i, op, s))
    print(f"function: {body[0].split(':')[0][:140]}")
    print(f"total instructions: {len(insts)}")
    for idx, (i, op, s) in enumerate(insts):
        if op.startswith(("s_cbranch", "s_branch")):
            tgt = s.split()[-1]
            if tgt in labels and labels[tgt] <= idx:
                loop = insts[labels[tgt]:idx + 1]
                c = Counter(klass(o) for _, o, _ in loop)
                vc = Counter(o for _, o, _ in loop if o.startswith("v_"))
                print(f"\nloop {tgt} ({len(loop)} insts): " + " ".join(f"{k}={v}" for k, v in sorted(c.items())))
                print("   " + " ".join(f"{o}:{n}" for o, n in vc.most_common(14)))
    meta = "\n".join(lines[end:end + 400])
    for key in ("NumVgprs", "NumAgprs", "NumSgprs", "ScratchSize", "Occupancy", "LDSByteSize"):
        mm = re.search(r"; " + key + r": (\d+)", meta)
        if mm:
            print(f"{key}={mm.group(1)}", end=" ")
    print()


if __name__ == "__main__":
    main()
