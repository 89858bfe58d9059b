"""Register usage of every kernel in a HIP object (build/*.o): VGPR / AGPR / SGPR counts
and spills from the code object's metadata notes.
  python scripts/kernel_regs.py zs3server_amd/build/fused_v2.hip.o [name-filter]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/llvm/bin"
obj, filt = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
with tempfile.TemporaryDirectory() as d:
    fb, co = os.path.join(d, "fb"), os.path.join(d, "co")
    subprocess.check_call([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj, os.path.join(d, "x")])
    subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                           "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"])
    notes = subprocess.run([f"{LLVM}/llvm-readobj", "--notes", co], capture_output=True, text=True).stdout
recs, cur = [], {}
for line in notes.splitlines():
    m = re.match(r"\s*-?\s*(\.[a-z_]+):\s+(\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == ".agpr_count" and cur:
        recs.append(cur)
        cur = {}
    cur[k] = v
if cur:
    recs.append(cur)
for r in recs:
    n = r.get(".name", "")
    if ".vgpr_count" not in r or filt not in n:
        continue
    dm = subprocess.run(["c++filt"], input=n, capture_output=True, text=True).stdout.strip()
    print(f"v{r['.vgpr_count']:>4} a{r.get('.agpr_count', '0'):>3} vspill{r.get('.vgpr_spill_count', '0'):>4} "
          f"s{r.get('.sgpr_count', '?'):>4} sspill{r.get('.sgpr_spill_count', '0'):>4}  {dm}")
