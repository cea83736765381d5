#!/usr/bin/env python3
"""Dev tool: the vector-memory / wait / barrier skeleton of one kernel in a hipcc object (gfx950).
usage: tools/isa_waits.py <object.o> <kernel-name-regex>"""
import re
import subprocess
import sys
import tempfile
from pathlib import Path

LLVM = Path("/opt/rocm/lib/llvm/bin")
obj, pat = sys.argv[1], sys.argv[2]
with tempfile.TemporaryDirectory() as td:
    fb, co = Path(td) / "fb.bin", Path(td) / "k.co"
    subprocess.run([str(LLVM / "llvm-objcopy"), f"--dump-section=.hip_fatbin={fb}", obj], check=True)
    subprocess.run([str(LLVM / "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fb}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    dis = subprocess.run([str(LLVM / "llvm-objdump"), "-d", str(co)], capture_output=True, text=True).stdout
m = re.search(r"^[0-9a-f]+ <([^>]*" + pat + r"[^>]*)>:\n(.*?)(?:\n\n|\Z)", dis, re.S | re.M)
lines = m.group(2).split("\n")
prev = None
for i, l in enumerate(lines):
    ins = l.strip().split("//")[0].strip()
    op = ins.split(" ")[0] if ins else ""
    key = None
    if re.match(r"(global|buffer|scratch|flat)_", op):
        key = op
    elif op == "s_waitcnt" and "vmcnt" in ins:
        key = ins
    elif op in ("s_barrier", "s_sleep") or op.startswith("s_cbranch") or op == "s_branch":
        key = ins if op.startswith("s_cbranch") or op == "s_branch" else op
    elif op.startswith("ds_read") or op.startswith("ds_write"):
        key = op.split("_")[0] + "_" + op.split("_")[1]
    elif op.startswith("v_fma_f64"):
        key = "v_fma_f64"
    if key is None:
        continue
    if key == prev and not key.startswith("s_"):
        continue
    print(i, key)
    prev = key
