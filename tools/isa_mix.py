#!/usr/bin/env python3
"""Dev tool: instruction-mix histogram of the kernels matching a regex in a hipcc object or in libmfhe.so
(gfx950 code objects).  Prints, per kernel, the VGPR / SGPR / scratch / LDS metadata line from the disassembly
header and the count of each opcode, VALU first.
usage: tools/isa_mix.py <object.o | libmfhe.so> <kernel-name-regex> [top]"""
import collections
import re
import subprocess
import sys
import tempfile
from pathlib import Path

LLVM = Path("/opt/rocm/lib/llvm/bin")


def code_objects(path: str):
    with tempfile.TemporaryDirectory() as td:
        fb = Path(td) / "fb.bin"
        subprocess.run([str(LLVM / "llvm-objcopy"), f"--dump-section=.hip_fatbin={fb}", path], check=True)
        data = fb.read_bytes()
        # one offload bundle per translation unit in a linked .so; each starts with the bundler magic
        magic = b"__CLANG_OFFLOAD_BUNDLE__"
        starts = [m.start() for m in re.finditer(re.escape(magic), data)]
        for i, s in enumerate(starts):
            e = starts[i + 1] if i + 1 < len(starts) else len(data)
            part, co = Path(td) / f"b{i}.bin", Path(td) / f"k{i}.co"
            part.write_bytes(data[s:e])
            r = subprocess.run([str(LLVM / "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={part}",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], capture_output=True)
            if r.returncode == 0 and co.exists() and co.stat().st_size:
                dis = subprocess.run([str(LLVM / "llvm-objdump"), "-d", str(co)], capture_output=True,
                                     text=True).stdout
                notes = subprocess.run([str(LLVM / "llvm-readelf"), "--notes", str(co)], capture_output=True,
                                       text=True).stdout
                yield dis, kernel_meta(notes)


def kernel_meta(notes: str):
    """{kernel symbol: "vgpr V agpr A sgpr S scratch B lds L"} from the code object's metadata note"""
    out = {}
    for blk in re.split(r"\n\s+- \.", notes):
        m = re.search(r"\.symbol:\s+(\S+)\.kd", blk)
        if not m:
            continue
        f = {k: re.search(rf"\.{k}:\s+(\d+)", blk) for k in
             ("vgpr_count", "agpr_count", "sgpr_count", "private_segment_fixed_size", "group_segment_fixed_size")}
        v = {k: (x.group(1) if x else "?") for k, x in f.items()}
        out[m.group(1)] = (f"vgpr {v['vgpr_count']} agpr {v['agpr_count']} sgpr {v['sgpr_count']} "
                           f"scratch {v['private_segment_fixed_size']} lds {v['group_segment_fixed_size']}")
    return out


def main():
    path, pat = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    for dis, meta in code_objects(path):
        for m in re.finditer(r"^[0-9a-f]+ <([^>]*)>:\n(.*?)(?:\n\n|\Z)", dis, re.S | re.M):
            name = m.group(1)
            if not re.search(pat, name):
                continue
            cnt = collections.Counter()
            for l in m.group(2).split("\n"):
                ins = l.strip().split("//")[0].strip()
                if ins:
                    cnt[ins.split(" ")[0]] += 1
            valu = sum(v for k, v in cnt.items() if k.startswith("v_"))
            print(f"== {name[:150]}\n   {meta.get(name, 'no metadata')}\n   total {sum(cnt.values())}  VALU {valu}")
            for k, v in sorted(cnt.items(), key=lambda kv: (not kv[0].startswith("v_"), -kv[1]))[:top]:
                print(f"   {v:6d} {k}")


if __name__ == "__main__":
    main()
