#!/usr/bin/env python3
"""Register use, spills and LDS of libyoda's kernels, from the built object (no GPU needed).

    python3 tools/kernel_regs.py [regex]      (default: the block kernels K1 / K2)
"""
import os
import re
import subprocess
import sys
import tempfile

L = "/opt/rocm/lib/llvm/bin"
OBJ = os.environ.get("OBJ") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                             "kubernetes-scheduler_amd", "csrc", "build",
                                             "yoda_kernels.o")


def notes(obj):
    with tempfile.TemporaryDirectory() as t:
        fat, co = os.path.join(t, "fat.bin"), os.path.join(t, "k.co")
        subprocess.run([f"{L}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj,
                        os.devnull], check=True)
        subprocess.run([f"{L}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"],
                       check=True)
        return subprocess.run([f"{L}/llvm-readelf", "--notes", co], check=True,
                              capture_output=True, text=True).stdout


def kernels(text):
    """One dict per kernel of the AMDGPU metadata (the keys after its `.args` list)."""
    rows, cur, in_args = [], {}, False
    for line in text.splitlines():
        m = re.match(r"(\s*)(- )?\.(\w+):\s*(.*)", line)
        if not m:
            continue
        indent, dash, k, v = len(m.group(1)), m.group(2), m.group(3), m.group(4).strip()
        if k == "args" and indent <= 4:
            if cur:
                rows.append(cur)
            cur, in_args = {}, True
            continue
        if in_args and indent > 4:
            continue
        in_args = False
        cur[k] = v
    if cur:
        rows.append(cur)
    return rows


def main():
    pat = re.compile(sys.argv[1] if len(sys.argv) > 1 else "k1_block_n32|k2_block_n32")
    for r in kernels(notes(OBJ)):
        n = r.get("name", "")
        if pat.search(n):
            print(f"{r.get('vgpr_count', '?'):>4} vgpr {r.get('vgpr_spill_count', '?'):>3} vspill"
                  f" {r.get('agpr_count', '?'):>3} agpr {r.get('sgpr_count', '?'):>4} sgpr"
                  f" {r.get('sgpr_spill_count', '?'):>3} sspill"
                  f" {r.get('group_segment_fixed_size', '?'):>6} lds  {n[:140]}")


if __name__ == "__main__":
    main()
