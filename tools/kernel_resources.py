"""Per-kernel register / scratch usage of the product library's gfx950 code objects.

Reads the AMDGPU metadata notes (.vgpr_count, .agpr_count, .private_segment_fixed_size = scratch bytes per lane,
.vgpr_spill_count) of every kernel in eventstreamgpt_amd/csrc/build/*.o: each object's gfx950 offload bundle is
extracted with llvm-objdump --offloading into a temporary directory and its notes parsed from llvm-readelf.

    python tools/kernel_resources.py [--scratch-only]
"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(REPO, "eventstreamgpt_amd", "csrc", "build")
LLVM = "/opt/rocm/lib/llvm/bin"
_KEYS = ("name", "private_segment_fixed_size", "vgpr_count", "agpr_count", "vgpr_spill_count", "sgpr_count")


def _parse_notes(text: str) -> list:
    kernels, cur = [], {}
    for line in text.splitlines():
        m = re.match(r"\s*-?\s*\.(\w+):\s+(\S+)", line)
        if not m or m.group(1) not in _KEYS:
            continue
        k, v = m.groups()
        if k == "agpr_count" and cur:  # every kernel's metadata map starts with .agpr_count (sorted keys)
            kernels.append(cur)
            cur = {}
        cur[k] = v if k == "name" else int(v)
    if cur:
        kernels.append(cur)
    return kernels


def demangle(names: list) -> list:
    try:
        out = subprocess.run([os.path.join(LLVM, "llvm-cxxfilt")], input="\n".join(names), capture_output=True,
                             text=True, check=True).stdout.splitlines()
        return out if len(out) == len(names) else names
    except (OSError, subprocess.CalledProcessError):
        return names


def kernel_resources(build_dir: str = BUILD) -> list:
    """[{object, name, private_segment_fixed_size, vgpr_count, agpr_count, vgpr_spill_count, ...}] for every kernel of
    every object in build_dir."""
    out = []
    with tempfile.TemporaryDirectory() as td:
        for f in sorted(os.listdir(build_dir)):
            if not f.endswith(".o"):
                continue
            local = os.path.join(td, f)
            shutil.copy(os.path.join(build_dir, f), local)
            subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", local], capture_output=True, check=True)
            cos = [c for c in os.listdir(td) if c.startswith(f + ".") and c.endswith("gfx950")]
            for co in cos:
                notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", os.path.join(td, co)],
                                       capture_output=True, text=True, check=True).stdout
                for k in _parse_notes(notes):
                    k["object"] = f[:-2]
                    out.append(k)
    return out


def main():
    ks = kernel_resources()
    if "--scratch-only" in sys.argv:
        ks = [k for k in ks if k.get("private_segment_fixed_size", 0) > 0]
    names = demangle([k["name"] for k in ks])
    for k, n in zip(ks, names):
        print(f"{k['object']:16s} scratch {k.get('private_segment_fixed_size', 0):4d} B  vgpr {k.get('vgpr_count', 0):3d}  "
              f"agpr {k.get('agpr_count', 0):3d}  spills {k.get('vgpr_spill_count', 0):3d}  {n[:160]}")


if __name__ == "__main__":
    main()
