"""Register / scratch / LDS usage of the gfx950 kernels in the built library (code-object metadata).

usage: python tools/kernel_regs.py [substring ...]   (default: every kernel)
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "iddgcn_amd", "libiddgcn_hip.so")
KEYS = (".vgpr_count", ".agpr_count", ".sgpr_count", ".vgpr_spill_count", ".private_segment_fixed_size",
        ".group_segment_fixed_size")


def notes(lib):
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section=.hip_fatbin=" + fat, lib,
                        os.path.join(d, "stripped.so")], check=True, capture_output=True)
        blob = open(fat, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(b"__CLANG_OFFLOAD_BUNDLE__"), blob)]
        out = []
        for i, a in enumerate(starts):
            part, dev = os.path.join(d, f"b{i}.bin"), os.path.join(d, f"b{i}.o")
            open(part, "wb").write(blob[a:starts[i + 1] if i + 1 < len(starts) else len(blob)])
            subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", "--input=" + part,
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + dev], check=True,
                           capture_output=True)
            out.append(subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", dev], check=True,
                                      capture_output=True, text=True).stdout)
    return "\n".join(out)


def main():
    pats = sys.argv[1:]
    for item in re.split(r"\n\s+- \.agpr_count", notes(LIB)):
        m = re.search(r"\.name:\s*(\S+)", item)
        if not m or m.group(1).endswith(".kd") or (pats and not any(p in m.group(1) for p in pats)):
            continue
        vals = {k: (re.search(re.escape(k) + r":\s*(\S+)", ".agpr_count:" + item) or [None, "?"])[1] for k in KEYS}
        print(m.group(1)[:90], " ".join(f"{k[1:]}={v}" for k, v in vals.items()))


if __name__ == "__main__":
    main()
