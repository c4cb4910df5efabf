"""List the s_waitcnt vmcnt instructions the compiler inserted (outside inline asm) in the pipelined
LDS-DMA kernels of libiddgcn_hip, with the instruction each one guards.  A compiler vmcnt wait inside a
main loop drains every DMA in flight (A tiles, slabs, stores) and defeats the software pipeline, so the
hot kernels should show none there except in rarely taken branches (e.g. `accumulate` loads).
usage: python tools/check_waits.py [--src file.hip] [kernel-substring ...]   (compiles iddgcn_hip.hip to gfx950 asm)
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(pats, src=None):
    src = src or os.path.join(ROOT, "iddgcn_amd", "csrc", "iddgcn_hip.hip")
    out = os.path.join(tempfile.gettempdir(), "iddgcn_hip_gfx950.s")
    flags = open(os.path.join(ROOT, "iddgcn_amd", "csrc", "device_flags.txt")).read().split()
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", *flags, "-I",
                    os.path.join(ROOT, "include"), "--cuda-device-only", "-S",
                    src, "-o", out], check=True,
                   stderr=subprocess.DEVNULL)
    lines = open(out).read().split("\n")
    starts = [(i, l[:-1]) for i, l in enumerate(lines) if re.match(r"^_Z\S+:", l)]
    for k, (st, name) in enumerate(starts):
        if not any(p in name for p in pats):
            continue
        en = starts[k + 1][0] if k + 1 < len(starts) else len(lines)
        body, inasm, hits = lines[st:en], False, []
        for j, l in enumerate(body):
            t = l.strip()
            if t.startswith(";;#ASMSTART"):
                inasm = True
            elif t.startswith(";;#ASMEND"):
                inasm = False
            elif not inasm and t.startswith("s_waitcnt") and "vmcnt" in t:
                nxt = next((x.strip() for x in body[j + 1:] if x.strip() and not x.strip().startswith(";")), "")
                hits.append(f"    {j:5d} {t:22s} -> {nxt}")
        scratch = sum(1 for l in body if l.strip().startswith("scratch_"))
        print(f"{name}  ({len(body)} lines, {len(hits)} compiler vmcnt waits, {scratch} scratch ops)")
        print("\n".join(hits))


if __name__ == "__main__":
    args = sys.argv[1:]
    src = None
    if args[:1] == ["--src"]:
        src, args = args[1], args[2:]
    main(args or ["rowgemm256_v3_kernel", "gemm_tn256_x3_kernel"], src)
