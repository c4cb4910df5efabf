"""Per-kernel digest of a built library's gfx950 code: disassemble every code object of the .so (one offload bundle
per translation unit) and hash each function's instruction text (addresses and encodings stripped).  Two builds
whose digests agree for a kernel run the same machine code for it: used to show that a source refactor (e.g.
removing experiment switches) left the product kernels unchanged.

usage: python tools/kernel_asm_digest.py lib.so > digest.txt ; diff digest_a.txt digest_b.txt
"""
import hashlib
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def disassemble(lib):
    out = []
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section=.hip_fatbin=" + fat, lib,
                        os.path.join(d, "stripped.so")], check=True, capture_output=True)
        blob = open(fat, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(b"__CLANG_OFFLOAD_BUNDLE__"), blob)]
        for i, a in enumerate(starts):
            part, dev = os.path.join(d, f"b{i}.bin"), os.path.join(d, f"b{i}.o")
            open(part, "wb").write(blob[a:starts[i + 1] if i + 1 < len(starts) else len(blob)])
            subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", "--input=" + part,
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + dev], check=True,
                           capture_output=True)
            out.append(subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn",
                                       "--no-leading-addr", dev], check=True, capture_output=True, text=True).stdout)
    return "\n".join(out)


def digests(asm):
    funcs, name, body = {}, None, []
    for line in asm.splitlines():
        m = re.match(r"^[0-9a-f]* ?<(.+)>:$", line.strip())
        if m:
            if name:
                funcs[name] = body
            name, body = m.group(1), []
        elif name and line.strip():
            # branch targets print as addresses / labels: keep only the mnemonic and operands
            body.append(re.sub(r"<[^>]*>|//.*$", "", line).strip())
    if name:
        funcs[name] = body
    # drop what follows a function's last s_endpgm (alignment padding, which depends on the code placed before it)
    for k, v in funcs.items():
        last = max((i for i, ln in enumerate(v) if ln.startswith("s_endpgm")), default=len(v) - 1)
        funcs[k] = v[:last + 1]
    return {k: (hashlib.sha1("\n".join(v).encode()).hexdigest()[:16], len(v)) for k, v in funcs.items()}


if __name__ == "__main__":
    for k, (h, n) in sorted(digests(disassemble(sys.argv[1])).items()):
        print(f"{h} {n:6d} {k}")
