"""The source digest that ties libiddgcn_hip.so to the tree it was built from.

``__graft_entry__.build()`` compiles the digest of the library's sources into the library itself
(``iddgcn_source_sha256()``, include/iddgcn.h); ``_lib.load`` recomputes it from the tree beside the library and
refuses a library whose digest differs, so a stale build can never be loaded and tested in place of HEAD's.
The digest covers every input of the device build: the HIP sources, the device code-generation flags and the
public headers.
"""
import glob
import hashlib
import os

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)


def source_files(root=ROOT):
    """Repo-relative paths of the build inputs, sorted."""
    pats = ("iddgcn_amd/csrc/*.hip", "iddgcn_amd/csrc/device_flags.txt", "include/*.h")
    files = set()
    for p in pats:
        files.update(os.path.relpath(f, root) for f in glob.glob(os.path.join(root, p)))
    return sorted(files)


def source_sha256(root=ROOT):
    """sha256 over (relative path, contents) of every build input, in sorted order."""
    h = hashlib.sha256()
    for rel in source_files(root):
        h.update(rel.replace(os.sep, "/").encode() + b"\0")
        with open(os.path.join(root, rel), "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()
