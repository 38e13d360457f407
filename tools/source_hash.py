#!/usr/bin/env python3
"""Build provenance: one sha256 over the sources libgpusdrpipeline.so is built from (the kernels, the
runtime, the C API, the public headers and the Makefile), path by path in sorted order. The Makefile
embeds it in the library (gsdrAmdBuildId); tests/test_abi_exports.py compares the two, so a stale
pushed .so fails loudly instead of testing other code than the tree's.
Usage: source_hash.py [repo root]   -> prints the 16-hex-digit id"""
import hashlib
import os
import sys

SUFFIXES = (".hip", ".cpp", ".h", ".hpp")


def source_files(root):
    pkg = os.path.join(root, "cuda-sdr_amd")
    files = [os.path.join(pkg, "Makefile")]
    for top in (os.path.join(pkg, "csrc"), os.path.join(root, "include")):
        for d, _, names in os.walk(top):
            files += [os.path.join(d, n) for n in names if n.endswith(SUFFIXES)]
    return sorted(files, key=lambda p: os.path.relpath(p, root))


def source_hash(root):
    h = hashlib.sha256()
    for p in source_files(root):
        rel = os.path.relpath(p, root).replace(os.sep, "/")
        with open(p, "rb") as f:
            data = f.read()
        h.update(rel.encode() + b"\0" + str(len(data)).encode() + b"\0" + data)
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(source_hash(os.path.abspath(sys.argv[1] if len(sys.argv) > 1 else
                                      os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))))
