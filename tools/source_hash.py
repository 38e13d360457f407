#!/usr/bin/env python3
"""Build provenance: one sha256 over what libgpusdrpipeline.so is built from - the sources (the kernels,
the runtime, the C API, the public headers and the Makefile, path by path in sorted order), the extra
compile flags (EXTRA_FLAGS: the -D switches of A/B and diagnostic builds) and the target architecture.
The Makefile embeds it in the library (gsdrAmdBuildId) and, beside it, the compiler's version
(gsdrAmdBuildCompiler: the HIP and clang version numbers, no install paths - r06, ADVICE r05: hashing
`hipcc --version` of the checking machine made the id depend on where ROCm is installed);
tests/test_abi_exports.py compares the two, so a stale pushed .so - or one built with a diagnostic or
A/B define - fails loudly instead of testing other code than the tree's.
Usage: source_hash.py [repo root] [--extra-flags FLAGS] [--arch ARCH]  -> prints the 16-hex-digit id
       source_hash.py --compiler-version [--hipcc PATH]                -> prints the compiler's version"""
import argparse
import functools
import hashlib
import os
import re
import subprocess

SUFFIXES = (".hip", ".cpp", ".h", ".hpp")
DEFAULT_HIPCC = "/opt/rocm/bin/hipcc"
DEFAULT_ARCH = "gfx950"


def source_files(root):
    pkg = os.path.join(root, "cuda-sdr_amd")
    files = [os.path.join(pkg, "Makefile")]
    for top in (os.path.join(pkg, "csrc"), os.path.join(root, "include")):
        for d, _, names in os.walk(top):
            files += [os.path.join(d, n) for n in names if n.endswith(SUFFIXES)]
    return sorted(files, key=lambda p: os.path.relpath(p, root))


@functools.lru_cache(maxsize=4)
def compiler_version(hipcc=DEFAULT_HIPCC):
    """The compiler's version numbers ("HIP 7.2.26015-fc0010cf6a; clang 22.0.0git roc-7.2.0 26014"), without
    the install paths of `hipcc --version`; '' where it cannot run."""
    try:
        r = subprocess.run([hipcc, "--version"], capture_output=True, text=True, timeout=60)
    except (OSError, subprocess.SubprocessError):
        return ""
    hip = re.search(r"HIP version:\s*(\S+)", r.stdout)
    clang = re.search(r"clang version\s+(\S+)(?:\s+\([^)]*?(roc-\S+\s+\d+))?", r.stdout)
    parts = []
    if hip:
        parts.append("HIP " + hip.group(1))
    if clang:
        parts.append("clang " + clang.group(1) + (" " + clang.group(2) if clang.group(2) else ""))
    return re.sub(r"[^A-Za-z0-9 ._;:+-]", "", "; ".join(parts))


def source_hash(root, extra_flags="", arch=DEFAULT_ARCH):
    """The build id of a library built from `root` with EXTRA_FLAGS=extra_flags (the product build:
    none) for `arch`."""
    h = hashlib.sha256()
    for p in source_files(root):
        rel = os.path.relpath(p, root).replace(os.sep, "/")
        with open(p, "rb") as f:
            data = f.read()
        h.update(rel.encode() + b"\0" + str(len(data)).encode() + b"\0" + data)
    for key, val in (("EXTRA_FLAGS", " ".join(extra_flags.split())), ("ARCH", arch)):
        h.update(b"\1" + key.encode() + b"=" + val.encode() + b"\0")
    return h.hexdigest()[:16]


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("root", nargs="?", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    ap.add_argument("--extra-flags", default="")
    ap.add_argument("--arch", default=DEFAULT_ARCH)
    ap.add_argument("--hipcc", default=DEFAULT_HIPCC)
    ap.add_argument("--compiler-version", action="store_true")
    a = ap.parse_args()
    if a.compiler_version:
        print(compiler_version(a.hipcc))
    else:
        print(source_hash(os.path.abspath(a.root), a.extra_flags, a.arch))
