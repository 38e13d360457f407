"""The C-ABI library builds, loads without a GPU and exports every symbol include/ declares."""
import os
import re
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "cuda-sdr_amd", "lib", "libgpusdrpipeline.so")
EXPORT_RE = re.compile(r"^\s*(?:GSDR_API|GSDR_CONV_API|GSP_API|GS_EXPORT)\b[^(]*?\b([A-Za-z_][A-Za-z0-9_]*)\s*\(", re.M)
NOISE_RE = re.compile(r"GS_FMT_ATTR\([^)]*\)|\[\[[^\]]*\]\]")


def declared_symbols():
    names = set()
    for root, _, files in os.walk(os.path.join(REPO, "include")):
        for f in files:
            if f.endswith(".h"):
                with open(os.path.join(root, f)) as fh:
                    names.update(EXPORT_RE.findall(NOISE_RE.sub("", fh.read())))
    return names


def exported_symbols():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], check=True, capture_output=True, text=True).stdout
    return {line.split()[-1] for line in out.splitlines() if len(line.split()) >= 3}


@pytest.fixture(scope="module")
def built():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(REPO, "cuda-sdr_amd")], check=True)
    return LIB


def test_every_declared_symbol_is_exported(built):
    declared = declared_symbols()
    assert {"gsdrFirFC", "gsdrQuadAmDemod", "gsdrInt8ToNormFloat"} <= declared
    missing = declared - exported_symbols()
    assert not missing, sorted(missing)


def test_library_is_gfx950_code(built):
    with open(built, "rb") as f:
        blob = f.read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"--gfx942" not in blob and b"--gfx90a" not in blob


def test_library_loads_without_gpu(built):
    code = ("import ctypes,sys; L=ctypes.CDLL(sys.argv[1]); "
            "assert L.gsdrFirFC and L.gsdrInt8FirFCAmDemod; print('ok')")
    r = subprocess.run([sys.executable, "-c", code, built], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr


# Every public header path of the reference's include/gpusdrpipeline that a drop-in caller may
# include (the reference's application-only headers SdrSession.h, am.h, fm.h and
# util/{ScopeExit,Thread,Window}.h are outside the hot path and not provided).
REFERENCE_HEADER_PATHS = [
    "CudaErrors.h", "Factories.h", "GSDefs.h", "GSErrors.h", "GSLog.h", "IMemory.h", "IRef.h",
    "Modulation.h", "Result.h", "SampleType.h", "Status.h", "util/CudaDevicePushPop.h", "util/CudaUtil.h",
]


def test_reference_header_paths_compile(tmp_path):
    """The reference's include paths exist and compile; the CUDA-named error / device-scope
    macros of CudaErrors.h and util/CudaDevicePushPop.h forward to the HIP ones."""
    src = tmp_path / "inc.cpp"
    body = "".join(f"#include <gpusdrpipeline/{h}>\n" for h in REFERENCE_HEADER_PATHS)
    body += """#include <stdexcept>
Status f(int d) {
  CUDA_DEV_PUSH_POP_OR_RET_STATUS(d);
  SAFE_CUDA_OR_RET_STATUS(hipDeviceSynchronize());
  CHECK_CUDA_OR_RET_STATUS("launch");
  return cudaErrorToStatus(hipErrorInvalidValue);
}
int main() { CudaDevicePushPop p(0); (void)p; return 0; }
"""
    src.write_text(body)
    r = subprocess.run(["/opt/rocm/lib/llvm/bin/clang++", "-std=c++20", "-fsyntax-only", "-D__HIP_PLATFORM_AMD__",
                        "-I/opt/rocm/include", "-I" + os.path.join(REPO, "include"), str(src)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr


def _library_build_id(path):
    code = ("import ctypes,sys; L=ctypes.CDLL(sys.argv[1]); f=L.gsdrAmdBuildId; "
            "f.restype=ctypes.c_char_p; print(f().decode())")
    r = subprocess.run([sys.executable, "-c", code, path], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return r.stdout.strip()


def _check_build_id(path):
    sys.path.insert(0, os.path.join(REPO, "tools"))
    from source_hash import source_hash
    tree = source_hash(REPO)
    lib_id = _library_build_id(path)
    assert lib_id == tree, (f"{path} was built from other sources (build id {lib_id}) than this tree "
                            f"({tree}): rebuild it (make -C cuda-sdr_amd) before testing")


def test_library_matches_source_tree(built):
    """Build provenance: the library's embedded source hash equals the tree's."""
    _check_build_id(built)


def test_build_id_folds_in_compile_flags():
    """the id covers EXTRA_FLAGS (the -D switches of A/B and diagnostic builds) and
    the target, so a library built with, e.g., -DGSDR_WS_RING_ZERO=0 (the r04 stale-LDS defect) cannot
    pass test_library_matches_source_tree; whitespace in the flags does not change it."""
    sys.path.insert(0, os.path.join(REPO, "tools"))
    from source_hash import source_hash
    product = source_hash(REPO)
    assert source_hash(REPO, extra_flags="-DGSDR_WS_RING_ZERO=0") != product
    assert source_hash(REPO, extra_flags="-DGSDR_WS_DIAG=1") != product
    assert source_hash(REPO, arch="gfx942") != product
    assert source_hash(REPO, extra_flags="  ") == product
    # the Makefile's stamp makes every object depend on the flags, and the id is computed with them
    mk = open(os.path.join(REPO, "cuda-sdr_amd", "Makefile")).read()
    assert "--extra-flags='$(EXTRA_FLAGS)'" in mk and "$(FLAGSTAMP)" in mk


def test_build_id_independent_of_compiler_location(built, tmp_path):
    """the id does not depend on the checking machine's compiler (a missing hipcc, or ROCm
    installed elsewhere, gave another id for the same sources); the compiler's version numbers are embedded
    beside it (gsdrAmdBuildCompiler) without install paths."""
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import source_hash as sh
    assert sh.compiler_version(str(tmp_path / "no-such-hipcc")) == ""
    assert "/" not in sh.compiler_version()
    code = ("import ctypes,sys; L=ctypes.CDLL(sys.argv[1]); f=L.gsdrAmdBuildCompiler; "
            "f.restype=ctypes.c_char_p; print(f().decode())")
    r = subprocess.run([sys.executable, "-c", code, built], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == sh.compiler_version()


@pytest.mark.gpu
def test_gpu_box_library_matches_source_tree():
    """The same check where the GPU suite runs: the pushed, prebuilt .so the box loads must be the one
    built from the tree it runs with, so a stale library fails loudly instead of passing the suite."""
    assert os.path.exists(LIB), LIB
    _check_build_id(LIB)
