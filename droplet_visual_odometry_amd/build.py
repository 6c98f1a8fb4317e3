"""Build libdvo_hip.so (the MI355X kernels + C ABI) in-tree with hipcc for gfx950.

Numerics flags are part of the product contract:
  -ffp-contract=off                          no FMA contraction: every float/double
                                             expression rounds like the CPU oracle
  -fhip-fp32-correctly-rounded-divide-sqrt   IEEE f32 division / sqrt
The shared object links the HIP runtime by the unversioned soname
``libamdhip64.so``; when PyTorch-ROCm is loaded first (the bench, the tests)
the dynamic linker reuses torch's copy, so torch tensors and the library share
one HIP runtime and one device address space.
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, "libdvo_hip.so")
ARCH = os.environ.get("DVO_OFFLOAD_ARCH", "gfx950")

CXXFLAGS = [
    "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
    "-ffp-contract=off", "-fno-fast-math", "-fhip-fp32-correctly-rounded-divide-sqrt",
    "-Wall", "-Wno-unused-function", "-Wno-unused-variable", "-Wno-unused-but-set-variable",
]

# Per-file code generation: the matcher's MFMA accumulators in VGPRs (no
# v_accvgpr_read of 32 accumulators per 32 trains before the epilogue; match
# stage 1.52 -> 1.43 ms per 1024 pairs, tools/ab_stages.sh).
FILE_FLAGS = {"match.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]}


def _torch_lib_dir():
    try:
        import torch  # noqa: F401  (location only; the library never calls torch)
        d = os.path.join(os.path.dirname(torch.__file__), "lib")
        if os.path.exists(os.path.join(d, "libamdhip64.so")):
            return d
    except Exception:
        pass
    return None


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def inputs():
    """Every file the library is compiled from."""
    return sources() + sorted(glob.glob(os.path.join(CSRC, "*.h"))) + [
        os.path.normpath(os.path.join(HERE, "..", "include", "dvo.h")),
        os.path.normpath(os.path.join(HERE, "..", "data", "orb_bit_pattern_31.inc"))]


def source_hash(defines=()) -> str:
    """Build id: sha256 over the source texts, the compiler flags and the
    defines (16 hex digits).  Compiled into the library (dvo_build_id) and
    checked when it is loaded, so a library built from other sources is
    rebuilt here and refused on the GPU box, whatever the file times say."""
    import hashlib
    h = hashlib.sha256()
    for path in inputs():
        h.update(os.path.relpath(path, os.path.dirname(HERE)).encode() + b"\0")
        with open(path, "rb") as f:
            h.update(f.read() + b"\0")
    h.update(repr((CXXFLAGS, sorted(FILE_FLAGS.items()), ARCH, list(defines))).encode())
    return h.hexdigest()[:16]


def library_build_id(lib=LIB):
    """dvo_build_id() of a built library, read from its bytes (no load)."""
    try:
        data = open(lib, "rb").read()
    except OSError:
        return None
    i = data.find(b"DVO_BUILD_ID=")
    return data[i + 13:i + 29].decode() if i >= 0 else None


def _stale(lib, want):
    return library_build_id(lib) != want


def build(force: bool = False, verbose: bool = False, out: str = LIB, defines=()) -> str:
    """Compile and link libdvo_hip.so.  `out`/`defines` build an experiment
    variant beside it (tools/: A/B timing through DVO_LIB_PATH); the product
    library is always the default build."""
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    LIB = out
    objdir = os.path.join(os.path.dirname(out), "obj" if out == globals()["LIB"] else "obj_" + os.path.basename(out))
    os.makedirs(objdir, exist_ok=True)
    srcs = sources()
    objs = [os.path.join(objdir, os.path.basename(s) + ".o") for s in srcs]
    bid = source_hash(defines)
    if not force and not _stale(LIB, bid):
        return LIB

    def compile_one(pair):
        src, obj = pair
        lang = ["-x", "hip"]
        extra = [t for d in defines for t in (d.split() if d.startswith("-") else [f"-D{d}"])]  # raw flags pass through
        cmd = [hipcc, *lang, *CXXFLAGS, *FILE_FLAGS.get(os.path.basename(src), []), *extra,
               f'-DDVO_BUILD_ID="{bid}"', "-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
        return r.stderr

    with ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        for warn in ex.map(compile_one, zip(srcs, objs)):
            if warn and verbose:
                print(warn)
    tl = _torch_lib_dir()
    link = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", LIB + ".tmp", *objs]
    if tl:
        # resolve -lamdhip64 to torch's soname-less copy first -> NEEDED libamdhip64.so
        link = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", LIB + ".tmp", *objs,
                f"-L{tl}", f"-Wl,-rpath,{tl}", "-Wl,-rpath,/opt/rocm/lib"]
    r = subprocess.run(link, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose="-v" in sys.argv))
