"""Development probe: per-phase shader cycles of the RANSAC kernel (block 0).

Builds a -DDVO_PROBE copy of the library into tools/probe_build/, runs one
bench-sized batch and prints the cycle split.  Not part of the product."""
import ctypes
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tools", "probe_build")


def build():
    from droplet_visual_odometry_amd import build as B
    os.makedirs(OUT, exist_ok=True)
    objs = []
    for src in B.sources():
        obj = os.path.join(OUT, os.path.basename(src) + ".o")
        lang = ["-x", "hip"] if src.endswith(".hip") else []
        subprocess.run(["hipcc", *lang, *B.CXXFLAGS, "-DDVO_PROBE", "-c", src, "-o", obj], check=True)
        objs.append(obj)
    lib = os.path.join(OUT, "libdvo_hip.so")
    import torch
    tl = os.path.join(os.path.dirname(torch.__file__), "lib")
    subprocess.run(["hipcc", "-shared", "-fPIC", f"--offload-arch={B.ARCH}", *objs, "-o", lib, f"-L{tl}",
                    f"-Wl,-rpath,{tl}:/opt/rocm/lib", "-lamdhip64"], check=True)
    return lib


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        print(build())
        return
    import torch
    from droplet_visual_odometry_amd import _native
    lib = _native.load_library(os.path.join(OUT, "libdvo_hip.so"))
    lib.dvo_debug_probe.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    from droplet_visual_odometry_amd.stream import FrameStream
    from droplet_visual_odometry_amd.synth import SceneStream
    W, H, B = 1280, 720, int(os.environ.get("B", "128"))
    sc = SceneStream(W, H, device="cuda")
    pool = torch.stack([sc.render(i) for i in range(B + 1)]).contiguous()
    fs = FrameStream(W, H, sc.K, nfeatures=2000, max_frames=B + 1)
    rec = fs.new_records(B)
    fs.process(pool, rec)
    fs.sync()
    buf = (ctypes.c_ulonglong * 32)()
    lib.dvo_debug_probe(buf, 32, 1)
    t0 = time.perf_counter()
    fs.process(pool, rec)
    fs.sync()
    dt = time.perf_counter() - t0
    lib.dvo_debug_probe(buf, 32, 1)
    r = FrameStream.records_numpy(rec, B)
    names = {0: "sample", 1: "solve", 2: "score", 3: "replay", 10: "fp_setup", 11: "fp_svd9", 12: "fp_coeff",
             13: "fp_lu", 14: "fp_bpoly", 15: "fp_roots", 16: "fp_backsub"}
    print(f"batch wall {dt * 1e3:.2f} ms; pair0 iters {r['ransac_iters'][0]} rounds {buf[4]}")
    for k, n in names.items():
        print(f"  {n:12s} {buf[k]:>14d} cycles")


if __name__ == "__main__":
    main()
