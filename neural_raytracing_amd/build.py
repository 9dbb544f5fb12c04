"""Build libnrt_hip.so in-tree with hipcc for gfx950 (no JIT cache, no CMake)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libnrt_hip.so")
SOURCES = ["nrt_common.hip", "nrt_pack.hip", "nrt_api_mlp.hip", "nrt_api_sdf.hip",
           "nrt_api_shade.hip", "nrt_api_cam.hip", "nrt_ring_march.hip", "nrt_ring_march32.hip", "nrt_ring_march3.hip", "nrt_ring_mixed.hip", "nrt_ring_normal.hip", "nrt_prog.hip", "nrt_shade_ring.hip", "nrt_ring_normal32.hip", "nrt_callable.hip", "nrt_api_nerf.hip",
           "nrt_api_path.hip", "nrt_api_train.hip", "nrt_refresh.hip", "nrt_sphere.hip", "nrt_sphere_smoothmin.hip", "nrt_api_tile.hip"]
HEADERS = ["nrt_kernels.h", "nrt_device.h", "nrt_internal.h", "nrt_launch.h", "nrt_ring3.h",
           "nrt_shade_ring.h", "nrt_train_ring.h"]
HEADER = os.path.join(os.path.dirname(HERE), "include", "nrt.h")

# -ffp-contract=off: elementwise math rounds like the reference's eager torch ops (no silent FMA
# contraction); MFMA and explicit fmaf() are unaffected.
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++20", "-fPIC", "-ffp-contract=off",
         "-fno-slp-vectorize", "-Wno-unused-result"]
OBJDIR = os.path.join(HERE, "build_obj")


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _obj(src):
    return os.path.join(OBJDIR, os.path.splitext(src)[0] + ".o")


def needs_build():
    """Any object older than its source or a header (an edit made while a build ran leaves the
    .so newer than the edit but its object stale), or the .so older than an object."""
    hdrs = [os.path.join(CSRC, h) for h in HEADERS] + [HEADER]
    if any(_stale(_obj(s), [os.path.join(CSRC, s)] + hdrs) for s in SOURCES):
        return True
    return _stale(OUT, [_obj(s) for s in SOURCES])


def build(force=False, verbose=True, jobs=None):
    """Compile every translation unit in parallel (one hipcc per TU), then link the .so."""
    if not force and not needs_build():
        return OUT
    from concurrent.futures import ThreadPoolExecutor
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    os.makedirs(OBJDIR, exist_ok=True)
    hdrs = [os.path.join(CSRC, h) for h in HEADERS] + [HEADER]

    def compile_one(src):
        obj = _obj(src)
        path = os.path.join(CSRC, src)
        if force or _stale(obj, [path] + hdrs):
            cmd = [hipcc, *FLAGS, "-c", path, "-o", obj]
            if verbose:
                print("[nrt build]", " ".join(cmd), flush=True)
            subprocess.run(cmd, check=True, cwd=CSRC)
        return obj

    jobs = jobs or min(len(SOURCES), os.cpu_count() or 4, 8)
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    cmd = [hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", OUT + ".tmp", *objs]
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
