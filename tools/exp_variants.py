"""Build timing variants of libnrt_hip.so into build_var/ (one box session then times them all).

A variant is NAME=FLAGS, e.g.  d3=-DNRT_RING_DEPTH=3  c32=-DNRT_RAY_CHUNK=32.  Only the SDF
translation units are recompiled (VARIED=a.hip,b.hip to choose others); the others come from the
normal build.  Usage:
    python tools/exp_variants.py d3=-DNRT_RING_DEPTH=3 c32=-DNRT_RAY_CHUNK=32
then on the box:  bash tools/exp_run.sh e1 d3
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from neural_raytracing_amd import build as B  # noqa: E402

B.build(verbose=False)
out = os.path.join(ROOT, os.environ.get("VAR_DIR", "build_var"))
os.makedirs(out, exist_ok=True)
VARIED = os.environ.get("VARIED", "nrt_api_sdf.hip,nrt_ring_march.hip,nrt_ring_normal.hip").split(",")
others = [os.path.join(B.OBJDIR, os.path.splitext(s)[0] + ".o") for s in B.SOURCES
          if s not in VARIED]


def compile_one(job):
    name, flags, src = job
    obj = os.path.join(out, f"{os.path.splitext(src)[0]}_{name}.o")
    subprocess.run(["/opt/rocm/bin/hipcc", *B.FLAGS, *flags.split(), "-c",
                    os.path.join(B.CSRC, src), "-o", obj], check=True)
    return obj


variants = [a.split("=", 1) for a in sys.argv[1:]]
jobs = [(n, f, src) for n, f in variants for src in VARIED]
with ThreadPoolExecutor(8) as ex:
    objs = list(ex.map(compile_one, jobs))
for i, (name, _) in enumerate(variants):
    lib = os.path.join(out, f"libnrt_hip_{name}.so")
    mine = objs[i * len(VARIED):(i + 1) * len(VARIED)]
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", lib,
                    *mine, *others, "-L/opt/rocm/lib", "-lrocblas", "-Wl,-rpath,/opt/rocm/lib"],
                   check=True)
    print(lib)
