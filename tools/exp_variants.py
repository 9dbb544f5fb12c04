"""Build timing-only variants of libnrt_hip.so (NRT_EXP bits, nrt_device.h) into build_var/.

Only the SDF translation units are recompiled; the others come from the normal build.  Variants
compute wrong results on purpose (no barrier, no activation, ...) and exist to price one
component of the march kernel: never ship or test them.  Usage:
    python tools/exp_variants.py 8 9 10 12 24
then on the box:  NRT_LIB=build_var/libnrt_hip_e9.so python bench.py ...
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from neural_raytracing_amd import build as B  # noqa: E402

B.build(verbose=False)
out = os.path.join(ROOT, "build_var")
os.makedirs(out, exist_ok=True)
VARIED = ["nrt_api_sdf.hip", "nrt_ring_march.hip", "nrt_ring_normal.hip"]
others = [os.path.join(B.OBJDIR, os.path.splitext(s)[0] + ".o") for s in B.SOURCES
          if s not in VARIED]


def one(v):
    objs = []
    for src in VARIED:
        obj = os.path.join(out, f"{os.path.splitext(src)[0]}_e{v}.o")
        subprocess.run(["/opt/rocm/bin/hipcc", *B.FLAGS, f"-DNRT_EXP={v}", "-c",
                        os.path.join(B.CSRC, src), "-o", obj], check=True)
        objs.append(obj)
    lib = os.path.join(out, f"libnrt_hip_e{v}.so")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", lib,
                    *objs, *others], check=True)
    return lib


with ThreadPoolExecutor(4) as ex:
    for lib in ex.map(one, [int(a) for a in sys.argv[1:]]):
        print(lib)
