"""Timing of the colocate scene's test render with shadow rays (colocate.py test(..., w_isect=True):
Direct's emitter sample marched by intersect_test, sdfs.py:162-181) against the same render
without them, per precision; kernel times from the library's HIP-event profile."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
import neural_raytracing_amd as nra  # noqa: E402
import neural_raytracing_amd.pathtracer as pt  # noqa: E402
from neural_raytracing_amd import _lib  # noqa: E402

KERNELS = ["k_occlusion", "k_intersect", "k_march16", "k_march32", "k_march3", "k_refine3",
           "k_shade_direct"]


def main():
    size = int(sys.argv[1]) if len(sys.argv) > 1 else 800
    precs = sys.argv[2].split(",") if len(sys.argv) > 2 else ["fp32", "mixed", "fp16"]
    dev = torch.device("cuda", 0)
    _lib.load(require_device=True)
    sc = bench.build_other_scene("colocate", dev, 64)
    for prec in precs:
        nra.set_precision(prec)
        for w in (False, True):
            def run():
                return pt.pathtrace(sc["shape"], sc["lights"], sc["cameras"], sc["integrator"],
                                    bsdf=sc["bsdf"], size=size, chunk_size=size // 4,
                                    bundle_size=1, with_noise=0.0, silent=True, w_isect=w)[0]
            with torch.no_grad():
                run()
                torch.cuda.synchronize()
                _lib.profile_reset()
                _lib.profile_enable(True)
                t0 = time.perf_counter()
                for _ in range(3):
                    run()
                torch.cuda.synchronize()
                el = (time.perf_counter() - t0) / 3
                _lib.profile_enable(False)
            ks = {k: _lib.profile_read(k)[0] / 3 for k in KERNELS}
            print(json.dumps({"precision": prec, "w_isect": w, "frame_ms": 1000 * el,
                              "kernel_ms": {k: v for k, v in ks.items() if v}}), flush=True)
    nra.set_precision("fp32")


if __name__ == "__main__":
    main()
