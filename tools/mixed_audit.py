"""NRT_MIXED flag audit (round-5 verdict item 5): on the headline frame (bench scene, 800^2),
how many rays the FP16 march flags for the split re-march, and how many of those the re-march
actually changes -- the FP16 frame's (hit, t) against the mixed frame's: every unflagged ray keeps
its FP16 march, so a ray whose (hit, t) differs between the two was flagged and re-marched to a
different result.  Also the FP32 frame's hit / step flips against both.  Per refine_d value
(units 1e-7, option mixed_refine_d; default 20000 = 2e-3): frame time, refined rays, changed
rays (hit or |dt| > 1e-4: a step flip; and |dt| > 1e-6: moved), pixels > 1e-4 vs FP32.
    python tools/mixed_audit.py [size] [refine_d,...]"""
import json
import math
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
import neural_raytracing_amd as nra  # noqa: E402
from neural_raytracing_amd import _lib  # noqa: E402
from neural_raytracing_amd.pathtracer.render import RowRenderer  # noqa: E402


def main():
    size = int(sys.argv[1]) if len(sys.argv) > 1 else 800
    ds = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [20000]
    dev = torch.device("cuda", 0)
    _lib.load(require_device=True)
    nra.set_precision("fp32")
    scene = bench.build_scene(dev, 64, light_gain=bench.LIGHT_GAIN)
    pt = scene["pt"]
    focal = float(0.5 * size / math.tan(0.5 * 0.6911))
    cams = pt.cameras.NeRFCamera(cam_to_world=bench.view_c2w(0, 1)[None].to(dev), focal=focal,
                                 device=dev)
    rr = RowRenderer(scene["shape"], scene["lights"], cams, scene["integrator"], scene["bsdf"],
                     size, range(size), background=0.0, with_noise=1e-3, device=dev)
    with torch.no_grad():
        want, rhit, rt = bench._frame_state(rr, 1234)
        nra.set_precision("fp16")
        f16, h16, t16 = bench._frame_state(rr, 1234)
        for d in ds:
            _lib.set_option("mixed_refine_d", d)
            nra.set_precision("mixed")
            el, ks, _ = bench._time_frames(rr.render, 3, 1, ["k_march16", "k_refine3", "k_best3"])
            _lib.profile_reset()
            _lib.profile_enable(False, evals=True)
            got, hm, tm = bench._frame_state(rr, 1234)
            torch.cuda.synchronize()
            refined = _lib.profile_refined()
            _lib.profile_enable(False)
            nra.set_precision("fp32")
            hit_ch = (hm != h16)
            both = hm & h16
            dt = (tm - t16).abs()
            step_ch = both & (dt > 1e-4)
            moved = both & (dt > 1e-6)
            acc = bench.frame_accuracy(got.cpu(), want.cpu(), hm.cpu(), rhit.cpu(), tm.cpu(),
                                       rt.cpu())
            acc16 = bench.frame_accuracy(f16.cpu(), want.cpu(), h16.cpu(), rhit.cpu(), t16.cpu(),
                                         rt.cpu())
            rays = size * size
            rec = {"refine_d": d * 1e-7, "frame_ms": 1000 * el / 3,
                   **{k + "_ms": v[0] / max(v[1], 1) for k, v in ks.items()},
                   "rays": rays, "refined": refined, "refined_frac": refined / rays,
                   "changed_hit": int(hit_ch.sum()), "changed_step": int(step_ch.sum()),
                   "moved_1e-6": int(moved.sum()),
                   "changed_frac_of_refined": (int(hit_ch.sum()) + int(step_ch.sum())) / max(refined, 1),
                   "moved_frac_of_refined": (int(hit_ch.sum()) + int(moved.sum())) / max(refined, 1),
                   "mixed_vs_fp32": {k: acc[k] for k in ("hit_flips", "step_flips",
                                                         "pixels_over_1e-4", "maxabs_agreeing")},
                   "fp16_vs_fp32": {k: acc16[k] for k in ("hit_flips", "step_flips",
                                                          "pixels_over_1e-4")}}
            print(json.dumps(rec), flush=True)
    _lib.set_option("mixed_refine_d", 20000)


if __name__ == "__main__":
    main()
