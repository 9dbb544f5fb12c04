"""NRT_MIXED threshold sweep on the headline frame (bench.py scene, 800^2): for each
mixed_refine_d / mixed_refine_s, the frame's accuracy against the FP32 frame (bench.frame_accuracy)
and the time of the frame, of k_march16, of the refinement march (k_refine3) and of sdf(best)
(k_best3)."""
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
    ds = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1200]
    ss = [int(v) for v in sys.argv[3].split(",")] if len(sys.argv) > 3 else [2000]
    rs = [int(v) for v in sys.argv[4].split(",")] if len(sys.argv) > 4 else [1]
    ms = [int(v) for v in sys.argv[5].split(",")] if len(sys.argv) > 5 else [0]
    zs = [int(v) for v in sys.argv[6].split(",")] if len(sys.argv) > 6 else [500000]
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
        for d, s, r, mdl, z in [(d, s, r, mdl, z) for z in zs for mdl in ms for r in rs
                                for d in ds for s in ss]:
            if True:
                _lib.set_option("mixed_zone", z)
                _lib.set_option("mixed_drift", mdl)
                _lib.set_option("mixed_restart", r)
                _lib.set_option("mixed_refine_d", d)
                _lib.set_option("mixed_refine_s", s)
                nra.set_precision("mixed")
                el, ks, evals = bench._time_frames(rr.render, 3, 1,
                                                   ["k_march16", "k_refine3", "k_best3"])
                got, hit, t = bench._frame_state(rr, 1234)
                nra.set_precision("fp32")
                acc = bench.frame_accuracy(got.cpu(), want.cpu(), hit.cpu(), rhit.cpu(), t.cpu(),
                                           rt.cpu())
                both = (hit & rhit).reshape(-1)
                dt = (t - rt).abs().reshape(-1)[both]
                rec = {"refine_d": d, "refine_s": s, "restart": r, "drift_model": mdl, "zone": z, "frame_ms": 1000 * el / 3,
                       **{k + "_ms": v[0] / max(v[1], 1) for k, v in ks.items()},
                       "evals": evals, "dt_q": torch.quantile(dt.float()[: 1 << 20], torch.tensor(
                           [0.5, 0.9, 0.99, 0.999], device=dt.device)).tolist(), **acc}
                print(json.dumps(rec), flush=True)
    _lib.reset_options() if hasattr(_lib, "reset_options") else None


if __name__ == "__main__":
    main()
