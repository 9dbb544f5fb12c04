"""Where the FP16 frame's error comes from: the headline frame (bench.py scene, 800^2, NeRFCamera)
rendered FP32, then with the intersect (march + scan + normals) and the shading at separate
precisions, each compared with the FP32 frame over the whole frame (bench.frame_accuracy)."""
import json
import math
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from neural_raytracing_amd import _lib  # noqa: E402
from neural_raytracing_amd.pathtracer import render as R  # noqa: E402


class _Prec:
    """render._lib stand-in: direct_kernels reads precision_code() once for the intersect, then
    once for the shading; answer each from the (intersect, shade) pair."""

    def __init__(self, pair):
        self.pair, self.k = pair, 0

    def __getattr__(self, name):
        return getattr(_lib, name)

    def precision_code(self):
        code = _lib._PRECISIONS[self.pair[self.k % 2]]
        self.k += 1
        return code


def main():
    size = int(sys.argv[1]) if len(sys.argv) > 1 else 800
    dev = torch.device("cuda", 0)
    _lib.load(require_device=True)
    _lib.set_precision("fp32")
    scene = bench.build_scene(dev, 64, light_gain=bench.LIGHT_GAIN)
    pt = scene["pt"]
    focal = float(0.5 * size / math.tan(0.5 * 0.6911))
    cams = pt.cameras.NeRFCamera(cam_to_world=bench.view_c2w(0, 1)[None].to(dev), focal=focal,
                                 device=dev)
    rows = list(range(size))
    rr = R.RowRenderer(scene["shape"], scene["lights"], cams, scene["integrator"], scene["bsdf"],
                       size, rows, background=0.0, with_noise=1e-3, device=dev)
    real = R._lib
    out = {}
    with torch.no_grad():
        want, rhit, rt = bench._frame_state(rr, 1234)
        rthr = next(iter(R._BUFS.values())).thr.clone()
        for pair in (("fp16", "fp16"), ("fp16", "fp32"), ("fp32", "fp16"),
                     ("fp32-split", "fp32"), ("fp16", "fp32-split"), ("mixed", "mixed")):
            R._lib = _Prec(pair)
            try:
                got, hit, t = bench._frame_state(rr, 1234)
                thr = next(iter(R._BUFS.values())).thr.clone()
            finally:
                R._lib = real
            acc = bench.frame_accuracy(got.cpu(), want.cpu(), hit.cpu(), rhit.cpu(), t.cpu(),
                                       rt.cpu())
            d = (thr - rthr).abs()
            acc["throughput_maxabs"] = float(d.max())
            acc["throughput_over_1e-3"] = int((d > 1e-3).sum())
            acc["t_maxabs_hits"] = float((t - rt).abs()[hit & rhit].max())
            key = f"intersect={pair[0]},shade={pair[1]}"
            out[key] = acc
            print(key, json.dumps(acc), flush=True)
        # the FP16 SDF error itself, on the points a march / scan visits: camera-ray points at
        # t in [0, 2.3], and the FP32 march's stop points
        from neural_raytracing_amd.pathtracer.shapes.sdfs import sdf_eval
        rays = cams.rays_tile(0, 0, size, size, size, 0.0, positions=rr.positions).reshape(-1, 6)
        g = torch.Generator(device=dev).manual_seed(0)
        sel = torch.randint(0, rays.shape[0], (1 << 20,), device=dev, generator=g)
        ts = torch.rand(1 << 20, 1, device=dev, generator=g) * 2.3
        pts = rays[sel, :3] + ts * rays[sel, 3:]
        stop = rays[:, :3] + rt.reshape(-1, 1).to(dev) * rays[:, 3:]
        sdf = scene["shape"].sdf
        for name, q in (("scan_points", pts), ("fp32_stop_points", stop[rhit.reshape(-1).to(dev)])):
            vals = {}
            for prec in ("fp32", "fp16", "fp32-split"):
                _lib.set_precision(prec)
                vals[prec] = sdf_eval(sdf, q.contiguous()).double()
            _lib.set_precision("fp32")
            for prec in ("fp16", "fp32-split"):
                e = (vals[prec] - vals["fp32"]).abs()
                qs = torch.quantile(e[: 1 << 20].float(), torch.tensor(
                    [0.5, 0.9, 0.99, 0.999, 0.9999], device=dev)).tolist()
                rec = {"points": int(e.numel()), "max": float(e.max()), "q50_90_99_999_9999": qs}
                out[f"sdf_err[{name},{prec}]"] = rec
                print(name, prec, json.dumps(rec), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
