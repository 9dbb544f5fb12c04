#!/usr/bin/env python
"""bench.py -- ray-samples/s of the MI355X ray-march render path (BASELINE.json metric).

One step = one frame batch: N views (N = number of ranks) of an 800x800 NeRF-camera render of a
learned SDF with the nerf_synthetic shading stack, rows dealt round-robin to the ranks in 10-row
tiles (each rank renders 800x800 rays per step: weak scaling), then one RCCL all-gather of the
row slabs at the end of the step.  Per frame the reference work is W*H*(S + 130) SDF-MLP
evaluations (S = 64 march steps, 130 = coarse scan, sdfs.py:119-131, 232-249) plus shading on the
hit rays; the headline unit is the metric's ray-sample = W*H*S per frame.

Scene (synthetic, seeded): SphereSDF-style prior (one sphere r=0.25) + an 8x256
SkipConnMLP shift (F=16, sigma=32, softplus, default torch init, output layer x0.1) -- the metric's
"8x256 MLP", evaluated at every sample; ComposeSpatialVarying([NeuralBSDF(Softplus)] x 8) with its
16x256 spatial MLP; LightField (10x256); NeRFIntegrator(Direct()).
"""
import argparse
import json
import math
import os
import random
import sys
import time

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FLOP_SDF_8x256 = 1_120_864  # per evaluation (F=16, in 3, out 1)
SCAN_EVALS = 130             # sdf(o) + 128 samples + sdf(best)
# k_march16 evaluates the march and the 129 scan points; sdf(best) is k_scan_best16's
MARCH_KERNEL_SCAN_EVALS = 129
PEAK_TFLOPS = {"fp16": 2500.0, "fp32": 157.3}  # MI355X dense MFMA (MI355X_MICROARCH.md)
PEAK_TFLOPS["fp32-split"] = PEAK_TFLOPS["fp16"]  # its MFMA work runs on the FP16 matrix cores
PEAK_TFLOPS["mixed"] = PEAK_TFLOPS["fp16"]  # the FP16 march (+ split refinement, also FP16 MFMA)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--size", type=int, default=None,
                    help="image side (default 800; 1600 for --scene nerfle, BASELINE cfg5)")
    ap.add_argument("--samples", type=int, default=None,
                    help="march steps per ray (max_steps) or NeRF depths per ray "
                         "(default 64; 256 for --scene nerfle, BASELINE cfg5)")
    ap.add_argument("--precision", default="fp32", choices=["fp16", "fp32", "fp32-split", "mixed"],
                    help="arithmetic of the headline frame (default fp32, the reference's; the "
                         "fp16 frame is reported as the `fp16` leg)")
    ap.add_argument("--tile-rows", type=int, default=10)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-crop", type=int, default=128, help="side of the CPU-baseline crop")
    ap.add_argument("--no-fp32-check", action="store_true", help="no-op (kept for tools/)")
    ap.add_argument("--no-extra-legs", action="store_true",
                    help="skip the FP32 (reference precision) and scan-free timing legs")
    ap.add_argument("--scene", default="nerf_synthetic",
                    choices=["nerf_synthetic", "colocate", "dtu", "nerfle", "train", "path"],
                    help="nerf_synthetic = the BASELINE metric (default); the others are "
                         "BASELINE.json configs[2..4] as one-GPU workloads")
    ap.add_argument("--views", type=int, default=6, help="--scene train: views per step (N)")
    ap.add_argument("--crop", type=int, default=80, help="--scene train: crop side")
    ap.add_argument("--envmap", action="store_true",
                    help="--scene nerfle: NeRF+LE (NeRFLE(envmap=True), the light's envmap as the "
                         "colour MLP's input, nerf.py:183-191) instead of NeRF+PT")
    ap.add_argument("--nrt-option", action="append", default=[], metavar="NAME=VALUE",
                    help="nrt_set_option before the run (include/nrt.h runtime options), e.g. "
                         "xcd_lines=0 for an A/B of a schedule switch; repeatable")
    ap.add_argument("--torch-profile", default=None,
                    help="--scene train: write a torch.profiler op table of one step here")
    args = ap.parse_args()
    if args.nrt_option:
        from neural_raytracing_amd import _lib
        for kv in args.nrt_option:
            k, _, v = kv.partition("=")
            _lib.set_option(k, int(v))
    import sys
    args.precision_set = any(a.startswith("--precision") for a in sys.argv[1:])
    if args.scene == "train":
        if args.size is None:
            args.size = 256
        if args.samples is None:
            args.samples = 64
        return args
    if args.scene == "path":
        if args.size is None:
            args.size = 200  # path_nerv.py:27 SIZE
        if args.samples is None:
            args.samples = 64  # path_nerv.py:48 max_steps
        return args
    big = args.scene == "nerfle"
    if args.size is None:
        args.size = 1600 if big else 800
    if args.samples is None:
        args.samples = 256 if big else 64
    return args


def look_at(eye):
    eye = torch.tensor(eye, dtype=torch.float)
    fwd = F.normalize(-eye, dim=0)
    right = F.normalize(torch.cross(fwd, torch.tensor([0.0, 1.0, 0.0]), dim=0), dim=0)
    up = torch.cross(right, fwd, dim=0)
    c2w = torch.zeros(3, 4)
    c2w[:, 0], c2w[:, 1], c2w[:, 2], c2w[:, 3] = right, up, -fwd, eye
    return c2w


def view_c2w(i, n):
    a = 2 * math.pi * i / max(n, 1) + 0.3
    return look_at((math.sin(a) * math.cos(0.4), math.sin(0.4), math.cos(a) * math.cos(0.4)))


def build_scene(device, samples, seed=0, light_gain=1.0):
    """Product objects of the bench scene (identical on every rank).  light_gain scales the
    LightField MLP's output layer, i.e. the light magnitude |v| (lights.py:191-194): the bench
    frame uses 10 so its RGB spans most of [0, 1] (at 1 it peaks near 0.09) and accuracy
    numbers are not flattered by a dark image; the work is unchanged."""
    import neural_raytracing_amd.pathtracer as pt
    from neural_raytracing_amd.pathtracer.bsdf import ComposeSpatialVarying, NeuralBSDF
    from neural_raytracing_amd.pathtracer.integrators import Direct, NeRFIntegrator
    from neural_raytracing_amd.pathtracer.lights import LightField
    from neural_raytracing_amd.pathtracer.neural_blocks import SkipConnMLP
    from neural_raytracing_amd.pathtracer.shapes import SDF, SphereSDF
    torch.manual_seed(seed)
    random.seed(seed)
    sphere = SphereSDF(n=1, device="cpu")
    with torch.no_grad():
        sphere.centers.zero_()
        sphere.radii.fill_(0.25)
    sphere.shift = SkipConnMLP(num_layers=8, hidden_size=256, in_size=3, out=1, freqs=16,
                               activation=F.softplus, device="cpu")
    with torch.no_grad():
        sphere.shift.out.weight.mul_(0.1)
        sphere.shift.out.bias.mul_(0.1)
    shape = SDF(sdf=sphere.to(device), device=device, max_steps=samples)
    bsdf = ComposeSpatialVarying([NeuralBSDF(activation=torch.nn.Softplus(), device="cpu")
                                  for _ in range(8)], device="cpu")
    for b in bsdf.bsdfs:
        b.mlp.to(device)
    bsdf.sp_var_fn.to(device)
    lights = LightField(device="cpu").to(device)
    if light_gain != 1.0:
        with torch.no_grad():
            lights.light_field_approx.out.weight.mul_(light_gain)
            lights.light_field_approx.out.bias.mul_(light_gain)
    return dict(shape=shape, bsdf=bsdf, lights=lights, integrator=NeRFIntegrator(Direct()),
                pt=pt)


def shape_mlp_sdf(mlp, radius=0.3, copies=40, scale=20.0, seed=0):
    """Give a randomly initialised SkipConnMLP(8, 256, in 3, out 1) a real zero level set.

    A default-initialised deep softplus MLP is constant to ~1e-3 over the unit ball (its output
    distribution collapses), so as an SDF every ray "hits" at t = 0.  This sets, in place:
      * init: 6*copies "carry" units u = +-a_c x_i (a_c = scale * [0.8, 1.2], one per copy);
      * every hidden layer: the carry units pass through exactly, t' = softplus(t) - softplus(-t)
        (weights +1 / -1 on the unit's pair, 0 on everything else incl. the skip encoding);
      * out: sum_c k_c (softplus(t) + softplus(-t)) over the carry pairs, k_c = 1 / (sqrt(3) a_c
        copies) x 0.99, plus the bias that puts the zero level set through (radius, 0, 0).  Since
        softplus(t) + softplus(-t) = |t| + 2 log(1 + e^-|t|), sdf(p) is a rounded octahedron,
        ~ (|x| + |y| + |z|) / sqrt(3) - const; every gradient component is at most 1 / sqrt(3),
        so the field is 1-Lipschitz and sphere tracing never oversteps.  The remaining
        256 - 6*copies units keep their random weights and feed the output through weights x 0.02.
    Works on the product SkipConnMLP and the oracle SkipMLP alike (same init / layers / out
    names); FLOPs and shapes are unchanged.  (A quadratic |p|^2 construction cancels a constant
    of 2 log 2 per unit pair and loses ~30x more to FP16 activations.)"""
    g = torch.Generator().manual_seed(seed)
    H = mlp.init.out_features
    nc = 6 * copies
    assert nc <= H and mlp.in_size == 3
    a = (scale * (0.8 + 0.4 * torch.rand(copies, generator=g, dtype=torch.float64))).tolist()

    def sp(x):
        return max(x, 0.0) + math.log1p(math.exp(-abs(x)))

    with torch.no_grad():
        W = mlp.init.weight
        W[:nc] = 0
        mlp.init.bias[:nc] = 0
        for c in range(copies):
            for i in range(3):
                W[6 * c + 2 * i, i] = a[c]
                W[6 * c + 2 * i + 1, i] = -a[c]
        for lin in mlp.layers:
            lin.weight[:nc] = 0
            lin.bias[:nc] = 0
            for u in range(0, nc, 2):
                lin.weight[u, u], lin.weight[u, u + 1] = 1.0, -1.0
                lin.weight[u + 1, u + 1], lin.weight[u + 1, u] = 1.0, -1.0
        mlp.out.weight.mul_(0.02)
        level = 0.0  # the carry part of sdf at (radius, 0, 0)
        for c in range(copies):
            k = 0.99 / (math.sqrt(3.0) * a[c] * copies)  # 1% headroom for the random units
            mlp.out.weight[0, 6 * c:6 * c + 6] = k
            level += k * (sp(a[c] * radius) + sp(-a[c] * radius) + 4 * math.log(2.0))
        mlp.out.bias[0] = mlp.out.bias[0] * 0.02 - level
    return mlp


def oracle_scene(scene):
    """The same weights in the CPU oracle (cpu_baseline leg only)."""
    from oracle import pathtracer_ref as R
    blob = R.SphereBlobSDF(n=1, shift_hidden=256, shift_freqs=16, shift_zero_init=False)
    src = scene["shape"].sdf
    with torch.no_grad():
        blob.centers.copy_(src.centers.cpu())
        blob.radii.copy_(src.radii.cpu())
        blob.tfs.copy_(src.tfs.cpu())
    _copy_to_oracle(blob.shift, src.shift)
    parts = [R.NeuralBSDFRef(activation="softplus") for _ in scene["bsdf"].bsdfs]
    for o, p in zip(parts, scene["bsdf"].bsdfs):
        _copy_to_oracle(o.mlp, p.mlp)
    bsdf = R.SpatialMixBSDF(parts)
    _copy_to_oracle(bsdf.sp_var_fn, scene["bsdf"].sp_var_fn)
    lights = R.LightFieldRef()
    _copy_to_oracle(lights.light_field_approx, scene["lights"].light_field_approx)
    shape = R.MarchedSDF(sdf=blob, max_steps=scene["shape"].max_steps)
    return dict(shape=shape, bsdf=bsdf, lights=lights,
                integrator=R.NeRFIntegratorRef(R.DirectRef()))


def _copy_to_oracle(dst, src):
    with torch.no_grad():
        dst.basis_p = src.basis_p.detach().cpu().clone()
        for a, b in zip([dst.init, *dst.layers, dst.out], src._linears()):
            a.weight.copy_(b.weight.cpu())
            a.bias.copy_(b.bias.cpu())


LIGHT_GAIN = 10.0  # bench frame light magnitude x10: RGB spans most of [0, 1] (build_scene)


def main():
    args = parse()
    if args.scene == "train":
        return bench_train(args)
    if args.scene == "path":
        return bench_path(args)
    if args.scene != "nerf_synthetic":
        return bench_other(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # a torch.distributed.run launch takes the process-group path even at one rank (so the RCCL
    # broadcast / all-gather / all-reduce run on a one-GPU box too)
    dist_on = world > 1 or "TORCHELASTIC_RUN_ID" in os.environ
    if dist_on:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    import neural_raytracing_amd as nra
    from neural_raytracing_amd import _lib
    from neural_raytracing_amd.pathtracer.render import RowRenderer, row_shard
    _lib.load(require_device=True)
    nra.set_precision(args.precision)

    size = args.size
    scene = build_scene(device, args.samples, light_gain=LIGHT_GAIN)
    if dist_on:
        # every rank built the scene from the same seed; broadcasting rank 0's tensors makes the
        # replication explicit (a model loaded from file on rank 0 is replicated the same way)
        from neural_raytracing_amd.pathtracer.render import broadcast_module
        for key in ("shape", "bsdf", "lights"):
            broadcast_module(scene[key])
    pt = scene["pt"]
    focal = float(0.5 * size / math.tan(0.5 * 0.6911))
    c2w = torch.stack([view_c2w(i, world) for i in range(world)]).to(device)
    cameras = pt.cameras.NeRFCamera(cam_to_world=c2w, focal=focal, device=device)
    rows = row_shard(size, rank, world, args.tile_rows)
    rr = RowRenderer(scene["shape"], scene["lights"], cameras, scene["integrator"], scene["bsdf"],
                     size, rows, background=0.0, with_noise=1e-3, device=device)
    step = make_step(rr.render, rows, size, rank, world, args.tile_rows, device, gather=dist_on)

    with torch.no_grad():
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        if dist_on:
            torch.distributed.barrier()
        _lib.profile_reset()
        _lib.profile_enable(True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        if dist_on:
            torch.distributed.barrier()
        elapsed = time.perf_counter() - t0
        _lib.profile_enable(False)
        march_kernel = MARCH_KERNEL[args.precision]
        k_ms, k_n = _lib.profile_read(march_kernel)
        i_ms, i_n = _lib.profile_read("k_intersect")
        evals = count_evals(step)
        elapsed = max_over_ranks(elapsed, world, device, force=dist_on)

    ms_step = 1000 * elapsed / args.steps
    rays_per_rank = len(rows) * size * world  # this rank's rows of every view
    rays_total = world * size * size * args.steps
    value = rays_total * args.samples / elapsed
    roof = march_roofline(march_kernel, "fp16" if args.precision == "mixed" else args.precision,
                          rays_per_rank, args.samples, k_ms, k_n, evals, size)
    roof["intersect_ms"] = i_ms / max(i_n, 1)

    extra = {}
    if rank == 0 and world == 1:
        with torch.no_grad():
            hit_frac = float(rr_hit_fraction(rr))
        extra["hit_fraction"] = round(hit_frac, 4)
        if not args.no_extra_legs:
            if args.precision == "fp32":
                extra["fp32_split"] = split_leg(rr, args, rows, size)
                extra["fp16"] = fp16_leg(rr, args, rows, size)
                extra["mixed"] = fp16_leg(rr, args, rows, size, precision="mixed")
            extra.update(extra_legs(scene, cameras, size, args, rows))
            extra["api_paths"] = api_path_legs(scene, args)
            # the training step (training_utils.py:246-285) at the reference's
            # arithmetic and with the mixed march, each with its backward roofline
            extra["train"] = {p: train_leg(p, 20, 3, cpu=(p == "fp32" and not args.no_cpu_baseline))
                              for p in ("fp32", "mixed")}
        if not args.no_cpu_baseline:
            extra.update(cpu_baseline(scene, size, args))

    if rank == 0:
        line = {
            "metric": "ray-samples/sec/GPU (800x800x64, 8x256 MLP); PSNR vs ref",
            "value": value,
            "unit": "ray-samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.precision,
            "data": "synthetic (seeded random-init weights, SphereSDF prior + 8x256 shift MLP)",
            "config": {
                "workload": f"{size}x{size} NeRFCamera frame per GPU, {args.samples} march steps + "
                            f"{SCAN_EVALS}-eval coarse scan per ray, SDF MLP 8x256 F16, "
                            "8x NeuralBSDF(6x96) + 16x256 spatial MLP + LightField(10x256, "
                            f"output x{LIGHT_GAIN:g}), NeRFIntegrator(Direct)",
                "image": [size, size],
                "samples_per_ray": args.samples,
                "views_per_step": world,
                "parallelism": f"row-tile shard x{world} ({args.tile_rows}-row tiles) + RCCL all-gather",
            },
            "roofline": roof,
            "sdf_evals_per_s": rays_total * (args.samples + SCAN_EVALS) / elapsed,
        }
        if "cpu_baseline" in extra:
            line["cpu_baseline"] = extra.pop("cpu_baseline")
        line.update(extra)
        print(json.dumps(line), flush=True)
    if dist_on:
        torch.distributed.destroy_process_group()


MARCH_KERNEL = {"fp16": "k_march16", "fp32": "k_march32", "fp32-split": "k_march3",
                "mixed": "k_march16"}


def march_roofline(kernel, precision, rays, samples, k_ms, k_n, evals, size):
    """Roofline object of one march + scan launch: algorithmic FLOP = every ray at every march
    step and scan point (the reference's count, sdfs.py:119-131, 232-249) x the 8x256 MLP's FLOP
    per evaluation, over the launch's HIP-event duration; `executed_*` counts the evaluations the
    job lists actually ran (device counter, one untimed frame) less the sdf(best) pass's.
    fp32-split: the kernel issues 3 f16 MFMA products per f32 product, so the MFMA work is 3x
    the algorithmic count, on the FP16 peak; fp32_equivalent_* is the algorithmic rate beside the
    FP32 peak."""
    split = precision == "fp32-split"
    products = 3 if split else 1
    flop_launch = rays * (samples + MARCH_KERNEL_SCAN_EVALS) * FLOP_SDF_8x256 * products
    avg_kernel_ms = k_ms / max(k_n, 1)
    achieved = flop_launch / (avg_kernel_ms * 1e-3) / 1e12
    peak = PEAK_TFLOPS[precision]
    exec_flop = (evals - rays) * FLOP_SDF_8x256 * products
    exec_achieved = exec_flop / (avg_kernel_ms * 1e-3) / 1e12
    traffic, source = None, None
    pmc_path = os.path.join(ROOT, "profiles", f"pmc_{kernel}.json")
    if os.path.exists(pmc_path):
        try:
            pm = json.load(open(pmc_path))
            if pm.get("size") == size and pm.get("precision") == precision:
                traffic = pm.get("hbm_bytes_per_launch")
                source = (f"committed PMC pass, profiles/pmc_{kernel}.json (FETCH_SIZE + "
                          f"WRITE_SIZE, {size}^2 {precision}); not measured in this run")
        except Exception:
            traffic = None
    out = {
        "bound": "mfma", "kernel": kernel, "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
        "frac": achieved / peak, "traffic": traffic, "traffic_source": source,
        "flop_per_launch": flop_launch,
        "flop_basis": "algorithmic: every ray at every march step and scan point "
                      "(sdfs.py:119-131, 232-249)",
        "executed_flop_per_launch": exec_flop, "executed_achieved": exec_achieved,
        "executed_frac": exec_achieved / peak, "avg_kernel_ms": avg_kernel_ms, "launches": k_n,
    }
    if split:
        out["flop_basis"] = ("MFMA work issued: 3 f16 products per f32 product (hi*hi, hi*lo, "
                             "lo*hi) x the algorithmic count (every ray at every march step and "
                             "scan point, sdfs.py:119-131, 232-249)")
        out["fp32_equivalent_achieved"] = achieved / 3
        out["fp32_equivalent_vs_fp32_peak"] = achieved / 3 / PEAK_TFLOPS["fp32"]
    return out


def _frame_state(rr, seed):
    """One render with fixed camera jitter / scan jitter draws; returns (image, hit, t) copies."""
    from neural_raytracing_amd.pathtracer import render as R
    torch.manual_seed(seed)
    random.seed(seed)
    img = rr.render().clone()
    b = next(iter(R._BUFS.values()))
    return img, b.hit.clone().bool(), b.t.clone()


def frame_accuracy(got, want, hit, rhit, t, rt):
    """Full-frame comparison of two renders of the same rays (RGBA [..., 4]): max |diff|, pixels
    with any channel off by more than 1e-4, hit flips, step flips (both hit, depth differs by
    more than 1e-4: one march stopped a step earlier on an SDF value within rounding of eps),
    RGB PSNR against the reference frame's own peak (mse2psnr with data range = the peak),
    and the alpha error."""
    err = (got - want).abs()
    px = err.amax(-1).reshape(-1)
    hit, rhit, t, rt = hit.reshape(-1), rhit.reshape(-1), t.reshape(-1), rt.reshape(-1)
    step = (hit & rhit) & ((t - rt).abs() > 1e-4)
    agree = (hit == rhit) & ~step
    peak = float(want[..., :3].max())
    mse = float(((got[..., :3] - want[..., :3]) ** 2).mean())
    return {
        "pixels": int(px.numel()), "hits": int(rhit.sum()),
        "maxabs": float(err.max()), "maxabs_rgb": float(err[..., :3].max()),
        "maxabs_alpha": float(err[..., 3].max()) if got.shape[-1] > 3 else None,
        "pixels_over_1e-4": int((px > 1e-4).sum()),
        "pixels_over_1e-3": int((px > 1e-3).sum()),
        "pixels_over_1e-2": int((px > 1e-2).sum()),
        "hit_flips": int((hit != rhit).sum()), "step_flips": int(step.sum()),
        "maxabs_agreeing": float(px[agree].max()) if bool(agree.any()) else 0.0,
        "rgb_peak": peak, "rgb_min": float(want[..., :3].min()),
        "psnr_peak": (10 * math.log10(peak * peak / mse)) if mse > 0 else float("inf"),
    }


def fp16_leg(rr, args, rows, size, steps=5, warmup=2, precision="fp16"):
    """The same frame on the FP16 MFMA path (march k_march16 on the 2.5 PF FP16 peak; sdf(best)
    FP32, option scan_best32) -- or with precision "mixed" (include/nrt.h NRT_MIXED: the same
    FP16 march + scan, the undecidable steps re-taken on the split engine by k_refine3, sdf(best)
    over the top two by k_best3, split normals and shading) -- timed, and compared over the whole
    frame with the FP32 frame of the same rays and weights."""
    import neural_raytracing_amd as nra
    from neural_raytracing_amd import _lib
    names = ["k_march16", "k_intersect", "k_scan_best32", "k_refine3", "k_best3"]
    with torch.no_grad():
        want, rhit, rt = _frame_state(rr, 1234)
        nra.set_precision(precision)
        try:
            el, ks, evals = _time_frames(rr.render, steps, warmup, names)
            got, hit, t = _frame_state(rr, 1234)
        finally:
            nra.set_precision(args.precision)
    frame_rays = len(rows) * size
    roof = march_roofline("k_march16", "fp16", frame_rays, args.samples, *ks["k_march16"],
                          evals, size)
    roof["intersect_ms"] = ks["k_intersect"][0] / max(ks["k_intersect"][1], 1)
    for k in names[2:]:
        if ks[k][1]:
            roof[k + "_ms"] = ks[k][0] / ks[k][1]
    if precision == "mixed":
        # the evaluation count includes the split refinement's (k_refine3 / k_best3), so the
        # executed rate divides it by the time of all three kernels; each split evaluation is
        # priced at one product although it issues three, so this is a lower bound
        k_ms = sum(ks[k][0] for k in ("k_march16", "k_refine3", "k_best3")) / max(ks["k_march16"][1], 1)
        roof["executed_achieved"] = roof["executed_flop_per_launch"] / (k_ms * 1e-3) / 1e12
        roof["executed_frac"] = roof["executed_achieved"] / roof["peak"]
        roof["executed_ms_per_launch"] = k_ms
        roof["note"] = ("executed_*: every counted evaluation (the FP16 march's and the split "
                        "refinement's, each priced at one product) over the time of k_march16 + "
                        "k_refine3 + k_best3 -- a lower bound, as a split evaluation issues three "
                        "products; frac / achieved: the algorithmic count over k_march16 alone")
    return {"value": frame_rays * args.samples * steps / el, "unit": "ray-samples/s",
            "ms_per_step": 1000 * el / steps, "steps": steps, "dtype": precision,
            "roofline": roof,
            "vs_fp32_full_frame": frame_accuracy(got.cpu(), want.cpu(), hit.cpu(), rhit.cpu(),
                                                 t.cpu(), rt.cpu())}


def make_step(render, rows, size, rank, world, tile_rows, device, channels=4, gather=None):
    """One bench step's frame assembly: `render()` gives this rank's rows of every view
    ([world, len(rows), size, channels]); the step returns the full [world, size, size, channels]
    frames on every rank -- a RowGather all-gather (RCCL) under a process group (world > 1, or
    `gather` forced on), an index copy otherwise.  The buffers and index tensors are built here,
    once."""
    from neural_raytracing_amd.pathtracer.render import RowGather
    full = torch.zeros(world, size, size, channels, device=device)
    rows_idx = torch.tensor(rows, dtype=torch.long, device=device)
    if gather is None:
        gather = world > 1
    gather = RowGather(size, rank, world, tile_rows, (world, size, channels), device) if gather else None

    def step():
        img = render()
        if gather is not None:
            gather(img, full)
        else:
            full.index_copy_(1, rows_idx, img)
        return full
    return step


def max_over_ranks(elapsed, world, device, force=False):
    """The bench's time: the slowest rank's (all-reduce MAX), on every rank."""
    if world <= 1 and not force:
        return elapsed
    t = torch.tensor([elapsed], device=device, dtype=torch.float64)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return t.item()


def count_evals(render):
    """SDF evaluations the ring marches execute in one more, untimed render (the device counter
    is one atomic per wave-evaluation, so it stays out of the timed steps)."""
    from neural_raytracing_amd import _lib
    _lib.profile_reset()
    _lib.profile_enable(False, evals=True)
    render()
    torch.cuda.synchronize()
    evals = _lib.profile_evals()
    _lib.profile_enable(False)
    return evals


def _time_frames(render, steps, warmup, kernels):
    """Wall time of `steps` renders after `warmup`, the HIP-event time of each kernel, and the
    SDF evaluations of one render."""
    from neural_raytracing_amd import _lib
    for _ in range(warmup):
        render()
    torch.cuda.synchronize()
    _lib.profile_reset()
    _lib.profile_enable(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        render()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    _lib.profile_enable(False)
    times = {k: _lib.profile_read(k) for k in kernels}
    return elapsed, times, count_evals(render)


def split_leg(rr, args, rows, size, steps=5, warmup=2):
    """The same frame in the fp32-split precision (include/nrt.h NRT_FP32_SPLIT): the march +
    coarse scan on k_march3 -- every SDF layer on v_mfma_f32_16x16x32_f16 with f32 operands
    split into two f16 halves, three products per block, f32 accumulation -- everything else as
    FP32.  Roofline: the MFMA work the kernel issues (3 x the algorithmic FLOP) on the 2.5 PF
    FP16 peak; `fp32_equivalent_*` puts the algorithmic FLOP beside the 157.3 TF FP32 peak.
    Compared over the whole frame with the FP32 frame of the same rays and weights."""
    import neural_raytracing_amd as nra
    with torch.no_grad():
        want, rhit, rt = _frame_state(rr, 1234)
        nra.set_precision("fp32-split")
        try:
            el, ks, evals = _time_frames(rr.render, steps, warmup,
                                         ["k_march3", "k_intersect", "k_scan_best3"])
            got, hit, t = _frame_state(rr, 1234)
        finally:
            nra.set_precision(args.precision)
    frame_rays = len(rows) * size
    roof = march_roofline("k_march3", "fp32-split", frame_rays, args.samples, *ks["k_march3"],
                          evals, size)
    roof["intersect_ms"] = ks["k_intersect"][0] / max(ks["k_intersect"][1], 1)
    roof["scan_best_ms"] = ks["k_scan_best3"][0] / max(ks["k_scan_best3"][1], 1)
    return {"value": frame_rays * args.samples * steps / el, "unit": "ray-samples/s",
            "ms_per_step": 1000 * el / steps, "steps": steps,
            "dtype": "fp32-split (f32 operands as f16 hi + lo, 3 f16 MFMA products, f32 accumulate)",
            "roofline": roof,
            "vs_fp32_full_frame": frame_accuracy(got.cpu(), want.cpu(), hit.cpu(), rhit.cpu(),
                                                 t.cpu(), rt.cpu())}


def extra_legs(scene, cameras, size, args, rows):
    """The same frame at the reference's precision when the headline ran FP16 (FP32: every MLP
    on exact-f32 MFMA, the 1e-4 parity path), and without the 130-eval coarse scan (SURVEY §8d
    cfg2 asks for both)."""
    import neural_raytracing_amd as nra
    from neural_raytracing_amd.pathtracer.integrators import Direct, NeRFIntegrator
    from neural_raytracing_amd.pathtracer.render import RowRenderer
    out = {}
    S = args.samples
    frame_rays = len(rows) * size * len(cameras)
    dev = cameras.cam_to_world.device
    if args.precision != "fp32":
        nra.set_precision("fp32")
        rr = RowRenderer(scene["shape"], scene["lights"], cameras, scene["integrator"],
                         scene["bsdf"], size, rows, background=0.0, with_noise=1e-3, device=dev)
        steps = 2
        el, ks, evals = _time_frames(rr.render, steps, 1, ["k_march32", "k_intersect"])
        out["fp32"] = {"value": frame_rays * S * steps / el, "unit": "ray-samples/s",
                       "ms_per_step": 1000 * el / steps, "steps": steps,
                       "roofline": march_roofline("k_march32", "fp32", frame_rays, S,
                                                  *ks["k_march32"], evals, size)}
        nra.set_precision(args.precision)
    # scan-free leg: Direct with training = False (the reference's Path / primary=False march)
    kernel = MARCH_KERNEL[args.precision]
    direct = Direct()
    direct.training = False
    rr = RowRenderer(scene["shape"], scene["lights"], cameras, NeRFIntegrator(direct),
                     scene["bsdf"], size, rows, background=0.0, with_noise=1e-3, device=dev)
    steps = 3
    el, ks, evals = _time_frames(rr.render, steps, 1, [kernel])
    k_ms = ks[kernel][0] / max(ks[kernel][1], 1)
    products = 3 if args.precision == "fp32-split" else 1  # f16 MFMA products per f32 product
    flop = frame_rays * S * FLOP_SDF_8x256 * products
    ach = flop / (k_ms * 1e-3) / 1e12
    peak = PEAK_TFLOPS[args.precision]
    # without the scan a ray stops at its hit (or at max_t): the algorithmic count (every ray at
    # every step, as the reference evaluates) is far above what the job lists execute, so the
    # executed fraction is the utilisation figure here
    exe = evals * FLOP_SDF_8x256 * products / (k_ms * 1e-3) / 1e12
    out["scan_free"] = {"value": frame_rays * S * steps / el, "unit": "ray-samples/s",
                        "ms_per_step": 1000 * el / steps, "steps": steps, "dtype": args.precision,
                        "roofline": {"bound": "mfma", "kernel": kernel, "achieved": exe,
                                     "peak": peak, "unit": "TFLOP/s", "frac": exe / peak,
                                     "avg_kernel_ms": k_ms,
                                     "executed_evals_per_ray": evals / frame_rays,
                                     "reference_count_flop_per_launch": flop,
                                     "reference_count_rate": ach,
                                     "reference_count_over_peak": ach / peak,
                                     "note": "frac = the evaluations the march executed (rays stop "
                                             "at their hit or max_t) over the peak: the kernel's "
                                             "utilisation; reference_count_* prices every ray x "
                                             "all 64 steps, as the reference evaluates them, and "
                                             "can exceed 1 since most rays stop early"}}
    return out


def api_path_legs(scene, args, reps=3):
    """The render calls the drivers make, timed through the public API:
    test_nerf's pathtrace(size=256, chunk_size=256) (training_utils.py:323-329), test_dtu's
    pathtrace(size=256, chunk_size=128) (training_utils.py:458-464) and the training step's
    forward, pathtrace_sample of a 6-view 80x80 crop of 256^2 (training_utils.py:256-266,
    nerf_synthetic.py), under torch.no_grad (the render path; training's autograd path is
    --scene train).  Each: ray-samples/s over the wall time and the march kernel's time / frac."""
    import neural_raytracing_amd as nra
    from neural_raytracing_amd import _lib
    pt = scene["pt"]
    S = args.samples
    prec = args.precision
    kernel = MARCH_KERNEL[prec]
    size = 256
    focal = float(0.5 * size / math.tan(0.5 * 0.6911))
    dev = scene["shape"].device

    def cam(n):
        c2w = torch.stack([view_c2w(i, n) for i in range(n)]).to(dev)
        return pt.cameras.NeRFCamera(cam_to_world=c2w, focal=focal, device=dev)

    cases = [
        ("test_nerf pathtrace(size=256, chunk_size=256)", cam(1), 256 * 256,
         lambda c: pt.pathtrace(scene["shape"], scene["lights"], c, scene["integrator"],
                                bsdf=scene["bsdf"], size=size, chunk_size=256, bundle_size=1,
                                background=0, silent=True, device=dev)),
        ("test_dtu pathtrace(size=256, chunk_size=128)", cam(1), 256 * 256,
         lambda c: pt.pathtrace(scene["shape"], scene["lights"], c, scene["integrator"],
                                bsdf=scene["bsdf"], size=size, chunk_size=128, bundle_size=1,
                                background=0, silent=True, device=dev)),
        ("train_nerf pathtrace_sample(6 views, crop 80 of 256, chunk_size=256) forward", cam(6),
         6 * 80 * 80,
         lambda c: pt.pathtrace_sample(scene["shape"], scene["lights"], c, scene["integrator"],
                                       bsdf=scene["bsdf"], size=size, chunk_size=256,
                                       bundle_size=1, crop_size=80, uv=(88, 88), background=0,
                                       device=dev)),
    ]
    out = {}
    with torch.no_grad():
        for name, c, rays, fn in cases:
            el, ks, evals = _time_frames(lambda: fn(c), reps, 1, [kernel])
            k_ms, k_n = ks[kernel]
            flop = rays * (S + MARCH_KERNEL_SCAN_EVALS) * FLOP_SDF_8x256 * \
                (3 if prec == "fp32-split" else 1)
            out[name] = {"value": rays * S * reps / el, "unit": "ray-samples/s",
                         "ms_per_call": 1000 * el / reps, "rays": rays,
                         "kernel": kernel, "kernel_launches_per_call": k_n / reps,
                         "kernel_ms_per_call": k_ms / reps,
                         "frac": flop / (k_ms / reps * 1e-3) / 1e12 / PEAK_TFLOPS[prec],
                         "dtype": prec}
    return out


FLOP_SHIFT_8x128 = 331_200      # SphereSDF shift MLP per evaluation
FLOP_NERFLE_SAMPLE = 327_840    # NeRFLE first (5x128, out 65) + second (8x64, in 70)
# NeRF+LE: the colour MLP reads 64 latent + 3 + 4^2 x 3 envmap values (in 115): per sample
# 2 x (dp H + L H^2 + skips dp H + H out + in F) = 2 x 72,432 for it (dp = 115 + 2 x 16)
FLOP_NERFLE_ENVMAP_SAMPLE = 207_456 + 144_864


def build_other_scene(name, device, samples, envmap=False, views=1):
    """BASELINE.json configs[2..4] (synthetic, seeded random init): colocate (cfg3: FoV camera,
    SphereSDF(n=64) + 8x128 shift, 4-component BSDF, point light), dtu (cfg4: DTU pinhole, 8x256
    MLP SDF, 10 NeuralBSDF + 6 Diffuse, LightField), nerfle (cfg5: NeRFLE, NeRF+PT, `samples`
    depths per ray).  views: camera views of the batch (bench_other renders one view per rank,
    each rank its rows of every view, as the headline; view 0 is the one-GPU scene's)."""
    import neural_raytracing_amd.pathtracer as pt
    from neural_raytracing_amd.pathtracer.bsdf import (ComposeSpatialVarying, Conductor, Diffuse,
                                                        NeuralBSDF)
    from neural_raytracing_amd.pathtracer.integrators import Direct, NeRFIntegrator, NeRFReproduce
    from neural_raytracing_amd.pathtracer.lights import LightField, PointLights
    from neural_raytracing_amd.pathtracer.neural_blocks import SkipConnMLP
    from neural_raytracing_amd.pathtracer.shapes import SDF, NeRFLE, SphereSDF
    torch.manual_seed(0)
    random.seed(0)
    if name == "colocate":
        sphere = SphereSDF(n=64, device="cpu")
        sphere.shift = SkipConnMLP(num_layers=8, hidden_size=128, in_size=3, out=1, freqs=32,
                                   activation=F.softplus, device="cpu")
        with torch.no_grad():
            sphere.shift.out.weight.mul_(0.1)
            sphere.shift.out.bias.mul_(0.1)
        comps = [NeuralBSDF(device="cpu"), NeuralBSDF(device="cpu"),
                 Diffuse(preprocess=torch.nn.Softplus(), device="cpu").random(),
                 Conductor(activation=torch.nn.Softplus(), device="cpu").random()]
        bsdf = ComposeSpatialVarying(comps, device="cpu")
        for c in comps[:2]:
            c.mlp.to(device)
        bsdf.sp_var_fn.to(device)
        R, T = pt.cameras.look_at_view_transform(
            dist=1.0, elev=30.0, azim=[45.0 + 360.0 * i / views for i in range(views)])
        cam = pt.cameras.OpenGLPerspectiveCameras(R=R, T=T, device=device)
        lights = PointLights(location=(cam.get_camera_center()[0] * 1.05).tolist(), scale=5.0,
                             device=device)
        return dict(kind="march", shape=SDF(sdf=sphere.to(device), max_steps=samples), bsdf=bsdf,
                    lights=lights, integrator=Direct(), cameras=cam, flop_eval=FLOP_SHIFT_8x128,
                    workload="colocate.py-like: OpenGLPerspectiveCameras(look_at dist 1, elev 30, "
                             "azim 45), SphereSDF(n=64) + 8x128 F32 shift MLP, "
                             "ComposeSpatialVarying([NeuralBSDF x2, Diffuse, Conductor]), "
                             "PointLights(scale 5) at 1.05 x camera centre, Direct()")
    if name == "dtu":
        sdf = SkipConnMLP(num_layers=8, hidden_size=256, in_size=3, out=1, freqs=16,
                          activation=F.softplus, device="cpu")
        shape_mlp_sdf(sdf, radius=0.2)  # random init alone has no zero level set
        comps = [NeuralBSDF(activation=torch.nn.Sigmoid(), device="cpu") for _ in range(10)] + \
                [Diffuse(preprocess=torch.sigmoid, device="cpu").random() for _ in range(6)]
        bsdf = ComposeSpatialVarying(comps, device="cpu")
        for c in comps[:10]:
            c.mlp.to(device)
        bsdf.sp_var_fn.to(device)
        K = torch.eye(4)
        K[0, 0], K[1, 1], K[0, 2], K[1, 2] = 2890.0, 2890.0, 800.0, 600.0
        poses = []
        for i in range(views):
            a = 2 * math.pi * i / views
            pose = torch.eye(4)
            pose[:3, :4] = look_at((0.866 * math.sin(a), 0.5, 0.866 * math.cos(a)))
            pose[:3, 1:3] *= -1  # DTU/IDR cameras look down +z
            poses.append(pose)
        cam = pt.cameras.DTUCamera(pose=torch.stack(poses).to(device),
                                   intrinsic=K[None].expand(views, 4, 4).contiguous().to(device),
                                   device=device)
        return dict(kind="march", shape=SDF(sdf=sdf.to(device), max_steps=samples), bsdf=bsdf,
                    lights=LightField(device="cpu").to(device), integrator=NeRFIntegrator(Direct()),
                    cameras=cam, flop_eval=FLOP_SDF_8x256,
                    workload="dtu.py-like: DTUCamera (fx=fy=2890, cx=800, cy=600, 1600x1200 "
                             "sensor), 8x256 F16 MLP SDF, ComposeSpatialVarying([NeuralBSDF x10, "
                             "Diffuse(sigmoid) x6]), LightField, NeRFIntegrator(Direct())")
    if name == "nerfle":
        nerf = NeRFLE(device="cpu", steps=samples, envmap=envmap).to(device)
        focal = float(0.5 * 800 / math.tan(0.5 * 0.6911))
        if envmap:
            workload = (f"NeRFLE (NeRF+LE, envmap=True, nerf.py:153-214, 183-191): 5x128 "
                        f"density/latent MLP + 8x64 colour MLP on 115 inputs (latent, view, the "
                        f"point light's 4x4 envmap) at {samples} depths per ray, NeRFReproduce; "
                        f"fp16: the fused k_nerfle16 with the frame-constant envmap folded into "
                        f"one input column (FLOP priced at the 115-input count)")
        else:
            workload = (f"NeRFLE (NeRF+PT, nerf.py:153-214): 5x128 density/latent MLP + "
                        f"8x64 colour MLP at {samples} depths per ray, point light, "
                        "NeRFReproduce")
        return dict(kind="nerfle", nerf=nerf, integrator=NeRFReproduce(),
                    lights=PointLights(location=[0.0, 1.0, 0.0], device=device),
                    c2w=torch.stack([view_c2w(i, views) for i in range(views)]),
                    flop_sample=FLOP_NERFLE_ENVMAP_SAMPLE if envmap else FLOP_NERFLE_SAMPLE,
                    workload=workload)
    raise ValueError(name)


def _dist_env():
    """(world, rank, local rank, process-group path on?) from torchrun's environment; a
    torch.distributed.run launch takes the process-group path even at one rank."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local, world > 1 or "TORCHELASTIC_RUN_ID" in os.environ


class NerfRowRenderer:
    """bench_other's NeRFLE rows: this rank's rows of every view -- NeRFCamera raygen on the rows'
    pixel positions, then NeRFReproduce's nerf(rays, lights) (integrators.py:260-267) -- into
    [views, rows, size, 3]."""

    def __init__(self, nerf, lights, cameras, size, rows, device):
        self.nerf, self.lights, self.cameras, self.size = nerf, lights, cameras, size
        R = len(rows)
        v = torch.tensor(list(rows), dtype=torch.float32, device=device)[:, None].expand(R, size)
        u = torch.arange(size, dtype=torch.float32, device=device)[None, :].expand(R, size)
        self.positions = torch.stack([u, v], dim=-1).contiguous()
        self.R = R

    def render(self):
        rays = self.cameras.rays_tile(0, 0, self.R, self.size, self.size, False,
                                      positions=self.positions)
        return self.nerf(rays, self.lights).reshape(len(self.cameras), self.R, self.size, 3)


def bench_other(args):
    """Bench line of a non-default scene (--scene colocate|dtu|nerfle): one view per rank (weak
    scaling, as the headline), each rank renders its rows of every view (row_shard, --tile-rows)
    and one RCCL all-gather per step assembles the frames (make_step) -- BASELINE cfg4 / cfg5 are
    8-GPU configurations.  Under torch.distributed.run the process-group path runs even at N = 1."""
    from neural_raytracing_amd import _lib
    import neural_raytracing_amd as nra
    import neural_raytracing_amd.pathtracer as pt
    from neural_raytracing_amd.pathtracer.render import RowRenderer, broadcast_module, row_shard
    world, rank, local, dist_on = _dist_env()
    if dist_on:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    _lib.load(require_device=True)
    if args.scene == "nerfle" and not args.precision_set:
        args.precision = "fp16"  # BASELINE cfg5 names the fp16 MFMA path
    nra.set_precision(args.precision)
    size = args.size
    sc = build_other_scene(args.scene, device, args.samples, envmap=args.envmap, views=world)
    if dist_on:
        for key in ("shape", "bsdf", "lights", "nerf"):
            if sc.get(key) is not None:
                broadcast_module(sc[key])
    rows = row_shard(size, rank, world, args.tile_rows)
    if sc["kind"] == "march":
        rr = RowRenderer(sc["shape"], sc["lights"], sc["cameras"], sc["integrator"], sc["bsdf"],
                         size, rows, background=0.0, with_noise=1e-3, device=device)
        render = rr.render
        kernel = MARCH_KERNEL[args.precision]
        channels = sc["integrator"].dims()
    else:
        focal = float(0.5 * size / math.tan(0.5 * 0.6911))
        cam = pt.cameras.NeRFCamera(cam_to_world=sc["c2w"].to(device), focal=focal, device=device)
        rr = NerfRowRenderer(sc["nerf"], sc["lights"], cam, size, rows, device)
        render = rr.render
        kernel = "k_nerfle"
        channels = 3
    step = make_step(render, rows, size, rank, world, args.tile_rows, device, channels=channels,
                     gather=dist_on)
    with torch.no_grad():
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        if dist_on:
            torch.distributed.barrier()
        _lib.profile_reset()
        _lib.profile_enable(True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        if dist_on:
            torch.distributed.barrier()
        elapsed = time.perf_counter() - t0
        _lib.profile_enable(False)
        k_ms, k_n = _lib.profile_read(kernel)
        evals = count_evals(render) if sc["kind"] == "march" else None
        elapsed = max_over_ranks(elapsed, world, device, force=dist_on)
    rays_rank = len(rows) * size * world  # this rank's rows of every view, per step
    rays_total = world * size * size * args.steps
    if sc["kind"] == "march":
        products = 3 if args.precision == "fp32-split" else 1  # f16 MFMA products per f32 one
        flop = rays_rank * args.steps * (args.samples + MARCH_KERNEL_SCAN_EVALS) * \
            sc["flop_eval"] * products
    else:
        flop = rays_rank * args.steps * args.samples * sc["flop_sample"]
    achieved = flop / (k_ms * 1e-3) / 1e12
    peak = PEAK_TFLOPS[args.precision]
    roof = {"bound": "mfma", "kernel": kernel, "achieved": achieved, "peak": peak,
            "unit": "TFLOP/s", "frac": achieved / peak, "traffic": None,
            "flop_per_step": flop / args.steps, "kernel_ms_per_step": k_ms / args.steps,
            "launches": k_n}
    if evals is not None:
        # the evaluations the job lists ran (device counter, one untimed frame), less the
        # sdf(best) pass's: the kernel's utilisation (the algorithmic count prices every ray at
        # every march step and can pass 1 when rays stop early, as on DTU)
        exe = (evals - rays_rank) * sc["flop_eval"] * products * args.steps
        roof["executed_flop_per_step"] = exe / args.steps
        roof["executed_achieved"] = exe / (k_ms * 1e-3) / 1e12
        roof["executed_frac"] = roof["executed_achieved"] / peak
        roof["executed_evals_per_ray"] = evals / rays_rank
        if args.precision == "mixed":
            # the split refinement's time too (its evaluations are in the count, priced at one
            # product though a split evaluation issues three: a lower bound)
            ex_ms = k_ms
            for k in ("k_refine3", "k_best3"):
                ex_ms += _lib.profile_read(k)[0]
            roof["executed_achieved"] = exe / (ex_ms * 1e-3) / 1e12
            roof["executed_frac"] = roof["executed_achieved"] / peak
    if sc["kind"] != "march":
        # every sample of every ray is evaluated (no early stop): executed = algorithmic, up to
        # the k_nerfle16 program's padding (which the algorithmic count does not price)
        roof["executed_frac"] = roof["frac"]
    pmc = _committed_pmc(kernel, args.scene, size, args.precision)
    if pmc is not None:
        roof["traffic"], roof["traffic_source"] = pmc
        if sc["kind"] != "march":
            roof["traffic_note"] = "per launch: the frame runs in %d launches" % max(k_n // max(args.steps, 1), 1)
    line = {
        "metric": f"ray-samples/sec/GPU ({args.scene} {size}x{size}x{args.samples})",
        "value": rays_total * args.samples / elapsed, "unit": "ray-samples/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1000 * elapsed / args.steps,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": args.precision, "data": "synthetic (seeded random-init weights)",
        "config": {"workload": sc["workload"], "image": [size, size],
                   "samples_per_ray": args.samples, "views_per_step": world,
                   "parallelism": f"row-tile shard x{world} ({args.tile_rows}-row tiles) + RCCL "
                                  "all-gather"},
        "roofline": roof,
    }
    if sc["kind"] == "march" and args.scene == "colocate":
        line["valu_roofline"] = colocate_valu_roofline(size, args, k_ms / max(k_n, 1))
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist_on:
        torch.distributed.destroy_process_group()


def _committed_pmc(kernel, scene, size, precision):
    """(HBM bytes per launch, source) from a committed PMC pass of this scene's kernel
    (profiles/pmc_<scene>_<precision>_<kernel>.json: FETCH_SIZE + WRITE_SIZE per launch,
    tools/r06_pmc_scenes.sh), or None; the pass must be of the same frame size and precision."""
    path = os.path.join(ROOT, "profiles", f"pmc_{scene}_{precision}_{kernel}.json")
    if not os.path.exists(path):
        return None
    try:
        pm = json.load(open(path))
    except Exception:
        return None
    if pm.get("size") != size or pm.get("precision") != precision:
        return None
    return pm.get("hbm_bytes_per_launch"), (f"committed PMC pass, profiles/pmc_{scene}_"
                                            f"{precision}_{kernel}.json ({size}^2); not measured "
                                            "in this run")


PATH_PASSES = 32  # path_nerv.py:86 run_tests(num_samples=32): pathtrace passes per frame
PATH_LIGHT = (0.8, 1.0, 0.6)
# the march kernels of a Path frame per precision: the primary / secondary march and the shadow
# march (k_occl*: intersect_test toward the point light, w_isect=True)
PATH_KERNELS = {"fp32": ("k_march32", "k_occl32"), "fp16": ("k_march16", "k_occl16"),
                "fp32-split": ("k_march3", "k_occl3"), "mixed": ("k_march16", "k_occl3")}


def build_path_scene(device, samples, seed=0):
    """path_nerv.py's scene (scripts/path_nerv.py:42-99; the models nerv.py:84-95 trains), seeded
    random init: SDF(SphereSDF(n=128)) with max_steps 64 (radii + 0.15 and the 8x128 F32 shift at
    default torch init, output x0.1, so the random blob has a surface), ComposeSpatialVarying of 7
    NeuralBSDFs with act = sigmoid (path_nerv.py:52), PointLights(intensity 1, scale 300)."""
    import neural_raytracing_amd.pathtracer as pt
    from neural_raytracing_amd.pathtracer.bsdf import ComposeSpatialVarying, NeuralBSDF
    from neural_raytracing_amd.pathtracer.lights import PointLights
    from neural_raytracing_amd.pathtracer.neural_blocks import SkipConnMLP
    from neural_raytracing_amd.pathtracer.shapes import SDF, SphereSDF
    torch.manual_seed(seed)
    random.seed(seed)
    sphere = SphereSDF(n=128, device="cpu")
    with torch.no_grad():
        sphere.radii.add_(0.15)
    sphere.shift = SkipConnMLP(num_layers=8, hidden_size=128, in_size=3, out=1, freqs=32,
                               activation=F.softplus, device="cpu")
    with torch.no_grad():
        sphere.shift.out.weight.mul_(0.1)
        sphere.shift.out.bias.mul_(0.1)
    shape = SDF(sdf=sphere.to(device), max_steps=samples)
    # act = sigmoid as path_nerv.py:52 sets it on the loaded models (here at construction: on a
    # NeuralBSDF built with a Softplus module, torch refuses the setattr of a function)
    comps = [NeuralBSDF(activation=torch.sigmoid, device="cpu") for _ in range(7)]
    for c in comps:
        c.mlp.to(device)
    bsdf = ComposeSpatialVarying(comps, device="cpu")
    bsdf.sp_var_fn.to(device)
    lights = PointLights(intensity=[1.0, 1.0, 1.0], location=list(PATH_LIGHT), scale=300.0,
                         device=device)
    return dict(shape=shape, bsdf=bsdf, lights=lights, pt=pt)


def bench_path(args):
    """`--scene path`: path_nerv.py's render (scripts/path_nerv.py:86-104) -- Path() (max_depth 2,
    the secondary-ray integrator of BASELINE cfg5, integrators.py:275-354) with shadow rays
    (w_isect=True), 200^2 in 100^2 tiles, 32 pathtrace passes averaged per frame.  One step = one
    frame; the unit is the metric's ray-sample (primary rays x max_steps, W H S per pass).  The
    passes run on pathtrace's batched Path (main._path_tiles: all tiles in one primary march, one
    bounce kernel and one compacted secondary march per bounce); the `per_tile` leg times the
    tile-by-tile loop of the reference.  Roofline: the march kernels (primary, secondary, shadow)
    over the SDF evaluations they executed (device counter).  One view per rank (replicas: the
    passes' draws depend on the ray count, so rows are not dealt; the MAX time over ranks)."""
    from neural_raytracing_amd import _lib
    import neural_raytracing_amd as nra
    from neural_raytracing_amd.pathtracer import main as ptmain
    from neural_raytracing_amd.pathtracer.integrators import Path
    world, rank, local, dist_on = _dist_env()
    if dist_on:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    _lib.load(require_device=True)
    nra.set_precision(args.precision)
    size, S = args.size, args.samples
    sc = build_path_scene(device, S)
    pt = sc["pt"]
    focal = float(0.5 * size / math.tan(0.5 * 0.6911))
    cam = pt.cameras.NeRFCamera(cam_to_world=view_c2w(rank, max(world, 1))[None].to(device),
                                focal=focal, device=device)
    integrator = Path()
    chunk = min(size, 100)

    def frame():
        got = None
        for _ in range(PATH_PASSES):
            sample = pt.pathtrace(sc["shape"], size=size, chunk_size=chunk, bundle_size=1,
                                  bsdf=sc["bsdf"], integrator=integrator, background=0,
                                  cameras=cam, lights=sc["lights"], device=device, silent=True,
                                  w_isect=True)[0]
            got = sample if got is None else got + sample
        return got / PATH_PASSES
    kernels = PATH_KERNELS[args.precision]
    with torch.no_grad():
        el, ks, evals = _time_frames(frame, args.steps, args.warmup,
                                     list(kernels) + ["k_path_sample", "k_light16", "k_bsdf16"])
        elapsed = max_over_ranks(el, world, device, force=dist_on)
        img = frame()
        lit = float((img.abs().sum(-1) > 0).float().mean())
        ptmain.BATCH_PATH = False
        try:
            el_tile, _, _ = _time_frames(frame, 1, 1, [])
        finally:
            ptmain.BATCH_PATH = True
    rays_frame = size * size * PATH_PASSES
    k_ms = sum(ks[k][0] for k in kernels) / args.steps
    peak = PEAK_TFLOPS[args.precision]
    products = 3 if args.precision == "fp32-split" else 1
    exe_flop = evals * FLOP_SHIFT_8x128 * products
    ach = exe_flop / (k_ms * 1e-3) / 1e12
    roof = {"bound": "mfma", "kernel": "+".join(kernels), "achieved": ach, "peak": peak,
            "unit": "TFLOP/s", "frac": ach / peak, "executed_frac": ach / peak, "traffic": None,
            "flop_basis": "executed: the SDF evaluations the primary, secondary and shadow "
                          "marches ran in one frame (device counter) x the 8x128 F32 shift MLP's "
                          f"{FLOP_SHIFT_8x128} FLOP (the 128 spheres' smooth-min is VALU, not "
                          "counted)",
            "executed_evals_per_frame": evals,
            "executed_evals_per_primary_ray": evals / rays_frame,
            "kernel_ms_per_frame": k_ms,
            "kernels_ms_per_frame": {k: ks[k][0] / args.steps for k in ks}}
    pmc = _committed_pmc(kernels[0], "path", size, args.precision)
    if pmc is not None:
        roof["traffic"], roof["traffic_source"] = pmc
        roof["traffic_note"] = "one launch of the primary march (40,000 rays) of the first pass"
    line = {
        "metric": f"ray-samples/sec/GPU (path {size}x{size}x{S}, {PATH_PASSES} passes)",
        "value": world * rays_frame * S * args.steps / elapsed, "unit": "ray-samples/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": 1000 * elapsed / args.steps, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": args.precision,
        "data": "synthetic (seeded random-init weights)",
        "config": {"workload": f"path_nerv.py-like: Path() max_depth 2 with shadow rays "
                               f"(w_isect=True), {size}^2 in {chunk}^2 tiles, {PATH_PASSES} "
                               f"passes per frame, SDF(SphereSDF(n=128) + 8x128 F32 shift), "
                               f"max_steps {S}, ComposeSpatialVarying(7 x NeuralBSDF, sigmoid), "
                               f"PointLights(scale 300)",
                   "image": [size, size], "samples_per_ray": S, "passes_per_frame": PATH_PASSES,
                   "parallelism": f"replicas x{world} (one view per rank)"},
        "roofline": roof,
        "lit_fraction": round(lit, 4),
        "per_tile": {"ms_per_step": 1000 * el_tile,
                     "note": "the same frame with pathtrace's tile loop (BATCH_PATH off: one "
                             "Path.sample per 100^2 tile, as the reference)"},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = path_cpu_baseline(sc, cam, size, S)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist_on:
        torch.distributed.destroy_process_group()


def path_cpu_baseline(sc, cam, size, S, crop=24):
    """The oracle's PathRef (oracle/pathtracer_ref.py, 'port') on this host's threads: one pass of
    a crop x crop window at the image centre with injected uniforms, and the GPU Path.sample of
    the same rays and uniforms beside it (max |diff|)."""
    from oracle import pathtracer_ref as R
    from neural_raytracing_amd.pathtracer.integrators import Path
    blob = R.SphereBlobSDF(n=128)
    src = sc["shape"].sdf
    with torch.no_grad():
        blob.centers.copy_(src.centers.cpu())
        blob.radii.copy_(src.radii.cpu())
        blob.tfs.copy_(src.tfs.cpu())
    _copy_to_oracle(blob.shift, src.shift)
    parts = [R.NeuralBSDFRef(activation="sigmoid") for _ in sc["bsdf"].bsdfs]
    for o, p in zip(parts, sc["bsdf"].bsdfs):
        _copy_to_oracle(o.mlp, p.mlp)
    bsdf = R.SpatialMixBSDF(parts)
    _copy_to_oracle(bsdf.sp_var_fn, sc["bsdf"].sp_var_fn)
    shape = R.MarchedSDF(sdf=blob, max_steps=S)
    lights = R.PointLightRef(location=PATH_LIGHT, scale=300.0)
    c0 = (size - crop) // 2
    ocam = R.NeRFCameraRef(cam.cam_to_world.cpu(), cam.focal)
    rays = ocam.sample_positions(R._tile_positions(c0, c0, crop), size)
    g = torch.Generator().manual_seed(5)
    lead = rays.shape[:-1]
    nc = len(parts)
    uniforms = [(torch.rand(*lead, nc, 2, generator=g), torch.rand(*lead, generator=g))
                for _ in range(2)]
    threads = torch.get_num_threads()
    t0 = time.perf_counter()
    with torch.no_grad():
        want, wmask, _ = R.PathRef().sample(shape, rays, bsdf, lights, w_isect=True,
                                            uniforms=uniforms)
    cpu_s = time.perf_counter() - t0
    with torch.no_grad():
        got, gmask, _ = Path().sample(sc["shape"], rays.cuda(), sc["bsdf"], lights=sc["lights"],
                                      w_isect=True, uniforms=uniforms)
    err = (got.cpu() - want).abs()
    return {"value": crop * crop * S / cpu_s, "unit": "ray-samples/s", "cores": threads,
            **host_cpu(), "kind": "port",
            "sample": f"one Path pass (max_depth 2, shadow rays) over a {crop}x{crop} window at "
                      f"the image centre with injected uniforms, oracle/pathtracer_ref.py "
                      f"PathRef, {cpu_s:.1f} s",
            "gpu_vs_port_maxabs": float(err.max()),
            "gpu_vs_port_pixels_over_1e-4": int((err.amax(-1) > 1e-4).sum()),
            "mask_equal": bool(torch.equal(gmask.cpu(), wmask)), "hits": int(wmask.sum())}


# VALU operations per SDF evaluation of the colocate scene's SphereSDF(n=64) (sdfs.py:37-43,
# utils.py:386-387), counted per sphere as issued lane-operations: the (I + tfs) p transform 9
# fma, the centre 3 sub, |q|^2 3 fma, sqrt, - r, * -k, exp, += : 20 ops, 2 of them quarter-rate
# transcendentals (x4 issue slots) -> 26 slot-equivalents; plus the 8x128 shift MLP's activations
# (softplus as exp + add + log, 2 transcendentals: 9 slot-equivalents per element) on 128 x 9
# layers -- the work the MFMA roofline does not count.
COLOCATE_SPHERES = 64
VALU_SLOTS_PER_SPHERE = 26
VALU_SLOTS_PER_ACT = 9


def colocate_valu_roofline(size, args, kernel_ms):
    """VALU roofline of the colocate march (k_march16): algorithmic lane-operations (every ray at
    every march step and scan point, as the MFMA count) over the kernel time, against the VALU
    issue peak -- 256 CUs x 4 SIMDs x 32 lanes per clock at 2.4 GHz = 78.6 T lane-ops/s (the
    157.3 TFLOP/s FP32 vector peak counts an fma as 2)."""
    evals = size * size * (args.samples + MARCH_KERNEL_SCAN_EVALS)
    per_eval = COLOCATE_SPHERES * VALU_SLOTS_PER_SPHERE + VALU_SLOTS_PER_ACT * 128 * 9
    ops = evals * per_eval
    peak = 256 * 4 * 32 * 2.4e9 / 1e12  # T lane-ops/s
    ach = ops / (kernel_ms * 1e-3) / 1e12
    return {"bound": "valu", "unit": "T lane-ops/s", "achieved": ach, "peak": peak,
            "frac": ach / peak, "ops_per_eval": per_eval,
            "note": "smooth-min over 64 spheres + shift-MLP activations per evaluation; add the "
                    "MFMA frac for the kernel's issue-bound picture"}


def bench_train(args):
    """`--scene train`: one JSON line of the training step (train_leg)."""
    if int(os.environ.get("WORLD_SIZE", "1")) != 1:
        raise SystemExit("--scene train runs on one GPU")
    device = torch.device("cuda", 0)
    torch.cuda.set_device(device)
    from neural_raytracing_amd import _lib
    _lib.load(require_device=True)
    # --precision fp16 / mixed / fp32-split: the gradient-free march (and, fp16, the MLP
    # forwards) at that precision, every backward FP32 (default fp32: the reference's arithmetic)
    prec = args.precision if args.precision_set else "fp32"
    line = train_leg(prec, args.steps, args.warmup, size=args.size, crop=args.crop,
                     views=args.views, samples=args.samples, cpu=not args.no_cpu_baseline,
                     torch_profile=args.torch_profile)
    print(json.dumps(line), flush=True)


TRAIN_KERNELS = ("k_mlp_backward32", "k_wgrad", "k_mlp_grad_backward32")


TRAIN_MARCH = {"fp32": ("k_march32",), "mixed": ("k_march16", "k_refine3", "k_best3"),
               "fp16": ("k_march16",), "fp32-split": ("k_march3",)}


def train_roofline(steps, prec, march_evals, rays, kt, kf):
    """Roofline of the training step over the timed steps, per kernel against the 157.3 TF FP32
    matrix peak (the mixed / fp16 march against the 2.5 PF FP16 one):
      * the gradient-free march + coarse scan (TRAIN_MARCH[prec]): EXECUTED FLOP = the SDF
        evaluations its job lists ran (device counter over one more, untimed step, less the
        sdf(best) pass's one per ray) x the SphereSDF shift MLP's 331,200 FLOP (8x128 F32; the 128
        spheres' smooth-min is VALU, not counted) over the march kernels' HIP-event time;
      * the backward launches: the algorithmic FLOP the library recorded (nrt_profile_flop: the MLP
        backward's forward recompute + input-gradient chain, the split-K weight gradients, the SDF
        normal's double backward, at the layers' real widths) over their HIP-event time.
    kt: {kernel: (total ms, launches)} and kf: {kernel: FLOP} of the timed steps.  The headline
    entry is the kernel with the most time."""
    per = {}
    mk = TRAIN_MARCH[prec]
    m_ms = sum(kt[k][0] for k in mk)
    m_n = kt[mk[0]][1]
    exe = max(march_evals - rays, 0) * FLOP_SHIFT_8x128 * steps
    m_peak = PEAK_TFLOPS["fp32"] if prec == "fp32" else PEAK_TFLOPS["fp16"]
    ach = exe / (m_ms * 1e-3) / 1e12 if m_ms > 0 else 0.0
    per["+".join(mk)] = {"ms_per_step": m_ms / steps, "launches_per_step": m_n / steps,
                         "flop_per_step": exe / steps, "achieved": ach, "peak": m_peak,
                         "frac": ach / m_peak, "executed_frac": ach / m_peak,
                         "executed_evals_per_ray": march_evals / max(rays, 1),
                         "flop_basis": "executed SDF evaluations (device counter) x 331,200"}
    for k in TRAIN_KERNELS:
        ms, n = kt[k]
        flop = kf[k]
        ach = flop / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
        per[k] = {"ms_per_step": ms / steps, "launches_per_step": n / steps,
                  "flop_per_step": flop / steps, "achieved": ach, "peak": PEAK_TFLOPS["fp32"],
                  "frac": ach / PEAK_TFLOPS["fp32"]}
    top = max(per, key=lambda k: per[k]["ms_per_step"])
    out = {"bound": "mfma", "kernel": top, "achieved": per[top]["achieved"],
           "peak": per[top]["peak"], "unit": "TFLOP/s", "frac": per[top]["frac"],
           "traffic": None, "flop_basis": per[top].get("flop_basis", "algorithmic: 2 FLOP per "
                                                       "multiply-add of every layer product at "
                                                       "its real width (nrt_profile_flop)"),
           "kernels": per}
    if "executed_frac" in per[top]:
        out["executed_frac"] = per[top]["executed_frac"]
    return out


def train_leg(prec, steps, warmup, size=256, crop=80, views=6, samples=64, cpu=True,
              torch_profile=None):
    """One-GPU training-step line: the nerf_synthetic training iteration of
    training_utils.py:246-285 / scripts/nerf_synthetic.py:61-116 -- N=6 views, an 80x80 crop of
    a 256^2 frame, SDF(SphereSDF(n=128), max_steps=64), 8 NeuralBSDF(Softplus) +
    ComposeSpatialVarying, LightField, NeRFIntegrator(Direct); loss = MSE + eikonal(raw_normals);
    backward through the fused path; AdamW with the script's three learning rates.  `prec` sets
    the gradient-free march's arithmetic (fp32 = the reference's; mixed = FP16 march with its
    undecidable steps at FP32 accuracy); every MLP forward and backward is FP32 except under
    fp16.  The process precision is restored afterwards."""
    from neural_raytracing_amd import _lib
    import neural_raytracing_amd as nra
    import neural_raytracing_amd.pathtracer as pt
    from neural_raytracing_amd.pathtracer.bsdf import ComposeSpatialVarying, NeuralBSDF
    from neural_raytracing_amd.pathtracer.integrators import Direct, NeRFIntegrator
    from neural_raytracing_amd.pathtracer.lights import LightField
    from neural_raytracing_amd.pathtracer.shapes import SDF, SphereSDF
    device = torch.device("cuda", torch.cuda.current_device())
    old_prec = nra.get_precision()
    nra.set_precision(prec)
    torch.manual_seed(0)
    random.seed(0)
    sdf = SphereSDF(n=128, device="cpu")
    with torch.no_grad():  # a non-trivial residual (the scripts load a trained one)
        for a in [sdf.shift.init, *sdf.shift.layers]:
            a.weight.normal_(0.0, 0.02)
        sdf.shift.out.weight.normal_(0.0, 0.002)
    shape = SDF(sdf=sdf.to(device), device=device, max_steps=samples)
    bsdf = ComposeSpatialVarying([NeuralBSDF(activation=torch.nn.Softplus(), device="cpu")
                                  for _ in range(8)], device="cpu")
    for b in bsdf.bsdfs:
        b.mlp.to(device)
    bsdf.sp_var_fn.to(device)
    lights = LightField(device="cpu").to(device)
    integrator = NeRFIntegrator(Direct())
    opt = torch.optim.AdamW([
        {"params": list(shape.parameters()), "lr": 8e-5},
        {"params": list(bsdf.parameters()), "lr": 8e-4},
        {"params": list(lights.parameters()), "lr": 8e-5},
    ], lr=8e-5, weight_decay=0)
    N = views
    focal = float(0.5 * size / math.tan(0.5 * 0.6911))
    c2w = torch.stack([view_c2w(i, N) for i in range(N)]).to(device)
    cameras = pt.cameras.NeRFCamera(cam_to_world=c2w, focal=focal, device=device)
    g = torch.Generator().manual_seed(1)
    target = torch.rand(N, crop, crop, 3, generator=g).to(device)

    def step(i):
        random.seed(i)
        opt.zero_grad()
        uv = ((37 * i) % (size - crop), (53 * i) % (size - crop))
        got, mi = pt.pathtrace_sample(shape, lights, cameras, integrator, bsdf=bsdf, size=size,
                                      chunk_size=size, bundle_size=1, crop_size=crop, uv=uv,
                                      background=0, addition=lambda m: m, squeeze_first=False,
                                      device=device)
        loss = F.mse_loss(got[..., :3], target)
        raw = getattr(mi, "raw_normals", None)
        if raw is not None:
            loss = loss + (raw.norm(dim=-1) - 1).square().mean()
        loss.backward()
        opt.step()
        return loss

    try:
        for i in range(warmup):
            step(i)
        torch.cuda.synchronize()
        if torch_profile:
            train_torch_profile(step, torch_profile)
        _lib.profile_reset()
        _lib.profile_enable(True)
        t0 = time.perf_counter()
        for i in range(steps):
            loss = step(warmup + i)
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        _lib.profile_enable(False)
        kms = {k: _lib.profile_read(k)[0] / steps
               for k in ("k_intersect",) + TRAIN_MARCH[prec] + TRAIN_KERNELS}
        kt = {k: _lib.profile_read(k) for k in TRAIN_MARCH[prec] + TRAIN_KERNELS}
        kf = {k: _lib.profile_flop(k) for k in TRAIN_KERNELS}
        # the march's executed evaluations: one more, untimed step with the device counter
        _lib.profile_reset()
        _lib.profile_enable(False, evals=True)
        step(warmup + steps)
        torch.cuda.synchronize()
        march_evals = _lib.profile_evals()
        _lib.profile_enable(False)
        roof = train_roofline(steps, prec, march_evals, N * crop * crop, kt, kf)
    finally:
        nra.set_precision(old_prec)
    rays = N * crop * crop
    line = {
        "metric": f"training ray-samples/sec/GPU (nerf_synthetic step, {N}x{crop}x{crop} crop "
                  f"of {size}^2, {samples} march steps)",
        "value": rays * samples * steps / elapsed, "unit": "ray-samples/s",
        "n_gpus": 1, "steps": steps, "warmup": warmup,
        "ms_per_step": 1000 * elapsed / steps, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None,
        "dtype": {"fp32": "fp32", "fp16": "fp16 forward / fp32 backward",
                  "fp32-split": "fp32-split forward (f16 hi/lo MFMA) / fp32 backward",
                  "mixed": "mixed march (fp16 + split refinement) / fp32 MLP forwards and "
                           "backward"}[prec],
        "data": "synthetic (seeded random-init weights, random target crops)",
        "config": {"workload": "forward (fused march + scan) + backward (MLP backward, SDF-normal "
                               "double backward, shading autograd) + AdamW",
                   "views": N, "crop": crop, "image": [size, size],
                   "samples_per_ray": samples, "precision": prec},
        "roofline": roof,
        "kernel_ms_per_step": kms, "final_loss": float(loss),
    }
    if cpu:
        line["cpu_baseline"] = cpu_train_baseline(sdf, bsdf, lights, size, focal, samples)
    return line


def train_torch_profile(step, path):
    """Op counts of one training step by Python call site and its host synchronisations (tools:
    where the launches come from), written to `path`."""
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
        step(10_000)
        torch.cuda.synchronize()
    # host synchronisations of one step by call site (torch.cuda sync debug mode)
    import collections
    import traceback
    import warnings
    sites = collections.Counter()

    def show(message, category, filename, lineno, file=None, line=None):
        stack = [f for f in traceback.extract_stack()[:-1]
                 if "site-packages" not in f.filename and "warnings" not in f.filename]
        sites[" <- ".join(f"{f.filename.split('/')[-1]}:{f.lineno}" for f in stack[-4:])] += 1
    old_show = warnings.showwarning
    warnings.showwarning = show
    torch.cuda.set_sync_debug_mode("warn")
    try:
        with warnings.catch_warnings():
            warnings.simplefilter("always")
            warnings.showwarning = show
            step(10_001)
            torch.cuda.synchronize()
    finally:
        torch.cuda.set_sync_debug_mode(0)
        warnings.showwarning = old_show
    with open(path, "w") as f:
        f.write(prof.key_averages().table(sort_by="count", row_limit=120,
                                          max_name_column_width=40))
        f.write("\n\nhost syncs by call site (one step)\n")
        for site, n in sites.most_common():
            f.write(f"{n:6d}  {site}\n")


def cpu_train_baseline(sdf, bsdf, lights, size, focal, samples, crop=176):
    """The oracle (torch-CPU restatement, 'port') running the same training step -- forward,
    create_graph normals, loss = MSE + eikonal, backward -- on one view's crop x crop window, on
    this host's threads; rate in training ray-samples/s like the GPU line."""
    from oracle import pathtracer_ref as R
    blob = R.SphereBlobSDF(n=sdf.centers.shape[0])
    with torch.no_grad():
        blob.centers.copy_(sdf.centers.cpu())
        blob.radii.copy_(sdf.radii.cpu())
        blob.tfs.copy_(sdf.tfs.cpu())
    _copy_to_oracle(blob.shift, sdf.shift)
    shape = R.MarchedSDF(sdf=blob, max_steps=samples, create_graph=True)
    parts = [R.NeuralBSDFRef(activation="softplus") for _ in bsdf.bsdfs]
    for a, b in zip(parts, bsdf.bsdfs):
        _copy_to_oracle(a.mlp, b.mlp)
    obsdf = R.SpatialMixBSDF(parts)
    _copy_to_oracle(obsdf.sp_var_fn, bsdf.sp_var_fn)
    olights = R.LightFieldRef()
    _copy_to_oracle(olights.light_field_approx, lights.light_field_approx)
    with torch.no_grad():
        olights.color.copy_(lights.color.cpu())
    cam = R.NeRFCameraRef(view_c2w(0, 1).unsqueeze(0), focal)
    integ = R.NeRFIntegratorRef(R.DirectRef())
    c0 = (size - crop) // 2
    target = torch.rand(crop, crop, 3, generator=torch.Generator().manual_seed(2))
    random.seed(9)
    t0 = time.perf_counter()
    img = R.render(shape, olights, cam, integ, obsdf, size=size, chunk_size=size, background=0.0,
                   with_noise=0.0, crop=(c0, c0, crop))
    rays = cam.sample_positions(R._tile_positions(c0, c0, crop), size, 0.0)
    o, d = rays.split(3, dim=-1)
    t, hit = shape.march(o, d)
    raw = shape.gradient((o + t * d)[hit])
    loss = F.mse_loss(img[..., :3], target) + (raw.norm(dim=-1) - 1).square().mean()
    loss.backward()
    cpu_s = time.perf_counter() - t0
    return {"value": crop * crop * samples / cpu_s, "unit": "ray-samples/s",
            "cores": torch.get_num_threads(), **host_cpu(), "kind": "port",
            "sample": f"one view, {crop}x{crop} crop, {samples} march steps + scan, forward + "
                      f"backward (oracle/pathtracer_ref.py autograd), {cpu_s:.1f} s"}


def host_cpu():
    """lscpu-style description of the host the CPU baseline ran on: model name, physical cores
    and logical CPUs of the machine (/proc/cpuinfo), next to ``cores`` = the torch threads the
    oracle actually used (the box's CPU share: OMP_NUM_THREADS)."""
    model, phys, logical = None, set(), 0
    try:
        with open("/proc/cpuinfo") as fh:
            pid = core = None
            for line in fh:
                k, _, v = line.partition(":")
                k, v = k.strip(), v.strip()
                if k == "processor":
                    logical += 1
                elif k == "model name" and model is None:
                    model = v
                elif k == "physical id":
                    pid = v
                elif k == "core id":
                    core = v
                    phys.add((pid, core))
    except OSError:
        pass
    return {"cpu_model": model, "physical_cores_on_host": len(phys) or None,
            "logical_cpus_on_host": logical or None, "threads_used": torch.get_num_threads()}


def rr_hit_fraction(rr):
    from neural_raytracing_amd.pathtracer import render as R
    for b in R._BUFS.values():
        return b.hit.float().mean().item()
    return 0.0


def single_camera(cameras):
    return type(cameras)(cam_to_world=cameras.cam_to_world[:1], focal=cameras.focal,
                         device=cameras.device)


def silhouette_crop(size, crop):
    """(row, column) origin of the accuracy crop: centred vertically, its columns across the left
    silhouette of the object (the metric-config parity test's crop, rows 368.., cols 72.. of the
    800 frame, scaled), so marches that can flip near the edge are in the number."""
    return (size - crop) // 2, int(round(72 * size / 800))


def crop_flips(scene, osc, gcam, ocam, c0, c1, crop, size):
    """Hit flips and step flips (both hit, depths differ by > 1e-4) between the GPU march and the
    oracle march of the crop's rays, and the per-pixel agreement mask."""
    from oracle import pathtracer_ref as R
    with torch.no_grad():
        it, h = scene["shape"].intersect(gcam.rays_tile(c0, c1, crop, crop, size), primary=False)
        o, d = ocam.sample_positions(R._tile_positions(c0, c1, crop), size).split(3, dim=-1)
        rt, rh = osc["shape"].march(o, d)
    h, rh = h.cpu().reshape(-1), rh.reshape(-1)
    t, rt = it.t.cpu().reshape(-1), rt.reshape(-1)
    step = (h & rh) & ((t - rt).abs() > 1e-4)
    return (h == rh) & ~step, int(rh.sum()), int((h != rh).sum()), int(step.sum())


def cpu_baseline(scene, size, args):
    """The CPU restatement (oracle/, 'port') on this host's cores over a bounded crop, plus the
    PSNR / max-abs of the GPU render of the same crop against it.  The crop straddles the
    silhouette (silhouette_crop); hit and step flips of the march are reported beside it."""
    import neural_raytracing_amd as nra
    from oracle import pathtracer_ref as R
    threads = torch.get_num_threads()
    osc = oracle_scene(scene)
    focal = float(0.5 * size / math.tan(0.5 * 0.6911))
    c2w = view_c2w(0, 1).unsqueeze(0)
    ocam = R.NeRFCameraRef(c2w, focal)
    crop = args.cpu_crop
    c0, c1 = silhouette_crop(size, crop)
    random.seed(7)
    t0 = time.perf_counter()
    with torch.no_grad():
        want = R.render(osc["shape"], osc["lights"], ocam, osc["integrator"], osc["bsdf"], size=size,
                        chunk_size=size, background=0.0, with_noise=0.0, crop=(c0, c1, crop))
    cpu_s = time.perf_counter() - t0
    rate = crop * crop * args.samples / cpu_s
    pt = scene["pt"]
    gcam = pt.cameras.NeRFCamera(cam_to_world=c2w.cuda(), focal=focal)
    acc = {}
    for prec in ("fp32", args.precision):
        nra.set_precision(prec)
        random.seed(7)
        with torch.no_grad():
            got, _ = pt.pathtrace_sample(scene["shape"], scene["lights"], gcam, scene["integrator"],
                                         bsdf=scene["bsdf"], size=size, chunk_size=size,
                                         bundle_size=1, crop_size=crop, uv=(c0, c1), background=0,
                                         with_noise=0.0)
        got = got.cpu()
        agree, hits, flips, steps = crop_flips(scene, osc, gcam, ocam, c0, c1, crop, size)
        err = (got - want).abs().amax(-1).reshape(-1)
        mse = ((got.clamp(0, 1) - want.clamp(0, 1)) ** 2).mean().item()
        acc[prec] = {"psnr": -10 * math.log10(max(mse, 1e-12)), "maxabs": err.max().item(),
                     "maxabs_agreeing": err[agree].max().item() if bool(agree.any()) else 0.0,
                     "pixels_over_1e-4": int((err > 1e-4).sum()), "hits": hits,
                     "hit_flips": flips, "step_flips": steps}
    nra.set_precision(args.precision)
    a = acc[args.precision]
    return {
        "cpu_baseline": {"value": rate, "unit": "ray-samples/s", "cores": threads, **host_cpu(),
                         "kind": "port",
                         "threads_note": "torch's intra-op threads = the CPU share this job is "
                                         "given (the GPU box's lease; the host's other cores "
                                         "belong to other jobs)",
                         "sample": f"{crop}x{crop} crop of the same frame (rows {c0}.., columns "
                                   f"{c1}.., across the silhouette), {args.samples} march steps + "
                                   f"coarse scan + shading, oracle/pathtracer_ref.py, {cpu_s:.1f} s"},
        "psnr_vs_ref": round(a["psnr"], 2),
        "fp32_maxabs_vs_ref": acc["fp32"]["maxabs"],
        "vs_ref_crop": {"origin": [c0, c1], "side": crop, "pixels": crop * crop, **a,
                        "precision": args.precision,
                        "note": "the oracle render of the crop is the reference; psnr over RGBA "
                                "clamped to [0, 1] (120 = the 1e-12 MSE floor); maxabs_agreeing "
                                "excludes the pixels whose march flipped (hit_flips + step_flips)"},
    }


if __name__ == "__main__":
    main()
