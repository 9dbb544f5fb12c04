"""Staged GPU diagnostic: each stage runs in its own process; stops at the first failure."""
import os
import subprocess
import sys

STAGES = {
    "torch": "import torch; x = torch.ones(4).cuda() * 2; torch.cuda.synchronize(); print(x.sum().item())",
    "raygen": """
import torch, neural_raytracing_amd.pathtracer as pt
c2w = torch.eye(4)[:3,:4].clone(); c2w[2,3] = 1
cam = pt.cameras.NeRFCamera(cam_to_world=c2w[None].cuda(), focal=100.0)
r = cam.rays_tile(0, 0, 8, 8, 64); torch.cuda.synchronize(); print(r.reshape(-1,6)[:2])
""",
    "unit_sdf": """
import torch
from neural_raytracing_amd.pathtracer.shapes import SDF, SPHERE_SDF
from neural_raytracing_amd.pathtracer.shapes.sdfs import sdf_eval
p = torch.rand(100, 3).cuda()
with torch.no_grad(): v = sdf_eval(SPHERE_SDF, p)
torch.cuda.synchronize(); print((v.cpu() - (p.cpu().norm(dim=-1) - 1)).abs().max())
""",
}
MLP = """
import torch, sys
sys.path.insert(0, '.')
from neural_raytracing_amd import set_precision
from oracle import pathtracer_ref as R
from tests.helpers import product_mlp_like
set_precision('{prec}')
torch.manual_seed(0)
ref = R.SkipMLP(num_layers={L}, hidden_size={H}, out={O}, freqs=16, activation='{act}')
mine = product_mlp_like(ref, '{act}')
x = torch.rand({M}, 3) * 2 - 1
with torch.no_grad():
    want = ref(x); got = mine(x.cuda()); torch.cuda.synchronize(); got = got.cpu()
print('maxdiff', (got - want).abs().max().item(), 'scale', want.abs().max().item())
"""
for name, prec, H, L, O, M, waves in [
    ("mlp16_h32", "fp16", 32, 2, 1, 64, 4),
    ("mlp32_h32", "fp32", 32, 2, 1, 64, 4),
    ("mlp32_h256_w1", "fp32", 256, 8, 1, 64, 1),
    ("mlp32_h256_w4", "fp32", 256, 8, 1, 64, 4),
    ("mlp16_h256", "fp16", 256, 8, 1, 64, 4),
]:
    STAGES[name] = (MLP.format(prec=prec, H=H, L=L, O=O, M=M, act="softplus"), waves)

for name, spec in STAGES.items():
    code, waves = (spec, 4) if isinstance(spec, str) else spec
    env = dict(os.environ, AMD_SERIALIZE_KERNEL="3", NRT_MAX_WAVES=str(waves))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=300)
    tail = (r.stdout + r.stderr).strip().splitlines()[-6:]
    print(f"[{name}] rc={r.returncode}", *tail, sep="\n    ", flush=True)
    if r.returncode != 0:
        sys.exit(1)
print("ALL STAGES OK")
