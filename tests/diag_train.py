"""Diagnostic script, not collected by pytest (test infrastructure): per-stage differences between the HIP training path and the
oracle on the perturbed BASELINE scene crop.  Writes gpurun_out/diag_train.txt."""
import random
import sys

import torch

sys.path.insert(0, ".")
from oracle import pathtracer_ref as R  # noqa: E402
import tests.test_gpu_train_render as T  # noqa: E402
from neural_raytracing_amd import set_precision  # noqa: E402
from neural_raytracing_amd.pathtracer import differentiable as D  # noqa: E402

set_precision("fp32")
ref, mine = T._perturbed_scene()
crop = (112, 112, 32)
rays_o = ref["camera"].sample_positions(R._tile_positions(*crop), 256, 0.0)
rays_m = mine["camera"].rays_tile(crop[0], crop[1], 32, 32, 256) if hasattr(mine["camera"], "rays_tile") else None
out = []
def rep(name, a, b):
    a = a.detach().cpu().reshape(-1, a.shape[-1] if a.dim() else 1).double()
    b = b.detach().cpu().reshape(a.shape).double()
    d = (a - b).abs()
    per = d.max(dim=-1).values
    top = per.argsort(descending=True)[:5]
    out.append(f"{name}: max {d.max().item():.3g} mean {d.mean().item():.3g} worst rows {top.tolist()} vals {per[top].tolist()}")
rep("rays", rays_m.reshape(-1, 6), rays_o.reshape(-1, 6))
random.seed(11)
it_o, hit_o = ref["shape"].intersect(rays_o, primary=True)
random.seed(11)
it_m, hit_m = mine["shape"].intersect(rays_m.reshape(rays_o.shape), primary=True)
out.append(f"hits {int(hit_o.sum())} {int(hit_m.sum())} equal {bool((hit_o.cpu() == hit_m.cpu()).all())}")
rep("t", it_m.t.reshape(-1, 1), it_o.t.reshape(-1, 1))
rep("p", it_m.p, it_o.p)
rep("n", it_m.n, it_o.n)
rep("wi", it_m.wi, it_o.wi)
rep("frame", it_m.frame.reshape(-1, 9), it_o.frame.reshape(-1, 9))
rep("throughput", it_m.throughput.reshape(-1, 1), it_o.throughput.reshape(-1, 1))
rep("raw", it_m.raw_normals, it_o.raw_normals)
act_o = hit_o
d_m, le_m, _ = D.light_sample(mine["lights"], it_m, hit_m.cuda())
ds_o, le_o = R.emitter(it_o, ref["shape"], ref["lights"], act_o, False)
rep("light d", d_m, ds_o.d)
rep("Le", le_m, le_o)
wo_m, wo_o = it_m.to_local(d_m), it_o.to_local(ds_o.d)
rep("wo", wo_m, wo_o)
rep("rusin", D.param_rusin2(it_m.wi, wo_m), R.rusinkiewicz(it_o.wi, wo_o))
for j in (0, 1, 2, 6):
    fm, _ = D.bsdf_eval(mine["bsdf"].bsdfs[j], it_m, wo_m, hit_m.cuda())
    fo, _ = ref["bsdf"].bsdfs[j].eval_and_pdf(it_o, wo_o, act_o)
    rep(f"f{j}", fm, fo)
k_m = mine["bsdf"].sp_var_fn(it_m.p).sigmoid()
k_o = ref["bsdf"].weights(it_o.p)
rep("k", k_m, k_o)
open("gpurun_out/diag_train.txt", "w").write("\n".join(out) + "\n")
print("\n".join(out))

# ---- isolate the NeuralBSDF MLP backward on the scene's own inputs
out2 = []
x = D.param_rusin2(it_m.wi, wo_m).detach()
dy = torch.randn(x.shape[:-1] + (3,), generator=torch.Generator().manual_seed(3))
mm = mine["bsdf"].bsdfs[0].mlp
mo = ref["bsdf"].bsdfs[0].mlp
for q in mm.parameters():
    q.grad = None
for q in mo.parameters():
    q.grad = None
(mm(x.reshape(-1, 3)) * dy.reshape(-1, 3).cuda()).sum().backward()
import copy
mo64 = copy.deepcopy(mo).double()
mo64.basis_p = mo.basis_p.double()
(mo64(x.reshape(-1, 3).cpu().double()) * dy.reshape(-1, 3).double()).sum().backward()
(mo(x.reshape(-1, 3).cpu()) * dy.reshape(-1, 3)).sum().backward()
for i, (a, b, c) in enumerate(zip(mm._linears(), [mo64.init, *mo64.layers, mo64.out], [mo.init, *mo.layers, mo.out])):
    e = (a.weight.grad.cpu().double() - b.weight.grad).abs().max().item()
    e32 = (c.weight.grad.double() - b.weight.grad).abs().max().item()
    out2.append(f"bsdf0 MLP W{i}: hip err {e:.3g} fp32-cpu err {e32:.3g} scale {b.weight.grad.abs().max().item():.3g}")
# near-zero pre-activations in the oracle forward
zs = []
def hook(m, i, o):
    zs.append(o.detach().abs().min().item())
hs = [l.register_forward_hook(hook) for l in [mo.init, *mo.layers]]
mo(x.reshape(-1, 3).cpu())
for h in hs:
    h.remove()
out2.append(f"min |z| per layer {zs}")
out2.append(f"x range {x.min().item():.3g} {x.max().item():.3g}; x rows with |x|<1e-6: {int((x.abs() < 1e-6).any(-1).sum())}")
open("gpurun_out/diag_train.txt", "a").write("\n".join(out2) + "\n")
print("\n".join(out2))
