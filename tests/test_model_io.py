"""Safe loading of the reference's saved models, CPU only.

The reference ships no model files, so the fixtures are made here: stand-in classes with the
reference's module paths and attribute layout (neural_blocks.py:12-86, sdfs.py:16-44,
bsdfs.py:90-140 / 480-536, lights.py:40-195) are pickled with ``torch.save`` and scripted with
``torch.jit.save``; ``model_io.load`` must rebuild this package's modules with identical tensors
without importing or running anything from the files.
"""
import sys
import types

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from neural_raytracing_amd.pathtracer import model_io


def _ref_identity_div_pi(x):
    return x / 3.141592653589793


class RefSkipConnMLP(nn.Module):
    def __init__(self, num_layers=3, hidden_size=32, in_size=3, out=3, skip=3, freqs=8,
                 activation=F.softplus, latent_size=0):
        super().__init__()
        self.in_size = in_size
        self.basis_p = 16 * torch.randn(freqs, in_size).T
        self.dim_p = 2 * freqs + in_size + latent_size
        self.skip = skip
        self.latent_size = latent_size
        self.layers = nn.ModuleList([
            nn.Linear(hidden_size + self.dim_p if (i % skip) == 0 and i != num_layers - 1
                      else hidden_size, hidden_size) for i in range(num_layers)])
        self.init = nn.Linear(self.dim_p, hidden_size)
        self.out = nn.Linear(hidden_size, out)
        self.activation = activation


class RefNeuralBSDF(nn.Module):
    def __init__(self, activation):
        super().__init__()
        self.mlp = RefSkipConnMLP(num_layers=2, hidden_size=32, freqs=8, activation=F.leaky_relu)
        self.act = activation


class RefDiffuse(nn.Module):
    def __init__(self):
        super().__init__()
        self.reflectance = torch.rand(3)
        self.preproc = _ref_identity_div_pi


class RefComposeSpatialVarying(nn.Module):
    def __init__(self, bsdfs):
        super().__init__()
        self.bsdfs = bsdfs
        self.sp_var_fn = RefSkipConnMLP(num_layers=2, hidden_size=32, out=len(bsdfs), freqs=8,
                                        activation=F.leaky_relu)


class RefLightField(nn.Module):
    def __init__(self):
        super().__init__()
        self.light_field_approx = RefSkipConnMLP(num_layers=2, hidden_size=64, freqs=8,
                                                 activation=F.leaky_relu)
        self.color = nn.Parameter(torch.tensor([0.1, -0.2, 0.3]))


class RefPointLights(nn.Module):
    def __init__(self):
        super().__init__()
        self.scale = torch.tensor(5.0)
        self.intensity = torch.tensor([[0.9, 0.5, 0.3]])
        self.location = torch.tensor([[0.2, 1.1, -0.4]])
        self.const = torch.tensor(1e-8)
        self.linear = torch.tensor(1e-8)
        self.square = torch.tensor(1.0)


_PATHS = {
    "pytorch3d.pathtracer.neural_blocks": {"SkipConnMLP": RefSkipConnMLP},
    "pytorch3d.pathtracer.bsdf.bsdfs": {"NeuralBSDF": RefNeuralBSDF, "Diffuse": RefDiffuse,
                                        "ComposeSpatialVarying": RefComposeSpatialVarying,
                                        "identity_div_pi": _ref_identity_div_pi},
    "pytorch3d.pathtracer.lights.lights": {"LightField": RefLightField,
                                           "PointLights": RefPointLights},
}


for _mod, _members in _PATHS.items():
    for _name, _obj in _members.items():
        _obj.__module__ = _mod  # test-local stand-ins: pickled under the reference's paths
        _obj.__qualname__ = _name


@pytest.fixture
def ref_paths(monkeypatch):
    """Make the reference's module paths importable while pickling the stand-ins."""
    for mod, members in _PATHS.items():
        parts = mod.split(".")
        for i in range(1, len(parts)):
            parent = ".".join(parts[:i])
            if parent not in sys.modules:
                monkeypatch.setitem(sys.modules, parent, types.ModuleType(parent))
        m = types.ModuleType(mod)
        for name, obj in members.items():
            setattr(m, name, obj)
        monkeypatch.setitem(sys.modules, mod, m)


def _assert_mlp(mine, ref):
    assert torch.equal(mine.basis_p.cpu(), ref.basis_p)
    refs = [ref.init, *ref.layers, ref.out]
    assert len(mine._linears()) == len(refs)
    for a, b in zip(mine._linears(), refs):
        assert torch.equal(a.weight.detach().cpu(), b.weight.detach())
        assert torch.equal(a.bias.detach().cpu(), b.bias.detach())


def test_pickled_bsdf_roundtrip(tmp_path, ref_paths):
    torch.manual_seed(0)
    ref = RefComposeSpatialVarying([RefNeuralBSDF(nn.Softplus()), RefNeuralBSDF(torch.sigmoid),
                                    RefDiffuse()])
    torch.save(ref, tmp_path / "bsdf.pt")
    mine = model_io.load(str(tmp_path / "bsdf.pt"), device="cpu")
    from neural_raytracing_amd.pathtracer.bsdf import ComposeSpatialVarying, Diffuse, NeuralBSDF
    from neural_raytracing_amd.pathtracer.bsdf import bsdfs as B
    assert isinstance(mine, ComposeSpatialVarying)
    assert [type(b) for b in mine.bsdfs] == [NeuralBSDF, NeuralBSDF, Diffuse]
    assert isinstance(mine.bsdfs[0].act, nn.Softplus)
    assert mine.bsdfs[1].act is torch.sigmoid
    assert mine.bsdfs[2].preproc is B.identity_div_pi
    assert torch.equal(mine.bsdfs[2].reflectance.detach(), ref.bsdfs[2].reflectance)
    for a, b in zip(mine.bsdfs[:2], ref.bsdfs[:2]):
        _assert_mlp(a.mlp, b.mlp)
    _assert_mlp(mine.sp_var_fn, ref.sp_var_fn)


def test_pickled_lights_roundtrip(tmp_path, ref_paths):
    torch.manual_seed(1)
    lf, pl = RefLightField(), RefPointLights()
    torch.save(lf, tmp_path / "lf.pt")
    torch.save(pl, tmp_path / "pl.pt")
    mine = model_io.load(str(tmp_path / "lf.pt"), device="cpu")
    _assert_mlp(mine.light_field_approx, lf.light_field_approx)
    assert torch.equal(mine.color.detach(), lf.color.detach())
    p = model_io.load(str(tmp_path / "pl.pt"), device="cpu")
    assert torch.equal(p.location.reshape(-1, 3), pl.location)
    assert torch.equal(p.intensity.reshape(-1, 3), pl.intensity)
    assert float(p.scale) == 5.0 and float(p.square) == 1.0


class _ScriptMLP(nn.Module):
    """Scriptable stand-in with SkipConnMLP's attributes (softplus, as SphereSDF.shift)."""

    def __init__(self, num_layers: int, hidden: int, freqs: int):
        super().__init__()
        self.in_size = 3
        self.basis_p = 32 * torch.randn(freqs, 3).T
        self.skip = 3
        self.latent_size = 0
        dp = 2 * freqs + 3
        self.layers = nn.ModuleList([
            nn.Linear(hidden + dp if (i % 3) == 0 and i != num_layers - 1 else hidden, hidden)
            for i in range(num_layers)])
        self.init = nn.Linear(dp, hidden)
        self.out = nn.Linear(hidden, 1)

    def forward(self, p):
        proj = p @ self.basis_p
        enc = torch.cat([p, proj.sin(), proj.cos()], dim=-1)
        x = self.init(enc)
        for i, layer in enumerate(self.layers):
            if i != len(self.layers) - 1 and i % 3 == 0:
                x = torch.cat([x, enc], dim=-1)
            x = layer(F.softplus(x))
        return self.out(F.softplus(x))


class SphereSDF(nn.Module):
    """Scriptable stand-in with the reference SphereSDF's attributes (sdfs.py:16-44)."""

    def __init__(self, n: int):
        super().__init__()
        self.centers = nn.Parameter(0.3 * torch.rand(n, 3) - 0.15)
        self.radii = nn.Parameter(0.2 * torch.rand(n) - 0.1)
        self.tfs = nn.Parameter(0.01 * torch.randn(n, 3, 3))
        self.shift = _ScriptMLP(8, 128, 32)

    def forward(self, p):
        q = p.reshape(-1, 1, 3) - self.centers.unsqueeze(0)
        sd = q.norm(p=2, dim=-1) - self.radii.unsqueeze(0)
        return -torch.logsumexp(-32 * sd, dim=-1) / 32 + self.shift(p.reshape(-1, 3)).squeeze(-1)


def test_torchscript_sphere_sdf(tmp_path):
    torch.manual_seed(2)
    ref = SphereSDF(16)
    torch.jit.save(torch.jit.script(ref), str(tmp_path / "sdf.pt"))
    mine = model_io.load(str(tmp_path / "sdf.pt"), device="cpu")
    from neural_raytracing_amd.pathtracer.shapes import SphereSDF as Mine
    assert isinstance(mine, Mine)
    for name in ("centers", "radii", "tfs"):
        assert torch.equal(getattr(mine, name).detach(), getattr(ref, name).detach())
    _assert_mlp(mine.shift, ref.shift)
    assert mine.shift.activation is F.softplus


def test_loader_runs_nothing_from_the_file(tmp_path, ref_paths):
    """A pickle that would call os.system on load only yields an inert record here."""
    class Evil:
        def __reduce__(self):
            import os
            return (os.system, ("echo should-not-run > " + str(tmp_path / "ran"),))
    torch.save({"x": Evil()}, tmp_path / "evil.pt")
    obj = model_io.read_archive(str(tmp_path / "evil.pt"))
    assert isinstance(obj["x"], model_io.Foreign)
    assert not (tmp_path / "ran").exists()
    with pytest.raises(ValueError):
        model_io.to_module(obj["x"])


class _WritesAFile:
    """A crafted pickle whose reduce calls the package's save_image (a side-effecting function)."""

    def __init__(self, path):
        self.path = path

    def __reduce__(self):
        from neural_raytracing_amd.pathtracer.utils import save_image
        return save_image, (self.path, torch.zeros(2, 2, 3))


def test_weights_only_load_rejects_package_functions(tmp_path):
    """the weights_only allow-list holds the package's module classes only -- a
    pickle that calls utils.save_image must be refused, and no file written."""
    import pytorch3d  # noqa: F401  -- registers the allow-list
    from pytorch3d import safe_global_entries
    from neural_raytracing_amd.pathtracer import utils
    listed = [e[0] if isinstance(e, tuple) else e for e in safe_global_entries()]
    assert utils.save_image not in listed
    pure = {"_leaky", "identity", "identity_div_pi"}
    assert all(isinstance(e, type) or getattr(e, "__module__", "").startswith("torch")
               or e.__name__ in pure for e in listed)
    target = tmp_path / "pwned.png"
    f = tmp_path / "evil.pt"
    torch.save(_WritesAFile(str(target)), f)
    with pytest.raises(Exception):
        torch.load(f, weights_only=True)
    assert not target.exists()
