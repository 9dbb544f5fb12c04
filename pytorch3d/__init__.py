"""The ``pytorch3d`` import surface of the reference's drivers, on the MI355X path.

The reference is a fork of PyTorch3D 0.3.0 whose drivers (scripts/nerf_synthetic.py, dtu.py,
colocate.py, ...) import ``pytorch3d.pathtracer.*``, ``pytorch3d.renderer`` and ``pytorch3d.io``
(SURVEY §2b).  This package makes those imports resolve to this repository's implementation so
the scripts run unchanged:

* ``pytorch3d.pathtracer`` and every submodule (``pytorch3d.pathtracer.shapes.sdfs``,
  ``.bsdf.bsdfs``, ``.integrators``, ``.training_utils``, ...) ARE the modules of
  ``neural_raytracing_amd.pathtracer`` (registered under both names in ``sys.modules``), so
  pickles that name ``pytorch3d.pathtracer.bsdf.bsdfs.ComposeSpatialVarying`` resolve to the HIP
  classes;
* ``pytorch3d.renderer`` -- camera math (look_at_view_transform, look_at_rotation, FoV /
  OpenGL perspective cameras); the mesh renderer names the scripts import but never call
  (MeshRasterizer, MeshRenderer, RasterizationSettings, HardPhongShader, PointLights) exist and
  raise when constructed: the mesh / point rasterisers and ``pytorch3d._C`` are out of scope;
* ``pytorch3d.io.load_objs_as_meshes`` -- likewise imported but unused by the drivers.

Nothing here imports a compiled ``_C`` module, torchvision, pytorch_msssim or cv2.
"""
import importlib
import pkgutil
import sys

__version__ = "0.3.0"

_SRC = "neural_raytracing_amd.pathtracer"
_DST = __name__ + ".pathtracer"


def _alias_pathtracer():
    root = importlib.import_module(_SRC)
    sys.modules[_DST] = root
    for info in pkgutil.walk_packages(root.__path__, _SRC + "."):
        mod = importlib.import_module(info.name)
        alias = _DST + info.name[len(_SRC):]
        sys.modules.setdefault(alias, mod)
    return root


pathtracer = _alias_pathtracer()


def safe_global_entries():
    """The allow-list for torch's ``weights_only=True`` unpickler: exactly the module classes a
    driver pickle of a BSDF / light / SDF holds (dtu.py:100, :108 ``torch.load`` them), under
    this package's and the reference's module paths, plus the torch layers and the pure
    activation functions those modules keep as attributes (neural_blocks.py:26, sdfs.py:29).

    Only ``nn.Module`` subclasses are listed (the unpickler rebuilds them with ``__new__`` +
    ``__setstate__``, running none of their code) plus three pure element-wise activation
    functions, never another free function of the package: the
    weights_only unpickler calls any allow-listed callable with arguments the file chooses, so a
    function such as ``utils.save_image`` on the list would let a crafted ``.pt`` write files."""
    import inspect

    import torch
    import torch.nn as nn
    import torch.nn.functional as F
    entries = []
    for name, mod in list(sys.modules.items()):
        if not name.startswith(_SRC + "."):
            continue
        for attr, obj in vars(mod).items():
            if getattr(obj, "__module__", None) != mod.__name__:
                continue
            if inspect.isclass(obj) and issubclass(obj, nn.Module):
                alias = _DST + name[len(_SRC):] + "." + attr
                entries += [obj, (obj, alias)]
    # the package's pure element-wise functions that modules keep as attributes: SkipConnMLP's
    # default activation (neural_blocks.py:26) and the BSDF preprocessors (bsdfs.py:80-96)
    from neural_raytracing_amd.pathtracer import neural_blocks
    from neural_raytracing_amd.pathtracer.bsdf import bsdfs
    for fn, mod in ((neural_blocks._leaky, "neural_blocks"), (bsdfs.identity, "bsdf.bsdfs"),
                    (bsdfs.identity_div_pi, "bsdf.bsdfs")):
        entries += [fn, (fn, f"{_DST}.{mod}.{fn.__name__}")]
    entries += [nn.Linear, nn.ModuleList, nn.Sequential, nn.Softplus, nn.Sigmoid, nn.LeakyReLU,
                nn.ReLU, nn.Tanh, nn.Identity, nn.Parameter, F.softplus, F.leaky_relu, F.relu,
                torch.sigmoid, torch.relu, torch.tanh]
    return entries


def _register_safe_globals():
    """Registered process-wide at import (not only inside ``model_io.load``, which has its own
    restricted unpickler) because the drivers call ``torch.load`` themselves."""
    import torch
    try:
        torch.serialization.add_safe_globals(safe_global_entries())
    except Exception:  # noqa: BLE001 -- an older torch without the allow-list: nothing to do
        pass


_register_safe_globals()
