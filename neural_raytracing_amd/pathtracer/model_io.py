"""Loaders for the reference's saved models that execute nothing from the file.

The reference's drivers load a TorchScript ``SphereSDF`` / MLP SDF with ``torch.jit.load``
(nerf_synthetic.py:63, dtu.py:93) and whole pickled modules -- ``ComposeSpatialVarying``,
``NeuralBSDF``, ``LightField``, ``PointLights``, an occlusion ``SkipConnMLP`` -- with
``torch.load`` (nerf_synthetic.py:118-121, dtu.py:105-113, nerv.py:75-82).  Both formats are zip
archives holding a ``data.pkl`` pickle plus raw tensor storages.  ``load`` reads them with a
restricted unpickler: every class or function the pickle names is materialised as an inert
``Foreign`` record (its pickled state kept as data), only tensor-rebuild helpers, ``OrderedDict``,
dtypes and TorchScript list builders are resolved to real code, and nothing from the archive is
imported, called or compiled.  The records are then converted into this package's modules by
attribute name (the reference's attribute layout: ``init`` / ``layers`` / ``out`` / ``basis_p``,
``centers`` / ``radii`` / ``tfs`` / ``shift``, ``bsdfs`` / ``sp_var_fn``, ...).

    shape = model_io.load("models/lego_sdf.pt")         # replaces torch.jit.load(...)
    bsdf = model_io.load("models/lego_bsdf.pt")          # replaces torch.load(...)
"""
import collections
import io
import pickle
import zipfile

import torch
import torch.nn as nn
import torch.nn.functional as F

__all__ = ["load", "read_archive", "to_module", "Foreign"]


class Foreign:
    """An object of a class (or a function) named by the pickle, kept as inert data."""
    qualname = "?"

    def __init__(self, *args, **kwargs):
        self.args = args
        self.state = {}

    def __setstate__(self, state):
        if isinstance(state, tuple) and len(state) == 2 and isinstance(state[0], (dict, type(None))):
            merged = dict(state[0] or {})
            merged.update(state[1] or {})
            state = merged
        self.state = state if isinstance(state, dict) else {"__state__": state}

    @property
    def short(self):
        return self.qualname.rsplit(".", 1)[-1]

    def get(self, name, default=None):
        st = self.state
        if name in st:
            return st[name]
        for sub in ("_parameters", "_buffers", "_modules"):
            d = st.get(sub)
            if isinstance(d, dict) and name in d:
                return d[name]
        return default

    def __repr__(self):
        return f"<Foreign {self.qualname}>"


_FOREIGN = {}


def _foreign(module, name):
    key = f"{module}.{name}"
    cls = _FOREIGN.get(key)
    if cls is None:
        cls = type(name, (Foreign,), {"qualname": key})
        _FOREIGN[key] = cls
    return cls


class _StorageType:
    def __init__(self, dtype):
        self.dtype = dtype


_STORAGE_DTYPES = {
    "FloatStorage": torch.float32, "DoubleStorage": torch.float64, "HalfStorage": torch.float16,
    "BFloat16Storage": torch.bfloat16, "LongStorage": torch.int64, "IntStorage": torch.int32,
    "ShortStorage": torch.int16, "CharStorage": torch.int8, "ByteStorage": torch.uint8,
    "BoolStorage": torch.bool, "UntypedStorage": torch.uint8,
}


def _rebuild_tensor_v2(storage, offset, size, stride, requires_grad=False, hooks=None,
                       metadata=None):
    t = torch.as_strided(storage, tuple(size), tuple(stride), offset).clone()
    t.requires_grad_(bool(requires_grad) and t.is_floating_point())
    return t


def _rebuild_parameter(data, requires_grad=True, hooks=None, state=None):
    return nn.Parameter(data, requires_grad=bool(requires_grad))


def _tag(value, *unused):
    return value


_ALLOWED = {
    ("torch._utils", "_rebuild_tensor_v2"): _rebuild_tensor_v2,
    ("torch._utils", "_rebuild_parameter"): _rebuild_parameter,
    ("torch._utils", "_rebuild_parameter_with_state"): _rebuild_parameter,
    ("collections", "OrderedDict"): collections.OrderedDict,
    ("torch", "device"): torch.device,
    ("torch", "Size"): torch.Size,
    ("torch.jit._pickle", "build_intlist"): list,
    ("torch.jit._pickle", "build_doublelist"): list,
    ("torch.jit._pickle", "build_boollist"): list,
    ("torch.jit._pickle", "build_tensorlist"): list,
    ("torch.jit._pickle", "restore_type_tag"): _tag,
}


class _Unpickler(pickle.Unpickler):
    def __init__(self, fh, zf, prefix):
        super().__init__(fh)
        self.zf, self.prefix = zf, prefix

    def find_class(self, module, name):
        fn = _ALLOWED.get((module, name))
        if fn is not None:
            return fn
        if module in ("torch", "torch.storage") and name in _STORAGE_DTYPES:
            return _StorageType(_STORAGE_DTYPES[name])
        if module == "torch" and isinstance(getattr(torch, name, None), torch.dtype):
            return getattr(torch, name)
        return _foreign(module, name)

    def persistent_load(self, pid):
        if not (isinstance(pid, tuple) and pid and pid[0] == "storage"):
            raise pickle.UnpicklingError(f"unsupported persistent id {pid!r}")
        _, stype, key, _location, _numel = pid[:5]
        dtype = stype.dtype if isinstance(stype, _StorageType) else torch.uint8
        raw = self.zf.read(f"{self.prefix}/data/{key}")
        if not raw:
            return torch.empty(0, dtype=dtype)
        return torch.frombuffer(bytearray(raw), dtype=dtype)


def read_archive(path):
    """The object tree of a torch.save / torch.jit.save zip archive (Foreign records, tensors,
    plain Python values)."""
    if not zipfile.is_zipfile(path):
        raise ValueError(f"{path}: not a zip-format torch archive (legacy pickles are not read)")
    with zipfile.ZipFile(path) as zf:
        names = [n for n in zf.namelist() if n.endswith("/data.pkl")]
        if not names:
            raise ValueError(f"{path}: no data.pkl in the archive")
        name = min(names, key=len)
        prefix = name[: -len("/data.pkl")]
        return _Unpickler(io.BytesIO(zf.read(name)), zf, prefix).load()


# ------------------------------------------------------------------------------------------
# record -> module conversion
# ------------------------------------------------------------------------------------------

def _linear(rec):
    return rec.get("weight"), rec.get("bias")


def _seq(mods):
    """Items of a pickled list / tuple / nn.ModuleList / nn.Sequential record."""
    if isinstance(mods, Foreign):
        items = mods.state.get("_modules")
        if isinstance(items, dict):
            return [items[k] for k in sorted(items, key=int)]
        return [mods.state[k] for k in sorted((k for k in mods.state if k.isdigit()), key=int)]
    return list(mods or [])


def _layers(rec):
    return _seq(rec.get("layers"))


def _activation(obj, default):
    from .bsdf import bsdfs as B
    if obj is None:
        return default
    name = obj.qualname if isinstance(obj, (Foreign, type)) and hasattr(obj, "qualname") else ""
    short = name.rsplit(".", 1)[-1]
    if isinstance(obj, Foreign) and short == "getattr" and len(obj.args) == 2:
        short = str(obj.args[1])  # builtins resolved by attribute, e.g. torch.sigmoid
        name = f"getattr(..., {short!r})"
    if isinstance(obj, Foreign):
        st = obj.state
        if short == "Softplus":
            return nn.Softplus(beta=st.get("beta", 1), threshold=st.get("threshold", 20))
        if short == "Sigmoid":
            return nn.Sigmoid()
        if short == "LeakyReLU":
            return nn.LeakyReLU(st.get("negative_slope", 0.01))
        if short == "ReLU":
            return nn.ReLU()
    table = {"softplus": F.softplus, "sigmoid": torch.sigmoid, "leaky_relu": F.leaky_relu,
             "relu": F.relu, "identity": B.identity, "identity_div_pi": B.identity_div_pi}
    if short in table:
        return table[short]
    raise ValueError(f"unsupported activation {name or obj!r} in the saved model")


def skip_conn_mlp(rec, device="cuda", activation=None):
    """SkipConnMLP (neural_blocks.py:12-86) from a record of one."""
    from .neural_blocks import SkipConnMLP
    init_w, init_b = _linear(rec.get("init"))
    out_w, _ = _linear(rec.get("out"))
    layers = _layers(rec)
    basis = rec.get("basis_p")
    in_size = int(rec.get("in_size", basis.shape[0]))
    latent = int(rec.get("latent_size", 0) or 0)
    act = activation if activation is not None else _activation(rec.get("activation"), None)
    kw = {} if act is None else {"activation": act}
    m = SkipConnMLP(num_layers=len(layers), hidden_size=init_w.shape[0], in_size=in_size,
                    out=out_w.shape[0], skip=int(rec.get("skip", 3)), freqs=basis.shape[1],
                    latent_size=latent, device="cpu", **kw)
    with torch.no_grad():
        m.basis_p = basis.detach().float().clone()
        for dst, src in zip(m._linears(), [rec.get("init"), *layers, rec.get("out")]):
            w, b = _linear(src)
            if dst.weight.shape != w.shape:
                raise ValueError(f"SkipConnMLP layer shape {tuple(w.shape)} != {tuple(dst.weight.shape)}")
            dst.weight.copy_(w)
            dst.bias.copy_(b)
    return m.to(device)


def sphere_sdf(rec, device="cuda"):
    """SphereSDF (sdfs.py:16-44): centres, radii, tfs and the softplus shift MLP."""
    from .shapes import SphereSDF
    centers = rec.get("centers")
    s = SphereSDF(n=centers.shape[0], device="cpu")
    with torch.no_grad():
        s.centers.copy_(centers)
        s.radii.copy_(rec.get("radii"))
        s.tfs.copy_(rec.get("tfs"))
    s.shift = skip_conn_mlp(rec.get("shift"), "cpu", activation=F.softplus)
    return s.to(device)


def _param(v, device):
    return v.detach().float().clone().to(device).requires_grad_(True)


def neural_bsdf(rec, device="cuda"):
    from .bsdf import NeuralBSDF
    b = NeuralBSDF(activation=_activation(rec.get("act"), torch.sigmoid), device="cpu")
    b.mlp = skip_conn_mlp(rec.get("mlp"), device)
    return b


def diffuse(rec, device="cuda"):
    from .bsdf import Diffuse
    from .bsdf import bsdfs as B
    d = Diffuse(preprocess=_activation(rec.get("preproc"), B.identity_div_pi), device=device)
    d.reflectance = _param(rec.get("reflectance"), device)
    return d


def conductor(rec, device="cuda"):
    from .bsdf import Conductor
    c = Conductor(activation=_activation(rec.get("act"), torch.sigmoid), device=device)
    c.specular = _param(rec.get("specular"), device)
    c.eta = _param(rec.get("eta"), "cpu")
    c.k = _param(rec.get("k"), "cpu")
    return c


def compose_spatial_varying(rec, device="cuda"):
    from .bsdf import ComposeSpatialVarying
    parts = [to_module(p, device) for p in _seq(rec.get("bsdfs"))]
    spatial = skip_conn_mlp(rec.get("sp_var_fn"), device)
    return ComposeSpatialVarying(parts, spatial_varying_fn=spatial, device=device)


def light_field(rec, device="cuda"):
    from .lights import LightField
    lf = LightField(device="cpu")
    lf.light_field_approx = skip_conn_mlp(rec.get("light_field_approx"), "cpu")
    with torch.no_grad():
        lf.color.copy_(rec.get("color"))
    return lf.to(device)


def point_lights(rec, device="cuda"):
    from .lights import PointLights
    loc = rec.get("location").detach().float().to(device)
    inten = rec.get("intensity").detach().float().to(device)
    return PointLights(intensity=inten, location=loc, const=float(rec.get("const")),
                       linear=float(rec.get("linear")), square=float(rec.get("square")),
                       scale=float(rec.get("scale")), device=device)


_CONVERT = {
    "SkipConnMLP": skip_conn_mlp, "SphereSDF": sphere_sdf, "NeuralBSDF": neural_bsdf,
    "Diffuse": diffuse, "Conductor": conductor, "ComposeSpatialVarying": compose_spatial_varying,
    "LightField": light_field, "PointLights": point_lights,
}


def to_module(rec, device="cuda"):
    """Convert a Foreign record of a reference class into this package's module."""
    if not isinstance(rec, Foreign):
        raise ValueError(f"expected a saved module, got {type(rec).__name__}")
    fn = _CONVERT.get(rec.short)
    if fn is None:
        raise ValueError(f"no converter for {rec.qualname} (supported: {sorted(_CONVERT)})")
    return fn(rec, device)


def load(path, device="cuda"):
    """Load a reference model file (TorchScript or pickled module) without executing it."""
    return to_module(read_archive(path), device)


jit_load = load
