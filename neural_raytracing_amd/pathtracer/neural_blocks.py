"""SkipConnMLP with the reference's constructor (neural_blocks.py:12-86); forward runs on the
fused HIP kernel ``nrt_mlp_forward`` (one wavefront = 32 rows, every layer an MFMA GEMM).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _lib
from ._handles import mlp_handle
from .utils import create_fourier_basis2


def _leaky(x):
    return F.leaky_relu(x)


def activation_code(fn):
    """Map a torch activation callable to an NRT_ACT code (raises for anything else)."""
    if fn is None or fn is _leaky or fn is F.leaky_relu:
        return "leaky_relu"
    if isinstance(fn, nn.LeakyReLU) and fn.negative_slope == 0.01:
        return "leaky_relu"
    if fn is F.softplus or (isinstance(fn, nn.Softplus) and fn.beta == 1 and fn.threshold == 20):
        return "softplus"
    if fn in (F.relu, torch.relu) or isinstance(fn, nn.ReLU):
        return "relu"
    if fn in (torch.sigmoid, F.sigmoid) or isinstance(fn, nn.Sigmoid):
        return "sigmoid"
    name = getattr(fn, "__name__", type(fn).__name__)
    raise _lib.NrtError(f"activation {name!r} has no HIP implementation "
                        "(supported: leaky_relu(0.01), softplus, relu, sigmoid)")


class SkipConnMLP(nn.Module):
    """MLP with skip connections and Fourier encoding (neural_blocks.py:12-86).

    Construction consumes the RNG exactly like the reference: Fourier basis, the hidden
    ``nn.Linear`` list, ``init``, ``out``, then optional zero / xavier re-initialisation.
    """

    def __init__(self, num_layers=8, hidden_size=64, in_size=3, out=3, skip=3, freqs=16,
                 sigma=2 << 4, device="cuda", activation=_leaky, latent_size=0,
                 zero_init=False, xavier_init=False):
        super().__init__()
        self.in_size = in_size
        assert type(freqs) == int
        self.basis_p, map_size = create_fourier_basis2(freqs, features=in_size, freq=sigma,
                                                       device=device)
        self.dim_p = map_size + latent_size
        self.skip = skip
        self.latent_size = latent_size
        skip_size = hidden_size + self.dim_p
        self.layers = nn.ModuleList([
            nn.Linear(skip_size if (i % skip) == 0 and i != num_layers - 1 else hidden_size,
                      hidden_size)
            for i in range(num_layers)
        ])
        self.init = nn.Linear(self.dim_p, hidden_size)
        self.out = nn.Linear(hidden_size, out)
        ordered = [self.init, self.out, *self.layers]
        if zero_init:
            for lin in ordered:
                nn.init.zeros_(lin.weight)
            for lin in ordered:
                nn.init.zeros_(lin.bias)
        if xavier_init:
            for lin in ordered:
                nn.init.xavier_uniform_(lin.weight)
            for lin in ordered:
                nn.init.zeros_(lin.bias)
        self.activation = activation

    def _apply(self, fn, *args, **kwargs):
        # basis_p is a plain tensor attribute in the reference too; move it with the module
        out = super()._apply(fn, *args, **kwargs)
        self.basis_p = fn(self.basis_p)
        return out

    def _linears(self):
        return [self.init, *self.layers, self.out]

    def activation_code(self):
        return activation_code(self.activation)

    def nrt(self):
        return mlp_handle(self).value

    def forward(self, p, latent=None):
        if not p.is_cuda:
            raise _lib.NrtError("SkipConnMLP evaluates on the HIP path only: move it and its "
                                "inputs to the GPU")
        if torch.is_grad_enabled() and (p.requires_grad or any(q.requires_grad for q in self.parameters())):
            raise NotImplementedError(
                "backward through the fused MLP is not implemented yet (SURVEY §8f row 1); "
                "call under torch.no_grad()")
        batches = p.shape[:-1]
        x = p.reshape(-1, self.in_size).float().contiguous()
        lat = None
        if latent is not None:
            lat = latent.reshape(-1, self.latent_size).float().contiguous()
        y = torch.empty(x.shape[0], self.out.out_features, device=p.device)
        _lib.call("nrt_mlp_forward", self.nrt(), _lib.ptr(x), _lib.ptr(lat), x.shape[0],
                  _lib.ptr(y), _lib.precision_code(), _lib.stream())
        return y.reshape(batches + (self.out.out_features,))
