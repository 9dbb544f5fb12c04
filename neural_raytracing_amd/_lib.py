"""ctypes binding of libnrt_hip.so (include/nrt.h).

The library is loaded lazily on first use, after torch (so the process has a single HIP
runtime: torch's libamdhip64.so.7 satisfies the library's NEEDED entry).  There is no CPU
fallback: any compute call without the library or without a gfx950 device raises.
"""
import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
# NRT_LIB: an alternative build of the same library (timing experiments, tools/exp_variants.sh)
LIB_PATH = os.environ.get("NRT_LIB") or os.path.join(HERE, "libnrt_hip.so")

NRT_FP32 = 0
NRT_FP16 = 1
NRT_FP32_SPLIT = 2
NRT_MIXED = 3
_PRECISIONS = {"fp32": NRT_FP32, "fp16": NRT_FP16, "fp32-split": NRT_FP32_SPLIT,
               "mixed": NRT_MIXED}

ACT = {"leaky_relu": 0, "softplus": 1, "none": 2, "sigmoid": 3, "relu": 4}

NRT_BSDF_NEURAL, NRT_BSDF_DIFFUSE, NRT_BSDF_CONDUCTOR = 0, 1, 2
NRT_CAM_NERF, NRT_CAM_DTU, NRT_CAM_FOV = 0, 1, 2


class NrtError(RuntimeError):
    pass


class MlpDesc(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in
                ("in_size", "hidden", "num_layers", "out", "freqs", "skip", "latent", "activation")]


class MarchParams(ctypes.Structure):
    _fields_ = [("max_steps", ctypes.c_int32), ("epsilon", ctypes.c_float),
                ("max_t", ctypes.c_float), ("primary", ctypes.c_int32),
                ("scan_max_t", ctypes.c_double), ("precision", ctypes.c_int32),
                ("scan_index", ctypes.c_void_p), ("scan_max_t_groups", ctypes.c_void_p),
                ("group_rays", ctypes.c_int64)]


class BsdfComponent(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("mlp", ctypes.c_void_p),
                ("activation", ctypes.c_int32), ("params", ctypes.c_float * 4)]


class Camera(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("size", ctypes.c_int32), ("focal", ctypes.c_float),
                ("mat", ctypes.c_float * 16), ("intrinsic", ctypes.c_float * 16),
                ("origin", ctypes.c_float * 3)]


_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_F = ctypes.c_float

_SIGNATURES = {
    "nrt_last_error": (ctypes.c_char_p, []),
    "nrt_version": (_I32, []),
    "nrt_device_ok": (_I32, []),
    "nrt_mlp_create": (_I32, [ctypes.POINTER(MlpDesc), _P, _P, _P, ctypes.POINTER(_P)]),
    "nrt_mlp_destroy": (_I32, [_P]),
    "nrt_mlp_refresh": (_I32, [_P, _P, _P, _P]),
    "nrt_mlp_forward": (_I32, [_P, _P, _P, _I64, _P, _I32, _P]),
    "nrt_mlp_forward_multi": (_I32, [_P, _I32, _P, _I64, _P, _P, _I32, _P]),
    "nrt_mlp_save_bytes": (ctypes.c_size_t, [_P, _I64]),
    "nrt_sdf_create_unit_sphere": (_I32, [ctypes.POINTER(_P)]),
    "nrt_sdf_create_mlp": (_I32, [_P, ctypes.POINTER(_P)]),
    "nrt_sdf_create_sphere_blob": (_I32, [_I32, _P, _P, _P, _F, _P, ctypes.POINTER(_P)]),
    "nrt_sdf_destroy": (_I32, [_P]),
    "nrt_sdf_refresh_spheres": (_I32, [_P, _P, _P, _P, _P]),
    "nrt_sphere_smoothmin_forward": (_I32, [_P, _I64, _P, _P, _P, _I32, _F, _P, _P, _P]),
    "nrt_sphere_smoothmin_workspace_bytes": (ctypes.c_size_t, [_I64]),
    "nrt_sphere_smoothmin_backward": (_I32, [_P, _I64, _P, _P, _P, _I32, _F, _P, _P, _P, _P, _P,
                                             _P, _P]),
    "nrt_sdf_eval": (_I32, [_P, _P, _I64, _P, _I32, _P]),
    "nrt_sdf_grad": (_I32, [_P, _P, _I64, _P, _P]),
    "nrt_intersect_workspace_bytes": (ctypes.c_size_t, [_P, _I64]),
    "nrt_sdf_intersect": (_I32, [_P, _P, _I64, ctypes.POINTER(MarchParams), _P, _P, _P, _P, _P,
                                 _P, _P, _P, _P, _P, _P]),
    "nrt_sdf_occlusion": (_I32, [_P, _P, _I64, _P, _I32, _F, _P, _I32, _P]),
    "nrt_march_callable_step": (_I32, [_P, _I64, _P, _F, _F, _I32, _P, _P, _P, _P, _P]),
    "nrt_scan_callable_step": (_I32, [_P, _I64, _P, _I32, ctypes.c_double, _I32, _P, _P, _P, _P]),
    "nrt_occlusion_callable_step": (_I32, [_P, _I64, _P, _F, _F, _P, _I32, _P, _P, _P, _P, _P]),
    "nrt_light_create_field": (_I32, [_P, _P, ctypes.POINTER(_P)]),
    "nrt_light_create_point": (_I32, [_P, _P, _F, _F, _F, _F, ctypes.POINTER(_P)]),
    "nrt_light_create_renderer_point": (_I32, [_P, _P, _F, ctypes.POINTER(_P)]),
    "nrt_light_destroy": (_I32, [_P]),
    "nrt_sphere_intersect": (_I32, [_P, ctypes.c_double, _P, _I64, _P, _P, _P, _P, _P, _P, _P, _P]),
    "nrt_sphere_cloud_intersect": (_I32, [_P, _I64, _I64, ctypes.c_double, _P, _I64, _P, _P, _P, _P,
                                          _P, _P, _P]),
    "nrt_bsdf_create": (_I32, [_I32, _P, _P, ctypes.POINTER(_P)]),
    "nrt_bsdf_destroy": (_I32, [_P]),
    "nrt_shade_direct": (_I32, [_P, _P, _P, _P, _P, _P, _P, _I64, _P, _P, _I32, _P]),
    "nrt_shadow_workspace_bytes": (ctypes.c_size_t, [_I64]),
    "nrt_shade_direct_shadowed": (_I32, [_P, _P, _P, _I32, _F, _P, _P, _P, _P, _P, _I64, _P, _P,
                                         _P, _P, _I32, _P]),
    "nrt_shade_direct_learned_occ": (_I32, [_P, _P, _P, _P, _I32, _F, _P, _P, _P, _P, _P, _I64,
                                            _P, _P, _P, _P, _I32, _P]),
    "nrt_raygen": (_I32, [_P, _I32, _I32, _I32, _I32, _I32, _F, _P, _P, _P, _P]),
    "nrt_path_workspace_bytes": (ctypes.c_size_t, [_I64]),
    "nrt_path_bounce": (_I32, [_P, _P, _P, _I32, _P, _I32, _F, _P, _P, _P, _I64, _P, _P, _P, _P, _P,
                               _P, _P, _I32, _P]),
    "nrt_render_tile_workspace_bytes": (ctypes.c_size_t, [_P, _I32, _I32, _I32]),
    "nrt_render_tile": (_I32, [_P, _I32, _I32, _I32, _I32, _I32, _F, _P, _P,
                               ctypes.POINTER(MarchParams), _P, _P, _I32, _F, _P, _I32, _I32, _I32,
                               _I32, _I32, _P, _P]),
    "nrt_nerfle_workspace_bytes": (ctypes.c_size_t, [_I64, _I32, _I32]),
    "nrt_nerfle_workspace_bytes_for": (ctypes.c_size_t, [_P, _P, _I64, _I32, _I32, _I32]),
    "nrt_nerfle_forward": (_I32, [_P, _P, _P, _I64, _P, _I32, _P, _I32, _P, _P, _I32, _P]),
    "nrt_light_envmap": (_I32, [_P, _I32, _P, _P]),
    "nrt_plain_nerf_workspace_bytes": (ctypes.c_size_t, [_P, _P, _I64, _I32]),
    "nrt_plain_nerf_forward": (_I32, [_P, _P, _P, _I64, _P, _I32, _P, _I64, _P, _P, _P, _I32, _P]),
    "nrt_mlp_backward_workspace_bytes": (ctypes.c_size_t, [_P, _I64]),
    "nrt_mlp_backward": (_I32, [_P, _P, _P, _I64, _P, _P, _P, _P, _P, _P, _P]),
    "nrt_mlp_backward_multi_workspace_bytes": (ctypes.c_size_t, [_P, _I32, _I64]),
    "nrt_mlp_backward_multi": (_I32, [_P, _I32, _P, _I64, _P, _P, _P, _P, _P, _P]),
    "nrt_mlp_backward_saved": (_I32, [_P, _I32, _P, _I64, _P, _P, _I64, _P, _P, _P, _P, _P, _P]),
    "nrt_mlp_grad_backward_workspace_bytes": (ctypes.c_size_t, [_P, _I64]),
    "nrt_mlp_grad_backward": (_I32, [_P, _P, _P, _I64, _P, _P, _P, _P, _P]),
    "nrt_frames": (_I32, [_P, _P, _I64, _P, _P, _P]),
    "nrt_profile_enable": (None, [_I32]),
    "nrt_profile_reset": (None, []),
    "nrt_profile_read": (_I32, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_double),
                                ctypes.POINTER(_I64)]),
    "nrt_profile_evals": (_I32, [ctypes.POINTER(ctypes.c_uint64)]),
    "nrt_profile_refined": (_I32, [ctypes.POINTER(ctypes.c_uint64)]),
    "nrt_profile_flop": (_I32, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_double)]),
    "nrt_set_option": (_I32, [ctypes.c_char_p, _I64]),
    "nrt_get_option": (_I32, [ctypes.c_char_p, ctypes.POINTER(_I64)]),
    "nrt_reset_options": (_I32, []),
    "nrt_composite": (_I32, [_P, _P, _P, _I32, _I32, _I32, _I32, _I32, _F, _P, _I32, _I32, _I32,
                             _I32, _I32, _P]),
}

_lib = None


def exported_symbols():
    return list(_SIGNATURES)


def load(require_device=False):
    """Load the library (once).  Raises NrtError if it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NrtError(f"{LIB_PATH} not built: run __graft_entry__.build() or "
                           "python -m neural_raytracing_amd.build")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    if require_device and not torch.cuda.is_available():
        raise NrtError("the HIP render path needs a gfx950 GPU (torch.cuda.is_available() is False)")
    return _lib


def check(rc, what=""):
    if rc != 0:
        msg = _lib.nrt_last_error().decode() if _lib is not None else ""
        raise NrtError(f"{what} failed ({rc}): {msg}")


def call(name, *args):
    lib = load(require_device=True)
    check(getattr(lib, name)(*args), name)


def ptr(t):
    """Raw device pointer of a contiguous tensor (None -> NULL)."""
    if t is None:
        return None
    if not t.is_contiguous():
        raise NrtError("tensor passed to the HIP library must be contiguous")
    return ctypes.c_void_p(t.data_ptr())


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


# ---------------------------------------------------------------------------------------------
# precision
# ---------------------------------------------------------------------------------------------
# NRT_PRECISION (fp32 | fp16 | fp32-split | mixed) picks the process-wide default; set_precision
# overrides it
_precision = {"value": _PRECISIONS.get(os.environ.get("NRT_PRECISION", "fp32"), NRT_FP32)}


def set_precision(p):
    """'fp32' (exact-f32 MFMA, parity with the reference), 'fp16' (f16 MFMA, f32 accumulate) or
    'fp32-split' ('fp32', with the SDF march + scan at FP32 accuracy on FP16 MFMA: every operand
    split into two f16 halves, three products; include/nrt.h NRT_FP32_SPLIT) or 'mixed'
    ('fp32-split', with the SDF march + scan at FP16 and every decision FP16 cannot make --
    a hit / max_t test near its threshold, a scan argmin between near-equal values -- taken
    again at FP32 accuracy; include/nrt.h NRT_MIXED)."""
    if p not in _PRECISIONS:
        raise ValueError(f"precision must be one of {sorted(_PRECISIONS)}")
    _precision["value"] = _PRECISIONS[p]


def get_precision():
    return {v: k for k, v in _PRECISIONS.items()}[_precision["value"]]


def precision_code():
    return _precision["value"]


def set_option(name, value):
    """nrt_set_option (include/nrt.h "Runtime options"): select an implementation or schedule."""
    check(load().nrt_set_option(name.encode(), int(value)), f"nrt_set_option({name})")


def get_option(name):
    v = ctypes.c_int64()
    check(load().nrt_get_option(name.encode(), ctypes.byref(v)), f"nrt_get_option({name})")
    return v.value


class options:
    """Context manager: ``with _lib.options(ring32=0): ...`` sets options and restores them."""

    def __init__(self, **kw):
        self.kw = kw
        self.old = {}

    def __enter__(self):
        for k, v in self.kw.items():
            self.old[k] = get_option(k)
            set_option(k, v)
        return self

    def __exit__(self, *exc):
        for k, v in self.old.items():
            set_option(k, v)
        return False


def profile_enable(on=True, evals=False):
    """HIP-event timing of the profiled launches (on); evals=True also counts the ring marches'
    SDF evaluations (a device atomic per wave-evaluation: keep it out of timed regions)."""
    load().nrt_profile_enable((1 if on else 0) | (2 if evals else 0))


def profile_reset():
    load().nrt_profile_reset()


def profile_evals():
    """SDF evaluations (ray x point) the ring marches executed since the last reset while profiling
    was enabled: the executed work behind an algorithmic FLOP count."""
    v = ctypes.c_uint64()
    check(load().nrt_profile_evals(ctypes.byref(v)), "nrt_profile_evals")
    return v.value


def profile_refined():
    """Rays the NRT_MIXED refinement re-marched (flagged by the FP16 march) since the last reset
    while evaluation counting was enabled."""
    v = ctypes.c_uint64()
    check(load().nrt_profile_refined(ctypes.byref(v)), "nrt_profile_refined")
    return v.value


def profile_read(name):
    """(total_ms, launches) of kernel `name` since the last reset (synchronises its events)."""
    tot = ctypes.c_double()
    n = ctypes.c_int64()
    check(load().nrt_profile_read(name.encode(), ctypes.byref(tot), ctypes.byref(n)),
          "nrt_profile_read")
    return tot.value, n.value


def profile_flop(name):
    """Algorithmic FLOP the library recorded for the timed launches of kernel `name` since the
    last reset (the training path's MLP backward / weight-gradient launches; 0 for others)."""
    v = ctypes.c_double()
    check(load().nrt_profile_flop(name.encode(), ctypes.byref(v)), "nrt_profile_flop")
    return v.value
