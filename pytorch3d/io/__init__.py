"""``pytorch3d.io`` names the drivers import (nerf_synthetic.py:8, dtu.py:9) but never call."""


def load_objs_as_meshes(*args, **kwargs):
    raise NotImplementedError("load_objs_as_meshes (pytorch3d.io, meshes) is out of scope for the "
                              "pathtracer render path")


def load_obj(*args, **kwargs):
    raise NotImplementedError("load_obj (pytorch3d.io, meshes) is out of scope for the pathtracer "
                              "render path")
