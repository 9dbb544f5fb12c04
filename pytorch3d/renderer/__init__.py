"""``pytorch3d.renderer`` for the pathtracer drivers: the camera math they use (host float32, the
reference's op order; renderer/cameras.py:280-575, 1275-1422) and import-only stand-ins for the
mesh-renderer classes they import (out of scope: the rasterisers need pytorch3d._C).  PointLights
is the fork's light with its pathtracer sample_direction (renderer/lighting.py:221-304)."""
from neural_raytracing_amd.pathtracer.cameras import (FoVPerspectiveCameras,  # noqa: F401
                                                      OpenGLPerspectiveCameras, look_at_rotation,
                                                      look_at_view_transform)


class _MeshRendererPart:
    """A mesh / point renderer class: importable, not constructible here."""

    def __init__(self, *args, **kwargs):
        raise NotImplementedError(f"pytorch3d.renderer.{type(self).__name__} belongs to the "
                                  "mesh / point rasteriser (pytorch3d._C), which is out of scope; "
                                  "render with pytorch3d.pathtracer.pathtrace")


class MeshRasterizer(_MeshRendererPart):
    pass


class MeshRenderer(_MeshRendererPart):
    pass


class RasterizationSettings(_MeshRendererPart):
    pass


class HardPhongShader(_MeshRendererPart):
    pass


class SoftPhongShader(_MeshRendererPart):
    pass


# the fork's PointLights (renderer/lighting.py:221-304) with its sample_direction: the light the
# pathtracer's sphere_examples / sphere_render_bsdf use
from neural_raytracing_amd.pathtracer.lights import RendererPointLights as PointLights  # noqa: E402,F401
