from .shapes import Shape, Sphere, SphereCloud  # noqa: F401
from .nerf import NeRFLE, PlainNeRF  # noqa: F401
from .sdfs import SDF, SPHERE_SDF, CapsuleSDF, RoundBoxSDF, SphereSDF  # noqa: F401
