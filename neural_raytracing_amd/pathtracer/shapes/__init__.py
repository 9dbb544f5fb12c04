from .nerf import NeRFLE  # noqa: F401
from .sdfs import SDF, SPHERE_SDF, SphereSDF  # noqa: F401
