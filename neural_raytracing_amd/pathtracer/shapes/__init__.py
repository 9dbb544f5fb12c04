from .sdfs import SDF, SPHERE_SDF, SphereSDF  # noqa: F401
