from .lights import Light, LightField, PointLights  # noqa: F401
