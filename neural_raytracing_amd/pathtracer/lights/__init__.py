from .lights import (Constant, Light, LightField, PointLights,  # noqa: F401
                     RendererPointLights)
