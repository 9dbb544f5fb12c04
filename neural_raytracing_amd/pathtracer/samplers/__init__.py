from .samplers import Sampler  # noqa: F401
