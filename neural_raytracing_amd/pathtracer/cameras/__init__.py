from .cameras import Camera, DTUCamera, NeRFCamera  # noqa: F401
