from .cameras import (Camera, DTUCamera, FoVPerspectiveCameras, NeRFCamera,  # noqa: F401
                      OpenGLPerspectiveCameras, look_at_view_transform)
