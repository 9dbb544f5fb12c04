from .cameras import (Camera, DTUCamera, FoVPerspectiveCameras, NeRFCamera,  # noqa: F401
                      NeRVCamera, OpenGLPerspectiveCameras, look_at_rotation,
                      look_at_view_transform)
