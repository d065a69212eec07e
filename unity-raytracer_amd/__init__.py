"""unity-raytracer_amd — MI355X-native (gfx950) per-pixel trace path of
vectorized-runner/unity-raytracer, behind the C-ABI in include/rt_mi355.h.

Import with ``_rt_pkg.load()`` from the repo root (the directory name has a
hyphen, so it is loaded under the module name ``unity_raytracer_amd``).
"""
from . import abi, bands, scene, scenes, raytracing  # noqa: F401
from .abi import load_library, RtError  # noqa: F401
from .scene import Scene, Mesh, MeshSource, MaterialData, TriangleData, SphereData  # noqa: F401
from .scenes import CameraData, ImagePlane, Frame, make  # noqa: F401
from .raytracing import Context, RayTracingSetup, params_struct, frame_params, pixel_dtype, write_ppm  # noqa: F401
