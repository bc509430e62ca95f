"""cad_amd — MI355X-native (gfx950) camera-aware depth training step.

Drop-in for the hot path of RyoK3N/Camera-Aware-Neural-Networks-for-Few-View-Depth-Estimation:
BaselineUNet forward/backward, CombinedDepthLoss (SI + gradient matching + smoothness +
reprojection) with its backward, clip_grad_norm_ and Adam, data-parallel over RCCL.  All compute is
in libcad_hip.so (hand-written HIP for CDNA4) behind the C ABI in include/cad/cad.h.

The directory name is not a Python identifier; import it with `cad_pkg.load()` from the repo root
(it registers the package as `cad_amd`).
"""
from ._abi import LIB_PATH, CadError, header_functions, load as load_library  # noqa: F401


def __getattr__(name):
    # lazy: importing the package must not require torch / a GPU (CPU tests only check the ABI)
    if name in ("BaselineUNet", "IntrinsicsConditionedUNet", "RayConditionedUNet", "CombinedDepthLoss", "Adam",
                "Trainer", "Communicator", "save", "load", "clip_grad_norm_", "depth_metrics", "ray_directions", "camera_from_K",
                "ResNetUNet", "GeometryAwareNetwork", "LightweightGeometryNetwork"):
        from . import model
        return getattr(model, name)
    if name in ("BatchAssembler", "AugSampler", "SunRGBDDataset", "PrefetchLoader"):
        from . import batch
        return getattr(batch, name)
    raise AttributeError(name)
