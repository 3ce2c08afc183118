"""transmvsnet_amd -- MI355X-native TransMVSNet depth-inference hot path.

    from transmvsnet_amd import TransMVSNet       # drop-in for models.TransMVSNet
    model = TransMVSNet().cuda().eval(); model.load_state_dict(sd, strict=True)
    outputs = model(imgs, proj_matrix, depth_values)

The hot path runs as hand-written gfx950 HIP kernels behind the C-ABI in
include/transmvs.h (libtransmvs_hip.so, built by ``python -m transmvsnet_amd.build``).
"""
from .model import TransMVSNet  # noqa: F401
from . import ops  # noqa: F401

__all__ = ["TransMVSNet", "ops"]
