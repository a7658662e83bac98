"""MI355X-native batched NMPC SQP-RTI solve path (drop-in for the acados solve of
JorgeDFR/nmpc_nav_control). The compute lives in libnmpc_amd.so (HIP, gfx950); this package is the
host-side mirror of the reference's controller interface plus device-memory plumbing."""
from ._lib import LIB_PATH, MODEL_IDS, MODEL_NAMES, ModelParams, default_params, lib, model_dims  # noqa: F401

__version__ = "0.1.0"
