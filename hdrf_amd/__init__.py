"""hdrf_amd — MI355X-native backend for HDRF's per-block reduction path.

chunk (window-max CDC) -> SHA-1/SHA-224 fingerprint -> GPU index -> container store,
implemented as hand-written gfx950 HIP kernels behind the C-ABI in include/hdrf.h.
"""
from .lib import Config, Context, HdrfError, build, default_config, load  # noqa: F401
from .scheme import HipReductionScheme, ReductionScheme  # noqa: F401
