"""Compute ops: every GPU path is a hand-written gfx950 HIP kernel from ``csrc/``."""
from .cross_section import xs_wls, xs_wls_reference, XsResult  # noqa: F401
from .ew_scan import newey_west_series, newey_west_single, ew_prefix_mean  # noqa: F401
