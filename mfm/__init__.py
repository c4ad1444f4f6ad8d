"""Drop-in replacement for the reference ``mfm`` package (Barra-master/mfm/__init__.py:11).

Same public names and pandas/numpy in-out contract (``CrossSection``, ``MFM``, ``utils``),
backed by the MI355X engine in :mod:`llm_driven_multi_factor_model_amd`.  Device selection:
``MFA_DEVICE`` env var (``cuda``/``cpu``), default ``cuda`` when a GPU is visible.
Set ``MFA_VERBOSE=1`` for the reference's per-date progress lines.
"""
from . import utils  # noqa: F401
from .CrossSection import CrossSection  # noqa: F401
from .MFM import MFM  # noqa: F401

__author__ = "llm_driven_multi_factor_model_amd"
__all__ = ["CrossSection", "utils", "MFM"]
