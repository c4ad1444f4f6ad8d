"""Model layer: panels, factor engine, post-processing and the risk model."""
from .panel import RiskPanel, synthetic_panel  # noqa: F401
