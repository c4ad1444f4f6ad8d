"""MI355X-native Barra multi-factor risk engine (capabilities of Izumighj/LLM-Driven-Multi-factor-Model).

Layers (see SURVEY.md §1 / §7 of the repository):

* :mod:`.ops`       — hand-written gfx950 HIP kernels (+ float64 CPU reference paths);
* :mod:`.models`    — device-resident panels, the factor (descriptor) engine, post-processing
  and the risk model (cross-sectional WLS -> Newey-West -> eigen adjustment -> VRA);
* :mod:`.parallel`  — date-sharded data parallelism over RCCL (``torch.distributed``);
* :mod:`.utils`     — configuration presets, CSV/IO, logging, timing, checkpoints.

The reference-compatible APIs live in the top-level ``mfm`` and ``barra_factor_cal`` packages.
"""
__version__ = "0.1.0"

from .models.panel import RiskPanel, synthetic_panel  # noqa: E402,F401
