"""Risk-model checkpoints: stage artifacts + the O(T K) scan history needed to append dates.

The reference keeps everything in memory lists and re-runs from scratch (SURVEY.md §5,
"Checkpoint / resume").  Here a finished :class:`~..models.risk_model.RiskModel` exports

* the factor-return history ``F`` [T, K] (what the Newey-West prefix scan and the VRA bias
  series are built from — the scan re-runs over it in O(T K^2), microseconds on the GPU),
* the VRA bias series ``B2`` [T],
* per-date R^2 / solver status, the last covariances, the config and the date index,

and :meth:`RiskModel.resume` continues on a panel of NEW dates without re-regressing or
re-adjusting the old ones.  Files are written with ``torch.save`` of tensors, strings and
plain containers only, and read back with ``torch.load(weights_only=True)`` (nothing from the
file is executed).  A config hash guards against resuming with different parameters.

Only MODEL parameters take part in that guard.  Execution-only settings (how the same numbers
are computed: the time-axis scan mode, the deterministic kernel, how the eigen sims are sharded
and chunked) may differ between the saved run and the resumed one, since every mode gives the
same results (bitwise, or to ~1e-13 for ``time_scan``).  Format 1 (round-2 files) hashed the
whole config dict; such files still load: their hash is verified the old way, and fields they
predate take their defaults.
"""
from __future__ import annotations

import hashlib
import json
from pathlib import Path

import torch

FORMAT_VERSION = 2
READABLE_FORMATS = (1, 2)

# RiskConfig fields that choose HOW a result is computed, not WHAT is computed
EXEC_KEYS = frozenset({"time_scan", "deterministic", "eigen_chunk", "eigen_shard"})


def model_config(cfg: dict) -> dict:
    """The model-defining part of a config dict (execution-only keys removed)."""
    return {k: v for k, v in cfg.items() if k not in EXEC_KEYS}


def _sha(d: dict) -> str:
    return hashlib.sha256(json.dumps(d, sort_keys=True, default=str).encode()).hexdigest()[:16]


def config_hash(cfg: dict, format_version: int = FORMAT_VERSION) -> str:
    """Hash of a config dict as written by checkpoint format ``format_version`` (1: the whole
    dict; 2: its model keys only)."""
    return _sha(cfg if format_version == 1 else model_config(cfg))


def save_state(state: dict, path: str | Path) -> Path:
    path = Path(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    out = {k: (v.detach().cpu() if torch.is_tensor(v) else v) for k, v in state.items()}
    out["format_version"] = FORMAT_VERSION
    tmp = path.with_suffix(path.suffix + ".tmp")
    torch.save(out, tmp)
    tmp.replace(path)  # atomic: a crash never leaves a half-written checkpoint
    return path


def load_state(path: str | Path) -> dict:
    state = torch.load(Path(path), map_location="cpu", weights_only=True)
    if state.get("format_version") not in READABLE_FORMATS:
        raise ValueError(f"unsupported checkpoint format {state.get('format_version')!r}")
    return state
