"""Typed configuration presets (the reference has module constants only).

* ``reference`` — the parameters the reference actually runs with
  (``Barra-master/demo.py:38-42``: NW q=2 tau=252, eigen M=100 scale 1.4, VRA tau=42;
  ``Barra_factor_cal/config.py``: descriptor windows / composites / orthogonalisation) and its
  quirks (``compat`` flags);
* ``use4s`` / ``use4l`` — USE4 short/long-horizon half-lives (MSCI USE4 methodology,
  Table 4.1: vol HL 84 / 252, NW lags 5 / 2 ... VRA HL 42 / 168).  Only fields that exist in the
  reference's model are exposed (no separate correlation half-life: quirk Q11).
"""
from __future__ import annotations

from dataclasses import asdict, dataclass, field, replace


@dataclass(frozen=True)
class RiskConfig:
    nw_lags: int = 2              # MFM.Newey_West_by_time(q=2)
    nw_half_life: float = 252.0   # tao=252
    eigen_sims: int = 100         # eigen_risk_adj_by_time(M=100)
    eigen_scale: float = 1.4      # scale_coef=1.4
    eigen_sim_length: int | None = None  # None = total #dates for every date (quirk Q9)
    eigen_seed: int = 1
    vra_half_life: float = 42.0   # demo.py:42 (MFM default is 84)
    pivot_mode: int = 0           # 0 = last non-empty industry; 1 = reference (quirk Q3)
    psd_tol: float = 0.0          # eigen adj requires D0 >= -psd_tol*max|D0| (reference: 0)
    vra_out_of_sample: bool = False  # True: B_t uses the forecast of t-1 (reference: in-sample, Q10)
    eigen_shard: str = "dates"    # "dates": each rank adjusts its own dates with all M sims;
                                  # "sims": ranks split the M sims of every date + all_reduce (C5)
    eigen_chunk: int = 256        # sims per launch in "sims" mode (bounds the [D, chunk, K] buffer)
    deterministic: bool | None = None  # bitwise-reproducible CS-WLS kernel (wave-owned LDS
                                       # replicas); None = whenever supported
                                       # (mfa_xs_det_supported: P <= 57 at Q = 10)
    time_scan: str = "gather"     # time-axis stages (Newey-West, VRA) across date shards:
                                  # "gather": all-gather the O(T K) series, every rank scans the
                                  # prefix (bitwise identical to one GPU); "carry": each rank
                                  # scans only its dates from carried-in block states (SURVEY
                                  # 2.5 SP design, O(T/world), equal to one GPU to ~1e-13)

    def __post_init__(self):
        if self.eigen_shard not in ("dates", "sims"):
            raise ValueError(f"eigen_shard must be 'dates' or 'sims', got {self.eigen_shard!r}")
        if self.time_scan not in ("gather", "carry"):
            raise ValueError(f"time_scan must be 'gather' or 'carry', got {self.time_scan!r}")

    def to_dict(self) -> dict:
        return asdict(self)


@dataclass(frozen=True)
class FactorConfig:
    """Descriptor windows (Barra_factor_cal/factor_calculator.py) and post-processing rules."""
    beta_window: int = 252
    beta_half_life: float = 63.0
    beta_min_periods: int = 42
    rstr_window: int = 504
    rstr_lag: int = 21
    rstr_half_life: float = 126.0
    rstr_min_periods: int = 42
    dastd_window: int = 252
    dastd_half_life: float = 42.0
    dastd_min_periods: int = 42
    cmra_window: int = 252
    cmra_partial: bool = False    # factor.py variant uses partial windows (quirk Q15)
    stom: tuple = (21, 15)
    stoq: tuple = (63, 42)
    stoa: tuple = (252, 126)
    winsor_n_std: float = 2.5
    composite: dict = field(default_factory=lambda: {
        "volatility": {"components": ["DASTD", "CMRA", "HSIGMA"], "weights": [0.7, 0.15, 0.15]},
        "leverage": {"components": ["MLEV", "DTOA", "BLEV"], "weights": [1 / 3, 1 / 3, 1 / 3]},
        "liquidity": {"components": ["STOM", "STOQ", "STOA"], "weights": [0.5, 0.25, 0.25]},
        "earnings": {"components": ["CETOP", "ETOP"], "weights": [0.5, 0.5]},
        "growth": {"components": ["YOYProfit", "YOYSales"], "weights": [0.5, 0.5]},
    })
    ortho: dict = field(default_factory=lambda: {
        "volatility": ["BETA", "SIZE"],
        "liquidity": ["SIZE"],
    })


PRESETS = {
    "reference": RiskConfig(),
    "use4s": RiskConfig(nw_lags=5, nw_half_life=84.0, vra_half_life=42.0),
    "use4l": RiskConfig(nw_lags=2, nw_half_life=252.0, vra_half_life=168.0),
    # BASELINE.json config 5: Newey-West + 10k-simulation eigen "bootstrap", sims over ranks
    "bootstrap10k": RiskConfig(eigen_sims=10_000, eigen_shard="sims"),
}


def preset(name: str = "reference", **overrides) -> RiskConfig:
    if name not in PRESETS:
        raise KeyError(f"unknown preset {name!r}; choose from {sorted(PRESETS)}")
    return replace(PRESETS[name], **overrides)
