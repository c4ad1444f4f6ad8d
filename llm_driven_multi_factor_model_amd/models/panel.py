"""Dense (date x stock) risk-model panel resident in device memory.

The reference keeps one long pandas frame and boolean-mask-selects every date
(``Barra-master/mfm/MFM.py:58``).  Here a panel is a set of dense device tensors:

* ``styles`` [D, Q, N] — style exposures, stocks contiguous per (date, style) so the
  regression kernel's loads are fully coalesced;
* ``cap``, ``ret`` [D, N] — capital (``circ_mv``) and t+1 return;
* ``ind`` [D, N] int16 — industry id in ``[0, P)``, ``-1`` where the stock is absent
  (ragged universes are masks, industries are ids — never one-hot columns).

``styles`` / ``cap`` / ``ret`` share one storage dtype: float64 (the reference's own input
precision: ``demo.py:21`` reads float64 CSV columns into ``CrossSection.reg``) or float32 (the
factor pipeline's downcast, ``load_data.py:18-21``).  Regression math is float64 either way.
At N = 5000, D = 2520 (10y all-A) an fp64 panel is 1.2 GB (fp32: 0.6 GB): trivially resident in
288 GB of HBM3E, so every stage runs batched over all dates of a rank's shard.
"""
from __future__ import annotations

from dataclasses import dataclass, field, replace

import numpy as np
import torch


@dataclass
class RiskPanel:
    styles: torch.Tensor          # [D, Q, N] f64 or f32
    cap: torch.Tensor             # [D, N]    same dtype
    ret: torch.Tensor             # [D, N]    same dtype
    ind: torch.Tensor | None      # [D, N] int16 or None (P == 0)
    P: int
    dates: np.ndarray             # [D] datetime64[ns]
    stocks: np.ndarray            # [N] object (ts_code)
    style_names: list[str] = field(default_factory=list)
    industry_names: list[str] = field(default_factory=list)
    date_offset: int = 0          # index of dates[0] in the global calendar (sharded panels)

    @property
    def D(self) -> int:
        return self.styles.shape[0]

    @property
    def Q(self) -> int:
        return self.styles.shape[1]

    @property
    def N(self) -> int:
        return self.styles.shape[2]

    @property
    def K(self) -> int:
        return 1 + self.P + self.Q

    @property
    def device(self) -> torch.device:
        return self.styles.device

    @property
    def dtype(self) -> torch.dtype:
        return self.styles.dtype

    def astype(self, dtype) -> "RiskPanel":
        """The same panel with styles / cap / ret stored in ``dtype``."""
        return replace(self, styles=self.styles.to(dtype), cap=self.cap.to(dtype),
                       ret=self.ret.to(dtype))

    @property
    def factor_names(self) -> list[str]:
        ind = self.industry_names or [f"ind{j}" for j in range(self.P)]
        sty = self.style_names or [f"style{q}" for q in range(self.Q)]
        return ["country", *ind, *sty]

    def to(self, device) -> "RiskPanel":
        return replace(self, styles=self.styles.to(device), cap=self.cap.to(device),
                       ret=self.ret.to(device),
                       ind=None if self.ind is None else self.ind.to(device))

    def slice_dates(self, a: int, b: int) -> "RiskPanel":
        return replace(self, styles=self.styles[a:b], cap=self.cap[a:b], ret=self.ret[a:b],
                       ind=None if self.ind is None else self.ind[a:b], dates=self.dates[a:b],
                       date_offset=self.date_offset + a)

    def valid(self) -> torch.Tensor:
        from ..ops.cross_section import valid_mask
        return valid_mask(self.styles, self.cap, self.ret, self.ind, self.P)

    def nbytes(self) -> int:
        e = self.styles.element_size()
        n = (self.styles.numel() + self.cap.numel() + self.ret.numel()) * e
        return n + (0 if self.ind is None else self.ind.numel() * 2)


def industry_order(ind: torch.Tensor, P: int) -> torch.Tensor:
    """Stock permutation that groups stocks by their modal industry over the panel's dates.

    SW-L1 membership of a stock changes rarely, so in this order almost every run of
    consecutive stocks shares one industry on every date.  The regression kernel then folds a
    whole run into the per-industry sums with one LDS atomic per run boundary instead of one
    per stock (csrc/xs_wls.hip, K1).  Stocks never assigned an industry go last; ties keep the
    original order (stable).
    """
    D, N = ind.shape
    if P <= 0:
        return torch.arange(N, device=ind.device)
    il = ind.long()
    ok = (il >= 0) & (il < P)
    counts = torch.zeros(N, P + 1, dtype=torch.int32, device=ind.device)
    idx = torch.where(ok, il, torch.full_like(il, P))                  # absent -> bucket P
    counts.scatter_add_(1, idx.T.contiguous(), torch.ones(N, D, dtype=torch.int32, device=ind.device))
    modal = counts[:, :P].argmax(1)
    modal = torch.where(counts[:, :P].sum(1) > 0, modal, torch.full_like(modal, P))
    key = modal * N + torch.arange(N, device=ind.device)
    return torch.argsort(key)


def order_by_industry(panel: "RiskPanel") -> "RiskPanel":
    """The same panel with its stock axis permuted by :func:`industry_order`.

    A pure layout change: every per-date regression result is identical up to the order of the
    stocks (``panel.stocks`` is permuted alongside, so stock labels stay attached).
    """
    if panel.ind is None:
        return panel
    perm = industry_order(panel.ind, panel.P)
    pc = perm.cpu().numpy()
    return replace(panel, styles=panel.styles[:, :, perm].contiguous(),
                   cap=panel.cap[:, perm].contiguous(), ret=panel.ret[:, perm].contiguous(),
                   ind=panel.ind[:, perm].contiguous(), stocks=np.asarray(panel.stocks)[pc])


def business_days(D: int, start: str = "2010-01-04") -> np.ndarray:
    return np.asarray(np.busday_offset(np.datetime64(start, "D"), np.arange(D), roll="forward"),
                      dtype="datetime64[ns]")


def synthetic_panel(D: int, N: int, P: int = 31, Q: int = 10, *, seed: int = 0,
                    device="cpu", missing_frac: float = 0.0, empty_industries: int = 0,
                    factor_vol: float = 0.01, noise_vol: float = 0.02,
                    return_truth: bool = False, dtype=torch.float32):
    """Synthetic Barra panel with planted factor returns (the reference ships no data).

    * caps log-normal (``circ_mv``-like, 10k CNY units), styles N(0,1) with a per-style offset,
      industries SW-L1-like with uneven sizes;
    * ``missing_frac`` of (date, stock) cells are absent (``ind = -1``, NaN exposures) to make
      universes ragged;
    * ``empty_industries`` industries are emptied on a subset of dates (rank-deficiency
      edge case of quirk Q3/Q4);
    * returns follow ``r = f_c + f_ind + sum_q z_q f_q + eps`` on the z-scored styles, so the
      regression should recover the planted ``f`` up to noise.

    ``dtype`` is the storage dtype of styles / cap / ret (float64 draws are not rounded
    through float32).  Generation runs on ``device`` (a 5000 x 2520 panel is generated on the
    GPU in milliseconds).
    """
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    dev = torch.device(device)
    styles = torch.randn(D, Q, N, generator=g, device=dev, dtype=dtype)
    styles += torch.linspace(-0.5, 0.5, Q, device=dev, dtype=dtype)[None, :, None]
    cap = torch.exp(torch.randn(D, N, generator=g, device=dev, dtype=dtype) * 1.2 + 13.0)
    if P > 0:
        # uneven industry sizes, stable per stock with occasional reclassification
        probs = torch.linspace(1.0, 3.0, P, device=dev)
        base = torch.multinomial(probs / probs.sum(), N, replacement=True, generator=g)
        ind = base[None, :].expand(D, N).clone()
        flip = torch.rand(D, N, generator=g, device=dev) < 0.002
        ind = torch.where(flip, torch.randint(0, P, (D, N), generator=g, device=dev), ind)
        ind = ind.to(torch.int16)
        if empty_industries > 0:
            nd = max(1, D // 4)
            for k in range(empty_industries):
                j = (k * 7 + 3) % P
                dsel = torch.arange(k % max(1, D - nd), min(D, k % max(1, D - nd) + nd), device=dev)
                sub = ind[dsel]
                ind[dsel] = torch.where(sub == j, torch.full_like(sub, (j + 1) % P), sub)
    else:
        ind = None
    K = 1 + P + Q
    f_true = torch.randn(D, K, generator=g, device=dev, dtype=torch.float64) * factor_vol
    if P > 0:
        # make the planted industry returns satisfy the cap-weighted neutrality constraint
        oh = torch.nn.functional.one_hot(ind.long(), P).double()
        s = (oh * cap.double()[..., None]).sum(1)
        fi = f_true[:, 1:1 + P]
        f_true[:, 1:1 + P] = fi - ((s * fi).sum(1) / s.sum(1))[:, None]
    z = styles.double()
    mu = (cap.double()[:, None, :] * z).sum(2) / cap.double().sum(1)[:, None]
    sig = z.reshape(D, -1).std(1, unbiased=False)
    zs = (z - mu[..., None]) / sig[:, None, None]
    r = f_true[:, :1] + (zs * f_true[:, 1 + P:, None]).sum(1)
    if P > 0:
        r = r + f_true[:, 1:1 + P].gather(1, ind.long())
    r = r + torch.randn(D, N, generator=g, device=dev, dtype=torch.float64) * noise_vol
    ret = r.to(dtype)
    if missing_frac > 0:
        miss = torch.rand(D, N, generator=g, device=dev) < missing_frac
        styles = styles.masked_fill(miss[:, None, :], float("nan"))
        ret = ret.masked_fill(miss, float("nan"))
        if ind is not None:
            ind = ind.masked_fill(miss, -1)
    panel = RiskPanel(
        styles=styles.contiguous(), cap=cap.contiguous(), ret=ret.contiguous(),
        ind=None if ind is None else ind.contiguous(), P=P, dates=business_days(D),
        stocks=np.array([f"{i:06d}.SZ" for i in range(N)], dtype=object),
        style_names=DEFAULT_STYLE_NAMES[:Q] if Q <= len(DEFAULT_STYLE_NAMES) else [f"style{q}" for q in range(Q)],
        industry_names=[f"ind{j:02d}" for j in range(P)])
    return (panel, f_true) if return_truth else panel


DEFAULT_STYLE_NAMES = [
    "size", "beta", "momentum", "residual_volatility", "non_linear_size",
    "book_to_price_ratio", "liquidity", "earnings_yield", "growth", "leverage",
]
