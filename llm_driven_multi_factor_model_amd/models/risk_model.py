"""Tensor-native Barra risk model: CS-WLS factor returns -> Newey-West -> eigen adjustment -> VRA.

Equivalent of ``Barra-master/mfm/MFM.py`` (``reg_by_time`` :48-76, ``Newey_West_by_time``
:80-101, ``eigen_risk_adj_by_time`` :105-126, ``vol_regime_adj_by_time`` :130-167) and the
diagnostics of ``mfm/utils.py`` (``eigenfactor_bias_stat`` :97-117, ``bayes_shrink`` :153-168),
re-designed for MI355X:

* no per-date Python loop: every stage is one batched launch over all dates of the shard;
* data-parallel over dates: a ``RiskPanel`` shard with ``date_offset`` runs on each rank; the
  factor-return series is all-gathered once (RCCL) and the Newey-West scan emits only the
  rank's own dates; the eigen adjustment of a date needs only that date's covariance; the VRA
  bias series is all-gathered once;
* outputs stay on the device as float64 tensors; pandas objects are built only on request;
* every stage is traced (ROCTX range, HIP-event GPU time, JSONL metrics: utils/trace.py);
* checkpoint / resume: :meth:`RiskModel.state_dict` exports the O(T K) history the scans need and
  :meth:`RiskModel.resume` appends new dates without re-running the old ones (utils/checkpoint.py).
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops import cross_section as xs
from ..ops import ew_scan, eigen
from ..parallel import dist as pdist
from ..utils import checkpoint as ckpt
from ..utils import trace
from ..utils.config import RiskConfig
from .panel import RiskPanel


class RiskModel:
    """Barra risk model over a (possibly date-sharded) panel.

    Attributes after the stages run (rank-local date block unless stated):
      factor_ret [D_loc, K], specific_ret [D_loc, N], r2 [D_loc], status [D_loc]
      factor_ret_global [T, K] (all ranks' dates), nw_cov / eigen_cov / vra_cov [D_loc, K, K],
      vra_lambda [D_loc]
    """

    def __init__(self, panel: RiskPanel, config: RiskConfig | None = None,
                 T_global: int | None = None, ctx: pdist.DistContext | None = None,
                 history: dict | None = None, sync_stages: bool = True):
        self.panel = panel
        self.cfg = config or RiskConfig()
        self.ctx = ctx or pdist.context()
        # dates already processed by an earlier run (checkpoint): global index offset
        self.history = history
        self.T_hist = int(history["T"]) if history is not None else 0
        # every rank's date-block length, exchanged once: the per-stage all-gathers then run
        # as single collectives without host synchronisation
        self.sizes = pdist.shard_sizes(panel.D, self.ctx)
        T_new = sum(self.sizes)
        if T_global is not None and int(T_global) != T_new:
            raise ValueError(f"T_global={T_global} but the ranks' date blocks sum to {T_new}")
        self.T = self.T_hist + T_new
        self.times = trace.Timer()
        self.sync_stages = sync_stages
        self.factor_ret = self.specific_ret = self.r2 = self.status = self.stats = None
        self.factor_ret_global = None
        self.nw_cov = self.eigen_cov = self.vra_cov = self.vra_lambda = None
        self.eigen_bias = None
        self.B2_global = self.B2 = None
        self.nw_params = None     # (q, tau) of the last newey_west() call

    def _stage(self, name: str):
        return trace.stage(name, self.times, self.device, sync=self.sync_stages,
                           dates=self.panel.D, K=self.K)

    @property
    def device(self):
        return self.panel.device

    @property
    def K(self) -> int:
        return self.panel.K

    @property
    def t_lo(self) -> int:
        """Global index of this rank's first date (history dates come first)."""
        return self.T_hist + self.panel.date_offset

    # --------------------------------------------------------------- stage 1: regression
    def regress(self, want_resid: bool = True):
        p = self.panel
        with self._stage("regress"):
            res = xs.xs_wls(p.styles, p.cap, p.ret, p.ind, p.P, pivot_mode=self.cfg.pivot_mode,
                            want_resid=want_resid, deterministic=self.cfg.deterministic)
        self.factor_ret, self.specific_ret, self.r2 = res.f, res.resid, res.r2
        self.status, self.stats = res.status, res.stats
        self.factor_ret_global = None
        if self.cfg.time_scan == "gather":
            self._gather_f()
        return self.factor_ret, self.specific_ret, self.r2

    def _gather_f(self) -> torch.Tensor:
        """[T, K] factor returns of every date (history first).  Collective."""
        if self.factor_ret_global is None:
            with self._stage("allgather_f"):
                F = pdist.all_gather_rows(self.factor_ret, self.ctx, self.sizes)
                if self.history is not None:
                    F = torch.cat([self.history["factor_ret"].to(F.device, F.dtype), F])
                self.factor_ret_global = F
        return self.factor_ret_global

    def _hist(self, key: str):
        if self.history is None:
            return None
        return self.history[key].to(self.device, torch.float64)

    # --------------------------------------------------------------- stage 2: Newey-West
    def newey_west(self, q: int | None = None, tau: float | None = None):
        if self.factor_ret is None:
            raise RuntimeError("please run regress() to get factor returns first")
        q = self.cfg.nw_lags if q is None else q
        tau = self.cfg.nw_half_life if tau is None else tau
        lo = self.t_lo
        self.nw_params = (int(q), float(tau))
        with self._stage("newey_west"):
            if self.cfg.time_scan == "carry":  # own dates only, block states carried across ranks
                self.nw_cov = ew_scan.newey_west_series_sharded(
                    self.factor_ret, q, tau, self.ctx, self.sizes, history=self._hist("factor_ret"))
            else:
                self.nw_cov = ew_scan.newey_west_series(self._gather_f(), q, tau, lo,
                                                        lo + self.panel.D)
        return self.nw_cov

    # --------------------------------------------------------------- stage 3: eigen adjustment
    def eigen_adjust(self, M: int | None = None, scale_coef: float | None = None,
                     T_sim: int | None = None, seed: int | None = None):
        if self.nw_cov is None:
            raise RuntimeError("please run newey_west() first")
        M = self.cfg.eigen_sims if M is None else M
        scale_coef = self.cfg.eigen_scale if scale_coef is None else scale_coef
        T_sim = T_sim or self.cfg.eigen_sim_length or self.T
        seed = self.cfg.eigen_seed if seed is None else seed
        with self._stage("eigen_adjust"):
            if self.cfg.eigen_shard == "sims":
                # Simulations sharded over ranks (10k-bootstrap configuration): every rank needs
                # the Newey-West covariances of ALL new dates, runs its block of sims on all of
                # them, and one all_reduce of the [T, K] bias sums (C5) completes the mean over M.
                lo_new = self.T_hist
                if self.cfg.time_scan == "carry":
                    # each rank scanned only its own dates: gather those blocks (no rescan, no
                    # factor-return gather), so the SP scan composes with C5 sharding
                    nw_all = pdist.all_gather_rows(self.nw_cov.contiguous(), self.ctx,
                                                   self.sizes)
                else:
                    # the gathered series is already on every rank: an O(T K^2) rescan is
                    # cheaper than gathering [T, K, K]
                    q_nw, tau_nw = self.nw_params  # the (q, tau) newey_west() actually used
                    nw_all = ew_scan.newey_west_series(self._gather_f(), q_nw, tau_nw, lo_new,
                                                       self.T)
                Fh, vb = eigen.eigen_risk_adjust_sharded(
                    nw_all, M=M, scale_coef=scale_coef, T_sim=T_sim, seed=seed,
                    chunk=self.cfg.eigen_chunk, ctx=self.ctx, psd_tol=self.cfg.psd_tol,
                    return_bias=True, date0=lo_new)
                a = self.t_lo - lo_new
                self.eigen_cov = Fh[a:a + self.panel.D].contiguous()
                self.eigen_bias = vb[a:a + self.panel.D].contiguous()
            else:
                self.eigen_cov, self.eigen_bias = eigen.eigen_risk_adjust(
                    self.nw_cov, M=M, scale_coef=scale_coef, T_sim=T_sim, seed=seed,
                    psd_tol=self.cfg.psd_tol, return_bias=True, date0=self.t_lo)
        return self.eigen_cov

    # --------------------------------------------------------------- stage 4: VRA
    def vol_regime_adjust(self, tau: float | None = None):
        """lambda_t^2 = EW mean of B_s^2 over valid s <= t; B_t^2 = mean_k f_tk^2 / sigma_tk^2.

        ``sigma_t`` is the eigen-adjusted forecast of date t itself (in-sample, quirk Q10); with
        ``config.vra_out_of_sample`` the forecast made at t-1 is used instead (USE4 practice).
        """
        if self.eigen_cov is None:
            raise RuntimeError("please run eigen_adjust() first")
        tau = self.cfg.vra_half_life if tau is None else tau
        with self._stage("vra"):
            var = torch.diagonal(self.eigen_cov, dim1=-2, dim2=-1)        # [D_loc, K]
            if self.cfg.vra_out_of_sample:
                var_all = pdist.all_gather_rows(var.contiguous(), self.ctx, self.sizes)
                if self.history is not None and "last_var" in self.history:
                    prev0 = self.history["last_var"].to(var.device, var.dtype)[None]
                else:
                    prev0 = torch.full_like(var_all[:1], float("nan"))
                prev = torch.cat([prev0, var_all[:-1]])
                lo = self.panel.date_offset
                var = prev[lo:lo + self.panel.D]
            B2 = (self.factor_ret ** 2 / var).mean(-1)                    # NaN where ER empty
            self.B2 = B2
            self.B2_global = None
            if self.cfg.time_scan == "carry":
                lam2 = ew_scan.ew_prefix_mean_sharded(B2, tau, self.ctx, self.sizes,
                                                      history=self._hist("B2"))
            else:
                lam2 = ew_scan.ew_prefix_mean(self._gather_b2(), tau)[
                    self.t_lo:self.t_lo + self.panel.D]
            # no valid date yet: the reference's sum over an empty selection gives lambda = 0
            lam2 = torch.nan_to_num(lam2, nan=0.0)
            self.vra_lambda = torch.sqrt(lam2)
            self.vra_cov = self.eigen_cov * lam2[:, None, None]
        return self.vra_cov, self.vra_lambda

    def _gather_b2(self) -> torch.Tensor:
        """[T] VRA bias statistics of every date (history first).  Collective."""
        if self.B2_global is None:
            B2_all = pdist.all_gather_rows(self.B2, self.ctx, self.sizes)
            if self.history is not None:
                B2_all = torch.cat([self.history["B2"].to(B2_all.device, B2_all.dtype), B2_all])
            self.B2_global = B2_all
        return self.B2_global

    def run(self):
        self.regress()
        self.newey_west()
        self.eigen_adjust()
        self.vol_regime_adjust()
        return self

    # --------------------------------------------------------------- checkpoint / resume
    def state_dict(self) -> dict:
        """History needed to append dates later (identical on every rank), plus artifacts.

        Call after :meth:`run`.  Collective in distributed mode (every rank must call it).
        """
        if self.vra_cov is None:
            raise RuntimeError("run all four stages before exporting a checkpoint")
        F_all, B2_all = self._gather_f(), self._gather_b2()
        r2 = pdist.all_gather_rows(self.r2, self.ctx, self.sizes)
        status = pdist.all_gather_rows(self.status, self.ctx, self.sizes)
        var = torch.diagonal(self.eigen_cov, dim1=-2, dim2=-1).contiguous()
        var_all = pdist.all_gather_rows(var, self.ctx, self.sizes)
        vra_last = pdist.all_gather_rows(self.vra_cov[-1:].contiguous(), self.ctx)[-1]
        if self.history is not None:
            r2 = torch.cat([self.history["r2"].to(r2.device), r2])
            status = torch.cat([self.history["status"].to(status.device), status])
        dates = [str(d) for d in self._global_dates()]
        if self.history is not None:
            dates = list(self.history["dates"]) + dates
        cfg = self.cfg.to_dict()
        return {
            "T": int(F_all.shape[0]), "K": int(self.K),
            "factor_names": list(self.panel.factor_names), "dates": dates,
            "config": {k: v for k, v in cfg.items()}, "config_hash": ckpt.config_hash(cfg),
            "factor_ret": F_all, "B2": B2_all,
            "r2": r2, "status": status, "last_var": var_all[-1], "last_vra_cov": vra_last,
        }

    def save(self, path) -> None:
        """Write a checkpoint (rank 0 writes; collective in distributed mode)."""
        st = self.state_dict()
        if self.ctx.rank == 0:
            ckpt.save_state(st, path)
        pdist.barrier(self.ctx)

    @classmethod
    def resume(cls, state, panel: RiskPanel, config: RiskConfig | None = None,
               T_global: int | None = None, ctx: pdist.DistContext | None = None, **kw):
        """A model for the NEW dates of ``panel`` continuing the run saved in ``state`` (a dict
        from :meth:`state_dict` or a checkpoint path).  Old dates are not recomputed: their
        factor returns feed the Newey-West prefix scan and the VRA series.  Results for the
        new dates equal those of one run over all dates (the eigen simulation length follows
        the total number of dates, quirk Q9, as in a full run)."""
        if not isinstance(state, dict):
            state = ckpt.load_state(state)
        stored = dict(state["config"])
        fv = int(state.get("format_version", ckpt.FORMAT_VERSION))
        if ckpt.config_hash(stored, fv) != state["config_hash"]:
            raise ValueError("checkpoint config does not match its hash (corrupt file?)")
        # fields a format-1 file predates take their defaults; unknown keys are ignored
        import dataclasses
        known = {f.name for f in dataclasses.fields(RiskConfig)}
        saved = RiskConfig(**{k: v for k, v in stored.items() if k in known})
        cfg = config or saved
        if ckpt.model_config(cfg.to_dict()) != ckpt.model_config(saved.to_dict()):
            raise ValueError("checkpoint was produced with a different RiskConfig")
        if int(state["K"]) != panel.K or list(state["factor_names"]) != list(panel.factor_names):
            raise ValueError("factor set of the new panel differs from the checkpoint")
        if len(panel.dates) and len(state["dates"]):
            import pandas as pd
            if pd.Timestamp(str(panel.dates[0])) <= pd.Timestamp(str(state["dates"][-1])):
                raise ValueError("resume panel must start after the last checkpointed date")
        return cls(panel, cfg, T_global=T_global, ctx=ctx, history=state, **kw)

    def diagnostics(self) -> dict:
        """Counters of the run (rank-local dates): solver status bits and NaN rates."""
        st = self.status.cpu() if self.status is not None else torch.zeros(0, dtype=torch.int32)
        out = {"dates": int(st.numel())}
        for name, bit in (("no_rows", xs.XS_NO_ROWS), ("pivot_empty", xs.XS_PIVOT_EMPTY),
                          ("near_singular", xs.XS_NEAR_SINGULAR), ("zero_pivot", xs.XS_ZERO_PIVOT),
                          ("pinv_cut", xs.XS_PINV_CUT), ("bad_sigma", xs.XS_BAD_SIGMA)):
            out[name] = int(((st & bit) != 0).sum())
        for name, t in (("factor_ret", self.factor_ret), ("nw_cov", self.nw_cov),
                        ("eigen_cov", self.eigen_cov), ("vra_cov", self.vra_cov)):
            if t is not None and t.numel():
                bad = ~torch.isfinite(t.reshape(t.shape[0], -1)).all(-1)
                out[f"{name}_nan_dates"] = int(bad.sum())
        return out

    # --------------------------------------------------------------- diagnostics
    def eigenfactor_bias(self, which: str = "eigen", start: int = 0, predlen: int = 1):
        """Eigenfactor bias statistic (``MFM.py:203-204`` runs it with predlen=21 on dates >=
        1000) of the chosen covariance series over GLOBAL dates t >= ``start`` with
        t + predlen < T.  Collective: each rank forms the z-scores of its own dates (the
        realised returns of later dates come from the gathered factor-return series), the z rows
        are all-gathered in calendar order and the std runs over all of them, so the result is
        the same on every rank and for every world size.  After :meth:`resume` only dates
        computed in this run have covariances: dates before the checkpoint's end are skipped
        with a RuntimeWarning."""
        cov = {"nw": self.nw_cov, "eigen": self.eigen_cov, "vra": self.vra_cov}[which]
        if cov is None:
            raise RuntimeError(f"covariance series {which!r} not computed yet")
        F = self._gather_f()                     # [T, K] with history first
        T, lo, D = self.T, self.t_lo, self.panel.D
        if self.T_hist > start and self.ctx.rank == 0:
            # a checkpoint keeps no covariance series: resumed runs cover their own dates only
            import warnings
            warnings.warn(f"eigenfactor_bias: dates [{start}, {self.T_hist}) precede this resumed "
                          f"run (no stored covariances); the statistic covers dates >= "
                          f"{self.T_hist} only", RuntimeWarning, stacklevel=2)
        a, b = max(start, lo), min(lo + D, T - predlen)
        z = torch.empty(0, self.K, dtype=torch.float64, device=self.device)
        if b > a:
            z = eigenfactor_z(cov[a - lo:b - lo], F[a + 1:b + predlen], predlen)
        Z = pdist.all_gather_rows(z.contiguous(), self.ctx)
        if Z.shape[0] == 0:
            return torch.full((self.K,), float("nan"), dtype=torch.float64)
        Z = Z[torch.isfinite(Z).all(-1)]
        return Z.std(0, unbiased=False)

    def specific_vol_series(self, window: int = 252, min_periods: int = 1) -> torch.Tensor:
        """[D_loc, N] trailing specific volatility, point in time: for date t the ddof-0 std of
        each stock's specific returns over the ``window`` dates ENDING at t (dates before t
        only; no later date enters).  The window crosses rank boundaries through a halo of the
        preceding window-1 rows (one collective), and every window is summed in the same fixed
        order whatever the sharding, so the result is bitwise rank-invariant.  Checkpoints keep
        no specific returns: after a resume the first window-1 new dates see only new dates."""
        e = self.specific_ret.double()
        D = e.shape[0]
        h = window - 1
        halo = pdist.halo_prev_rows(e, h, self.ctx, self.sizes)
        if e.is_cuda:  # HIP kernel, bitwise the loop below (csrc/attribution.hip)
            from ..ops.attribution import trailing_vol
            return trailing_vol(halo, e, window, min_periods)
        ext = torch.cat([halo, e])
        ok = torch.isfinite(ext)
        x = torch.where(ok, ext, torch.zeros((), dtype=torch.float64, device=e.device))
        okd = ok.double()
        n = torch.zeros_like(e)
        s1 = torch.zeros_like(e)
        s2 = torch.zeros_like(e)
        for j in range(window):  # fixed summation order: newest date first
            sl = slice(h - j, h - j + D)
            n += okd[sl]
            s1 += x[sl]
            s2 += x[sl] * x[sl]
        mean = s1 / n
        var = s2 / n - mean * mean
        vol = torch.sqrt(torch.clamp(var, min=0.0))
        return torch.where(n >= max(1, min_periods), vol,
                           torch.full_like(vol, float("nan")))

    def specific_risk_shrunk(self, window: int = 252, ngroup: int = 10, q: float = 1.0,
                             per_date: bool = True):
        """Cap-decile Bayesian shrinkage (``utils.bayes_shrink``, utils.py:153-168) of the
        point-in-time trailing specific volatility.  ``per_date``: [D_loc, N], date t shrunk
        with its own window and caps; otherwise [N] of the LAST global date, on every rank
        (broadcast from the rank that owns it).  Collective in distributed mode."""
        from ..ops.xs_reduce import bayes_shrink
        vol = self.specific_vol_series(window)
        s = bayes_shrink(vol, self.panel.cap.double(), ngroup, q).double()
        if per_date:
            return s
        return pdist.broadcast_last_row(s, self.ctx, self.sizes)

    def risk_attribution(self, h: torch.Tensor, which: str = "vra",
                         specific_vol: torch.Tensor | str | None = "shrunk"):
        """Risk decomposition of holdings ``h`` ([N] held every date, or [D_loc, N]) on this
        rank's dates against the chosen covariance series (``nw`` / ``eigen`` / ``vra``).

        ``specific_vol``: per-stock specific volatility [N] or [D_loc, N]; ``"shrunk"`` uses
        :meth:`specific_risk_shrunk` (cap-decile Bayesian shrinkage of each date's own trailing
        residual vol: point in time, identical for every world size; collective);
        None ignores specific risk.  Returns :class:`ops.attribution.RiskAttribution`.
        """
        from ..ops import attribution as attr
        if self.stats is None:
            raise RuntimeError("run regress() first")
        p = self.panel
        h = h.to(device=p.device, dtype=torch.float64)
        if h.dim() == 1:
            h = h[None, :].expand(p.D, -1)
        cov = {"nw": self.nw_cov, "eigen": self.eigen_cov, "vra": self.vra_cov}[which]
        if cov is None:
            raise RuntimeError(f"covariance series {which!r} not computed yet")
        x = attr.portfolio_exposure(p.styles, p.cap, p.ret, p.ind, h.contiguous(), self.stats, p.P)
        if isinstance(specific_vol, str):
            specific_vol = self.specific_risk_shrunk()
        svar = None if specific_vol is None else attr.portfolio_specific_var(h, specific_vol)
        return attr.risk_attribution(x, cov, svar)

    # --------------------------------------------------------------- pandas views
    def factor_returns_frame(self):
        import pandas as pd
        F = pdist.gather_to_root(self.factor_ret, self.ctx)
        if F is None:
            return None
        dates = self._global_dates()
        return pd.DataFrame(F.cpu().numpy(), index=pd.DatetimeIndex(dates), columns=self.panel.factor_names)

    def _global_dates(self):
        d = self.panel.dates
        if self.ctx.enabled:
            import torch.distributed as dist
            objs = [None] * self.ctx.world
            dist.all_gather_object(objs, np.asarray(d))
            d = np.concatenate(objs)
        return d


def eigenfactor_z(cov: torch.Tensor, fwd: torch.Tensor, predlen: int) -> torch.Tensor:
    """z-scores [n, K] of the eigen-factor portfolios of ``cov`` [n, K, K] (utils.py:103-110):
    U / colsum(U), sigma = sqrt(predlen diag(U^T cov U)), realised = U^T (prod(1 + f) - 1) over
    the next predlen dates.  ``fwd`` [n + predlen - 1, K] holds the factor returns of the
    dates after cov's first date."""
    cov = cov.double()
    n = cov.shape[0]
    w, U = eigen.eigh(cov)
    U = U / U.sum(-2, keepdim=True)
    sig = torch.sqrt(predlen * torch.einsum("dki,dkl,dli->di", U, cov, U))
    growth = (fwd.double()[:n + predlen - 1] + 1.0).unfold(0, predlen, 1).prod(-1) - 1.0  # [n, K]
    r = torch.einsum("dki,dk->di", U, growth)
    return r / sig


def eigenfactor_bias_stat(cov: torch.Tensor, ret: torch.Tensor, predlen: int = 1) -> torch.Tensor:
    """Bias statistic of eigen-factor portfolios (``utils.eigenfactor_bias_stat``, utils.py:97-117).

    For date i: eigen-portfolios U / colsum(U) of cov[i]; forecast sigma = sqrt(predlen *
    diag(U^T cov U)); realised = U^T (prod(1 + f[i+1 : i+1+predlen]) - 1); z = realised/sigma.
    Returns std over dates (ddof 0) per eigenfactor; dates with NaN covariances are skipped (the
    reference's bare ``except: pass``).  Eigenfactors ordered by descending variance.
    """
    cov = cov.double()
    ret = ret.double()
    n = cov.shape[0] - predlen
    if n <= 0:
        return torch.full((cov.shape[-1],), float("nan"), dtype=torch.float64)
    z = eigenfactor_z(cov[:n], ret[1:n + predlen], predlen)
    ok = torch.isfinite(z).all(-1)
    z = z[ok]
    return z.std(0, unbiased=False)
