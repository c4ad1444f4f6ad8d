"""Barra descriptor engine + post-processing + Barra export (L4-L6 of SURVEY.md §1).

Reference: ``Barra_factor_cal/factor_calculator.py`` (FactorCalculator, :11-576),
``post_processing.py`` and ``main.py:42-158``.  Semantics follow SURVEY.md §2.2.

MI355X design: the reference's master frame (sorted by ts_code, trade_date) lives on the device
as FLAT float32 rows plus three int32 index vectors (``seg_lo`` = first row of the row's stock,
``date_id``, ``stock_id``).  Time-series descriptors run as one rolling kernel launch each over
all stocks (``ops.rolling``); cross-sectional steps (NLSIZE, winsorize, orthogonalize) scatter
the rows into a dense [date, stock] grid in HBM, run one per-date kernel launch
(``ops.xs_reduce``) and gather back.  No per-stock or per-date Python loop anywhere.

Multi-GPU (DP with halos): every rank prepares the replicated master, keeps its
contiguous date block plus each stock's ``halo_rows()`` preceding rows (the longest window reach,
504 for RSTR), and runs descriptors and the per-date post-processing on that slice only
(:meth:`FactorEngine.date_shard`); rank 0 gathers the blocks for the Barra export.  Returns are
formed on the full history before slicing, so no halo row starts a fresh ``pct_change``.
"""
from __future__ import annotations

import logging
import os
import time
import warnings

import numpy as np
import pandas as pd
import torch

from ..ops import rolling as RL
from ..ops import xs_reduce as XR
from ..utils.config import FactorConfig

log = logging.getLogger("mfa.factors")

BARRA_RENAME = {
    "trade_date": "date", "ts_code": "stocknames", "l1_code": "industry", "circ_mv": "capital",
    "SIZE": "size", "BETA": "beta", "RSTR": "momentum", "volatility": "residual_volatility",
    "NLSIZE": "non_linear_size", "BP": "book_to_price_ratio", "earnings": "earnings_yield",
}
BARRA_OUTPUT_COLUMNS = [
    "date", "stocknames", "capital", "ret", "industry",
    "size", "beta", "momentum", "residual_volatility", "non_linear_size",
    "book_to_price_ratio", "liquidity", "earnings_yield", "growth", "leverage",
]
FACTORS_TO_RUN = ["SIZE", "BETA", "RSTR", "DASTD", "CMRA", "NLSIZE", "BP", "LIQUIDITY",
                  "EARNINGS", "GROWTH", "LEVERAGE"]
OUTPUT_ORDER = {  # columns each factor group appends (factor_calculator.py run :525-569)
    "SIZE": ["SIZE"], "BETA": ["BETA", "HSIGMA"], "RSTR": ["RSTR"], "DASTD": ["DASTD"],
    "CMRA": ["CMRA"], "NLSIZE": ["NLSIZE"], "BP": ["BP"], "LIQUIDITY": ["STOM", "STOQ", "STOA"],
    "EARNINGS": ["CETOP", "ETOP"], "GROWTH": ["YOYProfit", "YOYSales"],
    "LEVERAGE": ["MLEV", "DTOA", "BLEV"],
}


def _default_device():
    d = os.environ.get("MFA_DEVICE")
    if d:
        return torch.device(d)
    return torch.device("cuda:0" if torch.cuda.is_available() else "cpu")


class FactorEngine:
    """Descriptor computation on a stock-sorted master panel (``FactorCalculator`` semantics)."""

    NUMERIC = ["close", "total_mv", "circ_mv", "pb", "turnover_rate", "pe_ttm", "n_cashflow_act",
               "total_ncl", "total_hldr_eqy_inc_min_int", "debt_to_assets", "q_profit_yoy",
               "q_sales_yoy"]

    def __init__(self, prices_df: pd.DataFrame, index_df: pd.DataFrame, device=None,
                 config: FactorConfig | None = None):
        self.cfg = config or FactorConfig()
        self.device = torch.device(device) if device is not None else _default_device()
        t0 = time.perf_counter()
        self.master = self._prepare(prices_df, index_df)
        self.prep_s = time.perf_counter() - t0
        self.own = None  # row mask of the owned date block (date_shard); None = every row

    # ---------------------------------------------------------------- _prepare_data (:34-64)
    @staticmethod
    def _date_strings(td: pd.Series):
        """(codes, unique "%Y/%m/%d" strings) of a date column, formatting only the uniques
        (per-row strftime / to_datetime dominated host prep: 4.3 s at 2.5M rows)."""
        codes, uniq = pd.factorize(td)
        u = pd.Series(uniq)
        if not isinstance(u.dtype, pd.api.types.DatetimeTZDtype) and not np.issubdtype(u.dtype, np.datetime64):
            u = pd.to_datetime(u.astype(str), format="mixed")
        return codes, u.dt.strftime("%Y/%m/%d").to_numpy(dtype=object)

    def _prepare(self, prices_df, index_df) -> pd.DataFrame:
        # _prepare_data (:34-64): "%Y/%m/%d" dates, stable sort by (ts_code, trade_date), the
        # index's pct_change merged per date.  Done on integer codes: factorize the keys once,
        # format only the unique dates, lexsort, and look market_ret up by date code.
        dc, dstr = self._date_strings(prices_df["trade_date"])
        dnames = np.unique(dstr)                      # sorted "%Y/%m/%d" == chronological
        drank = np.searchsorted(dnames, dstr)         # unique-date code -> sorted date code
        tc = prices_df["ts_code"]
        if not (tc.dtype == object and pd.api.types.infer_dtype(tc, skipna=False) == "string"):
            tc = tc.astype(str)                       # (skip the 2.5M-string copy when already str)
        scodes, snames = pd.factorize(tc, sort=True)
        row_d = drank[dc]
        # stable sort by (ts_code, trade_date) on one int64 key; input already in that order
        # (the usual case for stored panels) is detected in O(n) and not permuted at all
        key = scodes.astype(np.int64) * len(dnames) + row_d
        if len(key) < 2 or bool((key[1:] >= key[:-1]).all()):
            order = np.arange(len(key))
            p = prices_df.copy(deep=False)
            p.index = pd.RangeIndex(len(p))
        else:
            order = np.argsort(key, kind="stable")
            p = prices_df.take(order)
            p.index = pd.RangeIndex(len(p))
        p["trade_date"] = dnames[row_d[order]]
        ix = index_df[["trade_date", "close"]].copy()
        ic, istr = self._date_strings(ix["trade_date"])
        ix["trade_date"] = istr[ic]
        ix = ix.sort_values("trade_date").reset_index(drop=True)
        ix["market_ret"] = ix["close"].pct_change()
        if ix["trade_date"].is_unique:
            pos = pd.Index(ix["trade_date"]).get_indexer(dnames)
            mr = np.where(pos >= 0, ix["market_ret"].to_numpy(np.float64)[np.maximum(pos, 0)], np.nan)
            master = p
            master["market_ret"] = mr[row_d[order]]
        else:  # duplicate index dates: keep the merge's row multiplication
            master = p.merge(ix[["trade_date", "market_ret"]], on="trade_date", how="left")
        master.insert(0, "original_index", np.arange(len(master)))
        dev = self.device
        if len(master) == len(p):
            codes, self.stock_names = scodes[order], pd.Index(snames)
            dcodes, self.date_names = row_d[order], pd.Index(dnames)
        else:
            codes, self.stock_names = pd.factorize(master["ts_code"].astype(str), sort=True)
            dcodes, self.date_names = pd.factorize(master["trade_date"], sort=True)
        self.R = len(master)
        self.D, self.N = len(self.date_names), len(self.stock_names)
        self.stock_id = torch.from_numpy(codes.astype(np.int32)).to(dev)
        self.date_id = torch.from_numpy(dcodes.astype(np.int32)).to(dev)
        self.seg_lo = RL.seg_lo_from_codes(self.stock_id)
        self.grid_idx = (self.date_id.long() * self.N + self.stock_id.long())
        self.cols = {}
        for c in self.NUMERIC + ["market_ret"]:
            if c in master.columns:
                self.cols[c] = torch.from_numpy(master[c].to_numpy(dtype=np.float32, na_value=np.nan)).to(dev)
        self.cols["ret"], self.cols["log_ret"] = RL.returns(self.cols["close"], self.seg_lo)
        # sorted by construction on the lexsort path (codes are sort=True factorize ranks);
        # only the merge path needs the O(n) string comparison
        if len(master) != len(p) and not master["ts_code"].is_monotonic_increasing:
            raise AssertionError("master frame must be sorted by ts_code")
        return master

    # ---------------------------------------------------------------- date sharding (DP + halo)
    def halo_rows(self) -> int:
        """Rows of a stock's history before an output row that the row's descriptors depend on:
        each window's reach back to the anchor of its segment-anchored kernel (ops.rolling
        ``*_reach``: 566 for RSTR's 504-row reach and 64-row segments).  A date shard that holds
        them computes its owned rows bit for bit as the full panel does."""
        c = self.cfg
        return max(RL.ew_reach(c.beta_window), RL.ew_reach(c.dastd_window),
                   RL.pos_reach(c.rstr_window - c.rstr_lag, c.rstr_lag),
                   RL.cmra_reach(c.cmra_window, c.cmra_partial),
                   *(RL.pos_reach(w) for w, _ in (c.stom, c.stoq, c.stoa)))

    @property
    def row_ord(self) -> torch.Tensor:
        """Each row's ordinal in its stock's FULL history (int32; rows of a shard keep the
        ordinals of the master they were cut from)."""
        ro = getattr(self, "_row_ord", None)
        if ro is None:
            ro = (torch.arange(self.R, device=self.seg_lo.device, dtype=torch.int32)
                  - self.seg_lo.to(torch.int32))
            self._row_ord = ro
        return ro

    def grid_map(self) -> "XR.GridMap":
        """Rows <-> the (date, stock) grid as an LDS-tiled transpose (built once per engine)."""
        gm = getattr(self, "_grid_map", None)
        if gm is None:
            gm = self._grid_map = XR.GridMap(self.stock_id, self.date_id, self.D, self.N)
        return gm

    def seg_layout(self) -> "RL.SegLayout":
        """The segment layout of the rolling descriptors (:class:`ops.rolling.SegLayout`, keyed
        by the rows' full-history ordinals), built once per engine with its virtual input
        series shared by every descriptor; None off the GPU."""
        if self.device.type != "cuda":
            return None
        lay = getattr(self, "_seg", None)
        if lay is None:
            # the rolling descriptors' four input series placed in the layout's own pass
            ser = [self.cols.get(c) for c in ("ret", "market_ret", "log_ret", "turnover_rate")]
            lay = self._seg = RL.SegLayout(self.seg_lo, self.row_ord, series=ser)
        return lay

    def date_shard(self, lo: int, hi: int, halo: int | None = None) -> "FactorEngine":
        """Engine over the rows of dates [lo, hi) plus each stock's ``halo`` preceding rows.

        Every window of an owned row then lies inside the slice, or starts at the stock's true
        first row, so the rolling descriptors of owned rows equal the full-panel ones (up to the
        summation order of the sliding kernels); per-date steps only see owned dates whole.
        The statement-row TTM (whose 4 distinct statements can reach further back than any
        row window) is formed on the full rows first and sliced.  Rows outside [lo, hi) are
        dropped again by :meth:`run` (or :meth:`owned`).
        """
        H = self.halo_rows() if halo is None else int(halo)
        dev = self.device
        sid = self.stock_id.long()
        row = torch.arange(self.R, device=dev, dtype=torch.int64)
        own = (self.date_id >= lo) & (self.date_id < hi)
        first = torch.full((self.N,), self.R, dtype=torch.int64, device=dev)
        first = first.scatter_reduce(0, sid[own], row[own], reduce="amin")  # first owned row
        f = first[sid]
        keep = own | ((f < self.R) & (row < f) & (row >= f - H))
        idx = torch.nonzero(keep).flatten()
        if self._has_statements():
            self.cashflow_ttm()
        sub = self._take(idx)
        sub.own = own[idx]
        sub.lo, sub.hi = lo, hi
        return sub

    def owned(self) -> "FactorEngine":
        """The owned rows of a :meth:`date_shard` as an engine of its own, on the LOCAL date
        axis [0, hi - lo) (``date_lo`` = global index of local date 0): the per-date
        post-processing then works on a [hi - lo, N] grid instead of the global one."""
        if self.own is None:
            return self
        sub = self._take(torch.nonzero(self.own).flatten(), self.lo, self.hi)
        sub.date_lo = self.lo
        return sub

    def _copy_labels(self, sub: "FactorEngine", d_lo: int, d_hi: int) -> None:
        sub.stock_names, sub.date_names = self.stock_names, self.date_names[d_lo:d_hi]

    def _take(self, idx: torch.Tensor, d_lo: int = 0, d_hi: int | None = None) -> "FactorEngine":
        """Rows ``idx`` (increasing, so still sorted by stock then date) as a new engine; dates
        renumbered to [0, d_hi - d_lo)."""
        d_hi = self.D if d_hi is None else d_hi
        sub = object.__new__(type(self))
        sub.cfg, sub.device, sub.prep_s = self.cfg, self.device, 0.0
        self._copy_labels(sub, d_lo, d_hi)
        sub.D, sub.N, sub.R = d_hi - d_lo, self.N, int(idx.numel())
        sub.master = None if self.master is None else \
            self.master.iloc[idx.cpu().numpy()].reset_index(drop=True)
        sub.stock_id = self.stock_id[idx]
        sub.date_id = self.date_id[idx] - d_lo if d_lo else self.date_id[idx]
        sub.seg_lo = RL.seg_lo_from_codes(sub.stock_id)
        sub.grid_idx = sub.date_id.long() * sub.N + sub.stock_id.long()
        sub.cols = {k: v[idx] for k, v in self.cols.items()}
        sub._row_ord = self.row_ord[idx]
        sub._seg = None
        sub._grid_map = None
        ttm = getattr(self, "_ttm", None)
        sub._ttm = None if ttm is None else ttm[idx]
        sub.own = None
        sub.date_lo = getattr(self, "date_lo", 0) + d_lo
        return sub

    # ---------------------------------------------------------------- grid helpers
    def to_grid(self, x: torch.Tensor) -> torch.Tensor:
        g = torch.full((self.D * self.N,), float("nan"), dtype=torch.float32, device=self.device)
        g[self.grid_idx] = x.to(torch.float32)
        return g.view(self.D, self.N)

    def from_grid(self, g: torch.Tensor) -> torch.Tensor:
        return g.reshape(-1)[self.grid_idx]

    def _need(self, *names):
        missing = [n for n in names if n not in self.cols]
        if missing:
            print(f"\nERROR: Missing required columns: {missing}\n")
            return False
        return True

    # ---------------------------------------------------------------- descriptors
    def compute_size(self):
        return {"SIZE": torch.log(self.cols["total_mv"])}

    def compute_beta_hsigma(self):
        c = self.cfg
        b, h = RL.beta_hsigma(self.cols["ret"], self.cols["market_ret"], self.seg_lo, c.beta_window,
                              c.beta_half_life, c.beta_min_periods, row_ord=self.seg_layout())
        return {"BETA": b, "HSIGMA": h}

    def compute_rstr(self):
        c = self.cfg
        return {"RSTR": RL.rstr(self.cols["log_ret"], self.seg_lo, c.rstr_window, c.rstr_lag,
                                c.rstr_half_life, c.rstr_min_periods, row_ord=self.seg_layout())}

    def compute_dastd(self):
        c = self.cfg
        return {"DASTD": RL.dastd(self.cols["ret"], self.cols["market_ret"], self.seg_lo, c.dastd_window,
                                  c.dastd_half_life, c.dastd_min_periods, row_ord=self.seg_layout())}

    def compute_cmra(self):
        c = self.cfg
        return {"CMRA": RL.cmra(self.cols["log_ret"], self.seg_lo, c.cmra_window, c.cmra_partial,
                                row_ord=self.seg_layout())}

    def compute_nlsize(self):
        # per date: -residual of SIZE^3 on [1, SIZE], SIZE = ln(total_mv) formed in fp64 in-kernel
        mv = self.to_grid(self.cols["total_mv"])
        out = XR.ols_resid(None, [mv], min_rows=2, sign=-1.0, log_x0=True, ypow=3)
        return {"NLSIZE": self.from_grid(out)}

    def compute_bp(self):
        if not self._need("pb"):
            return None
        pb = self.cols["pb"]
        return {"BP": torch.where(pb > 0, 1.0 / pb, torch.full_like(pb, float("nan")))}

    def compute_liquidity(self):
        if not self._need("turnover_rate"):
            return None
        c = self.cfg
        # the three turnover sums in one pass of the segment-anchored kernel
        sums = RL.window_sums(self.cols["turnover_rate"], self.seg_lo, [c.stom, c.stoq, c.stoa],
                              scale=0.01, log=True, row_ord=self.seg_layout())
        return dict(zip(("STOM", "STOQ", "STOA"), sums))

    def _has_statements(self) -> bool:
        return "n_cashflow_act" in self.cols and "end_date" in self.master.columns

    def cashflow_ttm(self) -> torch.Tensor:
        """[R] float64 statement-row TTM of ``n_cashflow_act`` (factor_calculator.py:392-410),
        computed once and kept (date shards slice the full-row result)."""
        if getattr(self, "_ttm", None) is None:
            m = self.master
            cf = self._ttm_by_codes(m)
            self._ttm = cf if cf is not None else self._ttm_by_merge(m)
        return self._ttm

    def compute_earnings_yield(self):
        if not (self._need("n_cashflow_act", "total_mv", "pe_ttm") and self._has_statements()):
            return None
        cf = self.cashflow_ttm()
        mv = self.cols["total_mv"].double()
        pe = self.cols["pe_ttm"].double()
        rows = getattr(self, "_ttm_rows", None)
        if rows is not None:  # merge-multiplied rows (see _ttm_by_merge)
            mv, pe = mv[rows], pe[rows]
        nan = torch.full_like(mv, float("nan"))
        cetop = torch.where((mv > 0) & (cf > 0), cf / mv, nan)  # unit mix-up kept (quirk Q17)
        etop = torch.where(pe > 0, 1.0 / pe, nan)
        return {"CETOP": cetop.float(), "ETOP": etop.float()}

    def _ttm_by_codes(self, m: pd.DataFrame):
        """Statement-row TTM (:392-410) on integer keys: (stock, end_date) rows deduplicated by
        np.unique, a 4-row rolling sum per stock on the device, gathered back by the inverse
        index.  None when one (stock, end_date) carries several values (the merge path's row
        multiplication is then kept by :meth:`_ttm_by_merge`)."""
        runs = self._ttm_runs(m)
        if runs is not None:
            return runs
        ecodes, _ = pd.factorize(m["end_date"], sort=True)
        ne = int(ecodes.max()) + 1 if len(ecodes) else 0
        sc = self.stock_id.cpu().numpy().astype(np.int64)
        key = sc * (ne + 1) + np.where(ecodes < 0, ne, ecodes)  # NaT last, as sort_values
        uk, first, inv = np.unique(key, return_index=True, return_inverse=True)
        v = m["n_cashflow_act"].to_numpy(np.float64, na_value=np.nan)
        vf = v[first]
        same = (v == vf[inv]) | (np.isnan(v) & np.isnan(vf[inv]))
        if not same.all():
            return None
        seg = RL.seg_lo_from_codes(torch.from_numpy(uk // (ne + 1))).to(self.device)
        with RL.direct_kernels():   # newest-first sums, as the run kernel (ttm_rows)
            ttm = RL.rolling_sum(torch.from_numpy(vf.astype(np.float32)).to(self.device), seg, 4, 4)
        return ttm.double()[torch.from_numpy(inv).to(self.device)]

    def _ttm_runs(self, m: pd.DataFrame):
        """O(n) fast path of :meth:`_ttm_by_codes`: the master frame is sorted by (stock,
        trade_date) and a point-in-time as-of join makes end_date non-decreasing within a stock,
        so the distinct (stock, end_date) rows are the RUN STARTS of the row order — no sort, no
        factorize.  None (caller falls back) when the order does not hold, e.g. a restatement
        that moves end_date backwards, or when a run carries several values."""
        ed = m["end_date"]
        if not np.issubdtype(ed.dtype, np.datetime64) or len(ed) == 0:
            return None
        ev = ed.to_numpy("datetime64[ns]").view(np.int64).copy()
        ev[ed.isna().to_numpy()] = np.iinfo(np.int64).max  # NaT last, as sort_values
        dev = self.device
        # the run detection, dedupe and gather run as device tensor ops (one sync: nonzero)
        e = torch.from_numpy(ev).to(dev)
        sc = self.stock_id.to(dev, torch.int64)
        ds, de = sc[1:] - sc[:-1], e[1:] - e[:-1]
        start = torch.ones(len(ev), dtype=torch.bool, device=dev)
        start[1:] = (ds != 0) | (de != 0)
        bad = (ds < 0) | ((ds == 0) & (de < 0))
        first = torch.nonzero(start).flatten()
        if bool(bad.any()):
            return None
        inv = torch.cumsum(start, 0) - 1
        v = torch.from_numpy(m["n_cashflow_act"].to_numpy(np.float64, na_value=np.nan)).to(dev)
        vf = v[first]
        vb = vf[inv]
        if not bool(((v == vb) | (v.isnan() & vb.isnan())).all()):
            return None
        seg = RL.seg_lo_from_codes(sc[first].to(torch.int32))
        with RL.direct_kernels():
            ttm = RL.rolling_sum(vf.float(), seg, 4, 4)
        return ttm.double()[inv]

    def _ttm_by_merge(self, m: pd.DataFrame):
        fin = m[["ts_code", "end_date", "n_cashflow_act"]].drop_duplicates().copy()
        fin = fin.sort_values(["ts_code", "end_date"], kind="stable").reset_index(drop=True)
        codes = torch.from_numpy(pd.factorize(fin["ts_code"].astype(str))[0].astype(np.int32))
        seg = RL.seg_lo_from_codes(codes).to(self.device)
        v = torch.from_numpy(fin["n_cashflow_act"].to_numpy(np.float32, na_value=np.nan)).to(self.device)
        with RL.direct_kernels():
            ttm = RL.rolling_sum(v, seg, 4, 4)  # statement-row TTM (quirk Q18)
        fin["n_cashflow_act_ttm"] = ttm.double().cpu().numpy()
        tmp = m[["original_index", "ts_code", "end_date"]].merge(
            fin[["ts_code", "end_date", "n_cashflow_act_ttm"]], on=["ts_code", "end_date"], how="left")
        tmp = tmp.sort_values("original_index")  # the reference's (unstable) default sort: same tie order
        if len(tmp) != len(m):
            # one statement with several values: the left merge multiplies its rows
            # (factor_calculator.py:403-410) and run() repeats every other column with them
            self._ttm_rows = torch.from_numpy(tmp["original_index"].to_numpy(np.int64)).to(self.device)
        return torch.from_numpy(tmp["n_cashflow_act_ttm"].to_numpy(np.float64, na_value=np.nan)).to(self.device)

    def ttm_multiplies_rows(self) -> bool:
        """True when the statement TTM merge multiplied rows (a statement with several values):
        the descriptor frame then has more rows than the master, as in the reference."""
        if not (self._need_quiet("n_cashflow_act") and self._has_statements()):
            return False
        self.cashflow_ttm()
        return getattr(self, "_ttm_rows", None) is not None

    def _need_quiet(self, *names) -> bool:
        return all(n in self.cols for n in names)

    def select_growth_factors(self):
        if not self._need("q_profit_yoy", "q_sales_yoy"):
            return None
        return {"YOYProfit": self.cols["q_profit_yoy"] / 100.0, "YOYSales": self.cols["q_sales_yoy"] / 100.0}

    def compute_leverage(self):
        if not self._need("total_mv", "total_ncl", "total_hldr_eqy_inc_min_int", "debt_to_assets"):
            return None
        if self.device.type == "cuda":  # one fused pass (csrc/rolling.hip leverage_kernel)
            mlev, blev = RL.leverage(self.cols["total_mv"], self.cols["total_ncl"],
                                     self.cols["total_hldr_eqy_inc_min_int"])
            return {"MLEV": mlev, "DTOA": self.cols["debt_to_assets"], "BLEV": blev}
        mv = self.cols["total_mv"].double()
        ncl = self.cols["total_ncl"].double()
        be = self.cols["total_hldr_eqy_inc_min_int"].double()
        nan = torch.full_like(mv, float("nan"))
        mlev = (mv + ncl) / mv
        mlev = torch.where(torch.isinf(mlev), nan, mlev)
        blev = torch.where(be > 0, (be + ncl) / be, nan)
        return {"MLEV": mlev.float(), "DTOA": self.cols["debt_to_assets"], "BLEV": blev.float()}

    METHODS = {
        "SIZE": "compute_size", "BETA": "compute_beta_hsigma", "RSTR": "compute_rstr",
        "DASTD": "compute_dastd", "CMRA": "compute_cmra", "NLSIZE": "compute_nlsize",
        "BP": "compute_bp", "LIQUIDITY": "compute_liquidity", "EARNINGS": "compute_earnings_yield",
        "GROWTH": "select_growth_factors", "LEVERAGE": "compute_leverage",
    }

    def compute(self, factors: list[str]) -> dict:
        """Run factor groups; returns ordered {column: flat tensor}."""
        out = {}
        self.timings = {}
        for name in factors:
            meth = self.METHODS.get(name.upper())
            if meth is None:
                print(f"Warning: Factor '{name}' not found.")
                continue
            t0 = time.perf_counter()
            res = getattr(self, meth)()
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            self.timings[name.upper()] = (time.perf_counter() - t0) * 1e3
            if res is None:
                print(f"Warning: Method for '{name}' returned None.")
                continue
            out.update(res)
        return out

    def run(self, factors: list[str]) -> pd.DataFrame:
        """``FactorCalculator.run``: [ts_code, trade_date, ret, circ_mv, <descriptors>] in master order."""
        res = self.compute(factors)
        df = self.master[["ts_code", "trade_date"]].copy()
        df["ret"] = self.cols["ret"].double().cpu().numpy()
        df["circ_mv"] = self.master["circ_mv"].to_numpy(np.float64, na_value=np.nan) if "circ_mv" in self.master else np.nan
        rows = getattr(self, "_ttm_rows", None)
        if rows is not None:
            # a statement with several values multiplied its rows in the TTM merge: every column
            # repeats with them, as the reference's merges on original_index do (:561-566)
            rc = rows.cpu().numpy()
            df = df.iloc[rc].reset_index(drop=True)
            for k, v in res.items():
                df[k] = v.double().cpu().numpy() if v.numel() == len(rc) else v.double().cpu().numpy()[rc]
            if self.own is not None:
                df = df.loc[self.own.cpu().numpy()[rc]].reset_index(drop=True)
            return df
        for k, v in res.items():
            df[k] = v.double().cpu().numpy()
        if self.own is not None:  # date shard: drop the halo rows
            df = df.loc[self.own.cpu().numpy()].reset_index(drop=True)
        return df


# ---------------------------------------------------------------------------------------------
# post-processing on a descriptor frame (post_processing.py) — per-date kernels on dense grids
# ---------------------------------------------------------------------------------------------
class _Grid:
    def __init__(self, df: pd.DataFrame, device):
        self.device = device
        dcodes, self.dates = pd.factorize(df["trade_date"], sort=True)
        scodes = None
        if "ts_code" in df.columns:
            scodes, self.stocks = pd.factorize(df["ts_code"].astype(str), sort=True)
            # frames in master order (ts_code, trade_date) are duplicate-free iff this key is
            # strictly increasing: an O(n) check instead of DataFrame.duplicated's hashing
            k = scodes.astype(np.int64) * (len(self.dates) + 1) + dcodes
            if not (len(k) < 2 or bool((k[1:] > k[:-1]).all())) and \
                    df.duplicated(["trade_date", "ts_code"]).any():
                scodes = None
        if scodes is None:  # no stock key (or duplicates): the row's rank within its date is its column
            scodes = df.groupby("trade_date").cumcount().to_numpy()
            self.stocks = np.arange(int(scodes.max()) + 1 if len(scodes) else 0)
        self.D, self.N = len(self.dates), len(self.stocks)
        self.idx = torch.from_numpy(dcodes.astype(np.int64) * self.N + scodes.astype(np.int64)).to(device)

    def put(self, col: np.ndarray) -> torch.Tensor:
        g = torch.full((self.D * self.N,), float("nan"), dtype=torch.float32, device=self.device)
        g[self.idx] = torch.from_numpy(np.asarray(col, dtype=np.float32)).to(self.device)
        return g.view(self.D, self.N)

    def take(self, g: torch.Tensor) -> np.ndarray:
        return g.reshape(-1)[self.idx].double().cpu().numpy()


def winsorize_frame(df: pd.DataFrame, factor_list: list, n_std: float = 2.5, device=None,
                    grid: _Grid | None = None, copy: bool = True) -> pd.DataFrame:
    """``grid`` (a :class:`_Grid` of the same keys) and ``copy=False`` let a pipeline build the
    (date, stock) index once and work in place; the defaults keep ``post_processing`` semantics."""
    dev = torch.device(device) if device else _default_device()
    out = df.copy() if copy else df
    grid = grid if grid is not None else _Grid(out, dev)
    for f in factor_list:
        if f not in out.columns:
            print(f"Warning: Factor '{f}' not found in DataFrame. Skipping.")
            continue
        out[f] = grid.take(XR.winsorize(grid.put(out[f].to_numpy(np.float64, na_value=np.nan)), n_std))
    return out


def composite_frame(df: pd.DataFrame, config: dict, device=None, copy: bool = True) -> pd.DataFrame:
    dev = torch.device(device) if device else _default_device()
    out = df.copy() if copy else df
    for new, cfg in config.items():
        xs, ws = [], []
        for c, w in zip(cfg["components"], cfg["weights"]):
            if c in out.columns:
                xs.append(torch.from_numpy(out[c].to_numpy(np.float32, na_value=np.nan)).to(dev))
                ws.append(w)
            else:
                print(f"Warning: Component '{c}' not found in DataFrame. Skipping.")
        if xs:
            out[new] = XR.composite(xs, ws).double().cpu().numpy()
        else:
            out[new] = np.nan
    return out


def orthogonalize_frame(df: pd.DataFrame, rules: dict, device=None, grid: _Grid | None = None,
                        copy: bool = True) -> pd.DataFrame:
    dev = torch.device(device) if device else _default_device()
    out = df.copy() if copy else df
    grid = grid if grid is not None else _Grid(out, dev)
    for target, against in rules.items():
        y = grid.put(out[target].to_numpy(np.float64, na_value=np.nan))
        xs = [grid.put(out[a].to_numpy(np.float64, na_value=np.nan)) for a in against]
        out[target] = grid.take(XR.ols_resid(y, xs, min_rows=len(against) + 2))
    return out


def _next_in_group(keys: pd.Series, values: np.ndarray) -> np.ndarray:
    """``values`` shifted by -1 within groups of ``keys`` in frame order (groupby().shift(-1));
    NaN keys are their own non-group (pandas dropna) and get NaN."""
    codes = pd.factorize(keys)[0]
    if len(codes) < 2 or bool((codes[1:] >= codes[:-1]).all()):
        order = np.arange(len(codes))  # frame already grouped (master order): no sort
    else:
        order = np.argsort(codes, kind="stable")
    out = np.full(len(values), np.nan)
    same = codes[order[1:]] == codes[order[:-1]]
    nxt = np.where(same, values[order[1:]], np.nan)
    out[order[:-1]] = nxt
    out[codes < 0] = np.nan
    return out


def barra_export(processed: pd.DataFrame, sw_industry: pd.DataFrame, _merge_path: bool = False):
    """main.py:98-137: industry merge, t+1 return, rename/select; plus industry_info.

    When every stock has one industry row (the usual case) the merge is an index lookup and
    only the exported columns are materialised; a stock with several memberships (quirk Q21:
    the merge multiplies its rows) takes the pandas merge path.
    """
    if not _merge_path and sw_industry["ts_code"].is_unique and "l1_code" not in processed.columns:
        pos = pd.Index(sw_industry["ts_code"]).get_indexer(processed["ts_code"])
        l1 = sw_industry["l1_code"].to_numpy(dtype=object)
        src = {"l1_code": pd.Series(np.where(pos >= 0, l1[np.maximum(pos, 0)], np.nan), dtype=object)}
        src["ret"] = _next_in_group(processed["ts_code"], processed["ret"].to_numpy(np.float64))
        inv = {v: k for k, v in BARRA_RENAME.items()}
        cols = {}
        for c in BARRA_OUTPUT_COLUMNS:
            s0 = inv.get(c, c)
            if s0 in src:
                cols[c] = src[s0]
            elif s0 in processed.columns and (s0 == c or c not in processed.columns):
                cols[c] = processed[s0].to_numpy()
        final = pd.DataFrame(cols)
    else:
        barra = processed.merge(sw_industry[["ts_code", "l1_code"]], on="ts_code", how="left")
        barra["ret"] = barra.groupby("ts_code")["ret"].shift(-1)
        barra = barra.rename(columns=BARRA_RENAME)
        final = barra[[c for c in BARRA_OUTPUT_COLUMNS if c in barra.columns]]
    stk = pd.DataFrame({"ts_code": pd.unique(final["stocknames"].to_numpy())})  # first-seen order
    cols = [c for c in ["ts_code", "l1_code", "l1_name", "in_date"] if c in sw_industry.columns]
    info = stk.merge(sw_industry[cols], on="ts_code", how="left")
    info = info.drop_duplicates(subset=[c for c in ["l1_code", "l1_name"] if c in info.columns]).rename(
        columns={"l1_code": "code", "l1_name": "industry_names", "in_date": "start_date"})
    info = info[[c for c in ["code", "industry_names", "start_date"] if c in info.columns]]
    return final, info


def postprocess_columns(eng: "FactorEngine", res: dict, cfg: FactorConfig) -> dict:
    """main.py:71-86 on device tensors in master order: winsorize every non-key column (incl.
    ret and circ_mv, quirk Q23), the composites, then the orthogonalisation, on the engine's
    own (date, stock) grid index.  Returns {column: flat tensor}."""
    dev, nan = eng.device, float("nan")
    D, N, idx = eng.D, eng.N, eng.grid_idx

    def put(x):
        return eng.grid_map().scatter(x.to(torch.float32)[None])[0].view(D, N)

    def take(g):
        return eng.grid_map().gather(g.contiguous(), 1)[0]

    col = {"ret": eng.cols["ret"],
           "circ_mv": eng.cols["circ_mv"] if "circ_mv" in eng.cols else torch.full((eng.R,), nan, device=dev)}
    col.update(res)
    # winsorize every non-key column (incl. ret, circ_mv: quirk Q23): all columns scattered onto
    # their (date, stock) grids in one launch, one per-date winsorize over the [C * D, N] stack,
    # one gather back
    names = list(col)
    gm = eng.grid_map()
    X = torch.stack([col[f].to(torch.float32) for f in names])
    G = XR.winsorize_(gm.scatter(X).view(len(names) * D, N), cfg.winsor_n_std)
    Xw = gm.gather(G, len(names))
    col = {f: Xw[k] for k, f in enumerate(names)}
    for new, cc in cfg.composite.items():
        xs, ws = [], []
        for c, w in zip(cc["components"], cc["weights"]):
            if c in col:
                xs.append(col[c].to(torch.float32))
                ws.append(w)
            else:
                print(f"Warning: Component '{c}' not found in DataFrame. Skipping.")
        col[new] = XR.composite(xs, ws) if xs else torch.full((eng.R,), nan, device=dev, dtype=torch.float64)
    for target, against in cfg.ortho.items():
        col[target] = take(XR.ols_resid(put(col[target]), [put(col[a]) for a in against],
                                        min_rows=len(against) + 2))
    return col


def next_return(eng: "FactorEngine", ret: torch.Tensor) -> torch.Tensor:
    """``groupby(ts_code).ret.shift(-1)`` (main.py:99, the t+1 return) in master order."""
    ret = ret.double()
    sid = eng.stock_id
    nxt = torch.full_like(ret, float("nan"))
    if eng.R > 1:
        nxt[:-1] = torch.where(sid[1:] == sid[:-1], ret[1:], ret.new_tensor(float("nan")))
    return nxt


def _pipeline_columnar(eng: "FactorEngine", factors, cfg: FactorConfig, sw_industry: pd.DataFrame, t: dict):
    """Single-process fast path of :func:`factor_pipeline` (same output frames, bit for bit):
    the descriptors stay device tensors through winsorize / composite / orthogonalize on the
    engine's own (date, stock) grid index (no re-factorisation of string keys), the t+1 return
    is a shift on stock ids, and the export frame is built once from ONE device->host copy.
    Mirrors main.py:42-137 (winsorize incl. ret / circ_mv, composites, orthogonalisation,
    industry merge, t+1 return, rename)."""
    t0 = time.perf_counter()
    res = eng.compute(factors)
    m = eng.master
    t["descriptors_s"] = t.pop("prep_s", 0.0) + time.perf_counter() - t0
    t0 = time.perf_counter()
    col = postprocess_columns(eng, res, cfg)
    t["postprocess_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    sid = eng.stock_id
    nxt = next_return(eng, col["ret"])
    inv = {v: k for k, v in BARRA_RENAME.items()}
    names, tens = [], []  # numeric export columns in output order
    for c in BARRA_OUTPUT_COLUMNS:
        s0 = inv.get(c, c)
        if s0 == "ret":
            names.append(c)
            tens.append(nxt)
        elif s0 not in ("ts_code", "trade_date", "l1_code") and s0 in col and (s0 == c or c not in col):
            names.append(c)
            tens.append(col[s0].double())
    host = torch.stack(tens).cpu().numpy()  # ONE device->host copy, [columns, rows]
    codes = m["ts_code"].to_numpy()
    first = np.r_[0, np.flatnonzero(np.diff(sid.cpu().numpy())) + 1]  # first row of each stock
    stock_keys = codes[first]
    pos = pd.Index(sw_industry["ts_code"]).get_indexer(stock_keys)
    l1 = sw_industry["l1_code"].to_numpy(dtype=object)
    l1_stock = np.where(pos >= 0, l1[np.maximum(pos, 0)], np.nan).astype(object)
    counts = np.diff(np.r_[first, eng.R])
    # the float block is the host array itself (no consolidation copy); key / industry object
    # columns are inserted at their output positions
    final = pd.DataFrame(host.T, columns=names, copy=False)
    for i, c in enumerate(BARRA_OUTPUT_COLUMNS):
        s0 = inv.get(c, c)
        at = sum(1 for x in BARRA_OUTPUT_COLUMNS[:i] if x in final.columns)
        if s0 == "trade_date":
            final.insert(at, c, m["trade_date"].to_numpy())
        elif s0 == "ts_code":
            final.insert(at, c, codes)
        elif s0 == "l1_code":
            final.insert(at, c, pd.Series(np.repeat(l1_stock, counts), dtype=object))
    stk = pd.DataFrame({"ts_code": pd.unique(stock_keys)})
    cols = [c for c in ["ts_code", "l1_code", "l1_name", "in_date"] if c in sw_industry.columns]
    info = stk.merge(sw_industry[cols], on="ts_code", how="left")
    info = info.drop_duplicates(subset=[c for c in ["l1_code", "l1_name"] if c in info.columns]).rename(
        columns={"l1_code": "code", "l1_name": "industry_names", "in_date": "start_date"})
    info = info[[c for c in ["code", "industry_names", "start_date"] if c in info.columns]]
    t["export_s"] = time.perf_counter() - t0
    return final, info


def factor_pipeline(prices_df, index_df, sw_industry_df, factors=None, config: FactorConfig | None = None,
                    device=None, ctx=None, columnar: bool = True):
    """main.py end to end: raw descriptors -> winsorize -> composite -> orthogonalize -> export.

    Single process (the default): :func:`_pipeline_columnar`, device tensors end to end and
    one export frame; ``columnar=False`` runs the frame-by-frame compat path (same output).
    With an enabled ``ctx`` (torchrun, one rank per GPU) the job is date-sharded on device
    tensors end to end (``e2e.run_factors``: each rank's block plus a halo, per-date steps on
    owned dates, the t+1 return across blocks by one collective, the owned rows gathered to
    rank 0 as one fp64 block); other ranks return ``(None, None, timings)``.  Input the device
    path does not model (duplicate (stock, date) rows, ...) runs on rank 0 alone.
    """
    cfg = config or FactorConfig()
    dist_on = ctx is not None and ctx.enabled
    if dist_on:
        from . import e2e
        if device is None:
            device = ctx.device
        try:
            return e2e.run_factors(prices_df, index_df, sw_industry_df, cfg, factors, device, ctx)
        except e2e.NeedsPandasPath as exc:
            log.warning("date-sharded factor pipeline: %s; rank 0 runs the whole panel", exc)
            if ctx.rank != 0:
                return None, None, {}
    t = {}
    t0 = time.perf_counter()
    eng = FactorEngine(prices_df, index_df, device=device, config=cfg)
    if (columnar and eng.R == len(prices_df) and sw_industry_df["ts_code"].is_unique
            and len(eng.master) == eng.R and eng.grid_map().strict
            and not eng.ttm_multiplies_rows()):
        # (duplicate (stock, date) rows take the frame path: its per-date grids give every row
        # a column of its own)
        t["prep_s"] = time.perf_counter() - t0
        final, info = _pipeline_columnar(eng, factors or FACTORS_TO_RUN, cfg, sw_industry_df, t)
        return final, info, dict(t, kernel_ms=getattr(eng, "timings", {}))
    raw = eng.run(factors or FACTORS_TO_RUN)
    t["descriptors_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    cols = [c for c in raw.columns if c not in ("ts_code", "trade_date")]
    # raw is this pipeline's own frame: one (date, stock) grid index, in-place steps
    grid = _Grid(raw, eng.device)
    w = winsorize_frame(raw, cols, cfg.winsor_n_std, device=eng.device, grid=grid, copy=False)  # incl. ret, circ_mv (Q23)
    c = composite_frame(w, cfg.composite, device=eng.device, copy=False)
    o = orthogonalize_frame(c, cfg.ortho, device=eng.device, grid=grid, copy=False)
    t["postprocess_s"] = time.perf_counter() - t0
    final, info = barra_export(o, sw_industry_df)
    return final, info, dict(t, kernel_ms=getattr(eng, "timings", {}))


def run_factor_pipeline(prices_csv, index_csv, industry_csv, out_dir, device=None, ctx=None):
    """``cli factors``: loader CSVs -> barra_data_csi.csv + industry_info.csv.  The native
    columnar reader feeds the device path (``e2e.run_factors``; date-sharded under torchrun);
    pandas frames only when the reader is unavailable or the input needs the pandas path."""
    from . import e2e
    sw = pd.read_csv(industry_csv, dtype={"ts_code": str, "l1_code": str})
    final = info = None
    done = False
    p, i = e2e.read_price_columns(prices_csv, index_csv)
    if p is not None:
        try:
            final, info, t = e2e.run_factors(p, i, sw, device=device, ctx=ctx)
            done = True
        except e2e.NeedsPandasPath as exc:
            log.info("factors: %s; pandas path", exc)
    if not done:
        prices = pd.read_csv(prices_csv)
        index = pd.read_csv(index_csv)
        for df in (prices, index):
            df["trade_date"] = pd.to_datetime(df["trade_date"].astype(str), format="mixed")
        final, info, t = factor_pipeline(prices, index, sw, device=device, ctx=ctx)
    if final is None:  # non-root rank of a sharded run
        return None, None
    os.makedirs(out_dir, exist_ok=True)
    final.to_csv(os.path.join(out_dir, "barra_data_csi.csv"), index=False)
    info.to_csv(os.path.join(out_dir, "industry_info.csv"), index=False)
    log.info("barra_data_csi.csv %s, industry_info %s, timings %s", final.shape, info.shape, t)
    return final, info


def synthetic_prices(N: int = 50, T: int = 300, seed: int = 0, n_ind: int = 8, suspend_frac: float = 0.0,
                     start: str = "2019-01-02"):
    """Synthetic (prices_df, index_df, sw_industry_df) in the loader's schema (load_data.py:66-431).

    Random-walk closes with a market component, lognormal caps, quarterly statement fields that
    step on announcement dates, and optional random suspensions (missing rows).
    """
    rng = np.random.default_rng(seed)
    dates = pd.bdate_range(start, periods=T)
    mkt = rng.normal(0.0003, 0.012, T)
    idx_close = 3000 * np.exp(np.cumsum(mkt))
    rows = []
    qends = pd.date_range(dates[0] - pd.Timedelta(days=400), dates[-1], freq="QE")
    for i in range(N):
        code = f"{600000 + i:06d}.SH" if i % 2 else f"{i:06d}.SZ"
        beta = rng.uniform(0.5, 1.5)
        r = beta * mkt + rng.normal(0, 0.02, T)
        close = 10 * np.exp(np.cumsum(r))
        shares = rng.lognormal(10, 1)
        keep = rng.random(T) >= suspend_frac
        ncf = rng.normal(1e8, 5e7, len(qends))
        ncl = rng.lognormal(20, 1, len(qends))
        eq = rng.lognormal(21, 1, len(qends))
        dta = rng.uniform(20, 80, len(qends))
        qp = rng.normal(10, 30, len(qends))
        qs = rng.normal(8, 20, len(qends))
        for t in range(T):
            if not keep[t]:
                continue
            k = np.searchsorted(qends, dates[t] - pd.Timedelta(days=45)) - 1
            k = max(k, 0)
            rows.append((code, dates[t], close[t], close[t] * shares, close[t] * shares * 0.7,
                         rng.uniform(0.5, 8), rng.uniform(0.1, 5), rng.uniform(5, 60),
                         ncf[k], qends[k], ncl[k], eq[k], dta[k], qp[k], qs[k]))
    prices = pd.DataFrame(rows, columns=["ts_code", "trade_date", "close", "total_mv", "circ_mv", "pb",
                                         "turnover_rate", "pe_ttm", "n_cashflow_act", "end_date",
                                         "total_ncl", "total_hldr_eqy_inc_min_int", "debt_to_assets",
                                         "q_profit_yoy", "q_sales_yoy"])
    for c in ["close", "total_mv", "circ_mv", "pb", "turnover_rate", "pe_ttm"]:
        prices[c] = prices[c].astype(np.float32).astype(np.float64)  # reference downcasts (Q27)
    index = pd.DataFrame({"ts_code": "000300.SH", "trade_date": dates, "close": idx_close})
    codes = prices["ts_code"].unique()
    sw = pd.DataFrame({"ts_code": codes, "l1_code": [f"80{j % n_ind:04d}.SI" for j in range(len(codes))],
                       "l1_name": [f"industry_{j % n_ind}" for j in range(len(codes))],
                       "in_date": "20000101", "out_date": None, "is_new": "Y"})
    return prices, index, sw


def synthetic_prices_fast(N: int = 5000, T: int = 2520, seed: int = 0, n_ind: int = 31,
                          suspend_frac: float = 0.0, start: str = "2019-01-02"):
    """Vectorised :func:`synthetic_prices` for benchmark-sized panels (5000 x 2520 in seconds
    instead of minutes): same schema and the same generating model, a different random stream
    (per-field arrays instead of per-row draws), so it does not reproduce the fixtures that
    :func:`synthetic_prices` feeds."""
    rng = np.random.default_rng(seed)
    dates = pd.bdate_range(start, periods=T)
    mkt = rng.normal(0.0003, 0.012, T)
    idx_close = 3000 * np.exp(np.cumsum(mkt))
    qends = pd.date_range(dates[0] - pd.Timedelta(days=400), dates[-1], freq="QE")
    nq = len(qends)
    kq = np.maximum(np.searchsorted(qends.values, (dates - pd.Timedelta(days=45)).values) - 1, 0)
    beta = rng.uniform(0.5, 1.5, N)
    close = 10 * np.exp(np.cumsum(beta[:, None] * mkt[None, :] + rng.normal(0, 0.02, (N, T)), axis=1))
    shares = rng.lognormal(10, 1, N)
    keep = (rng.random((N, T)) >= suspend_frac).ravel()
    q = {name: gen for name, gen in (("n_cashflow_act", rng.normal(1e8, 5e7, (N, nq))),
                                     ("total_ncl", rng.lognormal(20, 1, (N, nq))),
                                     ("total_hldr_eqy_inc_min_int", rng.lognormal(21, 1, (N, nq))),
                                     ("debt_to_assets", rng.uniform(20, 80, (N, nq))),
                                     ("q_profit_yoy", rng.normal(10, 30, (N, nq))),
                                     ("q_sales_yoy", rng.normal(8, 20, (N, nq))))}
    codes = np.array([f"{600000 + i:06d}.SH" if i % 2 else f"{i:06d}.SZ" for i in range(N)])
    mv = close * shares[:, None]
    cols = {"ts_code": np.repeat(codes, T), "trade_date": np.tile(dates.values, N),
            "close": close.ravel(), "total_mv": mv.ravel(), "circ_mv": (mv * 0.7).ravel(),
            "pb": rng.uniform(0.5, 8, N * T), "turnover_rate": rng.uniform(0.1, 5, N * T),
            "pe_ttm": rng.uniform(5, 60, N * T), "n_cashflow_act": q["n_cashflow_act"][:, kq].ravel(),
            "end_date": np.tile(qends.values[kq], N)}
    for name in ("total_ncl", "total_hldr_eqy_inc_min_int", "debt_to_assets", "q_profit_yoy",
                 "q_sales_yoy"):
        cols[name] = q[name][:, kq].ravel()
    prices = pd.DataFrame({k: v[keep] for k, v in cols.items()})
    for c in ["close", "total_mv", "circ_mv", "pb", "turnover_rate", "pe_ttm"]:
        prices[c] = prices[c].astype(np.float32).astype(np.float64)  # reference downcasts (Q27)
    index = pd.DataFrame({"ts_code": "000300.SH", "trade_date": dates, "close": idx_close})
    sw = pd.DataFrame({"ts_code": codes, "l1_code": [f"80{j % n_ind:04d}.SI" for j in range(N)],
                       "l1_name": [f"industry_{j % n_ind}" for j in range(N)],
                       "in_date": "20000101", "out_date": None, "is_new": "Y"})
    return prices, index, sw
