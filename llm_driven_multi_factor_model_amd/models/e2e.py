"""In-HBM end-to-end job: prices -> descriptors -> Barra exposures -> risk model -> results.

The reference runs two programs joined by a CSV file: ``Barra_factor_cal/main.py:42-158``
writes ``barra_data_csi.csv`` and ``Barra-master/demo.py:22-96`` reads it back, one-hot encodes
the industries, drops NaN rows and runs ``MFM``.  Here the whole job stays on the device:

1. :class:`DeviceFactorEngine` builds the master panel (sorted by stock, then date) from the
   native CSV reader's columnar buffers with device sorts: stock codes are fixed-width bytes
   compared as big-endian integers (lexicographic = the reference's string order), dates are
   YYYYMMDD integers, and no per-row Python object is ever created (the pandas master frame
   of :class:`FactorEngine` cost ~70 % of the factor pipeline's host time);
2. descriptors and post-processing run on device tensors (``factor_engine.postprocess_columns``);
3. :func:`risk_panel` turns the exported columns into a :class:`RiskPanel` with the demo.py
   semantics (t+1 return, industry id against ``industry_info``, rows with any NaN dropped,
   dates / stocks that keep at least one row) by scattering rows into the [D, Q, N] grid;
4. :class:`RiskModel` runs its four stages and ``write_risk_results`` writes the five CSVs.

The panel equals the one ``panel_from_barra_csv`` builds from the exported CSV bit for bit
(every value is a float32 descriptor widened to float64, which the CSV round trip preserves),
so results equal the two-step path.  ``barra_data_csi.csv`` is written only on request.
"""
from __future__ import annotations

import logging
import os
import time

import numpy as np
import pandas as pd
import torch

from ..ops import rolling as RL
from ..ops import xs_reduce as XR
from ..utils.config import FactorConfig, RiskConfig
from .factor_engine import (BARRA_OUTPUT_COLUMNS, BARRA_RENAME, FACTORS_TO_RUN, FactorEngine,
                            next_return, postprocess_columns)
from .panel import RiskPanel

log = logging.getLogger("mfa.e2e")

PRICE_STRING_COLS = ("ts_code",)
PRICE_DATE_COLS = ("trade_date", "end_date")
STYLE_COLUMNS = BARRA_OUTPUT_COLUMNS[5:]  # size ... leverage (demo.py's Q = 10 styles)


class NeedsPandasPath(Exception):
    """Input the device path does not model (duplicate (stock, date) rows, a stock whose
    statement runs break the point-in-time order): use :class:`FactorEngine`."""


def _s16_keys(a: np.ndarray):
    """(hi, lo) int64 keys of fixed-width byte strings whose numeric order is the strings'
    lexicographic order (big-endian words; ASCII keeps the sign bit clear)."""
    a = np.ascontiguousarray(a, dtype="S16")
    w = a.view(">u8").reshape(-1, 2)
    return w[:, 0].astype(np.int64), w[:, 1].astype(np.int64)


def _upload(x: np.ndarray, dev) -> torch.Tensor:
    """Host array -> device tensor; asynchronous when the array lives in pinned memory (the
    native reader's staging buffers)."""
    t = torch.from_numpy(np.ascontiguousarray(x))
    if dev.type != "cuda":
        return t.clone()  # never alias the caller's buffers
    return t.to(dev, non_blocking=t.is_pinned())


_BE_SHIFTS = {}


def _s16_keys_device(code_u8: torch.Tensor):
    """(hi, lo) int64 keys of [R * 16] code bytes (NUL padded), formed on the device: each 8-byte
    half read big-endian, so integer order is the strings' lexicographic order (ASCII keeps the
    sign bit clear).  Same keys as :func:`_s16_keys`."""
    b = code_u8.view(-1, 2, 8).to(torch.int64)
    sh = _BE_SHIFTS.get(b.device)
    if sh is None:
        sh = _BE_SHIFTS[b.device] = torch.arange(56, -8, -8, dtype=torch.int64, device=b.device)
    k = (b << sh).sum(-1)            # disjoint byte fields: the sum is the bitwise OR
    return k[:, 0].contiguous(), k[:, 1].contiguous()


def _unique_pairs(hi: torch.Tensor, lo: torch.Tensor):
    """Sorted unique (hi, lo) pairs on the device: (codes per row, index of one row per
    unique key, in key order)."""
    o1 = torch.argsort(lo, stable=True)
    perm = o1[torch.argsort(hi[o1], stable=True)]
    hs, ls = hi[perm], lo[perm]
    new = torch.ones(hs.numel(), dtype=torch.bool, device=hs.device)
    if hs.numel() > 1:
        new[1:] = (hs[1:] != hs[:-1]) | (ls[1:] != ls[:-1])
    rank = torch.cumsum(new.to(torch.int64), 0) - 1
    codes = torch.empty_like(rank)
    codes[perm] = rank
    return codes, perm[new]


def _ymd_to_datetime64(v: np.ndarray) -> np.ndarray:
    """YYYYMMDD ints -> datetime64[ns] (vectorised calendar arithmetic: pd.to_datetime on the
    string forms took ~2 ms for 2,500 dates)."""
    v = np.asarray(v, dtype=np.int64)
    y, m, d = v // 10000, v // 100 % 100, v % 100
    out = ((y - 1970).astype("datetime64[Y]") + (m - 1).astype("timedelta64[M]")).astype(
        "datetime64[D]") + (d - 1).astype("timedelta64[D]")
    if ((m < 1) | (m > 12) | (d < 1) | (d > 31)).any() or (
            (out.astype("datetime64[M]") - (y - 1970).astype("datetime64[Y]")).astype(np.int64) != m - 1).any():
        raise ValueError("invalid YYYYMMDD date")
    return out.astype("datetime64[ns]")


def _device_gather(srcs, ranges, offs, Rk, dev):
    """Row ranges of pinned host columns straight into device tensors (mfa_gather_host_ranges);
    None when not on a GPU, a column is not in pinned memory or has an unsupported width."""
    if dev.type != "cuda" or not srcs:
        return None
    try:
        pinned = all(torch.from_numpy(np.ascontiguousarray(x)).is_pinned() for x in srcs)
    except (TypeError, RuntimeError):
        return None
    if not pinned or any(x.dtype.itemsize not in (4, 8) or not x.flags.c_contiguous for x in srcs):
        return None
    from .. import _native
    import ctypes as C
    n = len(srcs)
    outs = [torch.empty(Rk, dtype=_TORCH_OF_NP[x.dtype.type], device=dev) for x in srcs]
    rg = torch.from_numpy(np.ascontiguousarray(ranges, dtype=np.int64)).to(dev)
    of = torch.from_numpy(np.ascontiguousarray(offs[:-1], dtype=np.int64)).to(dev)
    src_p = (C.c_void_p * n)(*[x.ctypes.data for x in srcs])
    dst_p = (C.c_void_p * n)(*[o.data_ptr() for o in outs])
    el = (C.c_int * n)(*[x.dtype.itemsize for x in srcs])
    rc = _native.lib().mfa_gather_host_ranges(src_p, dst_p, el, n, _native.ptr(rg), _native.ptr(of),
                                              int(rg.shape[0]), _native.stream(dev))
    return outs if rc == 0 else None


_TORCH_OF_NP = {np.float32: torch.float32, np.float64: torch.float64, np.int32: torch.int32,
                np.int64: torch.int64}


class DeviceFactorEngine(FactorEngine):
    """:class:`FactorEngine` whose master panel is built on the device from columnar arrays.

    ``prices``: {column: ndarray} with ``ts_code`` as ``S16`` bytes, ``trade_date`` (and
    ``end_date``) as int YYYYMMDD (-1 = missing), numeric columns float64 — the layout of
    ``utils.native_io.read_columns``.  ``index``: {``trade_date``: int YYYYMMDD, ``close``}.
    Same descriptors as ``FactorEngine(prices_df, index_df)`` on the equivalent frames (test:
    ``tests/test_e2e.py``); ``master`` is None (no pandas frame).
    """

    def __init__(self, prices: dict, index: dict, device=None, config: FactorConfig | None = None):
        self.cfg = config or FactorConfig()
        self.device = torch.device(device) if device is not None else torch.device(
            os.environ.get("MFA_DEVICE") or ("cuda:0" if torch.cuda.is_available() else "cpu"))
        t0 = time.perf_counter()
        self.master = None
        self._prepare_arrays(prices, index)
        self.prep_s = time.perf_counter() - t0
        self.own = None

    def _prepare_arrays(self, prices: dict, index: dict) -> None:
        from ..utils import native_io
        ix = prices.get(native_io.ROW_INDEX)
        if ix is not None and ix.rows == len(prices["ts_code"]) and ix.seg_first.size:
            self._prepare_indexed(prices, index, ix)
            return
        dev = self.device
        # every host -> device copy is issued first (asynchronous from the reader's pinned
        # buffers), in the dtype the reader produced: float32 loader columns (the reference's
        # load downcast, Q27) move half the bytes of float64; codes go up as raw S16 bytes and
        # dates as int32, and their keys are formed on the device
        code = _upload(np.ascontiguousarray(prices["ts_code"], dtype="S16").view(np.uint8), dev)
        td32 = _upload(np.asarray(prices["trade_date"]), dev)
        up = {c: _upload(np.asarray(prices[c]), dev) for c in self.NUMERIC if c in prices}
        ed = _upload(np.asarray(prices["end_date"]), dev) if "end_date" in prices else None
        hi, lo = _s16_keys_device(code)
        scodes, srep = _unique_pairs(hi, lo)                 # one sync (N)
        td = td32.long()
        dvals, dcodes = torch.unique(td, sorted=True, return_inverse=True)  # one sync (D)
        D = int(dvals.numel())
        key = scodes * D + dcodes
        R = int(key.numel())
        # input checks gathered into ONE host read: missing dates, sortedness, duplicates
        chk = torch.zeros(3, dtype=torch.bool, device=dev)
        chk[0] = (td < 0).any() if R else False
        if R > 1:
            chk[1] = (key[1:] < key[:-1]).any()
            chk[2] = (key[1:] == key[:-1]).any()
        missing, unsorted, dup = chk.tolist()
        if missing:
            raise NeedsPandasPath("missing trade_date")
        order = None
        if unsorted:
            order = torch.argsort(key, stable=True)      # _prepare_data's (ts_code, trade_date) sort
            key = key[order]
            dup = bool((key[1:] == key[:-1]).any())
        if dup:
            raise NeedsPandasPath("duplicate (ts_code, trade_date) rows")
        perm = (lambda x: x[order]) if order is not None else (lambda x: x)
        names = np.asarray(prices["ts_code"], dtype="S16")[srep.cpu().numpy()]
        self._finish_arrays(perm(scodes).to(torch.int32), perm(dcodes).to(torch.int32), names,
                            dvals.cpu().numpy(), {c: perm(x) for c, x in up.items()},
                            None if ed is None else perm(ed.long()), index)

    def _prepare_indexed(self, prices: dict, index: dict, ix) -> None:
        """The build from the reader's row-group index (``native_io.RowIndex``: segment starts in
        ascending code order, the sorted trade-date set, the (code, date) order checked while
        parsing): the stock ids are the segment ranks expanded on the device and the date ids a
        device searchsorted, so the 16-byte code column never crosses PCIe and no device
        unique / sort / order check runs.  Same ids, axes and columns as the key-based build."""
        dev = self.device
        codes = np.asarray(prices["ts_code"])
        td32 = _upload(np.asarray(prices["trade_date"]), dev)
        up = {c: _upload(np.asarray(prices[c]), dev) for c in self.NUMERIC if c in prices}
        ed = _upload(np.asarray(prices["end_date"]), dev) if "end_date" in prices else None
        R = int(codes.size)
        sf = np.ascontiguousarray(ix.seg_first, dtype=np.int64)
        N = int(sf.size)
        lens = torch.from_numpy(np.diff(np.append(sf, R))).to(dev)
        sid = torch.repeat_interleave(torch.arange(N, dtype=torch.int32, device=dev), lens,
                                      output_size=R)
        dv = np.asarray(ix.dates)
        did = torch.searchsorted(torch.from_numpy(dv.astype(np.int64)).to(dev),
                                 td32.long()).to(torch.int32)
        self._finish_arrays(sid, did, codes[sf].astype("S16"), dv, up,
                            None if ed is None else ed.long(), index)

    def _finish_arrays(self, stock_id, date_id, names, dv, cols, end_date, index) -> None:
        """Common tail of the full and the host-sharded builds: the global stock / date axes
        (``names`` S16 codes in id order, ``dv`` YYYYMMDD ints in id order), the per-row ids and
        columns already on the device, market returns, stock returns."""
        dev = self.device
        self.R, self.D = int(stock_id.numel()), int(len(dv))
        self.N = int(names.size)
        # the label indexes are built on first use (the writers need them, the device pipeline
        # does not): 6.5 ms of host string work at 5000 x 2520
        self._names_s16 = names
        self._stock_names = self._date_names = None
        self.date_ints = dv
        self.stock_id = stock_id
        self.date_id = date_id
        self.seg_lo = RL.seg_lo_from_codes(self.stock_id)
        self.grid_idx = self.date_id.long() * self.N + self.stock_id.long()
        # market_ret: the index close's pct_change (float64), looked up by date, then float32 as
        # every loaded column (load_data.py:18-21, Q27)
        it = np.asarray(index["trade_date"], dtype=np.int64)
        ic = np.asarray(index["close"], dtype=np.float64)
        if len(np.unique(it)) != len(it):
            raise NeedsPandasPath("duplicate index dates")
        io = np.argsort(it, kind="stable")
        it, ic = it[io], ic[io]
        mr_idx = np.full(len(ic), np.nan)
        if len(ic) > 1:
            mr_idx[1:] = ic[1:] / ic[:-1] - 1.0
        pos = np.searchsorted(it, dv)
        hit = (pos < len(it)) & (it[np.minimum(pos, len(it) - 1)] == dv)
        mr_date = np.where(hit, mr_idx[np.minimum(pos, len(it) - 1)], np.nan)
        mr = torch.from_numpy(mr_date).to(dev)[self.date_id.long()]
        self.cols = {c: x.to(torch.float32) for c, x in cols.items()}
        self.cols["market_ret"] = mr.to(torch.float32)
        self.cols["ret"], self.cols["log_ret"] = RL.returns(self.cols["close"], self.seg_lo)
        self.end_date = end_date

    @property
    def stock_names(self) -> pd.Index:
        if self._stock_names is None:
            self._stock_names = pd.Index(self._names_s16.astype("U16").astype(object))
        return self._stock_names

    @stock_names.setter
    def stock_names(self, v) -> None:
        self._stock_names = v

    @property
    def date_names(self) -> pd.Index:
        """YYYY/MM/DD labels of the date axis."""
        if self._date_names is None:
            dv = np.asarray(self.date_ints)
            y, m, d = dv // 10000, dv // 100 % 100, dv % 100
            self._date_names = pd.Index(np.char.add(np.char.add(np.char.add(
                np.char.zfill(y.astype(str), 4), "/"), np.char.add(np.char.zfill(m.astype(str), 2), "/")),
                np.char.zfill(d.astype(str), 2)).astype(object))
        return self._date_names

    @date_names.setter
    def date_names(self, v) -> None:
        self._date_names = v

    # ------------------------------------------------------------ host-side date sharding
    @classmethod
    def from_host_shard(cls, prices: dict, index: dict, rank: int, world: int, device=None,
                        config: FactorConfig | None = None, timing: bool = False):
        """The rows of date block ``rank`` of ``world`` -- exactly what ``DeviceFactorEngine(
        prices, index).date_shard(*shard_range(D, rank, world))`` keeps (its owned dates, each
        stock's ``halo_rows()`` preceding rows, plus the statement rows of the four most recent
        distinct end dates before them), selected on the HOST so a rank uploads and builds only
        its share instead of the whole master.

        The selection runs on the loader's row-group index (``native_io.RowIndex``: the first
        row of every stock and the trade-date set), which the CSV reader builds while it parses
        (``prices[native_io.ROW_INDEX]``); for columns from elsewhere it is built here in one
        threaded pass.  Per stock, binary searches find the kept range
        (``csrc_host/shard_rows.cpp``); global stock ids (segment ranks) and the global date axis
        come from the index, so every rank numbers stocks and dates identically without a
        collective.  None when the loader rows are not sorted by (code, date) or the native
        library is missing (the caller builds the full master and calls :meth:`date_shard`).
        ``timing``: synchronise the device at each sub-step of ``host_times`` (profiling)."""
        from ..parallel.dist import shard_range
        from ..utils import native_io
        cfg = config or FactorConfig()
        if "ts_code" not in prices or "trade_date" not in prices:
            return None
        codes = np.asarray(prices["ts_code"])
        if codes.dtype != np.dtype("S16"):
            return None
        ht = {}
        t0 = time.perf_counter()
        ix = prices.get(native_io.ROW_INDEX)
        if ix is not None and ix.rows != codes.size:
            ix = None   # the columns changed since the index was built
        ht["index"] = "reader" if ix is not None else "scan"
        if ix is None:
            ix = native_io.row_index(codes, prices["trade_date"])
            if ix is None:
                return None
        dv = ix.dates
        D = int(dv.size)
        if D == 0:
            return None
        lo, hi = shard_range(D, rank, world)
        big = np.iinfo(np.int32).max
        date_lo = int(dv[lo]) if lo < D else big
        date_hi = int(dv[hi]) if hi < D else big
        halo = FactorEngine.halo_rows(type("C", (), {"cfg": cfg})())
        ranges, seg_id = native_io.shard_rows_ix(ix, prices["trade_date"], prices.get("end_date"),
                                                 date_lo, date_hi, halo)
        seg_first = ix.seg_first
        ht["select_s"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        lens = ranges[:, 1] - ranges[:, 0]
        offs = np.zeros(lens.size + 1, np.int64)
        np.cumsum(lens, out=offs[1:])
        Rk = int(offs[-1])
        eng = object.__new__(cls)
        eng.cfg = cfg
        eng.device = torch.device(device) if device is not None else torch.device(
            os.environ.get("MFA_DEVICE") or ("cuda:0" if torch.cuda.is_available() else "cpu"))
        dev = eng.device
        sync = (lambda: torch.cuda.synchronize(dev)) if timing and dev.type == "cuda" else (lambda: None)
        # the kept rows of the columns the engine uses (codes are not needed: the stock ids come
        # from the index).  Pinned reader buffers on a GPU: the device reads the ranges straight
        # out of host memory (csrc/gather.hip, one pass over PCIe, only this rank's bytes);
        # otherwise a threaded host memcpy into pageable buffers and their upload.
        names_c = [c for c in prices if c in cls.NUMERIC or c in ("trade_date", "end_date")]
        srcs = [np.asarray(prices[c]) for c in names_c]
        dsel = _device_gather(srcs, ranges, offs, Rk, dev)
        if dsel is not None:
            sel = dict(zip(names_c, dsel))
            ht["gather"] = "device"
        else:
            sel = {c: _upload(native_io.gather_ranges(x, ranges, offs, np.empty(Rk, dtype=x.dtype)), dev)
                   for c, x in zip(names_c, srcs)}
            ht["gather"] = "host"
        sync()
        ht["gather_s"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        eng.master = None
        # per-row stock ids and full-history ordinals expanded on the device from the per-range
        # values (no host repeat of Rk rows, no sync: the output size is known)
        lt = torch.from_numpy(lens).to(dev)
        sid = torch.repeat_interleave(torch.from_numpy(seg_id).to(dev), lt, output_size=Rk)
        ord0 = torch.from_numpy(ranges[:, 0] - seg_first[seg_id] - offs[:-1]).to(dev)
        row_ord = (torch.repeat_interleave(ord0, lt, output_size=Rk)
                   + torch.arange(Rk, device=dev)).to(torch.int32)
        td = sel["trade_date"]
        up = {c: sel[c] for c in cls.NUMERIC if c in sel}
        edv = sel["end_date"].long() if "end_date" in sel else None
        did = torch.searchsorted(torch.from_numpy(dv.astype(np.int64)).to(dev), td.long()).to(torch.int32)
        names = codes[seg_first]
        sync()
        ht["ids_s"] = time.perf_counter() - t0
        t1 = time.perf_counter()
        eng._finish_arrays(sid, did, names, dv, up, edv, index)
        # each kept row's ordinal in its stock's full history (the aligned rank-invariant tiles)
        eng._row_ord = row_ord
        sync()
        ht["finish_s"] = time.perf_counter() - t1
        eng.prep_s = time.perf_counter() - t0
        ht["upload_build_s"] = eng.prep_s
        eng.own = (eng.date_id >= lo) & (eng.date_id < hi)
        eng.lo, eng.hi = lo, hi
        eng.host_shard_rows = Rk
        eng.host_times = ht
        return eng

    def _has_statements(self) -> bool:
        return "n_cashflow_act" in self.cols and self.end_date is not None

    def _copy_labels(self, sub, d_lo, d_hi) -> None:
        # still lazy in the sub-engine: its date labels come from its date_ints slice
        sub._names_s16, sub._stock_names, sub._date_names = self._names_s16, self._stock_names, None

    def _take(self, idx, d_lo=0, d_hi=None):
        sub = super()._take(idx, d_lo, d_hi)
        sub.end_date = None if self.end_date is None else self.end_date[idx]
        sub.date_ints = self.date_ints[d_lo:sub.D + d_lo]
        return sub

    # statement-row TTM (factor_calculator.py:392-410) with integer end dates on the device
    def cashflow_ttm(self) -> torch.Tensor:
        if getattr(self, "_ttm", None) is not None:
            return self._ttm
        if self.device.type == "cuda":
            # run-based kernels, one host read (the error flags) instead of three syncs
            ttm, flags = RL.ttm_runs(self.stock_id, self.end_date, self.cols["n_cashflow_act"])
            f = int(flags.item())
            if f & RL.TTM_MULTIVALUE:
                raise NeedsPandasPath("several cash-flow values for one (stock, end_date)")
            if not f & RL.TTM_RESTATED:
                self._ttm = ttm
                return ttm
        dev = self.device
        e = torch.where(self.end_date < 0, torch.full_like(self.end_date, 2 ** 62), self.end_date)
        sc = self.stock_id.to(torch.int64)
        v = self.cols["n_cashflow_act"].double()  # float32-loaded like every column
        ds, de = sc[1:] - sc[:-1], e[1:] - e[:-1]
        start = torch.ones(self.R, dtype=torch.bool, device=dev)
        start[1:] = (ds != 0) | (de != 0)
        if bool(((ds == 0) & (de < 0)).any()):
            # a restatement moved end_date backwards: distinct (stock, end_date) rows by sort
            key = sc * (2 ** 40) + torch.clamp(e, max=2 ** 40 - 1)
            uk, inv = torch.unique(key, sorted=True, return_inverse=True)
            first = torch.full((uk.numel(),), self.R, dtype=torch.int64, device=dev)
            first = first.scatter_reduce(0, inv, torch.arange(self.R, device=dev), reduce="amin")
            seg_codes = (uk // (2 ** 40)).to(torch.int32)
        else:
            inv = torch.cumsum(start.to(torch.int64), 0) - 1
            first = torch.nonzero(start).flatten()
            seg_codes = sc[first].to(torch.int32)
        vf = v[first]
        vb = vf[inv]
        if not bool(((v == vb) | (v.isnan() & vb.isnan())).all()):
            raise NeedsPandasPath("several cash-flow values for one (stock, end_date)")
        with RL.direct_kernels():   # newest-first sums, as the run kernel (ttm_rows)
            self._ttm = RL.rolling_sum(vf.float(), RL.seg_lo_from_codes(seg_codes), 4, 4).double()[inv]
        return self._ttm

    def compute_earnings_yield(self):
        if not (self._need("n_cashflow_act", "total_mv", "pe_ttm") and self._has_statements()):
            return None
        ttm = self.cashflow_ttm()
        mv = self.cols["total_mv"].double()
        nan = torch.full_like(mv, float("nan"))
        cetop = torch.where((mv > 0) & (ttm > 0), ttm / mv, nan)  # unit mix-up kept (quirk Q17)
        pe = self.cols["pe_ttm"].double()
        etop = torch.where(pe > 0, 1.0 / pe, nan)
        return {"CETOP": cetop.float(), "ETOP": etop.float()}


def industry_info(eng: FactorEngine, sw_industry: pd.DataFrame) -> tuple[pd.DataFrame, np.ndarray]:
    """main.py:129-137 ``industry_info`` (first-seen stock order, one row per industry) and
    each engine stock's SW-L1 code (object array, NaN without membership).

    The reference's left merge of the stock list with ``sw_industry`` is a positional take here
    (``sw_industry`` has one row per code -- the lookup below requires it, as the reference's
    ``get_indexer`` does), followed by the same ``drop_duplicates``: 5000 stocks in ~1 ms on
    the host instead of ~4 ms."""
    keys = np.asarray(eng.stock_names, dtype=object)
    ix = pd.Index(sw_industry["ts_code"].astype(str))
    pos = ix.get_indexer(keys)
    l1 = sw_industry["l1_code"].to_numpy(dtype=object)
    l1_stock = np.where(pos >= 0, l1[np.maximum(pos, 0)], np.nan).astype(object)
    uk = pd.unique(keys)
    upos = ix.get_indexer(uk)
    miss = upos < 0
    cols = [c for c in ["l1_code", "l1_name", "in_date"] if c in sw_industry.columns]
    data = {"ts_code": uk}
    for c in cols:
        v = sw_industry[c].to_numpy(dtype=object)[np.maximum(upos, 0)]
        v[miss] = np.nan
        data[c] = v
    info = pd.DataFrame(data)
    info = info.drop_duplicates(subset=[c for c in ["l1_code", "l1_name"] if c in info.columns]).rename(
        columns={"l1_code": "code", "l1_name": "industry_names", "in_date": "start_date"})
    info = info[[c for c in ["code", "industry_names", "start_date"] if c in info.columns]]
    return info.reset_index(drop=True), l1_stock


def export_columns(col: dict, nxt: torch.Tensor) -> dict:
    """The numeric barra_data_csi.csv columns (main.py:98-112 rename) as float64 device
    tensors: capital, ret (t+1) and the ten styles."""
    inv = {v: k for k, v in BARRA_RENAME.items()}
    out = {}
    for c in BARRA_OUTPUT_COLUMNS:
        s0 = inv.get(c, c)
        if s0 == "ret":
            out[c] = nxt
        elif s0 not in ("ts_code", "trade_date", "l1_code") and s0 in col and (s0 == c or c not in col):
            out[c] = col[s0].double()
    return out


def next_return_global(eng: FactorEngine, ret: torch.Tensor, ctx=None) -> torch.Tensor:
    """``groupby(ts_code).ret.shift(-1)`` (main.py:99) on a rank's owned rows of a date-sharded
    run.  Inside the block it is the in-rank shift; the last owned row of a stock takes the
    stock's FIRST row on the next rank that has one (a stock may skip a whole block).  One
    collective: every rank contributes [first-row value, has-a-row] per stock ([2, N] fp64)."""
    from ..parallel import dist as pdist
    nxt = next_return(eng, ret)
    if ctx is None or not ctx.enabled:
        return nxt
    dev, N, R = eng.device, eng.N, eng.R
    sid = eng.stock_id.long()
    mine = torch.zeros(2, N, dtype=torch.float64, device=dev)
    mine[0].fill_(float("nan"))
    if R:
        first = torch.ones(R, dtype=torch.bool, device=dev)
        last = torch.ones(R, dtype=torch.bool, device=dev)
        first[1:] = sid[1:] != sid[:-1]
        last[:-1] = sid[1:] != sid[:-1]
        fr = torch.nonzero(first).flatten()
        mine[0, sid[fr]] = ret.double()[fr]
        mine[1, sid[fr]] = 1.0
    allr = pdist.all_gather_rows(mine[None], ctx, [1] * ctx.world)   # [world, 2, N]
    later = allr[ctx.rank + 1:]
    if later.shape[0] and R:
        has = later[:, 1] > 0                                            # [w', N]
        which = torch.argmax(has.to(torch.int8), 0)                      # first later rank
        val = later[:, 0].gather(0, which[None]).squeeze(0)
        val = torch.where(has.any(0), val, torch.full_like(val, float("nan")))
        lr = torch.nonzero(last).flatten()
        nxt[lr] = val[sid[lr]]
    return nxt


def risk_panel(eng: FactorEngine, cols: dict, l1_stock: np.ndarray, info: pd.DataFrame,
               dtype=torch.float64, ctx=None) -> RiskPanel:
    """demo.py:22-35 on device tensors: rows with any NaN (or no industry in ``info``) are
    dropped, industries become ids into ``info``'s rows, and the rows are scattered into the
    [D, Q, N] panel over the dates / stocks that keep at least one row (the panel
    ``panel_from_barra_csv`` builds from the exported CSV).

    Date-sharded (``ctx`` enabled, ``eng`` = a rank's owned rows on its local date axis): the
    stock axis is GLOBAL -- the keep masks are max-reduced over ranks (one [N] all_reduce) so
    every rank scatters into the same columns -- and the panel's ``date_offset`` counts the
    kept dates of the ranks before (one [world] all_gather)."""
    from ..parallel import dist as pdist
    dev = eng.device
    missing = [c for c in ["capital", "ret", *STYLE_COLUMNS] if c not in cols]
    if missing:
        raise ValueError(f"exposure columns missing for the risk panel: {missing}")
    codes = info["code"].astype(str).to_numpy()
    cidx = pd.Index(codes)
    if cidx.is_unique:  # l1_stock holds str codes or NaN (no membership: never a match)
        ind_stock = cidx.get_indexer(pd.Index(l1_stock, dtype=object)).astype(np.int64)
    else:  # a code listed twice in info: the last row wins, as a dict would
        cpos = {c: i for i, c in enumerate(codes)}
        ind_stock = np.array([cpos.get(str(x), -1) if isinstance(x, str) else -1 for x in l1_stock],
                             dtype=np.int64)
    ind_row = torch.from_numpy(ind_stock).to(dev)[eng.stock_id.long()]
    keep = ind_row >= 0
    for c in ["capital", "ret", *STYLE_COLUMNS]:
        keep &= torch.isfinite(cols[c])
    sid, did = eng.stock_id.long(), eng.date_id.long()
    # dates / stocks with a kept row (an integer index_add here contends on ~5000 rows per
    # date counter: slower than the compaction + plain stores)
    dk = torch.zeros(eng.D, dtype=torch.bool, device=dev)
    sk = torch.zeros(eng.N, dtype=torch.bool, device=dev)
    dk[did[keep]] = True
    sk[sid[keep]] = True
    offset = 0
    if ctx is not None and ctx.enabled:
        ski = sk.to(torch.int32)
        pdist.all_reduce_max_(ski, ctx)
        sk = ski > 0
        kept = pdist.shard_sizes(int(dk.sum()), ctx)
        offset = sum(kept[:ctx.rank])
    dnew = torch.cumsum(dk.to(torch.int64), 0) - 1
    snew = torch.cumsum(sk.to(torch.int64), 0) - 1
    Dp, Np = int(dk.sum()), int(sk.sum())
    rows = torch.nonzero(keep).flatten()
    d_r, s_r = dnew[did[rows]], snew[sid[rows]]
    flat = d_r * Np + s_r
    Q = len(STYLE_COLUMNS)
    nan = float("nan")
    # the kept rows of every column onto the panel grids in two LDS-tiled transposes
    # (ops.xs_reduce.GridMap: the kept rows are still sorted by (stock, date)): capital + ret
    # onto [2, Dp * Np], the styles onto [Dp, Q, Np] (style q of cell (d, s) at
    # d * Q * Np + q * Np + s: column stride Np, date stride Q * Np)
    gm = XR.GridMap(s_r, d_r, Dp, Np)
    names = ["capital", "ret", *STYLE_COLUMNS]
    Xk = torch.empty(len(names), rows.numel(), dtype=dtype, device=dev)
    for k, c in enumerate(names):
        torch.index_select(cols[c].to(dtype), 0, rows, out=Xk[k])
    cr = gm.scatter(Xk[:2].contiguous())
    cap, ret = cr[0], cr[1]
    sty = torch.full((Dp, Q, Np), nan, dtype=dtype, device=dev)
    if Q:
        gm.scatter(Xk[2:].contiguous(), out=sty.view(-1), gs=Np, ds=Q * Np)
    ind = torch.full((Dp * Np,), -1, dtype=torch.int16, device=dev)
    ind[flat] = ind_row[rows].to(torch.int16)
    dmask, smask = dk.cpu().numpy(), sk.cpu().numpy()
    dates = _ymd_to_datetime64(eng.date_ints[dmask]) if hasattr(eng, "date_ints") else \
        pd.to_datetime(pd.Index(np.asarray(eng.date_names)[dmask]), format="%Y/%m/%d").to_numpy(
            dtype="datetime64[ns]")
    return RiskPanel(styles=sty, cap=cap.view(Dp, Np), ret=ret.view(Dp, Np),
                     ind=ind.view(Dp, Np) if len(info) else None, P=len(info), dates=dates,
                     stocks=np.asarray(eng.stock_names, dtype=object)[smask],
                     style_names=list(STYLE_COLUMNS),
                     industry_names=list(info["industry_names"].astype(str).to_numpy()),
                     date_offset=offset)


def barra_frame(eng: FactorEngine, cols: dict, l1_stock: np.ndarray, ctx=None,
                date_names=None) -> pd.DataFrame | None:
    """The barra_data_csi.csv frame (only built when requested: it is I/O, not compute).

    Date-sharded: every rank's owned rows go to rank 0 in ONE collective ([R_r, C + 2] fp64:
    the numeric columns, stock id and global date id) and are put back in master order
    (stock, date) by one device sort; other ranks return None.  ``date_names``: the GLOBAL
    date strings (the full engine's)."""
    from ..parallel import dist as pdist
    names = [c for c in BARRA_OUTPUT_COLUMNS if c in cols]
    sid_t, did_t = eng.stock_id.long(), eng.date_id.long()
    if ctx is not None and ctx.enabled:
        did_t = did_t + getattr(eng, "date_lo", 0)
        block = torch.stack([cols[c].double() for c in names]
                            + [sid_t.double(), did_t.double()], 1)
        full = pdist.gather_to_root(block.contiguous(), ctx)
        if full is None:
            return None
        sid_t, did_t = full[:, -2].long(), full[:, -1].long()
        order = torch.argsort(sid_t * (1 << 32) + did_t)
        full = full[order]
        sid_t, did_t = sid_t[order], did_t[order]
        host = full[:, :len(names)].T.cpu().numpy()
    else:
        host = torch.stack([cols[c] for c in names]).cpu().numpy()
    final = pd.DataFrame(host.T, columns=names, copy=False)
    sid = sid_t.cpu().numpy()
    did = did_t.cpu().numpy()
    dn = eng.date_names if date_names is None else date_names
    final.insert(0, "date", np.asarray(dn, dtype=object)[did])
    final.insert(1, "stocknames", np.asarray(eng.stock_names, dtype=object)[sid])
    final.insert(4, "industry", pd.Series(l1_stock[sid], dtype=object))
    return final[[c for c in BARRA_OUTPUT_COLUMNS if c in final.columns]]


def read_price_columns(prices_csv: str, index_csv: str):
    """Columnar parse of the loader's CSVs by the native reader: codes as S16 bytes, dates as
    YYYYMMDD ints, the engine's numeric columns float32, anything else float64.  None if the
    native reader is unavailable."""
    from ..utils import native_io
    # numeric loader columns parse straight to float32 (the reference's load downcast, Q27)
    # into pinned staging buffers when a GPU is present
    types = {c: 3 for c in FactorEngine.NUMERIC}
    types.update({c: 1 for c in PRICE_STRING_COLS})
    types.update({c: 2 for c in PRICE_DATE_COLS})
    # the parser also builds the row-group index the date-sharded ranks select their rows on
    p = native_io.read_columns(prices_csv, types, pinned=_pin_default(), index=("ts_code", "trade_date"))
    i = native_io.read_columns(index_csv, {"ts_code": 1, "trade_date": 2})
    return p, i


def _pin_default() -> bool:
    """Pinned staging when a GPU is present (``MFA_PINNED=0`` turns it off).  Off by default
    when several ranks share one device (``MFA_DIST_BACKEND`` rehearsals): four processes
    copying from pinned buffers into ONE MI355X at once measured 65 s for what takes 0.05 s
    alone, pageable copies 0.57 s (profiles/r04/README.md)."""
    if os.environ.get("MFA_PINNED"):
        return torch.cuda.is_available() and os.environ["MFA_PINNED"] != "0"
    return torch.cuda.is_available() and not os.environ.get("MFA_DIST_BACKEND")


def stage_host_columns(prices: dict, pinned: bool | None = None) -> dict:
    """The layout :func:`read_price_columns` produces, from float64 columnar arrays (e.g.
    :func:`_columns_from_frames`): the engine's numeric columns rounded to float32 (Q27), codes /
    dates / numerics in pinned host memory when a GPU is present.  This is the native reader's
    parse-time work; benchmarks count it as I/O.  That includes the row-group index
    (``native_io.ROW_INDEX``), which the reader builds while parsing: here one threaded pass over
    the staged codes and dates."""
    from ..utils import native_io
    from ..utils.native_io import _host_buffer
    pinned = _pin_default() if pinned is None else pinned
    out = {}
    for c, x in prices.items():
        if c == native_io.ROW_INDEX:
            continue
        x = np.asarray(x)
        if c in FactorEngine.NUMERIC:
            dt = np.float32
        elif x.dtype.kind == "S":
            dt = "S16"
        elif c in PRICE_DATE_COLS:
            dt = np.int32
        else:
            out[c] = x
            continue
        buf = _host_buffer(len(x), dt, pinned)
        buf[...] = x
        out[c] = buf
    if "ts_code" in out and "trade_date" in out and out["ts_code"].dtype == np.dtype("S16"):
        ix = native_io.row_index(out["ts_code"], out["trade_date"])
        if ix is not None:
            out[native_io.ROW_INDEX] = ix
    return out


def _columns_from_frames(prices_df: pd.DataFrame, index_df: pd.DataFrame):
    """The columnar layout of :class:`DeviceFactorEngine` from pandas frames (tests, API)."""
    def ymd(s):
        d = pd.to_datetime(s)
        out = (d.dt.year * 10000 + d.dt.month * 100 + d.dt.day).to_numpy(dtype=np.float64)
        return np.where(np.isnan(out), -1, out).astype(np.int64)
    p = {}
    for c in prices_df.columns:
        if c == "ts_code":
            p[c] = prices_df[c].astype(str).to_numpy().astype("S16")
        elif c in PRICE_DATE_COLS:
            p[c] = ymd(prices_df[c])
        else:
            try:
                p[c] = prices_df[c].to_numpy(dtype=np.float64, na_value=np.nan)
            except (TypeError, ValueError):
                continue
    i = {"trade_date": ymd(index_df["trade_date"]),
         "close": index_df["close"].to_numpy(dtype=np.float64)}
    return p, i


def exposures(prices, index, sw_industry: pd.DataFrame, factor_cfg: FactorConfig | None = None,
              factors=None, device=None, ctx=None, sync: bool = True):
    """``main.py:42-137`` on device tensors: descriptors -> winsorize -> composites ->
    orthogonalisation -> t+1 return -> export columns.

    Single process: every row.  Date-sharded (``ctx`` enabled, torchrun one rank per GPU):
    every rank builds the device master from the same loader columns (no collective, C2),
    keeps its balanced date block plus each stock's ``halo_rows()`` preceding rows
    (``date_shard``: the RSTR window reaches 504 rows back), runs the descriptors on that
    slice, and the per-date post-processing on its owned dates only (local [D_r, N] grid);
    the t+1 return crosses the block boundary with one [2, N] collective.

    Returns ``(eng, cols, info, l1_stock, full_eng, timings)``: ``eng`` = the rows this rank
    owns, ``cols`` = {barra column: float64 tensor over those rows}."""
    t = {}
    t0 = time.perf_counter()
    if isinstance(prices, pd.DataFrame):
        prices, index = _columns_from_frames(prices, index)
    if ctx is not None and ctx.enabled and device is None:
        device = ctx.device
    # the rolling descriptors are rank-invariant by construction (segment-anchored kernels on
    # every path): a date-sharded run equals the single-process run bit for bit at any world size
    factor_cfg = factor_cfg or FactorConfig()
    if ctx is not None and ctx.enabled:
        from ..parallel import dist as pdist
        # each rank selects, uploads and builds only its rows (host-side selection from the
        # sorted loader columns); unsorted input falls back to the full master + date_shard
        sh = DeviceFactorEngine.from_host_shard(prices, index, ctx.rank, ctx.world, device,
                                                factor_cfg) \
            if os.environ.get("MFA_HOST_SHARD", "1") != "0" else None
        if sh is None:
            full = DeviceFactorEngine(prices, index, device=device, config=factor_cfg)
            sh = full.date_shard(*pdist.shard_range(full.D, ctx.rank, ctx.world))
        else:
            full = sh  # global date axis (date_names, D) for the writers
        t["host_shard"] = getattr(sh, "host_shard_rows", None) is not None
        if t["host_shard"] and sh._has_statements():
            # a host shard forms the statement TTM on its own rows, so a statement with two
            # values may sit in one rank's rows only: the fall-back decision is collective
            # (one MAX over ranks) so no rank walks on into the collectives alone
            bad = 0.0
            try:
                sh.cashflow_ttm()
            except NeedsPandasPath:
                bad = 1.0
            if pdist.all_reduce_max(bad, ctx) > 0:
                raise NeedsPandasPath("several cash-flow values for one (stock, end_date)")
        res = sh.compute(factors or FACTORS_TO_RUN)
        own = torch.nonzero(sh.own).flatten()
        res = {k: v[own] for k, v in res.items()}
        eng = sh.owned()
        eng.timings = sh.timings
    else:
        full = DeviceFactorEngine(prices, index, device=device, config=factor_cfg)
        eng = full
        res = eng.compute(factors or FACTORS_TO_RUN)
    t["descriptors_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    col = postprocess_columns(eng, res, eng.cfg)
    nxt = next_return_global(eng, col["ret"], ctx)
    cols = export_columns(col, nxt)
    info, l1_stock = industry_info(eng, sw_industry)
    if sync and eng.device.type == "cuda":
        torch.cuda.synchronize(eng.device)
    t["postprocess_s"] = time.perf_counter() - t0
    return eng, cols, info, l1_stock, full, t


def run_factors(prices, index, sw_industry: pd.DataFrame, factor_cfg: FactorConfig | None = None,
                factors=None, device=None, ctx=None):
    """``cli factors`` (main.py) on the device path: ``(barra frame, industry_info, timings)``
    on rank 0 (``(None, None, timings)`` on the other ranks of a date-sharded run)."""
    eng, cols, info, l1_stock, full, t = exposures(prices, index, sw_industry, factor_cfg,
                                                   factors, device, ctx)
    t0 = time.perf_counter()
    frame = barra_frame(eng, cols, l1_stock, ctx, full.date_names)
    t["export_s"] = time.perf_counter() - t0
    t["kernel_ms"] = getattr(eng, "timings", {})
    if frame is None:
        return None, None, t
    return frame, info, t


def run_pipeline(prices, index, sw_industry: pd.DataFrame, risk_cfg: RiskConfig | None = None,
                 factor_cfg: FactorConfig | None = None, factors=None, device=None,
                 want_barra: bool = False, sync: bool = True, ctx=None):
    """The whole job in HBM.  ``prices`` / ``index``: columnar dicts (``read_price_columns``)
    or pandas frames.  Returns ``(model, info, barra_frame or None, timings)``; the model has
    run all four stages.

    With an enabled ``ctx`` (torchrun, one rank per GPU) the job is date-sharded end to end
    (BASELINE config 3): :func:`exposures` on the rank's block, a :class:`RiskPanel` on the
    global stock axis, and :class:`RiskModel` over the ranks' date blocks.  With the default
    ``time_scan="gather"`` every output equals the single-process run to rounding-free
    equality of the regression and 1e-12 of the scans (tests/test_e2e_dist.py); "carry" scans
    only the rank's own dates and carries block states across ranks (the Newey-West series
    then differs from one process at ~1e-11 relative, which the eigen adjustment can amplify
    where eigenvalues nearly coincide).  Nothing leaves HBM until the CSV writers gather to
    rank 0; the barra frame (``want_barra``) is returned on rank 0 only."""
    from .risk_model import RiskModel
    dist_on = ctx is not None and ctx.enabled
    eng, cols, info, l1_stock, full, t = exposures(prices, index, sw_industry, factor_cfg,
                                                   factors, device, ctx, sync)
    t0 = time.perf_counter()
    panel = risk_panel(eng, cols, l1_stock, info, ctx=ctx)
    if sync and eng.device.type == "cuda":
        torch.cuda.synchronize(eng.device)
    t["exposures_to_panel_s"] = t.pop("postprocess_s") + time.perf_counter() - t0
    t0 = time.perf_counter()
    cfg = risk_cfg or RiskConfig()
    from ..parallel import dist as pdist
    # one process: an explicit single-rank context (a torchrun job's rank may also run a
    # whole-panel pipeline of its own, e.g. tools/pipeline_dist.py's comparison)
    model = RiskModel(panel, cfg, ctx=ctx if dist_on else pdist.DistContext(device=eng.device)).run()
    if sync and eng.device.type == "cuda":
        torch.cuda.synchronize(eng.device)
    t["risk_model_s"] = time.perf_counter() - t0
    t["kernel_ms"] = getattr(eng, "timings", {})
    frame = barra_frame(eng, cols, l1_stock, ctx, full.date_names) if want_barra else None
    return model, info, frame, t
