"""Load the read-only reference implementation as a numerical oracle for parity tests.

``statsmodels`` is not installed here, so a minimal, formula-faithful stub is installed for the
duration of the import: ``DescrStatsW(x, weights).mean`` (weighted column mean), and
``statsmodels.api`` ``add_constant`` / ``WLS`` / ``OLS`` backed by a weighted least-squares
solve that reports ``params``, ``resid`` (unweighted, ``y - X b``) and ``scale``
(``sum w e^2 / (n - k)``) exactly as statsmodels defines them.

The reference's top-level package is also named ``mfm``; it is loaded under its own name and
``sys.modules`` is restored afterwards so it never shadows this repo's ``mfm`` package.
Nothing prebuilt from the reference is executed: only its ``.py`` sources.
"""
from __future__ import annotations

import importlib
import importlib.util
import os
import sys
import types
from types import SimpleNamespace

import numpy as np
import pandas as pd

REF = os.environ.get("MFA_REFERENCE", "/root/reference")


class _DescrStatsW:
    def __init__(self, data, weights=None, ddof=0):
        self.data = np.asarray(data, dtype=float)
        self.weights = np.ones(len(self.data)) if weights is None else np.asarray(weights, dtype=float)

    @property
    def mean(self):
        w = self.weights
        return (self.data * w.reshape((-1,) + (1,) * (self.data.ndim - 1))).sum(0) / w.sum()


class _Fit:
    def __init__(self, y, X, w):
        yv = np.asarray(y, dtype=float)
        Xv = np.asarray(X, dtype=float)
        sw = np.sqrt(np.asarray(w, dtype=float))
        b, *_ = np.linalg.lstsq(Xv * sw[:, None], yv * sw, rcond=None)
        e = yv - Xv @ b
        n, k = Xv.shape
        names = list(X.columns) if isinstance(X, pd.DataFrame) else list(range(k))
        idx = y.index if isinstance(y, pd.Series) else None
        self.params = pd.Series(b, index=names)
        self.resid = pd.Series(e, index=idx) if idx is not None else e
        self.scale = float((np.asarray(w) * e * e).sum() / (n - k))


class _WLS:
    def __init__(self, y, X, weights=1.0):
        self.y, self.X = y, X
        self.w = np.broadcast_to(np.asarray(weights, dtype=float), (len(y),))

    def fit(self):
        return _Fit(self.y, self.X, self.w)


class _OLS(_WLS):
    def __init__(self, y, X):
        super().__init__(y, X, 1.0)


def _add_constant(x):
    if isinstance(x, pd.Series):
        x = x.to_frame()
    if isinstance(x, pd.DataFrame):
        out = x.copy()
        out.insert(0, "const", 1.0)
        return out
    x = np.asarray(x, dtype=float)
    return np.column_stack([np.ones(len(x)), x])


def _install_statsmodels_stub():
    if "statsmodels" in sys.modules and not getattr(sys.modules["statsmodels"], "_mfa_stub", False):
        return
    sm = types.ModuleType("statsmodels"); sm._mfa_stub = True; sm.__path__ = []
    stats = types.ModuleType("statsmodels.stats"); stats.__path__ = []
    ws = types.ModuleType("statsmodels.stats.weightstats")
    ws.DescrStatsW = _DescrStatsW
    api = types.ModuleType("statsmodels.api")
    api.add_constant, api.WLS, api.OLS = _add_constant, _WLS, _OLS
    sm.stats, sm.api, stats.weightstats = stats, api, ws
    sys.modules.update({"statsmodels": sm, "statsmodels.stats": stats,
                        "statsmodels.stats.weightstats": ws, "statsmodels.api": api})


_CACHE = {}


def load_reference():
    if "ref" in _CACHE:
        return _CACHE["ref"]
    mdir = os.path.join(REF, "Barra-master", "mfm")
    if not os.path.isdir(mdir):
        return None
    _install_statsmodels_stub()
    import matplotlib
    matplotlib.use("Agg")
    saved = {k: sys.modules.pop(k) for k in list(sys.modules) if k == "mfm" or k.startswith("mfm.")}
    old_dwb = sys.dont_write_bytecode
    sys.dont_write_bytecode = True
    try:
        pkg = types.ModuleType("mfm")
        pkg.__path__ = [mdir]
        sys.modules["mfm"] = pkg
        cs = importlib.import_module("mfm.CrossSection")
        ut = importlib.import_module("mfm.utils")
        mf = importlib.import_module("mfm.MFM")
        fc_dir = os.path.join(REF, "Barra_factor_cal")
        sys.path.insert(0, fc_dir)
        try:
            fc = importlib.import_module("factor_calculator")
            pp = importlib.import_module("post_processing")
        finally:
            sys.path.remove(fc_dir)
            for k in ("factor_calculator", "post_processing"):
                sys.modules.pop(k, None)
        # legacy CSV-era twin at the repository root (/factor.py)
        legacy = None
        if os.path.isfile(os.path.join(REF, "factor.py")):
            spec = importlib.util.spec_from_file_location("_mfa_ref_legacy_factor",
                                                          os.path.join(REF, "factor.py"))
            legacy = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(legacy)
    finally:
        for k in [k for k in sys.modules if k == "mfm" or k.startswith("mfm.")]:
            sys.modules.pop(k)
        sys.modules.update(saved)
        sys.dont_write_bytecode = old_dwb
    r = SimpleNamespace(CrossSection=cs, utils=ut, MFM=mf, factor_calculator=fc, post_processing=pp,
                        legacy_factor=legacy)
    _CACHE["ref"] = r
    return r
