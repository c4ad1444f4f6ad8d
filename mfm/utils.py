"""``mfm.utils`` compatibility API (reference: Barra-master/mfm/utils.py)."""
from __future__ import annotations

import math

import numpy as np
import pandas as pd
import torch

from llm_driven_multi_factor_model_amd.models.risk_model import eigenfactor_bias_stat as _bias
from llm_driven_multi_factor_model_amd.ops import eigen as _eigen
from llm_driven_multi_factor_model_amd.ops.ew_scan import newey_west_single
from llm_driven_multi_factor_model_amd.ops.xs_reduce import bayes_shrink as _bayes

from ._device import device as _device


def Newey_West(ret: pd.DataFrame, q=2, tao=252):
    """Newey-West covariance of one sample (utils.py:16-50); raises if T <= q or T <= K."""
    T, K = ret.shape
    if T <= q or T <= K:
        raise Exception("T <= q or T <= K")
    V = newey_west_single(torch.from_numpy(np.asarray(ret.values, dtype=np.float64)), q, tao)
    return pd.DataFrame(V.numpy(), columns=ret.columns, index=ret.columns)


def eigen_risk_adj(covmat: pd.DataFrame, T=1000, M=100, scale_coef=1.4, seed: int = 1):
    """Eigenfactor risk adjustment of one covariance (utils.py:55-92); raises if not PSD."""
    F0 = torch.from_numpy(np.asarray(covmat.values, dtype=np.float64))[None]
    dev = _device()
    out = _eigen.eigen_risk_adjust(F0.to(dev), M=M, scale_coef=scale_coef, T_sim=T, seed=seed)[0]
    if torch.isnan(out).any():
        raise ValueError("covariance is not symmetric positive-semidefinite")
    return pd.DataFrame(out.cpu().numpy(), columns=covmat.columns, index=covmat.columns)


def eigenfactor_bias_stat(cov, ret, predlen=1, plot: bool = False):
    """Bias statistic of eigen-factor portfolios (utils.py:97-117).  ``cov``: list of frames."""
    K = ret.shape[1]
    mats = np.stack([c.values if (isinstance(c, pd.DataFrame) and not c.empty) else np.full((K, K), np.nan)
                     for c in cov])
    b = _bias(torch.from_numpy(mats), torch.from_numpy(np.asarray(ret.values, dtype=np.float64)), predlen)
    b = b.numpy()
    if plot:
        import matplotlib.pyplot as plt
        plt.plot(b)
    return b


def progressbar(cur, total, txt):
    percent = "{:.2%}".format(cur / total)
    print("\r[%-50s] %s" % ("=" * int(math.floor(cur * 50 / total)), percent) + txt, end="")


def group_mean_std(x):
    m = sum(x.volatility * x.capital) / sum(x.capital)
    s = np.sqrt(np.mean((x.volatility - m) ** 2))
    return [m, s]


def shrink(x, group_weight_mean, q):
    a = q * np.abs(x["volatility"] - group_weight_mean[x["group"]][0])
    b = group_weight_mean[x["group"]][1]
    v = a / (a + b)
    return v * group_weight_mean[x["group"]][0] + (1 - v) * np.abs(x["volatility"])


def bayes_shrink(volatility, capital, ngroup=10, q=1):
    """Cap-decile Bayesian shrinkage (utils.py:153-168), batched kernel on the device."""
    v = torch.as_tensor(np.asarray(volatility, dtype=np.float32)).to(_device())
    c = torch.as_tensor(np.asarray(capital, dtype=np.float32)).to(_device())
    return _bayes(v, c, ngroup, q).cpu().double().numpy()
