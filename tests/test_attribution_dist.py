"""Rank-invariant risk attribution and eigenfactor bias statistic.

The shrunk specific volatility behind ``RiskModel.risk_attribution`` is point in time: date t
uses the trailing window of specific returns ending at t, across rank boundaries via a halo,
and every window is summed in a fixed order.  So a 2- or 3-rank gloo run must reproduce the
one-process attribution (and the CLI's ``risk_attribution.csv`` / ``eigenfactor_bias.csv``) to
1e-12, also for ``preset("bootstrap10k")`` (sims sharded over ranks, BASELINE config 5).
"""
import os
import socket
import subprocess
import sys
import tempfile

import numpy as np
import pandas as pd
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _panel():
    from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel
    return synthetic_panel(37, 64, 4, 3, seed=21, missing_frac=0.05)


def _cfg(name):
    from llm_driven_multi_factor_model_amd.utils.config import preset
    if name == "bootstrap10k":  # the preset's sharding, with few sims (CPU)
        return preset("bootstrap10k", eigen_sims=9, eigen_chunk=4, time_scan="carry")
    return preset("reference", eigen_sims=5)


def _outputs(m):
    h = torch.full((m.panel.N,), 1.0 / m.panel.N, dtype=torch.float64)
    h[::3] *= 2.0
    r = m.risk_attribution(h)
    g = r.grouped(m.panel.P)
    vol = m.specific_vol_series(window=10)
    out = dict(total=r.total_var, factor=r.factor_var, specific=r.specific_var,
               contrib=r.contrib, style=g["style"], vol=vol,
               shrunk=m.specific_risk_shrunk(window=10))
    return out, m.specific_risk_shrunk(window=10, per_date=False), \
        m.eigenfactor_bias("eigen", start=5, predlen=3)


def _worker(rank, world, port, path, name):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from llm_driven_multi_factor_model_amd.models.risk_model import RiskModel
    from llm_driven_multi_factor_model_amd.parallel import dist as pdist
    ctx = pdist.init_distributed(device="cpu")
    full = _panel()
    a, b = pdist.shard_range(full.D, ctx.rank, ctx.world)
    m = RiskModel(full.slice_dates(a, b), _cfg(name), T_global=full.D, ctx=ctx).run()
    per, last, bias = _outputs(m)
    got = {k: pdist.gather_to_root(v.contiguous(), ctx) for k, v in per.items()}
    # the last-date vector and the bias statistic are returned on EVERY rank
    lasts = pdist.all_gather_rows(last[None].contiguous(), ctx)
    biases = pdist.all_gather_rows(bias[None].contiguous(), ctx)
    if ctx.rank == 0:
        got.update(lasts=lasts, biases=biases)
        torch.save(got, path)
    pdist.barrier(ctx)
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("name", ["reference", "bootstrap10k"])
def test_attribution_rank_invariant(world, name):
    from llm_driven_multi_factor_model_amd.models.risk_model import RiskModel
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "att.pt")
        mp.spawn(_worker, args=(world, _free_port(), path, name), nprocs=world, join=True)
        got = torch.load(path, weights_only=True)
    m = RiskModel(_panel(), _cfg(name)).run()
    per, last, bias = _outputs(m)
    for k, v in per.items():
        torch.testing.assert_close(got[k], v, rtol=1e-12, atol=1e-15, equal_nan=True, msg=k)
    for r in range(world):
        torch.testing.assert_close(got["lasts"][r], last, rtol=1e-12, atol=1e-15, equal_nan=True)
        torch.testing.assert_close(got["biases"][r], bias, rtol=1e-12, atol=1e-15)
    assert torch.isfinite(bias).all()
    # point in time: date t's vol uses dates <= t only (changing a later date changes nothing)
    assert torch.isfinite(per["shrunk"][-1]).any()


def test_specific_vol_is_point_in_time():
    from llm_driven_multi_factor_model_amd.models.risk_model import RiskModel
    m = RiskModel(_panel(), _cfg("reference"))
    m.regress()
    v0 = m.specific_vol_series(window=8)
    m.specific_ret = m.specific_ret.clone()
    m.specific_ret[20:] = 0.5  # rewrite the future of date 19
    v1 = m.specific_vol_series(window=8)
    torch.testing.assert_close(v1[:20], v0[:20], rtol=0, atol=0, equal_nan=True)
    # direct check of one window
    e = m.specific_ret[12:20].double()
    ok = torch.isfinite(e)
    n = ok.sum(0)
    x = torch.where(ok, e, torch.zeros_like(e))
    var = (x * x).sum(0) / n - ((x.sum(0) / n) ** 2)
    torch.testing.assert_close(v1[19], torch.sqrt(var.clamp(min=0)), rtol=1e-12, atol=1e-15,
                               equal_nan=True)


def _cli(args, world=1):
    if world == 1:
        cmd = [sys.executable, "-m", "llm_driven_multi_factor_model_amd.cli", *args]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={world}", "--master-addr", "127.0.0.1", "--master-port",
               str(_free_port()), "-m", "llm_driven_multi_factor_model_amd.cli", *args]
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    return subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)


def test_cli_attribution_and_bias_stat_equal_across_ranks(tmp_path):
    d = str(tmp_path)
    r = _cli(["synth", "--out", d, "--dates", "45", "--stocks", "70", "--industries", "5"])
    assert r.returncode == 0, r.stderr
    outs = {}
    for world in (1, 2):
        o = f"{d}/res{world}"
        r = _cli(["risk", "--data", f"{d}/barra_data_csi.csv", "--industry",
                  f"{d}/industry_info.csv", "--out", o, "--sims", "4", "--attribution", "equal",
                  "--bias-stat", "5", "--bias-start", "10", "--time-scan", "carry",
                  "--device", "cpu"], world)
        assert r.returncode == 0, r.stderr[-3000:]
        outs[world] = (pd.read_csv(f"{o}/risk_attribution.csv", index_col=0),
                       pd.read_csv(f"{o}/eigenfactor_bias.csv", index_col=0))
    for a, b in zip(outs[1], outs[2]):
        assert list(a.columns) == list(b.columns) and a.shape == b.shape
        np.testing.assert_allclose(b.values, a.values, rtol=1e-12, atol=1e-15)
    bias = outs[1][1]
    assert list(bias.columns) == ["bias_nw", "bias_eigen", "bias_vra"]
    assert np.isfinite(bias.values).all()
