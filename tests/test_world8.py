"""The target world size: 8 ranks on gloo (CPU), before any 8-GPU node.

* the date-sharded end-to-end job at 8 ranks -- blocks of ~78 dates, so every block's 566-row
  descriptor halo reaches across up to 7 rank boundaries -- on both row-selection paths
  (device ``date_shard`` of the full master; host-side ``from_host_shard`` of sorted rows) and
  with the "carry" time scan, against ONE default-config process;
* the risk model at 8 ranks with fewer dates than ranks (D = 5: three ranks own no date) in
  both time-scan modes and both eigen-sharding modes (7 sims over 8 ranks: a rank with no sim);
* bench.py launched like the driver at 8 ranks, weak and strong (6 global dates: two ranks
  with no date);
* ``cli pipeline`` under torchrun with 8 ranks writing the same five result files as 1 rank.
"""
import os
import tempfile

import numpy as np
import pandas as pd
import pytest
import torch
import torch.multiprocessing as mp

from tests.test_e2e_dist import _compare, _free_port, _reference, _run

KEYS_RM = ("factor_ret", "r2", "nw_cov", "eigen_cov", "vra_cov", "vra_lambda")


def test_world8_pipeline_equals_single_process():
    """Device shard path (unsorted loader rows: full master + date_shard on every rank)."""
    model, frame, info = _reference("cpu")
    got = _run(8, "cpu")
    _compare(got, model, frame, info, rtol=1e-12, atol=1e-15, frame_rtol=1e-12, frame_atol=0)


def test_world8_pipeline_host_shard_equals_single_process():
    """Host shard path (sorted loader rows: every rank selects and uploads only its rows)."""
    model, frame, info = _reference("cpu")
    got = _run(8, "cpu", sorted_rows=True)
    _compare(got, model, frame, info, rtol=1e-12, atol=1e-15, frame_rtol=1e-12, frame_atol=0)


def test_world8_pipeline_carry_scan():
    model, frame, info = _reference("cpu")
    got = _run(8, "cpu", "carry")
    _compare(got, model, frame, info, rtol=0, atol=0, frame_rtol=1e-12, frame_atol=0,
             keys=("factor_ret", "r2", "specific_ret"))
    torch.testing.assert_close(got["nw_cov"], model.nw_cov, rtol=1e-9, atol=1e-12, equal_nan=True)


def _rm_worker(rank, world, port, out_path, D, scan, shard):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MFA_DIST_TIMEOUT_S="120")
    from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel
    from llm_driven_multi_factor_model_amd.models.risk_model import RiskModel
    from llm_driven_multi_factor_model_amd.parallel import dist as pdist
    from llm_driven_multi_factor_model_amd.utils.config import preset
    ctx = pdist.init_distributed(device="cpu")
    full = synthetic_panel(40, D, 3, 3, seed=4, missing_frac=0.05)
    a, b = pdist.shard_range(full.D, ctx.rank, ctx.world)
    cfg = preset("reference", eigen_sims=7, eigen_shard=shard, eigen_chunk=3, time_scan=scan)
    m = RiskModel(full.slice_dates(a, b), cfg, T_global=full.D, ctx=ctx)
    m.run()
    out = {k: pdist.gather_to_root(getattr(m, k).contiguous(), ctx) for k in KEYS_RM}
    if ctx.rank == 0:
        torch.save(out, out_path)
    pdist.barrier(ctx)
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("D", [5, 60])
@pytest.mark.parametrize("scan,shard", [("gather", "dates"), ("carry", "dates"), ("gather", "sims")])
def test_world8_risk_model(D, scan, shard):
    """D = 5 < 8 ranks: ranks 5-7 own no date and still take part in every collective."""
    from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel
    from llm_driven_multi_factor_model_amd.models.risk_model import RiskModel
    from llm_driven_multi_factor_model_amd.utils.config import preset
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "rm.pt")
        mp.spawn(_rm_worker, args=(8, _free_port(), path, D, scan, shard), nprocs=8, join=True)
        got = torch.load(path, weights_only=True)
    m = RiskModel(synthetic_panel(40, D, 3, 3, seed=4, missing_frac=0.05),
                  preset("reference", eigen_sims=7))
    m.run()
    for k in KEYS_RM:
        ref = getattr(m, k)
        tol = (1e-9, 1e-12) if scan == "carry" and k != "factor_ret" and k != "r2" else (1e-12, 1e-15)
        if scan == "carry" and k in ("eigen_cov", "vra_cov", "vra_lambda"):
            continue   # the carry scan's ~1e-11 NW reordering is amplified by the eigen stage
        torch.testing.assert_close(got[k], ref, rtol=tol[0], atol=tol[1], equal_nan=True, msg=k)


def test_world8_bench_contract():
    from tests.test_bench_contract import _run as bench
    r = bench(8)
    assert r["n_gpus"] == 8 and r["config"]["parallelism"] == "dp8"
    assert r["config"]["global_batch"] == 48
    s = r["strong"]   # 6 global dates over 8 ranks: ranks 6 and 7 own none
    assert s["global_dates"] == 6 and s["value"] > 0
    r = bench(8, ["--scaling", "strong"])
    assert r["scaling"] == "strong" and r["config"]["global_batch"] == 6


def test_world8_cli_pipeline(tmp_path):
    from tests.test_e2e_dist import _data, _torchrun_cli
    prices, index, sw = _data()
    d = tmp_path
    prices.to_csv(d / "prices.csv", index=False)
    index.to_csv(d / "index.csv", index=False)
    sw.to_csv(d / "sw.csv", index=False)
    common = ["--prices", str(d / "prices.csv"), "--index", str(d / "index.csv"),
              "--industry", str(d / "sw.csv")]
    for n in (1, 8):
        r = _torchrun_cli(n, "pipeline", *common, "--out", str(d / f"res{n}"), "--sims", "3",
                          "--device", "cpu")
        assert r.returncode == 0, r.stderr[-3000:]
    for f in ("factor_returns.csv", "r_squared.csv", "specific_returns.csv",
              "final_vol_regime_adj_covariance.csv", "volatility_multiplier_lambda.csv"):
        a = pd.read_csv(d / "res1" / f, index_col=0)
        b = pd.read_csv(d / "res8" / f, index_col=0)
        assert list(a.columns) == list(b.columns) and list(a.index) == list(b.index), f
        np.testing.assert_allclose(b.to_numpy(np.float64), a.to_numpy(np.float64), rtol=1e-12,
                                   atol=1e-15, err_msg=f)
