"""Date-sharded factor pipeline (DP over dates, rolling stages with a halo).

The owned rows of every date block, computed on the block plus each stock's ``halo_rows()``
preceding rows, must equal the full-panel descriptors; a 2-rank gloo run of the whole pipeline
(descriptors -> winsorize -> composite -> orthogonalize -> gather -> export) must equal the
single-process export.
"""
import os
import socket
import tempfile

import numpy as np
import pandas as pd
import pytest
import torch
import torch.multiprocessing as mp

from llm_driven_multi_factor_model_amd.models import factor_engine as FE

# 700 dates: with 2-3 blocks every later block needs the 504-row RSTR halo
N, T, SEED = 12, 700, 5


def _data():
    return FE.synthetic_prices(N=N, T=T, seed=SEED, suspend_frac=0.04)


def _check_blocks(device, nblk, rtol, atol, cfg=None):
    prices, index, _ = _data()
    eng = FE.FactorEngine(prices, index, device=device, config=cfg)
    full = eng.run(FE.FACTORS_TO_RUN)
    parts = []
    for r in range(nblk):
        lo, hi = (eng.D * r) // nblk, (eng.D * (r + 1)) // nblk
        sh = eng.date_shard(lo, hi)
        assert sh.R < eng.R or r > 0  # later blocks may reach back to row 0 through the halo
        parts.append(sh.run(FE.FACTORS_TO_RUN))
    got = pd.concat(parts, ignore_index=True).sort_values(["ts_code", "trade_date"], kind="stable")
    got = got.reset_index(drop=True)
    assert len(got) == len(full)
    assert (got["ts_code"].values == full["ts_code"].values).all()
    assert (got["trade_date"].values == full["trade_date"].values).all()
    for c in full.columns[2:]:
        if rtol == 0 and atol == 0:  # bitwise (NaN where NaN)
            np.testing.assert_array_equal(got[c].values, full[c].values, err_msg=c)
        else:
            np.testing.assert_allclose(got[c].values, full[c].values, rtol=rtol, atol=atol,
                                       equal_nan=True, err_msg=c)


def test_date_shards_with_halo_equal_full_cpu():
    _check_blocks("cpu", 3, rtol=1e-12, atol=0)


def test_too_short_halo_changes_rstr():
    """The halo is load-bearing: 10 rows instead of 504 breaks RSTR on the later block."""
    prices, index, _ = _data()
    eng = FE.FactorEngine(prices, index, device="cpu")
    full = eng.run(["RSTR"])
    lo = eng.D // 2
    part = eng.date_shard(lo, eng.D, halo=10).run(["RSTR"])
    ref = full[pd.to_datetime(full.trade_date) >= pd.Timestamp(eng.date_names[lo])].reset_index(drop=True)
    assert len(part) == len(ref)
    diff = np.abs(part["RSTR"].values - ref["RSTR"].values)
    assert np.nanmax(diff) > 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("nblk", [2, 3, 8])
def test_date_shards_with_halo_equal_full_gpu_bitwise(cuda, nblk):
    """The DEFAULT config: the segment-anchored rolling kernels make every date block's owned
    rows equal the full-panel descriptors BIT FOR BIT on the GPU; 8 blocks
    of ~88 dates put the 566-row halo across several block boundaries."""
    _check_blocks("cuda:0", nblk, rtol=0, atol=0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from llm_driven_multi_factor_model_amd.parallel import dist as pdist
    ctx = pdist.init_distributed(device="cpu")
    prices, index, sw = _data()
    final, info, _ = FE.factor_pipeline(prices, index, sw, device="cpu", ctx=ctx)
    if ctx.rank == 0:
        final.to_csv(os.path.join(out_dir, "final.csv"), index=False)
        info.to_csv(os.path.join(out_dir, "info.csv"), index=False)
    else:
        assert final is None
    pdist.barrier(ctx)
    torch.distributed.destroy_process_group()


def test_two_rank_gloo_factor_pipeline_matches_single_process():
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_worker, args=(2, _free_port(), td), nprocs=2, join=True)
        got = pd.read_csv(os.path.join(td, "final.csv"))
        got_info = pd.read_csv(os.path.join(td, "info.csv"))
    prices, index, sw = _data()
    final, info, _ = FE.factor_pipeline(prices, index, sw, device="cpu")
    with tempfile.TemporaryDirectory() as td:  # same CSV round trip for the reference side
        final.to_csv(os.path.join(td, "f.csv"), index=False)
        info.to_csv(os.path.join(td, "i.csv"), index=False)
        ref, ref_info = pd.read_csv(os.path.join(td, "f.csv")), pd.read_csv(os.path.join(td, "i.csv"))
    assert list(got.columns) == list(ref.columns) and len(got) == len(ref)
    pd.testing.assert_frame_equal(got_info, ref_info)
    for c in ref.columns:
        if ref[c].dtype.kind == "f":
            np.testing.assert_allclose(got[c].values, ref[c].values, rtol=1e-10, atol=1e-12,
                                       equal_nan=True, err_msg=c)
        else:
            assert (got[c].values == ref[c].values).all(), c
