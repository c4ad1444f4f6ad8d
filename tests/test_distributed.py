"""Date-sharded data parallelism: 2-rank gloo run == single process (CPU, world_size 2)."""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel
    from llm_driven_multi_factor_model_amd.models.risk_model import RiskModel
    from llm_driven_multi_factor_model_amd.parallel import dist as pdist
    from llm_driven_multi_factor_model_amd.utils.config import preset

    ctx = pdist.init_distributed(device="cpu")
    full = synthetic_panel(40, 60, 3, 3, seed=4, missing_frac=0.05)
    a, b = pdist.shard_range(full.D, ctx.rank, ctx.world)
    m = RiskModel(full.slice_dates(a, b), preset("reference", eigen_sims=6), T_global=full.D, ctx=ctx)
    m.run()
    out = {k: pdist.gather_to_root(v, ctx) for k, v in
           dict(f=m.factor_ret, r2=m.r2, nw=m.nw_cov, er=m.eigen_cov, vr=m.vra_cov, lam=m.vra_lambda).items()}
    if ctx.rank == 0:
        torch.save(out, out_path)
    pdist.barrier(ctx)
    torch.distributed.destroy_process_group()


def test_two_rank_gloo_matches_single_process():
    from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel
    from llm_driven_multi_factor_model_amd.models.risk_model import RiskModel
    from llm_driven_multi_factor_model_amd.utils.config import preset

    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "dist.pt")
        mp.spawn(_worker, args=(2, _free_port(), path), nprocs=2, join=True)
        got = torch.load(path, weights_only=True)
    full = synthetic_panel(40, 60, 3, 3, seed=4, missing_frac=0.05)
    m = RiskModel(full, preset("reference", eigen_sims=6))
    m.run()
    ref = dict(f=m.factor_ret, r2=m.r2, nw=m.nw_cov, er=m.eigen_cov, vr=m.vra_cov, lam=m.vra_lambda)
    for k in ref:
        torch.testing.assert_close(got[k], ref[k], rtol=1e-12, atol=1e-15, equal_nan=True, msg=k)


def test_shard_range_balanced():
    from llm_driven_multi_factor_model_amd.parallel.dist import shard_range
    blocks = [shard_range(10, r, 4) for r in range(4)]
    assert blocks == [(0, 3), (3, 6), (6, 8), (8, 10)]
