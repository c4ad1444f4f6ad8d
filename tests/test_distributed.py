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


def _worker(rank, world, port, out_path, shard="dates"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel
    from llm_driven_multi_factor_model_amd.models.risk_model import RiskModel
    from llm_driven_multi_factor_model_amd.parallel import dist as pdist
    from llm_driven_multi_factor_model_amd.utils.config import preset

    ctx = pdist.init_distributed(device="cpu")
    full = synthetic_panel(40, 60, 3, 3, seed=4, missing_frac=0.05)
    a, b = pdist.shard_range(full.D, ctx.rank, ctx.world)
    cfg = preset("reference", eigen_sims=7, eigen_shard=shard, eigen_chunk=3)
    m = RiskModel(full.slice_dates(a, b), cfg, T_global=full.D, ctx=ctx)
    m.run()
    out = {k: pdist.gather_to_root(v, ctx) for k, v in
           dict(f=m.factor_ret, r2=m.r2, nw=m.nw_cov, er=m.eigen_cov, vr=m.vra_cov, lam=m.vra_lambda).items()}
    if ctx.rank == 0:
        torch.save(out, out_path)
    pdist.barrier(ctx)
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("shard", ["dates", "sims"])
def test_two_rank_gloo_matches_single_process(shard):
    """Both eigen-adjustment sharding modes (dates over ranks; Monte-Carlo sims over ranks with
    one all_reduce of the bias sums) reproduce the single-process run."""
    from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel
    from llm_driven_multi_factor_model_amd.models.risk_model import RiskModel
    from llm_driven_multi_factor_model_amd.utils.config import preset

    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "dist.pt")
        mp.spawn(_worker, args=(2, _free_port(), path, shard), nprocs=2, join=True)
        got = torch.load(path, weights_only=True)
    full = synthetic_panel(40, 60, 3, 3, seed=4, missing_frac=0.05)
    m = RiskModel(full, preset("reference", eigen_sims=7))
    m.run()
    ref = dict(f=m.factor_ret, r2=m.r2, nw=m.nw_cov, er=m.eigen_cov, vr=m.vra_cov, lam=m.vra_lambda)
    for k in ref:
        torch.testing.assert_close(got[k], ref[k], rtol=1e-12, atol=1e-15, equal_nan=True, msg=k)


def test_shard_range_balanced():
    from llm_driven_multi_factor_model_amd.parallel.dist import shard_range
    blocks = [shard_range(10, r, 4) for r in range(4)]
    assert blocks == [(0, 3), (3, 6), (6, 8), (8, 10)]


def test_sim_shard_partition():
    from llm_driven_multi_factor_model_amd.ops.eigen import sim_shard
    assert [sim_shard(10, r, 3) for r in range(3)] == [(0, 4), (4, 7), (7, 10)]
    assert sim_shard(10_000, 7, 8) == (8750, 10_000)


def test_sharded_eigen_equals_unsharded_cpu():
    """Chunked accumulation of the bias sums == the one-shot adjustment (same sims)."""
    from llm_driven_multi_factor_model_amd.ops import eigen
    g = torch.Generator().manual_seed(0)
    A = torch.randn(300, 6, generator=g, dtype=torch.float64)
    F = torch.stack([torch.cov(A[:200].T), torch.cov(A[100:].T), torch.full((6, 6), float("nan"))])
    Cz = eigen.mc_cov(10, 6, 200, seed=3, device="cpu")
    Fh, v = eigen.eigen_risk_adjust(F, Cz=Cz, T_sim=200, return_bias=True)
    Fs, vs = eigen.eigen_risk_adjust_sharded(F, M=10, T_sim=200, seed=3, chunk=3, return_bias=True)
    torch.testing.assert_close(Fs, Fh, rtol=1e-12, atol=1e-15, equal_nan=True)
    torch.testing.assert_close(vs, v, rtol=1e-12, atol=1e-15, equal_nan=True)
    # sims drawn in pieces are the sims of one draw
    torch.testing.assert_close(torch.cat([eigen.mc_cov(4, 6, 50, 9, "cpu"),
                                          eigen.mc_cov(6, 6, 50, 9, "cpu", m0=4)]),
                               eigen.mc_cov(10, 6, 50, 9, "cpu"), rtol=0, atol=0)


def _hang_worker(rank, world, port, out_path):
    import time
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MFA_DIST_TIMEOUT_S="3")
    from llm_driven_multi_factor_model_amd.parallel import dist as pdist
    ctx = pdist.init_distributed(device="cpu")
    if ctx.rank == 1:      # a rank that stops participating (hung / dead)
        # stay alive (connections open) until rank 0 has reported, so rank 0 sees the timeout
        # rather than a closed peer even on a loaded machine
        t_end = time.time() + 30
        while not os.path.exists(out_path) and time.time() < t_end:
            time.sleep(0.2)
        return
    t0 = time.time()
    try:
        pdist.all_reduce_sum(torch.ones(4), ctx)
        msg = "no error"
    except Exception as e:  # noqa: BLE001
        msg = type(e).__name__
    with open(out_path, "w") as f:
        f.write(f"{msg} {time.time() - t0:.1f}")


def test_hung_rank_fails_fast_with_collective_timeout():
    """Failure detection: with MFA_DIST_TIMEOUT_S=3 a collective whose peer never joins raises
    on the waiting rank after ~3 s instead of hanging."""
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "hang.txt")
        mp.start_processes(_hang_worker, args=(2, _free_port(), path), nprocs=2, join=True,
                           start_method="spawn")
        msg, secs = open(path).read().split()
    assert msg != "no error"
    assert float(secs) < 8.0
