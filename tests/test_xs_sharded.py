"""Stock-sharded (TP) CS-WLS, SURVEY.md §2.5: all-reduced moments + redundant solve + all-reduced
R^2 sums reproduce the single-process regression on the full universe."""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel
from llm_driven_multi_factor_model_amd.ops import cross_section as X
from llm_driven_multi_factor_model_amd.ops import xs_sharded as S

SHAPE = dict(D=12, N=150, P=6, Q=4)


def _panel():
    c = SHAPE
    return synthetic_panel(c["D"], c["N"], c["P"], c["Q"], seed=21, missing_frac=0.05, empty_industries=1)


def _cols(p, lo, hi):
    return (p.styles[..., lo:hi].contiguous(), p.cap[:, lo:hi].contiguous(),
            p.ret[:, lo:hi].contiguous(), p.ind[:, lo:hi].contiguous())


def test_single_rank_cpu_equals_reference():
    p = _panel()
    ref = X.xs_wls_reference(p.styles, p.cap, p.ret, p.ind, p.P)
    got = S.xs_wls_stock_sharded(p.styles, p.cap, p.ret, p.ind, p.P)
    torch.testing.assert_close(got.f, ref.f, rtol=1e-9, atol=1e-12, equal_nan=True)
    torch.testing.assert_close(got.r2, ref.r2, rtol=1e-9, atol=1e-12, equal_nan=True)
    torch.testing.assert_close(got.resid, ref.resid, rtol=1e-5, atol=1e-6, equal_nan=True)
    assert torch.equal(got.status, ref.status)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from llm_driven_multi_factor_model_amd.parallel import dist as pdist
    ctx = pdist.init_distributed(device="cpu")
    p = _panel()
    lo, hi = pdist.shard_range(p.N, ctx.rank, ctx.world)  # stocks, not dates
    out = S.xs_wls_stock_sharded(*_cols(p, lo, hi)[:3], _cols(p, lo, hi)[3], p.P, ctx)
    e = pdist.all_gather_rows(out.resid.T.contiguous(), ctx).T
    if ctx.rank == 0:
        torch.save(dict(f=out.f, r2=out.r2, e=e, st=out.status), path)
    pdist.barrier(ctx)
    torch.distributed.destroy_process_group()


def test_two_rank_gloo_stock_sharded_equals_reference():
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "tp.pt")
        mp.spawn(_worker, args=(2, _free_port(), path), nprocs=2, join=True)
        got = torch.load(path, weights_only=True)
    p = _panel()
    ref = X.xs_wls_reference(p.styles, p.cap, p.ret, p.ind, p.P)
    torch.testing.assert_close(got["f"], ref.f, rtol=1e-9, atol=1e-12, equal_nan=True)
    torch.testing.assert_close(got["r2"], ref.r2, rtol=1e-9, atol=1e-12, equal_nan=True)
    torch.testing.assert_close(got["e"], ref.resid, rtol=1e-5, atol=1e-6, equal_nan=True)
    assert torch.equal(got["st"], ref.status)


@pytest.mark.gpu
def test_gpu_split_kernels_sum_over_stock_shards(cuda):
    """HIP moments of 3 stock shards, summed (what the all_reduce does), then the solve and the
    per-shard residual sums equal the fused single-kernel regression of the whole universe."""
    from llm_driven_multi_factor_model_amd import _native
    p = synthetic_panel(64, 3001, 31, 10, seed=5, missing_frac=0.02, empty_industries=2).to(cuda)
    full = X.xs_wls(p.styles, p.cap, p.ret, p.ind, 31, refine=False)
    edges = [0, 1000, 2203, 3001]
    moms, parts = [], []

    class _SumCtx:  # one process standing in for 3 ranks: the "all_reduce" is the sum below
        enabled = False
    for a, b in zip(edges[:-1], edges[1:]):
        r = S.xs_wls_stock_sharded(*_cols(p, a, b), 31, _SumCtx(), refine=False)
        parts.append(r)
    # re-run with the summed moments through the native pieces directly
    MS = _native.query("mfa_xs_moments_bytes", 31, 10) // 8
    D, K = p.D, 42
    mom = torch.zeros(D, MS, dtype=torch.float64, device=cuda)
    st = _native.stream(cuda)
    for a, b in zip(edges[:-1], edges[1:]):
        Xs, cs, rs, js = _cols(p, a, b)
        n = b - a
        npad = (n + 7) // 8 * 8
        if npad != n:
            Xs = torch.nn.functional.pad(Xs, (0, npad - n), value=float("nan"))
            cs = torch.nn.functional.pad(cs, (0, npad - n), value=float("nan"))
            rs = torch.nn.functional.pad(rs, (0, npad - n), value=float("nan"))
            js = torch.nn.functional.pad(js, (0, npad - n), value=-1)
        m = torch.empty_like(mom)
        _native.call("mfa_xs_moments", _native.ptr(Xs), _native.ptr(cs), _native.ptr(rs),
                     _native.ptr(js), D, npad, 31, 10, _native.ptr(m), st)
        mom += m
        moms.append((Xs, cs, rs, js, npad))
    f = torch.empty(D, K, dtype=torch.float64, device=cuda)
    coef = torch.empty(D, 42, dtype=torch.float64, device=cuda)
    stats = torch.empty(D, 12, dtype=torch.float64, device=cuda)
    status = torch.empty(D, dtype=torch.int32, device=cuda)
    _native.call("mfa_xs_solve", _native.ptr(mom), D, 31, 10, 0, 1e-14, _native.ptr(f),
                 _native.ptr(coef), _native.ptr(stats), _native.ptr(status), st)
    sums = torch.zeros(D, 5, dtype=torch.float64, device=cuda)
    es = []
    for Xs, cs, rs, js, npad in moms:
        e = torch.empty(D, npad, dtype=torch.float32, device=cuda)
        s5 = torch.empty(D, 5, dtype=torch.float64, device=cuda)
        _native.call("mfa_xs_resid_sums", _native.ptr(Xs), _native.ptr(cs), _native.ptr(rs),
                     _native.ptr(js), D, npad, 31, 10, _native.ptr(coef), _native.ptr(status),
                     _native.ptr(e), _native.ptr(s5), st)
        sums += s5
        es.append(e)
    torch.cuda.synchronize()
    torch.testing.assert_close(f, full.f, rtol=1e-10, atol=1e-13, equal_nan=True)
    torch.testing.assert_close(S._r2_from_sums(sums, status), full.r2, rtol=1e-10, atol=1e-13,
                               equal_nan=True)
    e = torch.cat([e[:, :b - a] for e, a, b in zip(es, edges[:-1], edges[1:])], 1)
    torch.testing.assert_close(e, full.resid, rtol=1e-4, atol=1e-6, equal_nan=True)
    assert torch.equal(status, full.status)
    # a single shard with no peers is the plain regression (r2 from its own sums)
    one = S.xs_wls_stock_sharded(p.styles, p.cap, p.ret, p.ind, 31, refine=False)
    torch.testing.assert_close(one.f, full.f, rtol=1e-10, atol=1e-13, equal_nan=True)
    torch.testing.assert_close(one.r2, full.r2, rtol=1e-10, atol=1e-13, equal_nan=True)
