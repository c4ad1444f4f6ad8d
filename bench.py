#!/usr/bin/env python
"""Headline benchmark: cross-sectional WLS regressions/sec (5000 stocks x 41 factors).

BASELINE.json metric: "cross-sectional WLS regressions/sec (5000 stocks x 41 factors) at
1/2/4/8 GPU".  One regression = one date of ``mfm.CrossSection.reg`` semantics
(``Barra-master/mfm/CrossSection.py:57-108``): cap-weighted z-scoring of 10 styles, sqrt-cap
WLS on [country | 31 SW-L1 industries | 10 styles] with the industry-neutral constraint
(K = 42 columns, 41 free parameters), factor returns, specific returns for every stock and R^2.

A step regresses every date of a rank's shard (weak scaling, the default: ``--dates`` per GPU,
2520 = 10 years of trading days; ``--scaling strong``: ``--dates`` in total, 2520 / world per
rank), replayed from a captured HIP graph: the fused moments -> solve -> residual kernel (one
workgroup per date), then all-gathers the factor-return series across ranks over RCCL (the
collective the downstream Newey-West stage needs).  After the headline loop a second loop
regresses a FIXED global problem (``--strong-dates``, default ``--dates``, split over the ranks)
and is reported in the JSON's ``"strong"`` record, so one 1 -> N sweep yields both the weak and
the strong scaling curve.  Data is a synthetic panel of the named shape with random-init exposures (the reference ships no data).

Storage: ``--storage fp64`` (default, the headline) keeps the panel in float64, the precision
the reference regresses (``demo.py:21`` reads float64 CSV columns into ``CrossSection.reg``);
``--storage fp32`` is the factor pipeline's downcast (``load_data.py:18-21``).  Moments, solve
and reductions are float64 in both.  Every step runs the production path of
``RiskModel.regress``: the fused kernel plus the device pseudo-inverse pass for near-singular
dates (``refine=True``), both inside the captured graph.

    python bench.py --gpus 1 --steps 20 --warmup 3
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

BASELINE_REG_PER_S = 9.6  # reference on the survey host, N=5000, K=42
METRIC = "cross-sectional WLS regressions/sec (5000 stocks × 41 factors) at 1/2/4/8 GPU"


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--dates", type=int, default=2520,
                    help="dates per GPU (weak scaling) or in total (strong scaling)")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak",
                    help="weak: --dates per GPU; strong: --dates in total, sharded over ranks")
    ap.add_argument("--strong-dates", type=int, default=None,
                    help="global dates of the extra strong-scaling record (default --dates; "
                         "0 = skip it)")
    ap.add_argument("--stocks", type=int, default=5000)
    ap.add_argument("--industries", type=int, default=31)
    ap.add_argument("--styles", type=int, default=10)
    ap.add_argument("--storage", choices=["fp64", "fp32"], default="fp64",
                    help="panel storage dtype (fp64 = the reference's input precision)")
    ap.add_argument("--no-resid", action="store_true", help="skip specific-return output (not the headline)")
    ap.add_argument("--check", action="store_true", help="verify a few dates against the fp64 oracle")
    ap.add_argument("--no-graph", action="store_true",
                    help="launch the kernels eagerly instead of replaying a captured HIP graph")
    ap.add_argument("--prewarm", type=int, default=200,
                    help="untimed setup steps before the W warmup steps (GPU clock ramp)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    use_cuda = torch.cuda.is_available()
    rehearse = bool(os.environ.get("MFA_BENCH_BACKEND"))
    # a rehearsal may place several ranks on one device (local rank modulo the visible GPUs)
    gpu = local % max(1, torch.cuda.device_count()) if use_cuda and rehearse else local
    dev = torch.device(f"cuda:{gpu}" if use_cuda else "cpu")
    if use_cuda:
        torch.cuda.set_device(dev)
    backend = None
    # MFA_FORCE_PG=1 keeps the process group and the collectives at world size 1 (one rank over
    # RCCL on one GPU: the all-gather next to the graph replays, the barrier, the MAX reduce)
    coll = world > 1 or os.environ.get("MFA_FORCE_PG") == "1"
    if coll:
        # MFA_BENCH_BACKEND=gloo rehearses the multi-rank flow with several ranks on ONE GPU;
        # the default on GPUs is nccl (= RCCL).
        backend = os.environ.get("MFA_BENCH_BACKEND") or ("nccl" if use_cuda else "gloo")
        dist.init_process_group(backend, rank=rank, world_size=world,
                                device_id=dev if use_cuda and backend == "nccl" else None)

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from llm_driven_multi_factor_model_amd import _native
    from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel
    from llm_driven_multi_factor_model_amd.ops.cross_section import (xs_wls, xs_wls_reference,
                                                                     xs_wls_workspace)

    N, P, Q = args.stocks, args.industries, args.styles

    def block(G):
        """This rank's balanced contiguous share of G global dates (ranks past G % world get
        one date fewer; with G < world some own none) and the largest share (gather rows)."""
        base, rem = divmod(G, world)
        return base + (1 if rank < rem else 0), base + (1 if rem else 0)

    if args.scaling == "strong":  # fixed global problem: this rank's contiguous date block
        D, Dpad = block(args.dates)
    else:
        D, Dpad = args.dates, args.dates
    K = 1 + P + Q
    sdt = torch.float64 if args.storage == "fp64" else torch.float32
    panel = synthetic_panel(max(D, Dpad, 1), N, P, Q, seed=1234 + rank, device=dev,
                            missing_frac=0.01, dtype=sdt)

    def sync():
        if use_cuda:
            torch.cuda.synchronize(dev)
        if coll:
            dist.barrier()

    def make_runner(Dl, Dpad=None):
        """Step closure over the first ``Dl`` dates of the panel (a contiguous view).

        Two output / gather buffers: step i's RCCL all-gather of the factor-return series runs
        on the collective stream underneath step i+1's regression (the write of buffer i%2 at
        step i+2 first waits for that gather).  Every collective completes inside the timed
        region (``drain``).  ``Dpad`` > ``Dl`` (an uneven strong split): every rank gathers
        ``Dpad`` rows, its factor returns copied into a zero-padded send buffer inside the step;
        a rank with no date only takes part in the gather."""
        Dpad = Dl if Dpad is None else Dpad
        sty, cap, ret = panel.styles[:Dl], panel.cap[:Dl], panel.ret[:Dl]
        ind = None if panel.ind is None else panel.ind[:Dl]
        NB = 2 if coll else 1
        gathered = [torch.empty(world * Dpad, K, dtype=torch.float64, device=dev)
                    for _ in range(NB)] if coll else None
        send = [torch.zeros(Dpad, K, dtype=torch.float64, device=dev)
                for _ in range(NB)] if coll and Dpad != Dl else None
        outs, handles, graphs = [None] * NB, [None] * NB, [None] * NB
        ws = xs_wls_workspace(Dl, P, Q, dev, N) if use_cuda and Dl else None
        it = [0]

        def regress(b):
            if Dl == 0:
                return
            outs[b] = xs_wls(sty, cap, ret, ind, P, want_resid=not args.no_resid, refine=True,
                             out=outs[b], workspace=ws)
            if send is not None:
                send[b][:Dl].copy_(outs[b].f)

        def drain():
            for b in range(NB):
                if handles[b] is not None:
                    handles[b].wait()
                    handles[b] = None

        def step():
            b = it[0] % NB
            it[0] += 1
            if handles[b] is not None:
                handles[b].wait()          # buffer b's previous gather has read outs[b].f
                handles[b] = None
            if graphs[b] is not None:
                graphs[b].replay()
            else:
                regress(b)
            if coll:
                src = send[b] if send is not None else outs[b].f
                handles[b] = dist.all_gather_into_tensor(gathered[b], src, async_op=True)

        for b in range(NB):
            regress(b)
        if use_cuda and not args.no_graph and Dl:
            # The kernel of a step is captured once per buffer into a HIP graph and replayed:
            # the same work, without per-launch host overhead.  The RCCL all-gather stays eager.
            # thread_local capture: the process group's watchdog thread keeps polling the events
            # of earlier collectives (the barrier before the strong-scaling loop) while this
            # thread captures, which a global-mode capture forbids.
            torch.cuda.synchronize(dev)
            for b in range(NB):
                graphs[b] = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graphs[b], capture_error_mode="thread_local"):
                    regress(b)
        return step, drain, outs

    def timed(step, drain, prewarm, warmup, steps):
        """W untimed warmup steps, then EXACTLY ``steps`` timed steps between barrier +
        synchronize fences; returns the max over ranks of the elapsed seconds."""
        for _ in range(prewarm):
            step()
        drain()
        sync()
        for _ in range(warmup):
            step()
        drain()
        sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        drain()
        sync()
        el = time.perf_counter() - t0
        elt = torch.tensor([el], dtype=torch.float64, device=dev)
        if coll:
            dist.all_reduce(elt, op=dist.ReduceOp.MAX)
        return float(elt.item())

    # Setup (prewarm): bring the GPU to its steady-state clocks (a cold MI355X runs the first
    # ~100 steps ~10 % slower: 0.308 vs 0.278 ms/step measured).  Same step, same count on every
    # rank (the all-gathers pair up), all before the W warmup steps and the timed region.
    step, drain, outs = make_runner(D, Dpad)
    el = timed(step, drain, args.prewarm, args.warmup, args.steps)
    out = outs[0]

    # Second, separately reported record: strong scaling of a FIXED global problem
    # (--strong-dates in total, split over the ranks), so the driver's 1 -> N runs record both
    # curves.  The headline fields above stay the weak-scaling (or --scaling) loop.
    strong = None
    G = args.strong_dates if args.strong_dates is not None else args.dates
    if G > 0 and args.scaling == "weak":
        Ds, Dsp = block(G)
        if Dsp > D:
            raise SystemExit(f"--strong-dates {G} needs {Dsp} dates per rank, the panel has {D}")
        s_step, s_drain, _ = make_runner(Ds, Dsp)
        s_el = timed(s_step, s_drain, max(1, args.prewarm // 4), args.warmup, args.steps)
        strong = {"global_dates": G, "dates_per_gpu": Dsp, "steps": args.steps,
                  "ms_per_step": round(s_el / args.steps * 1e3, 4),
                  "value": round(G * args.steps / s_el, 1), "unit": "regressions/s"}

    if args.check and rank == 0:
        sl = slice(0, 8)
        ref = xs_wls_reference(panel.styles[sl].cpu(), panel.cap[sl].cpu(), panel.ret[sl].cpu(),
                               panel.ind[sl].cpu(), P)
        err = (out.f[sl].cpu() - ref.f).abs().max().item()
        print(f"check: max |f - oracle| = {err:.3e}", file=sys.stderr)
        assert err < 1e-9

    chunks = _native.query("mfa_xs_chunks", max(D, 1), (N + 7) // 8 * 8) if use_cuda else 1
    # regressions actually run: every rank's dates (== --dates * steps under strong scaling)
    regs = (args.dates if args.scaling == "strong" else world * D) * args.steps
    value = regs / el
    ms = el / args.steps * 1e3
    if rank == 0:
        print(json.dumps({
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "regressions/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": round(value / BASELINE_REG_PER_S, 1),
            "dtype": args.storage,
            "data": "synthetic (random-init exposures, lognormal caps, planted factor returns)",
            "strong": strong,
            "config": {
                "model": f"Barra CS-WLS: 1 country + {P} SW-L1 industries + {Q} styles, "
                         "industry-neutral constraint",
                "global_batch": args.dates if args.scaling == "strong" else world * D,
                "seq_len": N,
                "stocks": N,
                "factors": K,
                "dates_per_gpu": Dpad,
                "stock_chunks_per_date": chunks,
                "parallelism": f"dp{world}",
                "specific_returns": not args.no_resid,
                "storage": args.storage,
                "backend": backend,
                "ranks_per_gpu": (world // max(1, torch.cuda.device_count())
                                  if use_cuda and rehearse else 1),
            },
        }), flush=True)
    if coll:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
