"""Command line entry points (the reference has none: scripts with hard-coded paths, Q25).

    python -m llm_driven_multi_factor_model_amd.cli synth  --out data/ --dates 250 --stocks 300
    python -m llm_driven_multi_factor_model_amd.cli risk   --data data/barra_data_csi.csv \
        --industry data/industry_info.csv --out results/ [--preset reference] [--sims 100] \
        [--checkpoint risk.ckpt] [--resume risk.ckpt] [--attribution equal] [--mongo-uri URI] \
        [--time-scan carry] [--no-deterministic] [--bias-stat 21 --bias-start 1000]
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m llm_driven_multi_factor_model_amd.cli risk ...
    python -m llm_driven_multi_factor_model_amd.cli factors --prices prices.csv --index index.csv \
        --industry sw_industry.csv --out data/
    python -m llm_driven_multi_factor_model_amd.cli pipeline --prices prices.csv --index index.csv \
        --industry sw_industry.csv --out results/ [--write-barra data/]   # main.py + demo.py in HBM
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m llm_driven_multi_factor_model_amd.cli \
        pipeline ...          # date-sharded end to end: each rank its date block + halo
    python -m llm_driven_multi_factor_model_amd.cli serve --data barra_data_csi.csv \
        --industry industry_info.csv --port 8000      # POST /risk {"portfolios": [...]}

``risk`` is ``Barra-master/demo.py`` (read -> one-hot -> MFM(data, P, Q) -> 4 stages -> 5 CSVs);
``factors`` is ``Barra_factor_cal/main.py`` (descriptors -> winsorize -> composite ->
orthogonalize -> barra_data_csi.csv + industry_info.csv).
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys
import time

import numpy as np
import pandas as pd
import torch

log = logging.getLogger("mfa")


def _setup_logging(rank: int = 0):
    logging.basicConfig(level=os.environ.get("MFA_LOGLEVEL", "INFO"),
                        format=f"%(asctime)s [rank{rank}] %(name)s %(levelname)s: %(message)s")


def cmd_synth(a):
    from .models.panel import synthetic_panel
    p = synthetic_panel(a.dates, a.stocks, a.industries, a.styles, seed=a.seed, missing_frac=a.missing)
    os.makedirs(a.out, exist_ok=True)
    D, N = p.D, p.N
    m = p.valid()
    dates = pd.DatetimeIndex(p.dates).strftime("%Y/%m/%d")
    codes = np.array([f"80{j:04d}.SI" for j in range(p.P)])
    di, si = torch.nonzero(m, as_tuple=True)
    df = pd.DataFrame({
        "date": dates.values[di.numpy()], "stocknames": p.stocks[si.numpy()],
        "capital": p.cap[di, si].double().numpy(), "ret": p.ret[di, si].double().numpy(),
        "industry": codes[p.ind[di, si].long().numpy()],
    })
    for q, name in enumerate(p.style_names):
        df[name] = p.styles[di, q, si].double().numpy()
    df.to_csv(os.path.join(a.out, "barra_data_csi.csv"), index=False)
    pd.DataFrame({"code": codes, "industry_names": [f"industry_{j:02d}" for j in range(p.P)],
                  "start_date": "20000101"}).to_csv(os.path.join(a.out, "industry_info.csv"), index=False)
    log.info("wrote %d rows x %d dates x %d stocks to %s", len(df), D, N, a.out)


def cmd_risk(a):
    from .models.risk_model import RiskModel
    from .parallel import dist as pdist
    from .utils.config import preset
    from .utils.io import panel_from_barra_csv, write_risk_results

    ctx = pdist.init_distributed(device=a.device)
    _setup_logging(ctx.rank)
    t0 = time.perf_counter()
    if a.mongo_uri:  # demo.ipynb: barra_factors + sw_industry_info_for_factors from MongoDB
        from pymongo import MongoClient
        from .utils.io import panel_from_mongo
        client = MongoClient(a.mongo_uri)
        full = panel_from_mongo(client[a.mongo_db], device="cpu")
        client.close()
    else:
        if not (a.data and a.industry):
            raise SystemExit("risk: give --data and --industry (CSV) or --mongo-uri")
        full = panel_from_barra_csv(a.data, a.industry, device="cpu")
    state = None
    if a.resume:
        from .utils.checkpoint import load_state
        state = load_state(a.resume)
        last = pd.Timestamp(str(state["dates"][-1]))
        new = np.nonzero(pd.DatetimeIndex(full.dates) > last)[0]
        if not len(new):
            raise SystemExit(f"no dates after the checkpoint's last date {last.date()}")
        full = full.slice_dates(int(new[0]), full.D)
        full = type(full)(**{**full.__dict__, "date_offset": 0})
        log.info("resuming after %s: %d new dates", last.date(), full.D)
    lo, hi = pdist.shard_range(full.D, ctx.rank, ctx.world)
    panel = full.slice_dates(lo, hi).to(ctx.device)
    log.info("panel %d dates x %d stocks x K=%d (shard [%d,%d)) loaded in %.2fs", full.D, full.N,
             full.K, lo, hi, time.perf_counter() - t0)
    # only flags the user actually set override the preset (e.g. bootstrap10k keeps M = 10000)
    over = {k: v for k, v in dict(eigen_sims=a.sims, vra_half_life=a.vra_tau, nw_lags=a.nw_q,
                                  nw_half_life=a.nw_tau, eigen_scale=a.scale,
                                  eigen_shard=a.eigen_shard, eigen_chunk=a.eigen_chunk,
                                  time_scan=a.time_scan, deterministic=a.deterministic).items()
            if v is not None}
    cfg = preset(a.preset, **over)
    log.info("config %s: %s", a.preset, json.dumps(cfg.to_dict()))
    if state is not None:
        model = RiskModel.resume(state, panel, cfg, T_global=full.D, ctx=ctx)
    else:
        model = RiskModel(panel, cfg, T_global=full.D, ctx=ctx)
    model.run()
    if a.checkpoint:
        model.save(a.checkpoint)
    paths = write_risk_results(model, a.out, long_specific=a.long_specific)
    if a.attribution:
        paths["risk_attribution"] = _write_attribution(model, a.attribution, a.out, ctx)
    if a.bias_stat is not None:
        paths["eigenfactor_bias"] = _write_bias_stat(model, a.bias_stat, a.bias_start, a.out, ctx)
    if ctx.rank == 0:
        log.info("stage ms: %s", json.dumps({k: round(v, 3) for k, v in model.times.ms.items()}))
        for k, v in paths.items():
            log.info("wrote %s -> %s", k, v)
    pdist.barrier(ctx)


def _write_attribution(model, spec: str, out_dir: str, ctx):
    """Per-date risk decomposition of a portfolio: ``spec`` = "equal" (equal weight over the
    panel's stocks) or a CSV with columns ``stocknames, weight`` (held on every date).
    Writes ``risk_attribution.csv`` (rank 0): total / factor / specific volatility and the
    country / industry / style / specific shares of variance."""
    from .parallel import dist as pdist
    N = model.panel.N
    if spec == "equal":
        h = torch.full((N,), 1.0 / N, dtype=torch.float64)
    else:
        w = pd.read_csv(spec)
        pos = {str(s): i for i, s in enumerate(model.panel.stocks)}
        h = torch.zeros(N, dtype=torch.float64)
        for s, v in zip(w["stocknames"].astype(str), w["weight"].astype(float)):
            if s in pos:
                h[pos[s]] = v
    r = model.risk_attribution(h.to(model.device))
    g = r.grouped(model.panel.P)
    cols = {"total_vol": torch.sqrt(r.total_var), "factor_vol": torch.sqrt(r.factor_var),
            "specific_vol": torch.sqrt(r.specific_var), **{f"{k}_share": v for k, v in g.items()}}
    got = {k: pdist.gather_to_root(v.contiguous(), ctx) for k, v in cols.items()}
    dates = model._global_dates()
    path = os.path.join(out_dir, "risk_attribution.csv")
    if ctx.rank == 0:
        df = pd.DataFrame({k: v.cpu().numpy() for k, v in got.items()},
                          index=pd.DatetimeIndex(dates, name="date"))
        os.makedirs(out_dir, exist_ok=True)
        df.to_csv(path)
    return path


def _write_bias_stat(model, predlen: int, start: int, out_dir: str, ctx):
    """``MFM.py:203-204``: the eigenfactor bias statistic of the Newey-West series (before the
    eigen adjustment) and of the eigen-adjusted series (after), over dates >= ``start`` with a
    ``predlen``-day forecast horizon; plus the VRA series.  Collective; rank 0 writes
    ``eigenfactor_bias.csv`` (one row per eigenfactor, descending variance)."""
    cols = {w: model.eigenfactor_bias(w, start=start, predlen=predlen)
            for w in ("nw", "eigen", "vra")}
    path = os.path.join(out_dir, "eigenfactor_bias.csv")
    if ctx.rank == 0:
        if not torch.isfinite(cols["nw"]).any():
            log.warning("eigenfactor bias: no date >= %d has %d later dates (T = %d)", start,
                        predlen, model.T)
        df = pd.DataFrame({f"bias_{k}": v.cpu().numpy() for k, v in cols.items()})
        df.index.name = "eigenfactor"
        os.makedirs(out_dir, exist_ok=True)
        df.to_csv(path)
    return path


def cmd_serve(a):
    """Fit the risk model on a barra_data_csi.csv (single process) and serve portfolio risk of
    its last date over HTTP (``serving.make_app``)."""
    from .models.risk_model import RiskModel
    from .serving import RiskService, make_app
    from .utils.config import preset
    from .utils.io import panel_from_barra_csv
    _setup_logging()
    dev = a.device or ("cuda:0" if torch.cuda.is_available() else "cpu")
    panel = panel_from_barra_csv(a.data, a.industry, device=dev)
    over = {"eigen_sims": a.sims} if a.sims is not None else {}
    model = RiskModel(panel, preset(a.preset, **over)).run()
    svc = RiskService(model, which=a.covariance)
    log.info("serving %s", json.dumps(svc.info()))
    import uvicorn
    uvicorn.run(make_app(svc), host=a.host, port=a.port, log_level="info")


def cmd_pipeline(a):
    """The whole job in HBM: loader CSVs -> descriptors -> exposures -> risk model -> the five
    results CSVs (main.py then demo.py without the barra_data_csi.csv round trip)."""
    from .models import e2e
    from .parallel import dist as pdist
    from .utils.config import preset
    from .utils.io import write_risk_results
    # torchrun: date-sharded end to end (each rank reads the loader columns, computes its date
    # block + halo, and the risk model runs over the ranks' blocks); rank 0 writes the CSVs
    ctx = pdist.init_distributed(device=a.device)
    _setup_logging(ctx.rank)
    t0 = time.perf_counter()
    prices, index = e2e.read_price_columns(a.prices, a.index)
    if prices is None:
        prices = pd.read_csv(a.prices)
        index = pd.read_csv(a.index)
    sw = pd.read_csv(a.industry, dtype={"ts_code": str, "l1_code": str})
    t_read = time.perf_counter() - t0
    over = {k: v for k, v in dict(eigen_sims=a.sims, vra_half_life=a.vra_tau, nw_lags=a.nw_q,
                                  nw_half_life=a.nw_tau, time_scan=a.time_scan).items()
            if v is not None}
    cfg = preset(a.preset, **over)
    pdist.barrier(ctx)
    model, info, frame, t = e2e.run_pipeline(prices, index, sw, risk_cfg=cfg,
                                             device=None if ctx.enabled else a.device,
                                             want_barra=bool(a.write_barra), ctx=ctx)
    t0 = time.perf_counter()
    paths = write_risk_results(model, a.out, long_specific=a.long_specific)
    if a.write_barra and frame is not None:
        os.makedirs(a.write_barra, exist_ok=True)
        frame.to_csv(os.path.join(a.write_barra, "barra_data_csi.csv"), index=False)
        info.to_csv(os.path.join(a.write_barra, "industry_info.csv"), index=False)
    t_write = time.perf_counter() - t0
    compute = {k: v for k, v in t.items() if k.endswith("_s")}
    if ctx.enabled:  # the job's time is the slowest rank's
        compute = {k: pdist.all_reduce_max(v, ctx) for k, v in compute.items()}
    compute = {k: round(v, 4) for k, v in compute.items()}
    T = sum(model.sizes)
    if ctx.rank == 0:
        log.info("pipeline: %d rank(s), panel %d dates x %d stocks x K=%d; read %.3fs, compute "
                 "%s (%.3fs), write %.3fs", ctx.world, T, model.panel.N, model.K, t_read,
                 json.dumps(compute), sum(compute.values()), t_write)
        if a.timings:
            with open(a.timings, "w") as fh:
                json.dump({"read_s": t_read, "write_s": t_write, **compute,
                           "non_io_s": sum(compute.values()), "D": T, "N": model.panel.N,
                           "K": model.K, "world": ctx.world}, fh)
        for k, v in paths.items():
            log.info("wrote %s -> %s", k, v)
    pdist.barrier(ctx)


def cmd_factors(a):
    from .models.factor_engine import run_factor_pipeline
    from .parallel import dist as pdist
    ctx = pdist.init_distributed(device=a.device)  # torchrun: date blocks per rank (+ halo)
    _setup_logging(ctx.rank)
    run_factor_pipeline(a.prices, a.index, a.industry, a.out,
                        device=a.device if not ctx.enabled else None, ctx=ctx)
    pdist.barrier(ctx)


def main(argv=None):
    ap = argparse.ArgumentParser(prog="mfa", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("synth", help="write a synthetic barra_data_csi.csv + industry_info.csv")
    s.add_argument("--out", required=True)
    s.add_argument("--dates", type=int, default=250)
    s.add_argument("--stocks", type=int, default=300)
    s.add_argument("--industries", type=int, default=28)
    s.add_argument("--styles", type=int, default=10)
    s.add_argument("--missing", type=float, default=0.02)
    s.add_argument("--seed", type=int, default=0)
    s.set_defaults(fn=cmd_synth)
    r = sub.add_parser("risk", help="demo.py equivalent: risk model on barra_data_csi.csv")
    r.add_argument("--data", default=None, help="barra_data_csi.csv")
    r.add_argument("--industry", default=None, help="industry_info.csv")
    r.add_argument("--mongo-uri", default=None,
                   help="read barra_factors / sw_industry_info_for_factors from MongoDB instead")
    r.add_argument("--mongo-db", default=os.environ.get("MFA_MONGO_DB", "barra_financial_data"))
    r.add_argument("--out", default="results")
    r.add_argument("--preset", default="reference",
                   help="reference | use4s | use4l | bootstrap10k (flags below override it)")
    r.add_argument("--sims", type=int, default=None, help="eigen-adjustment sims (preset: 100)")
    r.add_argument("--scale", type=float, default=None, help="eigen scale_coef (preset: 1.4)")
    r.add_argument("--nw-q", type=int, default=None, help="Newey-West lags (preset: 2)")
    r.add_argument("--nw-tau", type=float, default=None, help="Newey-West half-life (preset: 252)")
    r.add_argument("--vra-tau", type=float, default=None, help="VRA half-life (preset: 42)")
    r.add_argument("--eigen-shard", choices=["dates", "sims"], default=None,
                   help="shard the eigen adjustment over dates or Monte-Carlo sims across ranks")
    r.add_argument("--eigen-chunk", type=int, default=None, help="sims per launch in sims mode")
    r.add_argument("--time-scan", choices=["gather", "carry"], default=None,
                   help="time-axis stages across ranks: gather the series (default) or carry "
                        "block states (each rank scans only its dates)")
    r.add_argument("--deterministic", dest="deterministic", action="store_true", default=None,
                   help="bitwise-reproducible CS-WLS kernel (default: whenever supported)")
    r.add_argument("--no-deterministic", dest="deterministic", action="store_false",
                   help="shared-replica CS-WLS kernel (reproducible to rounding only)")
    r.add_argument("--bias-stat", type=int, default=None, metavar="PREDLEN",
                   help="write eigenfactor_bias.csv with this forecast horizon (MFM.py:203: 21)")
    r.add_argument("--bias-start", type=int, default=1000,
                   help="first date of the bias statistic (MFM.py:203: 1000)")
    r.add_argument("--attribution", default=None,
                   help="'equal' or a CSV (stocknames, weight): write risk_attribution.csv")
    r.add_argument("--device", default=None, help="cpu to force the CPU path")
    r.add_argument("--long-specific", action="store_true")
    r.add_argument("--checkpoint", default=None, help="write a resumable checkpoint here")
    r.add_argument("--resume", default=None,
                   help="continue from a checkpoint: only dates after its last date are run")
    r.set_defaults(fn=cmd_risk)
    v = sub.add_parser("serve", help="fit the risk model, then serve portfolio risk over HTTP")
    v.add_argument("--data", required=True, help="barra_data_csi.csv")
    v.add_argument("--industry", required=True, help="industry_info.csv")
    v.add_argument("--preset", default="reference")
    v.add_argument("--sims", type=int, default=None)
    v.add_argument("--covariance", choices=["nw", "eigen", "vra"], default="vra")
    v.add_argument("--device", default=None)
    v.add_argument("--host", default="127.0.0.1")
    v.add_argument("--port", type=int, default=8000)
    v.set_defaults(fn=cmd_serve)
    q = sub.add_parser("pipeline", help="main.py + demo.py in HBM: loader CSVs -> results/*.csv")
    q.add_argument("--prices", required=True)
    q.add_argument("--index", required=True)
    q.add_argument("--industry", required=True)
    q.add_argument("--out", default="results")
    q.add_argument("--write-barra", default=None, metavar="DIR",
                   help="also write barra_data_csi.csv + industry_info.csv here")
    q.add_argument("--preset", default="reference")
    q.add_argument("--sims", type=int, default=None)
    q.add_argument("--nw-q", type=int, default=None)
    q.add_argument("--nw-tau", type=float, default=None)
    q.add_argument("--vra-tau", type=float, default=None)
    q.add_argument("--time-scan", choices=["gather", "carry"], default=None,
                   help="time-axis stages across ranks: gather the factor-return series "
                        "(default, equal to one process) or carry block states")
    q.add_argument("--long-specific", action="store_true")
    q.add_argument("--device", default=None)
    q.add_argument("--timings", default=None, help="write stage timings (JSON) here")
    q.set_defaults(fn=cmd_pipeline)
    f = sub.add_parser("factors", help="main.py equivalent: descriptors -> Barra exposures")
    f.add_argument("--prices", required=True)
    f.add_argument("--index", required=True)
    f.add_argument("--industry", required=True)
    f.add_argument("--out", default="data")
    f.add_argument("--device", default=None)
    f.set_defaults(fn=cmd_factors)
    a = ap.parse_args(argv)
    if a.cmd not in ("risk", "factors", "serve", "pipeline"):
        _setup_logging()
    a.fn(a)
    return 0


if __name__ == "__main__":
    sys.exit(main())
