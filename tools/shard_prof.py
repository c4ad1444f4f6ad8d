"""Per-rank cost of the date-sharded exposures path on ONE process (collectives stubbed):
the work rank `rank` of `world` does at N stocks x T days, timed sub-step by sub-step.

  host  : host-side row selection + upload + build of the rank's rows only
          (DeviceFactorEngine.from_host_shard, the default for sorted loader rows)
  full  : round 4's path -- every rank uploads and builds the whole master, then date_shard

then descriptors on the slice, owned rows, per-date post-processing -- and, for the host path,
the rest of the rank's config-3 job: export columns, its RiskPanel and RiskModel.run over its
owned dates (collectives stubbed: the t+1 return of a block's last row and the time-axis scans
see only this rank's dates; the per-date regression and eigen adjustment -- the bulk of the risk
model -- are the rank's exact work).  The loader columns are staged like the native reader's
(float32 numerics in pinned memory, S16 codes, int32 dates).

    python tools/shard_prof.py [N] [T] [world] [rank]      # default 5000 2520 8 7
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd.models import e2e  # noqa: E402
from llm_driven_multi_factor_model_amd.models import factor_engine as FE  # noqa: E402
from llm_driven_multi_factor_model_amd.parallel.dist import shard_range  # noqa: E402
from llm_driven_multi_factor_model_amd.models.risk_model import RiskModel  # noqa: E402
from llm_driven_multi_factor_model_amd.parallel.dist import DistContext  # noqa: E402
from llm_driven_multi_factor_model_amd.utils.config import FactorConfig, preset  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
T = int(sys.argv[2]) if len(sys.argv) > 2 else 2520
world = int(sys.argv[3]) if len(sys.argv) > 3 else 8
rank = int(sys.argv[4]) if len(sys.argv) > 4 else 7
dev = torch.device("cuda:0")
prices, index, sw = FE.synthetic_prices_fast(N=N, T=T, seed=0, n_ind=31, suspend_frac=0.01)
prices = prices.sort_values(["ts_code", "trade_date"], kind="stable").reset_index(drop=True)
p, i = e2e._columns_from_frames(prices, index)
p["trade_date"] = p["trade_date"].astype("int32")
if "end_date" in p:
    p["end_date"] = p["end_date"].astype("int32")
p = e2e.stage_host_columns(p)
cfg = FactorConfig()
risk_cfg = preset("reference")
small = FE.synthetic_prices(N=60, T=300, seed=1, n_ind=31)
e2e.run_pipeline(*small, device=dev)


def tick(rec, name, t0):
    torch.cuda.synchronize()
    rec[name] = round(time.perf_counter() - t0, 4)
    return time.perf_counter()


for rep in range(4):
    timing = rep == 3   # the last rep: device synchronised at every sub-step (breakdown only)
    for path in ("host", "full"):
        rec = {"path": path, "rep": rep, "synced_breakdown": timing, "N": N, "T": T, "world": world, "rank": rank}
        t00 = t = time.perf_counter()
        if path == "host":
            sh = e2e.DeviceFactorEngine.from_host_shard(dict(p), dict(i), rank, world, dev, cfg,
                                                        timing=timing)
            assert sh is not None
            t = tick(rec, "select_upload_build", t)
            rec["host_times"] = {k: round(v, 4) if isinstance(v, float) else v for k, v in sh.host_times.items()}
        else:
            full = e2e.DeviceFactorEngine(dict(p), dict(i), device=dev, config=cfg)
            t = tick(rec, "full_engine", t)
            lo, hi = shard_range(full.D, rank, world)
            full.cashflow_ttm()
            sh = full.date_shard(lo, hi)
            t = tick(rec, "date_shard", t)
        res = sh.compute(FE.FACTORS_TO_RUN)
        t = tick(rec, "descriptors", t)
        own = torch.nonzero(sh.own).flatten()
        res = {k: v[own] for k, v in res.items()}
        eng = sh.owned()
        t = tick(rec, "owned", t)
        col = FE.postprocess_columns(eng, res, eng.cfg)
        t = tick(rec, "postprocess", t)
        if path == "host":   # the rest of the rank's job: its risk panel and risk model
            cols = e2e.export_columns(col, e2e.next_return_global(eng, col["ret"], None))
            info, l1_stock = e2e.industry_info(eng, sw)
            panel = e2e.risk_panel(eng, cols, l1_stock, info)
            t = tick(rec, "risk_panel", t)
            RiskModel(panel, risk_cfg, ctx=DistContext(device=dev)).run()
            t = tick(rec, "risk_model", t)
            rec["panel_dates"] = panel.D
        rec["non_io_s"] = round(time.perf_counter() - t00, 4)
        rec["rows_slice"], rec["rows_owned"] = sh.R, eng.R
        print(json.dumps(rec), flush=True)
