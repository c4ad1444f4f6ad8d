"""One-rank process groups (``MFA_FORCE_PG=1``): every collective of the date-sharded paths runs
even at world size 1.  Two ranks cannot share one GPU under RCCL, so on a one-GPU box this is
how the RCCL paths themselves execute: communicator init with ``device_id``, the async
all-gather on RCCL's stream next to the captured HIP graphs in ``bench.py``, the gathers /
all-reduces / broadcasts of the sharded pipeline.  On CPU the same flow runs over gloo."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _torchrun(script_args, gpu: bool, timeout=600):
    env = dict(os.environ, MFA_FORCE_PG="1", PYTHONPATH=ROOT, OMP_NUM_THREADS="4")
    if not gpu:
        env.update(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", *script_args]
    return subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout,
                          env=env)


def _json_lines(out):
    return [json.loads(x) for x in out.splitlines() if x.startswith("{")]


def _bench(gpu):
    r = _torchrun(["bench.py", "--gpus", "1", "--steps", "5", "--warmup", "2", "--prewarm", "2",
                   "--dates", "64", "--stocks", "600" if not gpu else "2000", "--check"], gpu)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_lines(r.stdout)[-1]
    assert rec["value"] > 0 and rec["n_gpus"] == 1 and rec["steps"] == 5
    return rec


def test_bench_one_rank_process_group_cpu():
    rec = _bench(gpu=False)
    assert rec["config"]["backend"] == "gloo"


def _pipeline(gpu):
    r = _torchrun(["tools/pipeline_dist.py", "300", "620"], gpu)
    assert r.returncode == 0, r.stderr[-3000:]
    recs = _json_lines(r.stdout)
    diff = recs[-1]["vs_one_process"]
    for k, v in diff.items():   # the gathered outputs ARE the one-process outputs
        assert v["nan_mismatch"] == 0, k
        assert v["max_abs"] in (0.0, None), (k, v)
    return recs


def test_pipeline_one_rank_process_group_cpu():
    recs = _pipeline(gpu=False)
    assert recs[0]["backend"] == "gloo" and recs[0]["world"] == 1


@pytest.mark.gpu
def test_bench_one_rank_rccl(cuda):
    """bench.py's RCCL flow on one GPU: nccl communicator, graph replays + async all-gather."""
    rec = _bench(gpu=True)
    assert rec["config"]["backend"] == "nccl"


@pytest.mark.gpu
def test_pipeline_one_rank_rccl_bitwise(cuda):
    """The date-sharded pipeline with every collective over RCCL (world 1) == one process."""
    recs = _pipeline(gpu=True)
    assert recs[0]["backend"] == "nccl" and recs[0]["world"] == 1
