"""bench.py driver contract: launched like the driver does (torch.distributed.run, 127.0.0.1),
rank 0 prints ONE JSON line with the BASELINE metric; runs on CPU/gloo at a tiny shape."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(n, extra=()):
    args = ["--gpus", str(n), "--steps", "2", "--warmup", "1", "--dates", "6", "--stocks", "64",
            "--industries", "3", "--styles", "2", *extra]
    if n == 1:
        cmd = [sys.executable, "bench.py", *args]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", *args]
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_bench_single_process_json():
    r = _run(1)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in r
    assert r["metric"].startswith("cross-sectional WLS regressions/sec")
    assert r["n_gpus"] == 1 and r["steps"] == 2 and r["scaling"] == "weak"
    assert r["config"]["global_batch"] == 6 and r["value"] > 0
    assert r["dtype"] == "fp64"
    s = r["strong"]  # separately reported fixed-global-problem loop
    assert s["global_dates"] == 6 and s["dates_per_gpu"] == 6 and s["value"] > 0
    assert abs(s["value"] - 6 * 2 / (s["ms_per_step"] * 2 / 1e3)) / s["value"] < 0.02


def test_bench_dtype_follows_storage():
    r = _run(1, ["--storage", "fp32"])
    assert r["dtype"] == "fp32" and r["config"]["storage"] == "fp32"


def test_bench_two_ranks_aggregate():
    r = _run(2)
    assert r["n_gpus"] == 2
    assert r["config"]["global_batch"] == 12 and r["config"]["parallelism"] == "dp2"
    assert abs(r["value"] - 12 * 2 / (r["ms_per_step"] * 2 / 1e3)) / r["value"] < 0.02
    s = r["strong"]  # 6 global dates = 3 per rank; headline fields untouched
    assert s["global_dates"] == 6 and s["dates_per_gpu"] == 3 and s["value"] > 0


def test_bench_strong_scaling_two_ranks():
    """--scaling strong: the global date count is fixed and sharded over the ranks."""
    r = _run(2, ["--scaling", "strong"])
    assert r["scaling"] == "strong" and r["n_gpus"] == 2
    assert r["config"]["global_batch"] == 6 and r["config"]["dates_per_gpu"] == 3
    assert abs(r["value"] - 6 * 2 / (r["ms_per_step"] * 2 / 1e3)) / r["value"] < 0.02
    assert r["config"]["storage"] == "fp64"
