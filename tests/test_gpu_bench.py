"""bench.py keeps the driver's contract: one JSON line with the BASELINE metric, the roofline
and CPU-baseline objects (small shape, run as its own process on cuda:0)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_json_contract():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--pixels", "512",
                        "--samples", "8192", "--steps", "2", "--warmup", "1", "--cpu-pixels", "16"],
                       capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert out["metric"] == base["metric"]
    for key in ("value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert key in out, key
    assert out["n_gpus"] == 1 and out["steps"] == 2 and out["dtype"] == "f64"
    assert out["value"] > 0 and out["higher_is_better"] is True
    rl = out["roofline"]
    assert rl["bound"] == "hbm" and rl["unit"] == "GB/s" and rl["peak"] == 8000.0
    assert abs(rl["frac"] - rl["achieved"] / rl["peak"]) < 1e-3
    cb = out["cpu_baseline"]
    assert cb["kind"] == "port" and cb["cores"] >= 1 and cb["value"] > 0
    assert out["fits"]["nan"] == 0


def test_bench_two_ranks_rehearsal():
    """The multi-rank path of bench.py (torch.distributed.run, barrier, max-over-ranks time,
    gather of the records to rank 0, one JSON line from rank 0) with two ranks sharing cuda:0
    under gloo (GPD_DIST_BACKEND) — the scaling runs use RCCL with one rank per GPU."""
    import socket
    with socket.socket() as so:  # a free rendezvous port on this box
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ, GPD_DIST_BACKEND="gloo")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                        "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--pixels", "256", "--samples", "4096", "--steps", "2", "--warmup", "1",
                        "--no-cpu"], capture_output=True, text=True, timeout=110, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["total_series"] == 512
    assert out["scaling"] == "weak" and out["value"] > 0
