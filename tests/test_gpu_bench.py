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
                        "--samples", "8192", "--steps", "2", "--warmup", "1", "--cpu-pixels", "16",
                        "--sustain", "0.3"],
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
    su = out["sustained"]
    assert su["steps"] >= 10 and su["ms_per_step_min"] <= su["ms_per_step_mean"] <= su["ms_per_step_max"]


def _run_bench(nproc, extra, tmp, tag, backend="gloo", launcher=None):
    import socket
    dump = os.path.join(tmp, f"rec_{tag}.npy")
    args = [os.path.join(ROOT, "bench.py"), "--pixels", "520", "--samples", "4096", "--steps", "2",
            "--warmup", "1", "--no-cpu", "--no-f64", "--dump-records", dump, *extra]
    if nproc == 1 and not launcher:
        cmd = [sys.executable, *args]
    else:
        with socket.socket() as so:  # a free rendezvous port on this box
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
               str(nproc), "--master-addr", "127.0.0.1", "--master-port", str(port), *args,
               "--gpus", str(nproc)]
    env = dict(os.environ, GPD_DIST_BACKEND=backend)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    import numpy as np
    return json.loads(lines[0]), np.load(dump)


@pytest.mark.parametrize("nproc", [2, 3, 4])
def test_bench_multi_rank_strong_scaling_bitwise(tmp_path, nproc):
    """The multi-rank path of bench.py (torch.distributed.run, barrier, max-over-ranks time,
    gather of the records to rank 0, one JSON line from rank 0) with `nproc` ranks sharing
    cuda:0 under gloo (GPD_DIST_BACKEND) — the scaling runs use RCCL with one rank per GPU.
    Strong scaling (BASELINE C4): the one batch of 520 series is split into whole-FC-group
    shards (3 ranks: 43/43/44 groups, unequal), and the records gathered on rank 0 are the
    1-rank run's bit for bit."""
    one, r1 = _run_bench(1, [], str(tmp_path), "1")
    out, rn = _run_bench(nproc, [], str(tmp_path), str(nproc))
    assert out["n_gpus"] == nproc and out["config"]["total_series"] == 520
    assert out["scaling"] == "strong" and out["value"] > 0
    assert one["config"]["total_series"] == 520 and len(r1) == 520 and len(rn) == 520
    assert r1.tobytes() == rn.tobytes(), "sharded records differ from the 1-rank run"
    # the line diagnoses itself: every rank's shard, step time, kernels and gather time
    di = out["distributed"]
    assert di["world_size"] == nproc and di["backend"] == "gloo"
    pr = di["per_rank"]
    assert [r["rank"] for r in pr] == list(range(nproc))
    assert sum(r["series"] for r in pr) == 520
    assert [r["series_range"] for r in pr][0][0] == 0 and pr[-1]["series_range"][1] == 520
    for r in pr:
        assert r["step_ms"] > 0 and r["gather_ms"] is not None and r["gather_ms"] >= 0
        assert {"moments", "fit_harmonic", "reduce"} <= set(r["kernels_ms"]), r["kernels_ms"]
    assert di["step_ms_max_over_min"] >= 1.0
    assert one["distributed"] is None


def test_bench_weak_scaling_label(tmp_path):
    out, rn = _run_bench(2, ["--scaling", "weak"], str(tmp_path), "w")
    assert out["scaling"] == "weak" and out["config"]["total_series"] == 1040 and len(rn) == 1040


def test_bench_rccl_branch_at_world_one(tmp_path):
    """The branch an 8-GPU node runs (BASELINE C4), executed on one GPU: bench.py under
    torch.distributed.run with one rank and the default "nccl" backend (= RCCL), --dist-always
    sending the records through shard.gather_records (dist.gather of device uint8 records), the
    barriers and the max-over-ranks time through a device all_reduce.  The gathered records
    equal the plain run's byte for byte (src/Modulation.jl:387-389: series are independent)."""
    one, r1 = _run_bench(1, [], str(tmp_path), "plain")
    out, rd = _run_bench(1, ["--dist-always"], str(tmp_path), "rccl", backend="nccl",
                         launcher="torchrun")
    assert out["config"]["gather"].startswith("RCCL gather"), out["config"]
    assert out["n_gpus"] == 1 and out["value"] > 0
    assert len(rd) == 520 and r1.tobytes() == rd.tobytes(), "RCCL-gathered records differ"
    di = out["distributed"]
    assert di["world_size"] == 1 and di["backend"] == "nccl"
    assert di["per_rank"][0]["series"] == 520 and di["per_rank"][0]["gather_ms"] > 0
