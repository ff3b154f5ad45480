"""bench.py's multi-GPU contract rehearsed on CPU: the driver launches it as
``python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`` (one rank per GPU);
here the same command runs N gloo ranks on the CPU and rank 0 must print exactly one JSON line
with the whole-job numbers (n_gpus = N, global batch = N x per-GPU batch, dpN, comm fields)."""
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


@pytest.mark.parametrize("n", [2, 4])
def test_bench_torchrun_json_line(n):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(n), "--steps", "1", "--warmup", "1", "--image", "32", "--batch", "2"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd="/tmp")
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["steps"] == 1 and d["warmup"] == 1
    assert d["config"]["global_batch"] == 2 * n and d["config"]["parallelism"] == f"dp{n}"
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["higher_is_better"] is True
    assert d["scaling"] == "weak" and d["dtype"] == "bf16" and d["data"] == "synthetic"
    for k in ("comm_ms", "exposed_comm_ms", "bucket_mb", "buckets", "grad_mb", "backend"):
        assert k in d["config"], k
    assert d["config"]["backend"] == "gloo"


@pytest.mark.parametrize("model,extra", [("resnet50", ["--image", "32"]), ("vgg16", ["--image", "32"]),
                                         ("bert", ["--layers", "1", "--seq", "32"])])
def test_bench_torchrun_n8_every_dp_config(model, extra):
    """The driver's N=8 launch, rehearsed with 8 gloo ranks for each BASELINE.json DP config
    (tiny shapes): one JSON line, whole-job value, dp8, bucket / comm fields; bf16 wire for bert."""
    n = 8
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--model", model, "--gpus", str(n), "--steps", "1", "--warmup", "1", "--batch", "2", *extra]
    if model == "bert":
        cmd += ["--reduce-dtype", "bf16"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env, cwd="/tmp")
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["config"]["parallelism"] == "dp8" and d["config"]["global_batch"] == 2 * n
    assert d["value"] > 0 and d["config"]["buckets"] >= 1 and d["config"]["backend"] == "gloo"
    if model == "bert":
        assert d["config"]["reduce_dtype"] == "bf16" and d["config"]["bf16_algo"] == "a2a"
        assert d["unit"] == "tokens/sec"
