"""Data parallelism on the GPU fused path: 2 ranks (gloo transport, both on the one GPU of
the test box) with overlapped per-layer bucket hooks must equal a single-process emulation
(per-replica gradients averaged, then the same optimizer step)."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_ddp_overlap_hooks_match_emulation(tmp_path):
    from distributeddeeplearningspark_amd.models.optimizers import SGD
    from distributeddeeplearningspark_amd.models.resnet import ResNet
    from distributeddeeplearningspark_amd.parallel.launcher import free_port

    out = str(tmp_path / "ddp.pt")
    env = dict(os.environ, DDL_DIST_BACKEND="gloo", PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.join(ROOT, "tests", "ddp_gpu_worker.py"),
           out]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = torch.load(out, weights_only=True)

    torch.manual_seed(0)
    x = torch.randn(2, 16, 32, 32, 3)
    y = torch.randint(0, 10, (2, 16))
    m = ResNet(blocks=(2, 1), input_shape=(32, 32, 3), num_classes=10)
    m.compile(SGD(lr=0.05, momentum=0.9), "sparse_categorical_crossentropy")
    m.place("cuda", seed=3)
    for step in range(2):
        g = torch.zeros_like(m.arena.grad)
        for r_ in range(2):
            m.backward_step(m.to_input(x[r_]), m.to_target(y[r_]))
            g += m.arena.grad
        m.arena.grad.copy_(g)
        m.optimizer.step(grad_scale=0.5)
    ref = m.arena.master.detach().cpu()
    rel = ((res["master"] - ref).norm() / ref.norm()).item()
    assert rel < 1e-3, rel


@pytest.mark.parametrize("rd", ["fp32", "bf16"])
def test_forced_rccl_world1_matches_plain_step(tmp_path, rd):
    """RCCL on the 1-GPU box: a forced world-1 "nccl" group runs the bucket hooks, the
    (bf16-cast) bucket all-reduces and the broadcast; the result equals plain training."""
    from distributeddeeplearningspark_amd.models.optimizers import SGD
    from distributeddeeplearningspark_amd.models.resnet import ResNet

    out = str(tmp_path / "forced.pt")
    env = dict(os.environ, DDL_FORCE_DIST="1", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "ddp_forced_worker.py"), out, rd], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = torch.load(out, weights_only=True)

    torch.manual_seed(0)
    x = torch.randn(3, 16, 32, 32, 3)
    y = torch.randint(0, 10, (3, 16))
    m = ResNet(blocks=(2, 1), input_shape=(32, 32, 3), num_classes=10)
    m.compile(SGD(lr=0.05, momentum=0.9), "sparse_categorical_crossentropy")
    m.place("cuda", seed=3)
    for s in range(3):
        m.train_on_batch(x[s], y[s])
    ref = m.arena.master.detach().cpu()
    rel = ((res["master"] - ref).norm() / ref.norm()).item()
    assert rel < (1e-4 if rd == "fp32" else 3e-3), rel
    print(f"forced RCCL ({rd}): exposed {res['exposed_ms']:.3f} ms/step, full all-reduce {res['allreduce_ms']:.3f} ms")
