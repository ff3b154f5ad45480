"""Worker of tests/test_gpu_ddp.py::test_forced_rccl_world1_matches_plain_step: DDL_FORCE_DIST=1
builds a real "nccl" (RCCL) process group at world size 1, so DataParallel installs its bucket
hooks and issues RCCL all-reduces / broadcasts from a single MI355X."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributeddeeplearningspark_amd.models.optimizers import SGD
from distributeddeeplearningspark_amd.models.resnet import ResNet
from distributeddeeplearningspark_amd.parallel import comm
from distributeddeeplearningspark_amd.parallel.ddp import DataParallel


def main():
    out, rd = sys.argv[1], sys.argv[2]
    pg = comm.init_from_env(prefer_gpu=True)
    assert pg.forced and pg.distributed and pg.backend == "nccl", pg
    torch.manual_seed(0)
    x = torch.randn(3, 16, 32, 32, 3)
    y = torch.randint(0, 10, (3, 16))
    m = ResNet(blocks=(2, 1), input_shape=(32, 32, 3), num_classes=10)
    m.compile(SGD(lr=0.05, momentum=0.9), "sparse_categorical_crossentropy")
    m.place(pg.device, seed=3)
    ddp = DataParallel(m, pg, bucket_mb=0.25, overlap=True,
                       reduce_dtype=torch.bfloat16 if rd == "bf16" else torch.float32, timing=True)
    ddp.broadcast_parameters()
    assert len(ddp.buckets) > 3, len(ddp.buckets)
    n = [0]
    orig = ddp._launch
    ddp._launch = lambda i: (n.__setitem__(0, n[0] + 1), orig(i))[1]
    losses = [float(ddp.train_step(m.to_input(x[s]), m.to_target(y[s]))) for s in range(3)]
    torch.cuda.synchronize()
    assert n[0] == 3 * len(ddp.buckets), (n, len(ddp.buckets))
    exposed = ddp.exposed_comm_ms()
    master = m.arena.master.detach().cpu().clone()
    full = ddp.measure_allreduce(iters=3)
    assert exposed is not None and exposed >= 0.0 and full is not None and full > 0.0, (exposed, full)
    ddp.check_replicas()
    torch.save({"master": master, "losses": losses, "exposed_ms": exposed, "allreduce_ms": full}, out)
    pg.shutdown()


if __name__ == "__main__":
    main()
