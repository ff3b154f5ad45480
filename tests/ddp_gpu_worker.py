"""Worker of tests/test_gpu_ddp.py (run under torch.distributed.run): data-parallel training
of a small ResNet on the HIP fused path with overlapped bucket all-reduce hooks."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributeddeeplearningspark_amd.models.optimizers import SGD
from distributeddeeplearningspark_amd.models.resnet import ResNet
from distributeddeeplearningspark_amd.parallel import comm
from distributeddeeplearningspark_amd.parallel.ddp import DataParallel


def main():
    out = sys.argv[1]
    pg = comm.init_from_env(prefer_gpu=True)
    torch.manual_seed(0)
    x = torch.randn(2, 16, 32, 32, 3)
    y = torch.randint(0, 10, (2, 16))
    m = ResNet(blocks=(2, 1), input_shape=(32, 32, 3), num_classes=10)
    m.compile(SGD(lr=0.05, momentum=0.9), "sparse_categorical_crossentropy")
    m.place(pg.device, seed=3)
    ddp = DataParallel(m, pg, bucket_mb=0.25, overlap=True)
    ddp.broadcast_parameters()
    assert len(ddp.buckets) > 3, len(ddp.buckets)
    losses = []
    for step in range(2):
        xb, yb = m.to_input(x[pg.rank]), m.to_target(y[pg.rank])
        losses.append(float(ddp.train_step(xb, yb)))
    ddp.check_replicas()
    if pg.rank == 0:
        torch.save({"master": m.arena.master.detach().cpu(), "losses": losses}, out)
    pg.shutdown()


if __name__ == "__main__":
    main()
