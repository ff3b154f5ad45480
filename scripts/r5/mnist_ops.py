"""List the ATen ops (with their kernel launches) of one eager MNIST replica step (batch 16)."""
import sys, os
sys.path.insert(0, os.getcwd())
import torch
from torch.profiler import profile, ProfilerActivity
from distributeddeeplearningspark_amd.models import Activation, Conv2D, Dense, Flatten, MaxPooling2D, Sequential
from distributeddeeplearningspark_amd.ops._native import C

m = Sequential()
m.add(Conv2D(32, kernel_size=(3, 3), input_shape=(28, 28, 1), padding="valid"))
m.add(Activation("relu"))
m.add(Conv2D(32, kernel_size=(3, 3)))
m.add(Activation("relu"))
m.add(MaxPooling2D(pool_size=(2, 2)))
m.add(Flatten())
m.add(Dense(225))
m.add(Activation("relu"))
m.add(Dense(10))
m.add(Activation("softmax"))
m.compile("adam", "categorical_crossentropy")
m.place("cuda")
X = torch.rand(64, 28, 28, 1, device="cuda").to(torch.bfloat16)
Y = torch.nn.functional.one_hot(torch.randint(0, 10, (64,), device="cuda"), 10).float()
sx, sy = torch.empty_like(X[:16]), torch.empty_like(Y[:16])
ctr = torch.zeros(1, dtype=torch.int32, device="cuda")
hist = torch.zeros(100, device="cuda")
m.optimizer.enable_device_step()
def step():
    C().batch_fetch([X, Y], [sx, sy], ctr, 4)
    loss = m.backward_step(m.to_input(sx), m.to_target(sy))
    m.optimizer.captured_update(1.0)
    C().step_record(loss.detach().float().reshape(1), hist, ctr)
for _ in range(3):
    step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as p:
    step()
    torch.cuda.synchronize()
ev = [e for e in p.events()]
# print every CPU aten op that has device kernels, in order
for e in ev:
    if e.device_type == torch.autograd.DeviceType.CPU and e.name.startswith("aten::"):
        ks = [k.name[:60] for k in e.kernels]
        if ks:
            print(f"{e.name:32s} {str(e.input_shapes)[:70]:70s} {ks}")
print("---- kernels in order")
for e in ev:
    if e.device_type != torch.autograd.DeviceType.CPU:
        print(e.name[:100])
