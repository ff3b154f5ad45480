"""Per-step time of the reference's GRU/LSTM regressors (batch 32, 25x1 -> 128 units) with the
hipGraph-captured step; run under rocprofv3 for the kernel breakdown."""
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from distributeddeeplearningspark_amd.models import zoo  # noqa: E402
from distributeddeeplearningspark_amd.models.step import CompiledTrainStep  # noqa: E402

for name, build, opt in (("GRU", zoo.gru_regressor, "adagrad"), ("LSTM", zoo.lstm_regressor, "adam")):
    m = build()
    m.compile(opt, "mean_squared_error")
    m.place("cuda:0", seed=0)
    st = CompiledTrainStep(m)
    x = m.to_input(torch.rand(32, 25, 1))
    y = m.to_target(torch.rand(32, 1))
    for _ in range(5):
        st(x, y)
    torch.cuda.synchronize()
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    t0 = time.perf_counter()
    for _ in range(n):
        st(x, y)
    torch.cuda.synchronize()
    print(f"{name}: {(time.perf_counter() - t0) / n * 1e6:.1f} us/step (graph={st.captured})", flush=True)
