"""Print the deterministic GPU windows of the envelope task: unmutated, one block's shortcut dropped, all dropped."""
import os
import sys

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np

import test_gpu_convergence as T

for mut in (None, ("drop_shortcut", "resnet50/s3b6"), ("drop_shortcut", None)):
    h = T._hard_curve(mut)
    print(mut, [round(float(h[a:a + 10].mean()), 3) for a in range(0, len(h), 10)], flush=True)
