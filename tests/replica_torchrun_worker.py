"""torchrun entry for tests/test_replicas_cpu.py::test_replica_groups_under_torchrun: a dist-keras trainer with
more workers than ranks (k workers per rank as one replica group, commit sums over the job's gloo group).
Rank 0 writes the result as JSON to argv[2]."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributeddeeplearningspark_amd import trainers as T  # noqa: E402
from distributeddeeplearningspark_amd.context import SparkSession  # noqa: E402
from distributeddeeplearningspark_amd.models import Dense, Sequential  # noqa: E402


def main():
    algo, out = sys.argv[1], sys.argv[2]
    spark = SparkSession.builder.master("local[2]").getOrCreate()
    rng = np.random.default_rng(3)
    x = rng.normal(size=(70, 5)).astype(np.float32)
    y = (x @ np.arange(1, 6, dtype=np.float32)[:, None] * 0.1 + 0.3).astype(np.float32)
    df = spark.createDataFrame({"f": list(x), "l": list(y)}).repartition(3)
    base = Sequential([Dense(4, activation="relu", input_shape=(5,)), Dense(1)])
    base.set_weights([np.full_like(w, 0.05 * (i + 1)) + np.linspace(-0.1, 0.1, w.size, dtype=np.float32).reshape(w.shape)
                      for i, w in enumerate(base.get_weights())])
    tr = getattr(T, algo)(keras_model=base, worker_optimizer="adam", loss="mean_squared_error", num_workers=4,
                          batch_size=4, num_epoch=2, features_col="f", label_col="l", device="cpu",
                          communication_window=3)
    model = tr.train(df)
    if int(os.environ["RANK"]) == 0:
        json.dump({"num_updates": tr.parameter_server.num_updates, "history": tr.get_history(),
                   "weights": [w.tolist() for w in model.get_weights()],
                   "replica_group": [r.get("replica_group") for r in tr._results]}, open(out, "w"))


if __name__ == "__main__":
    main()
