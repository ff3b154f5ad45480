#!/usr/bin/env python
"""MNIST CNN trained with ADAG — the reference's ``ddl_mnist_aztk.py`` workflow on this
framework: Spark bootstrap -> storage attach -> CSV ingest -> feature
transformers (VectorAssembler, OneHot, MinMax, Reshape, Dense) -> ``repartition(num_workers)``
-> Keras-style CNN -> ``ADAG(...).train(df)`` -> ``ModelPredictor`` + ``AccuracyEvaluator``.

Differences: the CSVs are synthetic MNIST-shaped files written into a local
mount of the ``wasbs://`` container (no network, no account key), ``local[N]`` replaces the
AZTK master, and each worker is one process per MI355X (or CPU executor).

    python examples/ddl_mnist.py [--executors 4] [--processes 2] [--epochs 1] [--device auto|cpu]

Attribution: the pipeline (transformer sequence, trainer and evaluation calls) follows the
reference script ``ddl_mnist_aztk.py`` (chenhuims/DistributedDeepLearningSpark, GPLv3), whose
public dist-keras/Spark API this framework reproduces.
"""
from __future__ import annotations

import argparse
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributeddeeplearningspark_amd.context import SparkConf, SparkContext, SparkSession, SQLContext  # noqa: E402
from distributeddeeplearningspark_amd.data.synthetic import mnist_like  # noqa: E402
from distributeddeeplearningspark_amd.evaluators import AccuracyEvaluator  # noqa: E402
from distributeddeeplearningspark_amd.ml.feature import VectorAssembler  # noqa: E402
from distributeddeeplearningspark_amd.models import Activation, Conv2D, Dense, Flatten, MaxPooling2D  # noqa: E402
from distributeddeeplearningspark_amd.models import Sequential  # noqa: E402
from distributeddeeplearningspark_amd.predictors import ModelPredictor  # noqa: E402
from distributeddeeplearningspark_amd.trainers import ADAG  # noqa: E402
from distributeddeeplearningspark_amd.transformers import (DenseTransformer, LabelIndexTransformer,  # noqa: E402
                                                            MinMaxTransformer, OneHotTransformer, ReshapeTransformer)
from distributeddeeplearningspark_amd.utils import get_os_username  # noqa: E402
from distributeddeeplearningspark_amd.utils.storage import attach_storage_container  # noqa: E402

ACCOUNT, CONTAINER = "ddlstorage", "mnist"


def write_synthetic_csvs(root: str, n_train: int, n_test: int):
    import pandas as pd

    base = os.path.join(root, ACCOUNT, CONTAINER)
    os.makedirs(base, exist_ok=True)
    for name, n, seed in (("mnist_train.csv", n_train, 0), ("mnist_test.csv", n_test, 1)):
        pd.DataFrame(mnist_like(n, seed=seed)).to_csv(os.path.join(base, name), index=False)


def evaluate_accuracy(model, test_set, features="matrix"):
    """Accuracy of ``model`` on ``test_set``: predict -> argmax class index -> AccuracyEvaluator,
    the same three steps as the reference's helper (``ddl_mnist_aztk.py:202-210``; the
    reference is GPLv3, this workflow mirrors its API calls, not its code)."""
    scored = ModelPredictor(keras_model=model, features_col=features).predict(test_set.select(features, "label"))
    indexed = LabelIndexTransformer(output_dim=10).transform(scored)
    return AccuracyEvaluator(prediction_col="prediction_index", label_col="label").evaluate(indexed)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--executors", type=int, default=2)
    ap.add_argument("--processes", type=int, default=2)
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--train-rows", type=int, default=4096)
    ap.add_argument("--test-rows", type=int, default=1024)
    ap.add_argument("--device", default="auto")
    ap.add_argument("--workers-per-gpu", type=int, default=None,
                    help="co-locate replicas on one MI355X (the reference's 8 workers on a smaller node)")
    args = ap.parse_args()
    if args.workers_per_gpu:
        os.environ["DDL_WORKERS_PER_GPU"] = str(args.workers_per_gpu)

    num_workers = args.executors * args.processes  # A4: workers = executors x processes
    print("Number of desired executors: " + str(args.executors))
    print("Number of desired processes / executor: " + str(args.processes))
    print("Total number of workers: " + str(num_workers))

    conf = SparkConf()
    conf.set("spark.app.name", "Distributed Deep Learning on MI355X")
    conf.set("spark.master", f"local[{num_workers}]")
    conf.set("spark.executor.cores", str(args.processes))
    conf.set("spark.executor.instances", str(args.executors))
    conf.set("spark.locality.wait", "0")
    conf.set("spark.serializer", "org.apache.spark.serializer.KryoSerializer")
    conf.set("spark.local.dir", "/tmp/" + get_os_username() + "/spark/")
    # executors come up (torch import, HIP init, process group) while the driver runs the ETL
    conf.set("spark.ddl.prestartExecutors", "true").set("spark.ddl.device", args.device)
    sc = SparkContext(conf=conf)
    sqlc = SQLContext(sc)
    spark = SparkSession.builder.getOrCreate()
    spark.sparkContext.setLogLevel("ERROR")

    root = tempfile.mkdtemp(prefix="ddl_storage_")
    write_synthetic_csvs(root, args.train_rows, args.test_rows)
    attach_storage_container(spark, ACCOUNT, key=None, root=root)
    url = f"wasbs://{CONTAINER}@{ACCOUNT}.blob.core.windows.net/"
    raw_dataset_train = sqlc.read.format("com.databricks.spark.csv").options(header="true", inferSchema="true") \
        .load(url + "mnist_train.csv")
    raw_dataset_test = sqlc.read.format("com.databricks.spark.csv").options(header="true", inferSchema="true") \
        .load(url + "mnist_test.csv")

    features = [c for c in raw_dataset_train.columns if c != "label"]
    vector_assembler = VectorAssembler(inputCols=features, outputCol="features")
    dataset_train = vector_assembler.transform(raw_dataset_train)
    dataset_test = vector_assembler.transform(raw_dataset_test)
    encoder = OneHotTransformer(10, input_col="label", output_col="label_encoded")
    dataset_train = encoder.transform(dataset_train)
    dataset_test = encoder.transform(dataset_test)
    transformer = MinMaxTransformer(n_min=0.0, n_max=1.0, o_min=0.0, o_max=250.0, input_col="features",
                                    output_col="features_normalized")
    dataset_train = transformer.transform(dataset_train)
    dataset_test = transformer.transform(dataset_test)
    reshape_transformer = ReshapeTransformer("features_normalized", "matrix", (28, 28, 1))
    dataset_train = reshape_transformer.transform(dataset_train)
    dataset_test = reshape_transformer.transform(dataset_test)
    dense_transformer = DenseTransformer(input_col="features_normalized", output_col="features_normalized_dense")
    dataset_train = dense_transformer.transform(dataset_train)
    dataset_test = dense_transformer.transform(dataset_test)
    dataset_train = dataset_train.select("features_normalized_dense", "matrix", "label", "label_encoded")
    dataset_test = dataset_test.select("features_normalized_dense", "matrix", "label", "label_encoded")
    dataset_train = dataset_train.repartition(num_workers)
    dataset_test = dataset_test.repartition(num_workers)
    dataset_train.cache()
    dataset_test.cache()
    print("Training set size: " + str(dataset_train.count()))

    mnist = Sequential()
    mnist.add(Conv2D(32, kernel_size=(3, 3), input_shape=(28, 28, 1), padding="valid"))
    mnist.add(Activation("relu"))
    mnist.add(Conv2D(32, kernel_size=(3, 3)))
    mnist.add(Activation("relu"))
    mnist.add(MaxPooling2D(pool_size=(2, 2)))
    mnist.add(Flatten())
    mnist.add(Dense(225))
    mnist.add(Activation("relu"))
    mnist.add(Dense(10))
    mnist.add(Activation("softmax"))
    mnist.summary()

    optimizer_mnist = "adam"
    loss_mnist = "categorical_crossentropy"
    device = None if args.device == "auto" else args.device
    sc.awaitExecutors()  # session start-up ends here (the reference's executors were up before training)
    trainer = ADAG(keras_model=mnist, worker_optimizer=optimizer_mnist, loss=loss_mnist, num_workers=num_workers,
                   batch_size=16, communication_window=5, num_epoch=args.epochs, features_col="matrix",
                   label_col="label_encoded", device=device)
    trained_model = trainer.train(dataset_train)
    print("Training time: " + str(trainer.get_training_time()))
    print("Accuracy: " + str(evaluate_accuracy(trained_model, dataset_test)))
    print("Number of parameter server updates: " + str(trainer.parameter_server.num_updates))
    rs = getattr(trainer, "_results", [])
    print("Workers:", [{k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()
                        if k in ("rank", "time", "commit_s", "commit_wait_s", "commit_xfer_s", "graph", "ingest")} for r in rs])
    groups = [r["replica_group"] for r in rs if "replica_group" in r]
    if groups:
        print("Replica groups: batched", [g["batched"] for g in groups], "shard rows", trainer.worker_rows)
    return trainer, trained_model


if __name__ == "__main__":
    np.set_printoptions(precision=4)
    main()
