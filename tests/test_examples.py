"""End-to-end runs of the reference workflows (examples/) on CPU executors."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "examples"))


@pytest.fixture(autouse=True)
def _fresh_session():
    from distributeddeeplearningspark_amd.context import SparkSession

    yield
    if SparkSession._active is not None:
        SparkSession._active.stop()


def test_ddl_mnist_workflow(monkeypatch, capsys):
    import ddl_mnist

    monkeypatch.setattr(sys, "argv", ["ddl_mnist.py", "--executors", "2", "--processes", "1", "--device", "cpu",
                                      "--train-rows", "512", "--test-rows", "128"])
    trainer, model = ddl_mnist.main()
    out = capsys.readouterr().out
    assert "Total params: 1,048,853" in out
    # 512 rows / 2 workers = 256 rows -> 16 batches of 16 -> floor(16 / 5) = 3 commits per worker
    assert trainer.parameter_server.num_updates == 6
    acc = float(out.strip().splitlines()[-2].split(": ")[1])
    assert acc > 0.8


def test_storage_attach_resolves_wasb_uri(tmp_path):
    from distributeddeeplearningspark_amd.context import SparkSession
    from distributeddeeplearningspark_amd.utils.storage import attach_storage_container, resolve

    spark = SparkSession.builder.master("local[1]").getOrCreate()
    attach_storage_container(spark, "acct", key="secret-not-kept", root=str(tmp_path))
    assert resolve("wasbs://c@acct.blob.core.windows.net/a/b.csv") == os.path.join(str(tmp_path), "acct", "c", "a/b.csv")
    assert "secret" not in str(spark.conf.get("fs.azure.account.key.acct.blob.core.windows.net"))
    with pytest.raises(IOError):
        resolve("wasbs://c@other.blob.core.windows.net/x")
