"""distributeddeeplearningspark_amd — an MI355X-native data-parallel deep-learning framework
with the Spark-DataFrame / Distributed-Keras front end of chenhuims/DistributedDeepLearningSpark.

Layers:
  * ``sql`` / ``ml`` / ``context``  Spark-API-compatible DataFrame engine (no JVM)
  * ``transformers`` / ``predictors`` / ``evaluators`` / ``trainers``  dist-keras API
  * ``models``   Keras-compatible model API + model zoo (ResNet-50, VGG-16, BERT, LeNet-5, CNN, GRU/LSTM)
  * ``ops``      HIP/CDNA4 kernels (MFMA implicit GEMM, BN, pooling, losses, optimizers)
  * ``parallel`` one process per GPU, RCCL (torch.distributed "nccl") bucketed all-reduce over xGMI
  * ``utils``    checkpoint/resume, tracing, metrics, fault injection
"""
__version__ = "0.1.0"
