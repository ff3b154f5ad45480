"""Keras-compatible model API and model zoo."""
from .core import Layer, Model, Sequential, model_from_json  # noqa: F401
from .layers import (Activation, AveragePooling2D, BatchNormalization, Conv2D, Dense, Dropout, Embedding,  # noqa: F401
                     Flatten, GlobalAveragePooling2D, GRU, LSTM, MaxPooling2D, Reshape, SimpleRNN)
from .resnet import ResNet, ResNet50, ResNet101  # noqa: F401
from . import optimizers  # noqa: F401
from .bert import BertConfig, BertForMaskedLM, bert_base_mlm  # noqa: F401
