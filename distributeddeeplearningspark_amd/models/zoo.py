"""Model zoo: the reference's three models and the north-star configs.

* ``mnist_cnn``       conv32-conv32-pool-dense225-dense10 (``ddl_mnist_aztk.py:180-192``),
                      1,048,853 params.
* ``gru_regressor``   GRU(128, input (25,1)) + Dense(1) (``ddl_nyiso_aztk.py:201-203``), 50,049.
* ``lstm_regressor``  LSTM(128) + Dense(1) (``ddl_nyiso_aztk.py:249-251``), 66,689.
* ``lenet5``          LeNet-5 on MNIST shape (BASELINE.json config #1).
* ``vgg16``           VGG-16 (BN) in the CIFAR shape (BASELINE.json config #4).
* ResNet-50 lives in ``resnet.py``; BERT-base in ``bert.py``.
"""
from __future__ import annotations

from .core import Sequential
from .layers import (GRU, LSTM, Activation, BatchNormalization, Conv2D, Dense, Dropout, Flatten,
                     MaxPooling2D)


def mnist_cnn(nb_classes: int = 10, input_shape=(28, 28, 1), nb_filters: int = 32) -> Sequential:
    m = Sequential()
    m.add(Conv2D(nb_filters, (3, 3), padding="valid", input_shape=input_shape))
    m.add(Activation("relu"))
    m.add(Conv2D(nb_filters, (3, 3)))
    m.add(Activation("relu"))
    m.add(MaxPooling2D(pool_size=(2, 2)))
    m.add(Flatten())
    m.add(Dense(225))
    m.add(Activation("relu"))
    m.add(Dense(nb_classes))
    m.add(Activation("softmax"))
    return m


def gru_regressor(units: int = 128, seq_len: int = 25, features: int = 1, outputs: int = 1) -> Sequential:
    m = Sequential()
    m.add(GRU(units, input_shape=(seq_len, features)))
    m.add(Dense(outputs, activation="linear"))
    return m


def lstm_regressor(units: int = 128, seq_len: int = 25, features: int = 1, outputs: int = 1) -> Sequential:
    m = Sequential()
    m.add(LSTM(units, input_shape=(seq_len, features)))
    m.add(Dense(outputs, activation="linear"))
    return m


def lenet5(nb_classes: int = 10, input_shape=(28, 28, 1)) -> Sequential:
    m = Sequential()
    m.add(Conv2D(6, (5, 5), padding="same", activation="relu", input_shape=input_shape))
    m.add(MaxPooling2D((2, 2)))
    m.add(Conv2D(16, (5, 5), activation="relu"))
    m.add(MaxPooling2D((2, 2)))
    m.add(Flatten())
    m.add(Dense(120, activation="relu"))
    m.add(Dense(84, activation="relu"))
    m.add(Dense(nb_classes, activation="softmax"))
    return m


def vgg16(nb_classes: int = 10, input_shape=(32, 32, 3), batch_norm: bool = True) -> Sequential:
    cfg = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]
    m = Sequential()
    first = True
    for v in cfg:
        if v == "M":
            m.add(MaxPooling2D((2, 2)))
            continue
        kw = {"input_shape": input_shape} if first else {}
        first = False
        m.add(Conv2D(v, (3, 3), padding="same", use_bias=not batch_norm, kernel_initializer="he_normal", **kw))
        if batch_norm:
            m.add(BatchNormalization(momentum=0.9, epsilon=1e-5))
        m.add(Activation("relu"))
    m.add(Flatten())
    m.add(Dense(512, activation="relu"))
    m.add(Dropout(0.5))
    m.add(Dense(512, activation="relu"))
    m.add(Dropout(0.5))
    m.add(Dense(nb_classes, activation="softmax"))
    return m
