"""dist-keras ``distkeras.utils`` equivalents.

``serialize_keras_model`` / ``deserialize_keras_model`` keep the reference's de-facto
model/checkpoint format: ``{'model': <architecture JSON>, 'weights': [arrays in Keras
get_weights() order and layouts]}``.  The flat fp32 arena is shipped
alongside (``'flat'``) so workers rebuild replicas with one copy, plus the BN running
statistics (``'states'``).
"""
from __future__ import annotations

import getpass
import os
import pwd

import numpy as np


def get_os_username() -> str:
    """Username used by the reference for ``spark.local.dir`` (``ddl_mnist_aztk.py:71``)."""
    try:
        return pwd.getpwuid(os.getuid()).pw_name
    except KeyError:  # pragma: no cover - container without passwd entry
        return getpass.getuser()


def serialize_keras_model(model) -> dict:
    model.build_model()
    d = {"model": model.to_json(), "weights": model.get_weights()}
    if model.arena is not None:
        d["flat"] = model.arena.get_flat().detach().cpu().numpy().copy()  # canonical layout (params.py)
    d["states"] = {f"{l.name}/{k}": v.detach().cpu().numpy().copy()
                   for l in model.all_layers() for k, v in l._states.items()}
    if model.optimizer is not None:
        d["optimizer"] = model.optimizer.get_config()
        d["loss"] = model.loss if isinstance(model.loss, str) else None
    return d


def deserialize_keras_model(d: dict, device=None):
    import torch

    from ..models.core import model_from_json

    m = model_from_json(d["model"])
    m.build_model()
    m.set_weights(d["weights"])
    if device is not None:
        m.place(device)
    if d.get("states"):
        set_states(m, d["states"])
    if d.get("optimizer") and d.get("loss"):
        m.compile(d["optimizer"], d["loss"])
    _ = torch
    return m


def set_states(model, states: dict):
    import torch

    for l in model.all_layers():
        for k in list(l._states):
            key = f"{l.name}/{k}"
            if key in states:
                l._states[k].copy_(torch.as_tensor(states[key]).to(l._states[k].device))


def get_states(model) -> dict:
    return {f"{l.name}/{k}": v.detach().cpu().numpy().copy() for l in model.all_layers() for k, v in l._states.items()}


def uniform_weights(model, constraints=(-0.5, 0.5), seed=None):
    rng = np.random.default_rng(seed)
    ws = model.get_weights()
    model.set_weights([rng.uniform(constraints[0], constraints[1], w.shape).astype(np.float32) for w in ws])


def weights_mean(weights_list):
    return [np.mean(np.stack(ws), axis=0) for ws in zip(*weights_list)]


def shuffle(dataframe, seed=None):
    """Row shuffle of a DataFrame (dist-keras ``shuffle``)."""
    rng = np.random.default_rng(seed)
    return dataframe._select_rows(rng.permutation(dataframe.count()), parts=[0, dataframe.count()])


def precache(dataframe):
    dataframe.cache()
    dataframe.count()
    return dataframe


def history_executors_average(history):
    """Average the per-worker loss histories step by step (dist-keras helper)."""
    if not history:
        return []
    n = min(len(h) for h in history)
    return [float(np.mean([h[i] for h in history])) for i in range(n)]


__all__ = ["get_os_username", "serialize_keras_model", "deserialize_keras_model", "uniform_weights",
           "weights_mean", "shuffle", "precache", "history_executors_average", "set_states", "get_states"]
