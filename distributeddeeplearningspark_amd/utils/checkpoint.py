"""Checkpoint / resume.

The checkpoint format IS the reference's serialization, extended with what a restart
needs.  ``serialize_keras_model`` (``{'model': json, 'weights': get_weights()}``, reference
dist-keras ``utils.serialize_keras_model`` used by every trainer) is stored as

    <dir>/step_<n>/model.json        architecture (Keras-style JSON, ``model_from_json``)
    <dir>/step_<n>/weights.npz       Keras ``get_weights()`` arrays in order (w_000, w_001, ...)
    <dir>/step_<n>/state.safetensors fp32 master arena, optimizer slots, layer states (BN stats)
    <dir>/step_<n>/meta.json         step, optimizer config + iterations, RNG, user extras
    <dir>/latest                     name of the newest complete checkpoint
    <dir>/ranks/step_<n>/rank_<r>.safetensors
                                     per-worker state of the dist-keras worker algorithms
                                     (ADAG / DynSGD / DOWNPOUR / EASGD): that worker's weights,
                                     optimizer slots, layer states and the center variable it
                                     holds — worker-local state that differs between ranks

Writes go to a temporary directory renamed into place (a crash never leaves a torn
checkpoint); ``keep`` bounds how many are retained.  Loading never unpickles: npz with
``allow_pickle=False``, safetensors, JSON.
"""
from __future__ import annotations

import json
import os
import shutil
import tempfile

import numpy as np
import torch
from safetensors.torch import load_file, save_file


def _states_in_order(model):
    out = []
    for l in model.all_layers():
        for k, v in l._states.items():
            out.append(v)
    return out


def save_checkpoint(directory: str, model, step: int = 0, optimizer=None, extra: dict | None = None, keep: int = 3,
                    rank: int = 0) -> str | None:
    """Write a checkpoint (rank 0 only by default; data-parallel replicas are identical)."""
    if rank != 0:
        return None
    os.makedirs(directory, exist_ok=True)
    name = f"step_{int(step):09d}"
    final = os.path.join(directory, name)
    tmp = tempfile.mkdtemp(prefix=".tmp_", dir=directory)
    try:
        with open(os.path.join(tmp, "model.json"), "w") as f:
            f.write(model.to_json())
        ws = model.get_weights()
        np.savez(os.path.join(tmp, "weights.npz"), **{f"w_{i:03d}": np.asarray(w) for i, w in enumerate(ws)})
        tensors = {"arena.master": model.arena.get_flat().detach().float().cpu().contiguous()}
        for i, s in enumerate(_states_in_order(model)):
            tensors[f"layer_state.{i:04d}"] = s.detach().float().cpu().contiguous()
        opt = optimizer if optimizer is not None else model.optimizer
        meta = {"step": int(step), "format": "ddl-keras-v1", "num_weights": len(ws), "extra": extra or {}}
        if opt is not None:
            sd = opt.state_dict()
            meta["optimizer"] = {"config": opt.get_config(), "iterations": int(sd.pop("iterations", 0))}
            for k, v in sd.items():
                tensors[f"optim.{k}"] = v.float().contiguous()
        meta["rng"] = {"torch": torch.get_rng_state().tolist()}
        save_file(tensors, os.path.join(tmp, "state.safetensors"))
        with open(os.path.join(tmp, "meta.json"), "w") as f:
            json.dump(meta, f)
        if os.path.exists(final):
            shutil.rmtree(final)
        os.replace(tmp, final)
    except BaseException:
        shutil.rmtree(tmp, ignore_errors=True)
        raise
    with open(os.path.join(directory, "latest.tmp"), "w") as f:
        f.write(name)
    os.replace(os.path.join(directory, "latest.tmp"), os.path.join(directory, "latest"))
    _prune(directory, keep)
    return final


def _prune(directory, keep):
    ck = sorted(d for d in os.listdir(directory) if d.startswith("step_"))
    if keep <= 0 or not ck:
        return
    for d in ck[:-keep]:
        shutil.rmtree(os.path.join(directory, d), ignore_errors=True)
    # per-rank state is pruned against the keep window on its own: a run killed after the rank
    # files were written but before rank 0 published that step leaves a ranks/step_<n> with no
    # published step_<n>; anything older than the oldest kept step is stale either way
    oldest = ck[-keep] if len(ck) >= keep else ck[0]
    rdir = os.path.join(directory, "ranks")
    if os.path.isdir(rdir):
        for d in os.listdir(rdir):
            if d.startswith("step_") and d < oldest:
                shutil.rmtree(os.path.join(rdir, d), ignore_errors=True)


def _rank_file(directory: str, step: int, rank: int) -> str:
    return os.path.join(directory, "ranks", f"step_{int(step):09d}", f"rank_{int(rank):05d}.safetensors")


def save_rank_state(directory: str, model, step: int, rank: int, extra: dict | None = None) -> str:
    """Write THIS worker's state for checkpoint ``step``: its master weights, optimizer slots,
    layer states and any ``extra`` tensors (e.g. the center variable).  Call on every rank
    BEFORE rank 0's :func:`save_checkpoint` of the same step (with a barrier in between), so
    ``latest`` never names a step whose rank files are missing."""
    path = _rank_file(directory, step, rank)
    os.makedirs(os.path.dirname(path), exist_ok=True)
    tensors = {"arena.master": model.arena.get_flat().detach().float().cpu().contiguous()}
    for i, st in enumerate(_states_in_order(model)):
        tensors[f"layer_state.{i:04d}"] = st.detach().float().cpu().contiguous()
    opt = model.optimizer
    meta = {"rank": str(int(rank)), "step": str(int(step))}
    if opt is not None:
        sd = opt.state_dict()
        meta["iterations"] = str(int(sd.pop("iterations", 0)))
        for k, v in sd.items():
            tensors[f"optim.{k}"] = v.float().cpu().contiguous()
    for k, v in (extra or {}).items():
        tensors[f"extra.{k}"] = v.detach().float().cpu().contiguous()
    tmp = path + ".tmp"
    save_file(tensors, tmp, metadata=meta)
    os.replace(tmp, path)
    return path


def load_rank_state(checkpoint_path: str, model, rank: int) -> dict | None:
    """Restore this worker's state saved next to ``checkpoint_path`` (``<dir>/step_<n>``).
    Returns the ``extra`` tensors (on the model's device), or None if no rank file exists."""
    directory, name = os.path.split(os.path.normpath(checkpoint_path))
    step = int(name.split("_")[1])
    path = _rank_file(directory, step, rank)
    if not os.path.exists(path):
        return None
    from safetensors import safe_open

    with safe_open(path, framework="pt") as f:
        meta = f.metadata() or {}
    t = load_file(path)
    model.arena.set_flat(t["arena.master"])
    for i, st in enumerate(_states_in_order(model)):
        key = f"layer_state.{i:04d}"
        if key in t:
            st.copy_(t[key].to(st.device, st.dtype))
    opt = model.optimizer
    if opt is not None:
        if opt.arena is not model.arena:
            opt.bind(model.arena)
        sd = {k[len("optim."):]: v for k, v in t.items() if k.startswith("optim.")}
        sd["iterations"] = int(meta.get("iterations", 0))
        opt.load_state_dict(sd)
    dev = model.arena.master.device
    return {k[len("extra."):]: v.to(dev) for k, v in t.items() if k.startswith("extra.")}


def latest_checkpoint(directory: str) -> str | None:
    p = os.path.join(directory, "latest")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        name = f.read().strip()
    full = os.path.join(directory, name)
    return full if os.path.isdir(full) else None


def load_checkpoint(path: str, model=None, device=None, restore_rng: bool = False):
    """Restore a checkpoint directory (or the ``latest`` of a checkpoint root).

    Returns ``(model, meta)``.  With ``model=None`` the model is rebuilt from
    ``model.json``; otherwise weights/states/optimizer are loaded into ``model`` in place."""
    if os.path.exists(os.path.join(path, "latest")):
        path = latest_checkpoint(path)
    with open(os.path.join(path, "meta.json")) as f:
        meta = json.load(f)
    if model is None:
        from ..models.core import model_from_json

        with open(os.path.join(path, "model.json")) as f:
            model = model_from_json(f.read())
        if "optimizer" in meta:
            from ..models import optimizers as O

            model.compile(O.get(meta["optimizer"]["config"]), model.loss or "mean_squared_error")
    if model.arena is None or (device is not None and torch.device(device) != model.device):
        model.place(device or ("cuda" if torch.cuda.is_available() else "cpu"))
    t = load_file(os.path.join(path, "state.safetensors"))
    model.arena.set_flat(t["arena.master"])
    for i, s in enumerate(_states_in_order(model)):
        key = f"layer_state.{i:04d}"
        if key in t:
            s.copy_(t[key].to(s.device, s.dtype))
    if model.optimizer is not None and "optimizer" in meta:
        if model.optimizer.arena is not model.arena:
            model.optimizer.bind(model.arena)
        sd = {k[len("optim."):]: v for k, v in t.items() if k.startswith("optim.")}
        sd["iterations"] = meta["optimizer"]["iterations"]
        model.optimizer.load_state_dict(sd)
    if restore_rng and "rng" in meta:
        torch.set_rng_state(torch.tensor(meta["rng"]["torch"], dtype=torch.uint8))
    return model, meta


def load_keras_weights(path: str) -> list[np.ndarray]:
    """The reference-format weight list of a checkpoint (``get_weights()`` order)."""
    with np.load(os.path.join(path, "weights.npz"), allow_pickle=False) as z:
        return [z[k] for k in sorted(z.files)]
