"""Asynchronous parameter server (driver-hosted center variable), backed by the native
C++ TCP server in ``csrc/runtime/param_server.cpp``.

This is the reference's execution model for ADAG / DynSGD / DOWNPOUR / AEASGD
(``distkeras/parameter_servers.py`` SocketParameterServer + ``distkeras/workers.py``
NetworkWorker.pull/commit): workers train locally, and every
``communication_window`` mini-batches commit a residual and pull the newest center —
without any barrier between workers, so updates can be stale.

Differences by design: fixed binary framing (1-byte action + int64 header + raw fp32)
instead of pickled dicts over sockets, one native thread per connection, the center
update applied in C++ under one mutex, and DynSGD's staleness rule
(``1/(num_updates - last_update + 1)``) evaluated server-side.

On MI355X nodes the synchronous RCCL path (``trainers`` default ``mode="sync"``) is the
fast one; ``mode="async"`` exists for semantic parity with the reference's true
asynchrony.  The server binds 127.0.0.1 (single node).
"""
from __future__ import annotations

import torch

from ..ops._native import C

RULE_ADD = 0
RULE_DYNSGD = 1


class ParameterServerProcess:
    """Driver side: owns the center variable; ``port`` is what workers connect to."""

    def __init__(self, center: torch.Tensor, rule: int = RULE_ADD, port: int = 0):
        self._init = center.detach().to("cpu", torch.float32).contiguous().clone()
        self._srv = C().ParamServer(self._init, int(rule), int(port))

    @property
    def port(self) -> int:
        return self._srv.port

    @property
    def num_updates(self) -> int:
        return self._srv.num_updates

    def center(self) -> torch.Tensor:
        out = torch.empty_like(self._init)
        self._srv.get_center(out)
        return out

    def stop(self):
        if self._srv is not None:
            self._srv.stop()
            self._srv = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.stop()


class ParameterServerClient:
    """Worker side: ``pull()`` the center into a host buffer, ``commit()`` a residual."""

    def __init__(self, port: int, worker_id: int, numel: int, host: str = "127.0.0.1"):
        self._c = C().PSClient(host, int(port), int(worker_id))
        self._buf = torch.empty(int(numel), dtype=torch.float32).pin_memory() if torch.cuda.is_available() \
            else torch.empty(int(numel), dtype=torch.float32)
        self.last_update = 0

    def pull(self) -> torch.Tensor:
        self.last_update = self._c.pull(self._buf)
        return self._buf

    def commit(self, residual: torch.Tensor):
        r = residual.detach().to("cpu", torch.float32).contiguous()
        self._c.commit(r, self.last_update)

    def close(self):
        self._c.close()
