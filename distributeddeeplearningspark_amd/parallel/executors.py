"""Long-lived executor processes — the Spark executor analog.

In the reference, executors are JVM processes that YARN/AZTK start with the session
(``ddl_nyiso_hdi.ipynb:102-125``: 2 executors x 2 cores) and every ``trainer.train(df)``
ships tasks to those already-running processes (``mapPartitionsWithIndex``).
Here an :class:`ExecutorPool` is N worker interpreters (one per data-parallel replica,
bound to one MI355X each, or co-located per ``DDL_WORKERS_PER_GPU``) that import torch,
initialise HIP and join ONE process group (RCCL over xGMI, or gloo) once, then run any
number of tasks.  The driver talks to them over an authenticated local socket
(``multiprocessing.connection``); results come back pickled.

* Pools are cached by (world size, devices, backend) and reused by every trainer call, so
  ``get_training_time()`` measures training, not interpreter start-up — as in Spark, where
  the executors are up before the job is submitted.  ``SparkContext`` can pre-start the
  pool (``spark.ddl.prestartExecutors=true``) so it warms up while the driver runs the ETL.
* ``DDL_*`` environment variables of the driver are forwarded with every task (fault
  injection, restart counters and knobs set after the pool started still apply).
* Any task failure, worker death or timeout tears the whole pool down (a collective of
  the surviving ranks may be stuck); the launcher's restart logic then starts a new one.
* ``DDL_EXECUTOR_POOL=0`` disables caching (a fresh pool per call, stopped afterwards).
* Partition arrays do not travel through the task pickle: every numpy array of at least
  ``DDL_SHM_MIN_MB`` (default 1 MB) in a task's arguments is placed in POSIX shared memory
  (``/dev/shm``) once and the executors map it as a zero-copy ``np.ndarray`` view — the analog of
  the reference's cached partitions living on the executors (``repartition(num_workers)`` +
  ``cache()``, ``ddl_mnist_aztk.py:155-161``).  Blocks are cached per source array (a repeated
  ``train`` / ``predict`` on the same cached frame re-sends only a descriptor) and unlinked when the
  source array is freed or the pool shuts down.
"""
from __future__ import annotations

import atexit
import os
import pickle
import secrets
import subprocess
import sys
import threading
import time
import traceback
from multiprocessing.connection import Client, Listener

_POOLS: dict = {}
_LOCK = threading.Lock()


# ============================================================================ shared-memory shards
class ShmArray:
    """Picklable descriptor of a numpy array held in a POSIX shared-memory block."""

    __slots__ = ("name", "shape", "dtype", "offset")

    def __init__(self, name, shape, dtype, offset=0):
        self.name, self.shape, self.dtype, self.offset = name, tuple(shape), str(dtype), int(offset)

    def __getstate__(self):
        return (self.name, self.shape, self.dtype, self.offset)

    def __setstate__(self, st):
        self.name, self.shape, self.dtype, self.offset = st


_SHM_BLOCKS: dict = {}  # key -> (SharedMemory, ShmArray, weakref.finalize, content hash)
_SHM_LOCK = threading.Lock()


def _shm_min_bytes() -> int:
    return int(float(os.environ.get("DDL_SHM_MIN_MB", "1")) * (1 << 20))


def _release_block(key):
    with _SHM_LOCK:
        e = _SHM_BLOCKS.pop(key, None)
    if e is not None:
        try:
            e[0].close()
            e[0].unlink()
        except Exception:
            pass


def _fingerprint(a, base=None) -> int | None:
    """Content hash of a source array whose memory can change (None when the root buffer ``base``
    is read-only: then nothing can write it under the cache).  A read-only VIEW of a writable base
    is still hashed, since the base can be modified in place.  xxh3 runs at memory speed: ~10 ms
    per 150 MB shard."""
    import numpy as np

    root = a if base is None else base
    if not root.flags.writeable and not a.flags.writeable:
        return None
    buf = memoryview(np.ascontiguousarray(a)).cast("B")
    try:
        import xxhash

        return xxhash.xxh3_64_intdigest(buf)
    except ImportError:  # pragma: no cover - xxhash ships with the image
        import zlib

        return zlib.crc32(buf)


def share_array(a):
    """The shared-memory descriptor of ``a`` (copied into /dev/shm once per source array).

    The cache is keyed by the source buffer (zero-copy views of the user's arrays reach here), so a
    hit is re-validated against a content hash taken at copy time: an array the user modified in
    place between two ``train()`` / ``predict()`` calls is copied again, never served stale."""
    import weakref

    import numpy as np
    from multiprocessing import shared_memory

    base = a
    while isinstance(getattr(base, "base", None), np.ndarray):
        base = base.base
    key = (id(base), a.__array_interface__["data"][0], a.shape, a.strides, a.dtype.str)
    fp = _fingerprint(a, base)
    with _SHM_LOCK:
        e = _SHM_BLOCKS.get(key)
    if e is not None:
        if e[3] == fp:
            return e[1]
        c = np.ascontiguousarray(a)  # mutated in place since it was shared: refresh the block
        np.ndarray(c.shape, c.dtype, buffer=e[0].buf)[...] = c
        with _SHM_LOCK:
            _SHM_BLOCKS[key] = (e[0], e[1], e[2], fp)
        return e[1]
    c = np.ascontiguousarray(a)
    shm = shared_memory.SharedMemory(create=True, size=max(1, c.nbytes))
    np.ndarray(c.shape, c.dtype, buffer=shm.buf)[...] = c
    desc = ShmArray(shm.name, c.shape, c.dtype)
    try:
        fin = weakref.finalize(base, _release_block, key)
    except TypeError:  # not weak-referenceable: lives until the pool shuts down
        fin = None
    with _SHM_LOCK:
        _SHM_BLOCKS[key] = (shm, desc, fin, fp)
    return desc


def release_all_shared():
    for key in list(_SHM_BLOCKS):
        _release_block(key)


def _share_args(obj):
    import numpy as np

    if isinstance(obj, np.ndarray) and obj.nbytes >= _shm_min_bytes() and obj.dtype != object:
        return share_array(obj)
    if isinstance(obj, tuple):
        return tuple(_share_args(o) for o in obj)
    if isinstance(obj, list):
        return [_share_args(o) for o in obj]
    if isinstance(obj, dict):
        return {k: _share_args(v) for k, v in obj.items()}
    return obj


def _map_args(obj, opened):
    """Executor side: descriptors -> zero-copy ndarray views (the SharedMemory objects stay open
    in ``opened`` for the duration of the task)."""
    import numpy as np
    from multiprocessing import shared_memory

    if isinstance(obj, ShmArray):
        shm = opened.get(obj.name)
        if shm is None:
            shm = opened[obj.name] = shared_memory.SharedMemory(name=obj.name)
            try:  # the driver owns the block: this process's resource tracker must not unlink it at exit
                from multiprocessing import resource_tracker

                resource_tracker.unregister(shm._name, "shared_memory")
            except Exception:
                pass
        return np.ndarray(obj.shape, np.dtype(obj.dtype), buffer=shm.buf, offset=obj.offset)
    if isinstance(obj, tuple):
        return tuple(_map_args(o, opened) for o in obj)
    if isinstance(obj, list):
        return [_map_args(o, opened) for o in obj]
    if isinstance(obj, dict):
        return {k: _map_args(v, opened) for k, v in obj.items()}
    return obj


class PoolFailure(RuntimeError):
    def __init__(self, msg, short):
        super().__init__(msg)
        self.short = short


def _ddl_env() -> dict:
    return {k: v for k, v in os.environ.items() if k.startswith("DDL_")}


class ExecutorPool:
    def __init__(self, devices: list[str], backend: str | None, start_timeout_s: float = 600.0):
        from .launcher import free_port

        self.devices = list(devices)
        self.world = len(devices)
        self.backend = backend
        self.key = pool_key(devices, backend)
        self._authkey = secrets.token_bytes(16)
        self._listener = Listener(("127.0.0.1", 0), authkey=self._authkey)
        self._conns: dict[int, object] = {}
        self._accept_err = None
        self.closed = False
        self._ready = False
        self.tasks_run = 0
        threads = max(1, cpu_budget() // self.world)
        pg_port = free_port()
        env = dict(os.environ)
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = os.pathsep.join([root] + ([env["PYTHONPATH"]] if env.get("PYTHONPATH") else []))
        host, port = self._listener.address
        self.procs = []
        for r, dev in enumerate(self.devices):
            cmd = [sys.executable, "-m", "distributeddeeplearningspark_amd.parallel.executors", str(port),
                   self._authkey.hex(), str(r), str(self.world), str(pg_port), dev, backend or "", str(threads)]
            self.procs.append(subprocess.Popen(cmd, env=env))
        self._acceptor = threading.Thread(target=self._accept_all, daemon=True)
        self._acceptor.start()
        self._start_deadline = time.time() + start_timeout_s

    # ------------------------------------------------------------------ start-up
    def _accept_all(self):
        try:
            while len(self._conns) < self.world:
                c = self._listener.accept()
                kind, rank = c.recv()
                assert kind == "hello"
                self._conns[int(rank)] = c
        except BaseException as e:  # listener closed during shutdown, or a bad peer
            self._accept_err = e

    def wait_ready(self):
        if self._ready:
            return self
        while True:
            conns = list(self._conns.values())  # filled by the acceptor thread
            ready = sum(1 for c in conns if c.poll(0)) if len(conns) == self.world else 0
            if ready == self.world:
                for r in range(self.world):
                    kind, payload = self._conns[r].recv()
                    if kind != "ready":
                        self.shutdown(force=True)
                        raise PoolFailure(f"executor {r} failed to start:\n{payload}", f"executor {r} start failed")
                self._ready = True
                return self
            for r, p in enumerate(self.procs):
                if p.poll() is not None:
                    self.shutdown(force=True)
                    raise PoolFailure(f"executor {r} exited with code {p.returncode} during start-up",
                                      f"executor {r} died")
            if time.time() > self._start_deadline:
                self.shutdown(force=True)
                raise PoolFailure("executors did not start in time", "executor start timeout")
            time.sleep(0.02)

    # ------------------------------------------------------------------ tasks
    def run(self, fn, args_per_rank, timeout_s: float = 3600.0, attempt: int = 0):
        self.wait_ready()
        env = _ddl_env()
        env["DDL_RESTART_COUNT"] = str(attempt)
        paths = []
        try:  # the task function's own directory, so test / script modules unpickle in the executor
            import inspect

            paths.append(os.path.dirname(os.path.abspath(inspect.getfile(fn))))
        except (TypeError, OSError):
            pass
        for r in range(self.world):
            payload = pickle.dumps((fn, _share_args(args_per_rank[r])), protocol=pickle.HIGHEST_PROTOCOL)
            self.last_payload_bytes = len(payload)
            self._conns[r].send(("task", paths, payload, env))
        results, errors = {}, {}
        deadline = time.time() + timeout_s
        while len(results) + len(errors) < self.world:
            progressed = False
            for r in range(self.world):
                if r in results or r in errors:
                    continue
                c = self._conns[r]
                try:
                    has = c.poll(0)
                except (EOFError, OSError):
                    has = False
                if has:
                    try:
                        status, payload = c.recv()
                    except (EOFError, OSError):
                        status, payload = "error", f"executor {r} connection lost"
                    (results if status == "ok" else errors)[r] = payload
                    progressed = True
                elif self.procs[r].poll() is not None:
                    errors[r] = f"worker {r} exited with code {self.procs[r].returncode} without a result"
                    progressed = True
            if errors:
                break
            if time.time() > deadline:
                self.shutdown(force=True)
                raise TimeoutError(f"workers did not finish within {timeout_s}s")
            if not progressed:
                time.sleep(0.002)
        if errors:
            self.shutdown(force=True)
            r = sorted(errors)[0]
            raise PoolFailure(f"worker {r} failed:\n{errors[r]}", f"worker {r} failed")
        self.tasks_run += 1
        return [results[r] for r in range(self.world)]

    # ------------------------------------------------------------------ teardown
    def shutdown(self, force: bool = False):
        if self.closed:
            return
        self.closed = True
        with _LOCK:
            if _POOLS.get(self.key) is self:
                del _POOLS[self.key]
        if not force:
            for c in self._conns.values():
                try:
                    c.send(("stop",))
                except Exception:
                    pass
        deadline = time.time() + (10.0 if not force else 0.0)
        for p in self.procs:
            try:
                p.wait(timeout=max(0.0, deadline - time.time()))
            except subprocess.TimeoutExpired:
                pass
        for p in self.procs:
            if p.poll() is None:
                p.kill()
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    pass
        for c in self._conns.values():
            try:
                c.close()
            except Exception:
                pass
        try:
            self._listener.close()
        except Exception:
            pass


def cpu_budget() -> int:
    """CPUs this process may use: the affinity mask, capped by OMP_NUM_THREADS when that is set (a batch
    slot's CPU share shows up there, while os.cpu_count() and the affinity can report the whole host:
    sizing per-executor torch threads from those oversubscribed a 16-CPU share 12x)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 2
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def pool_key(devices, backend):
    return (len(devices), tuple(devices), backend)


def get_pool(devices: list[str], backend: str | None) -> ExecutorPool:
    """The cached pool for this topology (started if needed)."""
    key = pool_key(devices, backend)
    with _LOCK:
        pool = _POOLS.get(key)
        if pool is not None and not pool.closed and all(p.poll() is None for p in pool.procs):
            return pool
        if pool is not None:
            del _POOLS[key]
    if pool is not None:
        pool.shutdown(force=True)
    # one topology at a time: other cached pools hold GPUs / ports that this one may need
    shutdown_all()
    pool = ExecutorPool(devices, backend)
    with _LOCK:
        _POOLS[key] = pool
    return pool


def pooling_enabled() -> bool:
    return os.environ.get("DDL_EXECUTOR_POOL", "1") != "0"


def shutdown_all():
    with _LOCK:
        pools = list(_POOLS.values())
    for p in pools:
        p.shutdown()
    release_all_shared()


atexit.register(shutdown_all)


# ============================================================================ executor side
def _executor_main(port, authkey_hex, rank, world, pg_port, device, backend, threads):
    conn = Client(("127.0.0.1", int(port)), authkey=bytes.fromhex(authkey_hex))
    conn.send(("hello", int(rank)))
    pg = None
    try:
        import torch

        torch.set_num_threads(max(1, int(threads)))
        from .comm import init_process_group

        pg = init_process_group(int(rank), int(world), "127.0.0.1", int(pg_port), device=device,
                                backend=backend or None, timeout_s=600.0)
        conn.send(("ready", None))
    except BaseException:
        conn.send(("error", traceback.format_exc()))
        return 1
    base_env = {k: v for k, v in os.environ.items() if not k.startswith("DDL_")}
    while True:
        try:
            msg = conn.recv()
        except (EOFError, OSError):
            break  # driver went away
        if msg[0] == "stop":
            break
        _, paths, payload, env = msg
        for k in [k for k in os.environ if k.startswith("DDL_")]:
            del os.environ[k]
        os.environ.update(env)
        os.environ.update({k: v for k, v in base_env.items() if k not in os.environ})
        for pth in paths:
            if pth not in sys.path:
                sys.path.append(pth)
        opened = {}
        try:
            fn, args = pickle.loads(payload)
            # this file runs as __main__ in the executor: unpickled descriptors are instances of the
            # PACKAGE module's ShmArray, so map them with that module's helper
            from distributeddeeplearningspark_amd.parallel import executors as _pkg

            args = _pkg._map_args(args, opened)
            out = ("ok", fn(int(rank), int(world), pg, *args))
        except BaseException:  # report every failure to the driver
            out = ("error", traceback.format_exc())
        finally:
            args = None
            for shm in opened.values():
                try:
                    shm.close()
                except BufferError:  # a view is still referenced by the task's result: leave it mapped
                    pass
        try:
            conn.send(out)
        except Exception:
            conn.send(("error", "result could not be pickled:\n" + traceback.format_exc()))
        if out[0] == "error":
            break  # the driver tears the pool down after a failure
    try:
        if pg is not None:
            pg.shutdown()
    finally:
        conn.close()
    return 0


if __name__ == "__main__":
    sys.exit(_executor_main(*sys.argv[1:9]))
