"""``pyspark.sql.window.Window``: partitionBy/orderBy specs evaluated by a stable
vectorised sort + per-group shift (lag/lead) — the reference builds its 24 lag and
1 lead feature columns this way (``ddl_nyiso_aztk.py:140-146``)."""
from __future__ import annotations

import numpy as np

from .column import ColumnData, _as_column


def _sort_keys(cds):
    keys = []
    for cd in cds:
        v = cd.values
        if v.dtype == object:
            # strings / mixed: rank by python ordering (None first, as Spark's nulls-first ascending)
            uniq = sorted({x for x in v if x is not None}, key=lambda x: (str(type(x)), x))
            pos = {u: i + 1 for i, u in enumerate(uniq)}
            v = np.array([0 if x is None else pos[x] for x in v], dtype=np.int64)
        elif cd.mask is not None:
            v = v.astype(np.float64) if v.dtype.kind in "iuf" else v.astype("datetime64[us]").astype(np.int64).astype(np.float64)
            v = np.where(cd.mask, v, -np.inf)
        keys.append(v)
    return keys


class WindowSpec:
    def __init__(self, part=(), order=()):
        self._part = list(part)
        self._order = list(order)

    def partitionBy(self, *cols):
        cols = cols[0] if len(cols) == 1 and isinstance(cols[0], (list, tuple)) else cols
        return WindowSpec(list(cols), self._order)

    def orderBy(self, *cols):
        cols = cols[0] if len(cols) == 1 and isinstance(cols[0], (list, tuple)) else cols
        return WindowSpec(self._part, list(cols))

    def rowsBetween(self, start, end):
        return self

    def _order_index(self, table):
        part = [_as_column(c)._expr.eval(table) for c in self._part]
        order_cols = [_as_column(c) for c in self._order]
        order = [c._expr.eval(table) for c in order_cols]
        asc = [getattr(c, "_ascending", True) for c in order_cols]
        pk = _sort_keys(part)
        ok = _sort_keys(order)
        ok = [k if a else (-k if k.dtype.kind in "if" else -k.astype(np.int64)) for k, a in zip(ok, asc)]
        keys = list(reversed(pk + ok))  # np.lexsort: last key is primary
        n = table.nrows
        idx = np.lexsort(keys) if keys else np.arange(n)
        # group ids (in sorted order)
        if pk:
            sp = np.stack([k[idx] for k in pk], 1) if len(pk) > 1 else pk[0][idx][:, None]
            change = np.ones(n, dtype=bool)
            if n:
                change[1:] = np.any(sp[1:] != sp[:-1], axis=1)
            gid = np.cumsum(change) - 1
        else:
            gid = np.zeros(n, dtype=np.int64)
        return idx, gid, (ok, asc)

    def _apply(self, wf, table) -> ColumnData:
        n = table.nrows
        idx, gid, _ = self._order_index(table)
        if wf.kind in ("lag", "lead"):
            src = wf.child.eval(table)
            sv = src.values[idx]
            svalid = src.valid()[idx]
            k = wf.offset if wf.kind == "lag" else -wf.offset
            pos = np.arange(n) - k  # sorted position to read from
            ok = (pos >= 0) & (pos < n)
            posc = np.clip(pos, 0, max(n - 1, 0))
            ok &= gid[posc] == gid
            out = np.empty_like(sv) if n else sv.copy()
            if n:
                out[:] = sv[posc]
            valid = ok & svalid[posc] if n else ok
            if wf.default is not None:
                out[~ok] = wf.default
                valid = valid | ~ok
            res_v = np.empty_like(out)
            res_m = np.empty(n, dtype=bool)
            res_v[idx] = out
            res_m[idx] = valid
            return ColumnData(res_v, None if res_m.all() else res_m, src.dtype)
        if wf.kind in ("row_number", "rank"):
            start = np.zeros(n, dtype=np.int64)
            if n:
                first = np.r_[True, gid[1:] != gid[:-1]]
                starts = np.maximum.accumulate(np.where(first, np.arange(n), 0))
                start = np.arange(n) - starts + 1
            res = np.empty(n, dtype=np.int32)
            res[idx] = start
            from .types import IntegerType

            return ColumnData(res, None, IntegerType())
        raise ValueError(wf.kind)


class Window:
    unboundedPreceding = -(1 << 62)
    unboundedFollowing = 1 << 62
    currentRow = 0

    @staticmethod
    def partitionBy(*cols):
        return WindowSpec().partitionBy(*cols)

    @staticmethod
    def orderBy(*cols):
        return WindowSpec().orderBy(*cols)
