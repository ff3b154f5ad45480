"""Object-storage attach (reference ``attach_storage_container`` in
``ddl_mnist_aztk.py:88-97`` / ``ddl_nyiso_aztk.py``).

The reference sets ``fs.azure.account.key.<account>.blob.core.windows.net`` in the Hadoop
configuration and reads ``wasb[s]://<container>@<account>.blob.core.windows.net/<path>``.
This framework runs without network access, so an attached account is MOUNTED on a local
directory instead: ``<root>/<account>/<container>/<path>`` with ``root`` from the call or
``DDL_STORAGE_ROOT`` (default ``~/.ddl_storage``).  The account key is never stored or
logged — only the fact that a key was supplied is recorded in the session conf.
"""
from __future__ import annotations

import os
import re

_MOUNTS: dict[str, str] = {}
_URI = re.compile(r"^(wasbs?|abfss?)://(?P<container>[^@/]+)@(?P<account>[^./]+)\.[^/]+/?(?P<path>.*)$")


def attach_storage_container(spark, account: str, key: str | None = None, root: str | None = None):
    root = root or os.environ.get("DDL_STORAGE_ROOT", os.path.expanduser("~/.ddl_storage"))
    _MOUNTS[account] = os.path.join(root, account)
    conf_key = f"fs.azure.account.key.{account}.blob.core.windows.net"
    try:
        spark.conf.set(conf_key, "<set>" if key else "<none>")
    except Exception:
        pass
    return _MOUNTS[account]


def resolve(uri: str) -> str:
    """Map a storage URI of an attached account to its local path (other strings unchanged)."""
    m = _URI.match(uri)
    if not m:
        return uri
    acct = m.group("account")
    if acct not in _MOUNTS:
        raise IOError(f"storage account {acct!r} is not attached: call attach_storage_container(spark, {acct!r}, ...)")
    return os.path.join(_MOUNTS[acct], m.group("container"), m.group("path"))
