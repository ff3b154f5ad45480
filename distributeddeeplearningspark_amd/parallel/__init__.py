"""Distributed runtime: process groups (RCCL / gloo), bucketed overlapped all-reduce,
the Spark-style worker launcher and the parameter-server facade."""
from .comm import ProcessGroup, init_from_env, init_process_group  # noqa: F401
