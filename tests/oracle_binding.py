"""Test-side binding of the parity oracle (oracle/build/liboracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this.
"""
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-kubernetes_amd"))
from ksg.abi import Backend  # noqa: E402

LIB = os.path.join(ROOT, "oracle", "build", "liboracle.so")
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        _lib = C.CDLL(LIB)
        _lib.ksgo_go_log.restype = C.c_double
        _lib.ksgo_go_log.argtypes = [C.c_double]
        _lib.ksgo_heap_root.restype = C.c_int32
        _lib.ksgo_heap_root.argtypes = [C.POINTER(C.c_int64), C.c_int32]
    return _lib


def oracle(config=None):
    return Backend(load(), "ksgo_", config)
