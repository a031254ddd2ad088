"""ksg: MI355X-native kube-scheduler node evaluation (host-side Python mirror).

The compute path is libksg.so (HIP kernels for gfx950 behind the C ABI in
include/ksg.h); this package only binds it and mirrors the reference's
scheduler/framework interface for tests and benchmarks.
"""
from . import abi, objects  # noqa: F401
from .abi import KsgError  # noqa: F401
