import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# (In-process node-sharded groups, tests/test_gpu_sharded.py, run every rank's persistent loop in one dispatch,
# DESIGN.md §6, so they need no hardware queue per rank: the tests run at HIP's default GPU_MAX_HW_QUEUES.)
sys.path.insert(0, os.path.join(ROOT, "kubernetes-kubernetes_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through libksg.so)")
    config.addinivalue_line("markers", "slow: long-running parity sweep")
