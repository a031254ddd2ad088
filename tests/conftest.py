import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# In-process node-sharded groups (tests/test_gpu_sharded.py) take the device exchange only when every rank's
# stream has a hardware queue of its own plus one spare; HIP's default is 4 queues, which
# holds a W = 2 group.  The test process asks HIP for 8 (read at HIP's initialisation, before any test runs),
# so W = 3 groups run the loops too.  One-process-per-GPU deployments (RCCL ranks) do not depend on it.
os.environ["GPU_MAX_HW_QUEUES"] = "8"
sys.path.insert(0, os.path.join(ROOT, "kubernetes-kubernetes_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through libksg.so)")
    config.addinivalue_line("markers", "slow: long-running parity sweep")
