"""Diagnostic: runs the pipeline-fallback test clusters with loopStamps on (prints each drain)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "kubernetes-kubernetes_amd"), os.path.join(ROOT, "tests")]
import test_gpu_parity as t  # noqa: E402
from ksg.native import Scheduler  # noqa: E402


def native(cfg):
    return Scheduler(dict(cfg, loopStamps=True))


t.test_pipeline_relayout_mid_batch(native)
t.test_pipeline_staging_outgrown_mid_batch(native)
print("pipeline fallback streams match the oracle")
