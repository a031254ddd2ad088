"""CPU-side checks of the product boundary: libksg.so builds, loads, exports every entry point
include/ksg.h declares, and refuses to run without a HIP device (no CPU fallback)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from ksg import native
from ksg.abi import KsgError

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ensure_built():
    if not os.path.exists(native.LIB):
        subprocess.check_call(["make", "-s", "-j8", "-C", native.PKG])
    return native.LIB


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "ksg.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ksg_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for want in ["ksg_create", "ksg_schedule_one", "ksg_schedule_batch", "ksg_run_filter_plugin",
                 "ksg_run_score_plugin", "ksg_forget", "ksg_add_pod", "ksg_add_node"]:
        assert want in syms


def test_library_exports_every_declared_symbol():
    lib = C.CDLL(_ensure_built())
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_library_is_built_for_gfx950():
    blob = open(_ensure_built(), "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_create_fails_loudly_without_a_device():
    _ensure_built()
    if os.path.exists("/dev/kfd"):
        pytest.skip("a GPU is visible: covered by the gpu tests")
    with pytest.raises(KsgError, match="no HIP device"):
        native.Scheduler({})


def test_config_errors_are_reported_before_device_probe():
    _ensure_built()
    with pytest.raises(KsgError):
        native.Scheduler({"nodeResourcesFit": {"scoringStrategy": {"type": "Bogus"}}})
