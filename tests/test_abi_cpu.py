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


def _kernel_notes(tmp_path):
    """The gfx950 code object's AMDHSA metadata, as llvm-readelf prints it."""
    bin_dir = "/opt/rocm/lib/llvm/bin"
    if not os.path.exists(os.path.join(bin_dir, "llvm-readelf")):
        pytest.skip("ROCm LLVM tools not present")
    so = tmp_path / "lib.so"
    so.write_bytes(open(_ensure_built(), "rb").read())
    subprocess.check_call([os.path.join(bin_dir, "llvm-objdump"), "--offloading", str(so)],
                          stdout=subprocess.DEVNULL, cwd=tmp_path)
    cos = sorted(p for p in tmp_path.iterdir() if p.name.endswith("gfx950"))
    assert cos, "no gfx950 code object in the library"
    return "".join(subprocess.check_output([os.path.join(bin_dir, "llvm-readelf"), "--notes", str(p)], text=True)
                   for p in cos)


def test_no_kernel_uses_scratch(tmp_path):
    """Every kernel runs without private (scratch) memory: a dispatch that needs scratch waits for the
    runtime's scratch grant before its waves start, and the persistent loop's ranks must start together."""
    notes = _kernel_notes(tmp_path)
    kernels = re.findall(r"\.name:\s+(_Z\S+)", notes)
    sizes = [int(x) for x in re.findall(r"\.private_segment_fixed_size:\s+(\d+)", notes)]
    assert kernels and len(kernels) == len(sizes)
    assert any("k_sched_loop" in k for k in kernels)
    used = {k: s for k, s in zip(kernels, sizes) if s}
    assert not used, used


def test_pod_resources_decode_matches_reference_vectors():
    """The library's host decode of a pod's requests (ksg_debug_pod_resources: CalculateResource with the
    in-place resize status resources, and Fit's spec-only request) against the reference's own vectors
    (tests/golden/pod_resources.json, make_fixtures_i.py) -- no device needed; the device check of the
    same vectors (the mirror's Requested column) is test_golden_vectors_on_device."""
    import json

    from golden_runner import debug_pod_resources, pod_resources_mismatches
    lib = C.CDLL(_ensure_built())
    here = os.path.dirname(os.path.abspath(__file__))
    cases = json.load(open(os.path.join(here, "golden", "pod_resources.json")))["cases"]
    assert len(cases) >= 30
    bad = {}
    for c in cases:
        errs = pod_resources_mismatches(debug_pod_resources(lib, "ksg_", c["pod"]), c)
        if errs:
            bad[c["name"]] = errs
    assert not bad, bad


def test_log_table_matches_oracle_go_log_bit_for_bit():
    """The table PodTopologySpread scores read on the device (Cluster::log_tab) against the
    oracle's math.Log restatement, for every log(size + 2) a 100k-node cluster can need
    (podtopologyspread/scoring.go:287-299).  Both are independent copies of Go's math/log.go."""
    import struct

    from oracle_binding import load as load_oracle
    n = 100005
    lib = C.CDLL(_ensure_built())
    lib.ksg_debug_log_table.argtypes = [C.POINTER(C.c_double), C.c_int32]
    buf = (C.c_double * n)()
    assert lib.ksg_debug_log_table(buf, n) == n
    ora = load_oracle()
    bad = [k for k in range(2, n)
           if struct.pack("<d", buf[k]) != struct.pack("<d", ora.ksgo_go_log(float(k)))]
    assert not bad, f"{len(bad)} mismatches, first {bad[:5]}"
