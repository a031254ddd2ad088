"""Per-kernel resources of libksg.so's gfx950 code object (SGPRs, VGPRs, AGPRs, spills, scratch, LDS), from the
AMDHSA metadata llvm-readelf prints.   python scripts/kernel_resources.py [lib] [name-filter]"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

lib = os.path.abspath(sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..",
                                                                         "kubernetes-kubernetes_amd/lib/libksg.so"))
flt = sys.argv[2] if len(sys.argv) > 2 else ""
bd = "/opt/rocm/lib/llvm/bin"
with tempfile.TemporaryDirectory() as d:
    shutil.copy(lib, os.path.join(d, "lib.so"))  # the bundles are extracted beside the file
    subprocess.check_call([f"{bd}/llvm-objdump", "--offloading", os.path.join(d, "lib.so")], cwd=d, stdout=subprocess.DEVNULL)
    notes = "".join(subprocess.check_output([f"{bd}/llvm-readelf", "--notes", os.path.join(d, p)], text=True)
                    for p in sorted(os.listdir(d)) if p.endswith("gfx950"))
for blk in notes.split("  - .agpr_count")[1:]:
    g = lambda k: (re.search(rf"\.{k}:\s+(\S+)", blk) or [None, "?"])[1]  # noqa: E731
    name = subprocess.run(["c++filt"], input=g("name"), capture_output=True, text=True).stdout.strip()
    if flt in name:
        print(f"{name[:70]:70s} sgpr {g('sgpr_count'):>3} vgpr {g('vgpr_count'):>3} "
              f"agpr {blk.split()[1]:>3} spill s{g('sgpr_spill_count')}/v{g('vgpr_spill_count')} "
              f"scratch {g('private_segment_fixed_size')} lds {g('group_segment_fixed_size')}")
