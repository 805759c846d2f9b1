"""Per-kernel register / scratch metadata of a built object (gfx950 code object notes).
    python tools/kres.py build/variants/NAME/k.o [substring]"""
import os
import re
import subprocess
import sys
import tempfile

B = "/opt/rocm/lib/llvm/bin"
obj, pat = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
with tempfile.TemporaryDirectory() as d:
    fb, co = os.path.join(d, "fb"), os.path.join(d, "co")
    subprocess.check_call([B + "/llvm-objcopy", "--dump-section=.hip_fatbin=" + fb, obj])
    subprocess.check_call([B + "/clang-offload-bundler", "--unbundle", "--type=o", "--input=" + fb,
                           "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co])
    notes = subprocess.check_output([B + "/llvm-readelf", "--notes", co], text=True)
for blk in notes.split("  - .agpr_count")[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk).group(1)
    if pat not in name:
        continue
    g = lambda k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, "-"])[1]
    print("%-60s scratch %4s vgpr %3s vspill %4s sgpr %3s sspill %4s" % (
        name[:60], g("private_segment_fixed_size"), g("vgpr_count"), g("vgpr_spill_count"),
        g("sgpr_count"), g("sgpr_spill_count")))
