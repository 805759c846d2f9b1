"""Disassemble one kernel / device function of a built object (gfx950), and count scratch
accesses and calls in it: python tools/kdis.py OBJ SYMBOL_SUBSTRING [--print]"""
import os
import re
import subprocess
import sys
import tempfile

B = "/opt/rocm/lib/llvm/bin"
obj, pat = sys.argv[1], sys.argv[2]
with tempfile.TemporaryDirectory() as d:
    fb, co = os.path.join(d, "fb"), os.path.join(d, "co")
    subprocess.check_call([B + "/llvm-objcopy", "--dump-section=.hip_fatbin=" + fb, obj])
    subprocess.check_call([B + "/clang-offload-bundler", "--unbundle", "--type=o", "--input=" + fb,
                           "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co])
    dis = subprocess.check_output([B + "/llvm-objdump", "-d", "--no-show-raw-insn", co], text=True)
funcs = re.split(r"\n(?=[0-9a-f]+ <)", dis)
for f in funcs:
    m = re.match(r"[0-9a-f]+ <([^>]+)>:", f)
    if not m or pat not in m.group(1):
        continue
    lines = [l for l in f.split("\n")[1:] if l.strip()]
    scr = sum(1 for l in lines if "scratch_" in l or ("buffer_" in l and "off," in l and "s[0:3]" in l))
    print("%s: %d instr, scratch ops %d, s_swappc/call %d, v_writelane %d, v_readlane %d, v_accvgpr %d" % (
        m.group(1)[:70], len(lines), scr, sum("s_swappc" in l or "s_setpc" in l for l in lines),
        sum("v_writelane" in l for l in lines), sum("v_readlane" in l for l in lines),
        sum("v_accvgpr" in l for l in lines)))
    if "--print" in sys.argv:
        print("\n".join(lines))
