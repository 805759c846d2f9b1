"""Source revision of the native library: a hash of the sources it is built from.

`make` compiles this hash into libsspp_hip.so (`sspp_build_id()`, build/obj/stamp.o), and
tools/build_variant.sh links the same stamp into profiling variants.  `_lib.lib()` compares
a loaded library's stamp with the hash of the tree it runs from, so a library built from other
sources (a stale profiling variant, a product library not rebuilt after an edit) is caught at
load time instead of failing later on a missing symbol or giving another revision's numbers.

    python3 sspp_amd/_stamp.py          # print the hash (Makefile)
"""
import hashlib
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_HERE)
_SUFFIXES = (".h", ".hip", ".cpp")


def source_files(root=_ROOT):
    """The product library's sources: sspp_amd/csrc/* and include/sspp_hip.h, sorted."""
    csrc = os.path.join(root, "sspp_amd", "csrc")
    if not os.path.isdir(csrc):
        return []
    files = [os.path.join(csrc, f) for f in sorted(os.listdir(csrc)) if f.endswith(_SUFFIXES)]
    hdr = os.path.join(root, "include", "sspp_hip.h")
    if os.path.exists(hdr):
        files.append(hdr)
    return files


def source_hash(root=_ROOT):
    """16 hex digits of sha256 over (relative path, contents) of every source file; None when
    the sources are not present."""
    files = source_files(root)
    if not files:
        return None
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.relpath(f, root).replace(os.sep, "/").encode())
        h.update(b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(source_hash())
