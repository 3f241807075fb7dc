"""Register / LDS / scratch usage of the gfx950 kernels in libmdx.so (or a
.o): the AMDGPU code-object metadata of every embedded code object, filtered
by a kernel-name substring.

    python tools/kernel_resources.py k_wino_f4 [path]
"""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "moseq2-detectron-extract_amd"))
import _isa_lint as L  # noqa: E402

KEYS = (".vgpr_count", ".agpr_count", ".sgpr_count", ".private_segment_fixed_size", ".group_segment_fixed_size",
        ".vgpr_spill_count", ".sgpr_spill_count")


def resources(path, pattern):
    out = []
    with tempfile.TemporaryDirectory() as td:
        fat = os.path.join(td, "fatbin")
        subprocess.run([os.path.join(L.LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", path,
                        os.path.join(td, "stripped")], check=True, capture_output=True)
        data = open(fat, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(L.MAGIC), data)]
        for k, a in enumerate(starts):
            b = starts[k + 1] if k + 1 < len(starts) else len(data)
            part, co = os.path.join(td, f"b{k}"), os.path.join(td, f"b{k}.co")
            with open(part, "wb") as fh:
                fh.write(data[a:b])
            subprocess.run([os.path.join(L.LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                            f"--input={part}", f"--targets={L.TARGET}", f"--output={co}"], check=True,
                           capture_output=True)
            notes = subprocess.run([os.path.join(L.LLVM, "llvm-readelf"), "--notes", co], check=True,
                                   capture_output=True, text=True).stdout
            for blk in notes.split("  - .agpr_count")[1:]:
                blk = ".agpr_count" + blk
                m = re.search(r"\.name:\s+(\S+)", blk)
                if not m or pattern not in m.group(1):
                    continue
                vals = {}
                for key in KEYS:
                    mm = re.search(re.escape(key) + r":\s+(\d+)", blk)
                    if mm:
                        vals[key.strip(".")] = int(mm.group(1))
                out.append((m.group(1), vals))
    return out


if __name__ == "__main__":
    pat = sys.argv[1] if len(sys.argv) > 1 else ""
    path = sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(L.__file__), "libmdx.so")
    for name, vals in resources(path, pat):
        print(name, vals)
