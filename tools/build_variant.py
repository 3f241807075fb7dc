"""Build libmdx_<name>.so: the in-tree objects, with the listed sources
recompiled under changed per-file device flags (A/B builds, loaded with
MDX_LIB_VARIANT=<name>).  Usage:
  python tools/build_variant.py pk conv.hip inpaint.hip   # those files WITH packed-FP32 ops
  python tools/build_variant.py f32 frameops.hip -DMDX_PREP_FPB=32   # with extra defines"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "moseq2-detectron-extract_amd"))
import _build  # noqa: E402


def main():
    name = sys.argv[1]
    files = [a for a in sys.argv[2:] if not a.startswith("-D")]
    defines = [a for a in sys.argv[2:] if a.startswith("-D")]
    _build.build()
    cc = _build.hipcc()
    objs = []
    for src in _build.sources():
        base = os.path.basename(src)
        o = os.path.join(_build.OBJ, base[:-4] + ".o")
        if base in files:
            o = os.path.join(_build.OBJ, f"{base[:-4]}_{name}.o")
            cmd = [cc, *_build._cmd_flags(base), *defines, "-c", src, "-o", o]
            subprocess.check_call(cmd)
        objs.append(o)
    out = os.path.join(_build.HERE, f"libmdx_{name}.so")
    subprocess.check_call([cc, "-shared", "-fPIC", f"--offload-arch={_build.ARCH}", *objs, "-o", out])
    print(out)


if __name__ == "__main__":
    main()
