"""Build the in-tree HIP library ``libmdx.so`` for gfx950.

``python -m`` is not needed: ``__graft_entry__.build()`` and the package loader
call :func:`build`.  Objects go to ``csrc/build/``; the shared library lands
next to this file so it travels with the repository snapshot to the GPU box
(git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(CSRC, "build")
LIB = os.path.join(HERE, "libmdx.so")
ARCH = "gfx950"


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: cannot build the mdx HIP library")


def _flags():
    return ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-Wall", "-Wno-unused-result",
            "-munsafe-fp-atomics", f"-I{os.path.dirname(HERE)}"]


# per-file host-code flags: the dense linear algebra of the Kalman recursions
# vectorises with AVX2 / FMA (every x86-64 host of an MI355X has them)
HOST_FLAGS = {"host_tracking.hip": ["-Xarch_host", "-mavx2", "-Xarch_host", "-mfma"]}

# model_ops.hip (GroupNorm, RPN, ROIAlign, box / mask / keypoint post-processing)
# is compiled without the packed FP32 VALU instructions.  Round 4 found why
# ("Item 6"): the form v_pk_add_f32 vD, vA, vB
# op_sel:[0,1] op_sel_hi:[1,0] (low result = A.lo + B.hi), which the compiler
# forms from two-lane vector code in GroupNorm / ROIAlign / upsample, returns
# wrong low halves on gfx950 while other waves on the CU issue bf16 / f16
# MFMAs (tools/native/pk_hazard.hip: 200 / 200 reps beside a register-only
# bf16 MFMA loop, never alone or beside f32 MFMAs; the plain, broadcast,
# multiply and FMA packed forms never fault).  With the forms, the fp16
# pipelined loop differed from the serial step in 133 of 150 steps.
# conv.hip and inpaint.hip keep the packed forms: they contain no op_sel
# variant, which tools/isa_lint.py checks on the built library
# (tests/test_isa_lint.py).  The target-feature switch reaches the host
# compile too, where clang ignores it with a warning.
NO_PACKED_FP32 = ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]
DEVICE_FLAGS = {"model_ops.hip": NO_PACKED_FP32}


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def _deps_newer(target: str, srcs) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    hdrs = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(os.path.dirname(HERE), "include", "*.h"))
    return any(os.path.getmtime(s) > t for s in list(srcs) + hdrs)


def _cmd_flags(base: str) -> list:
    return [*_flags(), *HOST_FLAGS.get(base, []), *DEVICE_FLAGS.get(base, [])]


def _flags_changed(obj: str, flags: list) -> bool:
    """The object was built with other flags (or its record is missing)."""
    try:
        with open(obj + ".flags") as fh:
            return fh.read() != " ".join(flags)
    except OSError:
        return True


def build(force: bool = False, verbose: bool = False, jobs: int = 8) -> str:
    os.makedirs(OBJ, exist_ok=True)
    cc = hipcc()
    srcs = sources()
    objs = []
    todo = []
    for s in srcs:
        o = os.path.join(OBJ, os.path.basename(s)[:-4] + ".o")
        objs.append(o)
        if force or _deps_newer(o, [s]) or _flags_changed(o, _cmd_flags(os.path.basename(s))):
            todo.append((s, o))

    def comp(so):
        s, o = so
        flags = _cmd_flags(os.path.basename(s))
        cmd = [cc, *flags, "-c", s, "-o", o]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {os.path.basename(s)}:\n{r.stderr[-6000:]}")
        with open(o + ".flags", "w") as fh:  # the flags this object was built with
            fh.write(" ".join(flags))
        return o

    if todo:
        with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, len(todo)))) as ex:
            list(ex.map(comp, todo))
    if force or todo or _deps_newer(LIB, objs):
        cmd = [cc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", LIB]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link of libmdx.so failed:\n{r.stderr[-6000:]}")
        check_symbols()
    return LIB


def check_symbols() -> None:
    """A shared link does not reject undefined symbols; a kernel whose host
    stub was not emitted only fails at dlopen on the GPU box.  Refuse the
    library here instead."""
    nm = shutil.which("nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    r = subprocess.run([nm, "-u", "-C", LIB], capture_output=True, text=True)
    if r.returncode != 0:
        return
    bad = [ln.strip() for ln in r.stdout.splitlines() if "mdx::" in ln]
    if bad:
        os.remove(LIB)
        raise RuntimeError("libmdx.so has undefined symbols of its own:\n" + "\n".join(bad[:20]))


if __name__ == "__main__":
    import sys
    print(build(force="-f" in sys.argv, verbose=True))
