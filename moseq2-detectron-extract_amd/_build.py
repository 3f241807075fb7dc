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
# inpaint.hip (its serial tap sums would pack with SGPR operands) is also
# compiled without them.  conv.hip keeps the packed forms: every packed
# instruction it compiles to is one of the forms tools/native/pk_hazard.hip cleared
# beside 16-bit MFMAs, which build() checks on every library it links
# (_isa_lint.py, a whitelist; the build fails on anything else).  The
# target-feature switch reaches the host compile too, where clang ignores it
# with a warning.
NO_PACKED_FP32 = ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]
DEVICE_FLAGS = {"model_ops.hip": NO_PACKED_FP32, "inpaint.hip": NO_PACKED_FP32}


def sources(csrc: str = CSRC):
    return sorted(glob.glob(os.path.join(csrc, "*.hip")))


def objects(csrc: str = CSRC, obj: str = OBJ):
    """The objects the library is linked from: exactly one per csrc/*.hip
    source.  Anything else left in the object directory (an experiment's
    object) is never linked."""
    return [os.path.join(obj, os.path.basename(s)[:-4] + ".o") for s in sources(csrc)]


# libraries libmdx.so may depend on: the HIP runtime and the C/C++ runtime.
# No vendor GEMM library (hipBLASLt / rocBLAS: the in-process copy is
# PyTorch's ROCm 7.0 build, DESIGN.md section 3 "fp32 GEMM against the
# library"), no MIOpen: every kernel of the hot path is this library's own.
ALLOWED_NEEDED = ("libamdhip64.so", "libstdc++.so", "libm.so", "libgcc_s.so", "libc.so", "ld-linux-x86-64.so")


def needed(lib: str = LIB):
    """DT_NEEDED entries of `lib`."""
    r = subprocess.run(["readelf", "-d", lib], capture_output=True, text=True, check=True)
    return [ln.split("[", 1)[1].rstrip("]").strip() for ln in r.stdout.splitlines() if "(NEEDED)" in ln]


def _deps_newer(target: str, srcs, csrc: str = CSRC) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    hdrs = glob.glob(os.path.join(csrc, "*.h")) + glob.glob(os.path.join(os.path.dirname(HERE), "include", "*.h"))
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


def build(force: bool = False, verbose: bool = False, jobs: int = 8, csrc: str = CSRC, obj: str = OBJ,
          lib: str = LIB) -> str:
    """Compile every csrc/*.hip for gfx950, link `lib`, then refuse it (delete
    and raise) if it has undefined symbols of its own or any packed
    instruction outside the whitelist of cleared forms (_isa_lint)."""
    os.makedirs(obj, exist_ok=True)
    cc = hipcc()
    srcs = sources(csrc)
    objs = objects(csrc, obj)
    todo = []
    for s, o in zip(srcs, objs):
        if force or _deps_newer(o, [s], csrc) or _flags_changed(o, _cmd_flags(os.path.basename(s))):
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
    if force or todo or _deps_newer(lib, objs, csrc):
        cmd = [cc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", lib]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link of {os.path.basename(lib)} failed:\n{r.stderr[-6000:]}")
        check_symbols(lib)
        check_needed(lib)
        check_isa(lib)
    return lib


def check_needed(lib: str = LIB) -> None:
    """Refuse (delete) a library that depends on anything but the HIP and
    C/C++ runtimes."""
    if not shutil.which("readelf"):
        return
    bad = [n for n in needed(lib) if not n.startswith(ALLOWED_NEEDED)]
    if bad:
        os.remove(lib)
        raise RuntimeError(f"{os.path.basename(lib)} depends on {bad}: only {ALLOWED_NEEDED} are allowed")


def check_symbols(lib: str = LIB) -> None:
    """A shared link does not reject undefined symbols; a kernel whose host
    stub was not emitted only fails at dlopen on the GPU box.  Refuse the
    library here instead."""
    nm = shutil.which("nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    r = subprocess.run([nm, "-u", "-C", lib], capture_output=True, text=True)
    if r.returncode != 0:
        return
    bad = [ln.strip() for ln in r.stdout.splitlines() if "mdx::" in ln]
    if bad:
        os.remove(lib)
        raise RuntimeError(f"{os.path.basename(lib)} has undefined symbols of its own:\n" + "\n".join(bad[:20]))


def check_isa(lib: str = LIB) -> None:
    """The packed-instruction whitelist (_isa_lint.py) on the linked
    library's device code: a form pk_hazard.hip has not cleared beside 16-bit
    MFMAs deletes the library and fails the build, so it never reaches the
    GPU box."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("_mdx_isa_lint", os.path.join(HERE, "_isa_lint.py"))
    lint = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(lint)
    if not lint.available():
        raise RuntimeError("ROCm LLVM tools (llvm-objcopy, clang-offload-bundler, llvm-objdump) absent: "
                           "cannot check the library's packed instruction forms")
    hits = lint.scan(lib)
    if hits:
        os.remove(lib)
        raise RuntimeError(f"{os.path.basename(lib)}: {len(hits)} packed instruction(s) outside the forms "
                           "cleared by tools/native/pk_hazard.hip (_isa_lint.CLEARED), e.g.\n" +
                           "\n".join(f"  {s}: {i}" for s, i in hits[:10]))


if __name__ == "__main__":
    import sys
    print(build(force="-f" in sys.argv, verbose=True))
