"""The shipped library carries only packed instruction forms cleared on
gfx950 beside 16-bit matrix instructions (moseq2-detectron-extract_amd/
_isa_lint.py, tools/native/pk_hazard.hip, DESIGN.md section 3 "Item 6"), and
build() itself refuses a library holding any other form.  CPU-only: the
device code is extracted and disassembled; positive controls compile the
faulting form and check both the lint and build() catch it."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "moseq2-detectron-extract_amd")
sys.path.insert(0, PKG)
LIB = os.path.join(PKG, "libmdx.so")
HIPCC = "/opt/rocm/bin/hipcc"

needs_llvm = pytest.mark.skipif(not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"),
                                reason="ROCm LLVM tools absent")
needs_hipcc = pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc absent")

FAULTING = (
    "#include <hip/hip_runtime.h>\n"
    "typedef float f2 __attribute__((ext_vector_type(2)));\n"
    "extern \"C\" __global__ void k(f2 *p) {\n"
    "  f2 a = p[threadIdx.x], b = p[threadIdx.x + 64];\n"
    "  asm volatile(\"v_pk_add_f32 %0, %0, %1 op_sel:[0,1] op_sel_hi:[1,0]\" : \"+v\"(a) : \"v\"(b));\n"
    "  p[threadIdx.x] = a;\n"
    "}\n")


@needs_llvm
def test_library_has_only_cleared_packed_forms():
    import _isa_lint
    if not os.path.exists(LIB):
        pytest.skip("libmdx.so not built")
    hits = _isa_lint.scan(LIB)
    assert hits == [], hits[:5]


def test_form_parser():
    import _isa_lint
    f = _isa_lint.form
    assert f("v_pk_add_f32 v[28:29], v[28:29], v[32:33]") == ("v_pk_add_f32", "", "vv")
    assert f("v_pk_add_f32 v[34:35], v[30:31], 0 op_sel_hi:[1,0]") == ("v_pk_add_f32", "op_sel_hi:[1,0]", "vk")
    assert f("v_pk_fma_f32 v[2:3], v[14:15], s[14:15], v[2:3] op_sel_hi:[1,0,1]") == \
        ("v_pk_fma_f32", "op_sel_hi:[1,0,1]", "vsv")
    assert f("v_pk_min_u16 v17, v1, s70 op_sel_hi:[1,0]") == ("v_pk_min_u16", "op_sel_hi:[1,0]", "vs")
    bad = f("v_pk_add_f32 v[0:1], v[0:1], v[2:3] op_sel:[0,1] op_sel_hi:[1,0]")
    assert bad not in _isa_lint.CLEARED
    assert f("v_pk_mov_b32 v[0:1], v[2:3], v[4:5] op_sel:[1,0]") not in _isa_lint.CLEARED
    assert f("v_add_f32 v0, v1, v2") is None


@needs_llvm
@needs_hipcc
def test_lint_finds_the_form(tmp_path):
    import _isa_lint
    src = tmp_path / "k.hip"
    src.write_text(FAULTING)
    obj = tmp_path / "k.o"
    subprocess.run([HIPCC, "-O2", "--offload-arch=gfx950", "-fPIC", "-c", str(src), "-o", str(obj)], check=True,
                   capture_output=True)
    hits = _isa_lint.scan(str(obj))
    assert len(hits) == 1 and "op_sel:[0,1]" in hits[0][1], hits


@needs_llvm
@needs_hipcc
def test_build_refuses_the_form(tmp_path):
    """build() links, lints, deletes and raises: the faulting form never
    leaves the build."""
    import _build
    csrc = tmp_path / "csrc"
    csrc.mkdir()
    (csrc / "k.hip").write_text(FAULTING)
    lib = tmp_path / "libk.so"
    with pytest.raises(RuntimeError, match="outside the forms"):
        _build.build(csrc=str(csrc), obj=str(tmp_path / "obj"), lib=str(lib))
    assert not lib.exists()


def test_library_depends_only_on_runtimes():
    """libmdx.so's DT_NEEDED: the HIP runtime and the C/C++ runtime only --
    no hipBLASLt / rocBLAS / MIOpen (round 5 routed fp32 GEMMs to hipBLASLt
    from inside the library and faulted: PyTorch's bundled ROCm 7.0 copy
    resolved against 7.2 headers; the route was removed
    and this keeps it out)."""
    import shutil
    import _build
    if not os.path.exists(LIB) or not shutil.which("readelf"):
        pytest.skip("libmdx.so not built or readelf absent")
    deps = _build.needed(LIB)
    assert any(d.startswith("libamdhip64.so") for d in deps), deps
    assert all(d.startswith(_build.ALLOWED_NEEDED) for d in deps), deps
    for bad in ("blas", "miopen", "rccl", "torch"):
        assert not any(bad in d.lower() for d in deps), deps


def test_build_links_only_the_sources_objects(tmp_path):
    """build() links exactly one object per csrc/*.hip: an experiment's
    object left in the object directory (round 5's blas.o) is never linked."""
    import _build
    csrc = tmp_path / "csrc"
    obj = tmp_path / "obj"
    csrc.mkdir()
    obj.mkdir()
    for n in ("a", "b"):
        (csrc / f"{n}.hip").write_text("")
    (obj / "blas.o").write_text("")
    assert _build.objects(str(csrc), str(obj)) == [str(obj / "a.o"), str(obj / "b.o")]
    real = _build.objects()
    assert sorted(os.path.basename(o) for o in real) == \
        sorted(os.path.basename(s)[:-4] + ".o" for s in _build.sources())
    assert not any("blas" in os.path.basename(o) for o in real)


@needs_hipcc
def test_build_refuses_a_vendor_blas_dependency(tmp_path):
    """check_needed() deletes a library linked against a GEMM library."""
    import _build
    if not os.path.exists("/opt/rocm/lib/librocblas.so"):
        pytest.skip("rocBLAS absent")
    src = tmp_path / "k.cpp"
    src.write_text("extern \"C\" int rocblas_create_handle(void **);\nint f(void **h) { return rocblas_create_handle(h); }\n")
    lib = tmp_path / "libk.so"
    subprocess.run(["g++", "-shared", "-fPIC", str(src), "-o", str(lib), "-L/opt/rocm/lib", "-lrocblas",
                    "-Wl,--no-as-needed"], check=True, capture_output=True)
    with pytest.raises(RuntimeError, match="depends on"):
        _build.check_needed(str(lib))
    assert not lib.exists()
