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
