"""Scan the device code of a HIP shared library or object for packed VALU
instruction forms that are not known to be safe on gfx950 (run by
_build.build() on every freshly linked libmdx.so, and by tools/isa_lint.py).

The hazard ("Item 6"): ``v_pk_add_f32 vD, vA, vB op_sel:[0,1]
op_sel_hi:[1,0]`` -- the low result taking the high half of a source --
returns wrong low halves while other waves on the CU issue bf16 / f16 MFMAs
(tools/native/pk_hazard.hip: 200 / 200 reps beside a bf16 MFMA loop, 187-191 /
200 beside f16, never alone or beside f32 MFMAs).  Its cause is not known, so
this is a whitelist: every packed instruction must have one of the
(mnemonic, modifiers, operand kinds) forms pk_hazard.hip ran beside 16-bit
MFMAs without a single differing bit (profiles/r04_pkh_AC_*.log,
profiles/r05_pkh_bg*.json: forms 0, 2-4, 6-13; r05_pkh14_*.json: form 14); anything else -- any op_sel
form, v_pk_mov_b32, a new modifier combination the compiler starts to emit
-- fails the build until the harness has cleared it."""
from __future__ import annotations

import os
import re
import subprocess
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"

# (mnemonic, modifiers, source operand kinds: v = VGPR, s = SGPR, k = constant)
CLEARED = {
    ("v_pk_add_f32", "", "vv"),                                          # form 0
    ("v_pk_add_f32", "op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]", "vv"),  # form 2
    ("v_pk_mul_f32", "", "vv"),                                          # form 3
    ("v_pk_fma_f32", "", "vvv"),                                         # form 4
    ("v_pk_add_f32", "neg_lo:[0,1] neg_hi:[0,1]", "vv"),                 # form 6
    ("v_pk_add_f32", "op_sel_hi:[1,0]", "vk"),                           # form 7
    ("v_pk_fma_f32", "op_sel_hi:[1,0,1]", "vkv"),                        # form 8
    ("v_pk_fma_f32", "op_sel_hi:[1,0,1]", "vsv"),                        # form 9
    ("v_pk_mul_f32", "", "vs"),                                          # form 10
    ("v_pk_mul_f32", "op_sel_hi:[1,0]", "vk"),                           # form 11
    ("v_pk_mul_f32", "op_sel_hi:[1,0]", "vs"),                           # form 12
    ("v_pk_min_u16", "", "vv"),                                          # form 13
    ("v_pk_max_u16", "", "vv"),                                          # form 13
    ("v_pk_min_u16", "op_sel_hi:[1,0]", "vs"),                           # form 13
    # form 14: 0 of 200 reps differ beside bf16 / f16 MFMA loops, with the
    # form-1 positive control differing in 200 / 193 of the same runs
    # (profiles/r05_pkh14_all_bg1.json, r05_pkh14_all_bg2.json)
    ("v_pk_minimum3_f16", "", "vvv"),
}

_INS = re.compile(r"^\s*(v_pk_\w+)\s+(\S+?),\s*(.*)$")
_MOD = re.compile(r"\b(op_sel(?:_hi)?|neg_lo|neg_hi):\[[01,]+\]")


def _kind(op: str) -> str:
    op = op.strip().lstrip("-|").rstrip("|")
    if re.match(r"^v(\d+|\[)", op):
        return "v"
    if re.match(r"^(s(\d+|\[)|vcc|exec|m0|ttmp)", op):
        return "s"
    return "k"


def form(line: str):
    """(mnemonic, modifiers, operand kinds) of a packed instruction line, or
    None for any other line."""
    m = _INS.match(line.split("//")[0])
    if not m:
        return None
    rest = m.group(3)
    mods = " ".join(x.group(0) for x in _MOD.finditer(rest))
    srcs = [x for x in _MOD.sub("", rest).split(",") if x.strip()]
    return m.group(1), mods, "".join(_kind(x) for x in srcs)


def device_disassembly(path: str) -> str:
    """Disassembly of every gfx950 code object embedded in a .so / .o (a
    shared library's .hip_fatbin holds one offload bundle per source file)."""
    outs = []
    with tempfile.TemporaryDirectory() as td:
        fat = os.path.join(td, "fatbin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", path,
                        os.path.join(td, "stripped")], check=True, capture_output=True)
        data = open(fat, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        for k, a in enumerate(starts):
            b = starts[k + 1] if k + 1 < len(starts) else len(data)
            part, co = os.path.join(td, f"b{k}"), os.path.join(td, f"b{k}.co")
            with open(part, "wb") as fh:
                fh.write(data[a:b])
            subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={part}",
                            f"--targets={TARGET}", f"--output={co}"], check=True, capture_output=True)
            out = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", co], check=True,
                                 capture_output=True, text=True)
            outs.append(out.stdout)
    return "\n".join(outs)


def available() -> bool:
    return all(os.path.exists(os.path.join(LLVM, t)) for t in ("llvm-objcopy", "clang-offload-bundler",
                                                                "llvm-objdump"))


def scan(path: str):
    """[(kernel symbol, instruction)] for every packed instruction whose form
    is not in CLEARED."""
    hits, sym = [], None
    for line in device_disassembly(path).splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            sym = m.group(1)
            continue
        f = form(line)
        if f is not None and f not in CLEARED:
            hits.append((sym, line.split("//")[0].strip()))
    return hits
