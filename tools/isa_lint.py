"""Scan the device code of a HIP shared library or object for the packed-FP32
instruction form that faults on gfx950 beside 16-bit matrix instructions.

tools/native/pk_hazard.hip (profiles/r04_experiments.json, call AC): of the
packed-FP32 forms, only ``v_pk_add_f32 ... op_sel:[0,1] op_sel_hi:[1,0]`` --
the low result taking the high half of a source -- gave wrong low-half
results, in 200 / 200 reps beside a register-only v_mfma_f32_16x16x32_bf16
loop on other waves (187 / 200 beside the f16 form), never alone or beside
the f32 MFMA; the plain, broadcast (op_sel_hi only), multiply and FMA forms
never did.  The compiler forms it from two-lane vector code; this check
flags every v_pk_*_f32 with a set op_sel bit (a low lane reading a high
half), which covers that form and its siblings.

Usage: python tools/isa_lint.py FILE [FILE ...]   (exit 1 on any hit)"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
BAD = re.compile(r"\bv_pk_(add|mul|fma)_f32\b[^/\n]*\bop_sel:\[([01],)*1")


MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


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


def scan(path: str):
    """[(kernel symbol, instruction)] for every flagged instruction."""
    hits, sym = [], None
    for line in device_disassembly(path).splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            sym = m.group(1)
        elif BAD.search(line):
            hits.append((sym, line.split("//")[0].strip()))
    return hits


def main():
    bad = 0
    for path in sys.argv[1:]:
        hits = scan(path)
        bad += len(hits)
        print(f"{path}: {len(hits)} flagged packed-FP32 op_sel instructions")
        for sym, ins in hits[:10]:
            print(f"   {sym}: {ins}")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
