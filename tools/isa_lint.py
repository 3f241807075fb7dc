"""CLI of the packed-instruction whitelist lint (the check itself lives in the
package, moseq2-detectron-extract_amd/_isa_lint.py, so build() runs it on
every library it links).

Usage: python tools/isa_lint.py FILE [FILE ...]   (exit 1 on any hit)"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "moseq2-detectron-extract_amd"))
from _isa_lint import device_disassembly, form, scan  # noqa: E402,F401


def main():
    bad = 0
    for path in sys.argv[1:]:
        hits = scan(path)
        bad += len(hits)
        print(f"{path}: {len(hits)} packed instructions outside the cleared forms")
        for sym, ins in hits[:10]:
            print(f"   {sym}: {ins}")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
