"""VGPR / SGPR / LDS / spill counts of the kernels of a HIP shared library (no GPU).

    python tools/kernel_regs.py LIB.so [NAME_SUBSTRING]
"""
from __future__ import annotations

import pathlib
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parent))
import isa_dump  # noqa: E402

FIELDS = (".vgpr_count", ".sgpr_count", ".group_segment_fixed_size", ".vgpr_spill_count")


def main() -> None:
    lib = pathlib.Path(sys.argv[1])
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    with tempfile.TemporaryDirectory() as td:
        for co in isa_dump.code_objects(lib, pathlib.Path(td)):
            out = subprocess.run([str(isa_dump.LLVM / "llvm-readelf"), "--notes", str(co)],
                                 capture_output=True, text=True).stdout
            # one kernel's metadata map per "- .agpr_count" entry
            for ent in out.split("- .agpr_count")[1:]:
                m = re.search(r"\.name:\s+(\S+)", ent)
                if not m or pat not in m.group(1):
                    continue
                vals = {f: (re.search(re.escape(f) + r":\s+(\d+)", ent) or [None, "?"])[1] for f in FIELDS}
                print(m.group(1)[:60], " ".join(f"{k[1:]}={v}" for k, v in vals.items()))


if __name__ == "__main__":
    main()
