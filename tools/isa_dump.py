"""Disassemble every gfx950 code object of a HIP shared library, kernel by kernel (no GPU).

A HIP library built from several translation units carries one offload bundle per unit,
concatenated in its .hip_fatbin section; each is unbundled and disassembled on its own.

    python tools/isa_dump.py LIB.so            # kernel names and instruction counts
    python tools/isa_dump.py A.so B.so         # kernels whose instructions differ (exit 1 if any)
"""
from __future__ import annotations

import pathlib
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = pathlib.Path("/opt/rocm/lib/llvm/bin")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def available() -> bool:
    return shutil.which("objcopy") is not None and (LLVM / "llvm-objdump").exists()


def code_objects(lib: pathlib.Path, work: pathlib.Path) -> list[pathlib.Path]:
    """The gfx950 code objects of `lib`, one per offload bundle."""
    work.mkdir(parents=True, exist_ok=True)
    # objcopy with no output file rewrites its input: work on a copy (the library may be
    # mapped by the calling process)
    copy, fat = work / "lib.so", work / "fat.bin"
    shutil.copyfile(lib, copy)
    subprocess.run(["objcopy", f"--dump-section=.hip_fatbin={fat}", str(copy),
                    str(work / "discard.so")], check=True, capture_output=True)
    data = fat.read_bytes()
    offs = [m.start() for m in re.finditer(re.escape(MAGIC), data)] + [len(data)]
    out = []
    for i in range(len(offs) - 1):
        part, co = work / f"b{i}.bin", work / f"b{i}.co"
        part.write_bytes(data[offs[i]:offs[i + 1]])
        r = subprocess.run([str(LLVM / "clang-offload-bundler"), "--unbundle", "--type=o",
                            f"--input={part}", f"--targets={TARGET}", f"--output={co}"],
                           capture_output=True)
        if r.returncode == 0 and co.exists() and co.stat().st_size:
            out.append(co)
    return out


def kernels(lib, work=None) -> dict[str, list[str]]:
    """{symbol: [instruction text]} over every code object, addresses and encodings dropped."""
    lib = pathlib.Path(lib)
    tmp = None
    if work is None:
        tmp = tempfile.TemporaryDirectory()
        work = pathlib.Path(tmp.name)
    try:
        funcs: dict[str, list[str]] = {}
        for co in code_objects(lib, pathlib.Path(work)):
            txt = subprocess.run([str(LLVM / "llvm-objdump"), "-d", "--no-show-raw-insn", str(co)],
                                 check=True, capture_output=True, text=True).stdout
            cur = None
            for line in txt.splitlines():
                m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
                if m:
                    cur = m.group(1)
                    funcs[cur] = []
                    continue
                if cur is None:
                    continue
                s = re.sub(r"//.*$", "", line).strip()
                s = re.sub(r"^[0-9a-f]+:\s*", "", s)
                s = re.sub(r"<[^>]*>", "", s).strip()
                if s:
                    funcs[cur].append(s)
        return funcs
    finally:
        if tmp is not None:
            tmp.cleanup()


def descriptors(lib, work=None) -> dict[str, dict[str, str]]:
    """{kernel: {".amdhsa_*" directive: value}} from the kernel descriptors (.kd symbols)."""
    lib = pathlib.Path(lib)
    tmp = None
    if work is None:
        tmp = tempfile.TemporaryDirectory()
        work = pathlib.Path(tmp.name)
    try:
        out: dict[str, dict[str, str]] = {}
        for co in code_objects(lib, pathlib.Path(work)):
            txt = subprocess.run([str(LLVM / "llvm-objdump"), "-D", "-j", ".rodata", str(co)],
                                 check=True, capture_output=True, text=True).stdout
            cur = None
            for line in txt.splitlines():
                s = line.strip()
                if s.startswith(".amdhsa_kernel "):
                    cur = s.split(None, 1)[1]
                    out[cur] = {}
                elif s.startswith(".end_amdhsa_kernel"):
                    cur = None
                elif cur is not None and s.startswith(".amdhsa_"):
                    k, _, v = s.partition(" ")
                    out[cur][k] = v.strip()
        return out
    finally:
        if tmp is not None:
            tmp.cleanup()


def main(argv):
    if len(argv) == 1:
        for k, v in sorted(kernels(argv[0]).items()):
            print(f"{len(v):7d}  {k}")
        return 0
    a, b = kernels(argv[0]), kernels(argv[1])
    diff = [k for k in sorted(set(a) | set(b)) if a.get(k) != b.get(k)]
    print(f"{len(a)} / {len(b)} symbols, {len(diff)} differ")
    for k in diff:
        print(f"   {k}  {len(a.get(k, []))} / {len(b.get(k, []))}")
    return 1 if diff else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
