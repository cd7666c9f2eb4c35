"""Guards on the built gfx950 code object of liborbx.so (CPU only: the device code is
extracted from the library's .hip_fatbin section and disassembled, no GPU needed).

A pointer the compiler cannot place in one address space (e.g. one picked at run time
between an LDS array and global scratch) is generic: its accesses become flat instructions,
which for LDS data run at memory latency instead of LDS latency.  Round 5 found two such
cases (k_octree's candidate arrays, k_pyr_chain's ping-pong buffers) costing 10-80 us per
launch; the hot kernels must have none."""
import pathlib
import re
import shutil
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
LIB = ROOT / "my_orb_slam2_amd" / "liborbx.so"
LLVM = pathlib.Path("/opt/rocm/lib/llvm/bin")
HOT = ("k_octree", "k_pyr_chain", "k_fast", "k_orient_desc", "k_level_strip", "k_stereo",
       "k_bow", "k_proj_search", "k_triangulate", "k_bf_mfma")


def _disasm(tmp_path):
    if not LIB.exists() or shutil.which("objcopy") is None or not (LLVM / "llvm-objdump").exists():
        pytest.skip("liborbx.so or the LLVM tools are missing")
    fat, co = tmp_path / "fat.bin", tmp_path / "k.co"
    # objcopy with no output file rewrites its input: work on a copy (the library is mapped
    # into this process by the other tests)
    lib = tmp_path / "liborbx.so"
    shutil.copyfile(LIB, lib)
    subprocess.run(["objcopy", f"--dump-section=.hip_fatbin={fat}", str(lib), str(tmp_path / "discard.so")],
                   check=True, capture_output=True)
    subprocess.run([str(LLVM / "clang-offload-bundler"), "--unbundle", "--type=o",
                    f"--input={fat}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                    f"--output={co}"], check=True, capture_output=True)
    out = subprocess.run([str(LLVM / "llvm-objdump"), "-d", str(co)], check=True,
                         capture_output=True, text=True).stdout
    funcs, cur = {}, None
    for line in out.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = m.group(1)
            funcs[cur] = []
        elif cur is not None and line.strip():
            funcs[cur].append(line)
    return funcs


def test_hot_kernels_have_no_flat_memory_ops(tmp_path):
    funcs = _disasm(tmp_path)
    hot = {n: body for n, body in funcs.items() if any(h in n for h in HOT)}
    assert hot, "no hot kernel found in the code object"
    bad = {n: sum(1 for l in body if re.search(r"\bflat_(load|store|atomic)", l))
           for n, body in hot.items()}
    bad = {n: c for n, c in bad.items() if c}
    assert not bad, f"flat (generic address space) memory ops in hot kernels: {bad}"
