"""Guards on the built gfx950 code objects of liborbx.so and on its sources (CPU only: the
device code is extracted from the library's .hip_fatbin section, one offload bundle per
translation unit, and disassembled; no GPU needed).

* A pointer the compiler cannot place in one address space (e.g. one picked at run time
  between an LDS array and global scratch) is generic: its accesses become flat instructions,
  which for LDS data run at memory latency instead of LDS latency.  Round 5 found two such
  cases (k_octree's candidate arrays, k_pyr_chain's ping-pong buffers) costing 10-80 us per
  launch; the hot kernels must have none.
* k_fast's arc score packs pixel bytes into fp16 subnormals (fast_arc_score_pk,
  orbx_extract.hip): a kernel whose fp16 denormals are flushed would score every corner 0.
  Every kernel must keep fp16/fp64 denormals (.amdhsa_float_denorm_mode_16_64 3).
* The product sources carry no compile-time variant switches (round 6 removed ~180 of them:
  diagnostic builds that wrote wrong outputs on purpose, losing branches of closed A/Bs), and
  the product library is built without extra -D flags (build.py refuses them)."""
import pathlib
import re
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))
import isa_dump  # noqa: E402

LIB = ROOT / "my_orb_slam2_amd" / "liborbx.so"
CSRC = ROOT / "my_orb_slam2_amd" / "csrc"
HOT = ("k_octree", "k_pyr_chain", "k_fast", "k_orient_desc", "k_level_strip", "k_stereo",
       "k_bow", "k_proj_search", "k_triangulate", "k_bf_mfma", "k_bf_top2")
# the only conditionals left in csrc/: the build's source-hash default and the host/device
# split of orbx_math.h (shared with the host oracle checks)
ALLOWED_CONDITIONALS = {("orbx_capi.hip", "#ifndef ORBX_SRC_HASH"),
                        ("orbx_math.h", "#if defined(__HIPCC__)")}


def _need_tools():
    if not LIB.exists() or not isa_dump.available():
        pytest.skip("liborbx.so or the LLVM tools are missing")


def test_every_translation_unit_is_inspected(tmp_path):
    _need_tools()
    funcs = isa_dump.kernels(LIB, tmp_path)
    for h in HOT:
        assert any(h in n for n in funcs), f"{h} not found in any code object"


def test_hot_kernels_have_no_flat_memory_ops(tmp_path):
    _need_tools()
    funcs = isa_dump.kernels(LIB, tmp_path)
    hot = {n: body for n, body in funcs.items() if any(h in n for h in HOT)}
    assert hot, "no hot kernel found in the code objects"
    bad = {n: sum(1 for l in body if re.search(r"\bflat_(load|store|atomic)", l))
           for n, body in hot.items()}
    bad = {n: c for n, c in bad.items() if c}
    assert not bad, f"flat (generic address space) memory ops in hot kernels: {bad}"


def test_fp16_denormals_kept(tmp_path):
    _need_tools()
    kd = isa_dump.descriptors(LIB, tmp_path)
    fast = [n for n in kd if "k_fast" in n]
    assert fast, "k_fast's kernel descriptor not found"
    bad = {n: d.get(".amdhsa_float_denorm_mode_16_64") for n, d in kd.items()
           if d.get(".amdhsa_float_denorm_mode_16_64") != "3"}
    assert not bad, f"kernels flushing fp16/fp64 denormals: {bad}"


def test_no_variant_switches_in_sources():
    found = set()
    for p in sorted(CSRC.iterdir()):
        if p.suffix not in (".hip", ".h", ".inc"):
            continue
        for line in p.read_text().splitlines():
            s = line.strip()
            if re.match(r"#\s*if", s):
                found.add((p.name, re.sub(r"\s+", " ", s.split("//")[0].strip())))
    assert found <= ALLOWED_CONDITIONALS, f"compile-time switches in csrc/: {found - ALLOWED_CONDITIONALS}"


def test_build_refuses_product_variants():
    from my_orb_slam2_amd import build
    with pytest.raises(ValueError):
        build.build(extra_flags=["-DSOME_DIAG=1"])
