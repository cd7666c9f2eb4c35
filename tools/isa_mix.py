#!/usr/bin/env python3
"""Static VALU instruction mix of every kernel in liborbx.so, weighted by the measured issue
cost of each opcode on gfx950 (profiles/r01_valu_issue_rates.txt: cycles per wave64
instruction per SIMD with several waves per SIMD; about 2 for the full-rate class, about 4
for the rest).  The mean cost per VALU instruction of a kernel turns its dynamic instruction
count (SQ_INSTS_VALU) into VALU-busy cycles; bench.py divides those by the SIMDs' cycles for
a mix-aware issue fraction (SQ_ACTIVE_INST_VALU counts every instruction as 4 cycles, so
VALUBusy overstates a kernel rich in full-rate instructions and can exceed 1).

The weights are the kernel's static opcode counts: its hot loops are unrolled (strip walk
blocks, FAST compass rows, rBRIEF samples), so they dominate the static code too; the
approximation is stated wherever the number is used.

    python tools/isa_mix.py [OUT.json]     # runs hipcc -S on each source (no GPU needed)
"""
from __future__ import annotations

import json
import pathlib
import re
import subprocess
import sys
import tempfile

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from my_orb_slam2_amd import build as b  # noqa: E402

RATES = ROOT / "profiles" / "r01_valu_issue_rates.txt"


def load_rates():
    rates = {}
    for line in RATES.read_text().splitlines():
        m = re.match(r"(v_\w+)\s+[\d.]+ ms\s+([\d.]+) cycles", line)
        if m:
            rates[m.group(1)] = float(m.group(2))
    return rates


def cost_of(op: str, rates: dict):
    """Measured cycles of an opcode, matching the measured variant names (e.g. v_add_u32_e32
    -> v_add_u32, v_add_co_u32 -> v_add_u32); None if nothing similar was measured."""
    base = re.sub(r"_(e32|e64|dpp|sdwa)$", "", op)
    cands = [base, base.replace("_co_", "_").replace("_nc_", "_"),
             re.sub(r"_[iu](16|32)$", lambda m: "_u" + m.group(1), base),
             re.sub(r"_b32$", "_u32", base), re.sub(r"_u32$", "_b32", base),
             re.sub(r"_i32$", "_u32", base), base.replace("fmac", "fma").replace("mac_", "mad_")]
    for c in cands:
        if c in rates:
            return rates[c]
    if base.startswith("v_pk_"):
        return 4.3                       # every measured packed op issues at the 4-cycle rate
    if base.startswith(("v_cvt_", "v_dot", "v_mfma", "v_readlane", "v_readfirstlane")):
        return 4.2
    if base.startswith(("v_cndmask", "v_cmp", "v_mov", "v_subrev", "v_addc", "v_subb")):
        return 2.4                       # VOP2/VOPC form of the full-rate class
    return None


def kernel_histograms(asm: str):
    """{kernel symbol: {opcode: static count}} of the VALU instructions in a .s file."""
    out, cur = {}, None
    for line in asm.splitlines():
        m = re.match(r"^(_Z[\w.]+):\s*(;|$)", line)
        if m and not m.group(1).startswith(".L"):
            cur = m.group(1)
            out.setdefault(cur, {})
            continue
        if cur is None:
            continue
        if line.startswith(".Lfunc_end"):   # a kernel may hold several s_endpgm
            cur = None
            continue
        m = re.match(r"^\s+(v_\w+)", line)
        if m:
            out[cur][m.group(1)] = out[cur].get(m.group(1), 0) + 1
    return out


def main():
    out_path = pathlib.Path(sys.argv[1]) if len(sys.argv) > 1 else ROOT / "profiles" / "r03_isa_mix.json"
    rates = load_rates()
    result = {}
    with tempfile.TemporaryDirectory() as d:
        for src in b.SOURCES:
            s = pathlib.Path(d) / (src + ".s")
            cmd = [b.hipcc()] + [f for f in b.FLAGS if f not in ("-shared", "-fPIC")] + \
                  ["-S", "--cuda-device-only", str(b.CSRC / src), "-o", str(s)]
            subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)
            for sym, hist in kernel_histograms(s.read_text()).items():
                n = sum(hist.values())
                if not n:
                    continue
                known = {op: c for op, c in hist.items() if cost_of(op, rates) is not None}
                nk = sum(known.values())
                mean = sum(c * cost_of(op, rates) for op, c in known.items()) / nk if nk else None
                result[sym] = {"static_valu": n, "covered": nk / n, "mean_cycles": mean,
                               "full_rate_frac": sum(c for op, c in known.items()
                                                     if cost_of(op, rates) < 3.0) / max(nk, 1),
                               "uncovered": sorted(op for op in hist if op not in known)}
    out_path.write_text(json.dumps(result, indent=1, sort_keys=True))
    for sym, r in sorted(result.items()):
        if any(k in sym for k in ("k_level", "k_fast", "k_octree", "k_orient", "k_stereo",
                                  "k_bow", "k_kfdb")):
            print(f"{sym[:60]:60s} n={r['static_valu']:5d} cov={r['covered']:.2f} "
                  f"mean={r['mean_cycles'] or 0:.2f} full={r['full_rate_frac']:.2f}")


if __name__ == "__main__":
    main()
