"""Host-side checks of bench.py's measurement helpers against the committed profiles (no GPU).

The headline roofline's `traffic` is FETCH_SIZE x2 + WRITE_SIZE from the rocprofv3 PMC passes
(MI355X_MICROARCH.md §HBM); the committed bench line must agree with the committed CSVs."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _bench():
    import bench
    return bench


def _latest(pattern):
    import glob
    def key(p):   # (round, version) of profiles/rNN_vM_*
        name = os.path.basename(p)
        return int(name[1:3]), int(name.split("_v")[1].split("_")[0])
    return sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)), key=key)[-1]


def test_headline_traffic_matches_committed_pmc():
    b = _bench()
    line = json.load(open(_latest("r[0-9][0-9]_v*_bench.json")))
    roof = line["roofline"]
    if "launches_per_step" not in roof:
        pytest.skip("headline line predates the per-step roofline (round 4)")
    # the PMC passes count one-stream dispatches; the entry is per launch of the timed schedule
    t = b.traffic_per_step(b.DEFAULT_PMC, roof["kernel"])
    assert t is not None and t > 0
    assert t / roof["launches_per_step"] == pytest.approx(roof["traffic"], rel=1e-9)
    # the algorithmic bytes and the achieved rate are consistent with the launch time (the HBM
    # figures sit in `hbm` when the counters name VALU issue as the binding roof)
    hbm = roof["hbm"] if roof.get("bound") == "valu" else roof
    assert hbm["achieved"] == pytest.approx(
        roof["algorithmic_bytes_per_launch"] / (roof["avg_launch_ms"] / 1000.0) / 1e9, rel=1e-9)
    assert roof["frac"] == pytest.approx(roof["achieved"] / roof["peak"], rel=1e-9)


def test_binding_roof_label():
    """`bound` names the roof the counters show.  A launch whose SIMDs issue VALU
    work most of the time is labelled "valu" (its fraction = the mix-aware busy fraction, the
    HBM figures kept beside it); one that does not stays "hbm"."""
    b = _bench()
    e = b.roofline_entry("k_fast", 10.0, 10, 10, 7.0e8, None)
    # 0.75 of 1024 SIMDs x 1 ms x 2.4 GHz at 3 cycles per instruction
    e["valu"] = {"busy_frac": 0.75, "valubusy_4cycle": 1.01, "wave_instr_per_launch": 6.144e8,
                 "mean_issue_cycles": 3.0}
    hbm_frac = e["frac"]
    b.label_binding_roof(e)
    assert e["bound"] == "valu" and e["frac"] == pytest.approx(0.75) and e["hbm"]["frac"] == hbm_frac
    assert e["frac"] == pytest.approx(e["achieved"] / e["peak"], rel=1e-9)
    # k_level1_7 in r05: VALU 0.60 busy against HBM 0.34-0.43 -> valu (round 5 said hbm)
    e = b.roofline_entry("k_level1_7", 10.0, 70, 10, 3.4e9, None)
    hbm_frac = e["frac"]
    e["valu"] = {"busy_frac": 0.60, "valubusy_4cycle": 0.64, "wave_instr_per_launch": 7e7,
                 "mean_issue_cycles": 3.66}
    b.label_binding_roof(e)
    assert hbm_frac < 0.6 and e["bound"] == "valu" and e["hbm"]["frac"] == hbm_frac
    # an entry whose HBM fraction exceeds its VALU busy fraction stays hbm
    e = b.roofline_entry("k_level0", 10.0, 10, 10, 7.0e9, None)
    e["valu"] = {"busy_frac": 0.30, "wave_instr_per_launch": 1e8, "mean_issue_cycles": 3.0}
    b.label_binding_roof(e)
    assert e["frac"] > 0.3 and e["bound"] == "hbm" and e["hbm"]["frac"] == e["frac"]
    # no VALU entry: hbm
    e = b.roofline_entry("k_octree", 1.0, 10, 10, 1e6, None)
    b.label_binding_roof(e)
    assert e["bound"] == "hbm"


def test_valu_floor_on_committed_r05_line():
    """the step's VALU issue floor = sum over the kernel groups of wave
    instructions per launch x launches per step x mean issue cycles, over 1024 SIMDs x 2.4 GHz.
    On the committed r05 line (its per_kernel entries come from the r05 PMC CSVs) that is
    2.61 ms, 0.67 of the 3.90 ms timed step."""
    b = _bench()
    line = json.load(open(os.path.join(ROOT, "profiles", "r05_v5_bench.json")))
    pk = line["roofline"]["per_kernel"]
    want = sum(pk[k]["valu"]["wave_instr_per_launch"] * pk[k]["launches_per_step"] *
               pk[k]["valu"]["mean_issue_cycles"] for k in b.HEADLINE_GROUPS) / (1024 * 2.4e9) * 1e3
    assert b.valu_floor_ms(pk) == pytest.approx(want, rel=1e-12)
    assert b.valu_floor_ms(pk) == pytest.approx(2.61, abs=0.01)
    roof = {"per_kernel": pk}
    b.add_valu_floor(roof, line["ms_per_step"])
    assert roof["valu_floor_frac"] == pytest.approx(0.67, abs=0.01)
    # the k_level union entry is not counted twice
    assert "k_level" in pk and "k_level" not in b.HEADLINE_GROUPS
    # an entry without PMC counts makes the floor unknown, not smaller
    pk2 = dict(pk, k_fast=dict(pk["k_fast"], valu=None))
    assert b.valu_floor_ms(pk2) is None


def test_latest_line_carries_valu_floor():
    b = _bench()
    roof = json.load(open(_latest("r[0-9][0-9]_v*_bench.json")))["roofline"]
    if "valu_floor_ms" not in roof:
        pytest.skip("headline line predates the VALU floor (round 6)")
    assert roof["valu_floor_ms"] == pytest.approx(b.valu_floor_ms(roof["per_kernel"]), rel=1e-9)
    for e in roof["per_kernel"].values():
        v = (e.get("valu") or {}).get("busy_frac")
        if v is not None:
            assert e["bound"] == ("valu" if v > e["hbm"]["frac"] else "hbm")


def test_roofline_entries_per_launch():
    """Per-step algorithmic bytes and traffic divide by the launches per step of the run the
    entry times: k_fast launched twice per step (the side branch) gets half a step's bytes per
    launch."""
    b = _bench()
    e = b.roofline_entry("k_level", 16.0, 160, 20, 2.4e9, None)
    assert e["launches_per_step"] == 8
    assert e["avg_launch_ms"] == pytest.approx(0.1)
    assert e["algorithmic_bytes_per_launch"] == pytest.approx(3.0e8)
    assert e["achieved"] == pytest.approx(3.0e8 / 1e-4 / 1e9)
    e = b.roofline_entry("k_fast", 10.0, 40, 20, 7.0e8, 1.4e9)
    assert e["launches_per_step"] == 2
    assert e["algorithmic_bytes_per_launch"] == pytest.approx(3.5e8)
    assert e["traffic"] == pytest.approx(7.0e8)
    assert e["frac"] == pytest.approx(e["achieved"] / b.HBM_PEAK_GBS)


def test_headline_picks_largest_one_stream_group():
    """roofline.kernel is the kernel group with the most one-stream time per step (VERDICT r3:
    k_fast, not the hard-coded k_level); k_level splits into level 0 and levels 1-7."""
    b = _bench()
    sprof = {"k_level": (30.0, 160), "k_level0": (5.0, 20), "k_fast": (28.0, 20),
             "k_octree": (6.0, 20), "k_orient_desc": (22.0, 20), "k_stereo": (5.0, 20)}
    g = b.split_level(sprof)
    assert g["k_level1_7"] == (25.0, 140)
    assert b.pick_dominant(g, 20) == "k_fast"


def test_traffic_needs_both_passes(tmp_path):
    b = _bench()
    f = tmp_path / "fetch.csv"
    f.write_text('"Dispatch_Id","Kernel_Name","Counter_Name","Counter_Value"\n'
                 '1,"orbx::k_level(x)","FETCH_SIZE",100\n2,"orbx::k_level(x)","FETCH_SIZE",300\n')
    assert b.traffic_from_csv(str(f), "k_level") is None   # WRITE_SIZE pass missing
    w = tmp_path / "write.csv"
    w.write_text('"Dispatch_Id","Kernel_Name","Counter_Name","Counter_Value"\n'
                 '1,"orbx::k_level(x)","WRITE_SIZE",50\n')
    # mean FETCH 200 KiB doubled + WRITE 50 KiB
    assert b.traffic_from_csv(f"{f},{w}", "k_level") == pytest.approx((2 * 200 + 50) * 1024.0)


def test_result_line_is_the_only_stdout():
    """Native chatter on fd 1 (RCCL's version banner) goes to stderr; stdout holds only the
    result line the driver parses."""
    import subprocess
    import sys
    code = ("import os, bench; bench.keep_stdout_for_result(); "
            "os.write(1, b'RCCL version : x\\n'); print('py noise'); bench.emit('{\"value\": 1}')")
    r = subprocess.run([sys.executable, "-c", code], cwd=str(ROOT), capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout == '{"value": 1}\n'
    assert "RCCL version" in r.stderr and "py noise" in r.stderr


def test_counted_bytes_capped_by_traffic():
    """Overlapping reads (k_orient_desc's patches) are credited at most the measured HBM
    bytes, so the per-kernel fraction never exceeds what the PMC passes saw."""
    b = _bench()
    assert b.counted_bytes(4.95e9, 3.07e9) == 3.07e9
    assert b.counted_bytes(6.1e8, 6.2e8) == 6.1e8
    assert b.counted_bytes(6.1e8, None) == 6.1e8
    e = b.roofline_entry("k_orient_desc", 13.6, 10, 10, 1e12,
                         b.traffic_per_step(b.DEFAULT_PMC, "k_orient_desc"))
    assert e["algorithmic_bytes_per_launch"] == e["traffic"] < e["requested_bytes_per_launch"]


def test_gpus_flag_must_match_world_size():
    """`--gpus 2` under a launcher that started one rank is an error, not a silent 1-GPU run."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                       cwd=str(ROOT), capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0
    assert "does not match WORLD_SIZE=1" in r.stderr


def test_valu_entry_from_pmc(tmp_path):
    """The roofline's VALU issue entry: SQ_INSTS_VALU averaged over a kernel's dispatches; the
    mix-aware busy fraction prices them at the kernel's mean issue cycles (tools/isa_mix.py)
    over 1024 SIMDs x the launch time at 2.4 GHz; rocprof's VALUBusy (4 cycles per
    instruction, over GRBM_GUI_ACTIVE / 8) rides along."""
    b = _bench()
    f = tmp_path / "insts.csv"
    f.write_text('"Dispatch_Id","Kernel_Name","Counter_Name","Counter_Value"\n'
                 '1,"void orbx::k_level_strip<4>(x)","SQ_INSTS_VALU",100\n'
                 '2,"void orbx::k_level_strip<3>(x)","SQ_INSTS_VALU",300\n'
                 '3,"orbx::k_fast(x)","SQ_INSTS_VALU",999\n'
                 '3,"orbx::k_fast(x)","SQ_INSTS_SALU",5\n'
                 '3,"orbx::k_fast(x)","SQ_ACTIVE_INST_VALU",1000\n'
                 '3,"orbx::k_fast(x)","GRBM_GUI_ACTIVE",8000\n')
    mix = tmp_path / "mix.json"
    mix.write_text(json.dumps({"_ZN4orbx6k_fastEPKNS_8G": {"mean_cycles": 3.0},
                               "_ZN4orbx13k_level_stripILi3EEEvPK": {"mean_cycles": 3.5},
                               "_ZN4orbx13k_level_stripILi4EEEvPK": {"mean_cycles": 2.5}}))
    assert b.valu_from_csv(str(f), "k_level") == pytest.approx(200.0)
    assert b.mix_cycles_from_csv(str(f), "k_level", str(mix)) == pytest.approx(
        (100 * 2.5 + 300 * 3.5) / 400)
    b.ISA_MIX = str(mix)
    e = b.valu_entry(str(f), "k_fast", 1e-6)
    b.ISA_MIX = os.path.join(ROOT, "profiles", "r04_isa_mix.json")
    assert e["wave_instr_per_launch"] == pytest.approx(999.0)
    assert e["busy_frac"] == pytest.approx(999.0 * 3.0 / (1024 * 1e-6 * 2.4e9))
    assert e["valubusy_4cycle"] == pytest.approx(4.0 * 1000 / (1024 * 1000))
    assert b.valu_entry(str(f), "k_stereo", 1e-6) is None


def test_headline_valu_entry_matches_committed_pmc():
    """The committed headline line's VALU entry is the committed SQ_INSTS_VALU pass over the
    line's own average launch duration."""
    b = _bench()
    roof = json.load(open(_latest("r[0-9][0-9]_v*_bench.json")))["roofline"]
    if "valu" not in roof:
        pytest.skip("headline line predates the VALU entry")
    if "launches_per_step" not in roof:
        pytest.skip("headline line predates the per-step roofline (round 4)")
    v = b.valu_from_csv(b.DEFAULT_INSTS, roof["kernel"]) * \
        b.ONE_STREAM_LAUNCHES.get(roof["kernel"], 1) / roof["launches_per_step"]
    assert roof["valu"]["wave_instr_per_launch"] == pytest.approx(v)
    assert roof["valu"]["issue_rate"] == pytest.approx(v / (roof["avg_launch_ms"] / 1000.0) / 1e12)
    assert 0 < roof["valu"]["busy_frac"] <= 1.0


def test_ta_busy_from_committed_pass():
    """The per-kernel `ta_busy` of the headline roofline: TA_BUSY_avr over GRBM_GUI_ACTIVE / 8
    from the committed one-stream TA pass.  k_orient_desc's patch staging keeps the texture
    addresser the busiest unit of that kernel; a kernel absent from the pass has
    none."""
    b = _bench()
    t = b.ta_busy_from_csv(b.DEFAULT_TA, "k_orient_desc")
    assert t is not None and 0.5 < t <= 1.0
    assert b.ta_busy_from_csv(b.DEFAULT_TA, "k_no_such_kernel") is None
