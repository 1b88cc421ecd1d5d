"""CPU: bench.py's measurement definitions -- the algorithmic byte model of the
RC pass and the gather roofline built from a PMC record."""
import json
import os

import pytest

from conftest import ROOT


@pytest.fixture(scope="module")
def bench():
    import sys

    sys.path.insert(0, ROOT)
    import bench as b

    return b


def test_rc_byte_model_matches_survey(bench):
    # 16·CW·CH·(2N−1) + 4·W·H·N = 3.355 GB per pass at 4096², N=6
    assert bench.b_rc(4096, 4096, 4096, 4096, 6) == 16 * 4096 * 4096 * 11 + 4 * 4096 * 4096 * 6
    assert abs(bench.b_rc(4096, 4096, 4096, 4096, 6) / 1e9 - 3.355) < 1e-3
    # C1 0.231 GB, C2 4.563 GB
    assert abs(bench.b_rc(1200, 900, 1216, 960, 6) / 1e9 - 0.231) < 1e-3
    assert abs(bench.b_rc(4096, 4096, 4096, 4096, 8) / 1e9 - 4.563) < 1e-3
    # RGBA16F cascades halve the cascade terms
    assert bench.b_rc(64, 64, 64, 64, 2, gi_bytes=8) == 8 * 64 * 64 * 3 + 4 * 64 * 64 * 2


def test_gather_roofline_blends_the_ceiling_by_hit_rate(bench):
    rec = {"per_level": {f"k_rc_level L{L}": {"l2_requests": 1e6 * (L + 1), "l2_hit": 1.0} for L in range(4)}}
    g = bench.gather_roofline(rec, 4, [0.1, 0.1, 0.1, 0.1])
    # upper half = L2, L3: 7e6 requests in 0.2 ms -> 35 G/s against the L2-resident ceiling
    assert g["kernel"] == "k_rc_level L2-L3"
    assert abs(g["achieved"] - 35.0) < 1e-9 and g["peak"] == bench.GATHER_L2_GLINES
    rec["per_level"]["k_rc_level L3"]["l2_hit"] = 0.0
    g = bench.gather_roofline(rec, 4, [0.1, 0.1, 0.1, 0.1])
    h = 3 / 7
    want = 1.0 / (h / bench.GATHER_L2_GLINES + (1 - h) / bench.GATHER_MALL_GLINES)
    assert abs(g["peak"] - round(want, 1)) < 1e-9 and abs(g["l2_hit"] - round(h, 4)) < 1e-9
    # a record without L2 counters gives no gather roofline
    assert bench.gather_roofline({"per_level": {}}, 4, [0.1] * 4) is None


def test_committed_pmc_record_has_the_gather_fields(bench):
    """Every committed PMC record is keyed on what it measured (config, rayRange, storage, scene, schedule,
    knobs), one record per key, and the headline's record (demo scene, committed schedule) is there."""
    path = os.path.join(ROOT, "profiles", "rc_level_pmc.json")
    with open(path) as f:
        recs = json.load(f)["records"]
    keys = [json.dumps(r["key"], sort_keys=True) for r in recs]
    assert len(set(keys)) == len(keys)
    for rec in recs:
        assert rec["config"] == rec["key"]["config"] and rec["hbm_bytes_per_launch"] > 0
        N = len(rec["key"]["rc_variant"])
        for L in range(N):
            lv = rec["per_level"][f"k_rc_level L{L}"]
            assert lv["l2_requests"] > 0 and 0.0 < lv["l2_hit"] < 1.0 and lv["dur_us"] > 0
    with open(os.path.join(ROOT, "radiancecascade2dglobalillumination_amd", "tuning", "4096x4096_N6_rr2_f32.json")) as f:
        sched = json.load(f)
    key = bench.pmc_key(4096, 4096, 6, 2.0, "f32", "demo", sched["rc_order"], sched["rc_variant"], sched.get("knobs"))
    assert bench.find_pmc_record(path, key) is not None
    # another scene (or schedule) finds nothing: its line carries traffic null, not the demo's counters
    assert bench.find_pmc_record(path, dict(key, scene="random:3")) is None
    assert bench.find_pmc_record(path, dict(key, rc_order=[0] * 6)) is None


def test_valu_roofline_is_issue_time_over_level_time(bench):
    """valu_roofline: wave instructions per frame, priced at each level's cycles per instruction
    (plain wave64 VALU: 2 cycles on a SIMD-32, MI355X_MICROARCH.md), over the level times, against
    256 CUs x 4 SIMDs at 2.4 GHz."""
    rec = {"per_level": {f"k_rc_level L{L}": {"valu_insts": 1228.8e6 / 4} for L in range(4)}}
    v = bench.valu_roofline(rec, 4, [0.25] * 4)  # 1228.8 M plain instructions in 1 ms: the peak
    assert abs(v["achieved"] - 1228.8) < 0.1 and abs(v["frac"] - 1.0) < 1e-3 and abs(v["floor_ms"] - 1.0) < 1e-3
    mix = {"levels": {f"L{L}": {"valu_cycles_per_inst": 4.0} for L in range(4)}}  # e.g. all v_pk_*_f32
    v = bench.valu_roofline(rec, 4, [0.25] * 4, mix)
    assert abs(v["frac"] - 2.0) < 1e-3 and abs(v["floor_ms"] - 2.0) < 1e-3
    assert bench.valu_roofline({"per_level": {}}, 4, [0.1] * 4) is None


def test_isa_mix_classes():
    import sys

    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import isa_mix

    assert isa_mix.classify("v_pk_fma_f32") == "valu_pk" and isa_mix.classify("v_fma_f32") == "valu"
    assert isa_mix.classify("v_rcp_f32_e32") == "valu_tr" and isa_mix.classify("v_lshl_add_u64") == "valu_64"
    assert isa_mix.classify("s_and_b64") == "salu" and isa_mix.classify("global_load_ushort") == "vmem"
    assert isa_mix.classify("ds_read_u8") == "lds" and isa_mix.classify("s_waitcnt") == "wait"


def _run_bench(args, env_extra=None, timeout=180):
    import subprocess
    import sys

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=timeout, env=env)


def test_gpus_n_spawns_n_ranks_over_gloo():
    # bench.py --gpus 2 outside torch.distributed.run launches two ranks itself (before any GPU call)
    # and the line reports the process group's world size, never a silent one-rank run
    r = _run_bench(["--gpus", "2", "--launch-check", "--backend", "gloo"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["pg_world"] == 2 and line["max_rank"] == 1


def test_world_size_mismatch_is_an_error():
    r = _run_bench(["--gpus", "4", "--launch-check", "--backend", "gloo"], {"WORLD_SIZE": "2"}, timeout=60)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


def test_strips_launch_check_world_8_over_gloo():
    """bench.py --gpus 8 --mode strips --launch-check --backend gloo: eight ranks rehearse the row-strip exchange of a
    C3 frame (8192^2, N=8) without a GPU -- every JumpFlood step's transfers of the library's plan as point-to-point
    messages carrying their global rows, checked at the receiver, every tap row of every strip own or delivered,
    the distRT strips partitioning the screen (bench.strips_launch_check)."""
    r = _run_bench(["--gpus", "8", "--mode", "strips", "--launch-check", "--backend", "gloo", "--size", "8192",
                    "--cascades", "8", "--ray-range", "64"], timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 8 and line["pg_world"] == 8 and line["mode"] == "strips"
    assert line["steps_checked"] == 12 and line["transfers"] > 0 and line["rows_exchanged"] > 0
    assert sorted(tuple(p) for p in line["strips"]) == [(1024 * k, 1024 * (k + 1)) for k in range(8)]
