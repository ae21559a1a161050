"""The committed bench line (profiles/r4_c2_bench.json, written by bench.py on an
MI355X) carries every field of the driver's contract: the headline metric of
BASELINE.json on config 2, the dominant kernel's roofline and the CPU baseline.
Its roofline fractions are physical (<= 1) and recomputable from profiles/
(tools/roofline_check.py)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = "r4_c2_bench.json"
SUMMARY = "r4_c2_timed_summary.txt"


def load(name):
    with open(os.path.join(REPO, "profiles", name)) as f:
        return json.loads(f.read().strip().splitlines()[-1])


def test_c2_bench_line_contract():
    d = load(BENCH)
    base = json.load(open(os.path.join(REPO, "BASELINE.json")))
    assert d["metric"] == base["metric"]
    for k in ("value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["unit"] == "Msamples/s" and d["higher_is_better"] is True and d["n_gpus"] == 1
    assert d["config"]["workload"] and (d["config"]["width"], d["config"]["height"], d["config"]["spp"]) == (1200, 800, 500)
    # value = samples / wall time of the timed steps
    assert abs(d["value"] - 1200 * 800 * 500 / (d["ms_per_step"] / 1e3) / 1e6) <= 0.01 * d["value"]
    r = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert r["bound"] == "valu" and r["unit"] == "Tlane-op/s"
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert 0 < r["frac"] <= 1 and 0 < r["hbm"]["frac"] <= 1 and r["hbm"]["peak"] == 8000.0
    assert 0 < r["valu"]["lane_util"] <= 1
    assert r["traffic"] and r["traffic"] > 0
    c = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in c, k
    assert c["kind"] in ("port", "reference") and c["cores"] >= 1 and c["value"] > 0
    # the reference's 8 threads AND all host cores
    assert c["legs"]["threads_8"]["threads"] == 8 and c["legs"]["threads_all"]["threads"] == c["cores_all"]
    assert c["value"] == max(v["value"] for v in c["legs"].values())


@pytest.mark.parametrize("config", ["c2", "c3", "c4", "c5", "cornell", "cornell_smoke", "simple_light"])
def test_roofline_recomputes_from_profiles(config):
    """Every committed round-4 bench line: VALU and HBM fractions <= 1 and recomputable from
    the PMC passes in profiles/ (taken on the same build: the line's build_id) and its HIP-event launch time."""
    line = os.path.join(REPO, "profiles", f"r4_{config}_bench.json")
    rc = subprocess.run([sys.executable, os.path.join(REPO, "tools", "roofline_check.py"), line],
                        capture_output=True, text=True)
    assert rc.returncode == 0, rc.stdout + rc.stderr
    d = load(f"r4_{config}_bench.json")
    r = d["roofline"]
    assert r["bound"] == "valu" and 0 < r["frac"] <= 1 and 0 < r["hbm"]["frac"] <= 1
    assert r["peak"] == 78.643 and "r4_valu_peak" in r["valu"]["peak_source"]
    for kind in ("valu", "traffic"):
        with open(os.path.join(REPO, "profiles", f"pmc_{kind}_{config}_sah.json")) as f:
            assert json.load(f)["_build"]["build_id"] == d["build_id"]


def test_rocprof_summary_agrees_with_bench_events():
    """profiles/r4_c2_timed_summary.txt (rocprofv3 --kernel-trace --stats of the bench
    command) and the bench's HIP-event average of the dominant kernel agree."""
    d = load(BENCH)
    kernel = d["roofline"]["kernel"].split("<")[0]
    for line in open(os.path.join(REPO, "profiles", SUMMARY)):
        if kernel + "<" in line:
            mean_us = float(line.split()[-3])
            assert abs(mean_us / 1e3 - d["roofline"]["avg_launch_ms"]) <= 0.05 * d["roofline"]["avg_launch_ms"]
            return
    raise AssertionError(f"{kernel} not in the rocprof summary")


PMC_CONFIGS = ["c2", "c3", "c4", "c5", "cornell", "cornell_smoke", "simple_light"]


@pytest.mark.parametrize("config", PMC_CONFIGS)
def test_pmc_passes_are_from_this_build(rtw, config):
    """Every committed PMC pass bench.py derives a roofline from (profiles/pmc_{valu,traffic}_<config>_sah.json)
    was taken on the library these sources build: its _build.build_id is rtw_build_id() (test_abi.py checks
    that the loaded library IS these sources).  bench.py uses no pass of another build (roofline.frac null)."""
    want = rtw.lib().rtw_build_id().decode()
    for kind in ("valu", "traffic"):
        with open(os.path.join(REPO, "profiles", f"pmc_{kind}_{config}_sah.json")) as f:
            d = json.load(f)
        assert d.get("_build", {}).get("build_id") == want, (kind, config, d.get("_build"), want)
        assert d["_build"].get("config") == config


def test_bench_refuses_a_stale_pmc_pass(tmp_path, monkeypatch):
    """bench.py's PMC readers return nothing (so roofline.frac is null) for a pass of another build."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    prof = tmp_path / "profiles"
    prof.mkdir()
    entry = {"lane_ops": 1e11, "insts_valu": 3e9, "active_inst_valu": 3e9, "thread_cycles_valu": 1e11,
             "kernels": ["wf_step_clds<0u>"], "lane_util": 0.5}
    json.dump({"wf_step": entry, "_build": {"build_id": "aaaa", "config": "c2"}}, open(prof / "pmc_valu_c2_sah.json", "w"))
    json.dump({"wf_step": {"traffic_bytes": 1e10}, "_build": {"build_id": "aaaa", "config": "c2"}},
              open(prof / "pmc_traffic_c2_sah.json", "w"))
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    monkeypatch.delenv("RTW_LIB", raising=False)

    class A:
        config, bvh, spp, tuning = "c2", "sah", 0, ""
    assert bench.pmc_valu(A, "wf_step", "aaaa")[0] == entry
    assert bench.pmc_traffic(A, "wf_step", "aaaa")[0] == 10_000_000_000
    e, src = bench.pmc_valu(A, "wf_step", "bbbb")
    assert e is None and "stale" in src
    t, src = bench.pmc_traffic(A, "wf_step", "bbbb")
    assert t is None and "stale" in src
