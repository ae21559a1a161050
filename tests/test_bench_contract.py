"""The committed bench line (profiles/r6_c2_bench.json, written by bench.py on an
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
ROUND = "r6"
BENCH = f"{ROUND}_c2_bench.json"
SUMMARY = f"{ROUND}_c2_timed_summary.txt"


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
    # the work-normalised walk roofline (round 5): device node visits per second against the walk ceiling of
    # the same build (diag/trav_bench.hip -> profiles/walk_ceiling_c2.json)
    w = r["walk"]
    assert w["frac"] is not None and 0 < w["frac"] <= 1 and w["ceiling"] > 0
    ceil = json.load(open(os.path.join(REPO, "profiles", "walk_ceiling_c2.json")))
    assert ceil["build_id"] == d["build_id"] and abs(ceil["ceiling"] - w["ceiling"]) <= 1e-6 * w["ceiling"]
    assert abs(w["frac"] - w["achieved"] / w["ceiling"]) < 1e-3
    c = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in c, k
    assert c["kind"] in ("port", "reference") and c["cores"] >= 1 and c["value"] > 0
    # the reference's 8 threads AND all host cores
    assert c["legs"]["threads_8"]["threads"] == 8 and c["legs"]["threads_all"]["threads"] == c["cores_all"]
    assert c["value"] == max(v["value"] for v in c["legs"].values())


@pytest.mark.parametrize("config", ["c2", "c3", "c4", "c5", "cornell", "cornell_smoke", "simple_light"])
def test_roofline_recomputes_from_profiles(config):
    """Every committed round-6 bench line: VALU and HBM fractions <= 1 and recomputable from
    the PMC passes in profiles/ (taken on the same build: the line's build_id) and its HIP-event launch time."""
    line = os.path.join(REPO, "profiles", f"{ROUND}_{config}_bench.json")
    rc = subprocess.run([sys.executable, os.path.join(REPO, "tools", "roofline_check.py"), line],
                        capture_output=True, text=True)
    assert rc.returncode == 0, rc.stdout + rc.stderr
    d = load(f"{ROUND}_{config}_bench.json")
    r = d["roofline"]
    assert r["bound"] == "valu" and 0 < r["frac"] <= 1 and 0 < r["hbm"]["frac"] <= 1
    assert r["peak"] == 78.643 and "r4_valu_peak" in r["valu"]["peak_source"]
    for kind in ("valu", "traffic"):
        with open(os.path.join(REPO, "profiles", f"pmc_{kind}_{config}_sah.json")) as f:
            assert json.load(f)["_build"]["build_id"] == d["build_id"]


def test_rocprof_summary_agrees_with_bench_events():
    """profiles/r6_c2_timed_summary.txt (rocprofv3 --kernel-trace --stats of the bench
    command) and the bench's HIP-event average of the dominant kernel agree."""
    d = load(BENCH)
    kernel = d["roofline"]["kernel"].split("<")[0]
    lines = open(os.path.join(REPO, "profiles", SUMMARY)).read().splitlines()
    # round 6: the dominant kernel is a family of instantiations (iteration 0 / later iterations); the summary's
    # family line averages the timed region's calls of all of them, as bench.py's HIP events do
    fam = [ln for ln in lines if ln.startswith("dominant family in the timed region:")]
    if fam:
        mean_us = float(fam[0].split("mean ")[1].split()[0])
        assert abs(mean_us / 1e3 - d["roofline"]["avg_launch_ms"]) <= 0.05 * d["roofline"]["avg_launch_ms"]
        assert d["roofline"]["kernels"] and all(k.split("<")[0] == kernel for k in d["roofline"]["kernels"])
        return
    for line in lines:
        if kernel + "<" in line:
            mean_us = float(line.split()[-3])
            assert abs(mean_us / 1e3 - d["roofline"]["avg_launch_ms"]) <= 0.05 * d["roofline"]["avg_launch_ms"]
            return
    raise AssertionError(f"{kernel} not in the rocprof summary")


PMC_CONFIGS = ["c2", "c3", "c4", "c5", "cornell", "cornell_smoke", "simple_light"]


@pytest.mark.parametrize("config", PMC_CONFIGS)
def test_pmc_passes_pair_with_the_bench_lines(config):
    """Every committed PMC pass bench.py derives a roofline from (profiles/pmc_{valu,traffic}_<config>_sah.json)
    was taken on the build of the committed bench line it prices (its _build.build_id), for that config and for
    the whole frame (n_shards 1).  (Whether a pass matches the library being run is bench.py's own check: it
    leaves the fractions null for a pass of another build, test_bench_refuses_a_stale_pmc_pass.)"""
    line = load(f"{ROUND}_{config}_bench.json")
    for kind in ("valu", "traffic"):
        with open(os.path.join(REPO, "profiles", f"pmc_{kind}_{config}_sah.json")) as f:
            d = json.load(f)
        assert d.get("_build", {}).get("build_id") == line["build_id"], (kind, config, d.get("_build"))
        assert d["_build"].get("config") == config
        assert int(d["_build"].get("n_shards") or 1) == 1


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
        config, bvh, spp, tuning, profiles_dir = "c2", "sah", 0, "", str(prof)
    assert bench.pmc_valu(A, "wf_step", "aaaa")[0] == entry
    assert bench.pmc_traffic(A, "wf_step", "aaaa")[0] == 10_000_000_000
    e, src = bench.pmc_valu(A, "wf_step", "bbbb")
    assert e is None and "stale" in src
    t, src = bench.pmc_traffic(A, "wf_step", "bbbb")
    assert t is None and "stale" in src


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    return bench


def _fake_pass(path, build, kind, n_shards=1, rank=0):
    b = {"build_id": build, "config": "c2", "n_shards": n_shards, "rank": rank}
    if kind == "valu":
        e = {"lane_ops": 1e11, "insts_valu": 3e9, "active_inst_valu": 3e9, "thread_cycles_valu": 1e11,
             "kernels": ["wf_step_clds<0u>"], "lane_util": 0.5}
    else:
        e = {"traffic_bytes": 1e10}
    json.dump({"wf_step": e, "_build": b}, open(path, "w"))


def test_bench_prices_a_rank_only_with_its_own_shard_pass(tmp_path, monkeypatch):
    """At N > 1 a rank's launches cover ~1/N of the frame: bench.py prices them only with a PMC pass of
    that rank's shard at that N (profiles/pmc_*_<config>_sah_n<N>_r<R>.json, stamped n_shards / rank), never
    with the whole-frame pass (which would read as frac ~1.5 at N = 8)."""
    bench = _bench_module()
    monkeypatch.delenv("RTW_LIB", raising=False)
    for kind in ("valu", "traffic"):
        _fake_pass(tmp_path / f"pmc_{kind}_c2_sah.json", "aaaa", kind)

    class A:
        config, bvh, spp, tuning, profiles_dir = "c2", "sah", 0, "", str(tmp_path)
    assert bench.pmc_valu(A, "wf_step", "aaaa", 1, 0)[0] is not None
    e, src = bench.pmc_valu(A, "wf_step", "aaaa", 8, 0)
    assert e is None and "no pass of this rank's shard" in src
    t, src = bench.pmc_traffic(A, "wf_step", "aaaa", 8, 0)
    assert t is None and "no pass of this rank's shard" in src
    # a shard pass: used for that (N, R) only
    for kind in ("valu", "traffic"):
        _fake_pass(tmp_path / f"pmc_{kind}_c2_sah_n8_r0.json", "aaaa", kind, 8, 0)
    assert bench.pmc_valu(A, "wf_step", "aaaa", 8, 0)[0]["lane_ops"] == 1e11
    assert bench.pmc_traffic(A, "wf_step", "aaaa", 8, 0)[0] == 10_000_000_000
    assert bench.pmc_valu(A, "wf_step", "aaaa", 8, 1)[0] is None
    assert bench.pmc_valu(A, "wf_step", "aaaa", 4, 0)[0] is None
    # a file whose stamp does not match its name is refused
    _fake_pass(tmp_path / "pmc_valu_c2_sah_n4_r0.json", "aaaa", "valu", 1, 0)
    e, src = bench.pmc_valu(A, "wf_step", "aaaa", 4, 0)
    assert e is None and "not 0/4" in src
    # the single-process multi path runs other kernels: no pass at all
    assert bench.pmc_valu(A, "wf_step", "aaaa", 1, 0, single=True)[0] is None


@pytest.mark.parametrize("world_size", [2])
def test_bench_torchrun_line_never_carries_a_whole_frame_roofline(tmp_path, world_size):
    """bench.py's torchrun flow (--host-backend: no GPU) with a whole-frame PMC pass of the loaded build
    present: the N > 1 line leaves every roofline fraction null (or <= 1) and names why."""
    import socket
    from conftest import load_pkg
    build = load_pkg().lib().rtw_build_id().decode()
    for kind in ("valu", "traffic"):
        _fake_pass(tmp_path / f"pmc_{kind}_c1_sah.json", build, kind)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("RTW_LIB", None)
    rn = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world_size}",
                         "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(REPO, "bench.py"),
                         "--gpus", str(world_size), "--host-backend", "--config", "c1", "--steps", "1", "--warmup", "0",
                         "--no-cpu-baseline", "--profiles-dir", str(tmp_path)],
                        capture_output=True, text=True, timeout=300, cwd=REPO, env=env)
    assert rn.returncode == 0, rn.stderr[-2000:]
    d = json.loads([ln for ln in rn.stdout.splitlines() if ln.startswith("{")][-1])
    r = d["roofline"]
    assert d["n_gpus"] == world_size and d["config"]["shard"]["n_shards"] == world_size
    for frac in (r["frac"], r["hbm"]["frac"]):
        assert frac is None or 0 < frac <= 1
    assert r["valu"]["lane_ops_per_launch"] is None and r["traffic"] is None
    assert "no pass of this rank's shard" in r["valu"]["source"]
    assert "no pass of this rank's shard" in r["hbm"]["source"]


def test_prof_summary_keeps_only_the_timed_region(tmp_path):
    """tools/prof_summary.py: with the bench line, only the last steps x launches_per_step calls of the dominant
    kernel and the calls after the render before them count -- the counted passes before them may run other
    instantiations of the same kernels, so counting calls per name would misplace the region."""
    rows = []
    t = 0

    def call(name, dur):
        nonlocal t
        rows.append((name, t, t + dur))
        t += dur + 10

    call("wf_step<0u, true>(rtw_launch)", 5000)           # counted pass: another instantiation
    call("wf_reduce(rtw_launch, rtw_wf)", 100)
    for dur in (900, 800):                                # SAH counted pass: the dominant kernel, untimed
        call("wf_step_clds2<0u, 768u>(rtw_launch)", dur)
    call("wf_reduce(rtw_launch, rtw_wf)", 100)
    for _ in range(2):                                    # two timed steps, 2 launches each
        call("wf_tile_lists(rtw_launch, rtw_wf)", 5)
        for dur in (1000, 3000):
            call("wf_step_clds2<0u, 768u>(rtw_launch)", dur)
        call("wf_reduce(rtw_launch, rtw_wf)", 100)
    trace = tmp_path / "kt.csv"
    with open(trace, "w") as f:
        f.write("Kernel_Name,Start_Timestamp,End_Timestamp\n")
        for n, a, b in rows:
            f.write(f'"{n}",{a * 1000},{b * 1000}\n')
    line = {"steps": 2, "warmup": 0, "roofline": {"kernel": "wf_step_clds2<0u, 768u>", "launches_per_step": 2,
                                                  "avg_launch_ms": 2.0}}
    bench = tmp_path / "bench.json"
    bench.write_text(json.dumps(line) + "\n")
    rc = subprocess.run([sys.executable, os.path.join(REPO, "tools", "prof_summary.py"), str(trace), "--json", str(bench)],
                        capture_output=True, text=True)
    assert rc.returncode == 0, rc.stderr
    got = {}
    for ln in rc.stdout.splitlines()[1:]:  # kernel (70 columns), calls, total_ms, mean_us, min_us, max_us
        nums = ln[70:].split()
        if not ln.startswith("bench.py") and len(nums) == 5 and nums[0].isdigit():
            got[ln[:70].strip().split("(")[0]] = (int(nums[0]), float(nums[2]))
    assert got["wf_step_clds2<0u, 768u>"] == (4, 2000.0)  # 4 timed calls, mean 2000 us
    assert got["wf_reduce"][0] == 2 and got["wf_tile_lists"][0] == 2
    assert "wf_step<0u, true>" not in got
