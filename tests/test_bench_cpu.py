"""bench.py's multi-GPU plumbing on the CPU: per-rank chain arithmetic of the
weak (C2) and strong (C3 / C4 / C5) workloads, the child-rank launcher, and the
refusal of `--gpus N` without N devices."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_c3_divides_one_million_chains_over_the_node():
    # BASELINE.json configs[2]: 1M chains x 1 day sharded over 8 x MI355X
    for world in (1, 2, 4, 8):
        parts = [bench.rank_chains("c3", bench.DEFAULT_CHAINS["c3"], r, world) for r in range(world)]
        assert all(p[1] == 1_048_576 // world for p in parts)
        assert all(p[2] == 1_048_576 and p[3] == "strong" for p in parts)
        assert [p[0] for p in parts] == [r * (1_048_576 // world) for r in range(world)]
    assert bench.rank_chains("c3", 1_048_576, 7, 8)[:2] == (7 * 131_072, 131_072)


@pytest.mark.parametrize("wl,total", [("c4", 16_384), ("c5", 65_536), ("c3", 1_000_003)])
def test_strong_workloads_cover_node_total_once(wl, total):
    for world in (1, 3, 8):
        parts = [bench.rank_chains(wl, total, r, world) for r in range(world)]
        assert sum(p[1] for p in parts) == total
        for (a0, an, _, _), (b0, _, _, _) in zip(parts, parts[1:]):
            assert a0 + an == b0


def test_c2_is_weak_scaled_per_gpu():
    for world in (1, 2, 8):
        parts = [bench.rank_chains("c2", 4096, r, world) for r in range(world)]
        assert all(p[1] == 4096 and p[2] == 4096 * world and p[3] == "weak" for p in parts)
        # distinct global ids: rank r's batch-0 chains start at r * 4096
        assert [p[0] for p in parts] == [4096 * r for r in range(world)]


def test_launch_ranks_starts_n_children_with_rank_env(tmp_path):
    script = tmp_path / "child.py"
    out = tmp_path / "out"
    out.mkdir()
    script.write_text(
        "import json, os, sys\n"
        "keys = ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT')\n"
        f"open(os.path.join({str(out)!r}, os.environ['RANK']), 'w').write(json.dumps({{k: os.environ[k] for k in keys}}))\n"
        "sys.exit(0)\n")
    os.environ["TMH_BENCH_SHARE_GPU"] = "1"   # no device count check (no GPU here)
    try:
        rc = bench.launch_ranks(3, ["--gpus", "3"], script=str(script))
    finally:
        del os.environ["TMH_BENCH_SHARE_GPU"]
    assert rc == 0
    envs = [json.loads((out / str(r)).read_text()) for r in range(3)]
    assert [e["RANK"] for e in envs] == ["0", "1", "2"] == [e["LOCAL_RANK"] for e in envs]
    assert {e["WORLD_SIZE"] for e in envs} == {"3"}
    assert {e["MASTER_ADDR"] for e in envs} == {"127.0.0.1"}
    assert len({e["MASTER_PORT"] for e in envs}) == 1


def test_launch_ranks_reports_a_failed_rank(tmp_path):
    script = tmp_path / "child.py"
    script.write_text("import os, sys, time\n"
                      "if os.environ['RANK'] == '1': sys.exit(7)\n"
                      "time.sleep(30)\n")   # the others are terminated, not waited for
    os.environ["TMH_BENCH_SHARE_GPU"] = "1"
    try:
        rc = bench.launch_ranks(2, [], script=str(script))
    finally:
        del os.environ["TMH_BENCH_SHARE_GPU"]
    assert rc == 7


def test_gpus_2_without_two_devices_exits_nonzero():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "TMH_BENCH_SHARE_GPU")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "needs 2 visible GPUs" in r.stderr


def test_world_size_must_match_gpus():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr


def test_stale_pmc_record_never_reaches_a_bench_line(tmp_path, monkeypatch):
    """profiles/pmc_kernels.json records carry the build stamp of the library they
    were measured with; bench.py uses only records of the current build."""
    import argparse
    from tmhpvsim_amd.build import build_stamp
    key = dict(workload="c2", chains=4096, launch_seconds=86400, precision="fp32", mode="trace", cc="faithful")
    (tmp_path / "profiles").mkdir()
    args = argparse.Namespace(workload="c2", precision="fp32", mode="trace", cc="faithful", compact=0, seconds=86400)
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))

    def write(stamp):
        rec = dict(key, valu_insts_per_launch=1.0, salu_insts_per_launch=1.0, traffic_bytes_per_launch=1.0)
        if stamp is not None:
            rec["build_stamp"] = stamp
        (tmp_path / "profiles" / "pmc_kernels.json").write_text(json.dumps({"records": [rec]}))

    write(None)                     # an unstamped (pre-stamp) record
    assert bench.pmc_record(args, 4096, 86400) is None
    write("0123456789abcdef")       # another build's record
    assert bench.pmc_record(args, 4096, 86400) is None
    write(build_stamp())
    assert bench.pmc_record(args, 4096, 86400)["traffic_bytes_per_launch"] == 1.0


@pytest.mark.parametrize("argv,want", [([], "all"), (["--no-cpu-baseline"], "none"),
                                       (["--workload", "c3"], "none"), (["--precision", "fp64"], "none"),
                                       (["--secondary", "c3,c5"], "c3,c5")])
def test_secondary_lines_default_to_the_full_report_only(monkeypatch, argv, want):
    """The default C2 fp32 run (with its CPU baseline) adds the other configurations'
    lines; quick runs, other workloads and explicit choices do not change."""
    monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
    a = bench.parse()
    assert a.secondary == want
    assert {"c2_fp64", "c3", "c4", "c5"} <= set(bench.SECONDARY)
    proxies = {k for k in bench.SECONDARY if "_proxy" in k}      # one-GPU proxies of the strong-scaled configs
    assert proxies == {"c3_proxy8", "c4_proxy2", "c4_proxy4", "c4_proxy8", "c5_proxy8"}
    for k in proxies:
        argv = bench.SECONDARY[k]
        assert argv[argv.index("--proxy-world") + 1] == k.split("proxy")[1]


def test_secondary_lines_report_a_failed_child(monkeypatch):
    """A secondary configuration that fails reports its error; nothing raises."""
    import argparse

    class R:
        stdout = "not json"

    monkeypatch.setattr(subprocess, "run", lambda *a, **k: R())
    out = bench.secondary_lines(argparse.Namespace(secondary="c3", hw_queues=16, hw_queues_given=False))
    assert list(out) == ["c3"] and "error" in out["c3"]


def test_hw_queues_flag_defaults(monkeypatch):
    """16 hardware queues for C2 / C3; 32 for C4 / C5 (three streams per batch in flight)."""
    for argv, want in (([], 16), (["--workload", "c3"], 16), (["--workload", "c4"], 32),
                       (["--workload", "c5"], 32), (["--workload", "c4", "--hw-queues", "8"], 8)):
        monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
        a = bench.parse()
        assert a.hw_queues == want and a.hw_queues_given == ("--hw-queues" in argv)


def test_valu_busy_weights_the_instruction_classes():
    """The cycle-weighted VALU-busy fraction: class counts x issue cycles, the rest at 4,
    over 1024 SIMDs x 2.4 GHz."""
    rec = {"valu_insts_per_launch": 1000.0, "active_inst_valu": 600.0,
           "valu_mix": {"FMA_F32": 500.0, "TRANS_F32": 100.0, "FMA_F64": 100.0}}
    ms = 1e3 / bench.SIMD_CYCLES_PER_S   # one SIMD-cycle of the whole chip
    b = bench.valu_busy(rec, ms)
    assert b["valu_other_insts_per_launch"] == 300.0
    assert abs(b["valu_cycles_per_launch"] - (500 * 2 + 100 * 8 + 100 * 4 + 300 * 4)) < 1e-9
    assert abs(b["busy_frac_weighted"] - 3400.0) < 1e-6 and "busy_frac_active" not in b
    assert bench.valu_busy({"valu_insts_per_launch": 1.0}, 1.0) == {}


def test_pipeline_defaults_match_bench_schedule():
    """bench.py and the GPU tests of the timed schedule (tests/test_gpu_trace3.py) take the
    schedule from tmhpvsim_amd.pipeline.pipeline_defaults: C2 runs the gated schedule with
    five contexts, two walks in flight and construction four batches ahead; C3 two stats
    contexts; C4 30-day and C5 day windows (C5 compacted), three and five contexts."""
    import sys
    from tmhpvsim_amd.pipeline import pipeline_defaults
    c2 = pipeline_defaults("c2")
    assert (c2.mode, c2.pipeline, c2.walks, c2.build_ahead, c2.window, c2.schedule) == ("trace", 5, 2, 4, 86400, "gated")
    assert not c2.commit_stream and c2.walk_order and c2.queues == "dedicated"
    c3 = pipeline_defaults("c3")
    assert (c3.mode, c3.pipeline, c3.walks) == ("stats", 2, 1)
    c4, c5 = pipeline_defaults("c4"), pipeline_defaults("c5")
    assert c4.window == 30 * 86400 and c5.window == 86400 and c5.compact and not c4.compact
    assert (c4.pipeline, c5.pipeline) == (3, 5)
    import bench
    old = sys.argv
    try:
        sys.argv = ["bench.py"]
        a = bench.parse()
    finally:
        sys.argv = old
    assert a.cfg == c2


def test_build_stamp_ignores_comments():
    """The PMC records' build stamp hashes the code the compiler sees: comment and
    blank-line edits keep it, code edits change it."""
    from tmhpvsim_amd.build import _code_only
    a = 'int f(int x) { return x + 1; }  // one\n/* block\n comment */\n'
    b = 'int f(int x) { return x + 1; }\n\n// two\n'
    c = 'int f(int x) { return x + 2; }\n'
    d = 'const char* s = "// not a comment";\n'
    assert _code_only(a) == _code_only(b) != _code_only(c)
    assert "// not a comment" in _code_only(d)


def test_walk_lanes_defaults(monkeypatch):
    """8 walk lanes per chain for C3 / C4 batches above 8,192 chains, 16 for C5, the
    library's batch-size default (0) otherwise (C2, and the small C4 shards of N = 8)."""
    for argv, want in (([], 0), (["--workload", "c3"], 8), (["--workload", "c4"], 8),
                       (["--workload", "c4", "--proxy-world", "8"], 0), (["--workload", "c5"], 16),
                       (["--workload", "c3", "--proxy-world", "8"], 8), (["--workload", "c4", "--walk-lanes", "4"], 4)):
        monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
        assert bench.parse().walk_lanes == want, argv
