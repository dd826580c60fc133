"""bench.py's own multi-rank launcher: `python bench.py --gpus N` starts N rank
processes itself, as the reference's ddp/main.py:46-49 (`mp.spawn(main_worker, nprocs=ngpus)`) does,
instead of silently timing one GPU. CPU only: the rank processes here are a stand-in script."""
import json
import os
import subprocess
import sys
import textwrap
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    sys.path.insert(0, ROOT)
    import bench as b
    return b


def test_rank_envs_are_torchrun_shaped(bench):
    envs = bench.rank_envs(4, 29511, base={"KEEP": "1", "RANK": "9"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    for e in envs:
        assert (e["WORLD_SIZE"], e["LOCAL_WORLD_SIZE"], e["MASTER_ADDR"], e["MASTER_PORT"]) == ("4", "4", "127.0.0.1",
                                                                                                  "29511")
        assert e["KEEP"] == "1"  # the caller's environment travels (HSA_ENABLE_IPC_MODE_LEGACY, OMP_NUM_THREADS ...)


def test_spawn_ranks_propagates_argv_and_env(bench, tmp_path):
    child = tmp_path / "child.py"
    child.write_text(textwrap.dedent(f"""
        import json, os, sys
        keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
        out = {{k: os.environ[k] for k in keys}}
        out["argv"] = sys.argv[1:]
        open(os.path.join({str(tmp_path)!r}, "rank%s.json" % os.environ["RANK"]), "w").write(json.dumps(out))
    """))
    argv = ["--gpus", "3", "--steps", "7", "--opt", "graphs=1"]
    assert bench.spawn_ranks(3, argv, script=str(child), poll_s=0.01) == 0
    got = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(3)]
    assert [g["RANK"] for g in got] == ["0", "1", "2"] and [g["LOCAL_RANK"] for g in got] == ["0", "1", "2"]
    assert {g["WORLD_SIZE"] for g in got} == {"3"} and {g["MASTER_ADDR"] for g in got} == {"127.0.0.1"}
    assert len({g["MASTER_PORT"] for g in got}) == 1  # one rendezvous for the job
    assert all(g["argv"] == argv for g in got)


def test_spawn_ranks_failure_terminates_the_others(bench, tmp_path):
    child = tmp_path / "child.py"
    child.write_text("import os, sys, time\n"
                     "if os.environ['RANK'] == '1':\n    sys.exit(3)\n"
                     "time.sleep(120)\n")
    t0 = time.perf_counter()
    rc = bench.spawn_ranks(3, [], script=str(child), poll_s=0.01)
    assert rc == 3
    assert time.perf_counter() - t0 < 30  # the sleeping ranks were terminated, not waited for


def test_world_size_must_equal_gpus(bench):
    bench.check_world(4, 4)
    with pytest.raises(SystemExit, match="world size 1 != --gpus 8"):
        bench.check_world(1, 8)


def test_bench_refuses_more_gpus_than_visible():
    # no GPU in this container: `--gpus 2` must abort before starting anything, never time one rank
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, timeout=300, env={k: v for k, v in os.environ.items() if k != "RANK"})
    assert r.returncode != 0
    assert "GPU(s) visible" in r.stderr
    assert r.stdout.strip() == ""


def test_visible_gpus_counts_without_hip(bench, tmp_path):
    """the launcher counts GPUs from the environment or the KFD topology, never through HIP."""
    assert bench.visible_gpus({"HIP_VISIBLE_DEVICES": "0,1,2"}) == 3
    assert bench.visible_gpus({"ROCR_VISIBLE_DEVICES": ""}) == 0
    nodes = tmp_path / "nodes"
    for i, simd in enumerate((0, 256, 256)):  # a CPU node and two GPU agents
        d = nodes / str(i)
        d.mkdir(parents=True)
        (d / "properties").write_text(f"cpu_cores_count 0\nsimd_count {simd}\n")
    assert bench.visible_gpus({}, kfd=str(nodes)) == 2
    assert bench.visible_gpus({}, kfd=str(tmp_path / "missing")) is None


def test_traffic_file_selection_by_round_and_session(bench):
    """the newest PMC summary by round and session (r04ad after r04u), named in the line,
    and no traffic figure for a workload the summary did not measure."""
    names = ["profiles/r02_n_conv_traffic.json", "profiles/r04u_conv_traffic.json", "profiles/r04ad_conv_traffic.json",
             "profiles/r03ah_conv_traffic.json", "profiles/r01_s4_conv_traffic.json"]
    assert sorted(names, key=bench.profile_order_key)[-1] == "profiles/r04ad_conv_traffic.json"
    assert sorted(names + ["profiles/r05a_conv_traffic.json"], key=bench.profile_order_key)[-1].endswith("r05a_conv_traffic.json")
    val, src = bench.committed_traffic(256, 32)
    files = sorted([f for f in os.listdir(os.path.join(ROOT, "profiles")) if f.endswith("conv_traffic.json")],
                   key=bench.profile_order_key)
    assert src == os.path.join("profiles", files[-1])
    assert val == round(json.load(open(os.path.join(ROOT, src)))["hbm_bytes_per_call"], 1)
    val32, src32 = bench.committed_traffic(32, 32)
    assert val32 is None and "not this workload" in src32


def test_prof_summary_flops_follow_the_bench_batch(tmp_path):
    """a trace summary's fraction uses its own bench line's batch and size, and no
    fraction is printed without one (a B=256 figure divided by a B=32 trace's conv time read 0.51)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import prof_summary as ps

    line = {"roofline": {"algorithmic_gflop_per_step": 0.0}, "config": {"per_gpu_batch": 32, "image_size": 32}}
    f = tmp_path / "b.json"
    f.write_text(json.dumps(line) + "\n")
    g, _ = ps.bench_gflop(str(f))
    assert abs(g - 852.215 / 8) < 1e-6
    line["config"] = {"per_gpu_batch": 512, "image_size": 224}
    f.write_text(json.dumps(line) + "\n")
    assert abs(ps.bench_gflop(str(f))[0] - 852.215 * 2 * 49) < 1e-3
    line["roofline"]["algorithmic_gflop_per_step"] = 123.0
    f.write_text(json.dumps(line) + "\n")
    assert ps.bench_gflop(str(f))[0] == 123.0
    f.write_text("not json\n")
    assert ps.bench_gflop(str(f))[0] is None


def test_comm_timing_fields(bench):
    """the N>1 line carries comm_exposed_us (tail + weight-gradient join wait) and buckets_us
    (per bucket start / end / duration) from dtc_rn18_comm_timing_result's arrays."""
    bus = [10.0, 60.0, 50.0, 70.0, 95.0, 25.0, 300.0, 310.0, 10.0]
    exu = [12.0, 30.0, 42.0, 1200.0, 5.0]
    exposed, buckets = bench.comm_fields(bus, exu, 5, [32.22, 10.01, 0.57])
    assert {"tail_us", "side_join_us", "total_us", "backward_us", "steps"} <= set(exposed)
    assert exposed["total_us"] == 42.0 and exposed["steps"] == 5
    assert [b["bucket"] for b in buckets] == [0, 1, 2]
    assert buckets[1] == {"bucket": 1, "mb": 10.01, "start_us": 70.0, "end_us": 95.0, "duration_us": 25.0}
    assert bench.comm_fields(bus, exu, 0, [1.0]) == (None, None)
