"""The N>1 bench path on CPU: bench.py's own launcher (`--gpus 2` with no
WORLD_SIZE starts torch.distributed.run as a child) runs two gloo ranks that
each checksum their own shard through the library's host engine, time it in
the same timed region (barrier + sync both sides, max over ranks) and report
per rank; the shard assignment gives every rank a disjoint buffer range with
no data-path collective. CPU only."""
import json
import os
import socket
import subprocess
import sys
import time

import pytest
import torch.multiprocessing as mp

import bench


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    delay = 0.002 * (rank + 1)          # rank 1 is the slow one
    step = lambda: time.sleep(delay)    # noqa: E731
    elapsed, per_step, _, _ = bench.timed_region(step, steps=10, warmup=2, sync=lambda: None, dist=dist)
    q.put((rank, elapsed, per_step))
    dist.destroy_process_group()


def test_timed_region_max_over_ranks_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # Every rank reports the same (max) time, and it is the slow rank's.
    assert res[0][1] == res[1][1] and res[0][2] == res[1][2]
    assert res[0][1] >= 10 * 0.004
    # Whole-job value counts every rank's bytes over that time.
    v = bench.aggregate_gibps(1 << 30, 10, world, res[0][1])
    assert v == pytest.approx(2 * 10 / res[0][1])


@pytest.mark.parametrize("config", ["c2", "c3", "c4", "c5"])
def test_shards_are_disjoint(config):
    cfg = bench.CONFIGS[config]
    slots = cfg["count"] * cfg.get("nseg", 1)
    ranges = [(bench.shard_seed_base(r, slots), bench.shard_seed_base(r, slots) + slots) for r in range(8)]
    for a, b in zip(ranges, ranges[1:]):
        assert a[1] == b[0]  # contiguous, non-overlapping global buffer ids per rank


def test_bench_defaults():
    a = bench.parse([])
    assert a.gpus == 1 and a.config == "c2" and a.steps > 0 and a.warmup > 0
    # Every N runs the same per-GPU workload (C2 per GPU, weak scaling), so the
    # driver's 1/2/4/8-GPU lines compare like with like;
    # the 8-GPU config's shard stays available as --config c4.
    for n in (2, 4, 8):
        assert bench.parse(["--gpus", str(n)]).config == "c2"
    assert bench.CONFIGS["c4"]["count"] * 8 == 256 * 1024
    # tuning arguments default to the product's choices (0 = not set)
    assert a.rows == 0 and a.msg_rows == 0 and a.lanes == 0
    assert bench.parse(["--rows", "4", "--msg-rows", "2"]).rows == 4


def _run_bench(*argv, timeout=240):
    if "--cpu-seconds" not in argv:  # rank 0's CPU baseline leg, kept short on CPU
        argv = (*argv, "--cpu-seconds", "0.2")
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    return subprocess.run([sys.executable, os.path.join(bench.REPO, "bench.py"), *argv], capture_output=True,
                          text=True, timeout=timeout, env=env, cwd=bench.REPO)


def test_launcher_two_ranks_cpu(oracle):
    """`bench.py --gpus 2` (no WORLD_SIZE) launches 2 ranks itself; the line
    says n_gpus 2, and each rank checksummed ITS shard (global ids r*64..)."""
    from photonlibos_amd import datagen
    r = _run_bench("--gpus", "2", "--cpu-rehearsal", "--steps", "3", "--warmup", "1")
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, r.stdout  # rank 0 prints ONE line
    res = json.loads(line[0])
    assert res["n_gpus"] == 2 and res["steps"] == 3 and res["warmup"] == 1 and res["scaling"] == "weak"
    assert [p["rank"] for p in res["per_rank"]] == [0, 1]
    for p in res["per_rank"]:
        want = oracle.crc32c(datagen.stream_bytes(bench.shard_seed_base(p["rank"], 64), 65536))
        assert p["first_crc"] == want
        assert len(p["launch_ms"]["first5"]) == 3
    # whole-job value = both ranks' bytes over the slowest rank's wall time
    slow = max(p["wall_s"] for p in res["per_rank"])
    assert res["value"] == pytest.approx(2 * 3 * 64 * 65536 / slow / (1 << 30), rel=0.05)


def test_scaling_lines_name_one_workload():
    """The N = 1 and N = 2 lines of a scaling sweep (plain `--gpus 1`, and
    `--gpus 2` through bench.py's own launcher) name the same per-GPU
    workload, the metric's C2 config."""
    lines = {}
    for n in (1, 2):
        r = _run_bench("--gpus", str(n), "--cpu-rehearsal", "--steps", "2", "--warmup", "1")
        assert r.returncode == 0, r.stderr[-2000:]
        res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
        assert res["n_gpus"] == n and res["scaling"] == "weak"
        lines[n] = res["config"]
    assert lines[1]["workload"] == lines[2]["workload"] == bench.CONFIGS["c2"]["workload"]
    assert lines[1]["config"] == lines[2]["config"] == "c2"


def test_launcher_refuses_missing_gpus():
    """--gpus 2 with fewer visible GPUs (none here) exits non-zero instead of
    silently measuring one GPU."""
    r = _run_bench("--gpus", "2", "--steps", "1", "--warmup", "0", timeout=120)
    assert r.returncode == 2 and "visible" in r.stderr


def test_world_size_must_match_gpus():
    env_args = ("--gpus", "4", "--cpu-rehearsal", "--steps", "1", "--warmup", "0")
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(bench.REPO, "bench.py"), *env_args], capture_output=True,
                       text=True, timeout=120, env=env, cwd=bench.REPO)
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr


def test_two_rank_line_carries_c4_leg():
    """the C2 line (value, config.workload = C2) also carries
    a `config_c4` sub-record for BASELINE configs[3] timed in
    the same ranks after the C2 leg; each rank checksummed ITS part of the C4
    batch (global ids r*32768..)."""
    from photonlibos_amd import datagen
    r = _run_bench("--gpus", "2", "--cpu-rehearsal", "--steps", "2", "--warmup", "1")
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert res["config"]["workload"] == bench.CONFIGS["c2"]["workload"]
    c4 = res["config_c4"]
    assert c4["workload"] == bench.CONFIGS["c4"]["workload"] and c4["config"] == "c4"
    assert c4["buffers_total"] == 2 * 32768 and c4["steps"] == 2 and c4["warmup"] == 1
    assert [p["rank"] for p in c4["per_rank"]] == [0, 1]
    for p in c4["per_rank"]:
        want = oracle_crc(datagen.stream_bytes(bench.shard_seed_base(p["rank"], 32768), 1 << 20))
        assert p["first_crc"] == want
    # the C4 leg's value is its own bytes over its own slowest-rank time
    slow = max(p["wall_s"] for p in c4["per_rank"])
    assert c4["value"] == pytest.approx(2 * 2 * 4 * (1 << 20) / slow / (1 << 30), rel=0.05)
    # the one-GPU line carries it too (the driver's 1/2/4/8 sweep measures
    # C4 weak scaling), and --no-c4-leg drops it
    r1 = _run_bench("--gpus", "1", "--cpu-rehearsal", "--steps", "1", "--warmup", "0")
    one = json.loads([ln for ln in r1.stdout.splitlines() if ln.startswith("{")][0])
    assert one["config_c4"]["buffers_total"] == 32768 and one["config"]["config"] == "c2"
    r0 = _run_bench("--gpus", "2", "--cpu-rehearsal", "--steps", "1", "--warmup", "0", "--no-c4-leg")
    assert "config_c4" not in json.loads([ln for ln in r0.stdout.splitlines() if ln.startswith("{")][0])


def oracle_crc(data):
    from tests import _oracle
    return _oracle.crc32c(data)


def test_two_rank_line_carries_cpu_baseline_and_traffic():
    """an N>1 line carries what `north_star` asks for "in the
    same run" -- Photon's CPU checksum timed on the host cores (rank 0, after
    the timed legs, the other ranks idle in a barrier) and the HBM traffic of
    the config's kernel with its source and scope (rank 0's device). Before
    round 6 both were gated on world == 1."""
    r = _run_bench("--gpus", "2", "--cpu-rehearsal", "--steps", "2", "--warmup", "1", "--cpu-seconds", "0.3")
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    base = res["cpu_baseline"]
    assert base["value"] > 0 and base["unit"] == "GiB/s" and base["cores"] >= 1
    assert base["kind"] in ("reference", "port") and "rank 0 of 2" in base["measured_by"]
    roof = res["roofline"]
    assert roof["traffic_source"] and "rank 0" in roof["traffic_scope"]
    # the committed C2 profile is what a rehearsal (no rocprofv3 child) reads
    assert roof["traffic"] == bench.load_traffic(None, "c2")
    # --no-cpu-baseline drops the leg at any N
    r0 = _run_bench("--gpus", "2", "--cpu-rehearsal", "--steps", "1", "--warmup", "0", "--no-cpu-baseline",
                    "--no-c4-leg")
    assert "cpu_baseline" not in json.loads([ln for ln in r0.stdout.splitlines() if ln.startswith("{")][0])


def test_pmc_child_env_leaves_the_rendezvous(monkeypatch):
    """The live FETCH_SIZE child of an N>1 rank must not join the job's
    rendezvous: live_traffic strips the torch.distributed.run variables and
    pins the child to the rank's device."""
    seen = {}

    def fake_run(cmd, **kw):
        seen["cmd"], seen["env"] = cmd, kw["env"]
        raise subprocess.TimeoutExpired(cmd, 1)
    monkeypatch.setattr(bench.shutil, "which", lambda _: sys.executable)
    monkeypatch.setattr(bench.subprocess, "run", fake_run)
    monkeypatch.setenv("WORLD_SIZE", "8")
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("LOCAL_RANK", "0")
    monkeypatch.setenv("MASTER_PORT", "29500")
    assert bench.live_traffic("c2", device=3) is None
    assert not {"WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"} & set(seen["env"])
    assert seen["cmd"][-2:] == ["--device", "3"] and "--pmc-child" in seen["cmd"]
