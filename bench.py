#!/usr/bin/env python3
"""Benchmark of the north-star path: CRC32C over device-resident buffers on
MI355X through the C-ABI engine (libphoton_checksum.so).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5|...]

One "step" = one pass of the hot path over one batch (BASELINE.json configs):
  c2 (the default at EVERY N, configs[1]): 65,536 x 64 KiB random buffers,
      device-resident, per GPU (weak scaling: N GPUs checksum N such batches,
      so the driver's 1/2/4/8-GPU lines compare like with like)
  c4 (configs[3]): 32,768 x 1 MiB per GPU = the 256 Ki x 1 MiB batch sharded
      over 8 GPUs (`--config c4 --gpus 8`); at every --gpus N the C2 line
      also carries a `config_c4` sub-record: the same ranks time their C4
      shard right after the C2 leg (so the driver's 1/2/4/8-GPU sweep also
      measures configs[3], weak-scaling, as SURVEY §8(d) asks; `value` stays
      C2's)
  c3: 1,048,576 x 4 KiB        c5: 65,536 messages x 8 non-contiguous 8 KiB
      segments, per-segment CRC + crc32c_combine fold (BASELINE.json configs[4])
  c5_chain: the C5 shape, one CRC per message chained through the seed
      (Crc32Hasher::extend_hash, rpc/serialize.h:244-251), no segment CRCs
  c2_crc64: the C2 shape with CRC-64/ECMA (next row f2)
  c3_crc64: the C3 shape with CRC-64/ECMA
  --h2d / --rpc-batch / --rpc-latency / --file-records: host-memory rates
      for DESIGN.md, never `value`; --extend: one long device buffer (the
      reference's perf shape) and the routed drop-in's costs, also DESIGN.md.

Multi-GPU: one process per GPU. The driver launches
`python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`;
a plain `python bench.py --gpus N` (no WORLD_SIZE in the environment) starts
that launcher itself as a child process, before anything touches the GPU,
and exits with its status. Every rank checksums its own independent shard
(no data-path collective; gloo carries only the timing barrier, the
max-over-ranks and the per-rank report). Rank 0 prints one JSON line.
Fewer visible GPUs than --gpus is an error (exit 2) unless --share-gpus
(a rehearsal: ranks share the visible GPUs round-robin, marked in the line).
--cpu-rehearsal runs the same launcher / timed region / report with a host
step (this library's crc32c() drop-in) for the CPU tests.
"""
import argparse
import json
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

ck = None  # photonlibos_amd.checksum, imported once this process is a rank (after the launcher decision)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec, MI355X_MICROARCH.md "Chip-level parameters"
GIB = float(1 << 30)
METRIC = "GiB/s CRC32C over device-resident buffers; % of HBM-read roofline"

CONFIGS = {
    "c2": dict(kind="strided", nbytes=65536, count=65536,
               workload="C2: 65536 x 64 KiB random buffers, device-resident, per GPU"),
    "c3": dict(kind="strided", nbytes=4096, count=1 << 20,
               workload="C3: 1048576 x 4 KiB RPC-payload buffers, device-resident, per GPU"),
    "c4": dict(kind="strided", nbytes=1 << 20, count=32768,
               workload="C4 shard: 32768 x 1 MiB buffers per GPU (256K x 1 MiB over 8 GPUs, no collective)"),
    "c5": dict(kind="msg", nbytes=8192, count=65536, nseg=8, seg_out=True,
               workload="C5: 65536 messages x 8 non-contiguous 8 KiB segments, per-segment CRC + "
                        "crc32c_combine fold per message (every segment's CRC and every message's CRC written)"),
    "c5_chain": dict(kind="msg", nbytes=8192, count=65536, nseg=8, seg_out=False,
                     workload="C5 shape, per-message CRC only (Crc32Hasher: crc32c_extend chained over the "
                              "segments through the seed)"),
    "c2_crc64": dict(kind="strided64", nbytes=65536, count=65536,
                     workload="C2 shape, CRC-64/ECMA (next row): 65536 x 64 KiB, device-resident, per GPU"),
    "c3_crc64": dict(kind="strided64", nbytes=4096, count=1 << 20,
                     workload="C3 shape, CRC-64/ECMA (next row): 1048576 x 4 KiB, device-resident, per GPU"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=25)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS),
                    help="default c2 per GPU at every --gpus N (one workload for the whole scaling sweep)")
    ap.add_argument("--share-gpus", action="store_true",
                    help="rehearsal: allow more ranks than visible GPUs (round-robin); marked in the output")
    ap.add_argument("--cpu-rehearsal", action="store_true",
                    help="no GPU: the same launcher and report with a host crc32c() step (CPU tests)")
    ap.add_argument("--h2d", action="store_true", help="host-memory end-to-end rate (for DESIGN.md)")
    ap.add_argument("--h2d-devices", type=int, default=1,
                    help="with --h2d: shard the host batch over this many devices of ONE process (0 = all)")
    ap.add_argument("--file-records", action="store_true", help="file records through the pread pipeline (DESIGN.md)")
    ap.add_argument("--rpc-batch", action="store_true", help="CheckedMessage batch over pinned host payloads (DESIGN.md)")
    ap.add_argument("--rpc-latency", action="store_true", help="submit+wait latency of small CheckedMessage batches")
    ap.add_argument("--extend", action="store_true",
                    help="one long device buffer at base+1 (1 GiB rate, 128 KiB latency, routed drop-in cost)")
    ap.add_argument("--lanes", type=int, default=0, help="lanes per buffer override (0 = auto)")
    ap.add_argument("--msg-rows", type=int, default=0, help="message kernel rows per step (tuning; 0 = default)")
    ap.add_argument("--rows", type=int, default=0, help="batch kernel rows per step (tuning; 0 = by lane count)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-live-pmc", action="store_true",
                    help="do not run the rocprofv3 FETCH_SIZE child pass; read profiles/pmc_<config>.json instead")
    ap.add_argument("--no-shape64", action="store_true", help="skip the one-wavefront-per-buffer (G=64) side line")
    ap.add_argument("--no-c4-leg", action="store_true",
                    help="skip the C4 (BASELINE configs[3]) shard leg timed after the C2 leg")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--device", type=int, default=None, help=argparse.SUPPRESS)
    ap.add_argument("--traffic-json", default=None,
                    help="PMC summary (profiles/*.json) giving HBM bytes per launch (fallback when no live pass)")
    return ap.parse_args(argv)


# ------------------------------------------------------------------ launcher

def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launcher_cmd(args, argv, port):
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def launch_ranks(args, argv):
    """Start one rank process per GPU (torch.distributed.run as a CHILD; this
    process never touches the GPU: torch.cuda.device_count() does not
    initialise it on this image) and return the launcher's exit status."""
    if not args.cpu_rehearsal:
        visible = torch.cuda.device_count()
        if visible < args.gpus and not args.share_gpus:
            print(f"bench.py: --gpus {args.gpus} but only {visible} GPU(s) visible "
                  "(--share-gpus runs a rehearsal with ranks sharing them)", file=sys.stderr)
            return 2
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(launcher_cmd(args, argv, free_port()), env=env)


# -------------------------------------------------------------- timed region

def shard_seed_base(rank, count):
    """Rank r checksums buffers with global ids [r*count, (r+1)*count):
    splitmix streams 0x5EED0001 + global id (disjoint shards, no collective)."""
    return 0x5EED0001 + rank * count


def timed_region(step, steps, warmup, sync, dist=None, on_step=None):
    """Run `warmup` untimed steps, then exactly `steps` steps bracketed by a
    barrier + device sync on both sides. Returns (max over ranks of the wall
    time, max over ranks of the mean per-launch ms from `on_step`, this rank's
    wall time, this rank's per-launch ms list)."""
    for _ in range(warmup):
        step()
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    marks = []
    t0 = time.perf_counter()
    for s in range(steps):
        if on_step:
            marks.append(on_step(s, step))
        else:
            step()
    sync()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        dist.barrier()
    launch_ms = [m() for m in marks] if marks else [elapsed / steps * 1e3] * steps
    per_step_ms = float(np.mean(launch_ms))
    local = (elapsed, launch_ms)
    if dist is not None:
        t = torch.tensor([elapsed, per_step_ms], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, per_step_ms = float(t[0]), float(t[1])
    return elapsed, per_step_ms, local[0], local[1]


def gather_ranks(dist, rec):
    """Every rank's small report dict, in rank order (gloo all_gather_object)."""
    if dist is None:
        return [rec]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, rec)
    return out


def aggregate_gibps(bytes_per_step_per_rank, steps, world, elapsed):
    """Whole-job throughput: every rank's bytes over the slowest rank's time."""
    return bytes_per_step_per_rank * steps * world / elapsed / GIB


def launch_summary(ms):
    a = np.asarray(ms, dtype=np.float64)
    return {"first5": [round(float(x), 4) for x in a[:5]], "mean": round(float(a.mean()), 4),
            "median": round(float(np.median(a)), 4), "min": round(float(a.min()), 4), "max": round(float(a.max()), 4)}


# ------------------------------------------------------------------ workload

class Workload:
    """Device-resident synthetic batch for one config on the current device."""

    def __init__(self, cfg, rank, stream):
        self.cfg = cfg
        self.stream = stream
        n, cnt = cfg["nbytes"], cfg["count"]
        slots = cnt if cfg["kind"] in ("strided", "strided64") else cnt * cfg["nseg"]
        seed_base = shard_seed_base(rank, slots)
        self.payload = torch.empty(n * slots, dtype=torch.uint8, device="cuda")
        ck.fill_splitmix(self.payload, n, n, slots, seed_base, stream=stream)
        self.bytes_per_step = n * slots
        if cfg["kind"] == "strided":
            self.out = torch.zeros(cnt, dtype=torch.int32, device="cuda")
        elif cfg["kind"] == "strided64":
            self.out = torch.zeros(cnt, dtype=torch.int64, device="cuda")
        else:
            nseg = cfg["nseg"]
            # C5 layout: message m's segment j lives at pool slot perm[m*nseg + j].
            rng = np.random.default_rng(0x5EED0005 + rank)
            perm = rng.permutation(slots).astype(np.uint64)
            iov = np.empty((slots, 2), np.uint64)
            iov[:, 0] = np.uint64(self.payload.data_ptr()) + perm * np.uint64(n)
            iov[:, 1] = n
            self.iov = torch.from_numpy(iov.view(np.int64)).cuda()
            self.start = torch.from_numpy(np.arange(0, slots + 1, nseg, dtype=np.uint64).view(np.int64)).cuda()
            self.seg_out = torch.zeros(slots, dtype=torch.int32, device="cuda")
            self.out = torch.zeros(cnt, dtype=torch.int32, device="cuda")

    def step(self):
        c = self.cfg
        if c["kind"] == "strided":
            ck.batch_strided(self.payload, c["nbytes"], c["nbytes"], c["count"], self.out, stream=self.stream)
        elif c["kind"] == "strided64":
            ck.batch64_strided(self.payload, c["nbytes"], c["nbytes"], c["count"], self.out, stream=self.stream)
        else:
            ck.batch_msg_n(self.iov, self.start, c["count"], c["count"] * c["nseg"],
                           self.seg_out if c.get("seg_out") else None, self.out, stream=self.stream)

    def self_check(self):
        """Spot-check the LAST timed step's results against the product's own
        host engine (crc32c_hw / crc32c_extend / crc64ecma_sw), not the oracle."""
        c = self.cfg
        n = c["nbytes"]
        if c["kind"] == "strided64":
            out = self.out.cpu().numpy().view(np.uint64)
            for i in (0, c["count"] - 1):
                host = self.payload[i * n:(i + 1) * n].cpu().numpy().tobytes()
                if ck.crc64ecma_sw(host) != int(out[i]):
                    return False
            return True
        out = self.out.cpu().numpy().view(np.uint32)
        if c["kind"] == "strided":
            for i in (0, 1, c["count"] // 2, c["count"] - 1):
                host = self.payload[i * n:(i + 1) * n].cpu().numpy().tobytes()
                if ck.crc32c_hw(host) != out[i]:
                    return False
            return True
        iov = self.iov.cpu().numpy().view(np.uint64)
        seg = self.seg_out.cpu().numpy().view(np.uint32)
        base = self.payload.data_ptr()
        for m in (0, c["count"] - 1):
            acc = 0
            for j in range(c["nseg"]):
                off = int(iov[m * c["nseg"] + j, 0]) - base
                data = self.payload[off:off + n].cpu().numpy().tobytes()
                if c.get("seg_out") and ck.crc32c_hw(data) != seg[m * c["nseg"] + j]:
                    return False
                acc = ck.crc32c_extend(data, acc)
            if acc != out[m]:
                return False
        return True


# --------------------------------------------------------------- CPU baseline

def usable_cores():
    """Cores this process may run on: the affinity mask, capped by a cgroup CPU
    quota when one is set (a GPU box grants each GPU's job a CPU share while
    nproc / the affinity mask show the whole machine)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()
            if q != "max":
                quota = float(q) / float(period)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = float(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                period = float(f.read())
            if q > 0:
                quota = q / period
        except (OSError, ValueError):
            pass
    used = aff if quota is None else max(1, min(aff, int(quota)))
    return used, {"affinity_cpus": aff, "cgroup_cpu_quota": quota}


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            return [ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")][0]
    except Exception:
        return ""


def _run_harness(cmd, nbuf, n, threads, seconds):
    r = subprocess.run(cmd + [str(nbuf), str(n), str(threads), str(seconds)], capture_output=True, text=True,
                       timeout=seconds * 4 + 120)
    if r.returncode != 0:
        return None
    return json.loads(r.stdout.strip().splitlines()[-1])


def cpu_baseline(cfg, seconds):
    """Photon's own CPU checksum (reference crc.cpp compiled unmodified into
    oracle/_ref/ref_harness) on this host, over a bounded 256 MiB sample of the
    same workload, on 1 thread and on every usable core (persistent pinned
    thread pool, tests/cpp/spin_pool.h); the oracle's C port as fallback."""
    n = cfg["nbytes"]
    nbuf = max(1, (256 << 20) // n)
    cores, cinfo = usable_cores()
    harness = os.path.join(REPO, "oracle", "_ref", "ref_harness")
    sample = f"{nbuf} x {n} B random host buffers (256 MiB, stream 0x5EED0001+i), best pass"
    if os.path.exists(harness):
        allc = _run_harness([harness, "bench"], nbuf, n, cores, seconds)
        one = _run_harness([harness, "bench"], nbuf, n, 1, seconds / 2)
        if allc is not None:
            model = cpu_model()
            return {"value": round(allc["gib_per_s"], 3), "unit": "GiB/s", "cores": cores, "kind": "reference",
                    "sample": sample + f"; Photon crc32c() auto-dispatch (crc.cpp:339-358) on {cores} pinned "
                    "threads" + (f" of {model}" if model else ""),
                    "median_pass_gib_per_s": round(allc["gib_per_s_median"], 3),
                    "single_thread": round(one["gib_per_s"], 3) if one else None, **cinfo}
    # Fallback: the oracle's C restatement (slicing-by-8), one thread.
    from tests import _oracle
    from photonlibos_amd import datagen
    bufs = [datagen.stream_bytes(0x5EED0001 + i, n).tobytes() for i in range(min(nbuf, 256))]
    t0, done = time.perf_counter(), 0
    while time.perf_counter() - t0 < seconds:
        for b in bufs:
            _oracle.crc32c(b)
        done += len(bufs) * n
    return {"value": round(done / (time.perf_counter() - t0) / GIB, 3), "unit": "GiB/s", "cores": 1,
            "kind": "port", "sample": f"{len(bufs)} x {n} B, oracle slicing-by-8, 1 thread"}


def cpu_reference_c1(seconds):
    """Config C1 (1024 x 4 KiB, the reference's CPU-runnable case, cache-
    resident) with Photon's own crc32c() and this library's drop-in, on 1
    thread and on every usable core. Empty when the reference build is absent."""
    harness = os.path.join(REPO, "oracle", "_ref", "ref_harness")
    if not os.path.exists(harness):
        return {}
    dropin = os.path.join(REPO, "tests", "cpp", "bin", "host_bench")
    cores, _ = usable_cores()
    out = {}
    for threads in sorted({1, cores}):
        for key, cmd in ((f"threads_{threads}", [harness, "bench"]), (f"dropin_threads_{threads}", [dropin])):
            if os.path.exists(cmd[0]):
                r = _run_harness(cmd, 1024, 4096, threads, seconds)
                if r is not None:
                    out[key] = round(r["gib_per_s"], 3)
    return {"unit": "GiB/s", "workload": "C1: 1024 x 4 KiB random buffers (cache-resident), Photon crc32c(); "
            "dropin_*: this library's crc32c() drop-in on the same buffers; persistent pinned thread pool",
            **out} if out else {}


# ------------------------------------------------------------- HBM traffic

def load_traffic(path, config):
    if path is None:
        path = os.path.join(REPO, "profiles", f"pmc_{config}.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    v = d.get("hbm_bytes_per_launch")
    return int(v) if v else None


def live_traffic(config, device=0, timeout=150):
    """HBM read bytes per launch of the config's main kernel, measured now: a
    child `rocprofv3 --pmc FETCH_SIZE` pass (counters only, no tracing) over
    `bench.py --pmc-child` (3 launches of the same workload), FETCH_SIZE KiB
    x 1024 x 2 (gfx950 counts half the bytes of wide coalesced reads,
    MI355X_MICROARCH.md HBM section). None if rocprofv3 is unavailable."""
    import csv
    import glob
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as d:
        cmd = [prof, "--pmc", "FETCH_SIZE", "--output-format", "csv", "-d", d, "-o", "pmc", "--",
               sys.executable, os.path.abspath(__file__), "--config", config, "--steps", "3", "--warmup", "1",
               "--pmc-child"]
        # The child is a fresh 1-process run on this rank's device: drop the
        # torch.distributed.run variables so it does not join the job's
        # rendezvous, and pin it to the device this rank timed.
        env = {k: v for k, v in os.environ.items()
               if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                            "ROLE_WORLD_SIZE", "GROUP_WORLD_SIZE", "TORCHELASTIC_RUN_ID", "MASTER_PORT")}
        try:
            r = subprocess.run(cmd + ["--device", str(device)], capture_output=True, text=True, timeout=timeout,
                               cwd=d, env=env)
        except subprocess.TimeoutExpired:
            return None
        if r.returncode != 0:
            return None
        per = {}
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    if row.get("Counter_Name") == "FETCH_SIZE":
                        per.setdefault(row["Kernel_Name"], []).append(float(row["Counter_Value"]))
    if not per:
        return None
    name = max(per, key=lambda k: float(np.mean(per[k])))
    return {"bytes": int(round(float(np.mean(per[name])) * 1024 * 2)), "kernel": name, "launches": len(per[name])}


def rank0_tail(args, cfg, rank, world, dist, gpu=True, device=0):
    """What `north_star` asks for "in the same run" beside the throughput, at
    EVERY N: after the last timed leg and its barrier, rank 0 (a) takes live
    FETCH_SIZE of the config's kernel on its own device in a child rocprofv3
    process (a subprocess, never an exec of this GPU-initialised process) and
    (b) times Photon's own CPU checksum (crc.cpp:339-358) on its host cores,
    while the other ranks wait in a barrier, so the GPU ranks are idle and
    the timed legs are untouched. The traffic is per launch of ONE rank's
    shard (each rank runs the same per-GPU workload). Returns the fields for
    the line; every rank returns after the barrier."""
    tail = {"traffic": None, "traffic_source": None,
            "traffic_scope": f"per launch on rank 0's device (device {device}); every rank runs the same "
                             "per-GPU workload" if world > 1 else "per launch"}
    if rank == 0:
        if gpu and not args.no_live_pmc:
            lt = live_traffic(args.config, device)
            if lt is not None:
                tail["traffic"] = lt["bytes"]
                tail["traffic_source"] = (f"live rocprofv3 --pmc FETCH_SIZE x1024x2, {lt['launches']} launches, "
                                          "child process after the timed legs")
        if tail["traffic"] is None:
            tail["traffic"] = load_traffic(args.traffic_json, args.config)
            tail["traffic_source"] = (f"committed, not this run: profiles/pmc_{args.config}.json (an earlier "
                                      "rocprofv3 --pmc FETCH_SIZE pass of this config on one GPU)"
                                      if tail["traffic"] else "none: no live pass and no committed profile")
        if not args.no_cpu_baseline:
            base = cpu_baseline(cfg, args.cpu_seconds)
            base["measured_by"] = (f"rank 0 of {world}, after the timed legs, other ranks idle in a barrier"
                                   if world > 1 else "the bench process, after the timed legs")
            tail["cpu_baseline"] = base
            c1 = cpu_reference_c1(min(2.0, args.cpu_seconds))
            if c1:
                tail["cpu_reference_c1"] = c1
    if dist is not None:
        dist.barrier()
    return tail


# ------------------------------------------------------------- host-memory modes

def run_h2d(args, stream):
    """Host-memory end-to-end rate for the c2 batch (pinned host -> CRCs on host)."""
    cfg = CONFIGS["c2"]
    n, cnt = cfg["nbytes"], cfg["count"]
    dev = torch.empty(n * cnt, dtype=torch.uint8, device="cuda")
    ck.fill_splitmix(dev, n, n, cnt, shard_seed_base(0, cnt), stream=stream)
    host = torch.empty(n * cnt, dtype=torch.uint8, pin_memory=True)
    host.copy_(dev)
    del dev
    torch.cuda.synchronize()
    out = torch.zeros(cnt, dtype=torch.int32, pin_memory=True)
    ndev = args.h2d_devices
    if ndev == 1:
        step = lambda: ck.host_batch_strided(host, n, n, cnt, out)  # noqa: E731
    else:
        step = lambda: ck.host_batch_strided_multi(host, n, n, cnt, out, ndev=ndev)  # noqa: E731
    used = torch.cuda.device_count() if ndev <= 0 else min(ndev, torch.cuda.device_count())
    steps = max(2, min(args.steps, 10))
    elapsed, _, _, _ = timed_region(step, steps, 2, torch.cuda.synchronize)
    ok = ck.crc32c_hw(host[:n].numpy().tobytes()) == int(out[0].item()) & 0xFFFFFFFF
    print(json.dumps({"metric": "GiB/s CRC32C host-resident (pinned) end to end: H2D + kernel + D2H",
                      "value": round(n * cnt * steps / elapsed / GIB, 3), "unit": "GiB/s", "n_gpus": used,
                      "steps": steps, "ms_per_step": round(elapsed / steps * 1e3, 3), "self_check": ok,
                      "config": {"workload": cfg["workload"].replace("device-resident", "pinned host memory")}}))


def run_rpc_batch(args, stream):
    """§8(f) row 1: CheckedMessage validation batched over RPC payloads held in
    pinned host memory (the pinned IOAlloc pool), C5 shape: 65536 messages x 8
    non-contiguous 8 KiB segments. One step = submit + wait of the whole batch
    (kernels reading descriptors and payload in place over the host link and
    writing the verdicts to pinned memory). Reported in DESIGN.md, never as `value`."""
    from photonlibos_amd.checked import MessageBatch, PinnedAlloc
    cfg = CONFIGS["c5"]
    n, cnt, nseg = cfg["nbytes"], cfg["count"], cfg["nseg"]
    slots = cnt * nseg
    alloc = PinnedAlloc()
    region = 64 << 20  # receive-buffer regions from the IOAlloc pool
    per_region = region // n
    regions = [alloc.alloc(region) for _ in range((slots + per_region - 1) // per_region)]
    for r, a in enumerate(regions):
        ck.fill_splitmix(a, n, n, per_region, shard_seed_base(0, slots) + r * per_region, stream=stream)
    torch.cuda.synchronize()
    rng = np.random.default_rng(0x5EED0005)
    perm = rng.permutation(slots)
    addr = [regions[p // per_region] + (p % per_region) * n for p in perm.tolist()]
    batch = MessageBatch(cnt, slots)
    t0 = time.perf_counter()
    for m in range(cnt):
        batch.add([(addr[m * nseg + j], n) for j in range(nseg)])
    add_s = time.perf_counter() - t0
    batch.submit(stream.cuda_stream)
    batch.wait()
    check = []
    for m in (0, cnt - 1):
        acc = 0
        for j in range(nseg):
            acc = ck.crc32c_extend(PinnedAlloc.view(addr[m * nseg + j], n).tobytes(), acc)
        check.append(acc == batch.result(m)[1])

    def step():
        batch.submit(stream.cuda_stream)
        batch.wait()

    steps = max(2, min(args.steps, 10))
    elapsed, _, _, _ = timed_region(step, steps, 2, torch.cuda.synchronize)
    nbytes = n * slots
    print(json.dumps({"metric": "GiB/s CRC32C CheckedMessage batch validation, payload in pinned host memory "
                                "(zero-copy: descriptors, payload and verdicts in pinned memory)",
                      "value": round(nbytes * steps / elapsed / GIB, 3), "unit": "GiB/s", "n_gpus": 1,
                      "steps": steps, "ms_per_step": round(elapsed / steps * 1e3, 3),
                      "add_us_per_message_python": round(add_s / cnt * 1e6, 2), "self_check": all(check),
                      "config": {"workload": cfg["workload"] + ", pinned host memory (IOAlloc pool)"}}))
    batch.close()
    for a in regions:
        alloc.dealloc(a)


def run_rpc_latency(args, stream):
    """Latency of one CheckedMessage batch submit + wait (zero-copy descriptors
    and verdicts, one launch) for 1..4096 messages of 8 x 8 KiB segments in
    pinned host memory, beside Photon's own crc32c() on one core over the same
    byte count (oracle/_ref harness, when built). Median of 50. DESIGN.md."""
    from photonlibos_amd.checked import MessageBatch, PinnedAlloc
    n, nseg = 8192, 8
    alloc = PinnedAlloc()
    region = 64 << 20
    per_region = region // n
    maxmsg = 4096
    regions = [alloc.alloc(region) for _ in range((maxmsg * nseg + per_region - 1) // per_region)]
    for r, a in enumerate(regions):
        ck.fill_splitmix(a, n, n, per_region, 0x5EED0001 + r * per_region, stream=stream)
    torch.cuda.synchronize()
    addr = [regions[s // per_region] + (s % per_region) * n for s in range(maxmsg * nseg)]
    rows = []
    for k in (1, 16, 256, 4096):
        batch = MessageBatch(k, k * nseg)
        for m in range(k):
            batch.add([(addr[m * nseg + j], n) for j in range(nseg)])
        ts = []
        for _ in range(55):
            t0 = time.perf_counter()
            batch.submit(stream.cuda_stream)
            batch.wait()
            ts.append(time.perf_counter() - t0)
        gpu_us = float(np.median(ts[5:])) * 1e6
        row = {"messages": k, "payload_bytes": k * nseg * n, "gpu_submit_wait_us": round(gpu_us, 1)}
        harness = os.path.join(REPO, "oracle", "_ref", "ref_harness")
        if os.path.exists(harness):  # Photon's crc32c() over the same byte count, one core
            r = _run_harness([harness, "bench"], k * nseg, n, 1, 1)
            if r is not None:
                row["photon_cpu_1core_us"] = round(r["best_s"] * 1e6, 1)
        rows.append(row)
        batch.close()
    for a in regions:
        alloc.dealloc(a)
    print(json.dumps({"metric": "CheckedMessage batch latency (submit + wait), 8 x 8 KiB messages in pinned host memory",
                      "rows": rows}))


def run_extend(args, stream):
    """One long device buffer (photon_crc32c_extend_device, the routed drop-in
    crc32c_extend on device memory): the reference's own perf shape
    (common/checksum/test/test_checksum.cpp:125-168 times one 128 KiB and one
    1 GiB buffer at buf+1). 1 GiB: GiB/s and % of 8 TB/s from HIP events
    around each call on the launch stream; 128 KiB: latency per call (enqueue
    + wait); the routed drop-in crc32c_extend on a device pointer (sync); and
    the price of routing on HOST pointers (hipPointerGetAttributes per call,
    C1's 4 KiB buffers), dispatch off vs on. Reported in DESIGN.md, never `value`."""
    import ctypes
    res = {"metric": "photon_crc32c_extend_device: one long device buffer at base+1 (reference perf shape)"}
    n = 1 << 30
    d = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    ck.fill_splitmix(d, n + 64, n + 64, 1, 0x5EED0900, stream=stream)
    out = torch.zeros(64, dtype=torch.int32, device="cuda")
    # 1 MiB and 8 MiB: the mid layout (the small kernel's code over 512
    # workgroups); 64 MiB: the long kernel's smallest full-chip cut
    for label, nbytes, steps in (("1GiB", n, max(10, min(args.steps, 50))), ("128KiB", 128 << 10, 200),
                                 ("1MiB", 1 << 20, 200), ("8MiB", 8 << 20, 200), ("64MiB", 64 << 20, 100)):
        ms = []
        for k in range(steps + 5):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            ck.extend_device(d.data_ptr() + 1, nbytes, 0, out[k % 64:k % 64 + 1], stream=stream)
            b.record(stream)
            ms.append((a, b))
        torch.cuda.synchronize()
        t = np.array([a.elapsed_time(b) for a, b in ms[5:]])
        # enqueue + wait latency, one call at a time
        lat = []
        for _ in range(50):
            t0 = time.perf_counter()
            ck.extend_device(d.data_ptr() + 1, nbytes, 0, out[:1], stream=stream)
            stream.synchronize()
            lat.append(time.perf_counter() - t0)
        gbps = nbytes / (float(np.mean(t)) * 1e-3) / 1e9
        res[label] = {"bytes": nbytes, "kernel_ms_mean": round(float(np.mean(t)), 4),
                      "kernel_ms_median": round(float(np.median(t)), 4), "GiB_per_s": round(gbps * 1e9 / GIB, 1),
                      "frac_of_8TBps": round(gbps / HBM_PEAK_GBPS, 4),
                      "frac_of_8TBps_median_launch": round(nbytes / (float(np.median(t)) * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                      "call_wait_us_median": round(float(np.median(lat)) * 1e6, 1)}
    # What the same bytes can do as independent pieces, interleaved with the
    # long kernel in rounds (the clock moves with launch history): the strided
    # batch over 16 Ki x 64 KiB from an aligned base (no cross-chunk combine,
    # no cross-workgroup reduce) and the read-only grid-stride stream.
    pieces = torch.zeros(n >> 16, dtype=torch.int32, device="cuda")
    sink = torch.zeros(1 << 22, dtype=torch.int32, device="cuda")
    cmp_fns = {"long_kernel": lambda k: ck.extend_device(d.data_ptr() + 1, n, 0, out[k:k + 1], stream=stream),
               "batch_64KiB_pieces": lambda k: ck.batch_strided(d.data_ptr(), 65536, 65536, n >> 16, pieces,
                                                                stream=stream),
               "read_stream": lambda k: ck.read_stream(d.data_ptr(), n, sink, sink.numel(), stream=stream)}
    cmp_t = {k: [] for k in cmp_fns}
    for r in range(6):
        for name in (list(cmp_fns) if r % 2 == 0 else list(cmp_fns)[::-1]):
            evs = []
            for k in range(8):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                cmp_fns[name](k)
                b.record(stream)
                evs.append((a, b))
            torch.cuda.synchronize()
            cmp_t[name] += [a.elapsed_time(b) for a, b in evs]
    res["1GiB_interleaved"] = {name: {"ms_median": round(float(np.median(v)), 4),
                                      "frac_median_launch": round(n / (float(np.median(v)) * 1e-3) / 1e9 /
                                                                  HBM_PEAK_GBPS, 4)} for name, v in cmp_t.items()}
    want = ck.crc32c_hw(d[1:1 + (128 << 10)].cpu().numpy().tobytes())
    ck.extend_device(d.data_ptr() + 1, 128 << 10, 0, out[:1], stream=stream)
    torch.cuda.synchronize()
    ok = int(out[0].item()) & 0xFFFFFFFF == want
    # Routed drop-in: crc32c_extend through crc32c_auto on a device pointer
    # (default stream, synchronous), and the routing probe's price on host
    # pointers (C1: 1024 x 4 KiB).
    ck.set_device_dispatch(True)
    ck.set_small_service(0)  # the launch path first (the service: below)
    routed = []
    for _ in range(50):
        t0 = time.perf_counter()
        r = ck.crc32c_extend_at(d.data_ptr() + 1, 128 << 10, 0)
        routed.append(time.perf_counter() - t0)
    ok = ok and r == want
    routed_1g = []
    for _ in range(10):  # the same drop-in on the 1 GiB buffer (the long kernel, tagged result word)
        t0 = time.perf_counter()
        ck.crc32c_extend_at(d.data_ptr() + 1, n, 0)
        routed_1g.append(time.perf_counter() - t0)
    # The routed calls' wait policy (photon_crc_set_routed_wait): latency and
    # the calling thread's CPU time (CLOCK_THREAD_CPUTIME_ID) over >= 0.3 s of
    # back-to-back calls each, for spin windows / sleep-ahead on and off.
    policies = {}
    for spin_us, ahead in ((40, True), (30, True), (0, False), (100, True), (1000, False)):
        ck.set_routed_wait(spin_us, ahead)
        row = {}
        for label, nb in (("128KiB", 128 << 10), ("1GiB", n)):
            lat = []
            c0, w0 = time.thread_time(), time.perf_counter()
            while time.perf_counter() - w0 < 0.3 or len(lat) < 20:
                t0 = time.perf_counter()
                ck.crc32c_extend_at(d.data_ptr() + 1, nb, 0)
                lat.append(time.perf_counter() - t0)
            row[label] = {"us_median": round(float(np.median(lat)) * 1e6, 1),
                          "thread_cpu_frac": round((time.thread_time() - c0) / (time.perf_counter() - w0), 3),
                          "calls": len(lat)}
        policies[f"spin{spin_us}{'_sleep_ahead' if ahead else ''}"] = row
    ck.set_routed_wait(40, True)
    # The resident small-buffer services (photon_crc_set_small_service, the
    # default, 200 us idle): the same 128 KiB calls with no launch per call
    # (the first call of a launch takes the launch path and is not timed);
    # the calling thread's CPU time.
    ck.set_small_service(200)
    ok = ok and ck.crc32c_extend_at(d.data_ptr() + 1, 128 << 10, 0) == want
    svc0 = ck.small_service_stats()
    svc = []
    c0, w0 = time.thread_time(), time.perf_counter()
    for _ in range(400):
        t0 = time.perf_counter()
        r = ck.crc32c_extend_at(d.data_ptr() + 1, 128 << 10, 0)
        svc.append(time.perf_counter() - t0)
        ok = ok and r == want
    svc_cpu = (time.thread_time() - c0) / (time.perf_counter() - w0)
    svc1 = ck.small_service_stats()
    want64 = ck.crc64ecma_extend_at(d.data_ptr() + 1, 128 << 10, 0)  # starts the CRC-64 service
    svc64 = []
    for _ in range(400):
        t0 = time.perf_counter()
        r = ck.crc64ecma_extend_at(d.data_ptr() + 1, 128 << 10, 0)
        svc64.append(time.perf_counter() - t0)
        ok = ok and r == want64
    ck.set_small_service(0)
    launch64 = []
    for _ in range(100):
        t0 = time.perf_counter()
        r = ck.crc64ecma_extend_at(d.data_ptr() + 1, 128 << 10, 0)
        launch64.append(time.perf_counter() - t0)
        ok = ok and r == want64
    ck.set_small_service(200)
    ck.set_device_dispatch(False)
    hbuf = np.frombuffer(d[:1024 * 4096].cpu().numpy().tobytes(), np.uint8)
    base = hbuf.ctypes.data

    def per_call_us(on):
        ck.set_device_dispatch(on)
        fn = ck._auto("crc32c_auto", ctypes.CFUNCTYPE(ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t,
                                                       ctypes.c_uint32))
        best = 1e9
        for _ in range(5):
            t0 = time.perf_counter()
            for i in range(1024):
                fn(base + i * 4096, 4096, 0)
            best = min(best, time.perf_counter() - t0)
        ck.set_device_dispatch(False)
        return best / 1024 * 1e6
    off_us, on_us = per_call_us(False), per_call_us(True)
    # The CPU alternative for DEVICE-resident bytes: copy the 128 KiB at
    # buf+1 to pinned host memory (one stream-ordered copy + wait), then the
    # host engine (crc32c_auto = crc32c_hw, Photon's own choice on x86).
    from photonlibos_amd._native import lib as _lib
    L = _lib()
    hpin = torch.empty(128 << 10, dtype=torch.uint8).pin_memory()
    crc_fn = ck._auto("crc32c_auto", ctypes.CFUNCTYPE(ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t,
                                                       ctypes.c_uint32))
    sptr = ctypes.c_void_p(stream.cuda_stream)
    d2h = []
    for _ in range(50):
        t0 = time.perf_counter()
        L.photon_crc_memcpy_async(hpin.data_ptr(), d.data_ptr() + 1, 128 << 10, sptr)
        L.photon_crc_stream_sync(sptr)
        r2 = crc_fn(hpin.data_ptr(), 128 << 10, 0)
        d2h.append(time.perf_counter() - t0)
    ok = ok and r2 == want
    res["d2h_copy_then_host_crc32c_128KiB_us_median"] = round(float(np.median(d2h)) * 1e6, 1)
    res["routed_crc32c_extend_128KiB_device_us_median"] = round(float(np.median(routed)) * 1e6, 1)
    res["routed_crc32c_extend_1GiB_device_us_median"] = round(float(np.median(routed_1g)) * 1e6, 1)
    res["routed_wait_policies"] = policies
    res["routed_crc32c_extend_128KiB_service"] = {
        "us_median": round(float(np.median(svc)) * 1e6, 1), "us_p10": round(float(np.percentile(svc, 10)) * 1e6, 1),
        "us_p90": round(float(np.percentile(svc, 90)) * 1e6, 1), "thread_cpu_frac": round(svc_cpu, 3),
        "served": svc1[0] - svc0[0], "calls": len(svc), "starts": svc1[1] - svc0[1]}
    res["routed_crc64ecma_extend_128KiB_us_median"] = {
        "service": round(float(np.median(svc64)) * 1e6, 1), "launch_path": round(float(np.median(launch64)) * 1e6, 1)}
    res["host_pointer_call_us"] = {"dispatch_off": round(off_us, 3), "dispatch_on": round(on_us, 3),
                                   "note": "C1 (1024 x 4 KiB host buffers) through crc32c_auto from Python "
                                           "ctypes; the difference is the per-call hipPointerGetAttributes probe"}
    res["self_check"] = ok
    print(json.dumps(res))


def run_file_records(args):
    """§8(f) row 4: CRC32C of the 4 KiB records of a 1 GiB file (page-cache
    hot, buffered pread into pinned chunks + GPU pipeline), end to end.
    Reported in DESIGN.md, never as `value`."""
    n, size = 4096, 1 << 30
    count = size // n
    with tempfile.NamedTemporaryFile(dir=os.environ.get("TMPDIR", "/tmp"), delete=True) as f:
        rng = np.random.default_rng(0x5EED0F11)
        for _ in range(size // (64 << 20)):
            f.write(rng.integers(0, 256, 64 << 20, dtype=np.uint8).tobytes())
        f.flush()
        fd = os.open(f.name, os.O_RDONLY)
        try:
            out = ck.file_strided(fd, 0, n, n, count)  # warm the page cache and the pipeline
            steps = max(2, min(args.steps, 5))
            t0 = time.perf_counter()
            for _ in range(steps):
                out = ck.file_strided(fd, 0, n, n, count)
            el = time.perf_counter() - t0
            ok = out[7] == ck.crc32c_hw(os.pread(fd, n, 7 * n))
            # two concurrent callers (per-call chunk buffers, shared reader pool)
            import threading
            outs = [None, None]

            def one(k):
                outs[k] = ck.file_strided(fd, 0, n, n, count)
            t1 = time.perf_counter()
            th = [threading.Thread(target=one, args=(k,)) for k in range(2)]
            for t in th:
                t.start()
            for t in th:
                t.join()
            el2 = time.perf_counter() - t1
            ok = ok and all(np.array_equal(o, out) for o in outs)
        finally:
            os.close(fd)
    print(json.dumps({"metric": "GiB/s CRC32C of 4 KiB file records (pread into pinned chunks + GPU pipeline), "
                                "page-cache hot", "value": round(size * steps / el / GIB, 3), "unit": "GiB/s",
                      "n_gpus": 1, "steps": steps, "ms_per_step": round(el / steps * 1e3, 3),
                      "two_concurrent_callers_ms": round(el2 * 1e3, 3), "self_check": ok,
                      "config": {"workload": "1 GiB file, 262144 x 4 KiB records"}}))


def event_marks(stream):
    """timed_region's on_step: one HIP event per launch boundary on the launch
    stream (see main)."""
    bounds = {}

    def on_step(s, step):
        if s == 0:
            bounds.clear()
        if s not in bounds:
            bounds[s] = torch.cuda.Event(enable_timing=True)
            bounds[s].record(stream)
        step()
        bounds[s + 1] = torch.cuda.Event(enable_timing=True)
        bounds[s + 1].record(stream)
        a, b = bounds[s], bounds[s + 1]
        return lambda: a.elapsed_time(b)
    return on_step


def c4_leg(args, rank, world, device, stream, dist):
    """BASELINE configs[3] in the same ranks after the C2 leg,
    at every N (the same per-GPU shard at 1/2/4/8 GPUs):
    every rank checksums its 32 Ki x 1 MiB shard of the 256 Ki x 1 MiB batch
    (global ids r*32768.., no collective), timed like the C2 leg (barrier +
    sync both sides, max over ranks). At N = 8 this is the whole configs[3]
    batch; at N < 8, N/8 of it."""
    cfg = CONFIGS["c4"]
    wl = Workload(cfg, rank, stream)
    elapsed, kernel_ms, local_el, local_ms = timed_region(wl.step, args.steps, args.warmup, torch.cuda.synchronize,
                                                          dist, event_marks(stream))
    ok = wl.self_check()
    ranks = gather_ranks(dist, {"rank": rank, "device": device, "wall_s": round(local_el, 6),
                                "launch_ms": launch_summary(local_ms), "self_check": ok})
    per_launch = wl.bytes_per_step / (kernel_ms * 1e-3) / 1e9
    rec = {"workload": cfg["workload"], "config": "c4", "buffers_total": cfg["count"] * world,
           "buffer_bytes": cfg["nbytes"],
           "value": round(aggregate_gibps(wl.bytes_per_step, args.steps, world, elapsed), 3), "unit": "GiB/s",
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
           "frac": round(per_launch / HBM_PEAK_GBPS, 4),
           "frac_wall": round(wl.bytes_per_step * args.steps * world / elapsed / 1e9 / (HBM_PEAK_GBPS * world), 4),
           "per_rank": ranks, "self_check": all(r["self_check"] for r in ranks)}
    del wl
    torch.cuda.empty_cache()
    return rec


# ------------------------------------------------------------- CPU rehearsal

def run_cpu_rehearsal(args, rank, world, dist):
    """The N-rank launcher, timed region and report with no GPU: every rank
    checksums its own shard of 64 x 64 KiB host buffers through this library's
    crc32c() drop-in (the C-ABI library's host engine). For the CPU tests.
    `config` names the GPU workload this --gpus N / --config would run (the
    same at every N, so a scaling sweep compares like with like); the host
    step itself is `rehearsal_step`."""
    from photonlibos_amd import datagen
    n, cnt = 65536, 64
    bufs = [datagen.stream_bytes(shard_seed_base(rank, cnt) + i, n).tobytes() for i in range(cnt)]
    out = [0] * cnt

    def step():
        for i, b in enumerate(bufs):
            out[i] = ck.crc32c(b)
    def on_step(s, f):
        t0 = time.perf_counter()
        f()
        dt = (time.perf_counter() - t0) * 1e3
        return lambda: dt

    elapsed, _, local_el, local_ms = timed_region(step, args.steps, args.warmup, lambda: None, dist, on_step)
    ranks = gather_ranks(dist, {"rank": rank, "wall_s": round(local_el, 6), "first_crc": int(out[0]),
                                "launch_ms": launch_summary(local_ms)})
    c4 = None
    if args.config == "c2" and not args.no_c4_leg:
        # the C4 leg's host stand-in: 4 x 1 MiB per rank (global ids as the C4 shard's)
        n4, cnt4 = 1 << 20, 4
        bufs4 = [datagen.stream_bytes(shard_seed_base(rank, CONFIGS["c4"]["count"]) + i, n4).tobytes()
                 for i in range(cnt4)]
        out4 = [0] * cnt4

        def step4():
            for i, b in enumerate(bufs4):
                out4[i] = ck.crc32c(b)
        el4, _, lel4, lms4 = timed_region(step4, args.steps, args.warmup, lambda: None, dist, on_step)
        r4 = gather_ranks(dist, {"rank": rank, "wall_s": round(lel4, 6), "first_crc": int(out4[0]),
                                 "launch_ms": launch_summary(lms4)})
        c4 = {"workload": CONFIGS["c4"]["workload"], "config": "c4", "buffers_total": CONFIGS["c4"]["count"] * world,
              "value": round(aggregate_gibps(n4 * cnt4, args.steps, world, el4), 3), "unit": "GiB/s",
              "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el4 / args.steps * 1e3, 4),
              "per_rank": r4, "rehearsal_step": f"{cnt4} x {n4} B host buffers per rank, crc32c() drop-in"}
    tail = rank0_tail(args, CONFIGS[args.config], rank, world, dist, gpu=False)
    extra = {k: tail[k] for k in ("cpu_baseline", "cpu_reference_c1") if k in tail}
    if rank == 0:
        print(json.dumps({"metric": "GiB/s CRC32C host rehearsal of the N-rank bench path (no GPU)",
                          "value": round(aggregate_gibps(n * cnt, args.steps, world, elapsed), 3), "unit": "GiB/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(elapsed / args.steps * 1e3, 4), "scaling": "weak",
                          "rehearsal": "cpu", "per_rank": ranks,
                          "rehearsal_step": f"{cnt} x {n} B host buffers per rank, crc32c() drop-in",
                          "config": {"workload": CONFIGS[args.config]["workload"], "config": args.config,
                                     "parallelism": f"shard-per-gpu x{world}"},
                          "roofline": {"bound": "hbm", "traffic": tail["traffic"],
                                       "traffic_source": tail["traffic_source"],
                                       "traffic_scope": tail["traffic_scope"],
                                       "note": "rehearsal: no kernel was timed, only the tail's plumbing"},
                          **extra, **({"config_c4": c4} if c4 else {})}), flush=True)


# ----------------------------------------------------------------------- main

def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args, argv)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and not (args.pmc_child or args.h2d or args.rpc_batch or args.rpc_latency
                                   or args.file_records or args.extend):
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        return 2
    global ck
    from photonlibos_amd import checksum as _ck
    ck = _ck
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    if args.cpu_rehearsal:
        run_cpu_rehearsal(args, rank, world, dist)
        if dist:
            dist.destroy_process_group()
        return 0
    visible = torch.cuda.device_count()
    if visible < 1 or (world > visible and not args.share_gpus):
        print(f"bench.py: rank {rank}: {visible} GPU(s) visible for {world} ranks", file=sys.stderr)
        return 2
    device = args.device if args.device is not None else local % visible
    torch.cuda.set_device(device)
    ck.set_lanes_per_buffer(args.lanes)
    if args.msg_rows:
        ck.set_msg_rows(args.msg_rows)
    if args.rows:
        ck.set_generic_rows(args.rows)
    stream = torch.cuda.current_stream()
    if args.h2d or args.rpc_batch or args.rpc_latency or args.file_records or args.extend:
        if rank == 0:
            if args.h2d:
                run_h2d(args, stream)
            elif args.extend:
                run_extend(args, stream)
            elif args.rpc_batch:
                run_rpc_batch(args, stream)
            elif args.rpc_latency:
                run_rpc_latency(args, stream)
            else:
                run_file_records(args)
        return 0
    cfg = CONFIGS[args.config]
    wl = Workload(cfg, rank, stream)  # the fill kernel runs right before the warmup launches

    # Per-launch times from HIP events on the launch stream, ONE event per
    # launch boundary (K + 1 for K launches): every event record is a packet
    # between two launches, and the round-3 bench's two per launch cost the
    # wall clock ~1.3 % over the kernels' own time (r04a: 0.6441 ms per step
    # against a 0.636 ms mean launch). A launch's time is boundary to
    # boundary, so it includes the gap before the next launch.
    on_step = event_marks(stream)

    if args.pmc_child:  # the workload's launches under rocprofv3 --pmc (live_traffic)
        for _ in range(args.warmup + args.steps):
            wl.step()
        torch.cuda.synchronize()
        return 0
    elapsed, kernel_ms, local_el, local_ms = timed_region(wl.step, args.steps, args.warmup, torch.cuda.synchronize,
                                                          dist, on_step)
    ok = wl.self_check()  # the last timed step's results, checked after the timed region
    bytes_step = wl.bytes_per_step
    value = aggregate_gibps(wl.bytes_per_step, args.steps, world, elapsed)
    per_launch_gbps = wl.bytes_per_step / (kernel_ms * 1e-3) / 1e9
    ls = launch_summary(local_ms)
    ranks = gather_ranks(dist, {"rank": rank, "device": device, "wall_s": round(local_el, 6),
                                "launch_ms": ls, "self_check": ok})
    all_ok = all(r["self_check"] for r in ranks)

    shape64 = None
    if world == 1 and cfg["kind"] == "strided" and not args.no_shape64 and not args.lanes:
        # The north star's literal shape (one wavefront per buffer, G = 64)
        # beside the measured-best lane group, outside the timed region.
        ck.set_lanes_per_buffer(64)
        _, ms64, _, l64 = timed_region(wl.step, 20, 3, torch.cuda.synchronize, None, on_step)
        ck.set_lanes_per_buffer(0)
        shape64 = {"lanes_per_buffer": 64, "kernel_ms_mean": round(ms64, 4),
                   "kernel_ms_median": round(float(np.median(l64)), 4),
                   "frac": round(wl.bytes_per_step / (ms64 * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)}

    c4 = None
    if args.config == "c2" and not args.no_c4_leg:
        del wl
        torch.cuda.empty_cache()
        c4 = c4_leg(args, rank, world, device, stream, dist)
        all_ok = all_ok and c4["self_check"]

    tail = rank0_tail(args, cfg, rank, world, dist, gpu=True, device=device)
    traffic, traffic_src = tail["traffic"], tail["traffic_source"]

    if rank == 0:
        steady = bytes_step / (float(np.median([r["launch_ms"]["median"] for r in ranks])) * 1e-3) / 1e9
        res = {
            "metric": METRIC.replace("CRC32C", "CRC-64/ECMA") if cfg["kind"] == "strided64" else METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 random bytes generated on device)",
            "config": {"workload": cfg["workload"], "config": args.config, "buffers": cfg["count"],
                       "buffer_bytes": cfg["nbytes"],
                       "bytes_per_gpu_per_step": bytes_step, "parallelism": f"shard-per-gpu x{world}",
                       "lanes_per_buffer": args.lanes or "auto"},
            "roofline": {"bound": "hbm", "achieved": round(per_launch_gbps, 1), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(per_launch_gbps / HBM_PEAK_GBPS, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "algorithmic_bytes": bytes_step,
                         "frac_kernel": round(per_launch_gbps / HBM_PEAK_GBPS, 4),
                         "frac_wall": round(bytes_step * args.steps * world / elapsed / 1e9
                                            / (HBM_PEAK_GBPS * world), 4),
                         "frac_steady_median_launch": round(steady / HBM_PEAK_GBPS, 4),
                         "clock_note": "frac/frac_kernel: mean launch time between HIP events at the launch "
                                       "boundaries on the launch stream (slowest rank); frac_wall: value's wall "
                                       "clock; frac_steady: median launch"},
            "per_rank": ranks if world > 1 else None,
            "launch_ms": ls if world == 1 else None,
            "self_check": all_ok,
        }
        if args.share_gpus and world > visible:
            res["rehearsal"] = f"{world} ranks sharing {visible} visible GPU(s): not a scaling measurement"
        if shape64:
            res["north_star_shape_g64"] = shape64
        if c4:
            res["config_c4"] = c4
        res["roofline"]["traffic_scope"] = tail["traffic_scope"]
        for k in ("cpu_baseline", "cpu_reference_c1"):
            if k in tail:
                res[k] = tail[k]
        print(json.dumps(res), flush=True)
    if dist:
        dist.destroy_process_group()
    return 0 if all_ok else 1


if __name__ == "__main__":
    sys.exit(main())
