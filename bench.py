#!/usr/bin/env python3
"""Benchmark of the north-star path: CRC32C over device-resident buffers on
MI355X through the C-ABI engine (libphoton_checksum.so).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5] [--h2d]

One "step" = one pass of the hot path over one batch (BASELINE.json configs):
  c2 (default, configs[1]): 65,536 x 64 KiB random buffers, device-resident
  c3: 1,048,576 x 4 KiB        c4: 32,768 x 1 MiB per GPU (the 8-GPU config's shard)
  c5: 65,536 messages x 8 non-contiguous 8 KiB segments, per-message CRC (chained extend)
  c5_seg: the same with every segment's own CRC written too
  --h2d: the c2 batch starting and ending in pinned host memory (chunked
         H2D + kernel + D2H); reported in DESIGN.md, never as `value`.
Multi-GPU: one process per GPU (torchrun); every rank checksums its own
independent batch (weak scaling, no data-path collective; gloo carries only
the timing barrier and the max-over-ranks). Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from photonlibos_amd import checksum as ck  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec, MI355X_MICROARCH.md "Chip-level parameters"
GIB = float(1 << 30)
METRIC = "GiB/s CRC32C over device-resident buffers; % of HBM-read roofline"

CONFIGS = {
    "c2": dict(kind="strided", nbytes=65536, count=65536,
               workload="C2: 65536 x 64 KiB random buffers, device-resident, per GPU"),
    "c3": dict(kind="strided", nbytes=4096, count=1 << 20,
               workload="C3: 1048576 x 4 KiB RPC-payload buffers, device-resident, per GPU"),
    "c4": dict(kind="strided", nbytes=1 << 20, count=32768,
               workload="C4 shard: 32768 x 1 MiB buffers per GPU (256K x 1 MiB over 8 GPUs)"),
    "c5": dict(kind="msg", nbytes=8192, count=65536, nseg=8, seg_out=False,
               workload="C5: 65536 messages x 8 non-contiguous 8 KiB segments, per-message CRC "
                        "(Crc32Hasher: crc32c_extend chained over the segments = per-segment CRC + combine)"),
    "c5_seg": dict(kind="msg", nbytes=8192, count=65536, nseg=8, seg_out=True,
                   workload="C5 shape, per-segment CRCs also written (segment kernel + fold kernel)"),
    "c2_crc64": dict(kind="strided64", nbytes=65536, count=65536,
                     workload="C2 shape, CRC-64/ECMA (next row): 65536 x 64 KiB, device-resident, per GPU"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=25,
                    help="untimed steps; the first ~10 back-to-back launches run slower while clocks settle")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--h2d", action="store_true", help="host-memory end-to-end rate (for DESIGN.md)")
    ap.add_argument("--h2d-devices", type=int, default=1,
                    help="with --h2d: shard the host batch over this many devices of ONE process (0 = all)")
    ap.add_argument("--file-records", action="store_true", help="file records through the pread pipeline (DESIGN.md)")
    ap.add_argument("--rpc-batch", action="store_true", help="CheckedMessage batch over pinned host payloads (DESIGN.md)")
    ap.add_argument("--rpc-latency", action="store_true", help="submit+wait latency of small CheckedMessage batches")
    ap.add_argument("--lanes", type=int, default=0, help="lanes per buffer override (0 = auto)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--traffic-json", default=None,
                    help="PMC summary (profiles/*.json) giving HBM bytes per launch")
    return ap.parse_args(argv)


def shard_seed_base(rank, count):
    """Rank r checksums buffers with global ids [r*count, (r+1)*count):
    splitmix streams 0x5EED0001 + global id (disjoint shards, no collective)."""
    return 0x5EED0001 + rank * count


def timed_region(step, steps, warmup, sync, dist=None, on_step=None):
    """Run `warmup` untimed steps, then exactly `steps` steps bracketed by a
    barrier + device sync on both sides. Returns the max over ranks of the
    wall time and of the mean per-step time reported by `on_step` (ms)."""
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
    per_step_ms = float(np.mean([m() for m in marks])) if marks else elapsed / steps * 1e3
    if dist is not None:
        t = torch.tensor([elapsed, per_step_ms], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, per_step_ms = float(t[0]), float(t[1])
    return elapsed, per_step_ms


def aggregate_gibps(bytes_per_step_per_rank, steps, world, elapsed):
    """Whole-job throughput: every rank's bytes over the slowest rank's time."""
    return bytes_per_step_per_rank * steps * world / elapsed / GIB


class Workload:
    """Device-resident synthetic batch for one config on the current device."""

    def __init__(self, cfg, rank, stream):
        self.cfg = cfg
        self.stream = stream
        n, cnt = cfg["nbytes"], cfg["count"]
        if cfg["kind"] in ("strided", "strided64"):
            slots = cnt
        else:
            slots = cnt * cfg["nseg"]
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
        torch.cuda.synchronize()

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
        """Spot-check results against the product's own host engine (crc32c_hw
        and crc32c_combine), not the oracle."""
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
        base = self.payload.data_ptr()
        for m in (0, c["count"] - 1):
            acc = 0
            for j in range(c["nseg"]):
                off = int(iov[m * c["nseg"] + j, 0]) - base
                acc = ck.crc32c_extend(self.payload[off:off + n].cpu().numpy().tobytes(), acc)
            if acc != out[m]:
                return False
        return True


def cpu_baseline(cfg, seconds):
    """Photon's own CPU checksum (reference crc.cpp, oracle/_ref/ref_harness),
    timed on this host; the oracle's C port as fallback."""
    n = cfg["nbytes"]
    nbuf = max(1, (256 << 20) // n)  # bounded 256 MiB sample of the same workload
    threads = max(1, min(16, os.cpu_count() or 1))
    harness = os.path.join(REPO, "oracle", "_ref", "ref_harness")
    sample = f"{nbuf} x {n} B random host buffers (256 MiB, stream 0x5EED0001+i), best pass over >= {seconds:.0f} s"
    if os.path.exists(harness):
        out = subprocess.run([harness, "bench", str(nbuf), str(n), str(threads), str(seconds)],
                             capture_output=True, text=True, timeout=seconds * 4 + 120)
        if out.returncode == 0:
            r = json.loads(out.stdout.strip().splitlines()[-1])
            cpu = ""
            try:
                cpu = [ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name")][0]
            except Exception:
                pass
            return {"value": round(r["gib_per_s"], 3), "unit": "GiB/s", "cores": threads, "kind": "reference",
                    "sample": sample + f"; Photon crc32c() auto-dispatch (crc.cpp:339-358) on {threads} threads"
                    + (f" of {cpu}" if cpu else "")}
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
    """config C1 (1024 x 4 KiB, the reference's CPU-runnable
    case) with Photon's own crc32c() on 1 thread and on 16 threads, beside the
    main baseline. Empty when the reference build is absent."""
    harness = os.path.join(REPO, "oracle", "_ref", "ref_harness")
    if not os.path.exists(harness):
        return {}
    # beside it, this library's drop-in host engine (same header, same buffers)
    dropin = os.path.join(REPO, "tests", "cpp", "bin", "host_bench")
    out = {}
    for threads in (1, max(1, min(16, os.cpu_count() or 1))):
        for key, cmd in ((f"threads_{threads}", [harness, "bench"]), (f"dropin_threads_{threads}", [dropin])):
            if not os.path.exists(cmd[0]):
                continue
            r = subprocess.run(cmd + ["1024", "4096", str(threads), str(seconds)],
                               capture_output=True, text=True, timeout=seconds * 4 + 60)
            if r.returncode == 0:
                out[key] = round(json.loads(r.stdout.strip().splitlines()[-1])["gib_per_s"], 3)
    return {"unit": "GiB/s", "workload": "C1: 1024 x 4 KiB random buffers (cache-resident), Photon crc32c(); "
            "dropin_*: this library's crc32c() drop-in on the same buffers", **out} if out else {}


def load_traffic(path, config):
    if path is None:
        path = os.path.join(REPO, "profiles", f"pmc_{config}.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    v = d.get("hbm_bytes_per_launch")
    return int(v) if v else None  # HBM bytes per launch (PMC, corrected), vs the algorithmic bytes


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
    elapsed, _ = timed_region(step, steps, 2, torch.cuda.synchronize)
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
    elapsed, _ = timed_region(step, steps, 2, torch.cuda.synchronize)
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
            r = subprocess.run([harness, "bench", str(k * nseg), str(n), "1", "1"], capture_output=True, text=True,
                               timeout=120)
            if r.returncode == 0:
                row["photon_cpu_1core_us"] = round(json.loads(r.stdout.strip().splitlines()[-1])["best_s"] * 1e6, 1)
        rows.append(row)
        batch.close()
    for a in regions:
        alloc.dealloc(a)
    print(json.dumps({"metric": "CheckedMessage batch latency (submit + wait), 8 x 8 KiB messages in pinned host memory",
                      "rows": rows}))


def run_file_records(args):
    """§8(f) row 4: CRC32C of the 4 KiB records of a 1 GiB file (page-cache
    hot, buffered pread into pinned chunks + GPU pipeline), end to end.
    Reported in DESIGN.md, never as `value`."""
    import tempfile
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
        finally:
            os.close(fd)
    print(json.dumps({"metric": "GiB/s CRC32C of 4 KiB file records (pread into pinned chunks + GPU pipeline), "
                                "page-cache hot", "value": round(size * steps / el / GIB, 3), "unit": "GiB/s",
                      "n_gpus": 1, "steps": steps, "ms_per_step": round(el / steps * 1e3, 3), "self_check": ok,
                      "config": {"workload": "1 GiB file, 262144 x 4 KiB records"}}))


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    # one process per GPU; ranks beyond the visible devices (a rehearsal on a
    # smaller box) share them round-robin
    torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    ck.set_lanes_per_buffer(args.lanes)
    stream = torch.cuda.current_stream()
    if args.h2d:
        if rank == 0:
            run_h2d(args, stream)
        return
    if args.rpc_batch:
        if rank == 0:
            run_rpc_batch(args, stream)
        return
    if args.rpc_latency:
        if rank == 0:
            run_rpc_latency(args, stream)
        return
    if args.file_records:
        if rank == 0:
            run_file_records(args)
        return
    cfg = CONFIGS[args.config]
    wl = Workload(cfg, rank, stream)
    wl.step()
    torch.cuda.synchronize()
    ok = wl.self_check()

    def on_step(s, step):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        step()
        b.record(stream)
        return lambda: a.elapsed_time(b)

    elapsed, kernel_ms = timed_region(wl.step, args.steps, args.warmup, torch.cuda.synchronize, dist, on_step)
    value = aggregate_gibps(wl.bytes_per_step, args.steps, world, elapsed)
    per_launch_gbps = wl.bytes_per_step / (kernel_ms * 1e-3) / 1e9
    traffic = load_traffic(args.traffic_json, args.config)

    if rank == 0:
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
            "config": {"workload": cfg["workload"], "buffers": cfg["count"], "buffer_bytes": cfg["nbytes"],
                       "bytes_per_gpu_per_step": wl.bytes_per_step, "parallelism": f"shard-per-gpu x{world}",
                       "lanes_per_buffer": args.lanes or "auto"},
            "roofline": {"bound": "hbm", "achieved": round(per_launch_gbps, 1), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(per_launch_gbps / HBM_PEAK_GBPS, 4),
                         "traffic": traffic, "algorithmic_bytes": wl.bytes_per_step},
            "self_check": ok,
        }
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(cfg, args.cpu_seconds)
            res["cpu_reference_c1"] = cpu_reference_c1(min(5.0, args.cpu_seconds))
        print(json.dumps(res), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
