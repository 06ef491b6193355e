#!/usr/bin/env python3
"""Energy per payload byte of the C2 kernel against read-only controls
(bench-only probe; VERDICT r3 next #1: judge kernel changes by J/GiB).

In a fresh process, as bench.py: fill the C2 batch (65,536 x 64 KiB), then
per kernel -- `crc` (the product's batch kernel, or the stamped probe build
of it with --stamps), `rows` (the CRC kernel's own row pattern with the CRC
replaced by an XOR, probes.hip group_rows_stamped_kernel), `read` (the
grid-stride read stream) -- two measurements:
  * the driver's window: 25 back-to-back launches (bench.py --warmup 5
    --steps 20) right after the previous phase, HIP events per launch, the
    board energy counter read around the window (amdsmi), power and gfx
    clock sampled every ~2 ms by a host thread;
  * steady state: back-to-back launches for STEADY_S seconds, energy around it.
Per phase: GiB/s, mean board power (W), J/GiB, and for the stamped kernels
the in-kernel clock per launch (MI355X_MICROARCH.md 'DVFS give-back' item 6).
Energy comes from amdsmi_get_energy_count (accumulator x resolution, uJ);
without amdsmi the power sampler's mean power x time is used instead.
Phases are separated by IDLE_S seconds of idle GPU. One JSON line per phase.

  KERNELS=crc,rows,read,crc  STEADY_S=3  IDLE_S=2  [LANES=G] [ROWS64=2|4]  python scripts/probe_power.py [--stamps]
  (crc@W: the product kernel on a grid capped at W workgroups, photon_crc_set_batch_grid;
   c3: CRC-32C on the same 4 GiB as 1 Mi x 4 KiB buffers; c3_64 / c2_64: CRC-64/ECMA on
   4 KiB / 64 KiB buffers with the generic batch kernel (c5_64: 8 KiB), c3_64full / c2_64full: with the
   full-row kernel, cross-buffer prefetch, 2 rows per step; c4: CRC-32C on 4 Ki x 1 MiB; readp: the
   product's read-only row-pattern kernel, read_stream_kernel; crcsvc: the product kernel with a
   resident small-buffer service beside it -- after each group of launches is queued, one routed
   4 KiB call starts a service (1 s idle and life) that then idles, napping, beside the rest of
   the group; the next group's first launch ends it)
"""
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from photonlibos_amd import checksum as ck  # noqa: E402

P = ctypes.CDLL(os.environ.get("PHOTON_CRC_PROBES") or os.path.join(REPO, "photonlibos_amd", "lib", "libphoton_probes.so"))
vp, u64, ci = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
P.probe_crc_wave_times.argtypes = [vp, u64, u64, vp, vp, vp, ci, ci, ci, ci, vp]
P.probe_crc_wave_times.restype = ci
P.probe_read_stream_stamped.argtypes = [vp, u64, vp, vp, ci, vp]
P.probe_read_stream_stamped.restype = ci
P.probe_group_rows_stamped.argtypes = [vp, u64, u64, u64, vp, vp, ci, vp]
P.probe_group_rows_stamped.restype = ci

KERNELS = os.environ.get("KERNELS", "crc,rows,read,crc").split(",")
STEADY_S = float(os.environ.get("STEADY_S", "3"))
IDLE_S = float(os.environ.get("IDLE_S", "2"))
WINDOW = int(os.environ.get("WINDOW", "25"))
STAMPS = "--stamps" in sys.argv
GIB = float(1 << 30)


class Board:
    """Board energy / power / gfx clock of this process's GPU through amdsmi."""

    def __init__(self):
        self.h = None
        self.err = None
        try:
            import amdsmi
            self.m = amdsmi
            amdsmi.amdsmi_init()
            prop = torch.cuda.get_device_properties(0)
            for h in amdsmi.amdsmi_get_processor_handles():
                bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)
                dom, bus = bdf.split(":")[0], bdf.split(":")[1]
                if int(bus, 16) == prop.pci_bus_id and int(dom, 16) == prop.pci_domain_id:
                    self.h = h
                    self.bdf = bdf
            if self.h is None:
                self.err = "no amdsmi handle with this device's PCI bus id"
        except Exception as e:  # noqa: BLE001 -- the probe still reports times without the board
            self.err = f"amdsmi: {e!r}"

    def energy_uj(self):
        if self.h is None:
            return None
        try:
            e = self.m.amdsmi_get_energy_count(self.h)
            acc = e.get("energy_accumulator", e.get("power"))
            return float(acc) * float(e.get("counter_resolution", 1.0))
        except Exception as ex:  # noqa: BLE001
            self.err = f"energy: {ex!r}"
            return None

    def sample(self):
        if self.h is None:
            return None
        try:
            p = self.m.amdsmi_get_power_info(self.h)
            w = p.get("current_socket_power")
            if not isinstance(w, (int, float)) or w <= 0:
                w = p.get("average_socket_power")
            c = self.m.amdsmi_get_clock_info(self.h, self.m.AmdSmiClkType.GFX)
            return float(w), float(c.get("clk", c.get("cur_clk", 0)))
        except Exception as ex:  # noqa: BLE001
            self.err = f"sample: {ex!r}"
            return None


class Sampler(threading.Thread):
    def __init__(self, board, period=0.002):
        super().__init__(daemon=True)
        self.board, self.period, self.rows, self.stop_ev = board, period, [], threading.Event()

    def run(self):
        while not self.stop_ev.is_set():
            s = self.board.sample()
            if s is not None:
                self.rows.append((time.perf_counter(), s[0], s[1]))
            time.sleep(self.period)

    def stop(self):
        self.stop_ev.set()
        self.join()
        return self.rows


board = Board()
st = torch.cuda.current_stream()
cus = torch.cuda.get_device_properties(0).multi_processor_count
n, cnt = 65536, 65536
nbytes = n * cnt
buf = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
out = torch.zeros(cnt, dtype=torch.int32, device="cuda")
out3 = torch.zeros(nbytes // 4096, dtype=torch.int32, device="cuda")
out64 = torch.zeros(nbytes // 4096, dtype=torch.int64, device="cuda")
ticket = torch.zeros(256, dtype=torch.int32, device="cuda")
sink = torch.zeros(max(cus * 8 * 256, cus * 1024), dtype=torch.int32, device="cuda")
ts = [torch.zeros(6 * cus * 32, dtype=torch.int64, device="cuda") for _ in range(WINDOW)]


def launch(kernel, k):
    t = ts[k % WINDOW].data_ptr()
    if kernel == "read":
        rc = P.probe_read_stream_stamped(buf.data_ptr(), nbytes, sink.data_ptr(), t, cus * 8, st.cuda_stream)
    elif kernel == "rows":
        rc = P.probe_group_rows_stamped(buf.data_ptr(), n, n // 512, cnt, sink.data_ptr(), t, cus, st.cuda_stream)
    elif STAMPS:
        rc = P.probe_crc_wave_times(buf.data_ptr(), n, cnt, out.data_ptr(), t, ticket.data_ptr(), 32, 0, 0, cus,
                                    st.cuda_stream)
    elif kernel == "c3":
        ck.batch_strided(buf, 4096, 4096, nbytes // 4096, out3, stream=st)
        rc = 0
    elif kernel == "c4":
        ck.batch_strided(buf, 1 << 20, 1 << 20, nbytes >> 20, out3, stream=st)
        rc = 0
    elif kernel == "readp":  # the product's read-only reference kernel (read_stream_kernel, row pattern)
        ck.read_stream(buf, nbytes, sink, sink.numel(), stream=st)
        rc = 0
    elif kernel[:5] in ("c3_64", "c5_64", "c2_64"):  # c5_64: 8 KiB buffers
        if not kernel.endswith("full"):
            ck.set_full_rows64(0, 2)
        elif "ROWS64" in os.environ:  # the full-row kernel with that many rows per step
            ck.set_full_rows64(2, int(os.environ["ROWS64"]))
        else:  # the product's automatic choice
            ck.set_full_rows64(3, 2)
        b = {"c3": 4096, "c5": 8192, "c2": 65536}[kernel[:2]]
        ck.batch64_strided(buf, b, b, nbytes // b, out64, stream=st)
        rc = 0
    else:  # crc or crc@<workgroups>: the product kernel (on a capped grid)
        ck.batch_strided(buf, n, n, cnt, out, stream=st)
        rc = 0
    assert rc == 0, rc


ck.set_lanes_per_buffer(int(os.environ.get("LANES", "0")))  # LANES=8: lane groups of 8 for every batch phase
small = torch.zeros(8192, dtype=torch.uint8, device="cuda")
SVC = any(k.startswith("crcsvc") for k in KERNELS)
if SVC:
    ck.set_device_dispatch(True)
    ck.set_small_service(1000000)
    ck.set_small_service_life(1000000)


def svc_kick(kernel):
    """crcsvc: one routed call after the group is queued, so the service
    launch is resident beside the group's remaining launches."""
    if kernel == "crcsvc":
        ck.crc32c_extend_at(small.data_ptr() + 1, 4096, 0)


def clocks(k_count):
    """In-kernel clock (GHz) per launch of the window from the wave stamps."""
    res = []
    for k in range(k_count):
        v = ts[k].cpu().numpy().reshape(-1, 6).astype(np.int64)
        v = v[v[:, 1] > 0]
        if not len(v):
            return None
        dt = (v[:, 1] - v[:, 0]).astype(np.float64)
        dc = (v[:, 5] - v[:, 4]).astype(np.float64)
        res.append(round(float(np.median(dc / dt)) * 0.1, 3))
    return res


def phase(kernel, label):
    grid_cap = int(kernel.split("@")[1]) if "@" in kernel else 0
    kernel = kernel.split("@")[0]
    from photonlibos_amd._native import lib as _lib
    _lib().photon_crc_set_batch_grid(grid_cap)
    for t in ts:
        t.zero_()
    torch.cuda.synchronize()
    # the driver's window
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(WINDOW)]
    smp = Sampler(board)
    smp.start()
    e0, t0 = board.energy_uj(), time.perf_counter()
    for k in range(WINDOW):
        ev[k][0].record(st)
        launch(kernel, k)
        ev[k][1].record(st)
    svc_kick(kernel)
    st.synchronize()  # the launch stream only: a device-wide wait would wait out a live service
    e1, t1 = board.energy_uj(), time.perf_counter()
    ms = [round(a.elapsed_time(b), 4) for a, b in ev]
    clk = clocks(WINDOW) if (kernel in ("read", "rows") or STAMPS) else None
    # steady state
    e2, t2 = board.energy_uj(), time.perf_counter()
    launches = 0
    while time.perf_counter() - t2 < STEADY_S:
        for k in range(20):
            launch(kernel, k)
        svc_kick(kernel)
        launches += 20
        st.synchronize()
    e3, t3 = board.energy_uj(), time.perf_counter()
    rows = smp.stop()

    def seg(ea, eb, ta, tb, nl):
        r = {"s": round(tb - ta, 4), "GiB_per_s": round(nl * nbytes / (tb - ta) / GIB, 1)}
        pw = [w for (t, w, _) in rows if ta <= t <= tb]
        ck_ = [c for (t, _, c) in rows if ta <= t <= tb]
        if pw:
            r["power_w_mean_sampled"] = round(float(np.mean(pw)), 1)
            r["gfx_clk_mhz_sampled"] = round(float(np.mean(ck_)), 0)
        if ea is not None and eb is not None and eb > ea:
            joules = (eb - ea) * 1e-6
            r["power_w_energy"] = round(joules / (tb - ta), 1)
            r["J_per_GiB"] = round(joules / (nl * nbytes / GIB), 4)
        elif pw:
            r["J_per_GiB_sampled"] = round(float(np.mean(pw)) * (tb - ta) / (nl * nbytes / GIB), 4)
        return r

    res = {"phase": label, "kernel": kernel + ("+stamps" if kernel == "crc" and STAMPS else "") +
           (f"@{grid_cap}" if grid_cap else ""),
           "window": {"launch_ms": ms, "mean_ms": round(float(np.mean(ms)), 4),
                      "frac_of_8TBps": round(nbytes / (float(np.mean(ms)) * 1e-3) / 8e12, 4),
                      **seg(e0, e1, t0, t1, WINDOW)},
           "steady": {"launches": launches, "frac_of_8TBps": round(launches * nbytes / (t3 - t2) / 8e12, 4),
                      **seg(e2, e3, t2, t3, launches)}}
    if clk:
        res["window"]["clock_ghz"] = clk
    if SVC:
        res["service_stats_served_starts_missed"] = ck.small_service_stats()
        ck.set_small_service(0)  # ends a live service before the next phase
        ck.set_small_service(1000000)
    if board.err:
        res["board_note"] = board.err
    print(json.dumps(res), flush=True)


ck.fill_splitmix(buf, n, n, cnt, 0x5EED0001, stream=st)  # as bench.py: data generation, then launches
want = torch.zeros(cnt, dtype=torch.int32, device="cuda")
for i, kern in enumerate(KERNELS):
    if i:
        time.sleep(IDLE_S)
    phase(kern, "fresh process, right after the fill" if i == 0 else f"after {IDLE_S:g} s idle")
    from photonlibos_amd._native import lib as _lib
    _lib().photon_crc_set_batch_grid(0)
    if kern.startswith("crc"):
        ck.batch_strided(buf, n, n, cnt, want, stream=st)
        torch.cuda.synchronize()
        assert torch.equal(out, want), "probe CRCs differ from the product's"
print(json.dumps({"board": getattr(board, "bdf", None), "note": board.err}), flush=True)
