"""Soak of the resident small-buffer services (bench-only):
for SECONDS, routed crc32c_extend / crc64ecma_extend calls of random size
(up to 4 MiB: the service's small and rows forms, the mid layout),
offset and seed on device buffers that are rewritten between calls (a fill
kernel, a device-to-device copy on another stream, a host-to-device copy),
beside CRC32C and CRC-64 batch launches on another stream (the CRC-64 ones
end the services), with random idle gaps around the services' 200 us idle
time (their end / restart races). Every routed result is checked against the
host engine on a host copy of the same bytes; the batches' first and last
CRCs too. --flip: a further thread flips the service's doorbell (BAR /
pinned), its life (100 us .. 5 ms) and turns it off and on, every 2-50 ms,
while the calls run. One JSON line at the end.
Usage: python scripts/soak_service.py [--seconds 60] [--threads 1] [--flip]"""
import argparse
import json
import os
import random
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from photonlibos_amd import checksum as ck  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=60.0)
    ap.add_argument("--threads", type=int, default=1)
    ap.add_argument("--flip", action="store_true")
    args = ap.parse_args()
    ck.set_device_dispatch(True)
    nb, count = 64 << 10, 1024
    big = torch.empty(nb * count, dtype=torch.uint8, device="cuda")
    ck.fill_splitmix(big, nb, nb, count, 0x50A4)
    out32 = torch.zeros(count, dtype=torch.int32, device="cuda")
    out64 = torch.zeros(count, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    hb = big.cpu().numpy()
    want32 = (ck.crc32c_extend(hb[:nb].tobytes(), 0), ck.crc32c_extend(hb[-nb:].tobytes(), 0))
    want64 = (ck.crc64ecma(hb[:nb].tobytes(), 0), ck.crc64ecma(hb[-nb:].tobytes(), 0))
    side = torch.cuda.Stream()
    stats = {"calls": 0, "bad": 0, "batches32": 0, "batches64": 0, "bad_batches": 0}
    lock = threading.Lock()
    stop = time.perf_counter() + args.seconds

    def worker(t):
        rng = random.Random(1000 + t)
        cap = (4 << 20) + 64  # the small service (<= 256 KiB), its rows form (<= 2 MiB), the mid layout
        buf = torch.zeros(cap, dtype=torch.uint8, device="cuda")
        src = torch.zeros(cap, dtype=torch.uint8, device="cuda")
        stream = torch.cuda.Stream()
        k = 0
        while time.perf_counter() < stop:
            k += 1
            how = rng.randrange(3)
            with torch.cuda.stream(stream):
                if how == 0:
                    ck.fill_splitmix(buf, cap, cap, 1, rng.getrandbits(40), stream=stream)
                elif how == 1:
                    ck.fill_splitmix(src, cap, cap, 1, rng.getrandbits(40), stream=stream)
                    buf.copy_(src)
                else:
                    buf.copy_(torch.from_numpy(np.random.default_rng(k).integers(0, 256, cap, dtype=np.uint8)))
            stream.synchronize()
            host = buf.cpu().numpy()
            for _ in range(rng.randrange(1, 6)):
                off = rng.randrange(16)
                n = rng.choice([rng.randrange(1, 64), rng.randrange(1, 8192), rng.randrange(1, 256 << 10),
                                rng.randrange(1, cap - 64)])
                seed = rng.getrandbits(64)
                if rng.randrange(2):
                    got = ck.crc32c_extend_at(buf.data_ptr() + off, n, seed & 0xFFFFFFFF)
                    ok = got == ck.crc32c_extend(host[off:off + n].tobytes(), seed & 0xFFFFFFFF)
                else:
                    got = ck.crc64ecma_extend_at(buf.data_ptr() + off, n, seed)
                    ok = got == ck.crc64ecma(host[off:off + n].tobytes(), seed)
                with lock:
                    stats["calls"] += 1
                    stats["bad"] += 0 if ok else 1
            if rng.randrange(4) == 0:
                time.sleep(rng.choice([50e-6, 150e-6, 200e-6, 250e-6, 1e-3]))

    def batches():
        rng = random.Random(7)
        while time.perf_counter() < stop:
            if rng.randrange(3) == 0:
                ck.batch64_strided(big, nb, nb, count, out64, stream=side.cuda_stream)
                side.synchronize()
                g = out64.cpu().numpy().view(np.uint64)
                ok = (int(g[0]), int(g[-1])) == want64
                key = "batches64"
            else:
                ck.batch_strided(big, nb, nb, count, out32, stream=side.cuda_stream)
                side.synchronize()
                g = out32.cpu().numpy().view(np.uint32)
                ok = (int(g[0]), int(g[-1])) == want32
                key = "batches32"
            with lock:
                stats[key] += 1
                stats["bad_batches"] += 0 if ok else 1
            time.sleep(rng.choice([0, 1e-4, 1e-3, 5e-3]))

    flips = [0]

    def flipper():
        rng = random.Random(11)
        while time.perf_counter() < stop:
            what = rng.randrange(4)
            if what == 0:
                ck.set_service_doorbell(rng.randrange(2) == 1)
            elif what == 1:
                ck.set_small_service_life(rng.choice([100, 500, 2000, 5000]))
            elif what == 2:
                ck.set_small_service(0)
                ck.set_small_service(200)
            else:
                t0 = time.perf_counter()
                torch.cuda.synchronize()  # a device-wide wait beside the routed calls
                with lock:
                    stats["sync_max_ms"] = max(stats.get("sync_max_ms", 0.0), (time.perf_counter() - t0) * 1e3)
            flips[0] += 1
            time.sleep(rng.choice([2e-3, 10e-3, 50e-3]))
        ck.set_service_doorbell(True)
        ck.set_small_service_life(2000)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(args.threads)] + [threading.Thread(target=batches)]
    if args.flip:
        th.append(threading.Thread(target=flipper))
    for x in th:
        x.start()
    for x in th:
        x.join()
    served, starts, missed = ck.small_service_stats()
    stats.update({"served": served, "starts": starts, "missed": missed, "deferred": ck.small_service_deferred(),
                  "fallbacks": ck.dispatch_fallbacks(), "seconds": args.seconds, "threads": args.threads,
                  "flips": flips[0]})
    print(json.dumps(stats), flush=True)
    ck.set_device_dispatch(False)
    sys.exit(0 if stats["bad"] == 0 and stats["bad_batches"] == 0 and stats["fallbacks"] == 0 else 1)


if __name__ == "__main__":
    main()
