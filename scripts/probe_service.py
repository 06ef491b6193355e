"""Latency of routed crc32c_extend calls on device pointers by size: the
resident small-buffer service (photon_crc_set_small_service) against the
launch path, same buffers, interleaved in blocks (bench-only probe; one JSON
line per size). Usage: python scripts/probe_service.py [--calls 300]."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from photonlibos_amd import checksum as ck  # noqa: E402


def stamps(n):
    """Medians over 200 served calls, in us (100 MHz clock): the poll's round
    trip, seen -> decoded (barrier), -> loaded, -> value (small_value), ->
    done; the spread of the workgroups' seen times; the shader clock (MHz)."""
    import ctypes
    from photonlibos_amd._native import lib
    L = lib()
    L.photon_crc_test_service_area.restype = ctypes.c_void_p
    base = 272
    area = (ctypes.c_uint64 * (base + 16 * 32)).from_address(L.photon_crc_test_service_area())
    keys = ("poll_rt", "seen_to_decoded", "decoded_to_loaded", "loaded_to_column", "column_to_rows", "rows_to_finish",
            "finish_to_wavexor", "wavexor_to_wavefactor", "wavefactor_to_value", "seen_to_done")
    rows = {k: [] for k in keys}
    spread, mhz = [], []
    d = stamps.buf
    for _ in range(200):
        ck.crc32c_extend_at(d.data_ptr() + 1, n, 0)
        t = [[area[base + 16 * w + i] for i in range(16)] for w in range(32)]
        t = [x for x in t if x[1] and x[5]]
        for name, (i, j) in zip(keys, ((0, 1), (1, 2), (2, 3), (3, 8), (8, 9), (9, 10), (10, 11), (11, 12), (12, 4),
                                       (1, 5))):
            rows[name].append(np.median([x[j] - x[i] for x in t]))
        spread.append(max(x[1] for x in t) - min(x[1] for x in t))
        mhz.append(np.median([(x[7] - x[6]) / max(1, x[5] - x[1]) * 100 for x in t]))
    out = {k: round(float(np.median(v)) / 100, 2) for k, v in rows.items()}
    out["seen_spread"] = round(float(np.median(spread)) / 100, 2)
    out["shader_mhz"] = round(float(np.median(mhz)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=300)
    ap.add_argument("--idle-us", type=int, default=20000)
    ap.add_argument("--stamps", action="store_true",
                    help="a -DPCRC_SVC_STAMP=1 build (PHOTON_CRC_LIB): per-request s_memrealtime stamps")
    args = ap.parse_args()
    import torch
    d = torch.empty(1 << 20, dtype=torch.uint8, device="cuda")
    ck.fill_splitmix(d, 1 << 20, 1 << 20, 1, 0x5EED0001)
    torch.cuda.synchronize()
    stamps.buf = d
    ck.set_device_dispatch(True)
    for n in (16, 4096, 32768, 131072, 262143):
        want = ck.crc32c_extend_at(d.data_ptr() + 1, n, 0)
        res = {"bytes": n}
        for mode in ("launch", "service", "launch", "service"):
            ck.set_small_service(args.idle_us if mode == "service" else 0)
            assert ck.crc32c_extend_at(d.data_ptr() + 1, n, 0) == want  # starts the service
            s0 = ck.small_service_stats()[0]
            lat = []
            for _ in range(args.calls):
                t0 = time.perf_counter()
                r = ck.crc32c_extend_at(d.data_ptr() + 1, n, 0)
                lat.append(time.perf_counter() - t0)
                assert r == want
            served = ck.small_service_stats()[0] - s0
            if args.stamps and mode == "service":
                res["stamps_us"] = stamps(n)
            key = mode + ("_2" if mode in res else "")
            res[key] = {"us_median": round(float(np.median(lat)) * 1e6, 2),
                        "us_p10": round(float(np.percentile(lat, 10)) * 1e6, 2), "served": served}
        print(json.dumps(res), flush=True)
    ck.set_small_service(0)
    ck.set_device_dispatch(False)


if __name__ == "__main__":
    main()
