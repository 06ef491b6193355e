"""Mid layout vs long kernel (bench-only): for spans of 512 KiB
.. 32 MiB at buf+1, photon_crc32c_extend_device / photon_crc64ecma_extend_device
with the mid kernel on and off (photon_crc_set_mid_kernel), interleaved:
  call_us   one call + stream sync, median of 200;
  queued_us 200 calls queued back to back on one stream, per call (the
            kernels' own time plus launch gaps);
and the routed crc32c_extend / crc64ecma_extend on the same pointer, service
off (median of 200). Every
result is checked against the host engine. One JSON line per size and CRC.
Usage: python scripts/probe_mid.py"""
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from photonlibos_amd import checksum as ck  # noqa: E402


def main():
    sizes = [(512 << 10), 1 << 20, 2 << 20, 4 << 20, 8 << 20, 16 << 20, (32 << 20) - 16]
    cap = (32 << 20) + 64
    d = torch.empty(cap, dtype=torch.uint8, device="cuda")
    ck.fill_splitmix(d, cap, cap, 1, 0x3D1D)
    torch.cuda.synchronize()
    host = d.cpu().numpy()
    st = torch.cuda.Stream()
    reps = 200
    ck.set_small_service(0)  # routed calls: the launch path (the service takes up to 2 MiB)
    for crc64 in (False, True):
        out = torch.zeros(reps, dtype=torch.int64 if crc64 else torch.int32, device="cuda")
        for n in sizes:
            want = ck.crc64ecma(host[1:1 + n].tobytes(), 7) if crc64 else ck.crc32c_extend(host[1:1 + n].tobytes(), 7)
            row = {"crc": "crc64ecma" if crc64 else "crc32c", "bytes": n}
            for mid in (True, False, True, False):
                ck.set_mid_kernel(mid)
                key = "mid" if mid else "long"

                def call(k):
                    if crc64:
                        ck.extend64_device(d.data_ptr() + 1, n, out[k:k + 1], seed=7, stream=st)
                    else:
                        ck.extend_device(d.data_ptr() + 1, n, 7, out[k:k + 1], stream=st)

                call(0)
                st.synchronize()
                ts = []
                for k in range(reps):
                    t0 = time.perf_counter()
                    call(k)
                    st.synchronize()
                    ts.append(time.perf_counter() - t0)
                t0 = time.perf_counter()
                for k in range(reps):
                    call(k)
                st.synchronize()
                queued = (time.perf_counter() - t0) / reps
                got = out.cpu().numpy().view(np.uint64 if crc64 else np.uint32)
                ok = all(int(x) == want for x in got)
                ck.set_device_dispatch(True)
                rt = []
                for k in range(reps):
                    t0 = time.perf_counter()
                    r = ck.crc64ecma_extend_at(d.data_ptr() + 1, n, 7) if crc64 else \
                        ck.crc32c_extend_at(d.data_ptr() + 1, n, 7)
                    rt.append(time.perf_counter() - t0)
                    ok = ok and r == want
                ck.set_device_dispatch(False)
                row[key + "_call_us"] = round(statistics.median(ts) * 1e6, 2)
                row[key + "_queued_us"] = round(queued * 1e6, 2)
                row[key + "_routed_us"] = round(statistics.median(rt) * 1e6, 2)
                row[key + "_ok"] = ok
            print(json.dumps(row), flush=True)
    ck.set_mid_kernel(True)
    ck.set_small_service(200)


if __name__ == "__main__":
    main()
