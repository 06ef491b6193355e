"""C++ consumers of the drop-in headers and the C-ABI (tests/cpp/).

`dropin_test` is compiled against include/photon/common/checksum/*.h and
linked with libphoton_checksum.so the way Photon would link it; it re-runs the
checks of the reference's common/checksum/test/test_checksum.cpp:28-308
(golden file, sw/hw differential, combine/series/trim) with no Python in the
loop. `gpu_batch_example` drives the batched C-ABI from plain C++ built with g++ and
no HIP headers (the library's runtime shim: streams, device memory, copies,
completion callback).
"""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "bin")


def _golden_files(tmp_path):
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "checksum_in.json")))
    alpha = "abcdefghijklmnopqrstuvwxyz"
    lines_in, lines_64 = [], []
    for k, (c32, c64) in enumerate(zip(g["crc32c"], g["crc64ecma"]), 1):
        s = (alpha * (k // 26 + 1))[:k]
        lines_in.append(f"{c32} {s}")
        lines_64.append(str(c64))
    p_in, p_64 = tmp_path / "checksum.in", tmp_path / "checksum.crc64"
    p_in.write_text("\n".join(lines_in) + "\n")
    p_64.write_text("\n".join(lines_64) + "\n")
    return str(p_in), str(p_64)


def test_cpp_dropin_consumer(tmp_path):
    exe = os.path.join(BIN, "dropin_test")
    assert os.path.exists(exe), "build with make -C photonlibos_amd/csrc"
    p_in, p_64 = _golden_files(tmp_path)
    r = subprocess.run([exe, p_in, p_64], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "512 golden cases, 0 failures" in r.stdout


@pytest.mark.gpu
def test_cpp_gpu_batch_example():
    exe = os.path.join(BIN, "gpu_batch_example")
    assert os.path.exists(exe)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 mismatches" in r.stdout and "callback ran 1 time" in r.stdout


@pytest.mark.gpu
def test_cpp_rpc_batch_example():
    exe = os.path.join(BIN, "rpc_batch_example")
    assert os.path.exists(exe)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 wrong verdicts" in r.stdout


def test_host_engines_under_asan(tmp_path):
    # Host code only (no GPU sanitizer on this pool): the drop-in engines
    # compiled with -fsanitize=address,undefined and driven at every length
    # and misalignment.
    import shutil
    gxx = shutil.which("g++")
    if not gxx:
        pytest.skip("g++ not available")
    exe = str(tmp_path / "asan_host_engines")
    src = [os.path.join(ROOT, "tests", "cpp", "asan_host_engines.cpp"),
           os.path.join(ROOT, "photonlibos_amd", "csrc", "crc32c_cpu.cpp"),
           os.path.join(ROOT, "photonlibos_amd", "csrc", "crc64_cpu.cpp")]
    subprocess.run([gxx, "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-fno-omit-frame-pointer", "-I" + os.path.join(ROOT, "include")] + src + ["-o", exe],
                   check=True, timeout=300)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "asan64: 0 mismatches" in r.stdout


@pytest.mark.gpu
def test_cpp_concurrent_submitters():
    """16 threads on their own streams submit mixed batches while a 17th
    flips every tuning knob; every result equals the oracle's (reentrancy,
    crc.cpp:126-137)."""
    exe = os.path.join(BIN, "concurrency_test")
    assert os.path.exists(exe)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 mismatches, 0 errors" in r.stdout


def test_multi_device_plumbing_simulated_8_devices():
    """the shard plan and per-device switching behind
    photon_crc32c_host_batch_strided_multi / _batch_strided_shards /
    _extend_spans, and the per-device table images, run against a simulated
    runtime of 8 devices (tests/cpp/multi_device_test.cpp, CPU only): slices
    contiguous, disjoint, complete and balanced for 1-8 devices; every slice's
    work runs with its own device current and reads its own device's image;
    failures name their device; the caller's device is restored."""
    exe = os.path.join(BIN, "multi_device_test")
    assert os.path.exists(exe), "build with make -C photonlibos_amd/csrc"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr
