"""HIP vDMA target/initiator (include/photon_crc/vdma_hip.h) behind PhotonLibOS's
vDMA interface (net/vdma.h:13-77; behavioural model net/vdma/shm.cpp), driven
by the C++ program tests/cpp/vdma_test.cpp.

CPU: the library exports the factories and the batch helper with the C++
signatures the header declares; the program fails loudly without a GPU.
GPU: the single-process checks of the reference's net/test/test-vdma.cpp
(alloc/dealloc order, ids, exhaustion, 16 threads), register_memory, and
checksums of vDMA buffers vs the drop-in host engine; then a target and an
initiator in two processes sharing HBM through the published IPC handle:
the initiator's CRCs of the mapped buffers equal the target's, and bytes the
initiator writes are what the target checksums afterwards.
"""
import os
import re
import subprocess

import pytest

from photonlibos_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "bin", "vdma_test")


def test_vdma_symbols_exported():
    out = subprocess.check_output(["nm", "-DC", "--defined-only", _native.LIB_PATH], text=True)
    for sig in ("photon::new_hip_vdma_target(char const*, unsigned long, unsigned long, int)",
                "photon::new_hip_vdma_initiator(char const*, unsigned long)",
                "photon::crc32c_vdma_batch(photon::vDMABuffer* const*, unsigned long const*, unsigned long, "
                "unsigned int*, void*)"):
        assert sig in out, sig


def test_vdma_header_matches_reference_interface():
    # The interface header declares the reference's classes and virtual
    # methods in the reference's order (net/vdma.h:13-77).
    txt = open(os.path.join(ROOT, "include", "photon", "net", "vdma.h")).read()
    methods = re.findall(r"virtual [^;]*?(\w+)\([^)]*\)[^;]*= 0;", txt)
    assert methods == ["id", "address", "buf_size", "type_code", "is_registered", "is_valid",
                       "alloc", "dealloc", "register_memory", "unregister_memory",
                       "map", "unmap", "write", "read"]


@pytest.mark.skipif(os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK), reason="a GPU is present")
def test_vdma_program_fails_loudly_without_gpu():
    assert os.path.exists(EXE), "build with make -C photonlibos_amd/csrc"
    r = subprocess.run([EXE, "local"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "no device" in r.stderr


@pytest.mark.gpu
def test_vdma_local():
    r = subprocess.run([EXE, "local"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "vdma local: 0 failures" in r.stdout


@pytest.mark.gpu
def test_vdma_target_and_initiator_processes():
    name = f"/photon_crc_vdma_{os.getpid()}"
    tgt = subprocess.Popen([EXE, "target", name], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                           stderr=subprocess.PIPE, text=True)
    try:
        ids, crcs = [], []
        for _ in range(4):
            line = tgt.stdout.readline().strip()
            if line == "ready":
                break
            _, k, ident, crc = line.split()
            ids.append(ident)
            crcs.append(crc)
        assert len(ids) == 3, tgt.stderr.read() if tgt.poll() is not None else ids
        r = subprocess.run([EXE, "initiator", name] + ids, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stdout + r.stderr
        got = dict(re.findall(r"initiator-crc (\d) (\w+)", r.stdout))
        assert [got[str(k)] for k in range(3)] == crcs
        wrote = re.search(r"initiator-wrote2 (\w+)", r.stdout).group(1)
        tgt.stdin.write("check\n")
        tgt.stdin.flush()
        line = tgt.stdout.readline().split()
        assert line[:2] == ["target-crc2", "0"] and line[2] == wrote, line
        tgt.stdin.write("quit\n")
        tgt.stdin.flush()
        assert tgt.wait(timeout=60) == 0
    finally:
        if tgt.poll() is None:
            tgt.kill()
            tgt.wait()
    assert not os.path.exists("/dev/shm" + name)  # the target unlinked its handle
