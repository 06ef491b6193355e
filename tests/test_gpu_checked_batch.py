"""Batched CheckedMessage validation over pinned RPC payloads (SURVEY.md §8(f)
row 1): results equal Crc32Hasher::extend_hash over payload segments then the
message struct (rpc/serialize.h:244-275), checked against the pinned oracle's
chained crc32c_extend. Bit-exact."""
import random

import numpy as np
import pytest

from photonlibos_amd import checksum as ck
from photonlibos_amd.checked import DETACHED_BODY, MessageBatch, PinnedAlloc, TRUSTED
from photonlibos_amd.checksum import CrcError

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available()
    assert ck.device_count() >= 1
    return torch


def _messages(alloc, rng, nmsg, max_seg, seglen_max, struct_len=48):
    """Received messages laid out like a socket readv into pinned buffers:
    payload segments (ragged lengths, odd offsets) + a trailing struct."""
    msgs = []
    blocks = []
    for _ in range(nmsg):
        nseg = rng.randrange(0, max_seg + 1)
        segs = []
        for _ in range(nseg):
            ln = rng.choice([0, 1, 7, 64, 4095, 8192, rng.randrange(1, seglen_max + 1)])
            off = rng.randrange(0, 16)
            addr = alloc.alloc(ln + off + 1)
            blocks.append(addr)
            v = alloc.view(addr, ln + off + 1)
            v[:] = np.frombuffer(rng.randbytes(ln + off + 1), np.uint8)
            segs.append((addr + off, ln))
        saddr = alloc.alloc(struct_len)
        blocks.append(saddr)
        sv = alloc.view(saddr, struct_len)
        sv[:] = np.frombuffer(rng.randbytes(struct_len), np.uint8)
        sv[-4:] = 0  # m_checksum zeroed, as validate_checksum does (serialize.h:268)
        msgs.append((segs, (saddr, struct_len)))
    return msgs, blocks


def _expected(alloc, oracle, segs, body):
    data = [bytes(alloc.view(a, n)) for a, n in segs if n] + [bytes(alloc.view(*body))]
    return oracle.extend_chain(data, 0)


# These tests hash payload + a separate body buffer (DETACHED_BODY); the
# default, the body as the message object itself, is tested below.
@pytest.mark.parametrize("flags", [4, 6])  # zero-copy staging / STAGED copies
def test_validate_batch_matches_oracle(torch_dev, oracle, flags):
    rng = random.Random(11)
    alloc = PinnedAlloc()
    msgs, blocks = _messages(alloc, rng, 300, 9, 20000)
    b = MessageBatch(512, 4096, flags)
    exp = [_expected(alloc, oracle, s, body) for s, body in msgs]
    bad = set(rng.sample(range(len(msgs)), 17))
    for i, (segs, body) in enumerate(msgs):
        claimed = exp[i] ^ (1 << rng.randrange(32)) if i in bad else exp[i]
        assert b.add(segs, body, claimed) == i
    b.submit()
    assert b.wait() == len(bad)
    for i in range(len(msgs)):
        valid, crc = b.result(i)
        assert crc == exp[i]
        assert valid == (i not in bad)
    # reuse after reset; send side (add_checksum): expected 0, read the value
    b.reset()
    for segs, body in msgs[:50]:
        b.add(segs, body)
    b.submit()
    b.wait()
    assert [b.result(i)[1] for i in range(50)] == exp[:50]
    b.close()
    for a in blocks:
        alloc.dealloc(a)
    slab, used = alloc.stats()
    assert used == 0 and slab > 0
    assert alloc.release() == slab


@pytest.mark.parametrize("flags", [4, 6])
def test_payload_corruption_detected(torch_dev, oracle, flags):
    rng = random.Random(12)
    alloc = PinnedAlloc()
    msgs, blocks = _messages(alloc, rng, 64, 8, 8192)
    exp = [_expected(alloc, oracle, s, body) for s, body in msgs]
    # flip one payload bit in every odd message after computing its checksum
    for i, (segs, body) in enumerate(msgs):
        if i % 2:
            a, n = body if not any(n for _, n in segs) else next((a, n) for a, n in segs if n)
            v = alloc.view(a, n)
            v[rng.randrange(n)] ^= 1 << rng.randrange(8)
    b = MessageBatch(64, 1024, flags)
    for i, (segs, body) in enumerate(msgs):
        b.add(segs, body, exp[i])
    b.submit()
    assert b.wait() == 32
    assert [b.result(i)[0] for i in range(64)] == [i % 2 == 0 for i in range(64)]
    b.close()
    for a in blocks:
        alloc.dealloc(a)


def test_device_and_foreign_memory(torch_dev, oracle):
    torch = torch_dev
    # device memory is accepted; ordinary (pageable) host memory is refused loudly
    d = torch.randint(0, 256, (10000,), dtype=torch.uint8, device="cuda")
    host = d.cpu().numpy()
    b = MessageBatch(4, 16)
    b.add([(d.data_ptr(), 10000)], None, oracle.crc32c(host))
    pageable = np.zeros(4096, np.uint8)
    with pytest.raises(CrcError) as e:
        b.add([(pageable.ctypes.data, 4096)])
    assert e.value.code == -14  # EFAULT
    b.submit()
    assert b.wait() == 0
    assert b.result(0) == (True, oracle.crc32c(host))
    with pytest.raises(CrcError):
        b.add([(d.data_ptr(), 1)])  # EBUSY until reset
    b.close()


def test_capacity_and_empty(torch_dev):
    b = MessageBatch(2, 2, TRUSTED)
    b.submit()
    assert b.wait() == 0  # empty batch completes
    b.reset()
    alloc = PinnedAlloc()
    a = alloc.alloc(64)
    b.add([(a, 8), (a + 8, 8)])
    with pytest.raises(CrcError) as e:
        b.add([(a, 8)])
    assert e.value.code == -28  # ENOSPC
    b.add([], None, 0)  # an empty message: checksum 0 == init_value()
    b.submit()
    b.wait()
    assert b.result(1) == (True, 0)
    b.close()
    # a message-object body counts as ONE of max_segments (the
    # zero word standing for its m_checksum takes a slot the batch reserves
    # itself), as before the zero-word change: two bodies fit max_segments 2.
    b = MessageBatch(3, 2)
    bodies = []
    for k in range(2):
        body = alloc.alloc(64)
        v = PinnedAlloc.view(body, 64)
        v[:] = np.arange(64, dtype=np.uint8) + k
        bodies.append(body)
        z = v.copy()
        z[:4] = 0  # validate_checksum hashes the object with m_checksum = 0
        b.add([(a, 8)], (body, 64), oracle_crc32c(z))
    with pytest.raises(CrcError) as e:
        b.add([], (bodies[0], 64), 0)
    assert e.value.code == -28  # ENOSPC: the caller's two segments are used
    b.submit()
    assert b.wait() == 0
    assert b.result(0)[0] and b.result(1)[0]
    b.close()
    for body in bodies:
        alloc.dealloc(body)
    alloc.dealloc(a)


def oracle_crc32c(data):
    from tests import _oracle
    return _oracle.crc32c(data)


def test_resubmit_after_completion_without_wait(torch_dev, oracle):
    """A caller driven by completion (the `done` callback, or a stream sync)
    may resubmit a finished batch without calling wait(): no -EBUSY."""
    torch = torch_dev
    d = torch.randint(0, 256, (8192,), dtype=torch.uint8, device="cuda")
    want = oracle.crc32c(d.cpu().numpy())
    b = MessageBatch(1, 1)
    b.add([(d.data_ptr(), 8192)], None, want)
    for _ in range(3):
        b.submit()
        torch.cuda.synchronize()  # finished, never waited on
    assert b.wait() == 0 and b.result(0) == (True, want)
    b.close()


def test_segment_past_its_allocation_is_refused(torch_dev):
    """[p, p+n) must lie inside p's allocation: a segment running past the end
    of a hipMalloc'd block is -EFAULT, not a read of unmapped memory."""
    import ctypes
    from photonlibos_amd._native import lib
    p = ctypes.c_void_p()
    assert lib().photon_crc_device_alloc(ctypes.byref(p), 4096) == 0
    try:
        b = MessageBatch(2, 2)
        b.add([(p.value, 4096)])            # the whole block: fine
        with pytest.raises(CrcError) as e:
            b.add([(p.value + 16, 4096)])   # 16 bytes past the end
        assert e.value.code == -14
        b.close()
    finally:
        lib().photon_crc_device_free(p.value)


def _cm_fixture():
    import json
    import os
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "checked_message.json")) as f:
        return json.load(f)["messages"]


@pytest.mark.parametrize("flags", [4, 6])
def test_batch_matches_reference_checked_message(torch_dev, flags):
    """The device batch against the REFERENCE's own CheckedMessage template
    (serialize.h:239-279 run by oracle/ref/checked_message_fixtures.cpp, whose
    body is a buffer separate from the CheckedMessage object: DETACHED_BODY):
    every checksum add_checksum stored, every validate_checksum verdict."""
    from photonlibos_amd import datagen
    msgs = _cm_fixture()
    alloc = PinnedAlloc()
    blocks, specs = [], []
    for m in msgs:
        segs = []
        for seed, n, off in m["segs"]:
            a = alloc.alloc(n + off + 1)
            blocks.append(a)
            alloc.view(a + off, n)[:] = datagen.stream_bytes(seed, n) if n else []
            segs.append((a + off, n))
        b = alloc.alloc(m["body"][1])
        blocks.append(b)
        v = alloc.view(b, m["body"][1])
        v[:] = datagen.stream_bytes(*m["body"])
        v[-4:] = 0
        specs.append((segs, (b, m["body"][1])))
    for claim in ("right", "bad"):
        batch = MessageBatch(len(msgs), 2048, flags)
        for k, (m, (segs, body)) in enumerate(zip(msgs, specs)):
            c = m["checksum"] if claim == "right" else m["checksum"] ^ (1 << (k % 32))
            batch.add(segs, body, c)
        batch.submit()
        nbad = batch.wait()
        for k, m in enumerate(msgs):
            valid, crc = batch.result(k)
            assert crc == m["checksum"], k
            assert valid == (m["validate"] if claim == "right" else m["validate_bad_claim"]), (k, claim)
        assert nbad == (0 if claim == "right" else len(msgs))
        batch.close()
    for a in blocks:
        alloc.dealloc(a)


def test_resubmit_while_done_callback_runs_is_busy(torch_dev, oracle):
    """done_ev fires before the `done` host function runs. While a
    slow callback is still running (and may read the verdicts), a resubmit or
    reset from another thread is -EBUSY instead of overwriting them; result()
    inside the callback sees the settled batch; once the callback has
    returned, the batch resubmits."""
    import threading
    import time
    torch = torch_dev
    d = torch.randint(0, 256, (8192,), dtype=torch.uint8, device="cuda")
    want = oracle.crc32c(d.cpu().numpy())
    b = MessageBatch(1, 1)
    b.add([(d.data_ptr(), 8192)], None, want)
    entered, seen = threading.Event(), []

    def slow_done():
        seen.append(b.result(0))  # settled before the callback: no HIP call needed
        entered.set()
        time.sleep(0.5)

    b.submit(done=slow_done)
    assert entered.wait(30)
    with pytest.raises(CrcError) as e:
        b.submit()
    assert e.value.code == -16  # EBUSY: the callback has not returned
    with pytest.raises(CrcError) as e:
        b.reset()
    assert e.value.code == -16
    assert seen == [(True, want)]
    deadline = time.time() + 30
    while True:  # the callback returns after its sleep
        try:
            b.submit()
            break
        except CrcError as err:
            assert err.code == -16 and time.time() < deadline
            time.sleep(0.05)
    assert b.wait() == 0 and b.result(0) == (True, want)
    b.close()


def test_segment_past_its_pinned_block_is_refused(torch_dev):
    """a segment in pinned-pool memory must stay inside its own
    live IOAlloc block (not merely inside the 64 MiB slab)."""
    alloc = PinnedAlloc()
    a = alloc.alloc(4096)        # a 4 KiB-class block
    nb = alloc.alloc(4096)       # a neighbour, possibly the next block
    try:
        b = MessageBatch(4, 4)
        b.add([(a, 4096)])                  # the whole block: fine
        b.add([(a + 100, 3996)])            # ends exactly at the block end: fine
        with pytest.raises(CrcError) as e:
            b.add([(a + 16, 4096)])         # 16 bytes past the end of its block
        assert e.value.code == -14
        freed, nb = nb, None
        alloc.dealloc(freed)
        with pytest.raises(CrcError) as e:  # a freed block is not the caller's memory any more
            b.add([(freed, 64)])
        assert e.value.code == -14
        b.close()
    finally:
        alloc.dealloc(a)
        if nb:
            alloc.dealloc(nb)


def test_ioalloc_binding_against_reference_headers(torch_dev):
    """INTEGRATION.md §2.1 compiled verbatim against the
    reference's io-alloc.h / iovector.h / serialize.h (oracle/ref/
    ioalloc_binding.cpp, built in the build container into oracle/_ref/).
    On this box it builds 200 received requests with reference
    IOVector::push_back(size) allocating from photon_crc_pinned_allocate
    (rpc/rpc.cpp:216-220, 279), runs the reference CheckedMessage
    add_checksum / validate_checksum over the drop-in, then the §2.1 receive
    path hands every message to the GPU batch. Checked: the reference's
    checksums equal the committed fixture (tests/golden/ioalloc_binding.json,
    made over Photon's own crc.cpp), the batch reproduces every checksum, its
    verdicts flag exactly the corrupted claims, and every pinned block went
    back to the pool."""
    import json
    import os
    import subprocess
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(repo, "oracle", "_ref", "ioalloc_dropin")
    assert os.path.exists(exe), "oracle/_ref/ioalloc_dropin not built (make -C oracle/ref in the build container)"
    r = subprocess.run([exe, "pinned", "200"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = json.loads(r.stdout)
    with open(os.path.join(repo, "tests", "golden", "ioalloc_binding.json")) as f:
        gold = json.load(f)["messages"]
    assert got["pinned_in_use_bytes"] > 0 and got["pinned_in_use_after"] == 0
    assert len(got["messages"]) == len(gold) == 200
    for m, (g, w) in enumerate(zip(got["messages"], gold)):
        assert (g["lens"], g["seeds"], g["checksum"], g["validate"]) == \
            (w["lens"], w["seeds"], w["checksum"], w["validate"]), m
        assert g["batch_crc"] == w["checksum"], m
        assert g["batch_valid"] == (0 if m % 7 == 3 else 1), m



def test_trusted_device_memory_object_body(torch_dev, oracle):
    """a TRUSTED batch whose message object lives in device memory
    (no host write into it: the batch masks m_checksum itself)."""
    torch = torch_dev
    rng = random.Random(23)
    objs = torch.from_numpy(np.frombuffer(rng.randbytes(64 * 48), np.uint8).copy()).cuda()
    host = objs.cpu().numpy()
    b = MessageBatch(64, 128, TRUSTED)
    want = []
    for i in range(64):
        z = bytearray(host[48 * i:48 * i + 48].tobytes())
        z[:4] = b"\0\0\0\0"
        want.append(oracle.crc32c(bytes(z)))
        assert b.add([], (objs.data_ptr() + 48 * i, 48), want[-1] ^ (i % 2)) == i
    b.submit()
    assert b.wait() == 32
    for i in range(64):
        assert b.result(i) == (i % 2 == 0, want[i]), i
    assert np.array_equal(objs.cpu().numpy(), host)  # the objects were not written
    # a 4-byte object is m_checksum alone: crc32c of 4 zero bytes
    b.reset()
    b.add([], (objs.data_ptr(), 4), oracle.crc32c(bytes(4)))
    b.submit()
    assert b.wait() == 0
    b.close()


def _object_messages(alloc, rng, nmsg):
    """Photon's layout: payload segments, then the message struct whose first
    4 bytes are m_checksum (the CheckedMessage<> base), 48 bytes."""
    msgs, blocks = [], []
    for _ in range(nmsg):
        segs = []
        for _ in range(rng.randrange(0, 6)):
            ln = rng.randrange(1, 9000)
            a = alloc.alloc(ln)
            blocks.append(a)
            alloc.view(a, ln)[:] = np.frombuffer(rng.randbytes(ln), np.uint8)
            segs.append((a, ln))
        t = alloc.alloc(48)
        blocks.append(t)
        alloc.view(t, 48)[:] = np.frombuffer(rng.randbytes(48), np.uint8)
        msgs.append((segs, (t, 48)))
    return msgs, blocks


def _photon_checksum(alloc, oracle, segs, body):
    """The reference's value for a message object (oracle.checked_message_object:
    the in-place accumulation of serialize.h:244-275, 462-463)."""
    return oracle.checked_message_object([bytes(alloc.view(a, n)) for a, n in segs], bytes(alloc.view(*body)))


@pytest.mark.parametrize("flags", [0, 2])
def test_message_object_body_matches_reference_semantics(torch_dev, oracle, flags):
    """Default batches: the body is the message object (t->validate_checksum(
    iov, t, sizeof(*t)), serialize.h:462-463). The batch equals the
    reference's in-place accumulation computed step by step, which equals
    crc32c of the struct with m_checksum zeroed: a corrupted payload is NOT
    detected (as in Photon), a corrupted struct field is; DETACHED_BODY over
    the same messages covers the payload."""
    rng = random.Random(21)
    alloc = PinnedAlloc()
    msgs, blocks = _object_messages(alloc, rng, 120)
    want = [_photon_checksum(alloc, oracle, s, body) for s, body in msgs]
    for (s, (t, n)), w in zip(msgs, want):
        z = bytearray(alloc.view(t, n))
        z[:4] = b"\0\0\0\0"
        assert w == oracle.crc32c(bytes(z))  # the identity the batch relies on
    # corrupt one payload byte of every 3rd message that has a payload, one
    # struct byte (past m_checksum) of every 5th
    pay_bad, body_bad = set(), set()
    for i, (segs, (t, n)) in enumerate(msgs):
        if i % 3 == 0 and segs:
            a, ln = segs[0]
            alloc.view(a, ln)[rng.randrange(ln)] ^= 0x40
            pay_bad.add(i)
        if i % 5 == 0:
            alloc.view(t, n)[4 + rng.randrange(44)] ^= 0x01
            body_bad.add(i)
    b = MessageBatch(len(msgs), 4096, flags)
    claims = []
    for i, (segs, body) in enumerate(msgs):
        claims.append(rng.randbytes(4))
        alloc.view(body[0], 4)[:] = np.frombuffer(claims[-1], np.uint8)  # m_checksum holds the claim
        assert b.add(segs, body, want[i]) == i
    b.submit()
    assert b.wait() == len(body_bad)
    for i, (segs, body) in enumerate(msgs):
        assert b.result(i)[0] == (i not in body_bad), i
        # the batch reads m_checksum as 0 but never writes the caller's object
        assert bytes(alloc.view(body[0], 4)) == claims[i], i
    # resubmit after the bodies were refilled (new fields AND a new m_checksum
    # claim): the word is masked again, the verdicts follow the new contents
    for i, (segs, (t, n)) in enumerate(msgs):
        alloc.view(t, n)[:] = np.frombuffer(rng.randbytes(n), np.uint8)
    want2 = [_photon_checksum(alloc, oracle, s, body) for s, body in msgs]
    b.submit()
    b.wait()
    for i in range(len(msgs)):
        assert b.result(i)[1] == want2[i], i
    b.close()
    # the same messages, payload hashed (DETACHED_BODY: payload then struct)
    d = MessageBatch(len(msgs), 4096, flags | DETACHED_BODY)
    for i, (segs, body) in enumerate(msgs):
        d.add(segs, body, want[i])
    d.submit()
    d.wait()
    for i, (segs, body) in enumerate(msgs):
        data = [bytes(alloc.view(a, n)) for a, n in segs] + [bytes(alloc.view(*body))]
        assert d.result(i)[1] == oracle.extend_chain(data, 0), i
    d.close()
    for a in blocks:
        alloc.dealloc(a)
