"""The failure contract of the drop-in dispatch (failure row):
Photon's crc32c_extend has no error channel and always computes
(crc.cpp:114-117), so a routed call whose device work fails must still
return the reference's CRC -- recomputed on the host, reported loudly
(stderr, counter, errno, sticky -EIO) -- and never a made-up 0. The batched
C-ABI, which has an error channel, returns the error and computes nothing.
Failures are injected with tuning.h's photon_crc_test_fail_next."""
import numpy as np
import pytest

from photonlibos_amd import checksum as ck
from photonlibos_amd.checksum import CrcError

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available()
    return torch


def test_routed_failure_recomputes_on_host(torch_dev, oracle, capfd):
    torch = torch_dev
    n = (1 << 20) + 13
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    ck.fill_splitmix(d, n, n, 1, 0x5EED0600)
    torch.cuda.synchronize()
    host = d.cpu().numpy()
    before = ck.dispatch_fallbacks()
    ck.set_device_dispatch(True)
    try:
        ok = ck.crc32c_extend_at(d.data_ptr(), n, 5)  # healthy: the device engine
        assert ok == oracle.crc32c(host, 5)
        assert ck.dispatch_fallbacks() == before
        ck.inject_failures(1)
        got = ck.crc32c_extend_at(d.data_ptr(), n, 5)
        assert got == oracle.crc32c(host, 5)  # the right CRC, not 0
        assert ck.dispatch_fallbacks() == before + 1
        ck.inject_failures(1)
        assert ck.crc64ecma_extend_at(d.data_ptr(), n, 9) == oracle.crc64ecma(host, 9)
        # series into a device array and into a host array, each with a failure
        ps, np_ = 4096, n // 4096
        want = oracle.series(host, ps, np_, hw_quirk=True)
        out_d = torch.zeros(np_, dtype=torch.int32, device="cuda")
        ck.inject_failures(1)
        ck.crc32c_series_at(d.data_ptr(), ps, np_, out_d.data_ptr())
        assert list(out_d.cpu().numpy().view(np.uint32)) == want
        out_h = np.zeros(np_, np.uint32)
        ck.inject_failures(1)
        ck.crc32c_series_at(d.data_ptr(), ps, np_, out_h.ctypes.data)
        assert list(out_h) == want
        ck.inject_failures(1)
        assert ck.crc32c_combine_series_at(out_d.data_ptr(), ps, np_) == oracle.crc32c(host[:ps * np_])
        assert ck.dispatch_fallbacks() == before + 5
    finally:
        ck.inject_failures(0)
        with pytest.raises(CrcError) as e:  # the sticky flag reports the failures on the switch
            ck.set_device_dispatch(False)
        assert e.value.code == -5
    err = capfd.readouterr().err
    assert err.count("recomputing on the host") == 5


def test_batch_api_reports_instead_of_computing(torch_dev):
    """The batched C-ABI has an error channel: an injected failure returns
    -EIO and enqueues nothing (the output stays untouched)."""
    torch = torch_dev
    d = torch.zeros(4096 * 4, dtype=torch.uint8, device="cuda")
    out = torch.full((4,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    ck.inject_failures(1)
    with pytest.raises(CrcError) as e:
        ck.batch_strided(d, 4096, 4096, 4, out)
    assert e.value.code == -5 and "injected" in str(e.value)
    torch.cuda.synchronize()
    assert (out == 0x5A5A5A5A).all()
    ck.batch_strided(d, 4096, 4096, 4, out)  # the next call is healthy
    torch.cuda.synchronize()
    assert (out == 0).all()  # raw CRC-32C of zeros is 0
