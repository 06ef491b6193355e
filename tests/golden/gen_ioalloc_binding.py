#!/usr/bin/env python3
"""Writes tests/golden/ioalloc_binding.json: 200 seeded RPC messages built the
way the reference's RPC server receives them -- reference IOVectors whose
buffers come from IOVector::push_back(size) through an IOAlloc
(common/iovector.h:389-397, io-alloc.h:31-85, rpc/rpc.cpp:216-220, 279) --
with the reference's CheckedMessage<Crc32Hasher> add_checksum /
validate_checksum (rpc/serialize.h:239-279). oracle/ref/ioalloc_binding.cpp,
built twice by oracle/ref/Makefile: over Photon's own crc.cpp and over this
library's drop-in; run here with IOAlloc's default allocator (no GPU in the
build container), both builds must print the same. On the GPU box the
-m gpu test runs the drop-in build with the INTEGRATION.md §2.1 pinned pool
and the GPU batch and checks it against this fixture.
Build-container only (needs /root/reference):
    make -C oracle/ref && python tests/golden/gen_ioalloc_binding.py
Values only: per message the payload segment lengths and stream seeds, the
stored checksum and validate_checksum's verdict."""
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.path.join(HERE, "..", "..", "oracle", "_ref")


def main():
    outs = [subprocess.check_output([os.path.join(REF, b), "malloc", "200"], text=True)
            for b in ("ioalloc_ref", "ioalloc_dropin")]
    assert outs[0] == outs[1], "the reference template over Photon's crc.cpp and over the drop-in disagree"
    d = json.loads(outs[0])
    msgs = [{"lens": m["lens"], "seeds": m["seeds"], "checksum": m["checksum"], "validate": m["validate"]}
            for m in d["messages"]]
    assert all(m["validate"] for m in msgs)
    out = {"messages": msgs,
           "_source": "reference IOVector::push_back(size) via IOAlloc + rpc/serialize.h:239-279 "
                      "CheckedMessage<Crc32Hasher>, compiled with Photon's common/checksum/crc.cpp AND with "
                      "libphoton_checksum.so's drop-in header (identical output); oracle/ref/ioalloc_binding.cpp"}
    with open(os.path.join(HERE, "ioalloc_binding.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print(len(msgs), "messages")


if __name__ == "__main__":
    main()
