#!/usr/bin/env python3
"""Writes tests/golden/checked_message.json: the reference's own
rpc/serialize.h CheckedMessage<Crc32Hasher>::add_checksum / validate_checksum
(serialize.h:239-279) run on 160 seeded messages, by
oracle/ref/checked_message_fixtures.cpp built twice (oracle/ref/Makefile):
over Photon's own crc.cpp and over this library's drop-in. Both must print
the same fixtures. Build-container only (needs /root/reference):
    make -C oracle/ref && python tests/golden/gen_checked_message.py
The fixture holds values only: per message the (stream seed, length,
alignment offset) of each payload segment, the body (the serialized struct,
last 4 bytes = m_checksum zeroed) spec, the checksum add_checksum stored and
validate_checksum's verdicts for the right claim and a one-bit-off claim."""
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.path.join(HERE, "..", "..", "oracle", "_ref")


def main():
    outs = [subprocess.check_output([os.path.join(REF, b), "160"], text=True)
            for b in ("cm_fixtures_ref", "cm_fixtures_dropin")]
    assert outs[0] == outs[1], "serialize.h over Photon's crc.cpp and over the drop-in disagree"
    d = json.loads(outs[0])
    d["_source"] = ("reference rpc/serialize.h:239-279 CheckedMessage<Crc32Hasher> over reference IOVector "
                    "(common/iovector.h), compiled with Photon's common/checksum/crc.cpp AND with "
                    "libphoton_checksum.so's drop-in header (identical output); "
                    "oracle/ref/checked_message_fixtures.cpp")
    with open(os.path.join(HERE, "checked_message.json"), "w") as f:
        json.dump(d, f, separators=(",", ":"))
    print(len(d["messages"]), "messages")


if __name__ == "__main__":
    main()
