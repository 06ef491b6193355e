#!/usr/bin/env python3
"""Regenerate the committed golden fixtures from the reference (run HERE only;
/root/reference does not exist on the GPU box).

  checksum_in.json  <- the reference's own test data files
                       common/checksum/test/checksum.in   (512 x "<crc32c> <string>")
                       common/checksum/test/checksum.crc64 (512 x crc64ecma)
                       (loader: common/checksum/test/test_checksum.cpp:28-45).
                       Only the CRC values are kept; string k is the first k
                       characters of the cyclic alphabet (checked below).
  ref_vectors.json  <- `oracle/_ref/ref_harness vectors`: the reference's own
                       crc.cpp / crc_tables.cpp, compiled unmodified by
                       oracle/ref/Makefile, run on seeded splitmix64 inputs.

Usage: python tests/golden/gen_ref_vectors.py
"""
import json
import os
import string
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("PHOTON_REFERENCE", "/root/reference")
TESTDIR = os.path.join(REF, "common/checksum/test")


def checksum_in():
    crc32, strings = [], []
    with open(os.path.join(TESTDIR, "checksum.in")) as f:
        for line in f:
            if line.strip():
                c, s = line.split()
                crc32.append(int(c))
                strings.append(s)
    with open(os.path.join(TESTDIR, "checksum.crc64")) as f:
        crc64 = [int(x) for x in f.read().split()]
    alpha = string.ascii_lowercase * 40
    for k, s in enumerate(strings):
        if s != alpha[: k + 1]:
            sys.exit(f"checksum.in line {k + 1}: string is not the alphabet prefix")
    assert len(crc32) == len(crc64) == 512
    return {
        "source": "common/checksum/test/checksum.in + checksum.crc64 (reference test data)",
        "strings": "case k (1-based) = first k chars of 'abc...z' repeated",
        "crc32c": crc32,
        "crc64ecma": crc64,
    }


def main():
    with open(os.path.join(HERE, "checksum_in.json"), "w") as f:
        json.dump(checksum_in(), f)
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle/ref")])
    out = subprocess.check_output([os.path.join(REPO, "oracle/_ref/ref_harness"), "vectors"])
    data = json.loads(out)
    data["_source"] = ("reference common/checksum/crc.cpp + crc_tables.cpp built by oracle/ref/Makefile; "
                       "inputs: splitmix64 streams (see photonlibos_amd/datagen.py)")
    with open(os.path.join(HERE, "ref_vectors.json"), "w") as f:
        json.dump(data, f, separators=(",", ":"))
    print("wrote checksum_in.json, ref_vectors.json")


if __name__ == "__main__":
    main()
