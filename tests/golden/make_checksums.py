#!/usr/bin/env python3
"""Regenerate tests/golden/checksums.json from the reference's golden tables.

Reads the numeric (key1, key2, checksum) tuples of
  /root/reference/tests/constants/checksums/{1,2,3,4}d{Float,Double,Int32,Int64}.h
and records them as data, decoded with the key layout of
  tests/utils/zfpChecksums.c:75-136 (computeKey):
    key1 = test_type << 9 | subject << 7 | zfp_mode << 4 | param
    key2 = dims packed like zfp_field_metadata (n-1 per axis, x in the top field)
subject: 0 original input, 1 compressed stream, 2 decompressed array.
param:   fixed rate/precision 2^(p+3); accuracy 2^-(2^p)  (zfpCompressionParams.c).
Only the ARRAY_TEST (end-to-end, test_type 2) entries are kept.
"""
import json
import os
import re
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "checksums.json")

MODES = {0: "none", 2: "rate", 3: "precision", 4: "accuracy", 5: "reversible"}
SUBJECTS = {0: "input", 1: "stream", 2: "decompressed"}


def dims_of(key2, dims):
    bits = {1: 64, 2: 24, 3: 16, 4: 12}[dims]
    mask = (1 << bits) - 1
    vals = []
    for _ in range(dims):
        vals.append((key2 & mask) + 1)
        key2 >>= bits
    return list(reversed(vals))  # n[0] (x) first


def main():
    table = []
    for dims in (1, 2, 3, 4):
        for tname in ("Float", "Double", "Int32", "Int64"):
            path = os.path.join(REF, "tests", "constants", "checksums", "%dd%s.h" % (dims, tname))
            text = open(path).read()
            for m in re.finditer(r"\{UINT64C\((0x[0-9a-f]+)\),\s*UINT64C\((0x[0-9a-f]+)\),\s*UINT64C\((0x[0-9a-f]+)\)\}", text):
                k1, k2, ck = (int(g, 16) for g in m.groups())
                tt = k1 >> 9
                if tt != 2:
                    continue
                subject = (k1 >> 7) & 3
                mode = (k1 >> 4) & 7
                param = k1 & 15
                if mode == 2 or mode == 3:
                    value = 1 << (param + 3)
                elif mode == 4:
                    value = 2.0 ** -(1 << param)
                else:
                    value = None
                table.append({"dims": dims, "type": tname.lower(), "n": dims_of(k2, dims),
                              "subject": SUBJECTS[subject], "mode": MODES[mode], "param": value,
                              "checksum": "0x%x" % ck})
    with open(OUT, "w") as f:
        json.dump({"source": "reference tests/constants/checksums/*.h (ARRAY_TEST rows)",
                   "entries": table}, f, indent=1)
    print("wrote", len(table), "entries to", OUT)


if __name__ == "__main__":
    main()
