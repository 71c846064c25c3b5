"""Writes tests/golden/ref_exports.txt: the zfp_* and stream_* symbols exported
by the reference library built from the reference sources (oracle/_ref/
libzfp_ref.so, oracle/Makefile), one per line.  Run after building the oracle:
    python tests/golden/make_ref_exports.py
"""
import os
import subprocess

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
LIB = os.path.join(R, "oracle", "_ref", "libzfp_ref.so")

out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
names = sorted({ln.split()[-1] for ln in out.splitlines() if ln.split()[-1].startswith(("zfp_", "stream_"))})
with open(os.path.join(R, "tests", "golden", "ref_exports.txt"), "w") as f:
    f.write("\n".join(names) + "\n")
print(len(names), "symbols")
