"""Per-kernel VGPRs / scratch / occupancy of libzfp_hip (compile remarks).
usage: python tools/kres.py [extra hipcc flags...]"""
import re
import subprocess
import sys

R = __file__.rsplit("/tools/", 1)[0]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I" + R + "/include",
       "-I" + R + "/zfp-par_amd/csrc/hip", "-c", "-o", "/tmp/kres.o", R + "/zfp-par_amd/csrc/hip/zfp_hip.hip",
       "-Rpass-analysis=kernel-resource-usage"] + sys.argv[1:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).split()[0]] = int(m.group(2))
for k, v in rows.items():
    if "zfp_amd" not in k:
        continue
    name = re.sub(r"^_ZN7zfp_amd\d+", "", k)[:48]
    print("%-48s vgpr %3s scratch %4s occ %s lds %s" % (name, v.get("VGPRs"), v.get("ScratchSize"), v.get("Occupancy"),
                                                        v.get("LDS")))
