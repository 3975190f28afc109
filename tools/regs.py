"""Register use of every instantiation of a kernel (tooling): compiles a .hip file for gfx950 with
the resource-usage remarks and prints VGPRs / scratch / occupancy / LDS per kernel whose mangled
name contains PATTERN.  usage: python tools/regs.py vproxy_amd/csrc/kernels.hip [PATTERN]"""
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.abspath(sys.argv[1])
pat = sys.argv[2] if len(sys.argv) > 2 else "k_csum_d"
with tempfile.TemporaryDirectory() as td:
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
                        "-I", os.path.join(REPO, "include"), "-I", os.path.join(REPO, "vproxy_amd", "csrc"),
                        "-c", src, "-o", os.path.join(td, "x.o"), "-Rpass-analysis=kernel-resource-usage"],
                       capture_output=True, text=True, cwd=td)
cur, res = None, {}
for line in r.stderr.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        res[cur] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|Occupancy \[waves/SIMD\]|ScratchSize \[bytes/lane\]|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur:
        res[cur][m.group(1).split()[0]] = int(m.group(2))
for k, v in res.items():
    if pat in k:
        print(re.sub(r"EEEvPK.*", "", k), v)
