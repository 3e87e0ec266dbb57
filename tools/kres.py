"""Print per-kernel register / LDS / occupancy usage of an ops/csrc/*.hip file for gfx950.

usage: python tools/kres.py attention_decode.hip [kernel-substring]
(device-only compile with -Rpass-analysis=kernel-resource-usage; no GPU needed)
"""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from langstream_amd import _build  # noqa: E402

src = os.path.join(_build.CSRC, sys.argv[1])
inc, defs, _ = _build._torch_flags()
cmd = [_build.HIPCC, "--offload-arch=gfx950", "--cuda-device-only", "-O3", "-std=c++17", "-ffp-contract=fast",
       "-Wno-unused-result", "-Wno-deprecated-declarations", *defs, *inc, "-I", _build.CSRC, "-c", src,
       "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True).stdout
flt = sys.argv[2] if len(sys.argv) > 2 else ""
show = False
for line in out.splitlines():
    if "Function Name:" in line:
        show = flt in line
    if show and "remark" in line:
        print(line.split("remark: ")[-1])
