"""Device assembly of one ops/csrc/*.hip file for gfx950 (same flags as the build).

usage: python tools/dump_isa.py langstream_amd/ops/csrc/knn.hip /tmp/knn.s
"""
import subprocess
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from langstream_amd import _build as B  # noqa: E402


def main():
    src, out = sys.argv[1], sys.argv[2]
    inc, defs, _ = B._torch_flags()
    cmd = [B.HIPCC, f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", "-ffp-contract=fast", "-Wno-unused-result",
           "-Wno-deprecated-declarations", "--cuda-device-only", "-S", *defs, *inc, "-I", B.CSRC, src, "-o", out]
    subprocess.check_call(cmd)


if __name__ == "__main__":
    main()
