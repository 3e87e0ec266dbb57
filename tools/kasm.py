"""Compile one ops/csrc/*.hip for gfx950 with the extension's flags, keep the device
assembly, and print each matching kernel's resource usage (VGPR/AGPR/SGPR, spills, LDS)
plus instruction counts of interest.

usage: python tools/kasm.py gemm_prefill.hip [kernel-substring] [--dump]
"""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from langstream_amd import _build  # noqa: E402


def main():
    src = os.path.join(_build.CSRC, sys.argv[1])
    pat = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else ""
    inc, defs, _ = _build._torch_flags()
    d = tempfile.mkdtemp()
    cmd = [_build.HIPCC, f"--offload-arch={_build.ARCH}", "-O3", "-fPIC", "-std=c++17", "-ffp-contract=fast",
           "-Wno-unused-result", "-Wno-deprecated-declarations", "-Wno-unused-command-line-argument",
           *defs, *inc, "-I", _build.CSRC, "--cuda-device-only", "-S", src, "-o", os.path.join(d, "k.s")]
    subprocess.run(cmd, check=True)
    s = open(os.path.join(d, "k.s")).read()
    for m in re.finditer(r"\.amdhsa_kernel (\S+)\n(.*?)\.end_amdhsa_kernel", s, re.S):
        name, body = m.group(1), m.group(2)
        if pat and pat not in name:
            continue
        if ".amdhsa_next_free_vgpr" not in body:
            continue
        def g(k):
            mm = re.search(r"\." + k + r"\s+(\S+)", body)
            return mm.group(1) if mm else "?"
        # find the function body text
        fb = re.search(r"^" + re.escape(name) + r":.*?\n(.*?)\.Lfunc_end", s, re.S | re.M)
        text = fb.group(1) if fb else ""
        cnt = {k: len(re.findall(k, text)) for k in ("v_mfma", "s_barrier", "ds_read", "global_load_lds", "s_waitcnt vmcnt", "s_waitcnt lgkmcnt", "scratch_")}
        print(name[:110])
        print(f"   vgpr {g('amdhsa_next_free_vgpr')} accum_offset {g('amdhsa_accum_offset')} sgpr {g('amdhsa_next_free_sgpr')} "
              f"lds {g('amdhsa_group_segment_fixed_size')} scratch {g('amdhsa_private_segment_fixed_size')}  {cnt}")
        if "--dump" in sys.argv:
            open(os.path.join("/tmp", "kasm_" + re.sub(r"\W", "_", name)[:60] + ".s"), "w").write(text)


if __name__ == "__main__":
    main()
