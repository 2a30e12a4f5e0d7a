"""Build a variant of libdpg.so with extra -D flags (same-box A/B runs).

Usage: build_variant.py OUT_NAME FLAG [FLAG ...]
   e.g. build_variant.py libdpg_b.so -DDPG_HIST_U=8
"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "pipelinedp_amd", "csrc")


def main(name, flags):
    with tempfile.TemporaryDirectory() as tmp:
        out = os.path.join(tmp, "libdpg.so")
        subprocess.run(["/opt/rocm/bin/hipcc", *flags, "--offload-arch=gfx950", "-O3", "-std=c++17",
                        "-shared", "-fPIC", "-o", out, os.path.join(CSRC, "dpg_api.hip")],
                       check=True, cwd=tmp)
        os.replace(out, os.path.join(ROOT, "pipelinedp_amd", "lib", name))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
