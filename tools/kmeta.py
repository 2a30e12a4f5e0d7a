"""Register / spill / scratch summary of the kernels in a device asm file.

Usage: kmeta.py ASM_FILE [NAME_SUBSTRING]

Compile the device asm first, e.g.
  hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S \
      -o /tmp/dev.s pipelinedp_amd/csrc/dpg_api.hip -Iinclude
"""
import re
import sys


def main(path, sub=""):
    s = open(path).read()
    i = s.index("amdhsa.kernels:")
    for blk in s[i:].split("  - .agpr_count:")[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk).group(1)
        if sub not in name:
            continue

        def g(k):
            m = re.search(r"\.%s:\s+(\d+)" % k, blk)
            return m.group(1) if m else "?"

        print(f"{name[:70]:70s} vgpr {g('vgpr_count'):>3} vspill {g('vgpr_spill_count'):>3} "
              f"sspill {g('sgpr_spill_count'):>3} scratch {g('private_segment_fixed_size'):>4}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
