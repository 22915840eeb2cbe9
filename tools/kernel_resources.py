"""Print per-kernel VGPR/SGPR/scratch/LDS from an amdgcn .s (hipcc -S --cuda-device-only)."""
import re
import sys


def main(path):
    s = open(path).read()
    meta = s[s.index("amdhsa.kernels:"):]
    for blk in re.split(r"\n  - \.agpr_count:", meta)[1:]:
        def g(key):
            m = re.search(r"\n\s+" + re.escape(key) + r":\s+(\S+)", blk)
            return m.group(1) if m else "?"
        name = g(".name")
        if "gw" not in name and "cnn" not in name and "act" not in name:
            continue
        print("%-48s vgpr=%-4s sgpr=%-4s scratch=%-4s lds=%s" % (
            name[:48], g(".vgpr_count"), g(".sgpr_count"), g(".private_segment_fixed_size"),
            g(".group_segment_fixed_size")))


if __name__ == "__main__":
    main(sys.argv[1])
