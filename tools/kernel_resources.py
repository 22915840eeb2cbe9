"""Print per-kernel VGPR/SGPR/scratch/LDS from an amdgcn .s (hipcc -S --cuda-device-only)."""
import re
import sys


def main(path):
    s = open(path).read()
    for b in s.split(".name:")[1:]:
        name = b.split()[0]
        if "gw" not in name:
            continue
        head = b[:4000]

        def g(key):
            m = re.search(re.escape(key) + r":\s+(\d+)", head)
            return m.group(1) if m else "?"
        print("%-48s vgpr=%-4s sgpr=%-4s scratch=%-4s lds=%s" % (
            name[:48], g(".vgpr_count"), g(".sgpr_count"), g(".private_segment_fixed_size"),
            g(".group_segment_fixed_size")))


if __name__ == "__main__":
    main(sys.argv[1])
