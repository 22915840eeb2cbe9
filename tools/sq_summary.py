"""Mean SQ counter values per kernel from tools/gpu_sq.sh output (rocprofv3 counter_collection CSVs)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(root):
    acc = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> per-dispatch values
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row.get("Kernel_Name", "?")
                short = name.split("(")[0].split("<")[0].replace("void ", "").strip() + (
                    "<" + name.split("<", 1)[1].split(">")[0] + ">" if "<" in name else "")
                acc[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in sorted(acc.items()):
        print(k)
        for c, v in sorted(cs.items()):
            # each dispatch reports one row per counter (summed over the device by rocprofv3)
            print(f"  {c:24s} mean {sum(v) / len(v):16.1f}   dispatches {len(v)}")


if __name__ == "__main__":
    main(sys.argv[1])
