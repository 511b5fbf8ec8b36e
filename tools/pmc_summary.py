"""Summarise tools/pmc.sh output: one row per kernel, counters summed over dispatches."""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name):
    import re
    m = re.search(r"(gcm_kernel<[^>]*>|gcm_hy_kernel<[^>]*>|gcm_bs8?_kernel<[^>]*>|chacha_kernel<[^>]*>|chacha_wave_kernel<[^>]*>|k_copy_\w+)", name)
    return m.group(1) if m else None


def main(d):
    vals = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = short(row.get("Kernel_Name", ""))
            if not k:
                continue
            vals[k][row["Counter_Name"]] += float(row["Counter_Value"])
            disp[k].add(row.get("Dispatch_Id"))
    for k, v in vals.items():
        print("==", k, "dispatches:", len(disp[k]))
        for c in sorted(v):
            print("   %-34s %16.4g" % (c, v[c]))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
