"""HBM bytes per launch of the headline kernels from tools/traffic.sh output.

Corrections (MI355X_MICROARCH.md, HBM section): rocprofv3 FETCH_SIZE and
WRITE_SIZE are in KB (1024 B); on gfx950 FETCH_SIZE reports half the bytes of
a wide streaming read (128-B requests tallied at 64 B), so it is doubled;
WRITE_SIZE is taken as is.  Both count memory-side (fabric) requests, i.e.
Infinity-Cache hits are included; the headline working set (32 GiB) is far
past the 256 MiB Infinity Cache.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

NAMES = [(r"gcm_kernel<10, false", "aes128gcm_seal"), (r"gcm_kernel<10, true", "aes128gcm_open"),
         (r"chacha_kernel<false", "chacha20-poly1305_seal"),
         (r"chacha_kernel<true", "chacha20-poly1305_open")]


def label(name):
    for pat, lab in NAMES:
        if re.search(pat, name):
            return lab
    return None


def main(d):
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "*", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            lab = label(row.get("Kernel_Name", ""))
            if lab:
                vals[lab][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {}
    for lab, c in vals.items():
        fetch = sum(c["FETCH_SIZE"]) / max(len(c["FETCH_SIZE"]), 1) * 1024
        write = sum(c["WRITE_SIZE"]) / max(len(c["WRITE_SIZE"]), 1) * 1024
        out[lab] = {"fetch_size_bytes": fetch, "write_size_bytes": write,
                    "hbm_read_bytes": 2 * fetch, "hbm_write_bytes": write,
                    "hbm_bytes": 2 * fetch + write, "launches": len(c["FETCH_SIZE"])}
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1])
