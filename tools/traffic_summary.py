"""HBM bytes per launch of the headline kernels from tools/traffic.sh output,
calibrated per access shape.

rocprofv3 FETCH_SIZE / WRITE_SIZE are in KB (1024 B) and count memory-side
(fabric) requests.  On gfx950 their relation to the bytes moved depends on
the access shape (MI355X_MICROARCH.md: FETCH_SIZE reports half the bytes of a
wide coalesced streaming read; other widths are uncalibrated).  So
tools/fetch_calib.hip copies exactly 4 GiB with each shape the kernels use,
under the same counter passes, and the factor of a shape is
bytes / counter bytes; a kernel's traffic is its raw counters times the
factors of its shape:

  aes128gcm_*         gcm_hy_kernel, octet layout: 8 records x 128 B per
                      instruction -> the octet factors
  chacha20-poly1305_* chacha_kernel, line-pair tile: the same 8 records x
                      128 B per instruction -> the octet factors (round 1's
                      tile moved 16 records x 64 B: tile64)
  c4_kt_*             gcm_kth_kernel (round 4; gcm_kt_kernel before: config 4's
                      long records), whole-line layout -> the octet factors
  c4_lane_*           gcm_table_vkernel (config 4's short records), 16 B per
                      lane, one record per lane -> the lane factors
  aes128gcm_masks,    hy_mask_kernel, kt_mask_kernel, kth_jobkey_kernel: one
  c4_masks, c4_jobkey lane per record (or job), launched with every seal and
                      open (labels are per launch) -> the lane factors
  c5_prep, c5_seal    config 5 (bench.py --config c5, collected from its own
                      passes): seal_prep (one thread per record: header,
                      inner type, nonce / AAD rows -> the lane factors) and
                      the hybrid seal over the framed records (octet)

Config 4 (bench.py --config c4) is one seal and one open of the whole batch;
its traffic per operation is the sum over the kernels of that operation.

The headline working set (48 GiB) is far past the 256 MiB Infinity Cache, so
cache hits in the counters are negligible.

    python tools/traffic_summary.py <traffic.sh output dir>  > traffic.json
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

CAL_BYTES = 16384 * (1 << 18)
CAL = {"k_coalesced": "coalesced", "k_octet": "octet", "k_tile64": "tile64", "k_lane": "lane"}
# (kernel name pattern, label, access shape, calibration shape)
KERNELS = [(r"gcm_hy_kernel<10, false", "aes128gcm_seal", "octet", "octet"),
           (r"gcm_hy_kernel<10, true", "aes128gcm_open", "octet", "octet"),
           (r"chacha_kernel<false", "chacha20-poly1305_seal", "line-pair tile", "octet"),
           (r"chacha_kernel<true", "chacha20-poly1305_open", "line-pair tile", "octet"),
           (r"gcm_kt_kernel<14, false", "c4_kt_seal", "octet", "octet"),
           (r"gcm_kt_kernel<14, true", "c4_kt_open", "octet", "octet"),
           # round 4: the key-table hybrid (long records, 32 lanes per record:
           # each instruction moves 2 records x 512 B, whole lines -> octet)
           (r"gcm_kth_kernel<14, false", "c4_kt_seal", "octet", "octet"),
           (r"gcm_kth_kernel<14, true", "c4_kt_open", "octet", "octet"),
           (r"gcm_table_vkernel<14, false", "c4_lane_seal", "lane", "lane"),
           (r"gcm_table_vkernel<14, true", "c4_lane_open", "lane", "lane"),
           # round 4: the per-record keystream precomputes launched with each
           # seal and open (one lane per record: the lane factors)
           (r"hy_mask_kernel<10>", "aes128gcm_masks", "lane", "lane"),
           (r"kt_mask_kernel<14>", "c4_masks", "lane", "lane"),
           (r"kth_jobkey_kernel", "c4_jobkey", "lane", "lane")]
KERNELS_C5 = [(r"seal_prep", "c5_prep", "lane", "lane"),
              (r"gcm_hy_kernel<10, false", "c5_seal", "octet", "octet")]


def collect(d, pattern):
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, pattern, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            vals[row.get("Kernel_Name", "")][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return vals


def mean_kb(lst):
    return sum(lst) / max(len(lst), 1) * 1024


def main(d):
    cal_raw = collect(d, "cal_*")
    factors = {}
    for name, c in cal_raw.items():
        for k, shape in CAL.items():
            if re.search(r"\b%s\b" % k, name):
                fetch, write = mean_kb(c["FETCH_SIZE"]), mean_kb(c["WRITE_SIZE"])
                factors[shape] = {"fetch_size_bytes": fetch, "write_size_bytes": write,
                                  "fetch_factor": round(CAL_BYTES / fetch, 4) if fetch else None,
                                  "write_factor": round(CAL_BYTES / write, 4) if write else None}
    out = {}
    for name, c, kernels in ([(n, c, KERNELS) for n, c in collect(d, "bench_*").items()] +
                             [(n, c, KERNELS_C5) for n, c in collect(d, "c5_*").items()]):
        for pat, lab, shape, cal in kernels:
            if re.search(pat, name) and cal in factors:
                fetch, write = mean_kb(c["FETCH_SIZE"]), mean_kb(c["WRITE_SIZE"])
                ff, wf = factors[cal]["fetch_factor"], factors[cal]["write_factor"]
                out[lab] = {"fetch_size_bytes": fetch, "write_size_bytes": write, "shape": shape,
                            "calibrated_as": cal,
                            "fetch_factor": ff, "write_factor": wf,
                            "hbm_read_bytes": fetch * ff, "hbm_write_bytes": write * wf,
                            "hbm_bytes": fetch * ff + write * wf,
                            "launches": len(c["FETCH_SIZE"])}
    print(json.dumps({"calibration": factors, "calibration_bytes": CAL_BYTES, "kernels": out},
                     indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1])
