"""Summarise tools/pmc.sh / tools/pmc_roles.sh output: one row per kernel,
counters summed over dispatches; with a kernel-trace run beside the passes
(<dir>/kt, or --kernel-trace --stats in the counter passes themselves),
also the mean duration, the effective clock (GRBM_GUI_ACTIVE / 8
XCDs / duration, MI355X_MICROARCH.md "DVFS give-back") and the instructions
per 16-byte block (PROF_RECORDS x PROF_LEN records, default 2^18 x 16 KiB).
Counters are printed as means per dispatch."""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name):
    import re
    m = re.search(r"(gcm_kernel<[^>]*>|gcm_hy_kernel<[^>]*>|gcm_kth_kernel<[^>]*>|gcm_table_vkernel<[^>]*>|gcm_bs8?_kernel<[^>]*>|chacha_kernel<[^>]*>|chacha_wave_kernel<[^>]*>|ccm_\w*kernel<[^>]*>|kt_mask_kernel<[^>]*>|kth_jobkey_kernel|k_copy_\w+)", name)
    return m.group(1) if m else None


def main(d):
    # per kernel and counter: the mean over the dispatches that carried it
    # (each pass is its own run, so dispatch ids are not shared across passes)
    sums = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(lambda: defaultdict(int))
    for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = short(row.get("Kernel_Name", ""))
            if not k:
                continue
            sums[k][row["Counter_Name"]] += float(row["Counter_Value"])
            cnt[k][row["Counter_Name"]] += 1
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(d, "*", "**", "*kernel_stats.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = short(row.get("Name", ""))
            if k:
                dur[k].append(float(row["AverageNs"]))
    n_rec = int(os.environ.get("PROF_RECORDS", 1 << 18))
    blocks = n_rec * int(os.environ.get("PROF_LEN", 16384)) / 16
    for k in sums:
        v = {c: sums[k][c] / cnt[k][c] for c in sums[k]}
        print("==", k, "records per dispatch:", n_rec, "dispatches:", max(cnt[k].values()))
        for c in sorted(v):
            print("   %-34s %16.4g" % (c + " (per dispatch)", v[c]))
        if dur.get(k):
            ns = sum(dur[k]) / len(dur[k])
            print("   %-34s %16.4g" % ("duration_ms (kernel trace)", ns / 1e6))
            if "GRBM_GUI_ACTIVE" in v:
                print("   %-34s %16.4g" % ("effective_clock_GHz", v["GRBM_GUI_ACTIVE"] / 8 / ns))
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
            if c in v:
                print("   %-34s %16.4g" % (c + " lane-instr / 16 B", v[c] * 64 / blocks))
        if v.get("SQ_LDS_IDX_ACTIVE"):
            print("   %-34s %16.4g" % ("lds_bank_conflict / lds_active", v.get("SQ_LDS_BANK_CONFLICT", 0) /
                                       v["SQ_LDS_IDX_ACTIVE"]))

if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
