"""Per-role cycle accounting of the hybrid AES-GCM kernel.

Runs AES-128-GCM seal and open over 2^20 x 16 KiB records (the headline
shape, device resident) with a TG_ROLE_PROBE build of libtlsgpu.so
(tools/build_variant.sh aes_gcm_bs8 ... -DTG_ROLE_PROBE) under three role
mixes -- the default 10 T-table + 6 bitsliced waves, T-table waves only
(hy_t 16), bitsliced waves only (hy_t -1) -- and the tree's own library for
the probe's perturbation.  Each run is a child process; its device printf
lines (gcm_hy_kernel's role_probe_print) are parsed here.

    python tools/role_probe.py PROBE_LIB.so [--reps 3] > role_probe.json

For each role the probe sums, over every wave of the dispatch, the
wave-cycles (s_memtime) spent in each phase of its octet jobs: setup
(counter cache / first-state planes, AAD), keystream, consume (payload
loads, XOR, stores, GHASH), tail (lift, tag) and the job queue's atomic;
the blocks it encrypted; and each wave's span from its first grab to its
exit.  Per role: wave-cycles per 16-byte block by phase.  A CU runs n_r waves
of role r at once, so its blocks per cycle are sum_r n_r / w_r (w_r = the
role's wave-cycles per block) while every wave is busy.
"""
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import os, sys, json
sys.path[:0] = [%(root)r, os.path.join(%(root)r, "tlslite-ng_amd"), os.path.join(%(root)r, "tests", "golden")]
import torch, tlsgpu
from vectors import tls13_aad
n, L = 1 << 20, 16384
so = (L + 16 + 127) // 128 * 128
g = torch.Generator(device="cuda").manual_seed(0x7715)
inp = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
sealed = torch.empty(n * so, dtype=torch.uint8, device="cuda")
back = torch.empty_like(inp)
status = torch.zeros(n, dtype=torch.uint8, device="cuda")
nonces = torch.empty(12 * n, dtype=torch.uint8, device="cuda")
tlsgpu.make_nonces(bytes(range(12)), 0, n, nonces)
aad = torch.tensor(list(tls13_aad(L)), dtype=torch.uint8, device="cuda")
key = tlsgpu.HipAESGCM(bytearray(range(16)))
bs = tlsgpu.make_batch(n, inp, sealed, nonces, aad=aad, fixed_len=L, in_stride=L, out_stride=so, fixed_aad_len=5)
bo = tlsgpu.make_batch(n, sealed, back, nonces, aad=aad, fixed_len=L, in_stride=so, out_stride=L,
                       fixed_aad_len=5, status=status)
st = torch.cuda.current_stream()
for name, b, fn in (("seal", bs, tlsgpu.seal_batch), ("open", bo, tlsgpu.open_batch)):
    fn(key, b)
    torch.cuda.synchronize()
    sys.stdout.flush()
    print("PHASE %%s" %% name, flush=True)
    for r in range(%(reps)d):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        fn(key, b)
        e1.record(st)
        torch.cuda.synchronize()
        print("TIME %%s %%.4f" %% (name, e0.elapsed_time(e1)), flush=True)
ok = bool((status == 1).all()) and torch.equal(back, inp)
print("ROUNDTRIP %%s" %% ok, flush=True)
'''


def run(lib, hy_t, reps):
    env = dict(os.environ)
    if lib:
        env["TLSGPU_LIB"] = lib
        env["TLSGPU_ALLOW_MEASUREMENT_BUILD"] = "1"
    if hy_t is not None:
        env["TLSGPU_HY_T"] = str(hy_t)
    code = CHILD % {"root": ROOT, "reps": reps}
    p = subprocess.run([sys.executable, "-u", "-c", code], env=env, capture_output=True, text=True,
                       timeout=300)
    if p.returncode != 0:
        raise SystemExit("child failed: %s" % p.stderr[-2000:])
    out = {"seal": {"ms": [], "probe": []}, "open": {"ms": [], "probe": []}}
    phase = None
    for line in p.stdout.splitlines():
        if line.startswith("PHASE "):
            phase = line.split()[1]
        elif line.startswith("TIME "):
            _, name, ms = line.split()
            out[name]["ms"].append(float(ms))
        elif line.startswith("ROLE_PROBE") and phase:
            f = line.split()
            d = {f[i]: f[i + 1] for i in range(1, len(f) - 1, 2)}
            out[phase]["probe"].append(d)
        elif line.startswith("ROUNDTRIP"):
            out["roundtrip_ok"] = line.split()[1] == "True"
    return out


def summarise(runs, nt, waves_per_cu=16, cus=256):
    """Per role: wave-cycles per block by phase (the dispatch's sums over the
    timed launches, the warm-up launch's lines dropped)."""
    res = {}
    for name in ("seal", "open"):
        probe = runs[name]["probe"]
        ms = runs[name]["ms"]
        # the first two probe lines (both roles) belong to the warm-up launch
        lines = probe[2:] if len(probe) > 2 * len(ms) else probe
        roles = {}
        for role in ("ttable", "bitsliced"):
            rl = [d for d in lines if d["role"] == role]
            if not rl:
                continue
            tot = {k: sum(int(d[k]) for d in rl) for k in ("setup", "cipher", "consume", "tail", "grab",
                                                           "jobs", "blocks", "span", "waves")}
            if tot["blocks"] == 0:
                continue
            per_block = {k: round(tot[k] / tot["blocks"], 2) for k in ("setup", "cipher", "consume", "tail",
                                                                       "grab")}
            busy = sum(tot[k] for k in ("setup", "cipher", "consume", "tail", "grab"))
            per_block["jobs_total"] = round(busy / tot["blocks"], 2)
            per_block["span"] = round(tot["span"] / tot["blocks"], 2)
            nw = tot["waves"] / len(rl) / cus       # waves of this role per CU
            roles[role] = {"wave_cycles_per_block": per_block, "waves_per_cu": round(nw, 2),
                           "blocks_share": None, "jobs": tot["jobs"] // len(rl),
                           "mean_wave_span_cycles": round(tot["span"] / tot["waves"], 0),
                           "blocks": tot["blocks"] // len(rl)}
        allb = sum(r["blocks"] for r in roles.values())
        for r in roles.values():
            r["blocks_share"] = round(r["blocks"] / allb, 4) if allb else None
        # CU-cycles per block: the longest wave span (memtime cycles) over the
        # blocks one CU encrypts
        span = max(r["mean_wave_span_cycles"] for r in roles.values()) if roles else 0
        blocks_per_cu = allb / cus if allb else 0
        res[name] = {"ms_best": min(ms) if ms else None, "ms_mean": round(sum(ms) / len(ms), 4) if ms else None,
                     "roles": roles,
                     "cu_cycles_per_block": round(span / blocks_per_cu, 3) if blocks_per_cu else None,
                     "memtime_GHz": round(span / (min(ms) * 1e6), 3) if ms and span else None}
        # blocks per CU-cycle predicted from the roles: sum n_r / w_r
        if roles:
            pred = sum(r["waves_per_cu"] / r["wave_cycles_per_block"]["jobs_total"] for r in roles.values())
            res[name]["cu_cycles_per_block_from_roles"] = round(1 / pred, 3)
    return res


def main():
    lib = sys.argv[1]
    reps = 3
    if "--reps" in sys.argv:
        reps = int(sys.argv[sys.argv.index("--reps") + 1])
    report = {"probe_lib": lib}
    tree = run(None, None, reps)
    report["tree_no_probe"] = {k: {"ms_best": min(v["ms"]), "ms_mean": round(sum(v["ms"]) / len(v["ms"]), 4)}
                               for k, v in tree.items() if isinstance(v, dict)}
    for label, hy_t, nt in (("hybrid_10T_6B", None, 10), ("ttable_only_16T", 16, 16),
                            ("bitsliced_only_16B", -1, 0)):
        r = run(lib, hy_t, reps)
        report[label] = summarise(r, nt)
        report[label]["roundtrip_ok"] = r.get("roundtrip_ok")
        print(json.dumps({label: report[label]}), file=sys.stderr, flush=True)
    print(json.dumps(report, indent=1))


if __name__ == "__main__":
    main()
