"""Summarise a scripts/profile_round.sh run (gpurun_out/prof_<tag>) into profiles/.

Writes profiles/<tag>/ntt_kernel_stats.csv (rocprofv3 --stats), profiles/<tag>/pmc_counters.json
(per-kernel averages of every counter) and profiles/pmc_ntt_2p<log_n>_b<batch>.json, the HBM
traffic per bench step that bench.py reports as roofline.traffic.

Calibration (MI355X_MICROARCH.md, HBM section: FETCH_SIZE is exact only for 16-B-per-lane
streaming reads, "calibrate on a known byte count in your own access pattern"): the same run
profiles scripts/ubench/tile_copy, whose kernels move a known 256 MiB in the NTT pass's own
access patterns (8 B per lane, 64-B runs rows n/R apart); the ratio known bytes / counter
bytes of the matching tile_copy kernel converts the NTT kernels' FETCH_SIZE / WRITE_SIZE.
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


KNOWN = (1 << 20) * 32 * 8  # bytes each tile_copy kernel reads and writes
CAL_KERNEL = "k_tile<3, 8, 1>"  # strided 64-B runs on both sides, 8 B per lane


def counters(path):
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        out[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return out


def calibration(src):
    """bytes per counter unit for reads and writes, from the tile_copy runs (None if absent)."""
    cal = {}
    for f, cname in (("calib_fetch", "FETCH_SIZE"), ("calib_write", "WRITE_SIZE")):
        path = os.path.join(src, f + "_counter_collection.csv")
        if not os.path.exists(path):
            return None
        c = counters(path)
        ks = [k for k in c if CAL_KERNEL in k]
        assert len(ks) == 1, ks
        v = c[ks[0]][cname]
        cal[cname] = KNOWN / (sum(v) / len(v))  # bytes per counted unit
        cal[cname + "_all"] = {k: KNOWN / (sum(x) / len(x)) for k, d in c.items() for n, x in d.items()
                               if n == cname}
    return cal


def main(tag="r01", log_n=20, batch=32, steps=12):
    """steps: bench steps the profiled command ran (profile_round.sh: 10 timed + 2 warm-up);
    a kernel dispatched more than once per step (the grouped schedule) is summed per step."""
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace_kernel_stats.csv"), os.path.join(dst, f"ntt2p{log_n}_b{batch}_kernel_stats.csv"))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in ("fetch", "write", "sq"):
        for k, d in counters(os.path.join(src, f + "_counter_collection.csv")).items():
            for c, v in d.items():
                agg[k][c] += v
    summ = {k: {c: {"dispatches": len(v), "mean": sum(v) / len(v)} for c, v in d.items()} for k, d in agg.items()}
    cal = calibration(src)
    summ["_calibration"] = cal
    with open(os.path.join(dst, "pmc_counters.json"), "w") as fh:
        json.dump(summ, fh, indent=1)
    # one dispatch of each pass kernel per step
    ntt = sorted(k for k in summ if "ntt_gl_pass_kernel" in k or "ntt_pass_kernel" in k)
    assert ntt, list(summ)
    fk = cal["FETCH_SIZE"] if cal else 2.0 * 1024  # uncalibrated: the guide's 16-B-lane factor
    wk = cal["WRITE_SIZE"] if cal else 1024
    per = {}
    for k in ntt:
        per_step = summ[k]["FETCH_SIZE"]["dispatches"] / steps  # dispatches of this kernel per step
        per[k] = {"dispatches_per_step": per_step,
                  "fetch_bytes": summ[k]["FETCH_SIZE"]["mean"] * fk * per_step,
                  "write_bytes": summ[k]["WRITE_SIZE"]["mean"] * wk * per_step}
    data = (1 << log_n) * batch * 8
    hbm = sum(v["fetch_bytes"] + v["write_bytes"] for v in per.values())
    out = {"kernels": per, "log_n": log_n, "batch": batch, "passes_per_step": len(ntt),
           "note": "bytes per bench step (all dispatches of each pass kernel in one step)",
           "fetch_vs_input": {k: v["fetch_bytes"] / data for k, v in per.items()},
           "write_vs_output": {k: v["write_bytes"] / data for k, v in per.items()},
           "calibration_bytes_per_kib": {"FETCH_SIZE": fk, "WRITE_SIZE": wk, "kernel": CAL_KERNEL if cal else None},
           "hbm_bytes_per_step": hbm,
           "algorithmic_bytes_per_step": 2 * data,
           "source": f"profiles/{tag}/pmc_counters.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate "
                     f"passes; calibrated on scripts/ubench/tile_copy)"}
    with open(os.path.join(ROOT, "profiles", f"pmc_ntt_2p{log_n}_b{batch}.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*[a if i == 0 else int(a) for i, a in enumerate(sys.argv[1:])])
