"""Summarise a scripts/profile_round.sh run (gpurun_out/prof_<tag>) into profiles/.

Writes profiles/<tag>/ntt_kernel_stats.csv (rocprofv3 --stats), profiles/<tag>/pmc_counters.json
(per-kernel averages of every counter) and profiles/pmc_ntt_2p<log_n>_b<batch>.json, the HBM
traffic per bench step that bench.py reports as roofline.traffic.

Correction (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE reports half the bytes
of a coalesced streaming read, so FETCH bytes = 2 * FETCH_SIZE KiB * 1024; WRITE_SIZE is
taken as is. The NTT pass loads 8 B per lane in 128-B runs (a width the guide leaves
uncalibrated); with the factor 2 the fetch is 1.13x the pass input ('fetch_vs_input'), the
excess being consistent with L2 misses on pass 2's 8 MiB [r][k] twiddle table.
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(tag="r01", log_n=20, batch=32, passes=2):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace_kernel_stats.csv"), os.path.join(dst, f"ntt2p{log_n}_b{batch}_kernel_stats.csv"))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in ("fetch", "write", "sq"):
        for r in csv.DictReader(open(os.path.join(src, f + "_counter_collection.csv"))):
            agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    summ = {k: {c: {"dispatches": len(v), "mean": sum(v) / len(v)} for c, v in d.items()} for k, d in agg.items()}
    with open(os.path.join(dst, "pmc_counters.json"), "w") as fh:
        json.dump(summ, fh, indent=1)
    ntt = [k for k in summ if "ntt_pass_kernel" in k]
    assert len(ntt) == 1, ntt
    c = summ[ntt[0]]
    fetch = 2 * c["FETCH_SIZE"]["mean"] * 1024
    write = c["WRITE_SIZE"]["mean"] * 1024
    data = (1 << log_n) * batch * 8
    out = {"kernel": ntt[0], "log_n": log_n, "batch": batch, "passes_per_step": passes,
           "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
           "fetch_vs_input": fetch / data, "write_vs_output": write / data,
           "hbm_bytes_per_step": passes * (fetch + write),
           "algorithmic_bytes_per_step": passes * 2 * data,
           "source": f"profiles/{tag}/pmc_counters.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes)"}
    with open(os.path.join(ROOT, "profiles", f"pmc_ntt_2p{log_n}_b{batch}.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*[a if i == 0 else int(a) for i, a in enumerate(sys.argv[1:])])
