"""The prover under each fixed-base window width: python scripts/r04/prover_window_ab.py LOG_N C [C ...]
(scripts/bench_prover.run per PBF_MSM_FX_C; the proofs of every width must be identical)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import bench_prover  # noqa: E402
import torch  # noqa: E402

import pbf  # noqa: E402


def main(log_n, cs):
    ctx = pbf.Context(0)
    for c in cs:
        os.environ["PBF_MSM_FX_C"] = str(c)
        r = bench_prover.run(ctx, log_n, reps=3 if log_n >= 24 else 10, no_key=False)
        r["fx_c"] = c
        print(json.dumps(r), flush=True)
        ctx.release_caches()
        torch.cuda.empty_cache()
    ctx.close()


if __name__ == "__main__":
    main(int(sys.argv[1]), [int(a) for a in sys.argv[2:]] or [16, 20])
