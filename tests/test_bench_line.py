"""bench.py's printed line (CPU): the driver keeps only the last ~2 KB of stdout, so
compact_line must put the north-star 2^24 NTT roofline, config 3's roofline and the 2^24-gate
proof at the end of the line, keep the contract's top-level keys, and lose
no description (moved into extra.notes). Checked on the committed round-4 final-tree line."""
import importlib.util
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_compact_line_puts_headlines_in_the_tail():
    b = _bench()
    d = json.load(open(os.path.join(ROOT, "profiles", "r04", "bench_r04u.json")))
    d.pop("extra_keys", None)
    s = json.dumps(b.compact_line(d), separators=(",", ":"))
    tail = s[-1900:]  # what the driver keeps, less its stderr section
    for key in ('"ntt_2p24"', '"config3_bn254_polymul_2p22"', '"config5_prove_2p24"'):
        assert key in tail, key
    t24 = tail[tail.index('"ntt_2p24"'):]
    assert '"roofline"' in t24 and '"frac"' in t24 and '"traffic"' in t24
    t3 = tail[tail.index('"config3_bn254_polymul_2p22"'):]
    assert '"roofline"' in t3
    line = json.loads(s)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in line, k
    assert line["cpu_baseline"]["sample"] == d["cpu_baseline"]["sample"]  # top level keeps its strings
    notes = line["extra"]["notes"]
    assert notes["ntt_2p24.roofline.kernel"] == d["extra"]["ntt_2p24"]["roofline"]["kernel"]
    assert abs(line["value"] - d["value"]) / d["value"] < 1e-3
