"""bench.py's stdout line: the driver parses ONE JSON line (round 5's 29 KB
line was left unparsed).  Built here from a canned full result -- round 5's
final bench output with every side table, and eight ranks -- it must parse,
keep the contract's fields, and stay under bench.LINE_MAX_BYTES."""
import copy
import json
import os

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CANNED = os.path.join(ROOT, "profiles", "r05", "r05_final_bench.json")


def canned(world=1):
    line = json.load(open(CANNED))
    if world > 1:
        p = line["per_gpu"][0]
        line["per_gpu"] = [dict(copy.deepcopy(p), rank=r, device=r) for r in range(world)]
        line["n_gpus"] = world
    return line


def test_compact_line_parses_and_fits():
    full = canned()
    assert len(json.dumps(full)) > 20000            # the line that was not parsed
    for world in (1, 8):
        text = json.dumps(bench.compact_line(canned(world), bench.EXTRAS_PATH))
        assert "\n" not in text
        d = json.loads(text)
        assert len(text.encode()) <= bench.LINE_MAX_BYTES, len(text)
        for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                  "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
                  "roofline", "cpu_baseline", "per_gpu"):
            assert k in d, k
        assert d["value"] == full["value"] and d["n_gpus"] == world
        assert len(d["per_gpu"]) == world
        for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
            assert k in d["roofline"], k
        for k in ("value", "unit", "cores", "kind", "sample"):
            assert k in d["cpu_baseline"], k
        s = d["side"]
        for k in ("c1_64B_cold_frac", "c3_fill_ms", "c3_verify_ms", "c4_ms_per_step",
                  "lro_w64_ms", "rx_async_registered_blocked_us"):
            assert isinstance(s[k], (int, float)), k
        assert d["extras_file"] == "profiles/bench_extras_last.json"


def test_compact_line_without_extras():
    """--no-extras / N > 1 ranks: no side tables, still a valid line."""
    full = canned(2)
    for k in list(full):
        if k not in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                     "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
                     "gib_per_s", "roofline", "kernels_ms", "per_gpu", "settle_s",
                     "corrupted_frames_detected"):
            del full[k]
    d = json.loads(json.dumps(bench.compact_line(full)))
    assert "side" not in d and "cpu_baseline" not in d and "extras_file" not in d
    assert d["roofline"]["frac"] == full["roofline"]["frac"]


def test_zero_counters_dropped():
    s = {"config": {"MT_PIN": "1"}, "threads_1": {"us_per_call": 10.3, "gpu_span_us": 0.0,
                                                   "requests": 1200.0}}
    out = bench.drop_zero_counters(s)
    assert out["threads_1"] == {"us_per_call": 10.3, "requests": 1200.0}
    assert out["config"] == {"MT_PIN": "1"}
