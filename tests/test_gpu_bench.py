"""bench.py end to end on the GPU, short runs: the default line, the one-process-several-GPUs
form and the dispatch-carried events each print one JSON line with the contract's fields,
a verified round trip and per-kernel durations that add up to about the step."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("extra", [[], ["--dispatch-events"], ["--single-process"],
                                   ["--config", "raid5_4p1_64k"]])
def test_bench_line(extra):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "6",
                        "--warmup", "2", "--no-cpu-baseline"] + extra,
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config", "roofline"):
        assert key in d, key
    assert d["steps"] == 6 and d["warmup"] == 2 and d["n_gpus"] == 1 and d["dtype"] == "u8"
    assert d["verified_roundtrip"] is True
    assert d["value"] > 1000 and 0.3 < d["roofline"]["frac"] < 1.0
    b = d.get("breakdown")
    if b and "encode_ms" in b:  # the kernels' durations fill the step: nothing else runs in the timed region
        assert 0.8 * d["ms_per_step"] < b["encode_ms"] + b["reconstruct_ms"] < 1.1 * d["ms_per_step"]
