"""The other BASELINE configurations' bench entry points, each as a fresh child process.

- config 4 (``bench.py --model cgc_modified|cgc_vanilla``): the CGC benchmark models
  (``scripts/benchmark_models/cgc_*.py``) on the same synthetic lattices, at a reduced batch of
  8 graphs x 1024 nodes / 4096 edges (the driver's line uses 256);
- config 5 (``bench.py --config 5``): lmax 3, 5000-node / 20000-edge lattices, bf16 storage of
  the edge-sized tensors, at a reduced batch of 4 graphs (the line uses 32).

Checked on the JSON line: the metric and workload name the configuration, a finite positive
value and loss, the per-graph shapes, the roofline object of the fused kernel, and that the
line is a single-rank measurement.
"""
import json
import math
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*extra, timeout=300):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1",
           "--no-cpu-baseline", *extra]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("model", ["cgc_modified", "cgc_vanilla"])
def test_bench_config4_cgc_models(model):
    out = _bench("--model", model, "--batch", "8")
    assert model in out["metric"]
    assert math.isfinite(out["value"]) and out["value"] > 0
    assert math.isfinite(out["loss"])
    assert out["ranks"] == 1 and out["config"]["global_batch"] == 8
    assert out["config"]["parallelism"] == "graph-sharded dp1"
    roof = out["roofline"]
    assert roof is not None and roof["kernel"].startswith("cgc_fwd")
    assert 0 < roof["frac"] < 1.5 and roof["launches"] == 2 * 3      # 3 passes per step


def test_bench_config5_bf16_storage():
    out = _bench("--config", "5", "--batch", "4")
    assert "lmax 3" in out["metric"] and "bf16" in out["metric"]
    assert out["config"]["nodes_per_graph"] == 5000 and out["config"]["edges_per_graph"] == 20000
    assert out["config"]["global_batch"] == 4
    assert "bf16" in out["dtype"]
    assert math.isfinite(out["value"]) and out["value"] > 0 and math.isfinite(out["loss"])
    roof = out["roofline"]
    assert roof is not None and roof["kernel"].startswith("tp_fwd_tpB_l3")
    # frac from the 5 in-line steps after the timed region (bench --inline-steps), layers 1..3;
    # the overlapped timed region's own figure beside it (2 timed steps)
    assert roof["launches"] == 5 * 3 and roof["overlapped"]["launches"] == 2 * 3
    assert 0 < roof["frac"] < 1.5 and 0 < roof["overlapped"]["frac"] < 1.5
