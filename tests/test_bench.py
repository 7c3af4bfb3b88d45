"""bench.py contract: the global grid per GPU count (CPU) and one small end-to-end run whose
single JSON line carries the fields the driver and the judge read (GPU)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_global_dims_double_one_axis_per_doubling():
    assert bench.global_dims(1024, 1) == [1024, 1024, 1024]
    assert bench.global_dims(1024, 2) == [2048, 1024, 1024]
    assert bench.global_dims(1024, 4) == [2048, 2048, 1024]
    assert bench.global_dims(1024, 8) == [2048, 2048, 2048]    # BASELINE config 4
    assert bench.global_dims(64, 3) == [64, 64, 192]           # non-powers of two stack in z


@pytest.mark.gpu
def test_bench_small_run_prints_one_contract_line():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dst", "128", "--steps", "3",
                        "--warmup", "2", "--cpu-dst", "64"], capture_output=True, text=True, timeout=300,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert key in out, key
    assert out["n_gpus"] == 1 and out["steps"] == 3 and out["warmup"] == 2
    assert out["value"] > 0 and out["ms_per_step"] > 0 and out["higher_is_better"] is True
    roof = out["roofline"]
    assert roof["bound"] == "hbm" and roof["unit"] == "GB/s" and roof["peak"] == 8000.0
    assert 0 < roof["frac"] == pytest.approx(roof["achieved"] / roof["peak"], abs=1e-3)
    assert roof["traffic"] is None            # PMC traffic is keyed to the 1024^3 workload only
    assert out["copy_peak"]["achieved"] > 0 and roof["frac_vs_copy_peak"] > 0
    fp = out["mapping_m1_3"]
    assert fp["value"] > 0 and 0 < fp["SumRange_frac"] < 1.2
    f32 = out["f32_linear"]
    assert f32["value"] > 0 and f32["halo_planes_per_rank"] == 0 and "Float32 Linear" in f32["workload"]
    cpu = out["cpu_baseline"]
    assert cpu["kind"] == "port" and cpu["cores"] == 1 and cpu["value"] > 0
