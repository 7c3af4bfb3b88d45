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


@pytest.mark.parametrize("n", [1, 2, 4, 8])
def test_config4_strong_layout(n):
    """The fixed 2048^3 config-4 volume over n GPUs: dst slabs partition 2048 planes, each rank
    holds exactly its own source planes (2048 / n dst planes from 1024 / n), nothing moves."""
    planes = []
    for rank in range(n):
        (d0, d1), (s0, s1), plan = bench.config4_layout(2048, n, rank)
        assert d1 - d0 == 2048 // n and (s0, s1) == (d0 // 2, d1 // 2)
        assert plan.halo_planes == 0 and not plan.sends and not plan.recvs
        planes += list(range(d0, d1))
    assert planes == list(range(2048))


@pytest.mark.gpu
@pytest.mark.parametrize("layout", [0, 2, 4])
def test_bench_config4_layout_rehearsal(layout):
    """config4_2048 on one GPU: the whole fixed volume (layout 0) or rank 0's slab of the
    2- / 4-GPU layout, at a reduced edge."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--dst", "128", "--steps", "3", "--warmup", "1",
           "--no-cpu-baseline", "--no-copy-peak", "--no-secondary", "--config4-edge", "512"]
    if layout:
        cmd += ["--layout-gpus", str(layout)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    c4 = out["config4_2048"]
    assert "error" not in c4, c4
    assert c4["scaling"] == "strong" and c4["global_dst"] == [512] * 3 and c4["value"] > 0
    assert c4["dst_planes_per_rank"] == 512 // max(layout, 1) and c4["halo_planes_per_rank"] == 0
    assert ("rank 0's slab only" in c4["workload"]) == (layout > 1)


@pytest.mark.gpu
def test_bench_small_run_prints_one_contract_line():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dst", "128", "--steps", "3",
                        "--warmup", "2", "--cpu-dst", "64", "--config4-edge", "256"], capture_output=True, text=True,
                       timeout=300, cwd=ROOT)
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
    assert out["config4_2048"]["value"] > 0 and out["config4_2048"]["scaling"] == "strong"
    mig = out["migrate"]
    assert "error" not in mig, mig
    for kind in ("pageable", "pinned"):
        assert mig[kind]["H2D_GBs"] > 0 and mig[kind]["D2H_GBs"] > 0, mig
    cpu = out["cpu_baseline"]
    assert cpu["kind"] == "port" and cpu["cores"] == 1 and cpu["value"] > 0


@pytest.mark.gpu
def test_bench_native_comm_leg_on_one_rank():
    """the f32_linear_native leg (libvolkit's own C-ABI communicator:
    vktHipCommGetUniqueId -> vktHipCommInitRank -> vktHipSlabExchangeHalo + vktHipResampleSlab
    and vktHipResampleSlabOverlapped) end to end on a one-rank communicator; its dst bytes equal
    the torch-transport leg's.  At N>1 with the nccl backend the same leg moves the halo over
    RCCL between GPUs (the driver's 8-GPU run)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dst", "128", "--steps", "4",
                        "--warmup", "1", "--no-cpu-baseline", "--no-copy-peak", "--no-config4", "--no-migrate",
                        "--native-comm"], capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    nat = out["f32_linear_native"]
    assert "error" not in nat, nat
    assert nat["value"] > 0 and nat["exchange_ms"] >= 0 and nat["overlapped_ms"] > 0
    assert nat["matches_torch_transport"] is True, (nat, out["f32_linear"])
    assert nat["dst_checksum"] == out["f32_linear"]["dst_checksum"]
    assert "one-rank communicator" in nat["transport"]
