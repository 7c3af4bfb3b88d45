"""Failure detection on the multi-rank paths (SURVEY.md §5 "Failure detection"):
a rank whose peer never joins its side of an exchange errors out within the configured timeout
instead of hanging (gloo, two ranks on the CPU), and bench.py's watchdog turns an overrunning
secondary measurement into the headline line with that field {"error": "timeout"} and a non-zero
exit."""
import json
import os
import socket
import subprocess
import sys
import textwrap
import time

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, timeout_s, q):
    import numpy as np
    import torch
    import torch.distributed as dist
    from volkit_amd import slab
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        slab.set_exchange_timeout(timeout_s)
        # Float32 Linear chain, 2 ranks: rank 0 receives its z+1 halo plane from rank 1
        plan = slab.plan_resample(16, 8, world, rank, 1, chain=True)
        l0, l1 = plan.local_src
        flat = torch.zeros((l1 - l0) * 4 * 4 * 4, dtype=torch.uint8)

        def planes(g0, g1):
            return flat[(g0 - l0) * 64:(g1 - l0) * 64]

        t0 = time.monotonic()
        if rank == 1:
            q.put((rank, "skipped", 0.0, bool(plan.sends or plan.recvs)))   # never joins the round
            time.sleep(timeout_s * 3)
            return
        try:
            slab.exchange_planes(plan, planes)
            q.put((rank, "completed", time.monotonic() - t0, bool(plan.recvs)))
        except RuntimeError as e:
            q.put((rank, "error: " + str(e)[:200], time.monotonic() - t0, bool(plan.recvs)))
    except Exception as e:   # noqa: BLE001 -- surfaced in the parent
        q.put((rank, "exception: " + repr(e)[:200], -1.0, False))
    finally:
        q.close()
        q.join_thread()   # flush the result before leaving
        os._exit(0)   # no teardown handshake with a peer that left the protocol


def test_exchange_with_absent_peer_times_out():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    timeout_s = 3.0
    procs = [ctx.Process(target=_worker, args=(r, 2, port, timeout_s, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda r: r[0])
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    (r0, what0, dt0, has0), (r1, what1, _, has1) = res
    assert has0 and has1, "the case must exchange planes between the two ranks"
    assert what1 == "skipped"
    assert what0.startswith("error:") and "within 3.0 s" in what0, what0
    assert timeout_s * 0.8 <= dt0 <= timeout_s + 20, dt0


def test_bench_watchdog_prints_line_and_exits_nonzero():
    """bench.guarded: a secondary that overruns its deadline makes the watchdog print the line as
    it stands with that field {"error": "timeout"} and end the process with WATCHDOG_EXIT."""
    code = textwrap.dedent(f"""
        import sys, time
        sys.path.insert(0, {ROOT!r})
        import bench
        out = {{"metric": "m", "value": 1.0}}
        out["fast"] = bench.guarded(out, "fast", lambda: {{"ok": 1}}, 30.0, 0)
        out["slow"] = bench.guarded(out, "slow", lambda: time.sleep(60), 1.0, 0)
        print("not reached")
    """)
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert time.monotonic() - t0 < 30
    import bench
    assert r.returncode == bench.WATCHDOG_EXIT, (r.returncode, r.stderr[-1000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and "not reached" not in r.stdout, r.stdout
    out = json.loads(lines[0])
    assert out["value"] == 1.0 and out["fast"] == {"ok": 1}
    assert out["slow"]["error"] == "timeout"
    assert "watchdog" in r.stderr


def test_bench_watchdog_quiet_when_in_time():
    import bench
    out = {}
    calls = []
    assert bench.guarded(out, "x", lambda: {"v": 2}, 5.0, 0, exit_fn=calls.append) == {"v": 2}
    time.sleep(0.1)
    assert calls == [] and "x" not in out
    # an exception is still recorded in the line, not a watchdog exit
    got = bench.guarded(out, "y", lambda: 1 / 0, 5.0, 0, exit_fn=calls.append)
    assert "ZeroDivisionError" in got["error"] and calls == []
