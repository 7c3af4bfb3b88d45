"""Benchmark: Resample + SumRange on UInt16 volumes, BASELINE.json's headline metric.

One step = the metric pipeline on device-resident synthetic data:
    Resample(R, S, Linear)      S = 512^3 UInt16  ->  R = 1024^3 UInt16
    SumRange(D, R, B, 0, dims)  B, D = 1024^3 UInt16
per GPU.  With N GPUs (torchrun, one process per GPU, RCCL) the volumes are Z-slab
partitioned and the global grid doubles one axis per doubling of N (x, then y, then z):
N=1 1024^3, N=2 2048x1024x1024, N=4 2048x2048x1024, N=8 2048^3 (BASELINE config 4:
1024^3 -> 2048^3 + SumRange 2048^3), the source being half of it per axis.  Every rank owns
1024^3 dst voxels (weak scaling).  The exact z index table keeps every rank's reads in its
own source slab for this ratio and format, so no plane crosses ranks (the exchange plan is
still computed and executed -- it is empty).  --layout-gpus M runs rank 0's
slab of the M-GPU layout on one GPU (per-rank rehearsal of the multi-GPU shapes).

value = dst voxels of all ranks / wall time per step (Gvoxels/s).  roofline: the dominant
kernel (SumRange: 6 B/voxel algorithmic) timed with HIP events on the library's compute
stream.  After the timed region, secondary measurements go into the same JSON line (none of
them is `value`):
  * mapping_m1_3   -- the same pipeline with mapping [-1, 3] on every volume (the float-codec
                      kernels; SURVEY §8(d) "a second run uses mapping [-1,3]");
  * f32_linear     -- Float32 "Linear" Resample with the z+1 halo plane exchanged between
                      neighbour ranks over torch.distributed on device tensors (RCCL over
                      xGMI at N>1): per rank 512^3 -> 1024^3 of the same global layout;
  * f32_linear_native -- the same leg through the library's own C-ABI communicator
                      (vktHipCommGetUniqueId broadcast over the process group ->
                      vktHipCommInitRank -> vktHipSlabExchangeHalo + vktHipResampleSlab, and
                      vktHipResampleSlabOverlapped): at N>1 with the nccl backend, or with
                      --native-comm on a one-rank communicator; its dst equals the torch path's;
  * config4_2048   -- BASELINE config 4 in its STRONG-scaling form: the fixed global volume
                      1024^3 -> 2048^3 Resample + SumRange 2048^3 UInt16 Z-slab partitioned over
                      the N GPUs launched (at N=1 the whole 2048^3 on one GPU, ~50 GiB of
                      volumes): the denominator and numerator of BASELINE.md §4's speedup;
  * migrate        -- ManagedBuffer::migrate() host<->HBM GB/s of one 2 GiB UInt16 volume, pageable
                      and pinned host memory (N=1; SURVEY §8(a) A2, reported apart from the roofline);
  * copy_peak      -- the library's own Copy 1024^3 UInt16, the achievable streaming rate;
  * cpu_baseline   -- the oracle port (1 thread) on the full 1024^3 pipeline and on 512^3.
"""
import argparse
import ctypes as C
import datetime
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X spec (MI355X_MICROARCH.md: HBM3E 8.0 TB/s)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    # the first ~10-20 ms of sustained streaming run below the steady HBM rate (measured with
    # dev/kbench/libbench.cpp: 1.09 ms per SumRange in the first 10 launches, 1.01 ms after), so the
    # default warm-up covers ~35 ms; an explicit --warmup is honoured as given
    p.add_argument("--warmup", type=int, default=25)
    p.add_argument("--dst", type=int, default=1024, help="per-GPU dst cube edge (source = dst/2)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-copy-peak", action="store_true", help="skip the library-Copy achievable peak")
    p.add_argument("--no-secondary", action="store_true",
                   help="skip the mapping [-1,3] and Float32-Linear secondary measurements")
    p.add_argument("--cpu-dst", type=int, default=1024, help="dst edge of the CPU-baseline run")
    p.add_argument("--config4-edge", type=int, default=2048,
                   help="dst edge of the fixed global config-4 volume (strong scaling; source = edge/2)")
    p.add_argument("--no-config4", action="store_true", help="skip the strong-scaling config-4 measurement")
    p.add_argument("--no-migrate", action="store_true", help="skip the host<->HBM migrate() measurement (N=1 only)")
    p.add_argument("--layout-gpus", type=int, default=0,
                   help="single process: run rank 0's slab of the M-GPU global layout")
    p.add_argument("--dist-backend", default="nccl",
                   help="torch.distributed backend for N>1 (nccl = RCCL over xGMI; gloo only for rehearsal)")
    p.add_argument("--rehearse-one-device", action="store_true",
                   help="put every rank on device 0 (multi-rank rehearsal on a 1-GPU box, with --dist-backend gloo)")
    p.add_argument("--native-comm", action="store_true",
                   help="run the f32_linear_native leg also at N=1 (a one-rank communicator; at N>1 with the "
                        "nccl backend it always runs)")
    p.add_argument("--dist-timeout", type=float, default=300.0,
                   help="seconds: torch.distributed process-group timeout (collectives and p2p waits)")
    p.add_argument("--secondary-timeout", type=float, default=120.0,
                   help="seconds one secondary measurement may take before the watchdog prints the line "
                        "with that field {'error': 'timeout'} and exits non-zero")
    return p.parse_args()


def global_dims(edge, n):
    """Global dst dims for n GPUs: edge^3, doubling x, y, z in turn for each doubling of n
    (n=8 -> (2*edge)^3, BASELINE config 4).  Non-powers of two stack slabs in z."""
    dims = [edge, edge, edge]
    if n & (n - 1) == 0:
        k = 0
        while (1 << k) < n:
            dims[k % 3] *= 2
            k += 1
    else:
        dims[2] *= n
    return dims


def cpu_baseline(dst_edge):
    """Oracle (C restatement of the reference serial path, 1 thread) on the same pipeline at
    dst_edge^3; returns (Gvoxels/s of dst voxels, seconds)."""
    from oracle import binding as ob

    s = dst_edge // 2
    src = ob.Volume(ob.synth_codes((s, s, s), 5, 0x5EED), 5)
    b = ob.Volume(ob.synth_codes((dst_edge,) * 3, 5, 0x5EED + 1), 5)
    r = ob.Volume.zeros((dst_edge,) * 3, 5)
    d = ob.Volume.zeros((dst_edge,) * 3, 5)
    t0 = time.perf_counter()
    ob.resample(r, src, 1)
    ob.arith_range("Sum", d, r, b, (0, 0, 0), (dst_edge,) * 3)
    dt = time.perf_counter() - t0
    return dst_edge ** 3 / dt / 1e9, dt


class Ctx:
    """Process-group / stream context shared by the measurements."""

    def __init__(self, torch, dist, world, rank, backend):
        self.torch, self.dist, self.world, self.rank, self.backend = torch, dist, world, rank, backend

    def barrier_sync(self):
        self.torch.cuda.synchronize()
        if self.world > 1:
            self.dist.barrier()
        self.torch.cuda.synchronize()

    def max_over_ranks(self, x):
        if self.world == 1:
            return x
        dev = "cuda" if self.backend == "nccl" else "cpu"
        t = self.torch.tensor([x], device=dev, dtype=self.torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def timed(self, step, steps, warmup, nev):
        """warmup untimed steps, then `steps` timed steps between barrier + synchronize on both
        sides; step(ev) records nev+1 events.  Returns (max-over-ranks seconds, per-interval
        mean kernel ms)."""
        torch = self.torch
        for _ in range(warmup):
            step(None)
        self.barrier_sync()
        evs = []
        t0 = time.perf_counter()
        for _ in range(steps):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(nev + 1)]
            step(ev)
            evs.append(ev)
        self.barrier_sync()
        elapsed = self.max_over_ranks(time.perf_counter() - t0)
        ms = [sum(e[i].elapsed_time(e[i + 1]) for e in evs) / len(evs) for i in range(nev)]
        return elapsed, ms


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.rehearse_one_device:
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        # a dead or diverged peer fails the collective after --dist-timeout instead of hanging;
        # the secondaries' watchdog (below) fires first and still reports the headline
        pg_timeout = datetime.timedelta(seconds=args.dist_timeout)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=pg_timeout)
        else:
            dist.init_process_group(args.dist_backend, timeout=pg_timeout)
        from volkit_amd import slab as _slab
        _slab.set_exchange_timeout(args.dist_timeout)

    import volkit_amd.volkit as vkt
    from volkit_amd import slab
    from volkit_amd._lib import lib, HipVolumeView_t

    if lib.vktHipSetDevice(local) != 0:
        raise RuntimeError(vkt.last_error())
    # One dedicated (non-NULL) stream for our kernels and for torch's events / RCCL calls:
    # torch's default stream is the legacy NULL stream, which would serialise against the
    # backend's blocking stream at every event record.  Events are recorded on the stream the
    # library reports as its compute stream (the same one), so they bracket its kernels.
    own = torch.cuda.Stream()
    lib.vktHipSetComputeStream(C.c_void_p(own.cuda_stream))
    sp = C.c_void_p()
    lib.vktHipGetComputeStream(C.byref(sp))
    stream = torch.cuda.ExternalStream(sp.value)
    torch.cuda.set_stream(stream)
    ctx = Ctx(torch, dist, world, rank, args.dist_backend)

    ep = vkt.GetThreadExecutionPolicy()
    ep.device = vkt.ExecutionPolicy.Device_GPU
    vkt.SetThreadExecutionPolicy(ep)

    UINT16, FLOAT32, LINEAR = vkt.DataFormat_UInt16, vkt.DataFormat_Float32, vkt.FilterMode_Linear
    layout_n = world
    if args.layout_gpus:
        if world != 1:
            raise SystemExit("--layout-gpus is a single-process option")
        layout_n = args.layout_gpus
    DX, DY, dst_gdz = global_dims(args.dst, layout_n)
    SX, SY, src_gdz = DX // 2, DY // 2, dst_gdz // 2
    plan = slab.plan_resample(dst_gdz, src_gdz, layout_n, rank, LINEAR, chain=False)
    ls0, ls1 = plan.local_src
    dz0, dz1 = plan.dst

    # device-resident volumes (allocated on HBM directly: GPU policy at construction)
    Sv = vkt.StructuredVolume(SX, SY, ls1 - ls0, UINT16)
    Rv = vkt.StructuredVolume(DX, DY, dz1 - dz0, UINT16)
    Bv = vkt.StructuredVolume(DX, DY, dz1 - dz0, UINT16)
    Dv = vkt.StructuredVolume(DX, DY, dz1 - dz0, UINT16)
    for k, v in enumerate((Sv, Bv)):
        assert vkt.Synthesize(v, 0x5EED + k + 1000 * rank) == 0, vkt.last_error()
    sview, rview, bview, dview = Sv.hip_view(), Rv.hip_view(), Bv.hip_view(), Dv.hip_view()
    first = _lib_vec(0, 0, 0)
    last = _lib_vec(DX, DY, dz1 - dz0)
    plane_bytes = SX * SY * 2

    def planes(g0, g1):
        return slab.device_tensor(sview.data + (g0 - ls0) * plane_bytes, (g1 - g0) * plane_bytes)

    def pipeline(views):
        s_, r_, b_, d_ = views

        def step(ev):
            if plan.recvs or plan.sends:
                slab.exchange_planes(plan, planes)
            if ev:
                ev[0].record(stream)
            e1 = lib.vktHipResampleSlab(r_, s_, LINEAR, dst_gdz, dz0, src_gdz, ls0)
            if ev:
                ev[1].record(stream)
            e2 = lib.vktHipArithmeticRange(0, d_, r_, b_, first, last, _lib_vec(0, 0, 0))
            if ev:
                ev[2].record(stream)
            if e1 or e2:
                raise RuntimeError(vkt.last_error())
        return step

    elapsed, (res_ms, sum_ms) = ctx.timed(pipeline((sview, rview, bview, dview)), args.steps, args.warmup, 2)
    ms_per_step = elapsed * 1e3 / args.steps
    vox_rank = DX * DY * (dz1 - dz0)
    total_vox = vox_rank * world
    value = total_vox / (ms_per_step / 1e3) / 1e9

    # algorithmic bytes per launch: SumRange 6 B/voxel; Resample
    # N_src*2 + N_dst*2
    sum_bytes = 6 * vox_rank
    res_bytes = 2 * SX * SY * (ls1 - ls0) + 2 * vox_rank
    pipe_bytes = sum_bytes + res_bytes
    traffic = None
    tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tf):
        try:
            pm = json.load(open(tf))
            if pm.get("bench_dst_edge") == args.dst and layout_n == 1:   # only for the workload the counters were taken on
                traffic = pm.get("SumRange_bytes_per_launch")
        except Exception:
            traffic = None

    def gbs(nbytes, ms):
        return round(nbytes / (ms / 1e3) / 1e9, 1)

    out = {
        "metric": "Gvoxels/s + achieved HBM GB/s, Resample+SumRange 1024^3 UInt16",
        "value": round(value, 3),
        "unit": "Gvoxels/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u16",
        "data": "synthetic (splitmix64 codes, device-resident)",
        "config": {
            "workload": f"Resample {SX}x{SY}x{src_gdz}->{DX}x{DY}x{dst_gdz} UInt16 Linear + SumRange "
                        f"{DX}x{DY}x{dst_gdz} UInt16, Z-slab over {layout_n} GPU(s)"
                        + (" (rank 0's slab only, on 1 GPU)" if layout_n != world else ""),
            "global_dst": [DX, DY, dst_gdz], "global_src": [SX, SY, src_gdz],
            "slab_dst_per_rank": [DX, DY, dz1 - dz0],
            "parallelism": f"zslab{layout_n}", "halo_planes_per_rank": plan.halo_planes,
        },
        "pipeline_hbm_gbs": round(pipe_bytes * world / (ms_per_step / 1e3) / 1e9, 1),
        "kernels_ms": {"Resample": round(res_ms, 4), "SumRange": round(sum_ms, 4)},
        "roofline": {
            "kernel": "SumRange (arithmetic pointwise, UInt16)",
            "bound": "hbm",
            "achieved": gbs(sum_bytes, sum_ms),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(sum_bytes / (sum_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "resample_achieved": gbs(res_bytes, res_ms),
            "pipeline_frac": round(pipe_bytes / ((res_ms + sum_ms) / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "resample_note": "resample_achieved = algorithmic bytes (N_src*2 + N_dst*2) / event time, not a "
                             "sustained HBM rate: each source line is read by several dst rows and can be "
                             "served from the caches (Infinity Cache hits are counted in FETCH_SIZE too)",
        },
    }

    if not args.no_secondary:
        # same pipeline, same buffers, mapping [-1, 3] on every volume: the float codec runs
        # (the unit-mapping integer specialisations of DESIGN §4.1 do not apply)
        fp = [HipVolumeView_t(v.data, v.dimX, v.dimY, v.dimZ, v.dataFormat, -1.0, 3.0)
              for v in (sview, rview, bview, dview)]
        def mapping_m1_3():
            el_fp, (res_fp, sum_fp) = ctx.timed(pipeline(fp), args.steps, max(5, args.warmup // 2), 2)
            msfp = el_fp * 1e3 / args.steps
            return {
                "value": round(total_vox / (msfp / 1e3) / 1e9, 3), "unit": "Gvoxels/s",
                "ms_per_step": round(msfp, 4),
                "kernels_ms": {"Resample": round(res_fp, 4), "SumRange": round(sum_fp, 4)},
                "SumRange_achieved": gbs(sum_bytes, sum_fp),
                "SumRange_frac": round(sum_bytes / (sum_fp / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                "resample_achieved": gbs(res_bytes, res_fp),
                "note": "same workload and buffers, mapping [-1,3] on all volumes (float-codec kernels)",
            }
        # a failing secondary measurement is recorded in the line instead of losing the headline
        # (the failures these guard against -- a library error, an allocation -- are the same on
        # every rank, so no rank is left waiting in a collective); one that overruns (a peer that
        # never arrives in an exchange) trips the watchdog, which prints the line and exits
        out["mapping_m1_3"] = guarded(out, "mapping_m1_3", mapping_m1_3, args.secondary_timeout, rank)
        out["f32_linear"] = guarded(out, "f32_linear",
                                    lambda: f32_linear(ctx, vkt, slab, lib, args, layout_n, stream),
                                    args.secondary_timeout, rank)
        # the library's own RCCL transport (C ABI): where a real exchange runs, or on request
        if layout_n == world and (args.native_comm or (world > 1 and args.dist_backend == "nccl")):
            want = out["f32_linear"].get("dst_checksum") if isinstance(out["f32_linear"], dict) else None
            out["f32_linear_native"] = guarded(out, "f32_linear_native",
                                               lambda: f32_linear_native(ctx, vkt, slab, lib, args, stream, want),
                                               args.secondary_timeout, rank)
    if not args.no_config4:
        out["config4_2048"] = guarded(out, "config4_2048",
                                      lambda: config4_strong(ctx, vkt, slab, lib, args, layout_n, stream),
                                      args.secondary_timeout, rank)

    if not args.no_migrate and world == 1:
        out["migrate"] = guarded(out, "migrate", lambda: migrate_rates(vkt, lib, args.dst), args.secondary_timeout, rank)

    if not args.no_copy_peak:
        # achievable streaming rate on this box: the library's own CopyRange of one volume
        # (vector pointwise kernel, read + write bytes), after the timed regions
        def copy_step(ev):
            if ev:
                ev[0].record(stream)
            if lib.vktHipCopyRange(dview, bview, first, last, _lib_vec(0, 0, 0)):
                raise RuntimeError(vkt.last_error())
            if ev:
                ev[1].record(stream)
        _, (copy_ms,) = ctx.timed(copy_step, 10, 3, 1)
        copy_gbs = gbs(4 * vox_rank, copy_ms)
        out["copy_peak"] = {"kernel": f"CopyRange {DX}x{DY}x{dz1 - dz0} UInt16 (library)", "ms": round(copy_ms, 4),
                            "achieved": copy_gbs, "unit": "GB/s"}
        out["roofline"]["frac_vs_copy_peak"] = round(out["roofline"]["achieved"] / copy_gbs, 4)

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        gv, dt = cpu_baseline(args.cpu_dst)
        at512 = None
        if args.cpu_dst > 512:
            gv512, dt512 = cpu_baseline(512)
            at512 = {"value": round(gv512, 5), "seconds": round(dt512, 2)}
        # the compiled reference serial path, measured in the survey container
        # (1 thread, g++ -O2): SumRange UInt16 33.8-37.9 ns/voxel + Resample UInt16 Linear 41.5
        # ns/dst voxel -> ~77.4 ns per pipeline voxel.  The port skips the reference's per-voxel
        # migrate() + policy lookup; the calibration factor is reference ns / port ns, with the
        # port's ns measured here (the reference does not travel to the GPU box).
        ref_ns = (33.8 + 37.9) / 2 + 41.5
        port_ns = dt * 1e9 / args.cpu_dst ** 3
        out["cpu_baseline"] = {
            "value": round(gv, 5), "unit": "Gvoxels/s", "cores": 1, "kind": "port",
            "sample": f"oracle restatement of the reference serial path on the full headline workload: "
                      f"Resample {args.cpu_dst // 2}^3->{args.cpu_dst}^3 UInt16 Linear + SumRange "
                      f"{args.cpu_dst}^3, {dt:.1f} s, 1 thread of {os.cpu_count()} host CPUs",
            "at_512": at512,
            "reference_equivalent": {
                "value": round(1.0 / (ref_ns * 1e-9) / 1e9, 5), "unit": "Gvoxels/s",
                "calibration_factor": round(ref_ns / port_ns, 3),
                "basis": "BASELINE.md §2 survey probe of the compiled reference (1 core), "
                         "reference ns/voxel / port ns/voxel measured here"},
        }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def secondary(fn):
    """Run one secondary measurement; an exception becomes {"error": ...} in the JSON line."""
    try:
        return fn()
    except Exception as e:   # noqa: BLE001 -- reported, not swallowed
        print(f"bench: secondary measurement failed: {e!r}", file=sys.stderr, flush=True)
        return {"error": repr(e)[:300]}


WATCHDOG_EXIT = 3


def guarded(out, name, fn, seconds, rank, exit_fn=None):
    """secondary(fn) under a watchdog: if it has not returned after `seconds` (a peer that never
    joins an exchange or collective blocks every rank), the watchdog thread sets out[name] to
    {"error": "timeout"}, has rank 0 print the line as it stands -- the headline is measured
    before any secondary -- and ends the process with WATCHDOG_EXIT (no re-exec; exit_fn for
    tests).  Fires before the process-group timeout (--dist-timeout), whose handler would abort
    the process without a line."""
    fired = threading.Event()

    def fire():
        fired.set()
        out[name] = {"error": "timeout", "seconds": seconds,
                     "note": "watchdog: the measurement did not finish; line printed, process ended"}
        if rank == 0:
            print(json.dumps(out), flush=True)
        print(f"bench: watchdog: secondary '{name}' exceeded {seconds} s", file=sys.stderr, flush=True)
        (exit_fn or os._exit)(WATCHDOG_EXIT)

    t = threading.Timer(seconds, fire)
    t.daemon = True
    t.start()
    try:
        return secondary(fn)
    finally:
        t.cancel()


def f32_linear(ctx, vkt, slab, lib, args, layout_n, stream):
    """Float32 Linear Resample, per rank (dst/2)^3 -> dst^3 of the global layout, source
    uniform in [0, 1) (BASELINE config 3's input), with the chain's z+1 halo planes exchanged
    between neighbour ranks on device tensors (torch.distributed: RCCL over xGMI at N>1)."""
    torch = ctx.torch
    rank, world = ctx.rank, ctx.world
    LINEAR, FLOAT32 = vkt.FilterMode_Linear, vkt.DataFormat_Float32
    DX, DY, dgz = global_dims(args.dst, layout_n)
    SX, SY, sgz = DX // 2, DY // 2, dgz // 2
    plan = slab.plan_resample(dgz, sgz, layout_n, rank, LINEAR, chain=True)
    ls0, ls1 = plan.local_src
    o0, o1 = plan.owned_src
    dz0, dz1 = plan.dst
    S = vkt.StructuredVolume(SX, SY, ls1 - ls0, FLOAT32)
    R = vkt.StructuredVolume(DX, DY, dz1 - dz0, FLOAT32)
    sv, rv = S.hip_view(), R.hip_view()
    plane = SX * SY * 4
    src_t = slab.device_tensor(sv.data, (ls1 - ls0) * plane).view(torch.float32)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(0x5EED + rank)
    src_t.uniform_(0.0, 1.0, generator=gen)   # halo planes are overwritten by the exchange
    torch.cuda.synchronize()

    def planes(g0, g1):
        return slab.device_tensor(sv.data + (g0 - ls0) * plane, (g1 - g0) * plane)

    def step(ev):
        if ev:
            ev[0].record(stream)
        if exchanging:
            slab.exchange_planes(plan, planes)
        if ev:
            ev[1].record(stream)
        if lib.vktHipResampleSlab(rv, sv, LINEAR, dgz, dz0, sgz, ls0):
            raise RuntimeError(vkt.last_error())
        if ev:
            ev[2].record(stream)

    exchanging = world > 1 and bool(plan.recvs or plan.sends)   # (--layout-gpus: rank 0's slab alone)

    def step_overlapped(ev):
        # the exchange in flight while the interior dst planes (owned sources only) resample
        if ev:
            ev[0].record(stream)
        if slab.resample_slab_overlapped(rv, sv, LINEAR, plan, True, planes):
            raise RuntimeError(vkt.last_error())
        if ev:
            ev[1].record(stream)

    steps = max(5, args.steps // 2)
    elapsed, (ex_ms, res_ms) = ctx.timed(step, steps, 3, 2)
    ms = elapsed * 1e3 / steps
    serial_ms = ms
    if exchanging:
        elapsed_o, _ = ctx.timed(step_overlapped, steps, 3, 1)
        ms = elapsed_o * 1e3 / steps
    vox = DX * DY * (dz1 - dz0)
    nbytes = 4 * SX * SY * (o1 - o0) + 4 * vox
    checksum = dst_checksum(torch, rv)
    out = {
        "dst_checksum": checksum,
        "workload": f"Resample {SX}x{SY}x{sgz}->{DX}x{DY}x{dgz} Float32 Linear (source uniform [0,1)), "
                    f"Z-slab over {layout_n} GPU(s), z+1 halo exchanged on device tensors "
                    f"({'RCCL' if ctx.backend == 'nccl' and world > 1 else ctx.backend if world > 1 else 'none'})",
        "value": round(vox * world / (ms / 1e3) / 1e9, 3), "unit": "Gvoxels/s", "ms_per_step": round(ms, 4),
        "resample_ms": round(res_ms, 4), "exchange_ms": round(ex_ms, 4),
        "ms_per_step_serial_exchange": round(serial_ms, 4),
        "overlap": ("halo exchange overlapped with the interior planes (slab.resample_slab_overlapped), "
                    f"interior dst planes {slab.interior_split(plan, LINEAR, True) - dz0} of {dz1 - dz0}")
        if exchanging else "no exchange",
        "halo_planes_per_rank": plan.halo_planes, "halo_bytes_per_rank": plan.halo_planes * plane,
        "resample_achieved": round(nbytes / (res_ms / 1e3) / 1e9, 1),
        "resample_frac": round(nbytes / (res_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
    }
    del S, R
    return out


def dst_checksum(torch, view):
    """Sum of the dst slab's 32-bit words (int64): the bytes of one leg against another's."""
    from volkit_amd import slab
    words = slab.device_tensor(view.data, view.dimX * view.dimY * view.dimZ * 4).view(torch.int32)
    return int(words.sum(dtype=torch.int64).item())


def f32_linear_native(ctx, vkt, slab, lib, args, stream, want_checksum):
    """f32_linear's workload with the halo moved by the library's own communicator (the C-ABI
    multi-GPU surface, include/volkit_hip.h; design intent reference include/c/vkt/CudaContext.h:
    41-65): rank 0's vktHipCommGetUniqueId broadcast over the process group, vktHipCommInitRank,
    then per step (a) vktHipSlabExchangeHalo + vktHipResampleSlab (one RCCL group round on the
    library's compute stream, then the resample) and (b) vktHipResampleSlabOverlapped (the round
    on the communicator's stream under the interior planes).  Both legs' dst bytes are checked
    against the torch-transport leg's checksum."""
    import torch
    from volkit_amd._lib import HipCommId_t
    rank, world = ctx.rank, ctx.world
    LINEAR, FLOAT32 = vkt.FilterMode_Linear, vkt.DataFormat_Float32
    DX, DY, dgz = global_dims(args.dst, world)
    SX, SY, sgz = DX // 2, DY // 2, dgz // 2
    plan = slab.plan_resample(dgz, sgz, world, rank, LINEAR, chain=True)
    ls0, ls1 = plan.local_src
    dz0, dz1 = plan.dst
    uid = HipCommId_t()
    if rank == 0 and lib.vktHipCommGetUniqueId(C.byref(uid)) != 0:
        raise RuntimeError(vkt.last_error())
    if world > 1:
        dev = "cuda" if ctx.backend == "nccl" else "cpu"
        t = torch.frombuffer(bytearray(C.string_at(C.addressof(uid), C.sizeof(uid))), dtype=torch.uint8).to(dev)
        ctx.dist.broadcast(t, src=0)
        C.memmove(C.addressof(uid), bytes(t.cpu().numpy().tobytes()), C.sizeof(uid))
    comm = C.c_void_p()
    if lib.vktHipCommInitRank(C.byref(comm), world, uid, rank) != 0:
        raise RuntimeError(vkt.last_error())
    S = R = None
    try:
        if lib.vktHipCommSetTimeout(comm, int(args.dist_timeout * 1000)) != 0:
            raise RuntimeError(vkt.last_error())
        S = vkt.StructuredVolume(SX, SY, ls1 - ls0, FLOAT32)
        R = vkt.StructuredVolume(DX, DY, dz1 - dz0, FLOAT32)
        sv, rv = S.hip_view(), R.hip_view()
        src_t = slab.device_tensor(sv.data, (ls1 - ls0) * SX * SY * 4).view(torch.float32)
        gen = torch.Generator(device="cuda")
        gen.manual_seed(0x5EED + rank)              # the f32_linear leg's source, bit for bit
        src_t.uniform_(0.0, 1.0, generator=gen)
        torch.cuda.synchronize()

        def step(ev):
            if ev:
                ev[0].record(stream)
            if lib.vktHipSlabExchangeHalo(comm, sv, ls0, dgz, sgz, LINEAR, 1) != 0:
                raise RuntimeError(vkt.last_error())
            if ev:
                ev[1].record(stream)
            if lib.vktHipResampleSlab(rv, sv, LINEAR, dgz, dz0, sgz, ls0) != 0:
                raise RuntimeError(vkt.last_error())
            if ev:
                ev[2].record(stream)

        def step_overlapped(ev):
            if ev:
                ev[0].record(stream)
            if lib.vktHipResampleSlabOverlapped(comm, rv, sv, ls0, dgz, sgz, LINEAR, 1) != 0:
                raise RuntimeError(vkt.last_error())
            if ev:
                ev[1].record(stream)

        steps = max(5, args.steps // 2)
        elapsed, (ex_ms, res_ms) = ctx.timed(step, steps, 3, 2)
        if lib.vktHipCommSynchronize(comm) != 0:
            raise RuntimeError(vkt.last_error())
        serial_sum = dst_checksum(torch, rv)
        R_bytes = slab.device_tensor(rv.data, DX * DY * (dz1 - dz0) * 4)
        R_bytes.fill_(0)
        elapsed_o, (ov_ms,) = ctx.timed(step_overlapped, steps, 3, 1)
        if lib.vktHipCommSynchronize(comm) != 0:
            raise RuntimeError(vkt.last_error())
        overlapped_sum = dst_checksum(torch, rv)
        vox = DX * DY * (dz1 - dz0)
        ms = elapsed_o * 1e3 / steps
        return {
            "workload": f"Resample {SX}x{SY}x{sgz}->{DX}x{DY}x{dgz} Float32 Linear, Z-slab over {world} GPU(s), "
                        f"z+1 halo moved by libvolkit's communicator (RCCL, C ABI)",
            "transport": "vktHipCommInitRank + vktHipSlabExchangeHalo / vktHipResampleSlabOverlapped "
                         f"({'RCCL over xGMI' if world > 1 else 'one-rank communicator: no plane moves'})",
            "value": round(vox * world / (ms / 1e3) / 1e9, 3), "unit": "Gvoxels/s", "ms_per_step": round(ms, 4),
            "ms_per_step_serial_exchange": round(elapsed * 1e3 / steps, 4),
            "exchange_ms": round(ex_ms, 4), "resample_ms": round(res_ms, 4), "overlapped_ms": round(ov_ms, 4),
            "halo_planes_per_rank": plan.halo_planes,
            "matches_torch_transport": (want_checksum is not None and serial_sum == want_checksum
                                        and overlapped_sum == want_checksum),
            "dst_checksum": overlapped_sum,
        }
    finally:
        del S, R
        lib.vktHipCommDestroy(comm)


PCIE_PEAK_GBS = 63.0   # MI355X host link, PCIe Gen5 x16 per direction (MI355X_MICROARCH.md)


def migrate_rates(vkt, lib, edge, reps=3):
    """SURVEY §8(a) A2, reported apart from the kernel roofline: ManagedBuffer::migrate of one
    UInt16 edge^3 volume (2 GiB at 1024^3) between host memory and HBM at a device flip of the
    thread policy (reference include/cpp/vkt/ManagedBuffer.hpp:168-198 -> runtime/Memory.cpp
    MigrateBuffer: allocate on the new side, one copy on the side copy stream, free the old side).
    Pageable host buffers (malloc, the reference's behaviour) and pinned ones
    (vktHipSetPinnedHostAllocation).  H2D: the host volume (pages written) to HBM; D2H: back into
    the host buffer the H2D released (the library keeps it, pages resident, for the migration
    back), and `D2H_fresh_*`: one D2H after vktHipReleaseCachedMemory, into a FRESH host
    allocation whose pages the library faults in first.  Best of `reps` round trips; GB/s of the
    volume's bytes."""
    import numpy as np
    cpu, gpu = vkt.ExecutionPolicy.Device_CPU, vkt.ExecutionPolicy.Device_GPU

    def policy(dev):
        ep = vkt.GetThreadExecutionPolicy()
        ep.device = dev
        vkt.SetThreadExecutionPolicy(ep)

    res = {"volume": f"{edge}^3 UInt16", "bytes": 2 * edge ** 3, "pcie_peak_GBs": PCIE_PEAK_GBS,
           "note": "host<->HBM migrate() over PCIe; not part of value (inputs are device-resident)"}
    try:
        for pinned in (False, True):
            lib.vktHipSetPinnedHostAllocation(1 if pinned else 0)
            policy(cpu)
            v = vkt.StructuredVolume(edge, edge, edge, vkt.DataFormat_UInt16)
            v.from_numpy(np.full((edge, edge, edge), 0x1234, np.uint16))
            nbytes = v.getSizeInBytes()
            h2d, d2h = [], []
            for _ in range(reps):
                policy(gpu)
                t0 = time.perf_counter()
                v.migrate()
                if lib.vktHipSynchronize() != 0:
                    raise RuntimeError(vkt.last_error())
                h2d.append(time.perf_counter() - t0)
                policy(cpu)
                t0 = time.perf_counter()
                v.migrate()
                d2h.append(time.perf_counter() - t0)
            # one more round trip with the host caches emptied before the D2H
            policy(gpu)
            v.migrate()
            if lib.vktHipSynchronize() != 0 or lib.vktHipReleaseCachedMemory(None) != 0:
                raise RuntimeError(vkt.last_error())
            policy(cpu)
            t0 = time.perf_counter()
            v.migrate()
            d2h_fresh = time.perf_counter() - t0
            if v.getValue(3, 2, 1) != 0x1234 / 65536.0:
                raise RuntimeError("migrate round trip changed the data")
            del v
            key = "pinned" if pinned else "pageable"
            res[key] = {"H2D_GBs": round(nbytes / min(h2d) / 1e9, 2), "D2H_GBs": round(nbytes / min(d2h) / 1e9, 2),
                        "H2D_ms": round(min(h2d) * 1e3, 2), "D2H_ms": round(min(d2h) * 1e3, 2),
                        "D2H_fresh_GBs": round(nbytes / d2h_fresh / 1e9, 2), "D2H_fresh_ms": round(d2h_fresh * 1e3, 2)}
    finally:
        lib.vktHipSetPinnedHostAllocation(0)
        policy(gpu)
    return res


def config4_layout(edge, n, rank):
    """BASELINE config 4, strong scaling: ONE global volume -- source (edge/2)^3 UInt16, dst and
    SumRange edge^3 -- Z-slab partitioned over n GPUs.  Returns rank's (dst planes, source planes
    held, exchange plan); for edge/2 divisible by n every dst slab reads only its own source
    planes (UInt16 "Linear" = Nearest exactly), so the plan is empty."""
    from volkit_amd import slab
    plan = slab.plan_resample(edge, edge // 2, n, rank, 1, chain=False)
    return plan.dst, plan.local_src, plan


def config4_strong(ctx, vkt, slab, lib, args, layout_n, stream):
    """The fixed config-4 volume over the launched ranks: value = edge^3 dst voxels per step
    (each rank its slab; max-over-ranks time), so value(N) / value(1) is the strong-scaling
    speedup BASELINE.md §4 quotes (8.86 ms on 1 GPU vs 1.11 ms per GPU at 8 on A100s)."""
    torch = ctx.torch
    rank, world = ctx.rank, ctx.world
    E = args.config4_edge
    Sx = E // 2
    UINT16, LINEAR = vkt.DataFormat_UInt16, vkt.FilterMode_Linear
    (dz0, dz1), (ls0, ls1), plan = config4_layout(E, layout_n, rank)
    S = vkt.StructuredVolume(Sx, Sx, ls1 - ls0, UINT16)
    R = vkt.StructuredVolume(E, E, dz1 - dz0, UINT16)
    B = vkt.StructuredVolume(E, E, dz1 - dz0, UINT16)
    D = vkt.StructuredVolume(E, E, dz1 - dz0, UINT16)
    for k, v in enumerate((S, B)):
        assert vkt.Synthesize(v, 0x5EED + 40 + k + 1000 * rank) == 0, vkt.last_error()
    sv, rv, bv, dv = S.hip_view(), R.hip_view(), B.hip_view(), D.hip_view()
    plane = Sx * Sx * 2
    first, last, zero = _lib_vec(0, 0, 0), _lib_vec(E, E, dz1 - dz0), _lib_vec(0, 0, 0)

    def planes(g0, g1):
        return slab.device_tensor(sv.data + (g0 - ls0) * plane, (g1 - g0) * plane)

    def step(ev):
        if plan.recvs or plan.sends:
            with slab.library_stream():   # the halo moves in order with the library's kernels
                slab.exchange_planes(plan, planes)
        if ev:
            ev[0].record(stream)
        e1 = lib.vktHipResampleSlab(rv, sv, LINEAR, E, dz0, Sx, ls0)
        if ev:
            ev[1].record(stream)
        e2 = lib.vktHipArithmeticRange(0, dv, rv, bv, first, last, zero)
        if ev:
            ev[2].record(stream)
        if e1 or e2:
            raise RuntimeError(vkt.last_error())

    steps = max(3, args.steps // 10)
    elapsed, (res_ms, sum_ms) = ctx.timed(step, steps, 2, 2)
    ms = elapsed * 1e3 / steps
    vox = E * E * (dz1 - dz0)
    nbytes = 2 * Sx * Sx * (ls1 - ls0) + 2 * vox + 6 * vox
    out = {
        "workload": f"BASELINE config 4, strong scaling: Resample {Sx}^3->{E}^3 UInt16 Linear + SumRange {E}^3 "
                    f"UInt16, one fixed global volume Z-slab partitioned over {layout_n} GPU(s)"
                    + (" (rank 0's slab only, on 1 GPU)" if layout_n != world else ""),
        "scaling": "strong", "global_dst": [E, E, E], "dst_planes_per_rank": dz1 - dz0,
        "value": round(vox * world / (ms / 1e3) / 1e9, 3), "unit": "Gvoxels/s", "ms_per_step": round(ms, 4),
        "kernels_ms": {"Resample": round(res_ms, 4), "SumRange": round(sum_ms, 4)},
        "pipeline_frac": round(nbytes / ((res_ms + sum_ms) / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
        "halo_planes_per_rank": plan.halo_planes,
        "note": "speedup at N = config4_2048.value(N) / config4_2048.value(1); per-GPU work shrinks as N grows",
    }
    del S, R, B, D
    torch.cuda.synchronize()
    return out


def _lib_vec(x, y, z):
    from volkit_amd._lib import Vec3i_t
    return Vec3i_t(x, y, z)


if __name__ == "__main__":
    main()
