"""Benchmark: rrLU GFLOP/s at (m, n, r) = (8192, 8192, 256) on MI355X (BASELINE.json metric), plus
Pi-rows/s of the batch-evaluation kernel and the TCI2 sweep wall time of config 1.

A "step" is one rrlu(A; maxrank=r) on a synthetic U[0,1) Float64 matrix resident in HBM
(copy into the work buffer included, as rrlu = rrlu!(copy(A)), matrixlu.jl:462).
value = sum_{k=1..r} 2(m-k)(n-k) flops x ranks / max-over-ranks time.

  python bench.py [--gpus N --steps K --warmup W] [--m M --n N --r R] [--no-extras] [--no-cpu]
N > 1: launched by torch.distributed.run, one process per GPU; each rank factorises its own
matrix (weak scaling, no data-path collective; DESIGN.md "Multi-GPU").
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "tensorcrossinterpolation.jl_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec (6.29 measured copy)


def rrlu_flops(m, n, r):
    k = np.arange(1, r + 1, dtype=np.float64)
    return float(np.sum(2.0 * (m - k) * (n - k)))


def pass_bytes(m, n, r, nb, stride=1, shadow=True, sh_bytes=2, epochs=1, pass0_apart=False):
    """Algorithmic HBM bytes of the rrLU passes after pivots k = 0..r-1 with k % stride == 0
    (the ones bench times), each over the (m-k-1) x (n-k-1) trailing block, following the host
    schedule of tci_abi.cpp rrlu_device. Exact passes: a read-only pass reads 8 B/element, every
    nb-th pass also writes 8 B/element back. With the certified shadow search (DESIGN.md K2;
    sh_bytes = 1 for the 8-bit shadow, 2 for fp16, 4 for fp32) a read-only pass streams the shadow
    instead; with the narrow shadows (1 or 2 B) pass 0 is exact and writes the shadow of A (8 + s),
    and the two-level epoch ends every shadow epoch of nb pivots with a refresh (the shadow read and
    rewritten: s + s) and every epochs-th with a write-back (8 read + 8 + s written). The exact re-reads of candidate
    elements and the pending x / y vectors are data-dependent / small and not counted.
    Returns (read_only, write_back, refresh) as (bytes, launches); with pass0_apart the exact pass 0
    (narrow shadow: 8 + s B/element) is left out of read_only and returned fourth."""
    narrow = shadow and sh_bytes in (1, 2)  # the scaled narrow shadows (8-bit, fp16): two-level epoch
    if not (narrow and 2 <= nb <= 15):
        epochs = 1
    epochs = max(1, min(epochs, 32 // nb))
    nbx = nb * epochs
    ro_per, wb_per = (float(sh_bytes), 16.0 + sh_bytes) if shadow else (8.0, 16.0)
    ro_b = wb_b = rf_b = p0_b = 0.0
    ro_n = wb_n = rf_n = p0_n = 0
    te = ts = 0
    for k in range(r):
        PE, PS = k - te + 1, k - ts + 1
        last = k + 1 >= r
        flush = PE >= nbx and not last
        refresh = not flush and epochs > 1 and PS >= nb and not last
        elems = float(m - k - 1) * float(n - k - 1)
        if flush:
            te = ts = k + 1
        elif refresh:
            ts = k + 1
        if k % stride:
            continue
        if flush:
            wb_b += wb_per * elems
            wb_n += 1
        elif refresh:
            rf_b += 2.0 * sh_bytes * elems
            rf_n += 1
        elif narrow and k == 0 and pass0_apart:
            p0_b += (8.0 + sh_bytes) * elems
            p0_n += 1
        else:
            ro_b += (8.0 + sh_bytes if (narrow and k == 0) else ro_per) * elems
            ro_n += 1
    if pass0_apart:
        return (ro_b, ro_n), (wb_b, wb_n), (rf_b, rf_n), (p0_b, p0_n)
    return (ro_b, ro_n), (wb_b, wb_n), (rf_b, rf_n)


def len_sched(m, n, r, nb, epochs, shadow, sh_bytes):
    """(read-only, write-back, refresh) launch counts of one factorisation."""
    (_, a), (_, b), (_, c) = pass_bytes(m, n, r, nb, 1, shadow, sh_bytes, epochs)
    return a, b, c


_OUT_FD = 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--r", type=int, default=256)
    ap.add_argument("--no-extras", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-pivots", type=int, default=256)
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="diagnostic: no HIP events in the timed region (no roofline line)")
    ap.add_argument("--timing-stride", type=int, default=5,
                    help="time the rrLU pass of every s-th pivot with HIP events")
    ap.add_argument("--nb", type=int, default=int(os.environ.get("TCI_RRLU_NB", "10")),
                    help="shadow epoch of the rrLU: pending updates before the shadow is rewritten "
                         "(results are identical for every nb)")
    ap.add_argument("--epochs", type=int, default=int(os.environ.get("TCI_RRLU_EPOCHS", "0")),
                    help="shadow epochs per fp64 write-back (two-level epoch; identical results; "
                         "0 = the library's choice by shape)")
    ap.add_argument("--no-shadow", action="store_true",
                    help="exact fp64 read-only passes instead of the certified narrow-shadow search")
    args = ap.parse_args()
    # the result is ONE JSON line on stdout: native libraries' banners (RCCL prints its version
    # block to fd 1 when the sharded extras create a communicator) go to stderr instead
    global _OUT_FD
    _OUT_FD = os.dup(1)
    os.dup2(2, 1)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist  # control plane only: barrier + max of times
        dist.init_process_group(backend="gloo", init_method="env://")

    import tci_amd as T

    # one process per GPU (LOCAL_RANK); TCI_BENCH_DEVICE pins every rank to one device, only to
    # rehearse the multi-rank control flow on a one-GPU machine
    ctx = T.context(int(os.environ.get("TCI_BENCH_DEVICE", local_rank)))
    ctx.check(ctx.lib.tci_set_rrlu_flush(ctx.h, args.nb))
    ctx.check(ctx.lib.tci_set_rrlu_epochs(ctx.h, args.epochs))
    args.epochs = ctx.lib.tci_rrlu_epochs_for(ctx.h, args.m, args.n)  # the value the factorisation uses
    shadow = not args.no_shadow and os.environ.get("TCI_RRLU_SHADOW", "1") != "0"
    ctx.check(ctx.lib.tci_set_rrlu_shadow(ctx.h, int(shadow)))
    m, n, r = args.m, args.n, args.r
    A = T.DeviceMatrix(m, n, ctx=ctx)
    A.fill_uniform(seed=rank)
    W = T.DeviceMatrix(m, n, ctx=ctx)

    def step():
        # rrlu(A) = rrlu!(copy(A)) (matrixlu.jl:462): the copy into the work matrix W is fused into
        # the initial argmax pass (tci_rrlu_copy_d), A stays untouched
        return T.rrlu_inplace_device(W, maxrank=r, want_perms=False, src=A)

    for _ in range(args.warmup):
        step()

    def barrier():
        ctx.synchronize()
        if dist is not None:
            dist.barrier()

    # per-kernel device times: HIP events recorded on the context's stream around the passes of
    # every s-th pivot inside the timed region (s >= 5 prime to nb, so both pass kinds and every
    # pending depth are sampled; an event pair costs ~8 us of stream time, recording all 256 passes
    # would cost ~6 % of a step). --no-kernel-timing: diagnostic run without them.
    import math
    stride = args.timing_stride
    while math.gcd(stride, args.nb) != 1:  # sample every pending depth, both pass kinds
        stride += 1
    ctx.set_timing(not args.no_kernel_timing, stride=stride)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        np_, err, _, _, _ = step()
    barrier()
    dt = time.perf_counter() - t0
    assert np_ == min(r, m, n), np_
    wb_ms, wb_launches = ctx.kernel_stats(0)
    # read-only passes: per-pass launches (family 2, pass 0 excluded: family 43) and the persistent
    # shadow-epoch launches (41 first shadow epoch, 42 later ones; units = the passes they ran)
    ro1_ms, ro1_launches = ctx.kernel_stats(2)
    ep_ms, ep_launches, ep_passes = ctx.kernel_units(41)
    epx_ms, epx_launches, epx_passes = ctx.kernel_units(42)
    p0_ms, p0_launches = ctx.kernel_stats(43)
    ro_ms = ro1_ms + ep_ms + epx_ms
    ro_launches = ro1_launches + ep_passes + epx_passes  # passes, not launches
    rf_ms, rf_launches = ctx.kernel_stats(23)
    by_pending = {}  # read-only pass time by pending depth P (sub-families 3 + P)
    by_pending_ext = {}  # the same in the later shadow epochs of an exact epoch (EXT passes, 24 + P)
    for P in range(1, args.nb):
        pm, pn = ctx.kernel_stats(3 + P)
        if pn:
            by_pending[P] = round(pm / pn, 5)
        pm, pn = ctx.kernel_stats(24 + P)
        if pn:
            by_pending_ext[P] = round(pm / pn, 5)
    ctx.set_timing(False)
    # the benchmarked factorisation once more with permutations and pivot errors, for the parity
    # check against the CPU runs on the same matrix (rank 0 factorises the seed-0 matrix)
    npd, _, rpd, cpd, ped = T.rrlu_inplace_device(W, maxrank=r, want_perms=True, src=A)
    dev_res = (npd, rpd[:m].copy(), cpd[:n].copy(), ped.copy())
    if dist is not None:
        import torch
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    ms_per_step = dt / args.steps * 1e3
    flops = rrlu_flops(m, n, r)
    value = flops * world * args.steps / dt / 1e9  # GFLOP/s, whole job
    nb = args.nb
    sh_bytes = int(ctx.lib.tci_rrlu_shadow_bytes())
    # algorithmic bytes per pass from the whole schedule (every pass, stride 1): the sampled passes are
    # a uniform spread of it (every stride-th per-pass launch, every third persistent launch)
    (ro_b, ro_n), (wb_b, wb_n), (rf_b, rf_n), (p0_b, p0_n) = pass_bytes(m, n, r, nb, 1, shadow, sh_bytes,
                                                                       args.epochs, pass0_apart=True)
    # dominant kernel: the read-only pass when nb > 1, else the write-back pass
    if ro_n > 0 and ro_ms >= wb_ms:
        dom_key = "rrlu_read_only_pass"
        dom, dom_ms, dom_launches, dom_bytes, dom_n = (
            (("k_pass_mf<P> (read-only: " + ("8-bit" if sh_bytes == 1 else "fp16") + " shadow streamed, "
              "pending updates applied by f16-split MFMA with fp32 accumulation, certified abs2 argmax "
              "with exact fp64 re-reads of candidate elements)") if sh_bytes in (1, 2) else
             ("k_pass_sh<P> (read-only: fp32 shadow streamed, pending updates applied in fp32, "
              "certified abs2 argmax with exact fp64 re-reads of candidate chunks)")) if shadow else
            "k_pass2<P,false> (read-only: pending updates applied on the fly + abs2 argmax)",
            ro_ms, ro_launches, ro_b, ro_n)
    else:
        dom_key = "rrlu_write_back_pass"
        dom, dom_ms, dom_launches, dom_bytes, dom_n = ("k_pass2<P,true> (pending updates applied and "
                                                       "written back + abs2 argmax)", wb_ms, wb_launches,
                                                       wb_b, wb_n)
    # whole-step context: every pass's algorithmic bytes (stride 1), the initial argmax pass (8 B)
    # and the copy rrlu makes (16 B per element), over the measured step time
    step_bytes = ro_b + wb_b + rf_b + p0_b + 24.0 * m * n
    avg_launch_ms = dom_ms / max(dom_launches, 1)
    bytes_per_launch = dom_bytes / max(dom_n, 1)
    achieved = bytes_per_launch / (avg_launch_ms * 1e-3) / 1e9 if avg_launch_ms > 0 else 0.0
    other = {"write_back_pass": {"launches": wb_launches, "avg_ms": round(wb_ms / max(wb_launches, 1), 5),
                                 "GBps": round(wb_b / max(wb_n, 1) / (wb_ms / max(wb_launches, 1) * 1e-3) / 1e9, 1)
                                 if wb_launches else None},
             "read_only_pass": {"launches": ro_launches, "avg_ms": round(ro_ms / max(ro_launches, 1), 5),
                                "GBps": round(ro_b / max(ro_n, 1) / (ro_ms / max(ro_launches, 1) * 1e-3) / 1e9, 1)
                                if ro_launches else None,
                                "avg_ms_by_pending_depth": by_pending,
                                "avg_ms_by_pending_depth_ext": by_pending_ext},
             "read_only_pass_split": {
                 "per_pass_launches": {"passes": ro1_launches, "avg_ms": round(ro1_ms / max(ro1_launches, 1), 5)},
                 "persistent_first_epoch": {"launches": ep_launches, "passes": ep_passes,
                                            "avg_ms_per_pass": round(ep_ms / max(ep_passes, 1), 5)},
                 "persistent_ext": {"launches": epx_launches, "passes": epx_passes,
                                    "avg_ms_per_pass": round(epx_ms / max(epx_passes, 1), 5)}},
             "pass0": {"launches": p0_launches, "avg_ms": round(p0_ms / max(p0_launches, 1), 5),
                       "GBps": round(p0_b / max(p0_n, 1) / (p0_ms / max(p0_launches, 1) * 1e-3) / 1e9, 1)
                       if p0_launches else None,
                       "note": f"the exact pass after pivot 0 (reads A, writes the shadow: {8 + sh_bytes} B/element); "
                               "its own family, not in read_only_pass"},
             "refresh_pass": {"launches": rf_launches, "avg_ms": round(rf_ms / max(rf_launches, 1), 5),
                              "GBps": round(rf_b / max(rf_n, 1) / (rf_ms / max(rf_launches, 1) * 1e-3) / 1e9, 1)
                              if rf_launches else None},
             "step_share": {"write_back": round(wb_ms / max(wb_launches, 1) * len_sched(m, n, r, nb, args.epochs, shadow, sh_bytes)[1]
                                                / (ms_per_step), 4) if wb_launches else None}}
    out = {
        "metric": "rrLU GFLOP/s at (m,n,r)=(8192,8192,256)" if (m, n, r) == (8192, 8192, 256)
        else f"rrLU GFLOP/s at (m,n,r)=({m},{n},{r})",
        "value": round(value, 3),
        "unit": "GFLOP/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: U[0,1) splitmix64 matrix, seed = rank, resident in HBM",
        "config": {"workload": "rrlu(A; maxrank=r, reltol=1e-14, abstol=0, leftorthogonal=true)",
                   "m": m, "n": n, "r": r, "parallelism": f"replicas{world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "kernel": dom, "avg_launch_ms": round(avg_launch_ms, 5), "launches": dom_launches,
                     "launches_note": "read-only passes sampled by HIP events (every stride-th pass; pass 0 is "
                                      "its own family, passes.pass0); avg_launch_ms includes the event pair",
                     "algorithmic_bytes_per_launch": bytes_per_launch, "passes": other,
                     "deferred_depth_nb": nb, "epochs": args.epochs, "shadow_search": shadow, "shadow_bytes": sh_bytes,
                     "step_algorithmic_GBps": round(step_bytes / (ms_per_step * 1e-3) / 1e9, 1),
                     "step_note": "all passes' algorithmic bytes + initial pass + copy, per measured step; "
                                  "frac above is the dominant (read-only) kernel alone, most of whose "
                                  "~34 us is fixed per-pass cost (DESIGN.md K2)"},
    }
    # HBM bytes per launch from the committed PMC summary of this configuration (FETCH_SIZE x 2 +
    # WRITE_SIZE, scripts/profile_round.sh); null when none matches
    out["roofline"].update(pmc_traffic(dom_key, m, n, r, nb, args.epochs, shadow, sh_bytes))
    # the same fraction from the committed rocprofv3 kernel trace of this configuration: every
    # read-only pass's device time (no event overhead, pass 0 apart) over the schedule's pass count
    out["roofline"].update(trace_frac(m, n, r, nb, args.epochs, shadow, sh_bytes))
    # roofline calibration on the same buffers: 16-B stream read and stream copy, best grid
    import ctypes as C
    nel = A.ld * n
    best_r = best_c = 0.0
    for grid in (256, 512, 1024, 2048):
        ms_r, ms_c = C.c_double(), C.c_double()
        ctx.check(ctx.lib.tci_diag_stream_d(ctx.h, A.ptr, W.ptr, nel, 5, grid, C.byref(ms_r), C.byref(ms_c)))
        best_r = max(best_r, 8.0 * nel / (ms_r.value * 1e-3) / 1e9)
        best_c = max(best_c, 16.0 * nel / (ms_c.value * 1e-3) / 1e9)
    out["roofline"]["measured_stream_read_GBps"] = round(best_r, 1)
    out["roofline"]["measured_stream_copy_GBps"] = round(best_c, 1)
    A.free()
    W.free()

    if not args.no_extras:
        sh = sharded_pi(T, ctx, dist, world, rank)
        shq = sharded_pi(T, ctx, dist, world, rank, "quantics_osc")
        try:  # a failure of the multi-GPU extras must not cost the headline line
            shr = sharded_extras(T, ctx, dist, world, rank, dev_res if rank == 0 else None)
        except Exception as e:  # noqa: BLE001
            shr = {"sharded_extras_error": f"{type(e).__name__}: {e}"}
            sys.stderr.write(f"rank {rank}: sharded extras failed: {shr['sharded_extras_error']}\n")
        if rank == 0:
            out["extras"] = extras(T, ctx)
            out["extras"]["pi_lorentz_sharded"] = sh
            out["extras"]["pi_quantics_sharded"] = shq
            out["extras"].update(shr)
            # the paths that shard, as strong-scaling lines next to the replica
            # headline: fixed total work over N ranks, max-over-ranks time
            lines = {"n_gpus": world, "scaling": "strong"}
            for rec in shr.get("rrlu_sharded", []):
                lines[f"rrlu_sharded_{rec['m']}x{rec['n']}_r{rec['r']}"] = {
                    "value": rec["GFLOPs"], "unit": "GFLOP/s", "ms": rec["ms"],
                    "pivots_equal_unsharded": rec.get("pivots_equal_unsharded")}
            lines["pi_lorentz_sharded_8192x8192"] = {"value": sh["pi_rows_per_s"], "unit": "Pi-rows/s",
                                                     "ms": sh["ms_per_pi"]}
            lines["pi_quantics40_sharded_8192x8192"] = {"value": shq["pi_rows_per_s"], "unit": "Pi-rows/s",
                                                        "ms": shq["ms_per_pi"]}
            if "pi_sharded_with_gather" in shr:
                g = shr["pi_sharded_with_gather"]
                lines["pi_lorentz_gathered_8192x8192"] = {"value": g["pi_rows_per_s"], "unit": "Pi-rows/s",
                                                          "ms": g["ms"]}
            out["scaling_lines"] = lines
    parity_ok = True
    if rank == 0 and not args.no_cpu and world == 1:
        base, cpu_res = cpu_baseline(m, n, r, args.cpu_pivots)
        out["cpu_baseline"] = base
        out["parity"] = parity_vs_cpu(dev_res, cpu_res, r)
        parity_ok = out["parity"]["ok"]
    if rank == 0:
        sys.stdout.flush()
        os.write(_OUT_FD, (json.dumps(out) + "\n").encode())
    if dist is not None:
        dist.destroy_process_group()
    if not parity_ok:
        sys.stderr.write("bench: device rrLU differs from the CPU oracle on the benchmarked matrix\n")
        sys.exit(3)


PMC_SUMMARY = os.path.join(ROOT, "profiles", "r06_i1_pmc_summary.json")
TRACE_ROOFLINE = os.path.join(ROOT, "profiles", "r06_i1_trace_roofline.json")  # scripts/trace_roofline.py
PMC_CONFIG = {"m": 8192, "n": 8192, "r": 256, "nb": 10, "epochs": 2, "shadow": True, "sh_bytes": 1}  # the profiled command


def pmc_traffic(fam, m, n, r, nb, epochs, shadow, sh_bytes):
    """HBM bytes per launch of kernel family `fam` from the committed rocprofv3 PMC summary."""
    if ({"m": m, "n": n, "r": r, "nb": nb, "epochs": epochs, "shadow": shadow, "sh_bytes": sh_bytes} != PMC_CONFIG
            or not os.path.exists(PMC_SUMMARY)):
        return {"traffic": None}
    with open(PMC_SUMMARY) as fh:
        rec = json.load(fh).get(fam, {})
    if "hbm_bytes_per_launch" not in rec:
        return {"traffic": None}
    return {"traffic": rec["hbm_bytes_per_launch"],
            "traffic_source": os.path.relpath(PMC_SUMMARY, ROOT) + " (2 x FETCH_SIZE + WRITE_SIZE, "
                              f"{rec['dispatches_profiled']} dispatches)"}


def trace_frac(m, n, r, nb, epochs, shadow, sh_bytes):
    """roofline fraction of the read-only pass from the committed kernel trace summary (rocprof)."""
    if ({"m": m, "n": n, "r": r, "nb": nb, "epochs": epochs, "shadow": shadow, "sh_bytes": sh_bytes} != PMC_CONFIG
            or not os.path.exists(TRACE_ROOFLINE)):
        return {}
    with open(TRACE_ROOFLINE) as fh:
        rec = json.load(fh).get("read_only_pass")
    if not rec:
        return {}
    return {"frac_rocprof": rec["frac_of_8TBps"], "avg_us_per_pass_rocprof": rec["avg_us_per_pass"],
            "rocprof_source": os.path.relpath(TRACE_ROOFLINE, ROOT) + " (kernel trace of bench.py --steps 3 "
                              "--warmup 1 --no-extras --no-cpu: read-only passes' device time / passes)"}


def sharded_extras(T, ctx, dist, world, rank, full_res):
    """Multi-GPU data path on device buffers, every rank:
    * rrlu_sharded: one rrLU column-sharded over the ranks (tci_rrlu_sharded_d: per pivot one
      candidate record all-gathered over RCCL), on the metric matrix (8192^2, r = 256; its pivots
      must equal the unsharded device factorisation rank 0 ran above) and on a config-5-size
      matrix (32768^2 = 8 GiB, r = 1024) -- strong scaling: value = flops / max-over-ranks time;
    * pi_sharded_with_gather: the 8192^2 Lorentzian Pi evaluated by column blocks and all-gathered
      into a replicated device matrix on every rank (ncclAllGather in place)."""
    import ctypes as C

    from tci_amd.distributed import Comm, DeviceComm, column_blocks, rrlu_sharded

    host = Comm(device="cpu") if dist is not None else None
    if dist is not None:  # every rank reaches the communicator's creation, or none does (no hang)
        import torch
        t = torch.tensor([1.0], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
    dcomm = DeviceComm(ctx, host)

    def barrier():
        ctx.synchronize()
        if dist is not None:
            dist.barrier()

    def tmax(x):
        if dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    res = {}
    recs = []
    for (m, n, r, reps) in ((8192, 8192, 256, 3), (32768, 32768, 1024, 2)):
        j0, j1 = column_blocks(n, world)[rank]
        nloc = j1 - j0
        A0 = T.DeviceMatrix(m, nloc + 1, ctx=ctx)
        ctx.check(ctx.lib.tci_fill_uniform_block_d(ctx.h, A0.ptr, m, nloc, A0.ld, 0, m * j0))
        W = T.DeviceMatrix(m, nloc + 1, ctx=ctx)
        W.copy_from(A0)
        # one rank has nothing to exchange: the sharded driver then commits in the pass tail
        xc = dcomm if world > 1 else None
        out = rrlu_sharded(W, m, n, j0, nloc, comm=xc, maxrank=r)  # warm-up (+ pivots for parity)
        times = []
        for _ in range(reps):
            W.copy_from(A0)
            barrier()
            t0 = time.perf_counter()
            rrlu_sharded(W, m, n, j0, nloc, comm=xc, maxrank=r)
            barrier()
            times.append(time.perf_counter() - t0)
        dt = tmax(min(times))
        used = ctx.lib.tci_last_shard_exchange(ctx.h)
        rec = {"m": m, "n": n, "r": r, "ranks": world, "npivot": out[0], "ms": round(dt * 1e3, 3),
               "GFLOPs": round(rrlu_flops(m, n, out[0]) / dt / 1e9, 1),
               "exchange": {0: "none (one rank: the pass tail commits, as unsharded)",
                            1: "two collectives: all-gather of 32-B candidates, then the winning column from "
                               "its owner by an element-wise uint64 max (DESIGN.md 7)",
                            2: "fused: ONE all-gather per pivot of every rank's 32-B candidate and its own "
                               "candidate column (DESIGN.md 7)"}.get(used, used),
               "epochs": ctx.lib.tci_rrlu_epochs_for(ctx.h, m, n),
               "exchange_bytes_per_pivot": {"fused_allgather_recv": 8 * (m + 36) * world,
                                            "two_collective": {"allgather_candidates": 32 * world,
                                                               "allreduce_column": 8 * (m + 32)}}}
        if world == 1 and m == 8192:
            # the per-pivot exchange's own cost, measured through a one-rank RCCL communicator (the
            # collectives run, moving nothing across links): ms per factorisation in both forms
            xo = {}
            for xm in (1, 2):
                ctx.check(ctx.lib.tci_set_shard_exchange(ctx.h, xm))
                ts = []
                for _ in range(reps):
                    W.copy_from(A0)
                    barrier()
                    t0 = time.perf_counter()
                    o2 = rrlu_sharded(W, m, n, j0, nloc, comm=dcomm, maxrank=r)
                    barrier()
                    ts.append(time.perf_counter() - t0)
                xo[{1: "two_collective", 2: "fused"}[xm]] = {
                    "ms": round(min(ts) * 1e3, 3), "pivots_equal": bool(o2[0] == out[0] and
                                                                      np.array_equal(o2[2], out[2]) and
                                                                      np.array_equal(o2[3], out[3]))}
            ctx.check(ctx.lib.tci_set_shard_exchange(ctx.h, 0))
            for v in xo.values():
                v["us_per_pivot_over_unsharded"] = round((v["ms"] - rec["ms"]) * 1e3 / max(out[0], 1), 2)
            rec["one_rank_rccl_exchange"] = xo
        A0.free()
        W.free()
        if rank == 0:
            # the same matrix factorised unsharded on this GPU: pivots, permutations and pivot
            # errors must be bitwise equal (at 8192^2 the headline step ran it already)
            if (m, n, r) == (8192, 8192, 256) and full_res is not None:
                npd, rpd, cpd, ped = full_res
            else:
                Af = T.DeviceMatrix(m, n, ctx=ctx)
                Af.fill_uniform(seed=0)
                npd, _, rpd, cpd, ped = T.rrlu_inplace_device(Af, maxrank=r, want_perms=True)
                rpd, cpd = rpd[:m].copy(), cpd[:n].copy()
                Af.free()
            rec["pivots_equal_unsharded"] = bool(out[0] == npd and np.array_equal(out[2], rpd)
                                                 and np.array_equal(out[3], cpd) and np.array_equal(out[4], ped))
        recs.append(rec)
    res["rrlu_sharded"] = recs
    # Pi assembly + device all-gather of the column blocks (n divisible by world: equal blocks)
    m = n = 8192
    rng = np.random.default_rng(1)
    I = rng.integers(1, 11, (m, 10)).astype(np.int32)
    J = rng.integers(1, 11, (n, 10)).astype(np.int32)
    f = T.lorentz([10] * 20, ctx=ctx)
    w = n // world
    full = T.DeviceMatrix(m, w * world, ctx=ctx)
    blk_ptr = C.c_void_p(full.ptr.value + 8 * full.ld * w * rank)
    Jl = np.ascontiguousarray(J[rank * w:(rank + 1) * w])
    mx = C.c_double()

    def run():
        ctx.check(ctx.lib.tci_batcheval_d(ctx.h, f.h, T._lib.ptr(I), m, 10, T._lib.ptr(Jl), w, 10, 0, blk_ptr,
                                          full.ld, C.byref(mx)))
        dcomm.allgather(blk_ptr, full.ptr, 8 * full.ld * w)

    run()
    times = []
    for _ in range(5):
        barrier()
        t0 = time.perf_counter()
        run()
        barrier()
        times.append(time.perf_counter() - t0)
    dt = tmax(min(times))
    res["pi_sharded_with_gather"] = {"m": m, "n": w * world, "L": 20, "ranks": world,
                                     "ms": round(dt * 1e3, 4), "pi_rows_per_s": round(m / dt, 1),
                                     "gathered_GB": round(8.0 * full.ld * w * world / 1e9, 3),
                                     "note": "column blocks evaluated per rank, ncclAllGather into a replicated "
                                             "device Pi (no host staging)"}
    full.free()
    dcomm.close()
    return res


def sharded_pi(T, ctx, dist, world, rank, kind="lorentz"):
    """Pi assembly of one 8192 x 8192 Pi split by column blocks over the ranks: each
    rank evaluates its block on its own GPU, maxsample is all-reduced. Strong scaling: Pi-rows/s =
    m / (max over ranks of the block time). kind "lorentz": L = 20 legs of d = 10 (config 1's
    integrand, HBM-write-bound); "quantics_osc": config 4's integrand, L = 40 legs of d = 2
    (fp64-VALU-bound: the Pi that shards; config 4's own TCI2 Pi are <= 30^2 and run as replicas)."""
    import ctypes as C

    import torch

    m = n = 8192
    rng = np.random.default_rng(1)
    if kind == "lorentz":
        I = rng.integers(1, 11, (m, 10)).astype(np.int32)
        J = rng.integers(1, 11, (n, 10)).astype(np.int32)
        f = T.lorentz([10] * 20, ctx=ctx)
    else:
        rng.integers(1, 11, (m + n, 10))  # the draws of the Lorentzian inputs, as in extras()
        I = rng.integers(1, 3, (m, 20)).astype(np.int32)
        J = rng.integers(1, 3, (n, 20)).astype(np.int32)
        f = T.GPUBatchEvaluator(5, T.batcheval.QOSC_PARAMS, [2] * 40, ctx=ctx)
    nl, nr = I.shape[1], J.shape[1]
    j0, j1 = T.column_blocks(n, world)[rank]
    Jb = np.ascontiguousarray(J[j0:j1])
    dm = T.DeviceMatrix(m, max(j1 - j0, 1), ctx=ctx)
    mx = C.c_double()

    def run():  # tci_batcheval_d: host index tables uploaded by every call, max|Pi| synchronised
        if j1 > j0:
            ctx.check(ctx.lib.tci_batcheval_d(ctx.h, f.h, T._lib.ptr(I), m, nl, T._lib.ptr(Jb), j1 - j0, nr,
                                              0, dm.ptr, dm.ld, C.byref(mx)))
        else:
            mx.value = 0.0

    run()
    reps = 5
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    ctx.synchronize()
    dt_up = (time.perf_counter() - t0) / reps
    # device-resident index tables (a sweep's sets live on the device: uploaded once per bond, here
    # once) and tci_batcheval_dd: no host synchronisation per Pi; max|Pi| folded on the device into a
    # running maximum, reduced over the ranks once (updatemaxsample! per iteration)
    dI = T.DeviceMatrix(max(I.size // 2 + 1, 1), 1, ctx=ctx)  # (int32 tables in float64 buffers)
    dJ = T.DeviceMatrix(max(Jb.size // 2 + 1, 1), 1, ctx=ctx)
    dmax = T.DeviceMatrix(2, 1, ctx=ctx)
    ctx.check(ctx.lib.tci_memcpy_h2d(ctx.h, dI.ptr, T._lib.ptr(I), I.nbytes))
    if Jb.size:
        ctx.check(ctx.lib.tci_memcpy_h2d(ctx.h, dJ.ptr, T._lib.ptr(Jb), Jb.nbytes))
    zero = np.zeros(2, np.uint64)
    ctx.check(ctx.lib.tci_memcpy_h2d(ctx.h, dmax.ptr, T._lib.ptr(zero), 8))

    def run_dev():
        if j1 > j0:
            ctx.check(ctx.lib.tci_batcheval_dd(ctx.h, f.h, dI.ptr, m, nl, dJ.ptr, j1 - j0, nr, 0, dm.ptr, dm.ld,
                                               dmax.ptr))

    run_dev()
    reps_dev = 20
    ctx.synchronize()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps_dev):
        run_dev()
    bits = np.zeros(1, np.uint64)
    ctx.check(ctx.lib.tci_memcpy_d2h(ctx.h, T._lib.ptr(bits), dmax.ptr, 8))  # (synchronises the stream)
    gmx_dev = float(bits.view(np.float64)[0])
    if dist is not None:  # the once-per-iteration reduction of the running maximum over the ranks
        import torch
        tt = torch.tensor([gmx_dev], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        gmx_dev = float(tt.item())
    dt = (time.perf_counter() - t0) / reps_dev
    for x in (dI, dJ, dmax):
        x.free()
    gmx = mx.value
    if dist is not None:
        import torch
        t = torch.tensor([dt, dt_up, gmx], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, dt_up, gmx = float(t[0]), float(t[1]), float(t[2])
    dm.free()
    return {"m": m, "n": n, "L": nl + nr, "ranks": world, "pi_rows_per_s": round(m / dt, 1),
            "ms_per_pi": round(dt * 1e3, 4), "maxsample": gmx, "maxsample_device_path": gmx_dev,
            "ms_per_pi_host_tables": round(dt_up * 1e3, 4),
            "pi_rows_per_s_host_tables": round(m / dt_up, 1),
            "note": "column blocks per rank, no gather (strong scaling); ms_per_pi: device-resident index "
                    "tables, tci_batcheval_dd back to back (20 Pi), max|Pi| kept on the device and reduced "
                    "over the ranks once at the end; *_host_tables: tci_batcheval_d (index tables uploaded "
                    "and max|Pi| synchronised by every call)"}


def extras(T, ctx):
    """Pi-rows/s of the batch evaluation and the TCI2 wall time of BASELINE config 1."""
    res = {}
    # Pi assembly: 8192 x 8192, L = 20 legs, nl = nr = 10, d = 10, Lorentzian
    rng = np.random.default_rng(1)
    m = n = 8192
    I = rng.integers(1, 11, (m, 10)).astype(np.int32)
    J = rng.integers(1, 11, (n, 10)).astype(np.int32)
    for name, f in (("lorentz", T.lorentz([10] * 20, ctx=ctx)),
                    ("quantics_osc", T.GPUBatchEvaluator(5, T.batcheval.QOSC_PARAMS, [2] * 40, ctx=ctx))):
        if name == "quantics_osc":
            Ib = rng.integers(1, 3, (m, 20)).astype(np.int32)
            Jb = rng.integers(1, 3, (n, 20)).astype(np.int32)
        else:
            Ib, Jb = I, J
        dm = T.DeviceMatrix(m, n, ctx=ctx)
        import ctypes as C
        mx = C.c_double()
        for _ in range(2):
            ctx.check(ctx.lib.tci_batcheval_d(ctx.h, f.h, T._lib.ptr(Ib), m, Ib.shape[1], T._lib.ptr(Jb), n,
                                              Jb.shape[1], 0, dm.ptr, dm.ld, C.byref(mx)))
        ctx.set_timing(True)
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            ctx.check(ctx.lib.tci_batcheval_d(ctx.h, f.h, T._lib.ptr(Ib), m, Ib.shape[1], T._lib.ptr(Jb), n,
                                              Jb.shape[1], 0, dm.ptr, dm.ld, C.byref(mx)))
        wall = (time.perf_counter() - t0) / reps
        kms, kn = ctx.kernel_stats(1)
        ctx.set_timing(False)
        dev_s = kms / max(kn, 1) * 1e-3
        res[f"pi_{name}"] = {"m": m, "n": n, "L": Ib.shape[1] + Jb.shape[1],
                             "pi_rows_per_s_device": round(m / dev_s, 1),
                             "pi_rows_per_s_call": round(m / wall, 1),
                             "write_GBps_device": round(8.0 * m * n / dev_s / 1e9, 1)}
        dm.free()
    # roofline fractions of the Pi assembly: the Lorentzian is HBM-write-bound (8 B per element);
    # the quantics integrand is fp64 VALU-bound (exp/sin/pow per element), rated by its fp64 VALU
    # instruction count per element from rocprofv3 (profiles/, scripts/pmc_valu.sh) when present
    lz = res["pi_lorentz"]
    lz["roofline"] = {"bound": "hbm-write", "achieved": lz["write_GBps_device"], "peak": HBM_PEAK_GBS,
                      "unit": "GB/s", "frac": round(lz["write_GBps_device"] / HBM_PEAK_GBS, 4)}
    res["pi_quantics_osc"]["roofline"] = qosc_roofline(res["pi_quantics_osc"])
    # TCI2 sweep wall times of the BASELINE configs (scripts/tci2_configs.py), with the 1-core
    # oracle's wall time next to them where the oracle finishes in seconds (C1, C3, C4)
    res["tci2_configs"] = tci2_configs()
    # separable (CP-rank-K) Pi assembly of config 5 as an fp64 MFMA GEMM (K3): 8192^2, K = 1024,
    # 12 legs of d = 32, against the spec and the measured fp64 MFMA peak (two waves per SIMD)
    import ctypes as C
    peak, ghz = C.c_double(), C.c_double()
    ctx.check(ctx.lib.tci_diag_mfma_f64_ex(ctx.h, 2, C.byref(peak), C.byref(ghz)))
    K, L, d = 1024, 12, 32
    g = 0.5 + np.random.default_rng(2).random((K, L, d))
    fcp = T.cp_function(g, ctx=ctx)
    Ic = rng.integers(1, d + 1, (m, 6)).astype(np.int32)
    Jc = rng.integers(1, d + 1, (n, 6)).astype(np.int32)
    dm = T.DeviceMatrix(m, n, ctx=ctx)
    mx = C.c_double()
    for _ in range(2):
        ctx.check(ctx.lib.tci_batcheval_d(ctx.h, fcp.h, T._lib.ptr(Ic), m, 6, T._lib.ptr(Jc), n, 6, 0, dm.ptr,
                                          dm.ld, C.byref(mx)))
    ctx.set_timing(True)
    for _ in range(3):
        ctx.check(ctx.lib.tci_batcheval_d(ctx.h, fcp.h, T._lib.ptr(Ic), m, 6, T._lib.ptr(Jc), n, 6, 0, dm.ptr,
                                          dm.ld, C.byref(mx)))
    kms, kn = ctx.kernel_stats(1)
    ctx.set_timing(False)
    dm.free()
    tfl = 2.0 * m * n * K / (kms / kn * 1e-3) / 1e12
    res["pi_cp_gemm"] = {"m": m, "n": n, "K": K, "L": L, "ms_device": round(kms / kn, 3), "TFLOPs": round(tfl, 2),
                         "frac_of_spec": round(tfl / MFMA_F64_SPEC_TFLOPS, 4),
                         "mfma_f64_peak_measured_TFLOPs": round(peak.value, 2),
                         "frac_of_measured_peak": round(tfl / peak.value, 3)}
    # Contraction of two MPOs (contraction.jl, TCI_F_MPO): 20 sites, bonds 32 (K = 1024 environment
    # terms at the cut), d = 2 x 2 x 2; Pi 8192 x 8192 from 10 row legs and 10 column legs:
    # environments (k_mpo_env) + the MFMA GEMM
    N, chi = 20, 32
    bonds = [1] + [chi] * (N - 1) + [1]
    mrng = np.random.default_rng(5)
    Am = [mrng.standard_normal((bonds[t], 2, 2, bonds[t + 1])) / chi ** 0.5 for t in range(N)]
    Bm = [mrng.standard_normal((bonds[t], 2, 2, bonds[t + 1])) / chi ** 0.5 for t in range(N)]
    fm = T.Contraction(Am, Bm, ctx=ctx)
    Im = rng.integers(1, 5, (m, 10)).astype(np.int32)
    Jm = rng.integers(1, 5, (n, 10)).astype(np.int32)
    dm = T.DeviceMatrix(m, n, ctx=ctx)
    for _ in range(2):
        ctx.check(ctx.lib.tci_batcheval_d(ctx.h, fm.h, T._lib.ptr(Im), m, 10, T._lib.ptr(Jm), n, 10, 0, dm.ptr,
                                          dm.ld, C.byref(mx)))
    ctx.set_timing(True)
    for _ in range(3):
        ctx.check(ctx.lib.tci_batcheval_d(ctx.h, fm.h, T._lib.ptr(Im), m, 10, T._lib.ptr(Jm), n, 10, 0, dm.ptr,
                                          dm.ld, C.byref(mx)))
    kms, kn = ctx.kernel_stats(1)
    ctx.set_timing(False)
    dm.free()
    env_flops = 2 * 2.0 * (m + n) * 10 * 2 * chi ** 3  # two contractions per site and environment
    res["pi_mpo_contraction"] = {"m": m, "n": n, "sites": N, "bond": chi, "K": chi * chi,
                                 "ms_device": round(kms / kn, 3),
                                 "pi_rows_per_s_device": round(m / (kms / kn * 1e-3), 1),
                                 "TFLOPs_env_plus_gemm": round((env_flops + 2.0 * m * n * chi * chi)
                                                               / (kms / kn * 1e-3) / 1e12, 2)}
    # ComplexF64 rrLU (K8): 8192^2 r = 256, device-resident, U[0,1) re and im
    mc = nc = 8192
    rc = 256
    Ac = T.DeviceMatrix(2 * mc, nc, ctx=ctx)  # interleaved (re, im): complex ld = Ac.ld / 2
    Ac.fill_uniform(seed=0)
    Wc = T.DeviceMatrix(2 * mc, nc, ctx=ctx)
    npv, errc = C.c_int64(), C.c_double()
    walls = []
    for rep in range(3):
        Wc.copy_from(Ac)
        ctx.synchronize()
        t0 = time.perf_counter()
        ctx.check(ctx.lib.tci_rrlu_c128_inplace_d(ctx.h, Wc.ptr, mc, nc, Wc.ld // 2, rc, 1e-14, 0.0, 1,
                                                  None, None, C.byref(npv), C.byref(errc), None))
        walls.append(time.perf_counter() - t0)
    Ac.free()
    Wc.free()
    kk = np.arange(1, npv.value + 1, dtype=np.float64)
    elc = float(((mc - kk) * (nc - kk)).sum())
    tc = min(walls[1:])
    res["rrlu_c128"] = {"m": mc, "n": nc, "r": int(npv.value), "ms": round(tc * 1e3, 2),
                        "complex_GFLOPs": round(8 * elc / tc / 1e9, 1),
                        "search": "certified fp16 shadow (Re/Im planes) + f16-split MFMA, nb = 11 (DESIGN.md K8)"}
    # other rrLU configurations of SURVEY 8(d): config 2 (4096^2), right-orthogonal pivots, and a
    # 16384^2 matrix (2 GiB) for the scale curve
    res["rrlu_configs"] = []
    for (m2, n2, r2, lo) in ((4096, 4096, 256, True), (8192, 8192, 256, False), (16384, 16384, 256, True)):
        A = T.DeviceMatrix(m2, n2, ctx=ctx)
        A.fill_uniform(seed=0)
        W = T.DeviceMatrix(m2, n2, ctx=ctx)
        T.rrlu_inplace_device(W, maxrank=r2, leftorthogonal=lo, want_perms=False, src=A)
        ctx.synchronize()
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            T.rrlu_inplace_device(W, maxrank=r2, leftorthogonal=lo, want_perms=False, src=A)
        ctx.synchronize()
        dt = (time.perf_counter() - t0) / reps
        res["rrlu_configs"].append({"m": m2, "n": n2, "r": r2, "leftorthogonal": lo, "ms": round(dt * 1e3, 3),
                                    "GFLOPs": round(rrlu_flops(m2, n2, r2) / dt / 1e9, 1)})
        A.free()
        W.free()
    res["dense_mfma"] = dense_extras(T, ctx)
    return res


MFMA_F64_SPEC_TFLOPS = 78.6  # MI355X fp64 matrix peak (spec; 2.4 GHz x 256 CU x 4 SIMD x 32 flop/clk)


def dense_extras(T, ctx, only_k3=False):
    """fp64 MFMA dense kernels (tci_dense.hip), device time from HIP events on
    the context stream (timing families 20-22):
    * the fp64 MFMA probe at 1 / 2 / 4 waves per SIMD, with the shader clock it held;
    * K3, the blocked Schur-complement update C -= W V on 8192^2 at nb in {32, 64, 128, 256}
      (BASELINE.md:46, SURVEY 7 hard part 1): TFLOP/s as a fraction of the 78.6 TF spec, and the
      HBM-algorithmic rate (C read + written, W and V read once) as a fraction of 8 TB/s;
    * K5, setsitetensor!'s solve at the C5 shape (r = 1024, R = 32768) and the scaled one (256, 8192);
    * K4, the MatrixLUCI factor kernels of an 8192^2 matrix at np = 1024, both orthogonalities."""
    import ctypes as C
    out = {"spec_TFLOPs": MFMA_F64_SPEC_TFLOPS}
    probe = {}
    for w in (1, 2, 4):
        tf, ghz = C.c_double(), C.c_double()
        ctx.check(ctx.lib.tci_diag_mfma_f64_ex(ctx.h, w, C.byref(tf), C.byref(ghz)))
        probe[f"waves_per_simd_{w}"] = {"TFLOPs": round(tf.value, 2), "clock_GHz": round(ghz.value, 3)}
    out["probe"] = probe
    best = max(v["TFLOPs"] for v in probe.values())
    m = n = 8192
    Cm = T.DeviceMatrix(m, n, ctx=ctx)
    Cm.fill_uniform(seed=3)
    k3 = []
    for nb in (32, 64, 128, 256):
        W = T.DeviceMatrix(m, nb, ctx=ctx)
        W.fill_uniform(seed=4)
        V = T.DeviceMatrix(nb, n, ctx=ctx)
        V.fill_uniform(seed=5)
        T.schur_update_device(Cm, W, V)
        ctx.set_timing(True)
        for _ in range(5):
            T.schur_update_device(Cm, W, V)
        kms, kn = ctx.kernel_stats(22)
        ctx.set_timing(False)
        sec = kms / kn * 1e-3
        tfl = 2.0 * m * n * nb / sec / 1e12
        gbs = (16.0 * m * n + 8.0 * (m + n) * nb) / sec / 1e9
        k3.append({"m": m, "n": n, "nb": nb, "ms": round(sec * 1e3, 4), "TFLOPs": round(tfl, 2),
                   "frac_of_spec": round(tfl / MFMA_F64_SPEC_TFLOPS, 4),
                   "frac_of_probe": round(tfl / best, 4), "algorithmic_GBps": round(gbs, 1),
                   "hbm_frac": round(gbs / HBM_PEAK_GBS, 4)})
        W.free()
        V.free()
    Cm.free()
    out["schur_update_k3"] = k3
    if only_k3:
        return out
    solves = []
    for r, R in ((256, 8192), (1024, 32768), (1024, 64)):
        P0 = T.DeviceMatrix(r, r, ctx=ctx, ld=r)
        P0.fill_uniform(seed=6)
        P = T.DeviceMatrix(r, r, ctx=ctx, ld=r)
        Pi1 = T.DeviceMatrix(R, r, ctx=ctx, ld=R)
        Pi1.fill_uniform(seed=7)
        Tm = T.DeviceMatrix(R, r, ctx=ctx, ld=R)
        rec = {"r": r, "R": R}
        # mfma: the default (31: one cooperative getrf launch for r <= 1024); mfma_r5: round 5's
        # form (15: four launches per panel); mfma_lds_panel / round1_scalar / mfma_getrs_only:
        # older A/B points
        for tag, mask in (("mfma", 31), ("mfma_r5", 15), ("mfma_lds_panel", 7), ("round1_scalar", 0),
                          ("mfma_getrs_only", 4)):
            ctx.check(ctx.lib.tci_set_dense_mfma(ctx.h, mask))
            P.copy_from(P0)
            T.sitetensor_solve_device(P, Pi1, Tm)
            ctx.set_timing(True)
            for _ in range(3):
                P.copy_from(P0)
                T.sitetensor_solve_device(P, Pi1, Tm)
            kms, kn = ctx.kernel_stats(20)
            ctx.set_timing(False)
            sec = kms / kn * 1e-3
            fl = 2.0 / 3.0 * r ** 3 + 2.0 * R * r * r
            rec[tag] = {"ms": round(sec * 1e3, 3), "TFLOPs": round(fl / sec / 1e12, 2),
                        "frac_of_spec": round(fl / sec / 1e12 / MFMA_F64_SPEC_TFLOPS, 4)}
        ctx.check(ctx.lib.tci_set_dense_mfma(ctx.h, 31))
        solves.append(rec)
        for x in (P0, P, Pi1, Tm):
            x.free()
    out["sitetensor_solve_k5"] = solves
    lucis = []
    A = T.DeviceMatrix(8192, 8192, ctx=ctx)
    A.fill_uniform(seed=8)
    Ah = A.to_host()
    A.free()
    for lo in (True, False):
        npv = 1024
        # GEMM with K = np over the full np x n (or m x np) block + TRSM m np^2 (or n np^2)
        fl = 2.0 * npv * npv * 8192 + 1.0 * (8192 - npv) * npv * npv
        rec = {"m": 8192, "n": 8192, "np": npv, "leftorthogonal": lo}
        for tag, mask in (("mfma", 31), ("round1_scalar", 0)):
            ctx.check(ctx.lib.tci_set_dense_mfma(ctx.h, mask))
            ctx.set_timing(True)
            T.MatrixLUCI(Ah, maxrank=npv, leftorthogonal=lo, ctx=ctx).left()
            kms, kn = ctx.kernel_stats(21)
            ctx.set_timing(False)
            rec[tag] = {"ms": round(kms / max(kn, 1), 3), "TFLOPs": round(fl / (kms / max(kn, 1) * 1e-3) / 1e12, 2)}
        ctx.check(ctx.lib.tci_set_dense_mfma(ctx.h, 31))
        lucis.append(rec)
    out["luci_factors_k4"] = lucis
    return out


def _host_info():
    try:
        share = len(os.sched_getaffinity(0))
    except Exception:
        share = None
    info = {"nproc_machine": os.cpu_count(), "cpus_allowed": share,
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"),
            "note": "nproc_machine counts the whole host; the lease's share is OMP_NUM_THREADS "
                    "(the box sets it to 16) -- cores below is the thread count actually used"}
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    info["cpu_model"] = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in ("Socket(s)", "Core(s) per socket", "Thread(s) per core", "NUMA node(s)"):
                info["lscpu_" + k.strip().lower().replace("(s)", "s").replace(" ", "_")] = v.strip()
    except Exception:
        pass
    return info


def _native_omp_lib():
    """oracle/cpu_rrlu_omp.c built with -march=native for THIS host (a second, no GPU involved);
    falls back to the portable x86-64-v3 copy oracle/Makefile builds."""
    import subprocess
    import tempfile
    src = os.path.join(ROOT, "oracle", "cpu_rrlu_omp.c")
    out = os.path.join(tempfile.mkdtemp(prefix="tci_cpu_"), "libcpu_rrlu_omp_native.so")
    try:
        subprocess.run(["gcc", "-O3", "-march=native", "-ffp-contract=off", "-fno-fast-math", "-fPIC",
                        "-std=c11", "-fopenmp", "-shared", "-o", out, src, "-lm"], check=True,
                       capture_output=True, timeout=60)
        return out, "gcc -O3 -march=native -fopenmp -ffp-contract=off (built on this host)"
    except Exception:
        return None, "gcc -O3 -march=x86-64-v3 -fopenmp -ffp-contract=off (portable oracle/Makefile build)"


VALU_SUMMARY = os.path.join(ROOT, "profiles", "r02_qosc_valu.json")
FP64_VECTOR_PEAK_TF = 78.6  # MI355X spec fp64 vector (and matrix) rate


def qosc_roofline(rec):
    """fp64 VALU roofline of the quantics assembly: flops/element from the committed PMC count of
    fp64 VALU instructions (64 lanes; FMA = 2 flops), x elements / device time."""
    if not os.path.exists(VALU_SUMMARY):
        return {"bound": "valu-fp64", "achieved": None, "peak": FP64_VECTOR_PEAK_TF, "unit": "TFLOP/s",
                "frac": None, "note": "no PMC summary committed"}
    with open(VALU_SUMMARY) as fh:
        v = json.load(fh)
    fpe = v["fp64_flops_per_element"]
    dev_s = rec["m"] / rec["pi_rows_per_s_device"]  # device time of one m x n assembly
    tf = fpe * rec["m"] * rec["n"] / dev_s / 1e12
    return {"bound": "valu-fp64", "achieved": round(tf, 2), "peak": FP64_VECTOR_PEAK_TF, "unit": "TFLOP/s",
            "frac": round(tf / FP64_VECTOR_PEAK_TF, 4), "fp64_flops_per_element": fpe,
            "source": os.path.relpath(VALU_SUMMARY, ROOT)}


def tci2_configs():
    os.environ.setdefault("TCI2_CONFIGS_ORACLE", "1")
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import tci2_configs as TC
    TC.ORACLE = os.environ["TCI2_CONFIGS_ORACLE"] == "1"
    cs = TC.configs()
    out = {}
    for name in ("C1_lorentz8d_parity", "C1_lorentz8d_default", "C3_gauss20d", "C3_gaussmix20d", "C4_qosc40",
                 "C5_cp12d_K256", "C5_cp12d_K1024"):
        rec = cs[name]()
        rec.pop("linkdims", None)
        out[name] = rec
    return out


def cpu_baseline(m, n, r, pivots):
    """CPU baselines on the same seed-0 (m, n) matrix (SURVEY 8(d) "CPU baseline"):
      (ii) all host cores -- oracle/cpu_rrlu_omp.c (OpenMP over columns, update fused with the next
           argmax, bitwise the oracle's results), every pivot: the reported `value`;
      (i)  one core -- the loop-for-loop restatement oracle/tci_oracle.c, first `pivots` pivots.
    Returns (baseline dict, results of both for the parity check against the device)."""
    import oracle_lib as O
    a = O.fill_uniform(m * n, seed=0)
    path, build = _native_omp_lib()
    L = O.omp_lib(path)
    threads = int(L.cpu_rrlu_threads())
    w = a.copy()
    t0 = time.perf_counter()
    npo, erro, rpo, cpo = O.rrlu_inplace_omp(w, m, n, r, -1, path=path)
    dto = time.perf_counter() - t0
    pe_omp = np.concatenate([np.abs(w[np.arange(npo) * (m + 1)]), [erro]])
    del w
    t0 = time.perf_counter()
    npv, err, rp, cp = O.rrlu_inplace_sample(a, m, n, r, pivots)
    dt = time.perf_counter() - t0
    pe_one = np.concatenate([np.abs(a[np.arange(npv) * (m + 1)]), [err]])
    del a
    fl = rrlu_flops(m, n, npv)
    # Pi half of the metric: the oracle's _batchevaluate_dispatch restatement (one thread, the
    # reference's loop) on the bench's 8192^2 L = 20 Lorentzian tables, bounded to 1024 rows
    rng = np.random.default_rng(1)
    I = rng.integers(1, 11, (8192, 10)).astype(np.int32)
    J = rng.integers(1, 11, (8192, 10)).astype(np.int32)
    rows = 1024
    t0 = time.perf_counter()
    O.batcheval(1, [1.0], [10] * 20, I[:rows], J, 0)
    dtp = time.perf_counter() - t0
    pi_base = {"value": round(rows / dtp, 1), "unit": "Pi-rows/s", "cores": 1, "kind": "port",
               "sample": f"first {rows} of 8192 rows x 8192 columns of the L = 20 Lorentzian Pi (bench extras "
                         f"pi_lorentz inputs), oracle batch evaluation (batcheval.jl:131-175 loop), {dtp:.2f} s"}
    base = {"value": round(rrlu_flops(m, n, npo) / dto / 1e9, 4), "unit": "GFLOP/s", "cores": threads,
            "kind": "port",
            "sample": f"all {npo} of {r} pivots of rrlu on the same {m}x{n} seed-0 matrix, "
                      f"{dto:.2f} s: oracle/cpu_rrlu_omp.c (OpenMP over {threads} threads = the lease's CPU "
                      f"share, rank-1 update fused with the next argmax, bitwise the oracle's results)",
            "build": build,
            "host": _host_info(),
            "single_thread": {"value": round(fl / dt / 1e9, 4), "unit": "GFLOP/s", "cores": 1, "kind": "port",
                              "sample": f"oracle rrLU (tci_oracle.c, loop-for-loop, 1 thread) first {npv} of {r} "
                                        f"pivots on the same {m}x{n} matrix, {dt:.1f} s"},
            "pi_rows": pi_base}
    return base, {"omp": (npo, rpo, cpo, pe_omp), "one": (npv, rp, cp, pe_one)}


def parity_vs_cpu(dev, cpu, r):
    """Device step vs both CPU runs on the same matrix: npivot, pivot rows / columns in pivot order,
    the full permutations (all-pivot run) and the pivot errors, all bitwise."""
    npd, rpd, cpd, ped = dev
    res = {}
    ok = True
    for name, (npc, rpc, cpc, pec) in cpu.items():
        k = min(npc, npd)
        full = npc == npd
        chk = {"npivot_equal": bool(full) if name == "omp" else bool(npd >= npc),
               "pivots_compared": int(k),
               "rowindices_equal": bool(np.array_equal(rpd[:k] - 1, rpc[:k])),
               "colindices_equal": bool(np.array_equal(cpd[:k] - 1, cpc[:k])),
               "pivoterrors_equal": bool(np.array_equal(ped[:k], pec[:k]))}
        if name == "omp" and full:
            chk["permutations_equal"] = bool(np.array_equal(rpd - 1, rpc) and np.array_equal(cpd - 1, cpc))
            chk["lasterror_equal"] = bool(ped[npd] == pec[npc])
        res["vs_" + name] = chk
        ok = ok and all(v for kk, v in chk.items() if kk != "pivots_compared")
    res["ok"] = ok
    return res


if __name__ == "__main__":
    main()
